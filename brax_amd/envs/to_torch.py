"""`brax/envs/to_torch.py`: the reference converts JAX outputs to torch via
DLPack; brax_amd's outputs are torch device tensors already."""
from brax_amd.envs.wrappers import TorchWrapper

JaxToTorchWrapper = TorchWrapper
