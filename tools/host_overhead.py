"""Host cost of one Env.step call (Ant, 4096 envs): wall per call with the
launch queue absorbing the kernels, then the synchronised rate, plus a
cProfile of the Python path. Diagnostic, not part of the product."""
import cProfile, pstats, sys, time, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import envs
dev = torch.device('cuda', 0)
B = 4096
env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
st = env.reset(0)
acts = torch.rand((64, B, 8), device=dev) * 2 - 1
for k in range(50):
  st = env.step(st, acts[k % 64])
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for k in range(n):
  st = env.step(st, acts[k % 64])
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f'host us/step {1e6*(t1-t0)/n:.1f}  total us/step {1e6*(t2-t0)/n:.1f}')
pr = cProfile.Profile()
pr.enable()
for k in range(n):
  st = env.step(st, acts[k % 64])
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats('tottime').print_stats(18)

# the C entry point alone: prebuilt arguments, launches queued back to back
import ctypes as C  # noqa: E402
import bench  # noqa: E402
from brax_amd import _native, abi  # noqa: E402
from brax_amd.system import _stream, qp_struct  # noqa: E402
u = env.unwrapped
qp, obs, scal, met = u._alloc(B)
p = u._params({'episode_length': 1000, 'action_repeat': 1, 'auto_reset': True},
              st.info['first_qp'], st.info['first_obs'])
sin = abi.BxEnvState()
sin.qp = qp_struct(st.qp, True)
sin.done = st.done.data_ptr()
sin.steps = st.info['steps'].data_ptr()
sout = abi.BxEnvState()
sout.qp = qp_struct(qp, True)
sout.obs = obs.data_ptr()
base = scal.data_ptr()
sout.reward, sout.done, sout.steps, sout.truncation = base, base + 4 * B, base + 8 * B, base + 12 * B
sout.metrics = met.data_ptr()
lib = _native.lib()
a0 = acts[0]
args = (u.sys._h, C.byref(p), B, C.byref(sin), C.c_void_p(a0.data_ptr()), a0.stride(0), 8,
        C.byref(sout), _stream(0))
for _ in range(20):
  lib.bx_env_step(*args)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
  lib.bx_env_step(*args)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f'C entry point alone: host us/call {1e6*(t1-t0)/n:.1f}  total us/call {1e6*(t2-t0)/n:.1f}')
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
t0 = time.perf_counter()
for k in range(n):
  lib.bx_uniform(C.c_void_p(a0.data_ptr()), B * 8, 1, k, -1.0, 1.0, s)
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f'bx_uniform alone: host us/call {1e6*(t1-t0)/n:.1f}')
