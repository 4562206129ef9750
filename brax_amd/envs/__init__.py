"""Environment registry (`brax/envs/__init__.py:45-130`).

    env = brax_amd.envs.create('ant', batch_size=4096)   # Episode/AutoReset fused
    state = env.reset(rng)                                # batched State on HBM
    state = env.step(state, action)                       # one kernel launch
"""
import functools
from typing import Callable, Optional

from brax_amd.envs import wrappers
from brax_amd.envs.ant import Ant
from brax_amd.envs.env import Env, PhysicsEnv, State, Wrapper
from brax_amd.envs.half_cheetah import Halfcheetah
from brax_amd.envs.hopper import Hopper, Walker2d
from brax_amd.envs.pendulums import Acrobot, InvertedDoublePendulum, InvertedPendulum
from brax_amd.envs.tasks import Fetch, Grasp, Pusher, Reacher, ReacherAngle, Swimmer, Ur5e
from brax_amd.envs.humanoid import Humanoid
from brax_amd.envs.humanoid_standup import HumanoidStandup
from brax_amd.envs.fast import Fast

_envs = {
    'acrobot': Acrobot,
    'fast': Fast,
    'fetch': Fetch,
    'grasp': Grasp,
    'ant': functools.partial(Ant, use_contact_forces=True),
    'halfcheetah': Halfcheetah,
    'hopper': Hopper,
    'humanoid': Humanoid,
    'humanoidstandup': HumanoidStandup,
    'inverted_pendulum': InvertedPendulum,
    'inverted_double_pendulum': InvertedDoublePendulum,
    'pusher': Pusher,
    'reacher': Reacher,
    'reacherangle': ReacherAngle,
    'swimmer': Swimmer,
    'ur5e': Ur5e,
    'walker2d': Walker2d,
}


def get_environment(env_name, **kwargs) -> Env:
  return _envs[env_name](**kwargs)


def register_environment(env_name: str, env_class):
  _envs[env_name] = env_class


def create(env_name: str, episode_length: int = 1000, action_repeat: int = 1,
           auto_reset: bool = True, batch_size: Optional[int] = None,
           eval_metrics: bool = False, **kwargs) -> Env:
  """Creates an Env (`envs/__init__.py:74-92`); same wrapper order."""
  env = _envs[env_name](**kwargs)
  if episode_length is not None:
    env = wrappers.EpisodeWrapper(env, episode_length, action_repeat)
  if batch_size:
    env = wrappers.VectorWrapper(env, batch_size)
  if auto_reset:
    env = wrappers.AutoResetWrapper(env)
  if eval_metrics:
    env = wrappers.EvalWrapper(env)
  return env


def create_fn(env_name: str, **kwargs) -> Callable[..., Env]:
  return functools.partial(create, env_name, **kwargs)


def create_gym_env(env_name: str, batch_size: Optional[int] = None, seed: int = 0,
                   backend: Optional[str] = None, **kwargs):
  """`envs/__init__.py:118-130`: a gym-API env (VectorGymWrapper when batched);
  observations, rewards and dones are device tensors."""
  environment = create(env_name=env_name, batch_size=batch_size, **kwargs)
  if batch_size is None:
    return wrappers.GymWrapper(environment, seed=seed, backend=backend)
  if batch_size <= 0:
    raise ValueError('`batch_size` should either be None or a positive integer.')
  return wrappers.VectorGymWrapper(environment, seed=seed, backend=backend)
