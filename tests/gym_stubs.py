"""Minimal stand-in ``gymnasium`` and ``stable_baselines3`` packages (neither is installed here) for the
class-identity tests: just the names panda_gym_amd.envs binds when they import -- ``gymnasium.Env``,
``gymnasium.register`` / ``registry``, ``gymnasium.spaces.Box`` / ``Dict`` and SB3's abstract
``VecEnv`` with its 2.x constructor and abstract methods (stable_baselines3/common/vec_env/
base_vec_env.py: reset, step_async, step_wait, close, get_attr, set_attr, env_method,
env_is_wrapped; __init__ reads get_attr("render_mode")).  Test infrastructure, not a shim the
product loads."""
import os
import textwrap

GYM = '''
from . import spaces
registry = {}


class Env:
    metadata = {"render_modes": []}
    render_mode = None
    spec = None


def register(id, entry_point=None, kwargs=None, max_episode_steps=None, **extra):
    if id in registry:
        raise RuntimeError(f"{id} registered twice")
    registry[id] = {"entry_point": entry_point, "kwargs": dict(kwargs or {}), "max_episode_steps": max_episode_steps}
'''

SPACES = '''
import numpy as np


class Space:
    pass


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)


class Dict(Space):
    def __init__(self, spaces):
        self.spaces = dict(spaces)

    def __getitem__(self, key):
        return self.spaces[key]
'''

VEC = '''
import abc


class VecEnv(abc.ABC):
    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space
        self.reset_infos = [{} for _ in range(num_envs)]
        self._seeds = [None for _ in range(num_envs)]
        self._options = [{} for _ in range(num_envs)]
        self.render_mode = self.get_attr("render_mode")[0]

    @abc.abstractmethod
    def reset(self): ...

    @abc.abstractmethod
    def step_async(self, actions): ...

    @abc.abstractmethod
    def step_wait(self): ...

    @abc.abstractmethod
    def close(self): ...

    @abc.abstractmethod
    def get_attr(self, attr_name, indices=None): ...

    @abc.abstractmethod
    def set_attr(self, attr_name, value, indices=None): ...

    @abc.abstractmethod
    def env_method(self, method_name, *method_args, indices=None, **method_kwargs): ...

    @abc.abstractmethod
    def env_is_wrapped(self, wrapper_class, indices=None): ...
'''


def write_stubs(root: str) -> str:
    """Write the two stub packages under ``root``; returns ``root`` (put it first on PYTHONPATH)."""
    files = {
        "gymnasium/__init__.py": GYM,
        "gymnasium/spaces/__init__.py": SPACES,
        "stable_baselines3/__init__.py": "",
        "stable_baselines3/common/__init__.py": "",
        "stable_baselines3/common/vec_env/__init__.py": VEC,
    }
    for rel, text in files.items():
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(textwrap.dedent(text))
    return root
