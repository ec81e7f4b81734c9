"""panda-gym_amd: MI355X-native batched Panda manipulation environment.

The reference (RaikoPipe/panda-gym) steps one PyBullet env per process; here N
envs step in lockstep inside one HIP kernel launch per env step (libpgx.so,
C-ABI in include/pgx.h).  Public surface mirrors the reference's:

    import panda_gym_amd as pg
    pg.register_envs(50)                     # panda_gym.register_envs
    env = pg.make("PandaReach-v3")           # RobotTaskEnv + TimeLimit, one env
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=4096)   # SB3 VecEnv protocol
"""
from .envs import (Box, DictSpace, PandaEnv, PandaVecEnv, make, pcg64_from_record, pcg64_record, pcg64_records, register_envs,
                   registered_ids, seeded_goal, seeded_reset, spec, task_draws)
from .her import HerReplayBuffer
from ._native import PgxError, load as load_native
from .model import Model, load_model

__version__ = "0.1.0"

__all__ = ["Box", "DictSpace", "PandaEnv", "PandaVecEnv", "make", "register_envs", "registered_ids",
           "seeded_goal", "seeded_reset", "spec", "task_draws", "pcg64_record", "pcg64_records", "pcg64_from_record", "PgxError", "load_native", "Model", "load_model",
           "HerReplayBuffer"]
