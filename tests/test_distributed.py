"""World-size-2 gloo rehearsal of the multi-GPU sharding (CPU; the oracle stands in for the GPU step).

Checks the sharding contract bench.py relies on: each rank's envs are the
global ids [r*E, (r+1)*E), draws are keyed by global id, so the sharded run
equals the unsharded run env for env; timing is reduced with MAX and the
statistics all-gather returns one row per rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

E = 6
STEPS = 55  # crosses one auto-reset (50-step episodes)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rollout(n, offset, steps):
    from oracle import oracle as O
    from panda_gym_amd import abi
    from panda_gym_amd.model import load_model

    m = abi.make_model(load_model("panda_custom0"), ee_link=11)
    p = abi.default_sim_params()
    cfg = abi.make_config(abi.EnvSpec(), n, m, p, seed=77, env_id_offset=offset)
    env = O.OracleVecEnv(cfg, n)
    env.reset()
    obs = []
    for t in range(steps):
        obs.append(env.step(env.sample_actions(t))["obs"].copy())
    return np.stack(obs), env.goal.copy()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from panda_gym_amd.shard import gather_stats, max_over_ranks, shard_offset

    obs, goal = _rollout(E, shard_offset(rank, E), STEPS)
    t = max_over_ranks(float(rank + 1), dist)
    st = gather_stats([rank, 2.0 * rank, 0.5, 50.0], dist)
    gathered = [None] * world
    dist.all_gather_object(gathered, (obs, goal))
    if rank == 0:
        q.put((t, st.numpy(), gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_equals_single():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, st, gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0
    assert st.shape == (2, 4) and st[1, 1] == 2.0
    obs = np.concatenate([g[0] for g in gathered], axis=1)
    goal = np.concatenate([g[1] for g in gathered], axis=0)
    ref_obs, ref_goal = _rollout(world * E, 0, STEPS)
    assert np.array_equal(obs, ref_obs)
    assert np.array_equal(goal, ref_goal)
