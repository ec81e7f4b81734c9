"""The multi-GPU path of BASELINE configs[4] (ReachAO, 65536 envs = 8 x 8192), exercised on one GPU.

SURVEY.md §8e / DESIGN.md §7: rank r owns global env ids [r*E, (r+1)*E) through env_id_offset,
and every random draw (device Philox actions, auto-reset goals and obstacles) is keyed by the
global id, so a sharded run must equal the unsharded one env for env.  Checked here through the
C-ABI (libpgx): eight 8192-env handles with offsets r*8192 against one 65536-env handle, every
output of every step bit for bit over 30 steps with collisions, successes and resets; and the
bench's own multi-rank launcher (``bench.py --gpus 2 --dist-backend gloo``: two ranks sharing the
one GPU, gloo collectives on the host) against the single-rank run of the same global envs.
"""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pg():
    import panda_gym_amd as pg

    pg.load_native()
    return pg


def test_eight_shards_equal_one_handle(pg):
    env_id, E, W, steps = "PandaReachAO-v3", 8192, 8, 30
    full = pg.PandaVecEnv(env_id, num_envs=W * E, device="cuda:0", seed=1)
    shards = [pg.PandaVecEnv(env_id, num_envs=E, device="cuda:0", seed=1, env_id_offset=r * E) for r in range(W)]
    full.reset_tensors()
    for s in shards:
        s.reset_tensors()
    fields = ("obs", "achieved_goal", "desired_goal", "reward", "success", "terminated", "truncated",
              "task_trunc")
    finished = 0
    for t in range(steps):
        full.step_tensors(full.sample_actions(t))
        for s in shards:
            s.step_tensors(s.sample_actions(t))
        for f in fields:
            got = torch.cat([getattr(s, f) for s in shards])
            assert torch.equal(got, getattr(full, f)), (t, f)
        done = full.truncated.bool() | full.terminated.bool()
        if done.any():   # terminal outputs are written for the finished envs only
            for f in ("terminal_obs", "terminal_ag", "terminal_dg"):
                got = torch.cat([getattr(s, f) for s in shards])
                assert torch.equal(got[done], getattr(full, f)[done]), (t, f)
        finished += int(done.sum())
    fs = full.state()
    for k in ("q", "qd", "goal", "obstacles", "contacts", "elapsed", "episode"):
        got = torch.cat([s.state()[k] for s in shards], dim=-1)
        assert torch.equal(got, fs[k]), k
    assert finished > 0
    for s in shards:
        s.close()
    full.close()


def _bench(args, timeout=240):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_on_one_gpu_match_single_rank():
    """bench.py's launcher (a child torch.distributed.run job) with two gloo ranks on this one
    GPU: n_gpus 2, ReachAO global_envs 2 x 4096, and the final observations of every env equal
    the single-rank run of the same 8192 global envs (obs_digest)."""
    common = ["--steps", "5", "--warmup", "2", "--task-steps", "30", "--no-cpu-baseline", "--no-her", "--no-tasks",
              "--kernel-launches", "5"]
    two = _bench(["--gpus", "2", "--dist-backend", "gloo", "--envs", "1024", "--ao-envs", "4096"] + common)
    one = _bench(["--gpus", "1", "--envs", "1024", "--ao-envs", "8192"] + common)
    assert two["n_gpus"] == 2 and two["config"]["global_envs"] == 2048
    ao2, ao1 = two["reach_ao"], one["reach_ao"]
    assert ao2["n_gpus"] == 2 and ao2["global_envs"] == 8192 and ao1["global_envs"] == 8192
    assert ao2["obs_digest"] == ao1["obs_digest"]
