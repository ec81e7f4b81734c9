"""Run-to-run determinism of the step kernels: two handles with the same seed, stepped with the
same device Philox actions, give bit-identical observations and state in every layout.  (Round 4
found the runtime-model build's one-lane Reach kernel non-deterministic when compiled with SLP
vectorisation -- profiles/r04/rtmodel_slp_nan.log; the parity tests compare against the oracle
per step from the device state, so they cannot see run-to-run variation.)"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import panda_gym_amd as pg

    pg.load_native()
    return pg


def _rollout(pg, env_id, n, lanes, steps, **kw):
    v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=21, lanes_per_env=lanes, **kw)
    v.reset_tensors(seed=21)
    out = []
    for t in range(steps):
        v.step_tensors(v.sample_actions(t))
        st = v.state()
        out.append(torch.cat([v.obs, st["q"].T, st["qd"].T, st["contacts"].T], 1).cpu().numpy().copy())
    v.close()
    return np.stack(out)


@pytest.mark.parametrize("env_id,lanes", [("PandaReach-v3", 16), ("PandaReach-v3", 1), ("PandaPush-v3", 16),
                                          ("PandaPush-v3", 1), ("PandaPickAndPlaceJoints-v3", 1),
                                          ("PandaPickAndPlaceJoints-v3", 16), ("PandaReachAO-v3", 16)])
def test_step_kernels_are_deterministic(pg, env_id, lanes):
    a = _rollout(pg, env_id, 256, lanes, 30)
    b = _rollout(pg, env_id, 256, lanes, 30)
    diff = np.flatnonzero(~((a == b) | (np.isnan(a) & np.isnan(b))).all(axis=(1, 2)))
    assert diff.size == 0, f"first differing step {diff[:1]}"
    assert np.isfinite(a).all()


def test_runtime_model_library_is_deterministic(pg):
    from panda_gym_amd import _native

    path = os.path.join(os.path.dirname(_native.LIB_PATH), "libpgx_rtmodel.so")
    kw = {"lib_path": path, "sim_params": {"friction": 0.3}}
    for env_id, lanes in (("PandaReach-v3", 1), ("PandaReach-v3", 16), ("PandaPush-v3", 1)):
        a = _rollout(pg, env_id, 64, lanes, 10, **kw)
        b = _rollout(pg, env_id, 64, lanes, 10, **kw)
        assert np.isfinite(a).all(), (env_id, lanes)
        assert np.array_equal(a, b), (env_id, lanes)


@pytest.mark.parametrize("env_id,sort", [("PandaReach-v3", None), ("PandaPickAndPlace-v3", None),
                                         ("PandaPickAndPlace-v3", "1")])
def test_captured_steps_equal_eager_steps(pg, env_id, sort, monkeypatch):
    """capture_steps: k steps replayed from a HIP graph equal the same k steps launched eagerly, bit
    for bit (state and outputs), over two replays -- the kernels are graph-capturable (no host
    synchronisation or allocation on the step path; with PGX_SORT_ENVS=1 the heavy-first order's
    memset and sort kernels are captured too).  k spans an auto-reset (TimeLimit 3)."""
    if sort is not None:
        monkeypatch.setenv("PGX_SORT_ENVS", sort)
    n, k = 96, 4
    kw = dict(num_envs=n, device="cuda:0", seed=9, max_episode_steps=3)
    eager, graphed = pg.PandaVecEnv(env_id, **kw), pg.PandaVecEnv(env_id, **kw)
    eager.reset_tensors(seed=9)
    graphed.reset_tensors(seed=9)
    acts = torch.empty((k, n, eager.action_dim), device="cuda:0")
    g = graphed.capture_steps(k, acts)
    for rep in range(2):
        for i in range(k):
            acts[i].copy_(eager.sample_actions(100 * rep + i))
        for i in range(k):
            eager.step_tensors(acts[i])
        g.replay()
        torch.cuda.synchronize()
        se, sg = eager.state(), graphed.state()
        for key in ("q", "qd", "qc", "goal", "object", "contacts", "elapsed", "episode"):
            assert torch.equal(se[key], sg[key]), key
        for key in ("obs", "reward", "truncated", "terminal_obs"):
            assert torch.equal(getattr(eager, key), getattr(graphed, key)), key
    # the random-policy form: the draws of capture time, repeated on every replay
    g2 = graphed.capture_steps(2)
    g2.replay()
    for i in range(2):
        eager.step_tensors(eager.sample_actions(graphed._step_index + i))
    torch.cuda.synchronize()
    assert torch.equal(eager.state()["q"], graphed.state()["q"])
    eager.close()
    graphed.close()
