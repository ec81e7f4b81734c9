"""The fp32 build of the oracle (oracle/fp32_emul.cpp), the yardstick of test_gpu_fp32_envelope.py.

Checked on the CPU: the build really evaluates in fp32 (the joint state it integrates holds float
values, the fp64 build's do not), and it is the same algorithm (from the same states its
positions stay within 1e-3 of the fp64 build's; velocities carry the PGS residual exit's
~3e-4 rad/s resolution amplified by the IK, up to ~1e-2).
"""
import numpy as np

from oracle import count_flops as CF


def _run(oracle, key, n=16, steps=12):
    eid, cont, seed = next((e, c, s) for k, e, c, s in CF.CONFIGS if k == key)
    cfg, keep = CF.make_cfg(eid, n, cont, seed)
    a = oracle.OracleVecEnv(cfg, n)
    b = oracle.OracleVecEnv(cfg, n, fp32=True)
    a.reset()
    out = []
    for t in range(steps):
        act = a.sample_actions(t)
        for k in ("q", "qd", "qc", "goal", "obj", "elapsed", "episode"):
            getattr(b, k)[:] = getattr(a, k)
        r = a.step(act), b.step(act)
        out.append((r[0], r[1], a.q.copy(), b.q.copy()))
    del keep
    return out


def test_fp32_build_rounds_to_float(oracle):
    out = _run(oracle, "reach_table")
    q64 = np.concatenate([r[2] for r in out])   # the joint state (doubles in both builds)
    q32 = np.concatenate([r[3] for r in out])
    assert np.array_equal(q32, q32.astype(np.float32).astype(np.float64))
    assert not np.array_equal(q64, q64.astype(np.float32).astype(np.float64))


def test_fp32_build_is_the_algorithm(oracle):
    for key in ("reach_table", "push", "reach_ao"):
        out = _run(oracle, key)
        for r64, r32, _, _ in out:
            keep = r64["truncated"] == 0
            d = np.abs(r64["obs"][keep] - r32["obs"][keep])
            assert d[:, :3].max() <= 1e-3, key
            assert d[:, 3:6].max() <= 5e-2, key
