"""The frozen algorithmic FLOP counts (tests/golden/flops_per_env_step.json).

The counts come from the operation-counting build of the fp64 oracle (oracle/flops_count.cpp:
pgx_oracle.c compiled with a counting double).  Checked here: that build computes exactly what
the plain oracle computes (same outputs, bit for bit), and a recount of the fixture's own sample
reproduces every frozen total exactly (the counts are deterministic), so the constant bench.py
uses for the VALU roofline cannot drift from the restatement it is counted on.
"""
import json
import os

import numpy as np
import pytest

from oracle import count_flops as CF

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "flops_per_env_step.json")


@pytest.mark.parametrize("key,env_id,contacts,seed", CF.CONFIGS)
def test_counting_build_is_the_oracle(oracle, key, env_id, contacts, seed):
    n, steps = 8, 12
    cfg, keep = CF.make_cfg(env_id, n, contacts, seed)
    a = oracle.OracleVecEnv(cfg, n)
    b = oracle.OracleVecEnv(cfg, n, counting=True)
    ra, rb = a.reset(), b.reset()
    assert np.array_equal(ra["obs"], rb["obs"])
    for t in range(steps):
        oa = a.step(a.sample_actions(t))
        ob = b.step(b.sample_actions(t))
        for k in oa:
            assert np.array_equal(oa[k], ob[k]), (key, t, k)
    assert np.array_equal(a.q, b.q) and np.array_equal(a.qd, b.qd) and np.array_equal(a.obj, b.obj)
    del keep


def test_fixture_recount_is_exact(oracle):
    with open(FIXTURE) as f:
        doc = json.load(f)
    n, steps = doc["sample"]["envs"], doc["sample"]["steps"]
    from concurrent.futures import ProcessPoolExecutor

    with ProcessPoolExecutor(min(len(CF.CONFIGS), os.cpu_count() or 1)) as ex:
        futs = {key: ex.submit(CF.count, eid, cont, seed, n, steps) for key, eid, cont, seed in CF.CONFIGS}
        got = {key: CF.summarise(f.result()) for key, f in futs.items()}
    for key, v in doc["configs"].items():
        assert got[key]["totals"] == v["totals"], key
        assert got[key]["auto_resets"] == v["auto_resets"], key
        # the per-phase split adds up to the total
        assert abs(sum(v["by_phase_per_env_step"].values()) - v["flops_per_env_step"]) <= 1e-6 * v["flops_per_env_step"]


def test_fixture_magnitudes():
    """Sanity of the frozen numbers against SURVEY.md §8d's estimate (~1 MFLOP per Reach
    env-step): Reach with the table in [0.5, 2] MFLOP, the object tasks above Reach."""
    with open(FIXTURE) as f:
        c = json.load(f)["configs"]
    assert 0.5e6 <= c["reach_table"]["flops_per_env_step"] <= 2e6
    assert c["reach_no_table"]["flops_per_env_step"] < c["reach_table"]["flops_per_env_step"]
    assert c["push"]["flops_per_env_step"] > c["reach_table"]["flops_per_env_step"]
    assert c["reach_ao"]["by_phase_per_env_step"]["ao_collision_check"] > 0
