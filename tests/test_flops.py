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

    with ProcessPoolExecutor(min(len(CF.CONFIGS) * len(CF.FORMS), os.cpu_count() or 1)) as ex:
        futs = {(key, form): ex.submit(CF.count, eid, cont, seed, n, steps, fl)
                for key, eid, cont, seed in CF.CONFIGS for form, fl in CF.FORMS.items()}
        got = {k: CF.summarise(f.result()) for k, f in futs.items()}
    for key, c in doc["configs"].items():
        assert c["flops_per_env_step"] == c["recursive"]["flops_per_env_step"], key
        for form in CF.FORMS:
            v = c[form]
            assert got[key, form]["totals"] == v["totals"], (key, form)
            assert got[key, form]["auto_resets"] == v["auto_resets"], (key, form)
            # the per-phase split adds up to the total
            assert abs(sum(v["by_phase_per_env_step"].values()) - v["flops_per_env_step"]) <= 1e-6 * v["flops_per_env_step"]
        # the two forms differ in the dynamics phase only (the same trajectory to rounding)
        r, j = c["recursive"]["by_phase_per_env_step"], c["jacobian"]["by_phase_per_env_step"]
        assert r["dynamics"] < 0.5 * j["dynamics"], key
        assert abs(r["pgs_sweeps"] - j["pgs_sweeps"]) <= 0.02 * j["pgs_sweeps"], key


def test_fixture_magnitudes():
    """Sanity of the frozen numbers against SURVEY.md §8d's estimate (~1 MFLOP per Reach
    env-step): Reach with the table in [0.5, 2] MFLOP, the object tasks above Reach."""
    with open(FIXTURE) as f:
        c = json.load(f)["configs"]
    assert 0.5e6 <= c["reach_table"]["flops_per_env_step"] <= 2e6
    assert c["reach_no_table"]["flops_per_env_step"] < c["reach_table"]["flops_per_env_step"]
    assert c["push"]["flops_per_env_step"] > c["reach_table"]["flops_per_env_step"]
    assert c["reach_ao"]["recursive"]["by_phase_per_env_step"]["ao_collision_check"] > 0


@pytest.mark.parametrize("model_name", ["panda_custom0", "panda_upstream"])
def test_recursive_dynamics_equals_jacobian_form(oracle, model_name):
    """pgxo_dyn_recursive (CRBA + Newton-Euler, the kernel's formulation, counted under the
    "recursive" key) computes the oracle's M and b (Jacobian form) to rounding, at random poses and
    velocities, with and without gravity."""
    from panda_gym_amd import abi
    from panda_gym_amd.model import load_model

    model = abi.make_model(load_model(model_name), ee_link=11 if model_name == "panda_custom0" else 6)
    params = abi.default_sim_params()
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.uniform(-2.0, 2.0, model.n_dofs)
        qd = rng.uniform(-3.0, 3.0, model.n_dofs)
        for g in (True, False):
            M0 = oracle.mass_matrix(model, q)
            b0 = oracle.bias(model, params, q, qd, with_gravity=g)
            M1, b1 = oracle.dyn_recursive(model, params, q, qd, with_gravity=g)
            assert np.abs(M1 - M0).max() <= 1e-12 * max(1.0, np.abs(M0).max())
            assert np.abs(b1 - b0).max() <= 1e-12 * max(1.0, np.abs(b0).max())


def test_recursive_flag_runs_the_same_trajectory(oracle):
    """The substeps with PGX_FLAG_DYN_RECURSIVE follow the default oracle to rounding (Push, the
    random policy, contacts included)."""
    from panda_gym_amd import abi

    n = 8
    cfg, keep = CF.make_cfg("PandaPush-v3", n, True, 1)
    cfg2, keep2 = CF.make_cfg("PandaPush-v3", n, True, 1, flags=abi.FLAG_DYN_RECURSIVE)
    a, b = oracle.OracleVecEnv(cfg, n), oracle.OracleVecEnv(cfg2, n)
    a.reset(), b.reset()
    for t in range(10):
        oa, ob = a.step(a.sample_actions(t)), b.step(b.sample_actions(t))
        assert np.abs(oa["obs"] - ob["obs"]).max() <= 1e-5, t
    del keep, keep2
