"""Oracle and host logic against golden vectors made from the reference's own numpy code
(tests/golden/make_golden.py: panda_gym/utils.py distance + the task reward lines, and
PCG64 reset draws)."""
import os

import numpy as np

from panda_gym_amd import abi
from panda_gym_amd.envs import seeded_goal

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_distance_f32_f64_bit_exact(oracle):
    """Env-step path: utils.distance(float32 achieved_goal, float64 goal) (core.py:358,366)."""
    g = np.load(os.path.join(GOLD, "reward_golden.npz"))
    d = np.array([oracle.distance_f32_f64(a, b) for a, b in zip(g["ag32"], g["g64"])])
    assert np.array_equal(d, g["d_f32_f64"])
    assert np.array_equal(d < 0.05, g["success_f32_f64"])
    sparse = -np.array(d > 0.05, dtype=np.float32)
    assert np.array_equal(sparse.view(np.uint32), g["sparse_f32_f64"].view(np.uint32))  # includes -0.0


def test_compute_reward_f32_bit_exact(oracle):
    """HER path: compute_reward(float32 ag, float32 dg) keeps float32 arithmetic (reach.py:84-89)."""
    g = np.load(os.path.join(GOLD, "reward_golden.npz"))
    r = oracle.compute_reward_f32(g["ag32"], g["dg32"], abi.REWARD_SPARSE)
    assert np.array_equal(r.view(np.uint32), g["sparse_f32_f32"].view(np.uint32))
    r = oracle.compute_reward_f32(g["ag32"], g["dg32"], abi.REWARD_DENSE)
    assert np.array_equal(r.view(np.uint32), g["dense_f32_f32"].view(np.uint32))


def test_sparse_no_penalty_is_negative_zero():
    g = np.load(os.path.join(GOLD, "reward_golden.npz"))
    hit = g["d_f32_f64"] <= 0.05
    assert hit.any()
    assert np.all(np.signbit(g["sparse_f32_f64"][hit]))


def test_reset_draws_match_reference_values():
    """SURVEY §8c examples: Reach seed 12345, Push seed 6789 (goal then object)."""
    gold = np.load(os.path.join(GOLD, "reset_golden.npz"))
    i = list(gold["seeds"]).index(12345)
    assert np.array_equal(gold["reach_goal"][i],
                          [-0.08179919325984909, -0.054972498087074134, 0.23920963719982022])
    j = list(gold["seeds"]).index(6789)
    assert np.allclose(gold["push_goal_obj"][j], [0.016656701905313265, -0.08166345664461347, 0.02,
                                                  -0.1447002606327806, 0.07620567116508836, 0.02], atol=0, rtol=0)


def test_host_seeded_goal_matches_golden():
    gold = np.load(os.path.join(GOLD, "reset_golden.npz"))
    sp = abi.EnvSpec()
    for s, gl in zip(gold["seeds"], gold["reach_goal"]):
        assert np.array_equal(seeded_goal(sp, int(s)), gl)


def test_host_seeded_push_and_pnp_resets_match_golden():
    """Push / PickAndPlace reset draws (goal then object, PnP's z coin in between) against
    the fixture generated from the reference's task code order (make_golden.py)."""
    from panda_gym_amd.envs import seeded_reset

    gold = np.load(os.path.join(GOLD, "reset_golden.npz"))
    push = abi.EnvSpec(task=abi.TASK_PUSH)
    pnp = abi.EnvSpec(task=abi.TASK_PICK_AND_PLACE, block_gripper=False)
    for s, gp, gq in zip(gold["seeds"], gold["push_goal_obj"], gold["pnp_goal_obj"]):
        g, o = seeded_reset(push, int(s))
        assert np.array_equal(np.concatenate([g, o]), gp)
        g, o = seeded_reset(pnp, int(s))
        assert np.array_equal(np.concatenate([g, o]), gq)
