"""GPU parity: libpgx (HIP, fp32) against the fp64 oracle on the same seeded inputs.

Tolerances: observations/achieved goals within 1e-4 (BASELINE.json north star,
fp32 vs the fp64 restatement); integer/byte outputs (truncation, episode
counters, Philox draws, HER rewards on identical inputs) bit-exact; is_success
and sparse rewards bit-exact except where the distance lies within 1e-5 of the
threshold (the fp32 achieved goal legitimately differs from the fp64 one there).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

OBS_TOL = 1e-4
EDGE = 1e-5


@pytest.fixture(scope="module")
def pg():
    import panda_gym_amd as pg

    pg.load_native()
    return pg


def _state_to_oracle(venv, ref):
    from oracle import oracle as orc

    orc.set_robot_budget(venv.robot_contact_budget() or -1)   # the layout's budget
    st = venv.state()
    ref.q[:] = st["q"].double().cpu().numpy().T
    ref.qd[:] = st["qd"].double().cpu().numpy().T
    ref.qc[:] = st["qc"].double().cpu().numpy().T
    ref.goal[:] = st["goal"].cpu().numpy().T
    ref.elapsed[:] = st["elapsed"].cpu().numpy()
    ref.episode[:] = st["episode"].cpu().numpy().view(np.uint32)
    ref.obj[:, :13] = st["object"].double().cpu().numpy().T
    orc.set_contact_cache(ref.obj, st["contacts"].double().cpu().numpy().T)
    if "obstacles" in st:
        ref.obj[:, orc.OBJ_AO:orc.OBJ_AO + 24] = st["obstacles"].double().cpu().numpy().T
    # Bullet's persistent manifolds (the per-pair budget's object / ReachAO kernels)
    orc.set_manifolds(ref.obj, st["manifolds"].double().cpu().numpy().T if "manifolds" in st
                      else np.zeros((ref.obj.shape[0], 1)))


def _check_step(out_gpu, out_ref, goal):
    obs, ag, dg, rew, succ = out_gpu
    assert np.all(np.isfinite(obs))
    err = np.abs(obs - out_ref["obs"]).max()
    assert err <= OBS_TOL, f"obs error {err}"
    assert np.abs(ag - out_ref["ag"]).max() <= OBS_TOL
    assert np.array_equal(dg, out_ref["dg"])
    d = np.linalg.norm(out_ref["ag"].astype(np.float64) - goal, axis=-1)
    safe = np.abs(d - 0.05) > EDGE
    assert np.array_equal(succ[safe].astype(bool), out_ref["success"][safe].astype(bool))
    return err


def _gpu_out(venv):
    o = venv._obs_dict()
    return (o["observation"].cpu().numpy(), o["achieved_goal"].cpu().numpy(), o["desired_goal"].cpu().numpy(),
            venv.reward.cpu().numpy(), venv.success.cpu().numpy())


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaReachDense-v3", "PandaReachJoints-v3"])
def test_one_step_parity(pg, oracle, env_id, lanes):
    n = 512
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=3, lanes_per_env=lanes)
    venv.reset_tensors()
    ref = oracle.OracleVecEnv(venv._cfg, n)
    for k in range(3):  # a few steps so the start states are not all neutral
        venv.step_tensors(venv.sample_actions(100 + k))
    _state_to_oracle(venv, ref)
    goal = ref.goal.copy()
    acts = venv.sample_actions(7).clone()
    venv.step_tensors(acts)
    out = ref.step(acts.cpu().numpy())
    _check_step(_gpu_out(venv), out, goal)
    dense = env_id.find("Dense") >= 0
    r_gpu = venv.reward.cpu().numpy()
    if dense:
        assert np.abs(r_gpu - out["reward"]).max() <= OBS_TOL
    venv.close()


def test_episode_trajectory_parity(pg, oracle, lanes):
    """Free-running rollout across an auto-reset.

    Positions (ee position, achieved goal) stay within 1e-4 of the oracle for the whole episode.
    Velocities: the solver stops when the squared row residual <= 1e-7 (pybullet's
    solverResidualThreshold), so each joint velocity is only defined to sqrt(1e-7) = 3.2e-4 rad/s;
    an fp32/fp64 difference in the exit sweep moves the EE velocity by up to sum_j |J_ij| * 3.2e-4
    (~1e-3 m/s for the Panda's ~0.5 m lever arms).  Bound: max 2.5e-3, 99th percentile 3e-4
    (DESIGN.md §5).  Without the table: a free-running trajectory through contact events is
    chaotic at fp32 rounding (test_gpu_contacts.py holds those per step)."""
    n = 256
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=n, device="cuda:0", seed=11, contacts=False,
                          lanes_per_env=lanes)
    venv.reset_tensors()
    ref = oracle.OracleVecEnv(venv._cfg, n)
    _state_to_oracle(venv, ref)
    worst_pos, worst_vel, vel_err = 0.0, 0.0, []
    for t in range(60):
        acts = venv.sample_actions(t).clone()
        a_ref = ref.sample_actions(t)
        assert np.array_equal(acts.cpu().numpy(), a_ref), "device Philox actions differ from oracle"
        venv.step_tensors(acts)
        goal = ref.goal.copy()
        out = ref.step(a_ref)
        g = _gpu_out(venv)
        tr = venv.truncated.cpu().numpy()
        assert np.array_equal(tr, out["truncated"]), t
        if tr.any():
            # the episode just ended: compare terminal observations; new goals come from Philox
            te = np.abs(venv.terminal_obs.cpu().numpy() - out["terminal_obs"])
            assert te[:, :3].max() <= OBS_TOL and te[:, 3:].max() <= 10 * OBS_TOL
            assert np.array_equal(g[2], out["dg"])
            assert np.abs(g[0] - out["obs"]).max() <= 1e-6   # reset obs: neutral pose
            continue
        e = np.abs(g[0] - out["obs"])
        worst_pos = max(worst_pos, float(e[:, :3].max()), float(np.abs(g[1] - out["ag"]).max()))
        worst_vel = max(worst_vel, float(e[:, 3:].max()))
        vel_err.append(e[:, 3:].max(axis=1))
    assert worst_pos <= OBS_TOL, f"trajectory position error {worst_pos}"
    assert worst_vel <= 25 * OBS_TOL, f"trajectory velocity error {worst_vel}"
    assert np.percentile(np.concatenate(vel_err), 99) <= 3 * OBS_TOL
    venv.close()


def test_compute_reward_bit_exact_vs_reference_golden(pg):
    import os

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "reward_golden.npz"))
    for env_id, key in [("PandaReach-v3", "sparse_f32_f32"), ("PandaReachDense-v3", "dense_f32_f32")]:
        venv = pg.PandaVecEnv(env_id, num_envs=1, device="cuda:0")
        r = venv.compute_reward(g["ag32"], g["dg32"], {})
        assert r.dtype == np.float32
        assert np.array_equal(r.view(np.uint32), g[key].view(np.uint32)), key
        venv.close()


def test_seeded_reset_goals_match_reference_draws(pg):
    import os

    gold = np.load(os.path.join(os.path.dirname(__file__), "golden", "reset_golden.npz"))
    env = pg.make("PandaReach-v3")
    for s, gl in zip(gold["seeds"], gold["reach_goal"]):
        obs, info = env.reset(seed=int(s))
        st = env._vec.state()
        assert np.array_equal(st["goal"].cpu().numpy()[:, 0], gl)
        assert np.array_equal(obs["desired_goal"], gl.astype(np.float32))
    env.close()


def test_auto_reset_goals_match_oracle_philox(pg, oracle):
    n = 128
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=n, device="cuda:0", seed=1234, env_id_offset=5000,
                          max_episode_steps=2)
    venv.reset_tensors()
    ref = oracle.OracleVecEnv(venv._cfg, n)
    ref.reset()
    assert np.array_equal(venv.state()["goal"].cpu().numpy().T, ref.goal)
    for t in range(4):
        a = venv.sample_actions(t).clone()
        venv.step_tensors(a)
        ref.step(a.cpu().numpy())
    st = venv.state()
    assert np.array_equal(st["goal"].cpu().numpy().T, ref.goal)
    assert np.array_equal(st["episode"].cpu().numpy().view(np.uint32), ref.episode)
    assert np.array_equal(st["elapsed"].cpu().numpy(), ref.elapsed)
    venv.close()


def test_seed_determinism(pg):
    """test/seed_test.py:7-28 (PandaReach-v3, seed 12345, fixed 6-action sequence, twice)."""
    actions = [np.array([-0.931, 0.979, -0.385]), np.array([-0.562, 0.391, -0.532]),
               np.array([0.042, 0.254, -0.624]), np.array([0.465, 0.745, 0.284]),
               np.array([-0.237, 0.995, -0.425]), np.array([0.67, 0.472, 0.972])]
    finals = []
    env = pg.make("PandaReach-v3")
    for _ in range(2):
        env.reset(seed=12345)
        for a in actions:
            obs, _, term, trunc, _ = env.step(a)
            if term or trunc:
                obs, _ = env.reset()
        finals.append(obs)
    for k in ("observation", "achieved_goal", "desired_goal"):
        assert np.array_equal(finals[0][k], finals[1][k])
    env.close()


def test_save_and_restore_state(pg):
    """test/save_and_restore_test.py:9-27: save -> step -> reset -> restore -> step gives equal obs."""
    env = pg.make("PandaReach-v3")
    env.reset()
    sid = env.save_state()
    action = env.action_space.sample()
    o1, _, _, _, _ = env.step(action)
    env.reset()
    env.restore_state(sid)
    o2, _, _, _, _ = env.step(action)
    for k in ("observation", "achieved_goal", "desired_goal"):
        assert np.array_equal(o1[k], o2[k])
    env.close()


def test_remove_state(pg):
    """test/save_and_restore_test.py:30-36: restoring a removed state raises."""
    env = pg.make("PandaReach-v3")
    env.reset()
    sid = env.save_state()
    env.remove_state(sid)
    with pytest.raises(pg.PgxError):
        env.restore_state(sid)
    env.close()


def test_snapshot_ids_through_the_c_abi(pg):
    """pgx_snapshot / pgx_restore / pgx_release called through ctypes (include/pgx.h): ids are the
    first non-negative integer not in use (pybullet saveState, pybullet.py:79-86), a released id
    is handed out again, restoring or releasing an id not in use returns PGX_E_INVALID
    (save_and_restore_test.py:30-36: pybullet.error), and a restore brings back every state bit."""
    import ctypes as C

    import torch

    from panda_gym_amd import _native

    venv = pg.PandaVecEnv("PandaPush-v3", num_envs=64, device="cuda:0", seed=3)
    lib, h, st = venv.lib, venv._h, venv._stream()
    venv.reset_tensors()
    before = {k: v.clone() for k, v in venv.state().items()}
    ids = []
    for _ in range(3):
        sid = C.c_int32(-7)
        assert lib.pgx_snapshot(h, C.byref(sid), st) == 0
        ids.append(sid.value)
    assert ids == [0, 1, 2]
    assert lib.pgx_release(h, 1) == 0
    assert lib.pgx_restore(h, 1, st) == _native.PGX_E_INVALID
    assert b"no such saved state" in lib.pgx_last_error()
    assert lib.pgx_release(h, 1) == _native.PGX_E_INVALID
    assert lib.pgx_restore(h, 7, st) == _native.PGX_E_INVALID
    assert lib.pgx_restore(h, -1, st) == _native.PGX_E_INVALID
    sid = C.c_int32(-7)
    assert lib.pgx_snapshot(h, C.byref(sid), st) == 0 and sid.value == 1   # the freed id again
    for t in range(5):
        venv.step_tensors(venv.sample_actions(t))
    assert lib.pgx_restore(h, 0, st) == 0
    torch.cuda.synchronize()
    for k, v in venv.state().items():
        assert torch.equal(v, before[k]), k
    for i in (0, 1, 2):
        assert lib.pgx_release(h, i) == 0
    venv.close()


def test_single_env_time_limit(pg):
    env = pg.make("PandaReach-v3", max_episode_steps=5)
    env.reset(seed=0)
    truncs = []
    for _ in range(5):
        _, r, term, trunc, info = env.step(np.zeros(3, np.float32))
        truncs.append(trunc)
        assert term is False and isinstance(r, float) and "is_success" in info
    assert truncs == [False] * 4 + [True]
    env.close()


def test_sb3_vecenv_protocol(pg):
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=8, device="cuda:0", max_episode_steps=3)
    obs = venv.reset(seed=0)
    assert obs["observation"].shape == (8, 6)
    for t in range(3):
        obs, rew, dones, infos = venv.step(np.zeros((8, 3), np.float32))
    assert dones.all()
    assert all(i["TimeLimit.truncated"] for i in infos)
    assert infos[0]["terminal_observation"]["observation"].shape == (6,)
    r = venv.env_method("compute_reward", obs["achieved_goal"], obs["desired_goal"], infos)[0]
    assert r.shape == (8,)
    venv.close()


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaPush-v3", "PandaReachAO-v3"])
def test_sb3_host_path_matches_device_path(pg, env_id):
    """step_async/step_wait (pinned staging, one sync) returns exactly the device path's
    outputs, including the terminal observations of the auto-reset at the time limit."""
    n, T = 64, 7
    a_env = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, max_episode_steps=3)
    b_env = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, max_episode_steps=3)
    a_env.reset_tensors()
    b_env.reset()
    rng = np.random.default_rng(1)
    for t in range(T):
        act = rng.uniform(-1, 1, (n, a_env.action_dim)).astype(np.float32)
        obs, rew, term, trunc, succ = a_env.step_tensors(torch.as_tensor(act, device="cuda:0"))
        want = {k: v.cpu().numpy() for k, v in obs.items()}
        done = (term | trunc).bool().cpu().numpy()
        tobs = a_env.terminal_obs.cpu().numpy()
        o, r, d, infos = b_env.step(act)
        for k in want:
            assert np.array_equal(o[k], want[k]), (t, k)
        assert np.array_equal(r, rew.cpu().numpy())
        assert np.array_equal(d, done)
        assert [i["is_success"] for i in infos] == succ.bool().cpu().tolist()
        assert [i["is_truncated"] for i in infos] == a_env.task_truncated().tolist()
        te = term.bool().cpu().numpy()
        for i in np.nonzero(done)[0]:
            assert np.array_equal(infos[i]["terminal_observation"]["observation"], tobs[i])
            assert infos[i]["TimeLimit.truncated"] == bool(not te[i])
        if env_id != "PandaReachAO-v3":   # (ReachAO also ends episodes by success or collision)
            assert done.any() == ((t + 1) % 3 == 0)
    # device actions go straight through step_async
    o, *_ = b_env.step(torch.zeros((n, b_env.action_dim), device="cuda:0"))
    assert o["observation"].shape == (n, b_env.obs_dim)
    a_env.close()
    b_env.close()


def test_vecenv_seed_applies_to_next_reset(pg):
    """SB3 protocol: VecEnv.seed(s) then reset() seeds env i with s + i (as reset(seed=s))."""
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=8, device="cuda:0")
    assert venv.seed(123) == [123 + i for i in range(8)]
    a = venv.reset()["desired_goal"]
    b = venv.reset(seed=123)["desired_goal"]
    c = venv.reset()["desired_goal"]          # the pending seed was consumed: a fresh draw
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    want = np.stack([pg.seeded_goal(venv.spec, 123 + i) for i in range(8)]).astype(np.float32)
    assert np.array_equal(a, want)
    venv.close()


def test_large_batch_properties(pg):
    """Full-size batch (65536 envs): finite, bounded, deterministic, reward consistent with success."""
    n = 65536
    outs = []
    for _ in range(2):
        venv = pg.PandaVecEnv("PandaReach-v3", num_envs=n, device="cuda:0", seed=99)
        venv.reset_tensors()
        for t in range(12):
            venv.step_tensors(venv.sample_actions(t))
        torch.cuda.synchronize()
        o = venv.obs.cpu().numpy()
        outs.append((o, venv.reward.cpu().numpy(), venv.success.cpu().numpy()))
        venv.close()
    o, r, s = outs[0]
    assert np.all(np.isfinite(o)) and np.abs(o).max() < 10.0
    assert np.array_equal(outs[0][0], outs[1][0])  # bitwise deterministic
    assert np.array_equal(r == 0.0, s.astype(bool) | (r == 0.0))
    assert set(np.unique(r)).issubset({-1.0, 0.0})


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaReachAO-v3"])
def test_two_wave_variant_matches_one_wave_shards(pg, env_id):
    """8192 envs in the wide layout launch the two-waves-per-SIMD build of the step kernel;
    two 4096-env shards (global ids 0.. and 4096..) launch the one-wave build.  Same global
    ids, same Philox actions and resets: the results agree bit for bit."""
    n = 8192
    big = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, lanes_per_env=16)
    parts = [pg.PandaVecEnv(env_id, num_envs=n // 2, device="cuda:0", seed=5, lanes_per_env=16,
                            env_id_offset=k * (n // 2)) for k in range(2)]
    for v in [big] + parts:
        v.reset_tensors()
    for t in range(12):
        big.step_tensors(big.sample_actions(t))
        for v in parts:
            v.step_tensors(v.sample_actions(t))
        got = torch.cat([v.obs for v in parts])
        assert torch.equal(got.view(torch.int32), big.obs.view(torch.int32)), t
        assert torch.equal(torch.cat([v.reward for v in parts]), big.reward), t
        assert torch.equal(torch.cat([v.truncated for v in parts]), big.truncated), t
    for v in [big] + parts:
        v.close()


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaPush-v3", "PandaPickAndPlace-v3", "PandaReachAO-v3"])
@pytest.mark.parametrize("n", [3, 67])
def test_ragged_batches_match_oracle(pg, oracle, env_id, n, lanes):
    """Batches that fill neither the 16-lane layout's 4-env waves nor the one-lane layout's 64-env
    waves: the envs of the last, partial wave step like every other -- three random steps from the
    same state against the oracle, every output row (observation, goals, reward, flags) checked,
    so a write past env n - 1 into the next output array would show."""
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=17, lanes_per_env=lanes)
    venv.reset_tensors(seed=17)
    ref = oracle.OracleVecEnv(venv._cfg, n)
    for t in range(3):
        _state_to_oracle(venv, ref)
        acts = venv.sample_actions(t).clone()
        venv.step_tensors(acts)
        ao = env_id == "PandaReachAO-v3"
        out = ref.step(acts.cpu().numpy(), margins=ao)
        obs, ag, dg, rew, succ = _gpu_out(venv)
        tr = venv.truncated.cpu().numpy()
        # ReachAO: a collision decision may differ only where the oracle's own margin sat at
        # rounding level (test_gpu_reach_ao.py, FLIP_MARGIN)
        same = tr == out["truncated"]
        if ao:
            assert np.all(same | (out["margin_abs"] < 1e-6))
        else:
            assert np.all(same)
        keep = same & (tr == 0)
        assert obs.shape == out["obs"].shape and np.all(np.isfinite(obs))
        assert np.abs(obs[keep, :3] - out["obs"][keep, :3]).max(initial=0.0) <= OBS_TOL
        assert np.abs(ag[keep] - out["ag"][keep]).max(initial=0.0) <= OBS_TOL
        assert np.array_equal(dg[keep], out["dg"][keep])
        assert np.array_equal(rew[keep], out["reward"][keep])
    venv.close()


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaPickAndPlace-v3", "PandaReachAO-v3"])
def test_single_env_robot_task_sim_views(pg, env_id):
    """`env.robot`, `env.task`, `env.sim` of the single-env wrapper (RobotTaskEnv's attributes,
    SURVEY.md 8b): read-only views that agree with the observation the step returned and with the
    device state."""
    env = pg.make(env_id)
    obs, _ = env.reset(seed=123)
    a = env.action_space.sample() * 0.0 + 0.3
    obs, _, _, _, info = env.step(a)
    o = obs["observation"]
    assert np.array_equal(env.robot.get_ee_position(), o[0:3])
    assert np.array_equal(env.robot.get_ee_velocity(), o[3:6])
    assert np.array_equal(np.concatenate([env.robot.get_obs(), env.task.get_obs()]), o)
    assert np.array_equal(env.task.get_achieved_goal(), obs["achieved_goal"])
    assert np.array_equal(env.task.goal.astype(np.float32), obs["desired_goal"])
    assert env.task.goal.dtype == np.float64
    st = env._vec.state()
    for j in range(7):
        assert env.robot.get_joint_angle(j) == float(st["q"][j, 0].item())
    assert env.robot.get_joint_angle(9) == 0.0 and env.robot.get_fingers_width() == 0.0
    assert bool(env.task.is_success(obs["achieved_goal"], env.task.goal)) == info["is_success"]
    assert env.sim.dt == pytest.approx(0.04) and env.sim.n_substeps == 20
    if env_id == "PandaReachAO-v3":
        assert env.task.obstacles.shape == (6, 3) and len(env.robot.get_obs()) == 20
    else:
        assert env.task.obstacles is None
    sid = env.sim.save_state()
    env.sim.restore_state(sid)
    env.sim.remove_state(sid)
    env.close()
