"""GPU parity of the contact scene (table / plane / cube, robot capsules) against the fp64 oracle.

Away from contact events the step is as well conditioned as the Reach step (errors ~1e-6).  At a
contact event the truncated projected Gauss-Seidel (50 sweeps, residual exit 1e-7) amplifies
rounding: the fp64 oracle itself moves the EE by up to 7e-5 in one step when its input state is
perturbed by 1e-7 relative (tools/diag_contacts.py, DESIGN.md "Contacts"), so an fp32 step cannot
be held to 1e-4 at every contact event and a free-running contact trajectory diverges
chaotically.  The bar is therefore set per step, from the same state: 99th percentile <= 1e-5 of
the EE and object positions, the 99.9th inside the restated algorithm's own fp32 evaluation, and
every sample <= 1e-3 under the default physics (round 6; rounds 4-5 let one sample in 2000 reach
1e-2 where the oracle itself moved as far under a rounding-level, 1e-7 relative, change of its
input); plus the physical invariants the oracle tests pin (test_oracle_contacts.py) checked on
the device.

Where the tool bar slides on the table (test_reach_with_table_contacts, the runtime-model friction
test) the step is worse conditioned since round 4 gave the tool bar its own lateral friction
(panda.py:69-70: mu 0.5 against the table instead of 0.25): from the same state the device's p99
went 2.4e-6 -> 2.9e-5 while the restated algorithm evaluated in fp32 (oracle/fp32_emul.cpp) moves
by 9.0e-5 -> 1.8e-4 (tools/gpu_table_drive.py, profiles/r04/table_drive.log).  Those tests hold
the device inside that fp32 envelope, from the same state, percentile for percentile (p99, p99.9),
instead of an absolute p99; the tool bar at mu 0.25 (through libpgx_rtmodel.so) keeps the
absolute 1e-5 bar.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from test_gpu_parity import OBS_TOL, _state_to_oracle  # noqa: E402


@pytest.fixture(scope="module")
def pg():
    import panda_gym_amd as pg

    pg.load_native()
    return pg


def _obs(venv):
    return (venv.obs.cpu().numpy(), venv.achieved_goal.cpu().numpy(), venv.desired_goal.cpu().numpy())


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaPickAndPlace-v3", "PandaPushJoints-v3"])
def test_object_reset_and_one_step_parity(pg, oracle, env_id, lanes):
    n = 256
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, lanes_per_env=lanes)
    venv.reset_tensors(seed=100)
    spec = pg.spec(env_id)
    for i in (0, 17, 255):   # host PCG64 draws (RobotTaskEnv.reset(seed)) injected exactly
        g, o = pg.seeded_reset(spec, 100 + i)
        st = venv.state()
        assert np.array_equal(st["goal"].cpu().numpy()[:, i], g)
        assert np.array_equal(st["object"].cpu().numpy()[:3, i], o.astype(np.float32))
    ref = oracle.OracleVecEnv(venv._cfg, n)
    for k in range(4):
        venv.step_tensors(venv.sample_actions(k))
    _state_to_oracle(venv, ref)
    acts = venv.sample_actions(9).clone()
    venv.step_tensors(acts)
    out = ref.step(acts.cpu().numpy())
    obs, ag, dg = _obs(venv)
    assert obs.shape[1] == out["obs"].shape[1] == (19 if "PickAndPlace" in env_id else 18)
    err = np.abs(obs - out["obs"])
    assert err[:, :3].max() <= OBS_TOL and err[:, 6:12].max() <= 10 * OBS_TOL
    assert np.abs(ag - out["ag"]).max() <= OBS_TOL
    assert np.array_equal(dg, out["dg"])
    venv.close()


OUTLIER = 1e-3   # per-step errors above this must be explained by the oracle's own sensitivity


def _one_step_errors(pg, oracle, env_id, n, steps, seed, actions=None, lanes=0, outliers=None, full=False,
                     over=None, envelope=None, pools=None, **kw):
    """Per step, from the device state copied into the oracle: |device - oracle| of the EE
    position (obs 0:3) and the achieved goal (EE or object position).  With ``outliers`` (a
    list), every sample above OUTLIER is recorded with its oracle input for _self_sensitivity.
    With ``envelope`` (a dict), the fp32 build of the oracle steps from the same state too and
    its deviation from the fp64 oracle lands in envelope["ee"], envelope["ag"].
    ``kw``: more PandaVecEnv arguments (sim_params, lib_path)."""
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=seed, lanes_per_env=lanes, full_manifold=full,
                          **kw)
    venv.reset_tensors(seed=seed)
    ref = oracle.OracleVecEnv(venv._cfg, n)
    r32 = None
    if envelope is not None:
        r32 = oracle.OracleVecEnv(venv._cfg, n, fp32=True)
        oracle.fp32_lib().pgxo_set_robot_budget(venv.robot_contact_budget() or -1)
        envelope["ee"], envelope["ag"] = [], []
    ee_err, ag_err = [], []
    n_obj = 4   # the object-scene slots ahead of the robot slots in the contact cache
    for t in range(steps):
        _state_to_oracle(venv, ref)
        saved = (ref.q.copy(), ref.qd.copy(), ref.goal.copy(), ref.obj.copy(), ref.elapsed.copy(),
                 ref.episode.copy())
        if actions is None:
            a = venv.sample_actions(t).clone()
        elif callable(actions):   # a policy of the device observation before the step
            a = torch.as_tensor(actions(venv.obs.cpu().numpy(), t), device="cuda:0")
        else:   # one action for every env, or one per env
            at = np.asarray(actions[t], np.float32)
            a = torch.as_tensor(at if at.ndim == 2 else np.repeat(at[None], n, 0), device="cuda:0")
        if r32 is not None:
            for k in ("q", "qd", "qc", "goal", "obj", "elapsed", "episode"):
                getattr(r32, k)[:] = getattr(ref, k)
        venv.step_tensors(a)
        out = ref.step(a.cpu().numpy())
        o32 = r32.step(a.cpu().numpy()) if r32 is not None else None
        obs, ag, dg = _obs(venv)
        if over is not None:   # envs whose last substep held more than 4 robot points
            over[0] += int(((venv.state()["contacts"][2 * n_obj::2] >= 0).sum(dim=0) > 4).sum().item())
        assert np.array_equal(venv.truncated.cpu().numpy(), out["truncated"]), t
        if out["truncated"].any():
            continue
        e_ee = np.abs(obs[:, :3] - out["obs"][:, :3]).max(axis=1)
        e_ag = np.abs(ag - out["ag"]).max(axis=1)
        ee_err.append(e_ee)
        ag_err.append(e_ag)
        if o32 is not None:
            envelope["ee"].append(np.abs(o32["obs"][:, :3] - out["obs"][:, :3]).max(axis=1))
            envelope["ag"].append(np.abs(o32["ag"] - out["ag"]).max(axis=1))
        if pools is not None and "manifolds" in venv.state():
            # Bullet's persistent manifolds after the step from the same state: the device's and the
            # oracle's pools hold the same points (count and row ids, in pool order)
            from oracle import oracle as orc

            dm = venv.state()["manifolds"].cpu().numpy()
            for i in range(n):
                cnt = int(dm[0, i])
                dk = dm[1:1 + cnt * orc.MAN_PT:orc.MAN_PT, i]
                rk = orc.pool(ref.obj[i])[:, orc.MP_KID]
                pools["env_steps"] = pools.get("env_steps", 0) + 1
                pools["points"] = pools.get("points", 0) + cnt
                if cnt != len(rk) or not np.array_equal(dk, rk.astype(np.float32)):
                    pools["mismatch"] = pools.get("mismatch", 0) + 1
        if outliers is not None:
            for i in np.nonzero(np.maximum(e_ee, e_ag) > OUTLIER)[0]:
                outliers.append({"t": t, "env": int(i), "err_ee": float(e_ee[i]), "err_ag": float(e_ag[i]),
                                 "state": tuple(x[i:i + 1].copy() for x in saved),
                                 "action": a.cpu().numpy()[i:i + 1].copy(),
                                 "ee": out["obs"][i, :3].copy(), "ag": out["ag"][i].copy(),
                                 # the restated algorithm in fp32 from the same state: how far it moves
                                 "f32_ee": float(np.abs(o32["obs"][i, :3] - out["obs"][i, :3]).max())
                                 if o32 is not None else 0.0,
                                 "f32_ag": float(np.abs(o32["ag"][i] - out["ag"][i]).max()) if o32 is not None else 0.0})
    final = {k: v.clone() for k, v in venv.state().items()}   # views die with the handle
    cfg = type(venv._cfg).from_buffer_copy(venv._cfg)
    keep = (venv._model, venv._params)   # cfg points into these
    venv.close()
    if outliers is not None:
        outliers.append((cfg, keep))
    if envelope is not None:
        envelope["ee"], envelope["ag"] = np.stack(envelope["ee"]), np.stack(envelope["ag"])
    return np.stack(ee_err), np.stack(ag_err), final


def _inside_envelope(name, dev, f32, pcts=(99, 99.9), floor=1e-5):
    """The device's per-step deviation from the fp64 oracle is at most the fp32 evaluation's of
    the restated algorithm from the same state, percentile for percentile -- or below ``floor``
    (the absolute p99 bar), where both sit at rounding level (joint control, no IK: device
    p99.9 3.6e-7 vs fp32 oracle 3.3e-7 on PickAndPlaceJoints) and their order is noise."""
    for p in pcts:
        d, f = float(np.percentile(dev, p)), float(np.percentile(f32, p))
        print(f"{name} p{p}: device {d:.2e} | fp32 oracle {f:.2e}")
        assert d <= max(f, floor), (name, p, d, f)


def _self_sensitivity(oracle, cfg, rec, trials=16, rel=1e-7, seed=0):
    """The oracle's own one-step response (max |ee|, |ag| change over ``trials``) to its input
    state perturbed by ``rel`` relative -- the fp32 rounding scale of the device state.  Half the
    trials at rel, half at 3 rel: the device state carries the rounding of every operation of the
    step before (a few fp32 ulps), not one."""
    c1 = type(cfg).from_buffer_copy(cfg)
    c1.n_envs = 1
    rng = np.random.default_rng(seed)
    d_ee = d_ag = 0.0
    for t in range(trials):
        r = oracle.OracleVecEnv(c1, 1)
        q, qd, goal, obj, el, ep = (x.copy() for x in rec["state"])
        rt = rel if t % 2 == 0 else 3.0 * rel
        pert = lambda x: x * (1.0 + rt * rng.standard_normal(x.shape))  # noqa: E731
        r.q[:], r.qd[:], r.goal[:], r.obj[:] = pert(q), pert(qd), goal, obj
        r.obj[:, :13] = pert(obj[:, :13])
        # the persistent manifold points are state the device holds in fp32 too: their positions,
        # normals, distances and impulses (not the ids)
        from oracle import oracle as orc

        npool = int(obj[0, orc.OBJ_MAN])
        for i in range(npool):
            b = orc.OBJ_MAN + 1 + i * orc.MAN_PT
            r.obj[:, b + 1:b + orc.MAN_PT] = pert(obj[:, b + 1:b + orc.MAN_PT])
        r.elapsed[:], r.episode[:] = el, ep
        o = r.step(rec["action"])
        d_ee = max(d_ee, float(np.abs(o["obs"][0, :3] - rec["ee"]).max()))
        d_ag = max(d_ag, float(np.abs(o["ag"][0] - rec["ag"]).max()))
    return d_ee, d_ag


def test_reach_with_table_contacts(pg, oracle, lanes):
    """Drive the EE into the table (a = -z, each env with its own small lateral offset, so the 64
    envs are 64 samples per step): the tool-bar contact holds it at z ~ 0.042."""
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.2, 0.2, (64, 3)).astype(np.float32)
    off[:, 2] = 0.0
    acts = [np.clip(np.array([0.3, -0.2, -1.0], np.float32) + off, -1, 1)] * 30
    outl, env = [], {}
    ee, ag, _ = _one_step_errors(pg, oracle, "PandaReach-v3", 64, 30, 3, acts, lanes=lanes, outliers=outl,
                                 envelope=env)
    print(f"\ntable contacts: EE error p99 {np.percentile(ee, 99):.2e} max {ee.max():.2e}")
    _inside_envelope("ee", ee, env["ee"])
    assert np.percentile(ee, 99) <= 1e-4 and ee.max() <= 1e-3, (np.percentile(ee, 99), ee.max())
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=64, device="cuda:0", seed=3, lanes_per_env=lanes)
    venv.reset_tensors(seed=3)
    for a in acts:   # one action per env
        venv.step_tensors(torch.tensor(a, dtype=torch.float32, device="cuda:0"))
    z = venv.obs[:, 2].cpu().numpy()
    assert z.min() > 0.035, z.min()
    venv.close()


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaPickAndPlaceJoints-v3"])
def test_random_policy_one_step_parity(pg, oracle, env_id, lanes):
    """p99 <= 1e-5 in both layouts, p99.9 inside the fp32 envelope (round 3: <= 1e-4; with the tool
    bar's friction of round 4 the one-lane Push EE p99.9 measured 1.1e-4 against the fp32 oracle's
    2.8e-4), and every sample <= 1e-3.  Rounds 4-5 allowed one sample per 2000 up to 1e-2 at a
    contact bifurcation the oracle itself shows under a 1e-7 relative perturbation of its input
    (one one-lane Push sample of 12544 reached 1.7e-3); since the cube meets the table's side walls
    (round 6) the largest is 7.6e-4 (profiles/r06/pytest_gpu_v26.log), and the bar is 1e-3."""
    outl, env = [], {}
    ee, ag, final = _one_step_errors(pg, oracle, env_id, 256, 50, 21, lanes=lanes, outliers=outl, envelope=env)
    cfg, _keep = outl.pop()
    for name, e, f in (("ee", ee, env["ee"]), ("object", ag, env["ag"])):
        print(f"\n{env_id} {name}: p99 {np.percentile(e, 99):.2e} p99.9 {np.percentile(e, 99.9):.2e} max {e.max():.2e}, "
              f"{int((e > OUTLIER).sum())} of {e.size} above {OUTLIER:g}")
        assert np.percentile(e, 99) <= 1e-5, (name, np.percentile(e, 99))
        _inside_envelope(name, e, f, pcts=(99.9,))
        assert e.max() <= OUTLIER, (name, e.max())   # (round 6: 1e-3, was 1e-2)
    assert len(outl) <= ee.size // 2000, len(outl)
    for rec in outl:
        s_ee, s_ag = _self_sensitivity(oracle, cfg, rec, trials=32)
        assert rec["err_ee"] <= OUTLIER or s_ee >= rec["err_ee"], (rec["t"], rec["env"], rec["err_ee"], s_ee)
        assert rec["err_ag"] <= OUTLIER or s_ag >= rec["err_ag"], (rec["t"], rec["env"], rec["err_ag"], s_ag)
    cube = final["object"].cpu().numpy()
    assert cube[2].min() > -0.4


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaPickAndPlace-v3"])
def test_full_manifold_random_policy_one_step_parity(pg, oracle, env_id):
    """PGX_CONTACTS_FULL (16 lanes, robot budget 12): the same per-step bars as the default
    budget (p99 <= 1e-5, p99.9 inside the fp32 envelope, every sample <= 1e-3) over a random-policy
    run in which envs hold more than 4 robot points (the extra rows in LDS), against the oracle at
    the same budget."""
    outl, over, env, pools = [], [0], {}, {}
    ee, ag, final = _one_step_errors(pg, oracle, env_id, 256, 50, 21, lanes=16, outliers=outl, full=True, over=over,
                                     envelope=env, pools=pools)
    cfg, _keep = outl.pop()
    assert over[0] > 0, "no env held more than 4 robot points"
    for name, e, f in (("ee", ee, env["ee"]), ("object", ag, env["ag"])):
        print(f"\n{env_id} {name}: p99 {np.percentile(e, 99):.2e} p99.9 {np.percentile(e, 99.9):.2e} max {e.max():.2e}, "
              f"{int((e > OUTLIER).sum())} of {e.size} above {OUTLIER:g}")
        assert np.percentile(e, 99) <= 1e-5, (name, np.percentile(e, 99))
        _inside_envelope(name, e, f, pcts=(99.9,))
        assert e.max() <= OUTLIER, (name, e.max())   # (round 6: 1e-3, was 1e-2)
    assert len(outl) <= ee.size // 2000, len(outl)
    # Bullet's persistent manifolds: device and oracle pools agree point for point after (almost)
    # every step from the same state; a merge / break decision taken at the fp32 rounding edge may
    # differ (at most 1 env-step in 1000)
    print(f"\nmanifold pools: {pools}")
    assert pools["points"] > 0 and pools.get("mismatch", 0) <= pools["env_steps"] // 1000, pools
    for rec in outl:
        # an outlier sits where the oracle itself moves as far under a rounding-level perturbation
        # of its input, or where the restated algorithm evaluated in fp32 does
        s_ee, s_ag = _self_sensitivity(oracle, cfg, rec, trials=64)
        s_ee, s_ag = max(s_ee, rec["f32_ee"]), max(s_ag, rec["f32_ag"])
        assert rec["err_ee"] <= OUTLIER or s_ee >= rec["err_ee"], (rec["t"], rec["env"], rec["err_ee"], s_ee)
        assert rec["err_ag"] <= OUTLIER or s_ag >= rec["err_ag"], (rec["t"], rec["env"], rec["err_ag"], s_ag)
    assert final["object"].cpu().numpy()[2].min() > -0.4


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaPickAndPlace-v3"])
def test_persistent_manifold_branches_under_a_scripted_push(pg, oracle, env_id):
    """Bullet's persistent manifolds where the arm works the cube (tests/scripted_push.py: per env a
    randomised approach that brings the tool bar and the hand down beside the cube and pushes it),
    from the same state every step, 256 envs x 40 steps: every branch of the oracle's manifold --
    addContactPoint's merge (replaceContactPoint), append and sortCachedPoints replacement,
    refreshContactPoints' removal past the threshold and by sliding -- runs at least 100 times
    (oracle diagnostics), the device and oracle pools agree point for point in >= 999 of 1000
    env-steps, and the per-step positions hold the contact steps' bars (below)."""
    import ctypes as C

    from scripted_push import ScriptedPush

    n, steps = 256, 40
    pol = ScriptedPush(n, seed=7, obj_col=6 if env_id == "PandaPush-v3" else 7)
    act = (lambda obs, t: pol(obs, t)) if env_id == "PandaPush-v3" else \
        (lambda obs, t: np.concatenate([pol(obs, t), np.zeros((n, 1), np.float32)], axis=1))
    diag = np.zeros(128, np.int64)
    oracle.lib().pgxo_diag_read(diag.ctypes.data_as(C.c_void_p), 1)
    outl, env, pools = [], {}, {}
    ee, ag, final = _one_step_errors(pg, oracle, env_id, n, steps, 3, actions=act, lanes=16, outliers=outl,
                                     full=True, envelope=env, pools=pools)
    cfg, _keep = outl.pop()
    oracle.lib().pgxo_diag_read(diag.ctypes.data_as(C.c_void_p), 1)
    branches = {"merge": int(diag[121]), "append": int(diag[122]), "replace": int(diag[123]),
                "drop_distance": int(diag[124]), "drop_slide": int(diag[125]), "pool_full": int(diag[120])}
    print(f"\n{env_id} scripted push: manifold branches {branches}, pools {pools}")
    for k in ("merge", "append", "replace", "drop_distance", "drop_slide"):
        assert branches[k] >= 100, branches
    assert pools.get("mismatch", 0) <= pools["env_steps"] // 1000, pools
    # the random-policy test's bars (p99 <= 1e-5, p99.9 inside the fp32 envelope), here over contact
    # steps almost throughout, and the fp32 envelope at p99 as well
    for name, e, f in (("ee", ee, env["ee"]), ("object", ag, env["ag"])):
        print(f"{name}: p99 {np.percentile(e, 99):.2e} p99.9 {np.percentile(e, 99.9):.2e} max {e.max():.2e}")
        _inside_envelope(name, e, f, pcts=(99, 99.9))
        assert np.percentile(e, 99) <= 1e-5, (name, np.percentile(e, 99))
        assert e.max() <= OUTLIER, (name, e.max())   # (round 6: 1e-3, was 1e-2)
    assert len(outl) <= ee.size // 2000, len(outl)
    for rec in outl:
        s_ee, s_ag = _self_sensitivity(oracle, cfg, rec, trials=64)
        s_ee, s_ag = max(s_ee, rec["f32_ee"]), max(s_ag, rec["f32_ag"])
        assert rec["err_ee"] <= OUTLIER or s_ee >= rec["err_ee"], (rec["t"], rec["env"], rec["err_ee"], s_ee)
        assert rec["err_ag"] <= OUTLIER or s_ag >= rec["err_ag"], (rec["t"], rec["env"], rec["err_ag"], s_ag)


def test_scripted_push_moves_cube_like_oracle(pg, oracle):
    """The oracle's scripted push (test_oracle_contacts.py) on the GPU: same cube motion."""
    n = 8
    venv = pg.PandaVecEnv("PandaPush-v3", num_envs=n, device="cuda:0", seed=0)
    venv.reset_tensors(goals=np.tile([0.0, 0.1, 0.02], (n, 1)), objects=np.tile([0.0, 0.0, 0.02], (n, 1)))
    ref = oracle.OracleVecEnv(venv._cfg, n)
    _state_to_oracle(venv, ref)
    acts = [[1, 0, 0]] * 2 + [[0, -1, 0]] * 2 + [[0, 0, -1]] * 5 + [[0, 1, 0]] * 6
    for a in acts:
        at = torch.tensor([a] * n, dtype=torch.float32, device="cuda:0")
        venv.step_tensors(at)
        ref.step(at.cpu().numpy())
    cube = venv.state()["object"].cpu().numpy()[:3].T
    assert np.linalg.norm(cube[0, :2]) > 0.02
    assert np.abs(cube - ref.obj[:, :3]).max() <= 2e-3
    venv.close()


def test_auto_reset_object_draws_match_oracle(pg, oracle):
    n = 64
    for env_id in ("PandaPush-v3", "PandaPickAndPlace-v3"):
        venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=77, max_episode_steps=2)
        venv.reset_tensors()
        ref = oracle.OracleVecEnv(venv._cfg, n)
        ref.reset()
        st = venv.state()
        assert np.array_equal(st["goal"].cpu().numpy().T, ref.goal)
        assert np.array_equal(st["object"].cpu().numpy()[:3].T, ref.obj[:, :3].astype(np.float32))
        for t in range(4):
            a = venv.sample_actions(t).clone()
            venv.step_tensors(a)
            ref.step(a.cpu().numpy())
        st = venv.state()
        assert np.array_equal(st["goal"].cpu().numpy().T, ref.goal)
        assert np.array_equal(st["object"].cpu().numpy()[:3].T, ref.obj[:, :3].astype(np.float32))
        venv.close()


def test_push_large_batch_properties(pg):
    n = 16384
    venv = pg.PandaVecEnv("PandaPickAndPlace-v3", num_envs=n, device="cuda:0", seed=3)
    venv.reset_tensors()
    for t in range(10):
        venv.step_tensors(venv.sample_actions(t))
    torch.cuda.synchronize()
    o = venv.obs.cpu().numpy()
    assert np.all(np.isfinite(o))
    cube = venv.state()["object"].cpu().numpy()
    assert cube[2].min() > -0.4 and cube[2].max() < 0.5      # above the plane, nothing launched
    assert np.abs(np.linalg.norm(cube[3:7], axis=0) - 1).max() < 1e-5
    venv.close()


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaPush-v3", "PandaPickAndPlaceJoints-v3"])
def test_layouts_agree_per_step(pg, env_id):
    """The 16-lane and the one-lane kernels restate the same step; from the same state (copied
    through the state views) one random-policy step agrees to fp32 rounding (summation order
    of the row reductions, scaled row units).  Per step, as in the oracle parity above.  Both at
    the one-lane layout's robot budget (4 points): the 16-lane default keeps Bullet's per-pair
    manifolds up to 8 / 12 points, which the one-lane kernels do not hold."""
    n = 512
    a = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=4, lanes_per_env=16, full_manifold=False)
    b = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=4, lanes_per_env=1)
    a.reset_tensors(seed=4)
    errs = []
    for t in range(20):
        for k, v in a.state().items():
            b.state()[k].copy_(v)
        act = a.sample_actions(t).clone()
        a.step_tensors(act)
        b.step_tensors(act)
        assert torch.equal(a.truncated, b.truncated)
        errs.append((a.obs[:, :3] - b.obs[:, :3]).abs().max(dim=1).values.cpu().numpy())
    e = np.concatenate(errs)
    assert np.percentile(e, 99) <= 1e-5 and e.max() <= 1e-3, (np.percentile(e, 99), e.max())
    a.close()
    b.close()


@pytest.mark.parametrize("env_id,lanes", [("PandaReach-v3", 16), ("PandaPush-v3", 16), ("PandaReach-v3", 1),
                                          ("PandaPush-v3", 1), ("PandaPickAndPlace-v3", 1)])
def test_speculative_limit_skip_is_exact(pg, monkeypatch, env_id, lanes):
    """Both layouts (substep_g, substep) solve contact substeps without the joint-limit rows
    when the motor-impulse bound alone keeps them idle, check at every limit-block position
    that they would have computed a zero impulse, and redo the solve with them otherwise.  The
    claim is bit-exact equality with the all-rows solve: compared here against PGX_PGS_MODE=2
    (never speculate) and PGX_PGS_MODE=3 (always redo), on table-contact steps from the same
    states."""
    n = 256
    runs = {}
    for mode in ("0", "2", "3"):
        monkeypatch.setenv("PGX_PGS_MODE", mode)
        v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=9, lanes_per_env=lanes)
        v.reset_tensors(seed=9)
        outs = []
        for t in range(25):
            a = torch.zeros((n, v.action_dim), device="cuda:0")
            a[:, 2] = -1.0                          # press the tool bar onto the table
            a[:, :2] = v.sample_actions(t)[:, :2]
            v.step_tensors(a)
            outs.append(torch.cat([v.obs, v.state()["qd"].T], 1).cpu().numpy().copy())
        runs[mode] = np.stack(outs)
        v.close()
    assert np.array_equal(runs["0"], runs["2"])
    assert np.array_equal(runs["0"], runs["3"])


@pytest.mark.parametrize("env_id,n", [("PandaPickAndPlace-v3", 16384), ("PandaReach-v3", 16384)])
def test_one_lane_speculative_solve_exact_at_full_size(pg, monkeypatch, env_id, n):
    """The one-lane layout's speculative limit-row solve at its benchmark batch, random policy:
    every step bit-identical to the all-rows solve (PGX_PGS_MODE=2)."""
    runs = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("PGX_PGS_MODE", mode)
        v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=4, lanes_per_env=1)
        v.reset_tensors()
        outs = []
        for t in range(12):
            v.step_tensors(v.sample_actions(t))
            outs.append(torch.cat([v.obs, v.state()["qd"].T], 1).cpu().numpy().copy())
        runs[mode] = np.stack(outs)
        v.close()
    assert np.array_equal(runs["0"], runs["2"])


@pytest.mark.parametrize("env_id,contacts,n", [("PandaReach-v3", True, 4096), ("PandaReach-v3", False, 4096),
                                               ("PandaReach-v3", True, 8192), ("PandaReachAO-v3", True, 4096),
                                               ("PandaReachAO-v3", True, 8192), ("PandaPush-v3", True, 4096)])
def test_partial_limit_rows_are_exact(pg, monkeypatch, env_id, contacts, n):
    """Waves holding an env near a joint limit solve with only that dof's limit pair (a slot
    lane mirrors the dof) and check the other pairs as the speculative solve does.  Under the
    random policy ~1.4 % of substeps take that path; the claim is bit-exact equality with the
    all-rows solve (PGX_PGS_MODE=2), per step, in the one- and two-waves-per-SIMD builds."""
    runs = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("PGX_PGS_MODE", mode)
        v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, lanes_per_env=16, contacts=contacts)
        v.reset_tensors()
        outs = []
        for t in range(24):
            v.step_tensors(v.sample_actions(t))
            outs.append(torch.cat([v.obs, v.state()["qd"].T], 1).cpu().numpy().copy())
        runs[mode] = np.stack(outs)
        v.close()
    assert np.array_equal(runs["0"], runs["2"])


@pytest.mark.parametrize("env_id", ["PandaPush-v3", "PandaPickAndPlace-v3"])
def test_object_kernel_two_waves_per_simd_exact(pg, monkeypatch, env_id):
    """The object kernel's two-waves-per-SIMD build (256 registers, taken above 4096 envs; its
    all-rows solve inline, with the limit rows' rhs' and lambda' in LDS, and no partial solve)
    equals the one-wave build bit for bit, in the default solve and with every substep forced
    through the all-rows solve (PGX_PGS_MODE=2) or through a redo after the speculative solve
    (PGX_PGS_MODE=3)."""
    runs = {}
    for wm in ("1", "2"):
        for mode in ("0", "2", "3"):
            monkeypatch.setenv("PGX_WAVES_PER_SIMD", wm)
            monkeypatch.setenv("PGX_PGS_MODE", mode)
            v = pg.PandaVecEnv(env_id, num_envs=4096, device="cuda:0", seed=9, lanes_per_env=16)
            v.reset_tensors()
            outs = []
            for t in range(16):
                v.step_tensors(v.sample_actions(t))
                outs.append(torch.cat([v.obs, v.state()["qd"].T], 1).cpu().numpy().copy())
            runs[(wm, mode)] = np.stack(outs)
            v.close()
    ref = runs[("1", "0")]
    for k, r in runs.items():
        assert np.array_equal(ref, r), k


@pytest.mark.parametrize("case", ["two_links_on_table", "link_on_cube"])
def test_contact_budget_cases_keep_all_points(pg, oracle, case, lanes):
    """The oracle's manifold-rule cases (test_oracle_contacts.py) on the device: an arm with the
    hand and a finger on the table (5 robot points) and the cube at the closed fingertips.  The
    full-manifold kernels (16 lanes, PGX_CONTACTS_FULL) keep every table point (budget 8) and hold
    Bullet's persistent manifolds for the cube pairs: one new point per pair and substep, merged
    into at most 4 per pair; the one-lane kernels keep their default budget of 4, the deepest
    candidates.  One substep per env step, so after a step the device's contact cache holds the
    rows of that substep: the oracle's feature ids; and the step matches."""
    from test_oracle_contacts import TWO_LINKS_ON_TABLE_REL_Q as TWO_LINKS_ON_TABLE_Q   # (the device's rule)

    n = 4
    env_id = "PandaReach-v3" if case == "two_links_on_table" else "PandaPush-v3"
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0, lanes_per_env=lanes, n_substeps=1,
                          full_manifold=lanes == 16)
    venv.reset_tensors()
    st = venv.state()
    if case == "two_links_on_table":
        q = torch.tensor(TWO_LINKS_ON_TABLE_Q, dtype=torch.float32, device="cuda:0")[:, None]
        st["q"][:] = q
        st["qc"][:] = q
        st["qd"].zero_()
    else:
        venv.step_tensors(torch.zeros((n, 3), dtype=torch.float32, device="cuda:0"))
        st["object"][0:3] = venv.obs[:, 0:3].T       # the cube at the fingertips, at rest
        st["object"][3:6] = 0.0
        st["object"][6] = 1.0
        st["object"][7:13] = 0.0
    st["contacts"][0::2] = -1.0
    st["contacts"][1::2] = 0.0
    budget = venv.robot_contact_budget()
    assert budget == (abi_budget(case) if lanes == 16 else 4)
    ref = oracle.OracleVecEnv(venv._cfg, n)
    _state_to_oracle(venv, ref)
    a = torch.zeros((n, 3), dtype=torch.float32, device="cuda:0")
    venv.step_tensors(a)
    out = ref.step(a.cpu().numpy())
    err = np.abs(venv.obs.cpu().numpy() - out["obs"])
    assert err[:, 0:3].max() <= OBS_TOL and err.max() <= 1e-3, (err[:, 0:3].max(), err.max())   # as above
    if case == "link_on_cube":
        assert err[:, 6:9].max() <= OBS_TOL                   # the cube position
    from oracle import oracle as orc

    def ids():
        cache = venv.state()["contacts"].cpu().numpy()
        dev_ids = cache[2 * orc.OBJECT_POINTS::2]            # robot slots, id order
        ref_ids = ref.obj[:, orc.OBJ_CACHE1:orc.OBJ_AO:2]
        out = []
        for e in range(n):
            d = dev_ids[:, e][dev_ids[:, e] >= 0]
            r = ref_ids[e][ref_ids[e] >= 0]
            assert np.array_equal(d, r.astype(np.float32)), (e, d, r)
            out.append(d)
        return out

    persistent = case == "link_on_cube" and lanes == 16
    for d in ids():
        if persistent:   # Bullet's manifolds start from each pair's one new point (slot 0)
            assert len(d) >= 2 and np.all((d - 32) % 16 == 0), d
        else:
            assert len(d) == min(budget, 5 if case == "two_links_on_table" else 8), d
    if persistent:       # and gain at most one point per pair per substep, up to 4
        most = 0
        for _ in range(6):
            _state_to_oracle(venv, ref)
            venv.step_tensors(a)
            out = ref.step(a.cpu().numpy())
            err = np.abs(venv.obs.cpu().numpy() - out["obs"])
            assert err[:, 0:3].max() <= OBS_TOL and err[:, 6:9].max() <= OBS_TOL, err.max()
            for d in ids():
                per_pair = np.bincount(((d - 32) // 16).astype(int))
                assert per_pair.max() <= 4
                most = max(most, int(per_pair.max()))
        assert most >= 2
    venv.close()


def test_object_kernel_points_past_the_register_budget(pg, oracle):
    """Envs holding more robot points than the object kernels keep in register (Delassus) rows --
    PGX_CGR_OBJ = 6; the rest are the reduction rows read from LDS -- are rare under the random
    policy (0.015 % of Push env-steps, profiles/r05/point_hist.log), so a test over a few hundred
    envs may never reach them: found in a 4096-env rollout (below), their pre-step states are
    copied into a small handle and stepped once against the oracle from the same state (an env's
    result does not depend on its wave mates).  Bar: 1e-4, or the oracle's own move under a
    rounding-level perturbation of its input (the one-step tests' outlier rule)."""
    from oracle import oracle as orc

    from scripted_push import ScriptedPush

    import os

    from panda_gym_amd import _native

    # With Bullet's relative breaking thresholds (round 6: 0.73 mm for the cube pairs, 2-7 mm for the
    # table's) an env almost never holds seven robot points -- none in 2048 envs x 50 steps of a rough
    # scripted push (oracle search) -- so the rows past the register budget are
    # driven here through the runtime-model library (the same kernels, the physics block read from the
    # handle) at a 5x gContactBreakingThreshold (0.1: every pair's threshold x 5), under a rough push.
    rt = os.path.join(os.path.dirname(_native.LIB_PATH), "libpgx_rtmodel.so")
    kw = dict(lib_path=rt, sim_params={"contact_distance": 0.1})
    n, keys = 4096, ("q", "qd", "qc", "goal", "object", "contacts", "elapsed", "episode", "manifolds")
    big = pg.PandaVecEnv("PandaPush-v3", num_envs=n, device="cuda:0", seed=5, **kw)
    big.reset_tensors()
    pol = ScriptedPush(n, seed=11, height=(0.036, 0.06), rough=True)   # the bar pressed on the table too
    found = []
    for t in range(100):
        st = big.state()
        pre = {k: st[k].clone() for k in keys}
        a = torch.as_tensor(pol(big.obs.cpu().numpy(), t), device="cuda:0")
        big.step_tensors(a)
        cnt = (big.state()["contacts"][2 * orc.OBJECT_POINTS::2] >= 0).sum(0)
        idx = torch.nonzero(cnt > 6).flatten()
        if len(idx):
            found.append(({k: pre[k][..., idx] for k in keys}, a[idx]))
        if sum(len(f[1]) for f in found) >= 12:
            break
    big.close()
    assert found, "no env held more than six robot points"
    acts = torch.cat([f[1] for f in found], dim=0)
    m = acts.shape[0]
    small = pg.PandaVecEnv("PandaPush-v3", num_envs=m, device="cuda:0", seed=5, **kw)
    small.reset_tensors()
    st = small.state()
    for k in keys:
        st[k].copy_(torch.cat([f[0][k] for f in found], dim=-1))
    st["elapsed"].zero_()   # no TimeLimit reset inside the compared step
    ref = oracle.OracleVecEnv(small._cfg, m)
    _state_to_oracle(small, ref)
    saved = (ref.q.copy(), ref.qd.copy(), ref.goal.copy(), ref.obj.copy(), ref.elapsed.copy(), ref.episode.copy())
    small.step_tensors(acts)
    out = ref.step(acts.cpu().numpy())
    held = (small.state()["contacts"][2 * orc.OBJECT_POINTS::2] >= 0).sum(0).cpu().numpy()
    assert held.max() > 6, held                        # the step ran rows past the register budget
    obs, ag = small.obs.cpu().numpy(), small.achieved_goal.cpu().numpy()
    e_ee = np.abs(obs[:, :3] - out["obs"][:, :3]).max(axis=1)
    e_ag = np.abs(ag - out["ag"]).max(axis=1)
    print(f"\n{m} envs past six robot points (held {held.tolist()}): max |ee| {e_ee.max():.2e}, |object| {e_ag.max():.2e}")
    cfg = type(small._cfg).from_buffer_copy(small._cfg)
    for i in np.nonzero(np.maximum(e_ee, e_ag) > 1e-4)[0]:
        rec = {"state": tuple(x[i:i + 1].copy() for x in saved), "action": acts.cpu().numpy()[i:i + 1],
               "ee": out["obs"][i, :3].copy(), "ag": out["ag"][i].copy()}
        s_ee, s_ag = _self_sensitivity(oracle, cfg, rec, trials=32)
        assert e_ee[i] <= 1e-2 and e_ag[i] <= 1e-2, (i, e_ee[i], e_ag[i])
        assert e_ee[i] <= max(1e-4, s_ee) and e_ag[i] <= max(1e-4, s_ag), (i, e_ee[i], s_ee, e_ag[i], s_ag)
    small.close()


def abi_budget(case):
    from panda_gym_amd import abi

    return abi.ROBOT_POINTS_ARM if case == "two_links_on_table" else abi.ROBOT_POINTS


def test_runtime_model_library_other_frictions(pg, oracle):
    """libpgx_rtmodel.so (make runtime-model: the same kernels reading the handle's physics block)
    runs physics parameters the default library refuses -- here other lateral frictions (the
    reference sets them per link through changeDynamics, panda.py:69-72 -> pybullet.py:880-892) --
    and matches the oracle at the same parameters, per step from the same state."""
    import os

    from panda_gym_amd import _native

    path = os.path.join(os.path.dirname(_native.LIB_PATH), "libpgx_rtmodel.so")
    assert os.path.exists(path), "libpgx_rtmodel.so is built by __graft_entry__.build()"
    over = {"friction": 0.36, "link_friction": [0.3] * 9 + [0.8, 0.8] + [0.3] * 5}
    with pytest.raises(pg.PgxError):
        pg.PandaVecEnv("PandaPush-v3", num_envs=8, device="cuda:0", sim_params=over)
    env = {}
    ee, ag, _ = _one_step_errors(pg, oracle, "PandaPush-v3", 256, 40, 21, full=True, sim_params=over, lib_path=path,
                                 envelope=env)
    q = lambda x, p: float(np.percentile(x, p))  # noqa: E731
    print(f"\nruntime model, frictions {over['friction']} / {over['link_friction'][9]}: EE p99 {q(ee, 99):.2e} "
          f"max {ee.max():.2e}, object p99 {q(ag, 99):.2e} max {ag.max():.2e}")
    # the tool bar at mu 0.8 sliding on the table: the fp32 envelope (module docstring)
    _inside_envelope("ee", ee, env["ee"])
    _inside_envelope("object", ag, env["ag"])
    assert q(ee, 99) <= 1e-4 and q(ag, 99) <= 1e-5 and ee.max() <= 1e-2 and ag.max() <= 1e-2


@pytest.mark.parametrize("lanes_", [16, 1])
def test_table_drive_tool_bar_mu_025_absolute_bar(pg, oracle, lanes_):
    """The table drive of test_reach_with_table_contacts with every link at mu 0.25 against the
    table (round 3's friction, through libpgx_rtmodel.so): the absolute bar, p99 <= 1e-5."""
    import os

    from panda_gym_amd import _native

    path = os.path.join(os.path.dirname(_native.LIB_PATH), "libpgx_rtmodel.so")
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.2, 0.2, (64, 3)).astype(np.float32)
    off[:, 2] = 0.0
    acts = [np.clip(np.array([0.3, -0.2, -1.0], np.float32) + off, -1, 1)] * 30
    ee, _, _ = _one_step_errors(pg, oracle, "PandaReach-v3", 64, 30, 3, acts, lanes=lanes_,
                                sim_params={"link_friction": [0.25] * 16}, lib_path=path)
    print(f"\ntool bar mu 0.25: EE error p99 {np.percentile(ee, 99):.2e} max {ee.max():.2e}")
    assert np.all(np.isfinite(ee))
    assert np.percentile(ee, 99) <= 1e-5 and ee.max() <= 1e-3, (np.percentile(ee, 99), ee.max())


@pytest.mark.parametrize("env_id,points", [("PandaReach-v3", 8), ("PandaReachJoints-v3", 8), ("PandaPush-v3", 12),
                                           ("PandaPickAndPlace-v3", 12), ("PandaReachAO-v3", 8)])
def test_default_handles_keep_the_per_pair_manifold_budget(pg, env_id, points):
    """The default handle (PandaVecEnv / make) runs Bullet's per-pair manifold budget: 8 robot
    points in Reach / ReachAO, 12 in Push / PickAndPlace (include/pgx.h); 4 on request or in the
    one-lane layout; none without contacts."""
    v = pg.PandaVecEnv(env_id, num_envs=64, device="cuda:0")
    assert v.robot_contact_budget() == points
    v.close()
    if env_id != "PandaReachAO-v3":
        v = pg.PandaVecEnv(env_id, num_envs=64, device="cuda:0", full_manifold=False)
        assert v.robot_contact_budget() == 4
        v.close()
        v = pg.PandaVecEnv(env_id, num_envs=64, device="cuda:0", lanes_per_env=1)
        assert v.robot_contact_budget() == 4
        v.close()
    env = pg.make(env_id)
    assert env._vec.robot_contact_budget() == points
    env.close()
    if env_id.startswith("PandaReach-"):
        v = pg.PandaVecEnv(env_id, num_envs=64, device="cuda:0", contacts=False)
        assert v.robot_contact_budget() == 0
        v.close()


@pytest.mark.parametrize("env_id,n", [("PandaPush-v3", 8), ("PandaPickAndPlace-v3", 8)])
def test_free_fall_known_answer_on_the_device(pg, oracle, env_id, n, lanes):
    """test/pybullet_test.py:56-64 on the device: a cube released at rest, clear of every body,
    has linear velocity [0, 0, -0.392] (atol 1e-3, the reference's) one env step later -- the
    floating-base path (gravity, base damping, semi-implicit update) -- and equals the fp64
    oracle's step to fp32 rounding.  (The reference's box has half extent 0.5; free fall does not
    depend on the size or mass.)"""
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=3, lanes_per_env=lanes)
    venv.reset_tensors()
    st = venv.state()
    xs = torch.linspace(-0.2, 0.1, n, device="cuda:0")
    st["object"][0].copy_(xs)
    st["object"][1].zero_()
    st["object"][2].fill_(1.0)                    # 1 m above the table, 0.5 m above the arm's reach
    st["object"][3:6].zero_()
    st["object"][6].fill_(1.0)
    st["object"][7:13].zero_()
    torch.cuda.synchronize()
    ref = oracle.OracleVecEnv(venv._cfg, n)
    _state_to_oracle(venv, ref)
    venv.step_tensors(torch.zeros((n, venv.action_dim), device="cuda:0"))
    out = ref.step(np.zeros((n, venv.action_dim), np.float32))
    k = 6 + (0 if venv.spec.block_gripper else 1) + 6   # obs: ee pos, ee vel, [width], pos, euler, linvel
    lin = venv.obs.cpu().numpy()[:, k:k + 3]
    assert np.allclose(lin, [0.0, 0.0, -0.392], atol=1e-3), lin
    assert np.abs(lin - out["obs"][:, k:k + 3]).max() <= 1e-5
    assert np.all(venv.obs.cpu().numpy()[:, k + 3:k + 6] == 0.0)
    venv.close()


@pytest.mark.parametrize("lanes", [16, 1])
def test_cube_at_the_table_side_wall_and_edge(pg, oracle, lanes):
    """Round 6: the cube's vertices meet the whole table box (its side walls too), in the kernels as in
    the oracle.  Eight cubes on the plane sliding into the table's +x wall and eight sliding over its
    +x edge (small offsets in y and yaw), the arm away: per step from the same state the device
    follows the oracle (the cube position to 1e-3 at p99, 2e-3 at most: below) and no cube is ever
    thrown (|v| <= 3.5 m/s, free fall from the top is 2.8)."""
    n = 16
    venv = pg.PandaVecEnv("PandaPush-v3", num_envs=n, device="cuda:0", seed=4, lanes_per_env=lanes)
    venv.reset_tensors()
    rng = np.random.default_rng(5)
    st = venv.state()
    obj = np.zeros((13, n), np.float32)
    for i in range(n):
        yaw = rng.uniform(-0.3, 0.3)
        obj[3:7, i] = (0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2))
        if i < 8:   # on the plane, sliding into the wall at x = 0.25
            obj[0:3, i] = (0.25 + 0.035 + 0.02 * rng.random(), rng.uniform(-0.2, 0.2), -0.38)
            obj[7:10, i] = (-0.6, 0.0, 0.0)
        else:       # on the top, sliding over the edge
            obj[0:3, i] = (0.2 + 0.02 * rng.random(), rng.uniform(-0.2, 0.2), 0.02)
            obj[7:10, i] = (0.8, 0.0, 0.0)
    st["object"].copy_(torch.as_tensor(obj, device="cuda:0"))
    st["contacts"][0::2] = -1.0
    st["contacts"][1::2] = 0.0
    if "manifolds" in st:
        st["manifolds"].zero_()
    ref = oracle.OracleVecEnv(venv._cfg, n)
    r32 = oracle.OracleVecEnv(venv._cfg, n, fp32=True)
    oracle.fp32_lib().pgxo_set_robot_budget(venv.robot_contact_budget() or -1)
    zero = torch.zeros((n, 3), dtype=torch.float32, device="cuda:0")
    errs, e32, vmax = [], [], 0.0
    for t in range(25):
        _state_to_oracle(venv, ref)
        for k in ("q", "qd", "qc", "goal", "obj", "elapsed", "episode"):
            getattr(r32, k)[:] = getattr(ref, k)
        venv.step_tensors(zero)
        ref.step(zero.cpu().numpy())
        r32.step(zero.cpu().numpy())
        ob = venv.state()["object"].cpu().numpy()
        errs.append(np.abs(ob[0:3].T - ref.obj[:, 0:3]).max(axis=1))
        e32.append(np.abs(r32.obj[:, 0:3] - ref.obj[:, 0:3]).max(axis=1))
        vmax = max(vmax, float(np.abs(ob[7:10]).max()))
        assert np.all(np.isfinite(ob)), t
    e, f = np.stack(errs), np.stack(e32)
    print(f"\nside wall / edge: cube position p99 {np.percentile(e, 99):.2e} max {e.max():.2e} (fp32 evaluation "
          f"{np.percentile(f, 99):.2e} / {f.max():.2e}), max |v| {vmax:.2f}")
    # At the wall the cube rests on the plane with its four bottom vertices at one depth and touches
    # the wall with two or more: six candidates for the object group's four rows (PGX_OBJECT_POINTS),
    # the deepest four of near-equal depths, so fp32 rounding picks another subset than the fp64
    # oracle's at the impact step (tools/gpu_wall_diag.py, profiles/r06/wall_diag.log: ids 4, 9, 10,
    # 11 on the device against 4, 8, 10, 11) and the step differs by a few 1e-4: the bar is 1e-3 at
    # p99 there, 2e-3 at most.
    assert np.percentile(e, 99) <= 1e-3 and e.max() <= 2e-3, (np.percentile(e, 99), e.max())
    assert vmax <= 3.5
    final = venv.state()["object"].cpu().numpy()
    assert np.all(final[0, :8] > 0.25 + 0.02 - 3e-3), final[0, :8]     # held by the wall
    assert np.all(final[0, 8:] > 0.25)                                # over the edge
    venv.close()
