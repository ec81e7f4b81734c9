"""GPU parity of the device HER replay ring (pgx_her.hip) against the numpy oracle (oracle/her.py).

Everything here is integer/index work or float32 copies plus the float32
compute_reward: the bar is bit-exact (slots, envs, goal slots, episode arrays,
every copied row, relabelled rewards).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

FIELDS = ["obs", "achieved_goal", "desired_goal", "action", "reward", "next_obs", "next_achieved_goal",
          "next_desired_goal", "done", "slot", "env", "goal_slot"]


@pytest.fixture(scope="module")
def her_mod():
    import panda_gym_amd.her as her

    return her


def _pair(her_mod, N, C, od, ad, strategy="future", reward_type="sparse", seed=5, n_sampled_goal=4):
    from oracle import her as H

    buf = her_mod.HerReplayBuffer(C * N, device="cuda:0", n_envs=N, obs_dim=od, action_dim=ad,
                                  goal_selection_strategy=strategy, reward_type=reward_type, seed=seed,
                                  n_sampled_goal=n_sampled_goal)
    orc = H.HerOracle(N, C, od, ad, reward_type=0 if reward_type == "sparse" else 1,
                      strategy=her_mod.STRATEGIES[strategy], her_ratio=buf.her_ratio, seed=seed)
    return buf, orc


def _feed(buf, orc, steps, rng, min_len=2, max_len=11):
    N, od, ad = orc.N, orc.od, orc.ad
    left = rng.integers(min_len, max_len + 1, N)
    for t in range(steps):
        left -= 1
        done = (left == 0).astype(np.uint8)
        left[done == 1] = rng.integers(min_len, max_len + 1, int(done.sum()))
        timeout = (done & (rng.random(N) < 0.5)).astype(np.uint8)
        f = lambda *s: rng.standard_normal((N,) + s).astype(np.float32)  # noqa: E731
        # goals on a 0.05-scale so sparse rewards hit both sides of the threshold
        args = [f(od), f(3) * 0.05, f(3) * 0.05, f(ad), f(), f(od), f(3) * 0.05, f(3) * 0.05, done, timeout]
        orc.add(*args)
        buf.add_tensors(*args)


def _compare(buf, orc, B, draw):
    got = buf.sample_raw(B, draw=draw)
    want = orc.sample(B, draw)
    for k in FIELDS:
        g = got[k].cpu().numpy()
        w = want[k]
        assert g.shape == w.shape, k
        assert np.array_equal(g.view(np.uint32) if g.dtype == np.float32 else g,
                              w.view(np.uint32) if w.dtype == np.float32 else w), k
    s, l, _ = buf._arrays()
    assert np.array_equal(s.cpu().numpy(), orc.ep_start)
    assert np.array_equal(l.cpu().numpy(), orc.ep_length)


@pytest.mark.parametrize("steps", [12, 40, 97])
def test_sample_bit_exact_vs_oracle(her_mod, steps):
    rng = np.random.default_rng(steps)
    buf, orc = _pair(her_mod, N=64, C=29, od=19, ad=4)
    _feed(buf, orc, steps, rng)
    for draw in range(3):
        _compare(buf, orc, 4099, draw)
    buf.close()


@pytest.mark.parametrize("variant", ["default", "two_pass", "spb64"])
@pytest.mark.parametrize("od,ad", [(19, 4), (18, 3), (56, 7)])
def test_both_sample_kernels_bit_exact(her_mod, monkeypatch, od, ad, variant):
    """libpgx samples records of <= 16 float4 columns with the single-read kernel (sample_kernel_reg)
    and wider ones (ReachAO's 56-float observation) with the two-pass kernel; PGX_HER_TWO_PASS
    forces the latter, PGX_HER_SPB=64 the single-read kernel's 64-samples-per-block build.  All
    bit-exact against the restatement at PickAndPlace's, Push's and ReachAO's dimensions."""
    env = {"two_pass": ("PGX_HER_TWO_PASS", "1"), "spb64": ("PGX_HER_SPB", "64")}
    if variant in env:
        monkeypatch.setenv(*env[variant])
    rng = np.random.default_rng(od)
    buf, orc = _pair(her_mod, N=48, C=23, od=od, ad=ad)
    _feed(buf, orc, 60, rng)
    for draw in range(2):
        _compare(buf, orc, 2053, draw)
    buf.close()


@pytest.mark.parametrize("strategy,reward_type", [("final", "sparse"), ("episode", "dense"), ("future", "dense")])
def test_strategies_and_dense_reward(her_mod, strategy, reward_type):
    rng = np.random.default_rng(7)
    buf, orc = _pair(her_mod, N=33, C=16, od=6, ad=3, strategy=strategy, reward_type=reward_type)
    _feed(buf, orc, 50, rng)
    _compare(buf, orc, 1000, 11)
    buf.close()


def test_her_ratio_edges(her_mod):
    """n_sampled_goal=0 -> her_ratio 0 (no relabelling); odd batch sizes split like int(her_ratio*B)."""
    rng = np.random.default_rng(3)
    buf, orc = _pair(her_mod, N=8, C=12, od=6, ad=3, n_sampled_goal=0)
    _feed(buf, orc, 30, rng)
    _compare(buf, orc, 1, 0)
    _compare(buf, orc, 777, 1)
    buf.close()


def test_sample_before_first_episode_raises(her_mod):
    buf, orc = _pair(her_mod, N=4, C=8, od=6, ad=3)
    _feed(buf, orc, 1, np.random.default_rng(0), min_len=5, max_len=5)
    with pytest.raises(RuntimeError):
        buf.sample(16)
    buf.close()


def test_sb3_surface_and_vec_env_feed(her_mod):
    """add_from_vec_env over an auto-resetting PandaReach rollout: relabelled rewards equal
    env.compute_reward(next_achieved_goal, desired_goal); terminal next_obs; SB3 shapes."""
    import panda_gym_amd as pg

    N = 256
    venv = pg.PandaVecEnv("PandaReach-v3", num_envs=N, device="cuda:0", seed=1, max_episode_steps=10)
    venv.reset_tensors()
    buf = her_mod.HerReplayBuffer(1000 * N, env=venv, device="cuda:0", seed=2)
    assert buf.buffer_size == 1000 and abs(buf.her_ratio - 0.8) < 1e-12
    for t in range(25):
        obs = {k: v.clone() for k, v in venv._obs_dict().items()}
        a = venv.sample_actions(t).clone()
        venv.step_tensors(a)
        buf.add_from_vec_env(venv, obs, a)
        if t == 9:
            terminal = venv.terminal_obs.clone()
            assert bool(venv.truncated.bool().all())
    assert buf.size() == 25 and buf.pos == 25 and not buf.full
    s = buf.sample(4096)
    assert s.rewards.shape == (4096, 1) and s.dones.shape == (4096, 1)
    assert s.observations["observation"].shape == (4096, venv.obs_dim)
    rew = venv.compute_reward(s.next_observations["achieved_goal"], s.observations["desired_goal"])
    nbv = int(0.8 * 4096)
    assert torch.equal(rew[-nbv:], s.rewards[-nbv:, 0])
    # only the 20 transitions of the two finished episodes are valid; time-limit ends are not dones
    assert int((buf.ep_length > 0).sum()) == 20 * N
    assert float(s.dones.abs().sum()) == 0.0
    # next_obs of the last transition of an episode is the terminal observation, not the reset one
    r = buf.sample_raw(8192)
    last = r["slot"] == 9
    assert int(last.sum()) > 0
    assert torch.equal(r["next_obs"][last], terminal[r["env"][last].long()])
    assert torch.equal(r["next_achieved_goal"][last], terminal[r["env"][last].long()][:, :3])
    venv.close()
    buf.close()


def test_full_size_properties(her_mod):
    """C4 sizes (16384 envs x 50-step episodes, B = 2^20): invariants on device."""
    N, C, od, ad = 16384, 64, 19, 4
    buf = her_mod.HerReplayBuffer(C * N, device="cuda:0", n_envs=N, obs_dim=od, action_dim=ad, seed=9)
    g = torch.Generator(device="cuda:0").manual_seed(0)
    dev = torch.device("cuda:0")
    for t in range(100):  # two episodes of 50, the second wraps the ring
        done = torch.full((N,), 1 if t % 50 == 49 else 0, dtype=torch.uint8, device=dev)
        r = lambda *s: torch.randn(*s, generator=g, device=dev)  # noqa: E731
        buf.add_tensors(r(N, od), r(N, 3) * 0.05, r(N, 3) * 0.05, r(N, ad), r(N), r(N, od), r(N, 3) * 0.05,
                        r(N, 3) * 0.05, done, done)
    B = 1 << 20
    s = buf.sample_raw(B)
    s2 = buf.sample_raw(B, draw=buf._draw - 1)
    for k in FIELDS:
        assert torch.equal(s[k], s2[k]), k     # a sample is a pure function of (seed, draw, contents)
    l = buf.ep_length
    assert int((l > 0).sum()) == 50 * N      # first episode overwritten by the wrap, second valid
    nbv = int(0.8 * B)
    v = slice(B - nbv, B)
    st = buf.ep_start.long()
    slot, env, gs = s["slot"].long(), s["env"].long(), s["goal_slot"].long()
    start = st[slot, env]
    t_rel = (slot - start) % C
    g_rel = (gs[v] - start[v]) % C
    assert bool((g_rel >= t_rel[v]).all()) and bool((g_rel < 50).all())
    assert bool((s["goal_slot"][: B - nbv] == -1).all())
    rew = torch.empty(nbv, device=dev)
    import ctypes as C_
    lib = buf.lib
    ag = s["next_achieved_goal"][v].contiguous()
    dg = s["desired_goal"][v].contiguous()
    assert lib.pgx_compute_reward(C_.c_void_p(ag.data_ptr()), C_.c_void_p(dg.data_ptr()), C_.c_int64(nbv), 0,
                                  C_.c_double(0.05), C_.c_void_p(rew.data_ptr()), buf._stream()) == 0
    assert torch.equal(rew, s["reward"][v])
    assert bool((s["done"] == 0).all())      # every episode end here is a time-out
    buf.close()


def test_vec_env_feed_terminated_episodes_use_terminal_obs(her_mod):
    """terminate_on_success (ReachAO): a successful transition is stored with the terminal
    next_obs / next_achieved_goal, not the auto-reset episode's (SB3 _store_transition takes
    infos["terminal_observation"] of every done env)."""
    import panda_gym_amd as pg
    from oracle.oracle import fk

    N = 64
    venv = pg.PandaVecEnv("PandaReachAO-v3", num_envs=N, device="cuda:0", seed=1)
    com, _, _ = fk(venv._cfg.model.contents, np.array(pg.abi.NEUTRAL_Q[:7]))
    far = np.tile(np.array([99.9, 99.9, -99.9]), (N, 6, 1))
    venv.reset_tensors(goals=np.tile(com[11] + 0.01, (N, 1)), objects=far)
    buf = her_mod.HerReplayBuffer(16 * N, env=venv, device="cuda:0", seed=2)
    obs = {k: v.clone() for k, v in venv._obs_dict().items()}
    a = torch.zeros((N, 7), device="cuda:0")
    venv.step_tensors(a)
    assert bool(venv.terminated.bool().all()) and not bool(venv.truncated.bool().any())
    tag, tobs = venv.terminal_ag.clone(), venv.terminal_obs.clone()
    assert not torch.equal(tag, venv.achieved_goal)              # the reset moved the goal / pose
    buf.add_from_vec_env(venv, obs, a)
    r = buf.sample_raw(4096)
    e = r["env"].long()
    assert bool((r["slot"] == 0).all())
    assert torch.equal(r["next_achieved_goal"], tag[e])
    assert torch.equal(r["next_obs"], tobs[e])
    assert bool((r["done"] == 1).all())                         # terminated, not a time-out
    venv.close()
    buf.close()
