"""CPU tests of the HER oracle (oracle/her.py): Philox known answers, SB3 episode
bookkeeping against an independent episode tracker, "future" goal invariants."""
import numpy as np
import pytest

from oracle import her as H

# Random123 philox4x32-10 known-answer vectors (kat_vectors, Salmon et al. SC'11)
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_known_answers(oracle, ctr, key, want):
    got = H.philox4x32_10(*[np.array([c], np.uint64) for c in ctr], key[0], key[1])
    assert tuple(int(x[0]) for x in got) == want
    assert tuple(oracle.philox(ctr, key)) == want      # the C oracle (env resets/actions) agrees


def _fill(orc: H.HerOracle, steps: int, rng, min_len=3, max_len=9):
    """Random transitions with random episode lengths; returns per-env episode (start_t, end_t) lists."""
    N, od, ad = orc.N, orc.od, orc.ad
    left = rng.integers(min_len, max_len + 1, N)
    eps = [[] for _ in range(N)]
    cur = np.zeros(N, np.int64)
    for t in range(steps):
        left -= 1
        done = (left == 0).astype(np.uint8)
        timeout = (done & (rng.random(N) < 0.5)).astype(np.uint8)
        f = lambda *s: rng.standard_normal((N,) + s).astype(np.float32)  # noqa: E731
        orc.add(f(od), f(3), f(3), f(ad), f(), f(od), f(3) * 0.1, f(3), done, timeout)
        for e in np.flatnonzero(done):
            eps[e].append((cur[e], t + 1))
            cur[e] = t + 1
            left[e] = rng.integers(min_len, max_len + 1)
    return eps


@pytest.mark.parametrize("steps", [5, 23, 61, 150])
def test_episode_bookkeeping_matches_tracker(steps):
    """ep_length > 0 exactly on transitions of finished episodes none of whose slots was overwritten."""
    rng = np.random.default_rng(steps)
    C, N = 17, 6
    orc = H.HerOracle(N, C, 4, 2)
    eps = _fill(orc, steps, rng)
    want = np.zeros((C, N), np.int64)
    for e in range(N):
        for s, t in eps[e]:
            if s >= steps - C:       # still entirely in the ring
                for k in range(s, t):
                    want[k % C, e] = t - s
    assert np.array_equal(orc.ep_length, want)


@pytest.mark.parametrize("strategy", [H.FUTURE, H.FINAL, H.EPISODE])
def test_virtual_goals_come_from_the_same_episode(strategy):
    rng = np.random.default_rng(1)
    C, N = 23, 8
    orc = H.HerOracle(N, C, 5, 3, strategy=strategy)
    _fill(orc, 70, rng)
    B = 2000
    s = orc.sample(B, draw=3)
    nbv = int(0.8 * B)
    real, virt = slice(0, B - nbv), slice(B - nbv, B)
    assert np.all(s["goal_slot"][real] == -1) and np.all(s["goal_slot"][virt] >= 0)
    slot, env, gs = s["slot"][virt], s["env"][virt], s["goal_slot"][virt]
    start, length = orc.ep_start[slot, env], orc.ep_length[slot, env]
    t, tg = (slot - start) % C, (gs - start) % C
    assert np.all(tg < length)
    if strategy == H.FUTURE:
        assert np.all(tg >= t)
    if strategy == H.FINAL:
        assert np.all(tg == length - 1)
    assert np.array_equal(orc.ep_start[gs, env], start)   # same episode
    assert np.array_equal(s["desired_goal"][virt], orc.next_ag[gs, env])
    assert np.array_equal(s["next_desired_goal"][virt], orc.next_ag[gs, env])
    want = H.compute_reward_f32(orc.next_ag[slot, env], orc.next_ag[gs, env], 0)
    assert np.array_equal(s["reward"][virt].view(np.uint32), want.view(np.uint32))
    # real rows keep the stored goal/reward; dones mask time-outs
    rs, re = s["slot"][real], s["env"][real]
    assert np.array_equal(s["reward"][real], orc.reward[rs, re])
    assert np.array_equal(s["done"][real], (orc.done[rs, re] * (1 - orc.timeout[rs, re])).astype(np.float32))
    assert np.all(orc.ep_length[s["slot"], s["env"]] > 0)


def test_uniform_over_valid_transitions():
    rng = np.random.default_rng(2)
    orc = H.HerOracle(4, 13, 2, 2)
    _fill(orc, 40, rng)
    nv = int((orc.ep_length > 0).sum())
    B = 200_000
    s = orc.sample(B, draw=0)
    counts = np.bincount(s["slot"] * 4 + s["env"], minlength=13 * 4)
    valid = (orc.ep_length > 0).reshape(-1)
    assert np.all(counts[~valid] == 0)
    exp = B / nv
    assert np.all(np.abs(counts[valid] - exp) < 6 * np.sqrt(exp))


def test_sample_before_first_episode_raises():
    orc = H.HerOracle(2, 5, 2, 2)
    z = np.zeros((2, 3), np.float32)
    orc.add(np.zeros((2, 2), np.float32), z, z, np.zeros((2, 2), np.float32), np.zeros(2, np.float32),
            np.zeros((2, 2), np.float32), z, z, np.zeros(2, np.uint8), np.zeros(2, np.uint8))
    with pytest.raises(RuntimeError):
        orc.sample(4, 0)


def test_reward_matches_reference_golden():
    """The relabel reward is the reference's compute_reward (tests/golden/reward_golden.npz)."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "reward_golden.npz"))
    ag, dg = g["ag32"], g["dg32"]
    for rt, name in ((0, "sparse_f32_f32"), (1, "dense_f32_f32")):
        got = H.compute_reward_f32(ag, dg, rt)
        assert np.array_equal(got.view(np.uint32), g[name].view(np.uint32)), name


def test_episode_as_long_as_the_ring_is_never_valid():
    """SB3 edge case kept: an episode of exactly buffer_size transitions ends at pos == start,
    _compute_episode_length writes nothing, so it is never sampled."""
    orc = H.HerOracle(2, 6, 2, 2)
    z = np.zeros((2, 3), np.float32)
    for t in range(6):
        d = np.full(2, int(t == 5), np.uint8)
        orc.add(np.zeros((2, 2), np.float32), z, z, np.zeros((2, 2), np.float32), np.zeros(2, np.float32),
                np.zeros((2, 2), np.float32), z, z, d, d)
    assert not np.any(orc.ep_length > 0)
