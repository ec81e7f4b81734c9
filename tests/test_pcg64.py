"""CPU: the PCG64 arithmetic the device reset runs in its ``reset_rng="pcg64"`` mode, pinned
against numpy itself (gymnasium's seeding.np_random = Generator(PCG64(SeedSequence(seed))),
core.py:302), and the host records pgx_set_rng_streams takes.

The restatement below is the kernel's `pcg64_next64` / `pcg64_next_double` / `pcg64_next32` /
`pcg64_bounded` / `pcg64_interval` (csrc/pgx_kernels.hip) in Python integers: 128-bit LCG step with
numpy's PCG64 multiplier, XSL-RR output of the new state, (u >> 11) * 2^-53; next_uint32 hands out a
64-bit output's low half and keeps the high half (has_uint32 / uinteger); Generator.integers(4, 6)
by Lemire's bounded draw on next_uint32, Generator.shuffle of a list by random_interval."""
import numpy as np
import pytest

import panda_gym_amd as pg
from panda_gym_amd import abi

M128 = (1 << 128) - 1
M64 = (1 << 64) - 1
MULT = (0x2360ED051FC65DA4 << 64) | 0x4385DF649FCCF645


def _next64(rec):
    s = (rec[0] | (rec[1] << 64)) * MULT + (rec[2] | (rec[3] << 64))
    s &= M128
    rec[0], rec[1] = s & M64, s >> 64
    hi, lo = s >> 64, s & M64
    x, rot = hi ^ lo, hi >> 58
    return ((x >> rot) | (x << ((64 - rot) & 63))) & M64


def _next_double(rec):
    return (_next64(rec) >> 11) * (1.0 / 9007199254740992.0)


def _next32(rec):
    if rec[4]:
        v = rec[5]
        rec[4], rec[5] = 0, 0
        return v
    n = _next64(rec)
    rec[4], rec[5] = 1, n >> 32
    return n & 0xFFFFFFFF


def _bounded(rec, rng):
    excl = rng + 1
    m = _next32(rec) * excl
    left = m & 0xFFFFFFFF
    if left < excl:
        thr = (0xFFFFFFFF - rng) % excl
        while left < thr:
            m = _next32(rec) * excl
            left = m & 0xFFFFFFFF
    return m >> 32


def _interval(rec, mx):
    if mx == 0:
        return 0
    mask = mx
    for sh in (1, 2, 4, 8, 16):
        mask |= mask >> sh
    while True:
        v = _next32(rec) & mask
        if v <= mx:
            return v


@pytest.mark.parametrize("seed", [0, 1, 12345, 2 ** 40 + 7])
def test_restatement_matches_numpy_raw_and_doubles(seed):
    rec = [int(v) for v in pg.pcg64_records([seed])[0]]
    raw = np.random.PCG64(np.random.SeedSequence(seed)).random_raw(64)
    assert [_next64(rec) for _ in range(64)] == [int(v) for v in raw]
    rec = [int(v) for v in pg.pcg64_records([seed])[0]]
    gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    assert [_next_double(rec) for _ in range(16)] == list(gen.random(16))


def test_records_round_trip_and_continue_the_stream():
    recs = pg.pcg64_records([5, 6, 7])
    assert recs.dtype == np.uint64 and recs.shape == (3, abi.PCG64_WORDS)
    for sd, r in zip((5, 6, 7), recs):
        a = np.random.Generator(np.random.PCG64(np.random.SeedSequence(sd)))
        b = pg.pcg64_from_record(r)
        assert np.array_equal(a.random(9), b.random(9))
    # the record after k draws is the generator's own state after k draws
    g = np.random.Generator(np.random.PCG64(np.random.SeedSequence(11)))
    g.uniform(np.zeros(3), np.ones(3))
    rec = [int(v) for v in pg.pcg64_records([11])[0]]
    for _ in range(3):
        _next64(rec)
    assert rec == [int(v) for v in pg.pcg64_record(g)]


@pytest.mark.parametrize("seed", [0, 3, 77, 2024, 2 ** 33 + 5])
def test_uint32_draws_integers_and_shuffle_match_numpy(seed):
    """ReachAO.reset's integer draws (set_random_num_obs, reach_ao.py:1062-1082): integers(4, 6) and
    shuffle of the 6 obstacle names, after some doubles; the half-used 64-bit output carried in the
    record (has_uint32, uinteger) into the next reset's draws, as numpy carries it."""
    gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    rec = [int(v) for v in pg.pcg64_records([seed])[0]]
    for rnd in range(6):
        k = 5 + 3 * rnd
        assert [_next_double(rec) for _ in range(k)] == list(gen.random(k))
        n = int(gen.integers(4, 6))
        assert n == 4 + _bounded(rec, 1)
        keys = list(range(6))
        gen.shuffle(keys)
        perm = list(range(6))
        for j in range(5, 0, -1):
            r = _interval(rec, j)
            perm[j], perm[r] = perm[r], perm[j]
        assert perm == keys
        assert rec == [int(v) for v in pg.pcg64_record(gen)]
    # a record with the cached half round-trips through pcg64_from_record
    g2 = pg.pcg64_from_record(np.array(rec, dtype=np.uint64))
    assert int(g2.integers(0, 1000)) == int(gen.integers(0, 1000))


def test_reach_ao_reset_draw_order_from_the_record():
    """The device ReachAO reset's draws from a record (kernel ao_reset: hollow sphere = uniform phi,
    theta, r^3; obstacle coin random(); integers; shuffle) consume the stream exactly as the host
    sampler reach_ao.reset_draws does with numpy's Generator: same record after each reset."""
    from panda_gym_amd import reach_ao
    from panda_gym_amd.envs import _ao_geometry

    geom = _ao_geometry(tuple(pg.spec("PandaReachAO-v3").base_pos))
    for seed in (1, 42, 1000):
        gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        rec = [int(v) for v in pg.pcg64_records([seed])[0]]
        for _ in range(3):
            trace = []
            reach_ao.reset_draws(gen, geom, trace=trace)
            for kind, arg in trace:
                if kind == "double":
                    for _k in range(arg):
                        _next_double(rec)
                elif kind == "integers":
                    _bounded(rec, 1)
                else:
                    for j in range(5, 0, -1):
                        _interval(rec, j)
            assert rec == [int(v) for v in pg.pcg64_record(gen)]


@pytest.mark.parametrize("env_id", ["PandaReach-v3", "PandaPush-v3", "PandaPickAndPlace-v3"])
def test_task_draws_is_the_seeded_reset_and_the_device_order(env_id):
    """task_draws(spec, Generator(seed)) == seeded_reset(spec, seed); and the device's draw order
    (goal noise 0-2, PickAndPlace's z coin, object noise; kernel reset_env) from the restatement
    reproduces it bit for bit, for two consecutive resets of one stream."""
    sp = pg.spec(env_id)
    for seed in (3, 99, 2024):
        g0, o0 = pg.seeded_reset(sp, seed)
        gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        rec = [int(v) for v in pg.pcg64_records([seed])[0]]
        for rnd in range(2):
            g, o = pg.task_draws(sp, gen)
            if rnd == 0:
                assert np.array_equal(g, g0) and (o is None or np.array_equal(o, o0))
            lo, hi = sp.goal_bounds()
            noise = [lo[c] + ((hi[c] - lo[c]) * _next_double(rec)) for c in range(3)]
            half = abi.OBJECT_SIZE / 2
            if sp.task == abi.TASK_PICK_AND_PLACE and _next_double(rec) < 0.3:
                noise[2] = 0.0
            off = [0.0, 0.0, 0.0] if sp.task == abi.TASK_REACH else [0.0, 0.0, half]
            assert np.array_equal(g, np.array([off[c] + noise[c] for c in range(3)]))
            if sp.task != abi.TASK_REACH:
                olo, ohi = sp.obj_bounds()
                obj = [[0.0, 0.0, half][c] + (olo[c] + ((ohi[c] - olo[c]) * _next_double(rec))) for c in range(3)]
                assert np.array_equal(o, np.array(obj))
