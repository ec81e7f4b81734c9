"""CPU: the PCG64 arithmetic the device reset runs in its ``reset_rng="pcg64"`` mode, pinned
against numpy itself (gymnasium's seeding.np_random = Generator(PCG64(SeedSequence(seed))),
core.py:302), and the host records pgx_set_rng_streams takes.

The restatement below is the kernel's `pcg64_next_double` (csrc/pgx_kernels.hip) in Python
integers: 128-bit LCG step with numpy's PCG64 multiplier, XSL-RR output of the new state,
(u >> 11) * 2^-53."""
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
    assert recs.dtype == np.uint64 and recs.shape == (3, 4)
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
    st = g.bit_generator.state["state"]
    assert rec == [st["state"] & M64, st["state"] >> 64, st["inc"] & M64, st["inc"] >> 64]


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
