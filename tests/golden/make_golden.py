"""Generate golden reward/success/goal fixtures from the reference's own numpy code.

Run in the build container only (the reference tree is not on the GPU box):
    python tests/golden/make_golden.py

* ``panda_gym/utils.py`` (numpy-only) is loaded by file path and its
  ``distance`` produces the expected distances; the two compute_reward lines
  of Reach/Push/PickAndPlace (reach.py:84-89) and the is_success line
  (reach.py:80-82, with np.bool_ for the removed np.bool8) are applied to them.
  Cases: the env-step call (float32 achieved goal vs float64 goal) and the
  HER call (float32 vs float32), random pairs plus rounding and threshold edges.
* Goal/object draws of ``RobotTaskEnv.reset(seed)`` (core.py:302: a fresh
  ``np.random.Generator(PCG64(SeedSequence(seed)))`` per reset) for the task
  samplers (reach.py:75-78, push.py:69-87, pick_and_place.py:65-85),
  reproduced with numpy's PCG64 (gymnasium 0.29 seeding.np_random).
"""
import importlib.util
import os

import numpy as np

REF = os.environ.get("PGX_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def load_ref_utils():
    spec = importlib.util.spec_from_file_location("ref_utils", os.path.join(REF, "panda_gym", "utils.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def reward_cases(utils, rng):
    thr = 0.05
    n = 4000
    g64 = rng.uniform([-0.15, -0.15, 0.0], [0.15, 0.15, 0.3], size=(n, 3))
    direc = rng.normal(size=(n, 3))
    direc /= np.linalg.norm(direc, axis=-1, keepdims=True)
    kinds = rng.integers(0, 4, size=n)
    radius = np.where(kinds == 0, rng.uniform(0, 0.2, size=n), 0.0)
    radius = np.where(kinds == 1, thr + rng.uniform(-3e-6, 3e-6, size=n), radius)   # threshold edge
    radius = np.where(kinds == 2, (np.floor(rng.uniform(0, 0.1, size=n) * 1e6) + 0.5) / 1e6, radius)  # rounding edge
    radius = np.where(kinds == 3, rng.uniform(0, 1e-6, size=n), radius)  # ~zero
    ag32 = (g64 + direc * radius[:, None]).astype(np.float32)
    ag32[:8] = g64[:8].astype(np.float32)  # exact-ish zero distance
    dg32 = g64.astype(np.float32)
    out = {"ag32": ag32, "g64": g64, "dg32": dg32, "thr": np.float64(thr)}
    # env-step path: distance(float32 ag, float64 goal) -> float64
    d64 = np.array([utils.distance(ag32[i], g64[i]) for i in range(n)])
    out["d_f32_f64"] = d64
    out["success_f32_f64"] = np.array(d64 < thr, dtype=np.bool_)
    out["sparse_f32_f64"] = -np.array(d64 > thr, dtype=np.float32)
    out["dense_f32_f64"] = -d64.astype(np.float32)
    # HER path: vectorised distance over float32 batches
    d32 = utils.distance(ag32, dg32)
    assert d32.dtype == np.float32
    out["d_f32_f32"] = d32
    out["sparse_f32_f32"] = -np.array(d32 > thr, dtype=np.float32)
    out["dense_f32_f32"] = -d32.astype(np.float32)
    return out


def goal_draws():
    seeds = [0, 1, 42, 12345, 6789, 794512, 2**31 - 1]
    reach, push, pnp = [], [], []
    for s in seeds:
        r = np.random.Generator(np.random.PCG64(np.random.SeedSequence(s)))
        reach.append(r.uniform(np.array([-0.15, -0.15, 0.0]), np.array([0.15, 0.15, 0.3])))
        r = np.random.Generator(np.random.PCG64(np.random.SeedSequence(s)))
        g = np.array([0.0, 0.0, 0.02]) + r.uniform(np.array([-0.15, -0.15, 0]), np.array([0.15, 0.15, 0]))
        o = np.array([0.0, 0.0, 0.02]) + r.uniform(np.array([-0.15, -0.15, 0]), np.array([0.15, 0.15, 0]))
        push.append(np.concatenate([g, o]))
        r = np.random.Generator(np.random.PCG64(np.random.SeedSequence(s)))
        noise = r.uniform(np.array([-0.15, -0.15, 0]), np.array([0.15, 0.15, 0.2]))
        if r.random() < 0.3:
            noise[2] = 0.0
        g = np.array([0.0, 0.0, 0.02]) + noise
        o = np.array([0.0, 0.0, 0.02]) + r.uniform(np.array([-0.15, -0.15, 0]), np.array([0.15, 0.15, 0]))
        pnp.append(np.concatenate([g, o]))
    return {"seeds": np.array(seeds, dtype=np.int64), "reach_goal": np.array(reach),
            "push_goal_obj": np.array(push), "pnp_goal_obj": np.array(pnp)}


def main():
    utils = load_ref_utils()
    rng = np.random.default_rng(20251015)
    np.savez(os.path.join(OUT, "reward_golden.npz"), **reward_cases(utils, rng))
    np.savez(os.path.join(OUT, "reset_golden.npz"), **goal_draws())
    print("wrote", os.listdir(OUT))


if __name__ == "__main__":
    main()
