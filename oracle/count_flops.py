"""TEST INFRASTRUCTURE ONLY: algorithmic FLOPs per env-step, op-counted in the fp64 oracle.

SURVEY.md §8d: "the exact count to be op-counted in the CPU restatement and frozen as a
fixture constant".  Runs the operation-counting build of the oracle (oracle/flops_count.cpp:
pgx_oracle.c with every double replaced by a counting type) over the benchmark's workload --
device-Philox random actions U[-1,1) from the start of an episode, auto-reset included -- for
each BASELINE config, and writes the per-env-step means (total and per phase) to
tests/golden/flops_per_env_step.json, which bench.py reads for the VALU roofline and
tests/test_flops.py re-derives.

    python oracle/count_flops.py [--envs 256] [--steps 100]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden", "flops_per_env_step.json")

# (key, env id, contacts, seed): the bench's legs (bench.py main leg seed 0, task legs seed 1)
CONFIGS = [
    ("reach_table", "PandaReach-v3", True, 0),          # configs[1], the headline (table scene)
    ("reach_no_table", "PandaReach-v3", False, 1),      # configs[1] worded without contacts
    ("push", "PandaPush-v3", True, 1),                  # configs[2]
    ("pick_and_place", "PandaPickAndPlace-v3", True, 1),  # configs[3]
    ("reach_ao", "PandaReachAO-v3", True, 1),           # configs[4]
]
FLOP_KEYS = ("add", "mul", "div", "sqrt", "trans")


def make_cfg(env_id: str, n: int, contacts: bool, seed: int, flags: int = 0):
    """The bench's configuration of ``env_id`` (with contacts: Bullet's per-pair manifold budget, the
    default handle's); ``flags``: oracle modelling switches (PGX_FLAG_DYN_RECURSIVE)."""
    sys.path.insert(0, ROOT)
    from panda_gym_amd import abi, envs
    from panda_gym_amd.model import load_model

    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params(flags=flags)
    cfg = abi.make_config(envs.spec(env_id), n, model, params, seed=seed, contacts=contacts, full_manifold=contacts)
    return cfg, (model, params)


# the two formulations of the dynamics phase counted: "recursive" (composite rigid bodies +
# Newton-Euler + Cholesky, SURVEY.md section 8d's minimal form, the one the kernel computes: the
# roofline numerator) and "jacobian" (the oracle's default Jacobian-form M and b, kept labelled)
FORMS = {"recursive": 16, "jacobian": 0}   # PGX_FLAG_DYN_RECURSIVE


def count(env_id: str, contacts: bool, seed: int, n: int, steps: int, flags: int = 0) -> dict:
    """Per-phase operation counts summed over ``steps`` random-policy steps of ``n`` envs
    (the initial reset excluded), plus the number of auto-resets seen."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    cfg, keep = make_cfg(env_id, n, contacts, seed, flags)
    env = O.OracleVecEnv(cfg, n, counting=True)
    env.reset()
    O.read_flops(clear=True)
    resets = 0
    for t in range(steps):
        out = env.step(env.sample_actions(t))
        resets += int((out["truncated"] | out["terminated"]).sum())
    ph = O.read_flops(clear=True)
    del keep
    return {"phases": ph, "env_steps": n * steps, "auto_resets": resets}


def summarise(raw: dict) -> dict:
    es = raw["env_steps"]
    per_phase = {k: sum(v[f] for f in FLOP_KEYS) / es for k, v in raw["phases"].items()}
    tot = {f: sum(v[f] for v in raw["phases"].values()) for f in FLOP_KEYS + ("cmp",)}
    return {"flops_per_env_step": sum(tot[f] for f in FLOP_KEYS) / es,
            "by_kind_per_env_step": {f: tot[f] / es for f in FLOP_KEYS + ("cmp",)},
            "by_phase_per_env_step": per_phase, "env_steps": es, "auto_resets": raw["auto_resets"],
            "totals": tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    from oracle import oracle as O

    O.build()
    with ProcessPoolExecutor(min(len(CONFIGS) * len(FORMS), os.cpu_count() or 1)) as ex:
        futs = {(key, form): ex.submit(count, eid, cont, seed, args.envs, args.steps, fl)
                for key, eid, cont, seed in CONFIGS for form, fl in FORMS.items()}
        res = {k: f.result() for k, f in futs.items()}
    doc = {
        "about": "Algorithmic fp64 FLOPs per env-step, op-counted in the oracle's restatement "
                 "(oracle/count_flops.py, oracle/flops_count.cpp): add/sub, mul, div, sqrt and "
                 "transcendentals count 1 each, comparisons (cmp) are listed apart and not counted. "
                 "Workload: device-Philox random actions from a fresh reset, auto-resets included; "
                 "the contact configs at Bullet's per-pair manifold budget (the default handle's). "
                 "flops_per_env_step is the 'recursive' form: the dynamics by composite rigid bodies + "
                 "Newton-Euler + Cholesky (SURVEY.md 8d, the kernel's formulation); 'jacobian' is the "
                 "oracle's default Jacobian-form M and b (the same dynamics, more arithmetic), kept "
                 "for reference only.",
        "sample": {"envs": args.envs, "steps": args.steps},
        "configs": {key: {"env_id": eid, "contacts": cont, "seed": seed,
                          "flops_per_env_step": summarise(res[key, "recursive"])["flops_per_env_step"],
                          **{form: summarise(res[key, form]) for form in FORMS}}
                    for key, eid, cont, seed in CONFIGS},
    }
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=False)
        f.write("\n")
    for key, v in doc["configs"].items():
        print(f"{key:16s} {v['recursive']['flops_per_env_step'] / 1e3:9.1f} kFLOP/env-step recursive, "
              f"{v['jacobian']['flops_per_env_step'] / 1e3:9.1f} jacobian form  resets {v['recursive']['auto_resets']}")


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main()
