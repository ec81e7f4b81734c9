"""CPU analysis of the outliers tools/gpu_scripted_outlier.py dumped: for each, the fp64 oracle's own
one-step response to its input state perturbed by 1e-7 / 3e-7 relative (the fp32 rounding scale of the
device state), and the restated algorithm evaluated in fp32 (oracle/fp32_emul.cpp) from the same state
-- how far the reference algorithm itself moves there -- beside the device's deviation.

    python tools/analyze_outlier.py gpurun_out/scripted_outliers.npz [--env PandaPickAndPlace-v3]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from panda_gym_amd import abi, envs  # noqa: E402
from panda_gym_amd.model import load_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--env", default="PandaPickAndPlace-v3")
    ap.add_argument("--trials", type=int, default=64)
    args = ap.parse_args()
    d = np.load(args.npz)
    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params()
    cfg = abi.make_config(envs.spec(args.env), 1, model, params, seed=3, full_manifold=True)
    keys = ("q", "qd", "qc", "goal", "obj", "elapsed", "episode")
    for j in range(int(d["count"])):
        sfx = f"_{j}"
        rec = {k[:-len(sfx)]: d[k] for k in d.files if k.endswith(sfx) and k != "count"}
        a = rec["action"][None].astype(np.float32)

        def run(fp32=False, pert=0.0, seed=0):
            r = O.OracleVecEnv(cfg, 1, fp32=fp32)
            rng = np.random.default_rng(seed)
            for k in keys:
                v = rec["in_" + k].copy()
                if pert and k in ("q", "qd"):
                    v = v * (1.0 + pert * rng.standard_normal(v.shape))
                if pert and k == "obj":
                    v[:13] = v[:13] * (1.0 + pert * rng.standard_normal(13))
                getattr(r, k)[0] = v
            o = r.step(a)
            return o["obs"][0], r.obj[0, :3].copy()

        base_obs, base_obj = run()
        moves = []
        for t in range(args.trials):
            o, ob = run(pert=1e-7 if t % 2 == 0 else 3e-7, seed=t)
            moves.append(max(np.abs(o[:3] - base_obs[:3]).max(), np.abs(ob - base_obj).max()))
        o32, ob32 = run(fp32=True)
        f32 = max(np.abs(o32[:3] - base_obs[:3]).max(), np.abs(ob32 - base_obj).max())
        print(f"t {int(rec['t'])} env {int(rec['env'])}: device deviation {float(rec['err']):.3e}; the oracle under "
              f"1e-7/3e-7 perturbations: max {max(moves):.3e}, median {np.median(moves):.3e}; fp32 evaluation "
              f"{f32:.3e}; input cube {rec['in_obj'][:3]} (z of the table top 0)", flush=True)


if __name__ == "__main__":
    main()
