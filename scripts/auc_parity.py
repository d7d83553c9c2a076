#!/usr/bin/env python3
"""Accuracy parity at the headline size (BASELINE.md "Accuracy"): the MI355X learner
(fixed-point histograms, and gpu_use_dp=true) against the CPU oracle learner on the
SAME synthetic Higgs-shape rows, held-out AUC after the same number of iterations.
The reference's own CPU-vs-GPU table (docs/GPU-Performance.rst:136) is the model;
the target is |dAUC| <= 1e-3.

    python scripts/auc_parity.py --rows 10000000 --iters 100 --num-leaves 63

Prints one JSON line (per-learner AUC, wall time, it/s).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--valid-rows", type=int, default=500_000)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--num-leaves", type=int, default=63)
    ap.add_argument("--learners", default="gpu,gpu_dp,cpu")
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args()

    import lambdagap_amd as lgb
    from lambdagap_amd.utils import make_higgs_like
    from bench import _auc

    X, y = make_higgs_like(args.rows, seed=args.seed)
    Xv, yv = make_higgs_like(args.valid_rows, seed=args.seed + 1000)
    base = {"objective": "binary", "num_leaves": args.num_leaves, "max_bin": 255, "learning_rate": 0.1,
            "min_data_in_leaf": 1, "min_sum_hessian_in_leaf": 100, "verbosity": -1, "seed": args.seed}
    # one binning shared by every learner: identical bins, so only the learners differ
    ds = lgb.Dataset(X, y, params=dict(base, device_type="cpu"), free_raw_data=False).construct()
    out = {"rows": args.rows, "iters": args.iters, "num_leaves": args.num_leaves, "data": "synthetic"}
    for name in args.learners.split(","):
        p = dict(base, device_type="cpu" if name == "cpu" else "gpu")
        if name == "gpu_dp":
            p["gpu_use_dp"] = True
        t = time.perf_counter()
        b = lgb.train(p, ds, args.iters, keep_training_booster=True)
        el = time.perf_counter() - t
        auc = _auc(yv, b.predict(Xv))
        out[name] = {"auc": round(auc, 6), "train_s": round(el, 2), "it_s": round(args.iters / el, 2),
                     "device": b.device_name()}
        print(name, out[name], file=sys.stderr, flush=True)
    if "cpu" in out:
        for name in ("gpu", "gpu_dp"):
            if name in out:
                out[f"d_auc_{name}_vs_cpu"] = round(out[name]["auc"] - out["cpu"]["auc"], 6)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
