"""Fixed-point histogram precision with heavy-tailed gradients (tests/test_gpu_learner.py
test_fixed_point_heavy_tailed_regression_10m), with the round-3 scale for comparison:
held-out L2 against the noise-free target for the fixed-point learner with the sum|g| bound
(default), without it (LGAP_FIXED_SUMBOUND=0: rows * max|g| only) and for gpu_use_dp=true.

    python scripts/heavy_tail_precision.py [--rows 10000000] [--iters 30]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import lambdagap_amd as lgb  # noqa: E402


def make(rng, n, nf=8):
    X = rng.standard_normal((n, nf)).astype(np.float32)
    f = np.sin(2.0 * X[:, 0]) + 0.5 * X[:, 1] * X[:, 2] + np.where(X[:, 3] > 0.5, 1.0, -0.3)
    return X, f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--df", type=float, default=1.5)
    args = ap.parse_args()
    rng = np.random.default_rng(31)
    X, f = make(rng, args.rows)
    y = f + rng.standard_t(args.df, args.rows)
    out = rng.random(args.rows) < 1e-5
    y[out] *= 1e4
    Xv, fv = make(rng, 500_000)
    g0 = np.abs(y - y.mean())
    print(f"max|g| / median|g| at the first tree: {g0.max() / np.median(g0):.3g}", flush=True)
    base = {"objective": "regression", "num_leaves": 63, "learning_rate": 0.1, "min_data_in_leaf": 100,
            "verbosity": -1, "device_type": "gpu"}
    ds = lgb.Dataset(X, y, params=base, free_raw_data=False).construct()
    res = {}
    for name, extra, env in (("fixed_sumbound", {}, "1"), ("fixed_max_only", {}, "0"),
                             ("fp64", {"gpu_use_dp": True}, "1")):
        os.environ["LGAP_FIXED_SUMBOUND"] = env
        t0 = time.time()
        b = lgb.train(dict(base, **extra), ds, args.iters, keep_training_booster=True)
        dt = time.time() - t0
        l2 = float(np.mean((b.predict(Xv) - fv) ** 2))
        res[name] = {"heldout_l2_vs_clean": l2, "train_s": round(dt, 2)}
        print(name, json.dumps(res[name]), flush=True)
    ref = res["fp64"]["heldout_l2_vs_clean"]
    for k, v in res.items():
        v["rel_vs_fp64"] = (v["heldout_l2_vs_clean"] - ref) / ref
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
