#!/usr/bin/env python3
"""A/B timing of learner settings in ONE process on the same data (box-to-box and
run-to-run clock variation on the pool is larger than the effects we tune for).

    python scripts/ab_bench.py --rows 1250000 --variant graph=1 --variant graph=0

Each variant is a booster with its own parameter overrides; variants are timed in
alternating blocks of --block iterations after a warmup, and the median ms/iter
per variant is printed as JSON.
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
    ap.add_argument("--variant", action="append", default=[])
    ap.add_argument("--block", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--preset", default="higgs", choices=["higgs", "ltr", "goss"])
    ap.add_argument("--quantized", action="store_true", help="use_quantized_grad=true, 4 levels (goss / ltr)")
    ap.add_argument("--features", type=int, default=300)
    args = ap.parse_args()
    import lambdagap_amd as lgb
    from lambdagap_amd.parallel import device_synchronize
    from lambdagap_amd.utils import make_higgs_like

    if args.preset == "goss":
        from lambdagap_amd.models import preset
        from lambdagap_amd.utils import make_regression

        X, y = make_regression(args.rows, num_features=args.features, seed=7)
        base = preset("regression_goss", verbosity=-1, seed=7)
        if args.quantized:
            base.update(use_quantized_grad=True, num_grad_quant_bins=4)
        ds = lgb.Dataset(X, y, params=base, free_raw_data=True).construct()
        del X
    elif args.preset == "ltr":
        from lambdagap_amd.models import preset
        from lambdagap_amd.utils import make_ranking

        X, y, g = make_ranking(max(1, args.rows // 120), num_features=args.features, docs_per_query=(60, 180), seed=7)
        base = preset("ltr", verbosity=-1, seed=7)
        if args.quantized:
            base.update(use_quantized_grad=True, num_grad_quant_bins=4)
        ds = lgb.Dataset(X, y, group=g, params=base, free_raw_data=False).construct()
    else:
        X, y = make_higgs_like(args.rows, seed=7)
        base = {"objective": "binary", "num_leaves": 63, "max_bin": 255, "learning_rate": 0.1, "min_data_in_leaf": 1,
                "min_sum_hessian_in_leaf": 100, "device_type": "gpu", "verbosity": -1, "seed": 7}
        ds = lgb.Dataset(X, y, params=base, free_raw_data=False).construct()
    variants = args.variant or ["device_use_graph=1", "device_use_graph=0"]
    boosters, benvs = [], []

    class _Env:  # a variant's environment knobs, applied while its booster is set up and updated
        def __init__(self, envs):
            self.envs = envs

        def __enter__(self):
            self.saved = {k: os.environ.get(k) for k in self.envs}
            os.environ.update(self.envs)

        def __exit__(self, *exc):
            for k, old_v in self.saved.items():
                if old_v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = old_v

    for v in variants:
        p = dict(base)
        envs = {}
        for kv in v.split(","):
            k, val = kv.split("=")
            if k.startswith("env."):  # environment knobs read when the learner is set up
                envs[k[4:]] = val
            else:
                p[k] = val
        benvs.append(_Env(envs))
        with benvs[-1]:
            boosters.append(lgb.Booster(params=p, train_set=ds))
    for b, env in zip(boosters, benvs):
        with env:
            for _ in range(args.warmup):
                b.update()
    device_synchronize()
    times = [[] for _ in boosters]
    for _ in range(args.rounds):
        for i, b in enumerate(boosters):
            device_synchronize()
            with benvs[i]:
                t0 = time.perf_counter()
                for _ in range(args.block):
                    b.update()
                device_synchronize()
            times[i].append(1000.0 * (time.perf_counter() - t0) / args.block)
    out = {v: {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(np.min(t)), 4)}
           for v, t in zip(variants, times)}
    print(json.dumps({"rows": args.rows, "results": out}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
