#!/usr/bin/env python3
"""Secondary benchmark configurations of BASELINE.json on one GPU (bench.py is the headline).

    python scripts/bench_suite.py --config ltr --rows 5000000 --features 300
    python scripts/bench_suite.py --config regression_goss --rows 2000000 --features 500

`ltr`: LambdaRank on synthetic grouped queries (60-180 documents per query), NDCG@1/3/5/10 on a
held-out query set. `regression_goss`: wide mostly-zero regression (EFB bundles the sparse columns)
with GOSS sampling, l2 on a held-out set. Timed exactly like bench.py: W untimed iterations, then K
iterations between device synchronisations. Synthetic data, random labels of the named shape.
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["ltr", "regression_goss"], required=True)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--valid-rows", type=int, default=200_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--quantized", action="store_true", help="use_quantized_grad=true, 4 gradient levels")
    ap.add_argument("--learner", choices=["serial", "data", "voting"], default="serial",
                    help="data / voting on ONE GPU run through a one-rank RCCL communicator (the parallel "
                         "learner's kernels and exchanges, single rank)")
    args = ap.parse_args()
    if args.learner != "serial":
        import ctypes

        from lambdagap_amd.parallel import distributed as dd

        uid = dd.get_unique_id()
        dd._check(dd._LIB.LGBM_DeviceCommInit(dd._c_str(uid), ctypes.c_int64(len(uid)), ctypes.c_int(1),
                                              ctypes.c_int(0), ctypes.c_int(0)))
        # (one machine: the configuration trains serial, as the reference; the knob keeps the
        # parallel learner's path on the one-rank communicator)
        os.environ["LGAP_FORCE_DEVICE_DP"] = "1" if args.learner == "data" else "voting"

    import numpy as np

    import lambdagap_amd as lgb
    from lambdagap_amd.models import preset
    from lambdagap_amd.parallel import device_synchronize
    from lambdagap_amd.utils import make_ranking, make_regression

    t0 = time.time()
    if args.config == "ltr":
        nf = args.features or 300
        X, y, g = make_ranking(max(1, args.rows // 120), num_features=nf, docs_per_query=(60, 180), seed=7)
        Xv, yv, gv = make_ranking(max(1, args.valid_rows // 120), num_features=nf, docs_per_query=(60, 180), seed=8)
        params = preset("ltr", device_type=args.device, verbosity=-1)
    else:
        nf = args.features or 500
        X, y = make_regression(args.rows, num_features=nf, seed=7)
        Xv, yv = make_regression(args.valid_rows, num_features=nf, seed=8)
        g = gv = None
        params = preset("regression_goss", device_type=args.device, verbosity=-1, metric="l2")
    if args.learner == "voting":
        params["tree_learner"] = "voting"
    if args.quantized:
        params["use_quantized_grad"] = True
        params["num_grad_quant_bins"] = 4
    gen_s = time.time() - t0
    print(f"# data generated in {gen_s:.1f} s", file=sys.stderr, flush=True)
    t0 = time.time()
    train = lgb.Dataset(X, y, group=g, params=params, free_raw_data=True)
    valid = lgb.Dataset(Xv, yv, group=gv, reference=train)
    booster = lgb.Booster(params=params, train_set=train)
    rows = int(len(y))
    del X
    construct_s = time.time() - t0
    print(f"# dataset + booster in {construct_s:.1f} s ({booster.device_name()})", file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        booster.update()
    device_synchronize()
    print("# warmup done", file=sys.stderr, flush=True)
    t = time.perf_counter()
    for _ in range(args.steps):
        booster.update()
    device_synchronize()
    el = time.perf_counter() - t
    booster.add_valid(valid, "valid")
    ev = {name: round(v, 6) for _, name, v, _ in booster.eval_valid()}
    print(json.dumps({"config": args.config, "rows": rows, "features": nf, "value": round(args.steps / el, 3),
                      "unit": "iters/s", "ms_per_step": round(1000 * el / args.steps, 3), "steps": args.steps,
                      "warmup": args.warmup, "device": booster.device_name(), "valid": ev, "learner": args.learner, "quantized": args.quantized,
                      "num_leaves": params["num_leaves"], "max_bin": params["max_bin"],
                      "data_gen_s": round(gen_s, 1), "construct_s": round(construct_s, 1), "data": "synthetic"}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
