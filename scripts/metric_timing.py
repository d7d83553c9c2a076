#!/usr/bin/env python3
"""Cost of a training-set AUC every iteration on the 10M x 28 headline data: iterations/s
without a metric, with the device AUC (metric_kernels.hip) and with the host AUC
(LGAP_DEVICE_METRICS=0: score download + parallel-sort tie-aware loop). One JSON line each."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(lgb, X, y, metric, device_metrics, iters, warmup):
    os.environ["LGAP_DEVICE_METRICS"] = "1" if device_metrics else "0"
    params = {"objective": "binary", "num_leaves": 63, "learning_rate": 0.1, "min_data_in_leaf": 1,
              "min_sum_hessian_in_leaf": 100, "device_type": "gpu", "verbosity": -1, "metric": metric or "None"}
    ds = lgb.Dataset(X, y, params=params)
    b = lgb.Booster(params, ds)
    for _ in range(warmup):
        b.update()
    from lambdagap_amd.parallel import device_synchronize

    vals = []
    device_synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        b.update()
        if metric:
            vals.append(b.eval_train()[0][2])
    device_synchronize()
    el = time.perf_counter() - t0
    return iters / el, (vals[-1] if vals else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import lambdagap_amd as lgb
    from lambdagap_amd.utils import make_higgs_like

    X, y = make_higgs_like(a.rows, seed=7)
    for metric, dev in ((None, True), ("auc", True), ("auc", False)):
        it_s, v = run(lgb, X, y, metric, dev, a.iters, a.warmup)
        print(json.dumps({"rows": a.rows, "metric": metric, "where": "device" if dev else "host",
                          "it_per_s": round(it_s, 2), "ms_per_iter": round(1000 / it_s, 3),
                          "last_value": v}), flush=True)


if __name__ == "__main__":
    main()
