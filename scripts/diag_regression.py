#!/usr/bin/env python3
"""Diagnostic: per-iteration training / validation l2 of the regression + EFB + GOSS preset
across learners (CPU oracle, HIP learner with device / host sampling, without GOSS).

    python scripts/diag_regression.py ROWS LEARNERS ITERS
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import numpy as np

    import lambdagap_amd as lgb
    from lambdagap_amd.models import preset
    from lambdagap_amd.utils import make_regression

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    devs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["cpu", "gpu", "gpu_hostsample", "gpu_nogoss"]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    X, y = make_regression(rows, num_features=500, seed=7)
    Xv, yv = make_regression(20000, num_features=500, seed=8)
    for name in devs:
        p = preset("regression_goss", device_type="cpu" if name == "cpu" else "gpu", verbosity=-1, metric="l2")
        if name == "gpu_hostsample":
            p["device_sampling"] = False
        if name == "gpu_nogoss":
            p.pop("data_sample_strategy")
        ds = lgb.Dataset(X, y, params=p, free_raw_data=False)
        dv = lgb.Dataset(Xv, yv, reference=ds)
        ev = {}
        b = lgb.train(p, ds, iters, valid_sets=[ds, dv], valid_names=["t", "v"],
                      callbacks=[lgb.record_evaluation(ev)])
        pred = b.predict(Xv)
        leaves = [v for t in b.dump_model()["tree_info"] for v in _leaves(t["tree_structure"])]
        print(json.dumps({"learner": name, "train_l2": ev["t"]["l2"], "l2": ev["v"]["l2"],
                          "pred_l2": float(np.mean((pred - yv) ** 2)),
                          "max_abs_leaf": float(max(abs(v) for v in leaves))}), flush=True)
    return 0


def _leaves(n):
    if "leaf_value" in n:
        return [n["leaf_value"]]
    return _leaves(n["left_child"]) + _leaves(n["right_child"])


if __name__ == "__main__":
    sys.exit(main())
