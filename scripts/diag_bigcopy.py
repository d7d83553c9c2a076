#!/usr/bin/env python3
"""Diagnostic: one small tree on a wide dataset past 8M rows, CPU oracle vs HIP learner (split
structure, leaf values, training l2)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import lambdagap_amd as lgb  # noqa: E402
from lambdagap_amd.models import preset  # noqa: E402
from lambdagap_amd.utils import make_regression  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8_500_000
X, y = make_regression(rows, num_features=500, seed=7)
p = preset("regression_goss", device_type="cpu", verbosity=-1, metric="l2",
           num_leaves=int(sys.argv[3]) if len(sys.argv) > 3 else 4)
ds = lgb.Dataset(X, y, params=p, free_raw_data=False).construct()
print("groups/bins", ds.num_feature(), flush=True)
out = {}
for dev in sys.argv[2].split(",") if len(sys.argv) > 2 else ["gpu", "cpu"]:
    ev = {}
    b = lgb.train(dict(p, device_type=dev), ds, 1, valid_sets=[ds], valid_names=["t"],
                  callbacks=[lgb.record_evaluation(ev)], keep_training_booster=True)
    t = b.dump_model()["tree_info"][0]["tree_structure"]

    def walk(n, d=0):
        if "leaf_value" in n:
            return [("leaf", round(n["leaf_value"], 6), n.get("leaf_count"))]
        return [(n["split_feature"], round(n["threshold"], 6), n["internal_count"], round(n["split_gain"], 3))] + \
            walk(n["left_child"], d + 1) + walk(n["right_child"], d + 1)

    nodes = walk(t)
    out[dev] = nodes
    print(dev, ev["t"]["l2"], len(nodes), flush=True)
if len(out) == 2:
    a, b = out.values()
    for i, (u, v) in enumerate(zip(a, b)):
        if u[:3] != v[:3]:
            print("first difference at node", i, u, v, "context", a[max(0, i - 3):i + 2], b[max(0, i - 3):i + 2])
            break
    else:
        print("identical structure")
