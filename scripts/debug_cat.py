"""CPU vs GPU split-by-split comparison on data with NaN / zero / categorical columns."""
import sys

import numpy as np

sys.path.insert(0, ".")
import lambdagap_amd as lgb

rng = np.random.default_rng(12345)
n = 30000
X = rng.standard_normal((n, 6))
X[rng.random(n) < 0.2, 0] = np.nan
X[rng.random(n) < 0.5, 1] = 0.0
X[:, 2] = rng.integers(0, 12, n)
y = ((np.nan_to_num(X[:, 0]) > 0.3) ^ (X[:, 2] % 3 == 0) ^ (X[:, 1] > 0.5)).astype(float)
dp = len(sys.argv) > 1 and sys.argv[1] == "dp"
params = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "min_data_in_leaf": 20, "seed": 1,
          "categorical_feature": [2], "max_cat_to_onehot": 4}


def walk(node, out, depth=0):
    if "split_index" in node:
        out.append((node["split_index"], node["split_feature"], node["threshold"], node["default_left"],
                    round(node["split_gain"], 6), node["internal_count"], node.get("missing_type")))
        walk(node["left_child"], out, depth + 1)
        walk(node["right_child"], out, depth + 1)
    return out


bc = lgb.train({**params, "device_type": "cpu"}, lgb.Dataset(X, y, params=params), 3)
bg = lgb.train({**params, "device_type": "gpu", "gpu_use_dp": dp}, lgb.Dataset(X, y, params=params), 3)
for t in range(3):
    sc = sorted(walk(bc.dump_model()["tree_info"][t]["tree_structure"], []))
    sg = sorted(walk(bg.dump_model()["tree_info"][t]["tree_structure"], []))
    nd = 0
    for a, b in zip(sc, sg):
        if a[1:3] != b[1:3]:
            nd += 1
            if nd <= 4:
                print("tree", t, "DIFF", a, "|", b)
    print("tree", t, "splits", len(sc), len(sg), "diffs", nd)
