"""Per-split comparison of CPU and device extra-trees trees (test_extra_trees_on_frontier_matches_cpu[extra0])."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import lambdagap_amd as lgb


def walk(node, out, depth=0):
    if "split_index" not in node:
        return
    out.append((node["split_index"], depth, node["split_feature"], node["threshold"], round(node["split_gain"], 6),
                node["internal_count"], round(node["internal_value"], 6)))
    walk(node["left_child"], out, depth + 1)
    walk(node["right_child"], out, depth + 1)


variant = sys.argv[1] if len(sys.argv) > 1 else "default"
rng = np.random.default_rng(12345)
n = 30000
X = rng.standard_normal((n, 8))
X[:, 6] = rng.integers(0, 3, n)
X[:, 7] = rng.integers(0, 25, n)
z = X[:, 0] - 0.8 * X[:, 1] + 0.4 * (X[:, 7] % 5 == 1) + 0.3 * (X[:, 6] == 2) + 0.3 * rng.standard_normal(n)
y = (z > 0).astype(float)
kw = {"objective": "binary", "num_leaves": 15, "extra_trees": True, "categorical_feature": [6, 7],
      "min_data_per_group": 20, "cat_smooth": 5, "verbosity": -1, "seed": 1,
      "deterministic": True, "min_data_in_leaf": 20}
if variant == "nocat":
    kw["categorical_feature"] = []
elif variant == "onehot":
    kw["categorical_feature"] = [6]
elif variant == "manycat":
    kw["categorical_feature"] = [7]
res = {}
for dev, extra in (("cpu", {}), ("gpu", {"gpu_use_dp": True})):
    p = dict(kw, device_type=dev, **extra)
    b = lgb.train(p, lgb.Dataset(X, y, params=p), 5)
    res[dev] = b.dump_model()["tree_info"]
for t in range(5):
    a, g = [], []
    walk(res["cpu"][t]["tree_structure"], a)
    walk(res["gpu"][t]["tree_structure"], g)
    a.sort(); g.sort()
    same = [x[2:4] for x in a] == [x[2:4] for x in g]
    print(f"[{variant}] tree {t}: {'same' if same else 'DIFF'}")
    if not same:
        for x, y2 in zip(a, g):
            flag = "" if x[2:4] == y2[2:4] else "  <<<"
            print("  cpu", x, "\n  gpu", y2, flag)
        break
