"""Per-split comparison of CPU and device trees on the wide-data test
(test_wide_data_wave_scan_matches_cpu[extra1]); device variants chosen by env assignments,
e.g. `python scripts/dbg/wide_diff.py LGAP_SCAN_WAVE=0 LGAP_SCAN_WAVE=1`."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import lambdagap_amd as lgb


def walk(node, out, depth=0):
    if "split_index" not in node:
        return
    out.append((node["split_index"], depth, node["split_feature"], round(node["threshold"], 6), node["split_gain"],
                node["internal_count"], round(node["internal_value"], 6), node["default_left"]))
    walk(node["left_child"], out, depth + 1)
    walk(node["right_child"], out, depth + 1)


rng = np.random.default_rng(12345)
n, nf = 20000, 80
X = rng.standard_normal((n, nf))
X[rng.random((n, nf)) < 0.05] = np.nan
z = X[:, 0] - 0.7 * np.nan_to_num(X[:, 1]) + 0.4 * np.nan_to_num(X[:, 5]) * np.nan_to_num(X[:, 9])
y = (z + 0.3 * rng.standard_normal(n) > 0).astype(float)
kw = {"objective": "binary", "num_leaves": 63, "min_data_in_leaf": 20, "monotone_constraints": [1] + [0] * 79,
      "verbosity": -1, "seed": 1, "deterministic": True}
if os.environ.get("WIDE_NOMONO"):
    kw.pop("monotone_constraints")
variants = sys.argv[1:] or ["default"]
res = {}
p = dict(kw, device_type="cpu")
res["cpu"] = lgb.train(p, lgb.Dataset(X, y, params=p), 1).dump_model()["tree_info"]
for v in variants:
    saved = dict(os.environ)
    if "=" in v:
        k, val = v.split("=", 1)
        os.environ[k] = val
    p = dict(kw, device_type="gpu", gpu_use_dp=True)
    res[v] = lgb.train(p, lgb.Dataset(X, y, params=p), 1).dump_model()["tree_info"]
    os.environ.clear()
    os.environ.update(saved)
a = []
walk(res["cpu"][0]["tree_structure"], a)
a.sort()
for v in variants:
    g = []
    walk(res[v][0]["tree_structure"], g)
    g.sort()
    same = [x[2:4] for x in a] == [x[2:4] for x in g]
    print(f"[{v}] tree 0: {'same' if same else 'DIFF'}", flush=True)
    if not same:
        shown = 0
        for x, y2 in zip(a, g):
            if x[2:4] != y2[2:4] or shown < 0:
                print("  cpu", x, "\n  gpu", y2, "  <<<")
                shown += 1
                if shown >= 4:
                    break
