"""Debug: first split where the device frontier and the CPU learner differ (monotone methods)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import lambdagap_amd as lgb


def splits(node, out):
    if "split_index" in node:
        out.append((node["split_index"], node["split_feature"], node["split_gain"], node["internal_count"], node["threshold"]))
        splits(node["left_child"], out)
        splits(node["right_child"], out)
    return sorted(out)


import json
EXTRA = json.loads(os.environ.get("EXTRA", "{}"))


def run(method, n=int(os.environ.get("N", "60000")), leaves=int(os.environ.get("LEAVES", "127")),
        mind=int(os.environ.get("MIND", "5")), rounds=8):
    rng = np.random.default_rng(int(os.environ.get("SEED", "0")))
    X = rng.standard_normal((n, 6))
    z = 1.5 * X[:, 0] - X[:, 1] + 0.7 * X[:, 2] * X[:, 3] + 0.3 * rng.standard_normal(n)
    y = z if EXTRA.get("objective") == "regression" else (z > 0).astype(float)
    res = {}
    for dev in ("cpu", "gpu"):
        p = {"objective": "binary", **{k: v for k, v in EXTRA.items() if k == "objective"}, "num_leaves": leaves, "device_type": dev, "verbosity": -1, "min_data_in_leaf": mind,
             "seed": 1, "deterministic": True, "gpu_use_dp": True, **EXTRA}
        if method:
            p.update(monotone_constraints=[1, -1, 1, 0, -1, 0], monotone_constraints_method=method)
        b = lgb.train(p, lgb.Dataset(X, y, params=p), rounds)
        res[dev] = [splits(t["tree_structure"], []) for t in b.dump_model()["tree_info"]]
    print(method, "leaves cpu", [len(t) + 1 for t in res["cpu"]], "gpu", [len(t) + 1 for t in res["gpu"]])
    for ti, (a, b) in enumerate(zip(res["cpu"], res["gpu"])):
        for i, (x, y2) in enumerate(zip(a, b)):
            if x[:2] != y2[:2]:
                print(method, "tree", ti, "split", i, "cpu", x, "gpu", y2, flush=True)
                # the gains of the two candidates elsewhere in each tree
                print("   cpu near:", [s for s in a if abs(s[2] - y2[2]) < 1e-6 * max(1, abs(y2[2]))][:3])
                print("   gpu near:", [s for s in b if abs(s[2] - x[2]) < 1e-6 * max(1, abs(x[2]))][:3])
                return
    print(method, "all equal", flush=True)


for m in sys.argv[1:]:
    run(None if m == "none" else m)
