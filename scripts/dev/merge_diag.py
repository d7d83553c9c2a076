import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import lambdagap_amd as lgb
os.environ["LGAP_FRONTIER_SPEC"] = "fixed"
rng = np.random.default_rng(29)
n = 80000
X = rng.standard_normal((n, 16))
y = X[:, 0] + 0.5 * X[:, 1] * X[:, 2] - 0.4 * np.abs(X[:, 3]) + 0.3 * rng.standard_normal(n)
L = int(os.environ.get("LEAVES", "511"))
params = {"objective": "regression", "num_leaves": L, "min_data_in_leaf": 2, "device_type": "gpu",
          "verbosity": -1, "seed": 4, "deterministic": True}
res = {}
for tag, merge in (("m1", True), ("m2", True), ("f1", False), ("f2", False)):
    if merge:
        os.environ.pop("LGAP_KERNEL", None)
    else:
        os.environ["LGAP_KERNEL"] = "select_merge=0"
    b = lgb.train(params, lgb.Dataset(X, y, params=params), 12, keep_training_booster=True)
    res[tag] = [t["num_leaves"] for t in b.dump_model()["tree_info"]], b.model_to_string()
for a, b in (("m1", "m2"), ("f1", "f2"), ("m1", "f1")):
    print(a, b, "equal" if res[a][1] == res[b][1] else "DIFFER", res[a][0], res[b][0], flush=True)
