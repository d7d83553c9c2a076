"""Which bagging / GOSS configuration diverges between the host and the device learner."""
import sys
import os
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lambdagap_amd as lgb  # noqa: E402
from lambdagap_amd.utils import make_higgs_like  # noqa: E402

X, y = make_higgs_like(60000, seed=21)
base = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "min_data_in_leaf": 20, "seed": 1,
        "deterministic": True}
cases = [{"bagging_fraction": 0.7, "bagging_freq": 1},
         {"pos_bagging_fraction": 0.8, "neg_bagging_fraction": 0.5, "bagging_freq": 2},
         {"data_sample_strategy": "goss", "learning_rate": 0.5, "device_sampling": False},
         {"data_sample_strategy": "goss", "learning_rate": 0.5}]
for kw in cases:
    out = []
    for dev in ("cpu", "gpu"):
        p = dict(base, device_type=dev, **kw)
        b = lgb.train(p, lgb.Dataset(X, y, params=p), 5)
        out.append(b)
    for it in range(1, 6):
        pc = out[0].predict(X[:3000], raw_score=True, num_iteration=it)
        pg = out[1].predict(X[:3000], raw_score=True, num_iteration=it)
        print(kw, "iter", it, "maxdiff", float(np.abs(pc - pg).max()), flush=True)
    tc = out[0].dump_model()["tree_info"]
    tg = out[1].dump_model()["tree_info"]
    print("  leaf counts t0 cpu", tc[0]["tree_structure"].get("internal_count"),
          "gpu", tg[0]["tree_structure"].get("internal_count"), flush=True)
