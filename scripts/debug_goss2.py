"""Determinism of host-sampled GOSS on the CPU and the device learner within one process."""
import sys
import os
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lambdagap_amd as lgb  # noqa: E402
from lambdagap_amd.utils import make_higgs_like  # noqa: E402

X, y = make_higgs_like(60000, seed=21)
base = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "min_data_in_leaf": 20, "seed": 1,
        "deterministic": True, "data_sample_strategy": "goss", "learning_rate": 0.5, "device_sampling": False}
first = sys.argv[1] if len(sys.argv) > 1 else ""
if first == "bag":
    p = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "bagging_fraction": 0.7, "bagging_freq": 1,
         "device_type": "gpu"}
    lgb.train(p, lgb.Dataset(X, y, params=p), 5)
preds = {}
for rep in range(2):
    for dev in ("cpu", "gpu"):
        p = dict(base, device_type=dev)
        b = lgb.train(p, lgb.Dataset(X, y, params=p), 3)
        preds[(dev, rep)] = b.predict(X[:3000], raw_score=True)
for k, v in preds.items():
    print(k, "vs cpu0", float(np.abs(v - preds[("cpu", 0)]).max()), flush=True)
