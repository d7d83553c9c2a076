"""Intermediate monotone on the frontier at larger shapes: 255 leaves, 10M rows (timing + monotone check)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import lambdagap_amd as lgb
from lambdagap_amd.parallel import device_synchronize
from lambdagap_amd.utils import make_higgs_like
for rows, leaves, steps in ((1_000_000, 255, 20), (10_000_000, 63, 20)):
    X, y = make_higgs_like(rows, seed=7)
    for method in ("none", "intermediate"):
        p = {"objective": "binary", "num_leaves": leaves, "max_bin": 255, "device_type": "gpu", "verbosity": -1, "seed": 7,
             "min_data_in_leaf": 20}
        if method != "none":
            p.update(monotone_constraints=[1, -1, 1, -1] + [0] * (X.shape[1] - 4), monotone_constraints_method=method)
        b = lgb.Booster(p, lgb.Dataset(X, y, params=p))
        for _ in range(3):
            b.update()
        device_synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            b.update()
        device_synchronize()
        dt = time.perf_counter() - t
        ok = True
        if method != "none":
            grid = np.linspace(-3, 3, 40)
            for row in X[:5]:
                for f, s in ((0, 1), (1, -1)):
                    Z = np.repeat(row[None, :], len(grid), 0)
                    Z[:, f] = grid
                    ok = ok and bool(np.all(s * np.diff(b.predict(Z, raw_score=True)) >= -1e-10))
        print(json.dumps({"rows": rows, "leaves": leaves, "method": method, "it_s": round(steps / dt, 2), "monotone": ok,
                          "device": b.device_name()}), flush=True)
