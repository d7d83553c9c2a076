"""Per-iteration CPU vs GPU comparison for lambdarank (debug aid)."""
import sys

import numpy as np

sys.path.insert(0, ".")
import lambdagap_amd as lgb
from lambdagap_amd import ops
from lambdagap_amd.utils import make_ranking

target = sys.argv[1] if len(sys.argv) > 1 else "ndcg"
X, y, sizes = make_ranking(300, num_features=20, seed=3)
params = {"objective": "lambdarank", "lambdarank_target": target, "num_leaves": 15, "verbosity": -1,
          "lambdarank_truncation_level": 10}
bc = lgb.Booster({**params, "device_type": "cpu"}, lgb.Dataset(X, y, group=sizes))
bg = lgb.Booster({**params, "device_type": "gpu"}, lgb.Dataset(X, y, group=sizes))
for it in range(3):
    bc.update()
    bg.update()
    gc, hc = ops.booster_gradients(bc)
    gg, hg = ops.booster_gradients(bg)
    d = np.abs(gc - gg)
    print(f"iter {it}: grad maxdiff {d.max():.3e} at {d.argmax()} (cpu {gc[d.argmax()]:.6g} gpu {gg[d.argmax()]:.6g}) "
          f"hess maxdiff {np.abs(hc - hg).max():.3e}; sum|g| {np.abs(gc).sum():.4g}")
    tc = bc.dump_model()["tree_info"][-1]
    tg = bg.dump_model()["tree_info"][-1]
    print("  leaves", tc["num_leaves"], tg["num_leaves"], "root split", tc["tree_structure"].get("split_feature"),
          tc["tree_structure"].get("threshold"), "|", tg["tree_structure"].get("split_feature"),
          tg["tree_structure"].get("threshold"))
    pc, pg = bc.predict(X, raw_score=True), bg.predict(X, raw_score=True)
    print("  pred corr", np.corrcoef(pc, pg)[0, 1], "maxdiff", np.abs(pc - pg).max())
