"""Per-iteration wall times of the headline training loop (device synchronised after every
update): distribution and the slowest iterations. `python scripts/dbg/iter_times.py ROWS STEPS`"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import lambdagap_amd as lgb
from lambdagap_amd.parallel import device_synchronize
from lambdagap_amd.utils import make_higgs_like

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 150
X, y = make_higgs_like(rows, seed=7)
params = {"objective": "binary", "num_leaves": 63, "max_bin": 255, "learning_rate": 0.1, "min_data_in_leaf": 1,
          "min_sum_hessian_in_leaf": 100, "device_type": "gpu", "verbosity": -1, "seed": 7}
b = lgb.Booster(params=params, train_set=lgb.Dataset(X, y, params=params, free_raw_data=True))
ts = []
for i in range(steps):
    device_synchronize()
    t0 = time.perf_counter()
    b.update()
    device_synchronize()
    ts.append(1000 * (time.perf_counter() - t0))
ts = np.array(ts)
print(f"rows {rows}: mean {ts.mean():.3f} ms, median {np.median(ts):.3f}, p90 {np.percentile(ts, 90):.3f}, max {ts.max():.3f}")
for lo in range(0, steps, 25):
    seg = ts[lo:lo + 25]
    print(f"  iters {lo}-{lo + len(seg) - 1}: mean {seg.mean():.3f} median {np.median(seg):.3f} max {seg.max():.3f}")
slow = np.argsort(ts)[::-1][:8]
print("slowest:", ", ".join(f"{i}:{ts[i]:.2f}" for i in sorted(slow)))


def depth(node):
    if "split_index" not in node:
        return 0
    return 1 + max(depth(node["left_child"]), depth(node["right_child"]))


trees = b.dump_model()["tree_info"]
ds = np.array([depth(t["tree_structure"]) for t in trees])
for lo in range(0, len(ds), 25):
    print(f"  trees {lo}-{min(len(ds), lo + 25) - 1}: mean depth {ds[lo:lo + 25].mean():.1f} max {ds[lo:lo + 25].max()}")
