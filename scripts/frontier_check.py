#!/usr/bin/env python3
"""Frontier engine vs the sequential device chain vs the CPU learner on the same data.

    python scripts/frontier_check.py [rows] [num_leaves] [rounds]

Each engine runs in its own process (LGAP_FRONTIER=1 / 0); prints one JSON line with the
number of leading trees whose split structure is identical and the max |raw score| diff.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, %(root)r)
import numpy as np
import lambdagap_amd as lgb
from lambdagap_amd.utils import make_higgs_like
X, y = make_higgs_like(%(rows)d, seed=5)
p = {"objective": "binary", "num_leaves": %(leaves)d, "device_type": %(dev)r, "verbosity": -1,
     "min_data_in_leaf": 20, "seed": 1, "gpu_use_dp": %(dp)s, "max_bin": 255}
p.update(%(extra)s)
b = lgb.train(p, lgb.Dataset(X, y, params=p), %(rounds)d, keep_training_booster=True)
trees = []
for t in b.dump_model()["tree_info"]:
    out = []
    def walk(n):
        if "split_index" in n:
            out.append((n["split_feature"], n["threshold"], n["default_left"]))
            walk(n["left_child"]); walk(n["right_child"])
    walk(t["tree_structure"])
    trees.append(out)
pred = b.predict(X[:5000], raw_score=True).tolist()
print(json.dumps({"trees": trees, "pred": pred, "name": b.device_name()}))
"""


def run(dev, frontier, rows, leaves, rounds, dp, extra):
    env = dict(os.environ, LGAP_FRONTIER="1" if frontier else "0")
    code = CHILD % {"root": ROOT, "rows": rows, "leaves": leaves, "dev": dev, "dp": dp, "rounds": rounds,
                    "extra": repr(extra)}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 40000
    leaves = int(sys.argv[2]) if len(sys.argv) > 2 else 31
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    extra = json.loads(sys.argv[4]) if len(sys.argv) > 4 else {}
    import numpy as np

    res = {}
    for dp in ("True", "False"):
        f = run("gpu", True, rows, leaves, rounds, dp, extra)
        s = run("gpu", False, rows, leaves, rounds, dp, extra)
        c = run("cpu", False, rows, leaves, rounds, dp, extra)

        def lead(a, b):
            n = 0
            for x, y in zip(a["trees"], b["trees"]):
                if x != y:
                    break
                n += 1
            return n

        res[dp] = {"frontier_vs_seq_trees": lead(f, s), "frontier_vs_cpu_trees": lead(f, c),
                   "seq_vs_cpu_trees": lead(s, c),
                   "max_diff_vs_seq": float(np.max(np.abs(np.array(f["pred"]) - np.array(s["pred"])))),
                   "max_diff_vs_cpu": float(np.max(np.abs(np.array(f["pred"]) - np.array(c["pred"])))),
                   "leaves_first": [len(f["trees"][0]), len(s["trees"][0]), len(c["trees"][0])]}
    print(json.dumps({"rows": rows, "leaves": leaves, "rounds": rounds, "extra": extra, "gpu_use_dp": res}))


if __name__ == "__main__":
    main()
