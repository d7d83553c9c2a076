"""Trees of the host learner vs the device learner with the host GOSS sample: first differing node."""
import sys
import os
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lambdagap_amd as lgb  # noqa: E402
from lambdagap_amd.utils import make_higgs_like  # noqa: E402

X, y = make_higgs_like(60000, seed=21)
base = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "min_data_in_leaf": 20, "seed": 1,
        "deterministic": True, "data_sample_strategy": "goss", "learning_rate": 0.5,
        "device_sampling": len(sys.argv) > 1}


def walk(a, b, path=""):
    if ("split_index" in a) != ("split_index" in b):
        return f"{path}: leaf/internal mismatch"
    if "split_index" in a:
        if (a["split_feature"], a["threshold"]) != (b["split_feature"], b["threshold"]):
            return f"{path}: split {a['split_feature']}@{a['threshold']:.5f} cnt {a['internal_count']} vs " \
                   f"{b['split_feature']}@{b['threshold']:.5f} cnt {b['internal_count']}"
        return walk(a["left_child"], b["left_child"], path + "L") or walk(a["right_child"], b["right_child"], path + "R")
    if abs(a["leaf_value"] - b["leaf_value"]) > 1e-3 or a["leaf_count"] != b["leaf_count"]:
        return f"{path}: leaf {a['leaf_value']:.5f}/{a['leaf_count']} vs {b['leaf_value']:.5f}/{b['leaf_count']}"
    return None


bs = {}
for dev in ("cpu", "gpu"):
    p = dict(base, device_type=dev)
    bs[dev] = lgb.train(p, lgb.Dataset(X, y, params=p), 4)
tc, tg = bs["cpu"].dump_model()["tree_info"], bs["gpu"].dump_model()["tree_info"]
for i in range(len(tc)):
    print("tree", i, walk(tc[i]["tree_structure"], tg[i]["tree_structure"]), flush=True)
