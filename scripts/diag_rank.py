"""CPU vs GPU split-by-split comparison of a LambdaRank run (diagnostic; GPU needed).

usage: diag_rank.py <lambdarank_target> [extra k=v params...]
Prints every split (tree, split index) whose feature or threshold differs between
the host learner and the HIP learner, and the correlation of the raw predictions.
"""
import sys

import numpy as np

sys.path.insert(0, ".")
import lambdagap_amd as lgb  # noqa: E402
from lambdagap_amd.utils import make_ranking  # noqa: E402


def splits(node, out):
    if "split_index" in node:
        out.append((node["split_index"], node["split_feature"], round(node["threshold"], 6),
                    round(node["split_gain"], 6), node["internal_count"]))
        splits(node["left_child"], out)
        splits(node["right_child"], out)
    return out


def main():
    target = sys.argv[1]
    extra = dict(kv.split("=") for kv in sys.argv[2:])
    X, y, sizes = make_ranking(300, num_features=20, seed=3)
    y = (y >= 3).astype(np.float32)
    params = {"objective": "lambdarank", "lambdarank_target": target, "num_leaves": 15, "verbosity": -1,
              "lambdarank_truncation_level": 10, **extra}
    bc = lgb.train({**params, "device_type": "cpu"}, lgb.Dataset(X, y, group=sizes), 3)
    bg = lgb.train({**params, "device_type": "gpu"}, lgb.Dataset(X, y, group=sizes), 3)
    for i, (a, b) in enumerate(zip(bc.dump_model()["tree_info"], bg.dump_model()["tree_info"])):
        sa, sb = sorted(splits(a["tree_structure"], [])), sorted(splits(b["tree_structure"], []))
        for x, z in zip(sa, sb):
            if x[1:3] != z[1:3]:
                print("tree", i, "cpu", x, "gpu", z)
    pc, pg = bc.predict(X, raw_score=True), bg.predict(X, raw_score=True)
    print("corr", np.corrcoef(pc, pg)[0, 1])


if __name__ == "__main__":
    main()
