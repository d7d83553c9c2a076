#!/usr/bin/env python3
"""Multi-rank rehearsal of the parallel HIP learners (data / feature / voting) on ONE GPU.

Launched with ``torchrun --standalone --nproc-per-node P`` (P ranks share
cuda:0). The device learner's collectives are staged through host memory over
gloo (``LGAP_DEVICE_DP_TRANSPORT=host``) so that everything the 8-GPU RCCL run
depends on besides RCCL itself is exercised with P > 1 ranks: row sharding
with ``pre_partition``, distributed bin finding, root-sum and histogram
all-reduce, global leaf counts, identical split decisions on every rank, and
the score / metric bookkeeping. The same ranks then train the host
data-parallel learner on the same bins; both models must agree.

Rank 0 prints one JSON line.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch.distributed as dist

    import lambdagap_amd as lgb
    from lambdagap_amd.parallel import shard_range
    from lambdagap_amd.parallel.torch_network import init_torch_network

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group(backend="gloo", rank=rank, world_size=world)
    init_torch_network()
    os.environ["LGAP_DEVICE_DP_TRANSPORT"] = "host"
    n = int(os.environ.get("DP_ROWS", "120000"))
    rng = np.random.default_rng(11)
    X = rng.standard_normal((n, 10))
    X[rng.random(X.shape) < 0.03] = np.nan
    y = ((np.nan_to_num(X[:, 0]) - 0.8 * np.nan_to_num(X[:, 2]) + 0.4 * np.nan_to_num(X[:, 5]) ** 2
          + 0.3 * rng.standard_normal(n)) > 0.3).astype(float)
    learner = os.environ.get("DP_LEARNER", "data")
    # data parallel: each rank holds a row shard; feature parallel: every rank holds all rows
    a, b = shard_range(n, rank, world) if learner in ("data", "voting") else (0, n)
    # l2 regression: unit hessians make every histogram hessian sum and count estimate exact,
    # so no min_data / min_hessian boundary can flip between the fixed-point device sums
    # and the host's doubles; any model difference is then a transport or split-sync bug
    objective = os.environ.get("DP_OBJECTIVE", "regression")
    base = {"objective": objective, "num_leaves": 31, "verbosity": -1, "seed": 1, "min_data_in_leaf": 20,
            "tree_learner": learner, "num_machines": world, "pre_partition": True, "deterministic": True,
            "top_k": int(os.environ.get("DP_TOPK", "20"))}
    # extra options (JSON), e.g. extra_trees / cegb_penalty_split on the voting learner
    base.update(json.loads(os.environ.get("DP_EXTRA", "{}")))
    if os.environ.get("DP_QUANTIZED") == "1":
        # quantized gradients: packed level sums (one accumulator word per bin) all-reduced
        base.update({"use_quantized_grad": True, "num_grad_quant_bins": 4})
    ds = lgb.Dataset(X[a:b], y[a:b], params=dict(base, device_type="cpu"), free_raw_data=False).construct()
    models = {}
    devs = os.environ.get("DP_DEVICES", "gpu,cpu").split(",")
    for dev in devs:
        models[dev] = lgb.train(dict(base, device_type=dev), ds, 10, keep_training_booster=True)
    first = models[devs[0]]
    name = first.device_name()
    text = first.model_to_string()
    texts = [None] * world
    dist.all_gather_object(texts, text)
    pg, pc = first.predict(X), models[devs[-1]].predict(X)
    def splits(node, out):
        if "split_index" in node:
            out.append((node["split_feature"], round(node["threshold"], 6), node["split_gain"],
                        node["internal_count"]))
            splits(node["left_child"], out)
            splits(node["right_child"], out)
        return out

    ta = [splits(t["tree_structure"], []) for t in first.dump_model()["tree_info"]]
    tb = [splits(t["tree_structure"], []) for t in models[devs[-1]].dump_model()["tree_info"]]
    same = 0
    while same < min(len(ta), len(tb)) and [x[:2] for x in ta[same]] == [x[:2] for x in tb[same]]:
        same += 1
    if rank == 0 and os.environ.get("DP_DIAG"):
        for i, (u, v) in enumerate(zip(ta, tb)):
            if [x[:2] for x in u] != [x[:2] for x in v]:
                print("first differing tree", i, file=sys.stderr)
                for x, z in zip(u, v):
                    print("  ", x, z, file=sys.stderr)
                break
    if rank == 0:
        from sklearn.metrics import roc_auc_score

        print(json.dumps({"world": world, "device_name": name,
                          "ranks_identical": all(t == texts[0] for t in texts),
                          "num_trees": first.num_trees(),
                          "max_abs_diff_vs_cpu_dp": float(np.max(np.abs(pg - pc))),
                          "mean_abs_diff_vs_cpu_dp": float(np.mean(np.abs(pg - pc))),
                          "identical_leading_trees": same,
                          "auc_gpu": float(roc_auc_score(y, pg)), "auc_cpu": float(roc_auc_score(y, pc))}),
              flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
