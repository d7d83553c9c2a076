#!/usr/bin/env python3
"""Single-GPU rehearsal of the data-parallel HIP learner.

Creates a one-rank RCCL communicator, trains with LGAP_FORCE_DEVICE_DP=1 (the
learner then takes the owner-computes distributed path: slab rows folded into the
owner-permuted row, the owner exchange — ncclReduceScatter / ncclAllGather, or the
xGMI in-kernel exchange with LGAP_DP_TRANSPORT=xgmi —, scan of the owned features
from the exchanged rows, global leaf counts from the split records) and compares
against the single-device path on the same data.
Prints one JSON line; tests/test_gpu_learner.py runs this in a subprocess so the
communicator never outlives it.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import lambdagap_amd as lgb
    from lambdagap_amd.parallel import distributed as d

    uid = d.get_unique_id()
    import ctypes

    d._check(d._LIB.LGBM_DeviceCommInit(d._c_str(uid), ctypes.c_int64(len(uid)), ctypes.c_int(1), ctypes.c_int(0),
                                        ctypes.c_int(0)))
    rng = np.random.default_rng(3)
    X = rng.standard_normal((60000, 12))
    X[rng.random(X.shape) < 0.05] = np.nan
    y = ((np.nan_to_num(X[:, 0]) + 0.5 * np.nan_to_num(X[:, 3]) ** 2 + 0.3 * rng.standard_normal(60000)) > 0.4)
    y = y.astype(float)
    params = {"objective": "binary", "num_leaves": 31, "device_type": "gpu", "verbosity": -1, "seed": 1,
              "min_data_in_leaf": 20}
    if os.environ.get("DP_SELFTEST_QUANTIZED") == "1":
        # packed g32|h32 accumulators, one word per bin in the all-reduce
        params.update({"use_quantized_grad": True, "num_grad_quant_bins": 4})
    out = {}
    for mode in ("single", "dp", "dp_serial"):
        os.environ["LGAP_FORCE_DEVICE_DP"] = "0" if mode == "single" else "1"
        # dp: RCCL exchange pipelined with the histogram / scan halves (frontier engine);
        # dp_serial: LGAP_DP_PIPELINE=0, the same exchange in series on the compute stream
        os.environ["LGAP_DP_PIPELINE"] = "0" if mode == "dp_serial" else "1"
        b = lgb.train(params, lgb.Dataset(X, y, params=params), 8, keep_training_booster=True)
        out[mode] = b
    pa, pb = out["single"].predict(X), out["dp"].predict(X)
    ta = [t["tree_structure"].get("split_feature") for t in out["single"].dump_model()["tree_info"]]
    tb = [t["tree_structure"].get("split_feature") for t in out["dp"].dump_model()["tree_info"]]
    pc = out["dp_serial"].predict(X)
    print(json.dumps({"max_abs_diff": float(np.max(np.abs(pa - pb))), "root_features_equal": ta == tb,
                      "pipeline_vs_serial_equal": bool(np.array_equal(pb, pc)),
                      "dp_path": "data-parallel" in out["dp"].device_name(),
                      "dp_name": out["dp"].device_name(),
                      "single_path": "parallel" not in out["single"].device_name(),
                      "num_trees": [out["single"].num_trees(), out["dp"].num_trees()]}), flush=True)
    d.free_device_comm()
    return 0


if __name__ == "__main__":
    sys.exit(main())
