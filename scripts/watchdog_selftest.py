#!/usr/bin/env python3
"""Collective watchdog self-test on one GPU.

Builds a one-rank RCCL communicator, forces the data-parallel device learner
(its tree growth then waits through the watchdog) and sets the collective
timeout far below one tree's duration (LGAP_COMM_TIMEOUT_S): the watchdog must
abort the communicator and raise instead of waiting. Prints one JSON line.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    os.environ["LGAP_COMM_TIMEOUT_S"] = os.environ.get("LGAP_COMM_TIMEOUT_S", "1e-9")
    os.environ["LGAP_FORCE_DEVICE_DP"] = "1"
    import lambdagap_amd as lgb
    from lambdagap_amd.parallel import distributed as d

    uid = d.get_unique_id()
    d._check(d._LIB.LGBM_DeviceCommInit(d._c_str(uid), ctypes.c_int64(len(uid)), ctypes.c_int(1), ctypes.c_int(0),
                                        ctypes.c_int(0)))
    rng = np.random.default_rng(5)
    X = rng.standard_normal((400000, 16))
    y = (X[:, 0] + 0.3 * rng.standard_normal(len(X)) > 0).astype(float)
    params = {"objective": "binary", "num_leaves": 63, "device_type": "gpu", "verbosity": -1}
    out = {"raised": False, "message": ""}
    try:
        lgb.train(params, lgb.Dataset(X, y, params=params), 3)
    except lgb.basic.LightGBMError as e:
        out = {"raised": True, "message": str(e)}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
