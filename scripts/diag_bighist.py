#!/usr/bin/env python3
"""Diagnostic: device histogram of a wide dataset past 8M rows vs a numpy reference of the same
group bins (all rows, and a random subset), reporting the worst bins."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import lambdagap_amd as lgb  # noqa: E402
from lambdagap_amd import ops  # noqa: E402
from lambdagap_amd.models import preset  # noqa: E402
from lambdagap_amd.utils import make_regression  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8_500_000
X, y = make_regression(rows, num_features=500, seed=7)
p = preset("regression_goss", device_type="cpu", verbosity=-1)
ds = lgb.Dataset(X, y, params=p, free_raw_data=True).construct()
del X
ng, tb, bw, starts = ops.group_layout(ds)
print("groups", ng, "total bins", tb, "bin width", bw, flush=True)
bins = ops.group_bins(ds)
rng = np.random.default_rng(3)
g = rng.standard_normal(rows).astype(np.float32)
h = np.ones(rows, dtype=np.float32)


def ref_hist(sel):
    out = np.zeros((tb, 2))
    b = bins if sel is None else bins[sel]
    gg = g if sel is None else g[sel]
    hh = h if sel is None else h[sel]
    for k in range(ng):
        col = b[:, k].astype(np.int64)
        m = col != 0
        out[starts[k]:starts[k] + col.max() + 1, 0] += np.bincount(col[m], weights=gg[m])[:col.max() + 1] if m.any() else 0
        out[starts[k]:starts[k] + col.max() + 1, 1] += np.bincount(col[m], weights=hh[m])[:col.max() + 1] if m.any() else 0
    return out


for name, sel in (("all", None), ("subset", np.sort(rng.choice(rows, rows // 7, replace=False)).astype(np.int32)),
                  ("tail", np.arange(rows - 300000, rows, dtype=np.int32))):
    ref = ref_hist(sel)
    out = ops.device_histogram(ds, g, h, sel)
    err = np.abs(out - ref)
    worst = np.argsort(-err[:, 0])[:5]
    print(name, "max |dg|", float(err[:, 0].max()), "max |dh|", float(err[:, 1].max()),
          "worst bins", [(int(i), float(out[i, 0]), float(ref[i, 0]), float(out[i, 1]), float(ref[i, 1])) for i in worst],
          flush=True)
