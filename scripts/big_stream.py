#!/usr/bin/env python3
"""The BASELINE's largest configuration on ONE MI355X: synthetic 100M x 500 regression with EFB +
GOSS, tree_learner=voting on a one-rank RCCL communicator (the per-rank share of the 8-GPU run is
12.5M rows; here one GPU holds all 100M).

No 200 GB host float matrix is ever built. The rows are streamed:
  1. a 1M-row sample chunk builds the reference Dataset (bin mappers, EFB bundles);
  2. LGBM_DatasetCreateByReference sizes the 100M-row dataset, and LGBM_DatasetPushRowsWithMetadata
     bins every further chunk into it on the host (OpenMP), one chunk of floats alive at a time;
  3. the HIP learner uploads the packed rows once (row-major + group-major copies) and trains.
Chunks are drawn on the GPU with torch (the same distribution as utils.make_regression: 20 dense
normal columns, 480 columns 10% dense, target = X w + sin(x0) x1 + noise) and copied to the host.

Reference: c_api.h:177-323 (streaming push), config.h:730-734 (two_round: bins from a sample).

    python scripts/big_stream.py --rows 100000000 --steps 10 --warmup 2

Prints one JSON line: HBM footprint, setup time (generation, push, upload), it/s, held-out l2.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def gen_chunk(torch, n, nf, seed, w):
    """n rows of the make_regression distribution, drawn on the GPU (float32, row-major)."""
    dev = w.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    dense = min(20, nf)
    x = torch.randn((n, nf), generator=g, device=dev, dtype=torch.float32)
    if nf > dense:
        keep = torch.rand((n, nf - dense), generator=g, device=dev) < 0.1
        x[:, dense:] *= keep
    y = x @ w + torch.sin(x[:, 0]) * x[:, 1] + 0.1 * torch.randn((n,), generator=g, device=dev)
    return x.cpu().numpy(), y.cpu().numpy().astype(np.float32)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--features", type=int, default=500)
    ap.add_argument("--chunk", type=int, default=2_000_000)
    ap.add_argument("--sample-rows", type=int, default=1_000_000)
    ap.add_argument("--valid-rows", type=int, default=200_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--learner", choices=["serial", "voting"], default="voting")
    ap.add_argument("--device", default="gpu", help="cpu: a plumbing check of the streaming path (no GPU)")
    args = ap.parse_args()

    import torch

    import lambdagap_amd as lgb
    from lambdagap_amd.basic import _LIB, _c_str, _check
    from lambdagap_amd.models import preset
    from lambdagap_amd.parallel import device_synchronize
    from lambdagap_amd.parallel import distributed as dd

    gpu = args.device == "gpu"
    if args.learner == "voting" and gpu:
        uid = dd.get_unique_id()
        _check(_LIB.LGBM_DeviceCommInit(_c_str(uid), ctypes.c_int64(len(uid)), ctypes.c_int(1), ctypes.c_int(0),
                                        ctypes.c_int(0)))
        # (one machine trains serial, as in the reference: keep the voting learner's path)
        os.environ["LGAP_FORCE_DEVICE_DP"] = "voting"
    params = preset("regression_goss", verbosity=-1, metric="l2", device_type=args.device)
    if args.learner == "voting":
        params["tree_learner"] = "voting"
    nf = args.features
    w = torch.randn((nf,), generator=torch.Generator().manual_seed(1234), dtype=torch.float32) / np.sqrt(nf)
    if gpu:
        w = w.cuda()
    mem = torch.cuda.mem_get_info if gpu else (lambda: (0, 0))
    sync = device_synchronize if gpu else (lambda: None)
    free0, total = mem()
    t_all = time.time()
    t = time.time()
    Xs, ys = gen_chunk(torch, args.sample_rows, nf, 1, w)
    ref = lgb.Dataset(Xs, ys, params=dict(params, device_binning=False), free_raw_data=False).construct()
    t_ref = time.time() - t
    print(f"# reference dataset from {args.sample_rows} sample rows in {t_ref:.1f} s", file=sys.stderr, flush=True)
    out = ctypes.c_void_p()
    _check(_LIB.LGBM_DatasetCreateByReference(ref.handle, ctypes.c_int64(args.rows), ctypes.byref(out)))
    t_gen = t_push = 0.0
    for s0 in range(0, args.rows, args.chunk):
        n = min(args.chunk, args.rows - s0)
        t = time.time()
        X, y = gen_chunk(torch, n, nf, 100 + s0 // args.chunk, w)
        t_gen += time.time() - t
        t = time.time()
        _check(_LIB.LGBM_DatasetPushRowsWithMetadata(out, X.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(0),
                                                     ctypes.c_int32(n), ctypes.c_int32(nf), ctypes.c_int32(s0),
                                                     y.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), None, None,
                                                     None, ctypes.c_int32(0)))
        t_push += time.time() - t
        del X, y
        if (s0 // args.chunk) % 10 == 0:
            print(f"# pushed {s0 + n} rows (gen {t_gen:.1f} s, push {t_push:.1f} s)", file=sys.stderr, flush=True)
    if gpu:
        torch.cuda.empty_cache()
    streamed = lgb.Dataset(None, params=dict(params, device_binning=False))
    streamed.handle = out
    streamed._predictor = None
    t = time.time()
    booster = lgb.Booster(params, streamed)
    sync()
    t_upload = time.time() - t
    setup_s = time.time() - t_all
    free1, _ = mem()
    print(f"# booster on {booster.device_name()} in {t_upload:.1f} s; HBM used {(free0 - free1) / 2**30:.1f} GiB",
          file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        booster.update()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        booster.update()
        print(f"# iteration {i}", file=sys.stderr, flush=True)
    sync()
    el = time.perf_counter() - t0
    free2, _ = mem()
    Xv, yv = gen_chunk(torch, args.valid_rows, nf, 99, w)
    pv = booster.predict(Xv)
    res = {
        "config": f"regression_goss {args.rows} x {nf}, EFB + GOSS, tree_learner={args.learner} (1 rank)",
        "device": booster.device_name(),
        "rows": args.rows, "features": nf,
        "it_s": round(args.steps / el, 3), "ms_per_iter": round(1000 * el / args.steps, 2),
        "steps": args.steps, "warmup": args.warmup,
        "setup_s": round(setup_s, 1), "ref_s": round(t_ref, 1), "gen_s": round(t_gen, 1), "push_s": round(t_push, 1),
        "upload_s": round(t_upload, 1),
        "hbm_used_gib_after_setup": round((free0 - free1) / 2**30, 2),
        "hbm_used_gib_training": round((free0 - free2) / 2**30, 2),
        "hbm_total_gib": round(total / 2**30, 1),
        "valid_l2": float(np.mean((pv - yv) ** 2)), "valid_var": float(np.var(yv)),
        "data": "synthetic (GPU-drawn chunks, streamed)",
    }
    print(json.dumps(res), flush=True)
    del booster
    if args.learner == "voting" and gpu:
        dd.free_device_comm()
    return 0


if __name__ == "__main__":
    sys.exit(main())
