"""Kernel-level entry points of the native library.

These expose single HIP kernels (histogram construction, gradients) and the
packed bin layout they consume, so numerics can be checked against a plain
PyTorch / NumPy reference of the same op (tests/test_gpu_kernels.py).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from ..basic import _LIB, Booster, Dataset, _check

__all__ = ["group_layout", "group_bins", "device_histogram", "device_sample_rows", "booster_gradients",
           "frontier_histogram", "frontier_partition"]


def group_layout(ds: Dataset) -> Tuple[int, int, int, np.ndarray]:
    """(num_groups, num_total_bin, bin_width_bytes, hist_start[num_groups]) of a constructed Dataset."""
    ds.construct()
    ng, tb, bw = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    _check(_LIB.LGBM_DatasetGetGroupLayout(ds.handle, ctypes.byref(ng), ctypes.byref(tb), ctypes.byref(bw), None))
    starts = np.zeros(max(ng.value, 1), dtype=np.int32)
    _check(_LIB.LGBM_DatasetGetGroupLayout(ds.handle, ctypes.byref(ng), ctypes.byref(tb), ctypes.byref(bw),
                                           starts.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
    return ng.value, tb.value, bw.value, starts[:ng.value]


def group_bins(ds: Dataset) -> np.ndarray:
    """[num_data, num_groups] uint16 packed group bins (0 = every feature of the group at its most frequent bin)."""
    ng = group_layout(ds)[0]
    out = np.zeros((ds.num_data(), ng), dtype=np.uint16)
    _check(_LIB.LGBM_DatasetGetGroupBins(ds.handle, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))))
    return out


def device_histogram(ds: Dataset, grad: np.ndarray, hess: np.ndarray, rows: Optional[np.ndarray] = None
                     ) -> np.ndarray:
    """[num_total_bin, 2] (sum_grad, sum_hess) histogram built by the HIP kernel on the GPU."""
    ds.construct()
    tb = group_layout(ds)[1]
    g = np.ascontiguousarray(grad, dtype=np.float32)
    h = np.ascontiguousarray(hess, dtype=np.float32)
    out = np.zeros(2 * tb, dtype=np.float64)
    if rows is not None:
        r = np.ascontiguousarray(rows, dtype=np.int32)
        rp, n = r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), r.size
    else:
        rp, n = None, ds.num_data()
    _check(_LIB.LGBM_DeviceHistogram(ds.handle, g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                     h.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), rp, ctypes.c_int32(n),
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
    return out.reshape(tb, 2)


_SAMPLE_MODES = {"bagging": 1, "balanced": 2, "goss": 3}


def device_sample_rows(mode: str, grad: np.ndarray, hess: np.ndarray, label: Optional[np.ndarray] = None,
                       num_class: int = 1, fraction: float = 1.0, pos_fraction: float = 1.0,
                       neg_fraction: float = 1.0, top_rate: float = 0.2, other_rate: float = 0.1,
                       bagging_seed: int = 3, goss_seed: int = 0, rounds: int = 1
                       ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Run the HIP bagging / GOSS sampling kernels once (``rounds`` re-bags for bagging).

    Returns (kept rows ascending, grad, hess) where GOSS has scaled the sampled rows."""
    g = np.array(grad, dtype=np.float32, copy=True).ravel()
    h = np.array(hess, dtype=np.float32, copy=True).ravel()
    n = g.size // num_class
    lab = None if label is None else np.ascontiguousarray(label, dtype=np.float32)
    rows = np.zeros(max(n, 1), dtype=np.int32)
    cnt = ctypes.c_int32(0)
    fp = ctypes.POINTER(ctypes.c_float)
    _check(_LIB.LGBM_DeviceSampleRows(
        ctypes.c_int(_SAMPLE_MODES[mode]), ctypes.c_int32(n), ctypes.c_int(num_class), g.ctypes.data_as(fp),
        h.ctypes.data_as(fp), None if lab is None else lab.ctypes.data_as(fp), ctypes.c_double(fraction),
        ctypes.c_double(pos_fraction), ctypes.c_double(neg_fraction), ctypes.c_double(top_rate),
        ctypes.c_double(other_rate), ctypes.c_int(bagging_seed), ctypes.c_uint32(goss_seed), ctypes.c_int(rounds),
        rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.byref(cnt)))
    return rows[:cnt.value].copy(), g, h


def booster_gradients(booster: Booster) -> Tuple[np.ndarray, np.ndarray]:
    """Gradients / hessians of the booster's last round (class-major), read back from the device."""
    n = ctypes.c_int64(0)
    _check(_LIB.LGBM_BoosterGetGradients(booster.handle, ctypes.byref(n), None, None))
    g = np.zeros(n.value, dtype=np.float32)
    h = np.zeros(n.value, dtype=np.float32)
    _check(_LIB.LGBM_BoosterGetGradients(booster.handle, ctypes.byref(n), g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                         h.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return g, h


def _param_str(params: Optional[dict]) -> bytes:
    return " ".join(f"{k}={v}" for k, v in (params or {}).items()).encode()


def _subsets(subsets):
    rows = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int32) for s in subsets]), dtype=np.int32)
    offsets = np.zeros(len(subsets) + 1, dtype=np.int32)
    offsets[1:] = np.cumsum([len(s) for s in subsets])
    return rows, offsets


def frontier_histogram(ds: Dataset, grad: np.ndarray, hess: np.ndarray, subsets, params: Optional[dict] = None
                       ) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """One launch of the frontier engine's production histogram kernel (k_f_hist) over several row
    subsets at once, one expansion each, with a device learner set up by ``params``.

    Returns ([k, num_total_bin, 2] sums at the kernel's fixed-point scale -- integer level sums under
    use_quantized_grad --, and for quantized training the per-row levels as (g_level, h_level))."""
    ds.construct()
    tb = group_layout(ds)[1]
    rows, offsets = _subsets(subsets)
    k = len(subsets)
    g = np.ascontiguousarray(grad, dtype=np.float32)
    h = np.ascontiguousarray(hess, dtype=np.float32)
    out = np.zeros(k * tb * 2, dtype=np.float64)
    levels = np.zeros(ds.num_data(), dtype=np.uint16)
    i32 = ctypes.POINTER(ctypes.c_int32)
    _check(_LIB.LGBM_DeviceTestFrontierHist(
        ds.handle, ctypes.c_char_p(_param_str(params)), g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
        h.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), rows.ctypes.data_as(i32), offsets.ctypes.data_as(i32),
        ctypes.c_int(k), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
        levels.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))))
    lv = None
    if (params or {}).get("use_quantized_grad"):
        lv = np.stack([(levels >> 8).astype(np.uint8).view(np.int8).astype(np.int64),
                       (levels & 0xFF).astype(np.int64)], axis=1)
    return out.reshape(k, tb, 2), lv


def frontier_scan(ds: Dataset, grad: np.ndarray, hess: np.ndarray, params: Optional[dict] = None
                  ) -> Tuple[np.ndarray, np.ndarray]:
    """The frontier engine's production split scan (k_f_scan) of the root round over all rows, next
    to the host learner's split_math.h scan of the same rows' exact histogram.

    Returns (device, host) arrays [num_features, 8]: gain, threshold, left count, default_left,
    left sum g, left sum h, valid (a split exists), categorical thresholds."""
    ds.construct()
    nf = ds.num_feature()
    g = np.ascontiguousarray(grad, dtype=np.float32)
    h = np.ascontiguousarray(hess, dtype=np.float32)
    out = np.zeros(nf * 8, dtype=np.float64)
    ref = np.zeros(nf * 8, dtype=np.float64)
    dp = ctypes.POINTER(ctypes.c_double)
    _check(_LIB.LGBM_DeviceTestFrontierScan(
        ds.handle, ctypes.c_char_p(_param_str(params)), g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
        h.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), out.ctypes.data_as(dp), ref.ctypes.data_as(dp)))
    return out.reshape(nf, 8), ref.reshape(nf, 8)


def frontier_partition(ds: Dataset, subsets, splits, params: Optional[dict] = None):
    """One launch of the frontier engine's production partition kernel (k_f_partition) over several
    parents at once. ``splits``: per parent (inner feature, threshold bin, default_left, categorical
    bins or None). Returns (device children lists, device left counts, host learner's lists, host
    left counts); each parent's list holds its lefts in order, then its rights."""
    ds.construct()
    rows, offsets = _subsets(subsets)
    k = len(subsets)
    feats = np.array([s[0] for s in splits], dtype=np.int32)
    thr = np.array([s[1] for s in splits], dtype=np.int32)
    dleft = np.array([int(s[2]) for s in splits], dtype=np.int32)
    bits = np.zeros((k, 32), dtype=np.uint32)  # kMaxCatWords (split_math.h) words per parent
    for e, s in enumerate(splits):
        for b in (s[3] if len(s) > 3 and s[3] is not None else []):
            bits[e, b >> 5] |= np.uint32(1 << (b & 31))
    out_rows = np.zeros(max(rows.size, 1), dtype=np.int32)
    exp_rows = np.zeros(max(rows.size, 1), dtype=np.int32)
    out_left = np.zeros(k, dtype=np.int32)
    exp_left = np.zeros(k, dtype=np.int32)
    i32 = ctypes.POINTER(ctypes.c_int32)
    _check(_LIB.LGBM_DeviceTestFrontierPartition(
        ds.handle, ctypes.c_char_p(_param_str(params)), rows.ctypes.data_as(i32), offsets.ctypes.data_as(i32),
        ctypes.c_int(k), feats.ctypes.data_as(i32), thr.ctypes.data_as(i32), dleft.ctypes.data_as(i32),
        bits.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), out_rows.ctypes.data_as(i32),
        out_left.ctypes.data_as(i32), exp_rows.ctypes.data_as(i32), exp_left.ctypes.data_as(i32)))
    return out_rows[:rows.size], out_left, exp_rows[:rows.size], exp_left
