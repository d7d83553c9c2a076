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

__all__ = ["group_layout", "group_bins", "device_histogram", "device_sample_rows", "booster_gradients"]


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
