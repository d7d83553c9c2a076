"""Direct numerics tests of the frontier engine's production kernels.

k_f_hist (src/device/frontier_kernels.hip) is compared bin for bin with a float64 ``index_add``
histogram of the same rows (the plain PyTorch/NumPy reference of the op), in every accumulation
mode: MODE 0 fixed point (512 and 1024 threads, many LDS tiles), MODE 1 (gpu_use_dp), MODE 2 / 3
integer levels (use_quantized_grad, 64- and 32-bit LDS bins), 4-bit rows (max_bin <= 15) and
``tile.direct`` global accumulation (a group too wide for the LDS budget). Several row subsets go
through ONE launch, as the expansions of a frontier round do.

k_f_partition is compared with the host learner's stable partition (SerialTreeLearner::Split's
predicate, reference data_partition.hpp:101) for several parents in one launch: numerical splits
with NaN / zero missing handling both ways, and a categorical split.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(rng, n=40_000, nf=10, max_bin=255, cat=True):
    X = rng.standard_normal((n, nf))
    X[rng.random(n) < 0.05, 1] = np.nan          # NaN missing values
    X[rng.random(n) < 0.3, 2] = 0.0              # zero-heavy column
    if cat:
        X[:, 3] = rng.integers(0, 20, n)         # categorical
    y = (X[:, 0] + 0.3 * rng.standard_normal(n) > 0).astype(float)
    return X, y


def _expected(ops, ds, g, h, subsets):
    """float64 index_add of (g, h) into the group-bin histogram (group bin 0, every feature of the
    group at its most frequent bin, is implicit and stays 0, as in the kernels)."""
    _, tb, _, starts = ops.group_layout(ds)
    bins = ops.group_bins(ds).astype(np.int64)
    out = []
    for rows in subsets:
        hist = np.zeros((tb, 2))
        b = bins[rows]
        for gi in range(b.shape[1]):
            nz = b[:, gi] != 0
            idx = starts[gi] + b[nz, gi]
            np.add.at(hist[:, 0], idx, g[rows][nz])
            np.add.at(hist[:, 1], idx, h[rows][nz])
        out.append(hist)
    return np.stack(out), bins


def _subsets(rng, n):
    return [np.sort(rng.choice(n, m, replace=False)).astype(np.int32) for m in (1, 777, 5_000, 20_000)] + \
           [np.arange(n, dtype=np.int32)]


CASES = {
    "fixed_point_1024": ({}, {"LGAP_KERNEL": "fhist_threads=1024"}),
    "fixed_point_512_many_tiles": ({}, {"LGAP_KERNEL": "fhist_threads=512,hist_lds_kb=16"}),
    "fp64": ({"gpu_use_dp": True}, {}),
    "quantized_lds64": ({"use_quantized_grad": True, "num_grad_quant_bins": 4}, {"LGAP_KERNEL": "quant_lds32=0"}),
    "quantized_lds32": ({"use_quantized_grad": True, "num_grad_quant_bins": 16}, {"LGAP_KERNEL": "quant_lds32=1"}),
    "four_bit_rows": ({"max_bin": 15}, {}),
    "direct_tiles": ({"max_bin": 3000, "min_data_in_bin": 1}, {"LGAP_KERNEL": "hist_lds_kb=16"}),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_frontier_histogram_matches_index_add(lgb, gpu_required, rng, monkeypatch, case):
    from lambdagap_amd import ops

    params, env = CASES[case]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cat = case not in ("direct_tiles", "four_bit_rows")  # (4-bit rows: every group <= 16 bins)
    X, y = _data(rng, cat=cat)
    if case == "direct_tiles":
        X[:, 4] = rng.integers(0, 2900, len(X))  # one feature of ~2900 bins in a 16-bit group
    base = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "device_type": "gpu"}
    base.update(params)
    ds = lgb.Dataset(X, y, params=base, categorical_feature=[3] if cat else "auto").construct()
    n = len(y)
    g = rng.standard_normal(n).astype(np.float32)
    h = rng.uniform(0.05, 0.3, n).astype(np.float32)
    subsets = _subsets(rng, n)
    got, levels = ops.frontier_histogram(ds, g, h, subsets, base)
    if params.get("use_quantized_grad"):
        # integer level sums: exactly the index_add of the kernel's own levels
        want, _ = _expected(ops, ds, levels[:, 0].astype(np.float64), levels[:, 1].astype(np.float64), subsets)
        np.testing.assert_array_equal(got, want)
        assert np.abs(levels[:, 0]).max() <= params["num_grad_quant_bins"] // 2
        return
    want, _ = _expected(ops, ds, g.astype(np.float64), h.astype(np.float64), subsets)
    counts, _ = _expected(ops, ds, np.ones(n), np.ones(n), subsets)
    if params.get("gpu_use_dp"):
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-9)
        return
    # MODE 0: each row rounded once at its block's scale 2^bg >= 2^29 / (block rows * max|v|)
    for e, rows in enumerate(subsets):
        tol_g = counts[e, :, 0] * len(rows) * np.abs(g).max() * 2.0 ** -29 + 1e-12
        tol_h = counts[e, :, 0] * len(rows) * np.abs(h).max() * 2.0 ** -29 + 1e-12
        assert np.all(np.abs(got[e, :, 0] - want[e, :, 0]) <= tol_g), (case, e)
        assert np.all(np.abs(got[e, :, 1] - want[e, :, 1]) <= tol_h), (case, e)
    # and the error is far below the bound in practice (no misplaced row)
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("part_iters", ["4", "8", "16"])
def test_frontier_partition_matches_host(lgb, gpu_required, rng, monkeypatch, part_iters):
    from lambdagap_amd import ops

    monkeypatch.setenv("LGAP_KERNEL", f"part_iters={part_iters}")
    X, y = _data(rng, n=60_000)
    base = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "device_type": "gpu"}
    ds = lgb.Dataset(X, y, params=base, categorical_feature=[3]).construct()
    n = len(y)
    # disjoint parents of very different sizes (one row; a tile boundary; most of the data)
    perm = rng.permutation(n)
    cuts = [0, 1, 1 + 4096, 1 + 4096 + 9_000, 1 + 4096 + 9_000 + 777, n]
    subsets = [np.sort(perm[a:b]).astype(np.int32) for a, b in zip(cuts[:-1], cuts[1:])]
    nb = [ds.feature_num_bin(f) for f in range(X.shape[1])]
    splits = [
        (0, nb[0] // 2, False, None),
        (1, nb[1] // 3, True, None),   # NaN rows go left
        (1, nb[1] // 3, False, None),  # NaN rows go right
        (2, 1, True, None),            # zero-missing handling
        (3, 0, False, [1, 4, 5, 9, 13]),  # categorical bins to the left
    ]
    dev_rows, dev_left, host_rows, host_left = ops.frontier_partition(ds, subsets, splits, base)
    np.testing.assert_array_equal(dev_left, host_left)
    # the device writes each parent's lefts from the front in row order and its rights from the
    # back (so a right child's list is the host's in reverse): the same children, both stable
    off = np.cumsum([0] + [len(s) for s in subsets])
    for e, s in enumerate(subsets):
        seg, ref, nl = dev_rows[off[e]:off[e + 1]], host_rows[off[e]:off[e + 1]], dev_left[e]
        np.testing.assert_array_equal(seg[:nl], ref[:nl])
        np.testing.assert_array_equal(seg[nl:][::-1], ref[nl:])
        assert np.array_equal(np.sort(seg), s)  # nothing lost or duplicated


# gain tolerance: fp64-equivalent and integer-level accumulation are exact up to summation order;
# the default fixed point rounds each row once (a gain is a difference of squared sums, so its
# absolute error follows the root's scale: ~1e-5 here)
SCAN_CASES = {
    "fixed_point": ({}, 2e-5),
    "fp64": ({"gpu_use_dp": True}, 1e-9),
    # (quantized: the device sums integer levels x the scale in fp64, the host the fp32 de-quantized
    # values the learner keeps in gh: ~1e-7 apart)
    "quantized": ({"use_quantized_grad": True, "num_grad_quant_bins": 16}, 1e-6),
    # (the scan logic cases accumulate fp64-equivalent: their direction / threshold ties are exact)
    "missing_zero": ({"zero_as_missing": True, "gpu_use_dp": True}, 1e-9),
    "regularised": ({"lambda_l1": 0.5, "lambda_l2": 2.0, "min_data_in_leaf": 300, "max_delta_step": 0.7,
                     "gpu_use_dp": True}, 1e-9),
    "max_bin_63": ({"max_bin": 63, "gpu_use_dp": True}, 1e-9),
}


@pytest.mark.parametrize("case", sorted(SCAN_CASES))
def test_frontier_scan_matches_host_split_math(lgb, gpu_required, rng, case):
    """k_f_scan (numerical scans both directions with NaN / zero missing values, categorical one-hot
    and ctr-sorted scans, most-frequent-bin reconstruction from the leaf sums) against the host
    learner's split_math.h scans of the exact fp64 histogram of the same rows: the same features
    are splittable, with the same threshold, default direction and left count, and gains within
    the accumulation's precision."""
    from lambdagap_amd import ops

    params, rtol = SCAN_CASES[case]
    X, y = _data(rng)
    X[:, 5] = rng.integers(0, 3, len(y))            # one-hot categorical
    base = {"objective": "binary", "num_leaves": 31, "verbosity": -1, "device_type": "gpu", "cat_smooth": 5}
    base.update(params)
    ds = lgb.Dataset(X, y, params=base, categorical_feature=[3, 5]).construct()
    n = len(y)
    p = 1.0 / (1.0 + np.exp(-0.3 * rng.standard_normal(n)))
    g = (p - y).astype(np.float32)
    h = (p * (1.0 - p)).astype(np.float32)
    dev, ref = ops.frontier_scan(ds, g, h, base)
    np.testing.assert_array_equal(dev[:, 6], ref[:, 6])
    assert ref[:, 6].sum() >= 6, ref[:, 6]                   # most features have a split
    ok = ref[:, 6] > 0
    np.testing.assert_allclose(dev[ok, 0], ref[ok, 0], rtol=rtol, atol=5 * rtol)   # gain
    np.testing.assert_array_equal(dev[ok, 2], ref[ok, 2])                       # left count
    np.testing.assert_array_equal(dev[ok, 7], ref[ok, 7])                       # categorical thresholds
    num = ok & (ref[:, 7] == 0)
    np.testing.assert_array_equal(dev[num, 1], ref[num, 1])                     # threshold bin
    np.testing.assert_array_equal(dev[num, 3], ref[num, 3])                     # default direction
    np.testing.assert_allclose(dev[ok, 4:6], ref[ok, 4:6], rtol=rtol, atol=5 * rtol)      # left sums
