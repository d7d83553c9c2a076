"""Numerics of single HIP kernels against a plain PyTorch fp32 reference of the same op."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch_histogram(bins, starts, tb, g, h, rows=None):
    import torch

    b = torch.from_numpy(bins.astype(np.int64))
    gg = torch.from_numpy(g.astype(np.float32))
    hh = torch.from_numpy(h.astype(np.float32))
    if rows is not None:
        r = torch.from_numpy(rows.astype(np.int64))
        b, gg, hh = b[r], gg[r], hh[r]
    idx = b + torch.from_numpy(starts.astype(np.int64))[None, :]
    mask = b != 0  # group bin 0 is implicit (reconstructed from leaf totals)
    flat = idx[mask]
    gsum = torch.zeros(tb, dtype=torch.float32).index_add_(0, flat, gg[:, None].expand_as(b)[mask])
    hsum = torch.zeros(tb, dtype=torch.float32).index_add_(0, flat, hh[:, None].expand_as(b)[mask])
    return torch.stack([gsum, hsum], 1).numpy()


@pytest.mark.parametrize("max_bin", [15, 63, 255, 1023])
def test_histogram_kernel_matches_torch(lgb, gpu_required, rng, max_bin):
    from lambdagap_amd import ops

    n, f = 60000, 17
    X = rng.standard_normal((n, f)).astype(np.float32)
    X[:, 3] = np.where(rng.random(n) < 0.8, 0.0, X[:, 3])  # sparse-ish column
    X[:, 5] = np.round(X[:, 5] * 2)  # few distinct values
    ds = lgb.Dataset(X, params={"max_bin": max_bin, "verbosity": -1}).construct()
    ng, tb, bw, starts = ops.group_layout(ds)
    bins = ops.group_bins(ds)
    g = rng.standard_normal(n).astype(np.float32)
    h = rng.random(n).astype(np.float32) + 0.1
    ref = _torch_histogram(bins, starts, tb, g, h)
    out = ops.device_histogram(ds, g, h)
    np.testing.assert_allclose(out, ref, rtol=2e-4, atol=2e-3)
    rows = np.sort(rng.choice(n, 7777, replace=False)).astype(np.int32)
    ref2 = _torch_histogram(bins, starts, tb, g, h, rows)
    out2 = ops.device_histogram(ds, g, h, rows)
    np.testing.assert_allclose(out2, ref2, rtol=2e-4, atol=1e-3)


def test_binary_gradient_kernel_matches_torch(lgb, gpu_required, rng):
    import torch
    from lambdagap_amd import ops

    n = 50000
    X = rng.standard_normal((n, 5)).astype(np.float32)
    y = (rng.random(n) < 0.4).astype(np.float32)
    init = rng.standard_normal(n).astype(np.float64)
    params = {"objective": "binary", "device_type": "gpu", "verbosity": -1, "num_leaves": 7}
    b = lgb.Booster(params, lgb.Dataset(X, y, init_score=init, params=params))
    b.update()
    g, h = ops.booster_gradients(b)
    s = torch.from_numpy(init.astype(np.float32))
    p = torch.sigmoid(s)
    tg = (p - torch.from_numpy(y)).numpy()
    th = (p * (1 - p)).numpy()
    np.testing.assert_allclose(g, tg, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(h, th, rtol=1e-4, atol=1e-5)


def test_softmax_gradient_kernel_matches_torch(lgb, gpu_required, rng):
    import torch
    from lambdagap_amd import ops

    n, k = 30000, 4
    X = rng.standard_normal((n, 6)).astype(np.float32)
    y = rng.integers(0, k, n).astype(np.float32)
    init = rng.standard_normal((n, k))
    params = {"objective": "multiclass", "num_class": k, "device_type": "gpu", "verbosity": -1, "num_leaves": 7}
    b = lgb.Booster(params, lgb.Dataset(X, y, init_score=init, params=params))
    b.update()
    g, h = ops.booster_gradients(b)
    s = torch.from_numpy(init.astype(np.float32))
    p = torch.softmax(s, 1)
    onehot = torch.nn.functional.one_hot(torch.from_numpy(y.astype(np.int64)), k).float()
    tg = (p - onehot).T.reshape(-1).numpy()
    th = (k / (k - 1.0) * p * (1 - p)).T.reshape(-1).numpy()
    np.testing.assert_allclose(g, tg, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(h, th, rtol=1e-4, atol=1e-5)


def _torch_lambdarank_ndcg(score, label, sizes, k=30, sigmoid=1.0):
    """fp32 torch reference of the ndcg target (norm=true), pairs over sorted ranks."""
    import torch

    gains = (2.0 ** torch.arange(32, dtype=torch.float64)) - 1
    G = np.zeros(len(score), np.float32)
    H = np.zeros(len(score), np.float32)
    start = 0
    for c in sizes:
        s = torch.tensor(score[start:start + c], dtype=torch.float64)
        l = torch.tensor(label[start:start + c], dtype=torch.float64)
        order = torch.tensor(sorted(range(c), key=lambda i: (-float(s[i]), i)))
        ideal = torch.sort(l, descending=True).values[:k]
        disc = 1.0 / torch.log2(torch.arange(c, dtype=torch.float64) + 2)
        maxdcg = float((gains[ideal.long()] * disc[:len(ideal)]).sum())
        inv = 1.0 / maxdcg if maxdcg > 0 else 0.0
        best, worst = float(s[order[0]]), float(s[order[-1]])
        lam = torch.zeros(c, dtype=torch.float64)
        hes = torch.zeros(c, dtype=torch.float64)
        tot = 0.0
        for i in range(min(c - 1, k)):
            for j in range(i + 1, c):
                di, dj = int(order[i]), int(order[j])
                if l[di] == l[dj]:
                    continue
                hi_r, lo_r = (i, j) if l[di] > l[dj] else (j, i)
                hi, lo = int(order[hi_r]), int(order[lo_r])
                ds = float(s[hi] - s[lo])
                dp = float(gains[int(l[hi])] - gains[int(l[lo])]) * abs(float(disc[hi_r] - disc[lo_r])) * inv
                if best != worst:
                    dp /= 0.01 + abs(ds)
                pl = 1.0 / (1.0 + np.exp(sigmoid * ds))
                ph = pl * (1 - pl)
                pl *= -sigmoid * dp
                ph *= sigmoid * sigmoid * dp
                lam[lo] -= pl
                lam[hi] += pl
                hes[lo] += ph
                hes[hi] += ph
                tot -= 2 * pl
        if tot > 0:
            f = np.log2(1 + tot) / tot
            lam *= f
            hes *= f
        G[start:start + c] = lam.numpy()
        H[start:start + c] = hes.numpy()
        start += c
    return G, H


def test_lambdarank_gradient_kernel_matches_torch(lgb, gpu_required, rng):
    from lambdagap_amd import ops

    nq = 60
    sizes = rng.integers(2, 40, nq)
    n = int(sizes.sum())
    X = rng.standard_normal((n, 5)).astype(np.float32)
    y = rng.integers(0, 5, n).astype(np.float32)
    init = rng.standard_normal(n)
    params = {"objective": "lambdarank", "device_type": "gpu", "verbosity": -1, "num_leaves": 7,
              "lambdarank_target": "ndcg"}
    b = lgb.Booster(params, lgb.Dataset(X, y, group=sizes, init_score=init, params=params))
    b.update()
    g, h = ops.booster_gradients(b)
    tg, th = _torch_lambdarank_ndcg(init, y, sizes)
    # the kernel uses the 1M-entry sigmoid lookup table of the host objective
    np.testing.assert_allclose(g, tg, rtol=2e-3, atol=2e-4)
    np.testing.assert_allclose(h, th, rtol=2e-3, atol=2e-4)
