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


@pytest.mark.parametrize("n", [300_007, 1_234_567])
def test_histogram_constant_hessian_is_exact(lgb, gpu_required, rng, n):
    """Constant hessians (l2, quantile, ...) must histogram EXACTLY: the fixed-point scales are
    powers of two, so h = 1 quantizes without rounding and every bin's hessian is its row
    count. A non-power-of-two scale biased every row alike, and parent - smaller subtraction
    carried the root's error into small deep leaves (diverging l2 training at ~8M rows)."""
    from lambdagap_amd import ops

    X = rng.standard_normal((n, 6)).astype(np.float32)
    ds = lgb.Dataset(X, params={"max_bin": 63, "verbosity": -1}).construct()
    ng, tb, bw, starts = ops.group_layout(ds)
    bins = ops.group_bins(ds)
    g = rng.standard_normal(n).astype(np.float32)
    h = np.ones(n, dtype=np.float32)
    for rows in (None, np.sort(rng.choice(n, n // 3, replace=False)).astype(np.int32)):
        out = ops.device_histogram(ds, g, h, rows)
        b = bins if rows is None else bins[rows]
        for k in range(ng):
            cnt = np.bincount(b[:, k], minlength=64)
            nb = (starts[k + 1] if k + 1 < ng else tb) - starts[k]
            np.testing.assert_array_equal(out[starts[k] + 1:starts[k] + nb, 1], cnt[1:nb])


@pytest.mark.parametrize("dtype,max_bin", [(np.float32, 255), (np.float64, 63), (np.float32, 1023)])
def test_device_binning_matches_host_bit_for_bit(lgb, gpu_required, rng, dtype, max_bin):
    """Device feature binning (ValueToBin + EFB bundle packing on the GPU) produces exactly the
    host packer's group bins: NaN (missing as NaN and as zero), exact zeros and values under the
    zero threshold, categorical codes (incl. unseen / negative), and sparse bundled columns."""
    from lambdagap_amd import ops

    n = 120_000
    X = rng.standard_normal((n, 12))
    X[rng.random(n) < 0.1, 0] = np.nan                  # NaN -> missing bin
    X[rng.random(n) < 0.3, 1] = 0.0                     # zero-heavy
    X[rng.random(n) < 0.05, 1] = 1e-40                  # below the zero threshold
    X[:, 2] = rng.integers(-1, 40, n)                   # categorical (negative -> bin 0)
    X[rng.random(n) < 0.02, 2] = np.nan
    X[:, 3] = np.round(X[:, 3] * 3)                     # few distinct values
    for j in range(6, 12):                              # sparse columns EFB bundles together
        X[rng.random(n) < 0.93, j] = 0.0
    X[rng.random(n) < 0.05, 5] = np.nan
    X = X.astype(dtype)
    params = {"max_bin": max_bin, "verbosity": -1, "categorical_feature": [2], "enable_bundle": True,
              "use_missing": True}
    host = lgb.Dataset(X, params=dict(params, device_type="cpu")).construct()
    dev = lgb.Dataset(X, params=dict(params, device_type="gpu")).construct()
    assert ops.group_layout(host)[:3] == ops.group_layout(dev)[:3]
    np.testing.assert_array_equal(ops.group_bins(dev), ops.group_bins(host))
    # zero_as_missing routes zeros through the missing path
    host_z = lgb.Dataset(X, params=dict(params, device_type="cpu", zero_as_missing=True)).construct()
    dev_z = lgb.Dataset(X, params=dict(params, device_type="gpu", zero_as_missing=True)).construct()
    np.testing.assert_array_equal(ops.group_bins(dev_z), ops.group_bins(host_z))


def test_device_binned_dataset_trains_like_host_binned(lgb, gpu_required, rng):
    """The HIP learner adopts the device-binned rows (no second upload) and grows the same model
    as from host-binned rows."""
    from lambdagap_amd.utils import make_higgs_like

    X, y = make_higgs_like(200_000, seed=9)
    p = {"objective": "binary", "num_leaves": 31, "device_type": "gpu", "verbosity": -1}
    b_dev = lgb.train(p, lgb.Dataset(X, y, params=p), 5)
    b_host = lgb.train(p, lgb.Dataset(X, y, params=dict(p, device_binning=False)), 5)
    np.testing.assert_array_equal(b_dev.predict(X[:5000], raw_score=True), b_host.predict(X[:5000], raw_score=True))
    # the device packer ran (phase timer), not a silent host fallback
    import os
    import subprocess
    import sys
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import lambdagap_amd as lgb; "
            "X = np.random.default_rng(1).standard_normal((50000, 8)).astype(np.float32); "
            "lgb.Dataset(X, params={'device_type': 'gpu', 'verbosity': -1}).construct(); "
            "print(lgb.phase_timer_report())") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, LGAP_TIMETAG="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Device::PackRows" in r.stdout + r.stderr


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


LTR_TARGETS = ["ndcg", "lambdaloss-ndcg", "lambdaloss-ndcg-plus-plus", "bndcg", "lambdaloss-bndcg",
               "lambdaloss-bndcg-plus-plus", "precision", "arpk", "lambdaloss-arp1", "lambdaloss-arp2", "ranknet",
               "bin-ranknet", "lambdagap-s", "lambdagap-x", "lambdagap-s-plus", "lambdagap-x-plus",
               "lambdagap-s-plus-plus", "lambdagap-x-plus-plus"]


@pytest.mark.parametrize("target", LTR_TARGETS)
@pytest.mark.parametrize("variant", ["plain", "long_queries_positions"])
def test_lambdarank_gradient_kernel_all_targets(lgb, gpu_required, rng, target, variant):
    """Device lambdas / hessians of every LambdaGap target against the host objective (the
    correctness oracle of the 18 targets) on the same scores: short queries in LDS, queries over
    2048 documents in global scratch, and position-biased (unbiased LTR) scores."""
    from lambdagap_amd import ops

    if variant == "plain":
        sizes = rng.integers(2, 60, 80)
    else:
        sizes = np.array([30, 2500, 7, 4100, 90], dtype=np.int64)
    n = int(sizes.sum())
    X = rng.standard_normal((n, 5)).astype(np.float32)
    y = rng.integers(0, 5, n).astype(np.float32)
    if target in ("bndcg", "lambdaloss-bndcg", "lambdaloss-bndcg-plus-plus", "precision", "arpk", "bin-ranknet") or \
            target.startswith("lambdagap"):
        y = (y >= 3).astype(np.float32)
    init = rng.standard_normal(n)
    pos = np.concatenate([np.arange(s) % 7 for s in sizes]).astype(np.int32) if variant != "plain" else None
    grads = {}
    for dev in ("cpu", "gpu"):
        params = {"objective": "lambdarank", "device_type": dev, "verbosity": -1, "num_leaves": 7,
                  "lambdarank_target": target, "lambdarank_truncation_level": 12, "lambdagap_weight": 0.5}
        b = lgb.Booster(params, lgb.Dataset(X, y, group=sizes, init_score=init, position=pos, params=params))
        b.update()
        grads[dev] = ops.booster_gradients(b)
    (gc, hc), (gg, hg) = grads["cpu"], grads["gpu"]
    scale_g, scale_h = np.abs(gc).max() + 1e-12, np.abs(hc).max() + 1e-12
    np.testing.assert_allclose(gg, gc, rtol=1e-4, atol=1e-5 * scale_g)
    np.testing.assert_allclose(hg, hc, rtol=1e-4, atol=1e-5 * scale_h)


def _lcg_bags(n, seed, rounds, decide):
    """Host reference of the bagging streams: Random(seed + b) per 1024-row block, one
    NextFloat per row, continued across re-bags (sample_strategy.cpp / bagging.hpp)."""
    nb = (n + 1023) // 1024
    states = (seed + np.arange(nb, dtype=np.int64)) & 0xFFFFFFFF
    keep = None
    for _ in range(rounds):
        draws = np.zeros((nb, 1024), dtype=np.float32)
        s = states.copy()
        for j in range(1024):
            s = (214013 * s + 2531011) & 0xFFFFFFFF
            draws[:, j] = ((s >> 16) & 0x7FFF).astype(np.float32) / np.float32(32768.0)
        rows_per = np.minimum(1024, n - 1024 * np.arange(nb))
        # each block's stream advances by its own row count
        for b in range(nb):
            t = states[b]
            for _ in range(int(rows_per[b])):
                t = (214013 * t + 2531011) & 0xFFFFFFFF
            states[b] = t
        r = draws.reshape(-1)[:n].astype(np.float64)
        keep = decide(r)
    return np.flatnonzero(keep)


@pytest.mark.parametrize("rounds", [1, 3])
def test_device_bagging_matches_host_streams(lgb, gpu_required, rng, rounds):
    from lambdagap_amd import ops

    n = 50_000 + 123
    g = rng.standard_normal(n).astype(np.float32)
    h = np.ones(n, np.float32)
    rows, _, _ = ops.device_sample_rows("bagging", g, h, fraction=0.37, bagging_seed=11, rounds=rounds)
    ref = _lcg_bags(n, 11, rounds, lambda r: r < 0.37)
    np.testing.assert_array_equal(rows, ref)
    label = (rng.random(n) < 0.3).astype(np.float32)
    rows, _, _ = ops.device_sample_rows("balanced", g, h, label=label, pos_fraction=0.9, neg_fraction=0.2,
                                        bagging_seed=5, rounds=rounds)
    ref = _lcg_bags(n, 5, rounds, lambda r: np.where(label > 0, r < 0.9, r < 0.2))
    np.testing.assert_array_equal(rows, ref)


@pytest.mark.parametrize("num_class", [1, 3])
def test_device_goss_selection(lgb, gpu_required, rng, num_class):
    """Per 4096-row tile: every row with sum_k |g_k h_k| >= the top_k-th largest is kept, exactly
    min(other_k, rest) others are sampled and only those are scaled by (cnt - top_k) / other_k."""
    from lambdagap_amd import ops

    n = 3 * 4096 + 1000
    g = rng.standard_normal(num_class * n).astype(np.float32)
    h = rng.random(num_class * n).astype(np.float32) + 0.1
    g[:50] = 0.0  # ties at zero importance
    top, other = 0.2, 0.1
    rows, g2, h2 = ops.device_sample_rows("goss", g, h, num_class=num_class, top_rate=top, other_rate=other,
                                          goss_seed=99)
    assert np.all(np.diff(rows) > 0)
    imp = np.abs(g * h).reshape(num_class, n).sum(0, dtype=np.float32)
    kept = np.zeros(n, bool)
    kept[rows] = True
    for t0 in range(0, n, 4096):
        sl = slice(t0, min(n, t0 + 4096))
        cnt = sl.stop - sl.start
        top_k, other_k = max(1, int(cnt * top)), int(cnt * other)
        thr = np.sort(imp[sl])[::-1][top_k - 1]
        big = imp[sl] >= thr
        assert kept[sl][big].all()
        sampled = kept[sl] & ~big
        assert sampled.sum() == min(other_k, cnt - big.sum())
        mul = np.float32(cnt - top_k) / np.float32(other_k)
        for k in range(num_class):
            gk, gk2 = g.reshape(num_class, n)[k, sl], g2.reshape(num_class, n)[k, sl]
            np.testing.assert_allclose(gk2[sampled], gk[sampled] * mul, rtol=1e-6)
            np.testing.assert_array_equal(gk2[~sampled], gk[~sampled])


def _torch_xendcg(score, label, sizes, seed, weight=None):
    """rank_xendcg lambdas / hessians (rank_objective.hpp RankXENDCG::GetGradientsForOneQuery) in
    PyTorch fp64, with each query's Random(seed + q) NextFloat draws reproduced."""
    import torch

    g = torch.zeros(len(score), dtype=torch.float64)
    h = torch.zeros(len(score), dtype=torch.float64)
    start = 0
    for q, cnt in enumerate(sizes):
        cnt = int(cnt)
        if cnt > 1:
            s = torch.as_tensor(score[start:start + cnt], dtype=torch.float64)
            rho = torch.softmax(s, 0)
            x = (seed + q) & 0xFFFFFFFF
            draws = []
            for _ in range(cnt):
                x = (214013 * x + 2531011) & 0xFFFFFFFF
                draws.append(float(np.float32((x >> 16) & 0x7FFF) / np.float32(32768.0)))
            params = torch.pow(2.0, torch.as_tensor(label[start:start + cnt]).to(torch.int64).double()) \
                - torch.as_tensor(draws, dtype=torch.float64)
            inv_den = 1.0 / max(1e-15, float(params.sum()))
            t1 = -params * inv_den + rho
            p1 = t1 / (1 - rho)
            t2 = rho * (p1.sum() - p1)
            p2 = t2 / (1 - rho)
            t3 = rho * (p2.sum() - p2)
            g[start:start + cnt] = t1 + t2 + t3
            h[start:start + cnt] = rho * (1 - rho)
        start += cnt
    if weight is not None:
        g, h = g * torch.as_tensor(weight, dtype=torch.float64), h * torch.as_tensor(weight, dtype=torch.float64)
    return g.numpy(), h.numpy()


@pytest.mark.parametrize("weighted", [False, True])
def test_xendcg_gradient_kernel_matches_torch(lgb, gpu_required, rng, weighted):
    from lambdagap_amd import ops

    nq = 80
    sizes = rng.integers(1, 60, nq)
    sizes[3] = 700  # a query wider than the workgroup
    n = int(sizes.sum())
    X = rng.standard_normal((n, 5)).astype(np.float32)
    y = rng.integers(0, 5, n).astype(np.float32)
    w = rng.uniform(0.5, 2.0, n).astype(np.float32) if weighted else None
    init = rng.standard_normal(n)
    params = {"objective": "rank_xendcg", "device_type": "gpu", "verbosity": -1, "num_leaves": 7,
              "objective_seed": 11}
    b = lgb.Booster(params, lgb.Dataset(X, y, group=sizes, init_score=init, weight=w, params=params))
    b.update()
    g, h = ops.booster_gradients(b)
    tg, th = _torch_xendcg(init, y, sizes, 11, w)
    np.testing.assert_allclose(g, tg, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(h, th, rtol=1e-4, atol=1e-6)


def test_xendcg_device_training_matches_host(lgb, gpu_required):
    """Several rounds: the device's per-query LCG states advance exactly like the host's."""
    from lambdagap_amd.utils import make_ranking

    X, y, sizes = make_ranking(300, num_features=20, seed=5)
    params = {"objective": "rank_xendcg", "num_leaves": 15, "verbosity": -1, "objective_seed": 3}
    bc = lgb.train({**params, "device_type": "cpu"}, lgb.Dataset(X, y, group=sizes), 4)
    bg = lgb.train({**params, "device_type": "gpu"}, lgb.Dataset(X, y, group=sizes), 4)
    pc, pg = bc.predict(X, raw_score=True), bg.predict(X, raw_score=True)
    assert np.corrcoef(pc, pg)[0, 1] > 0.999
    close = np.isclose(pg, pc, rtol=5e-3, atol=5e-3)
    assert close.mean() > 0.995, close.mean()
