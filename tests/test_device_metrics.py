"""AUC / average precision / NDCG@k / MAP@k / precision@k evaluated where the score lives.

Host path: the tie-aware AUC loop over a parallel sort (reference binary_metric.hpp:159-268,
Common::ParallelSort at :200). Device path (src/device/metric_kernels.hip): radix sort by score,
deterministic reduce-by-key over tied scores and a group scan for AUC / AP; a segmented stable
sort per query and one wave per query for the query metrics. The device values must equal the
host metric's (LGAP_DEVICE_METRICS=0) on the same scores within 1e-12.
"""
import numpy as np
import pytest


def _metric_values(lgb, X, y, params, rounds, valid=None, **ds_kw):
    evals = {}
    ds = lgb.Dataset(X, y, params=params, **ds_kw)
    sets, names = [ds], ["train"]
    if valid is not None:
        Xv, yv, vkw = valid
        sets.append(lgb.Dataset(Xv, yv, reference=ds, params=params, **vkw))
        names.append("valid")
    lgb.train(params, ds, rounds, valid_sets=sets, valid_names=names,
              callbacks=[lgb.record_evaluation(evals)])
    return evals


def _auc_ap_reference(y, s, w):
    from sklearn.metrics import average_precision_score, roc_auc_score

    return roc_auc_score(y, s, sample_weight=w), average_precision_score(y, s, sample_weight=w)


@pytest.mark.parametrize("weighted", [False, True])
def test_host_auc_parallel_sort_matches_sklearn(lgb, rng, weighted):
    """200k rows with heavy ties (scores rounded to 3 decimals): the parallel-sort AUC and
    average precision equal sklearn's tie-aware values."""
    n = 200_000
    s = np.round(rng.standard_normal(n), 3)
    y = (s + rng.standard_normal(n) > 0).astype(float)
    w = rng.uniform(0.5, 2.0, n) if weighted else None
    X = rng.standard_normal((n, 2))
    params = {"objective": "binary", "metric": ["auc", "average_precision"], "verbosity": -1}
    booster = lgb.Booster(params, lgb.Dataset(X, y, init_score=s, weight=w, params=params))
    ev = {m: v for _, m, v, _ in booster.eval_train()}  # the init scores, before any tree
    auc, ap = _auc_ap_reference(y, s, w)
    assert ev["auc"] == pytest.approx(auc, rel=1e-10)
    assert ev["average_precision"] == pytest.approx(ap, rel=1e-10)


def _ranking_data(rng, nq=300, max_len=40):
    sizes = rng.integers(1, max_len, nq)
    n = int(sizes.sum())
    X = rng.standard_normal((n, 5))
    rel = X[:, 0] + 0.5 * rng.standard_normal(n)
    y = np.digitize(rel, [-0.5, 0.5, 1.2]).astype(float)
    return X, y, sizes


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
def test_device_auc_ap_match_host(lgb, gpu_required, rng, weighted, monkeypatch):
    """Training and validation AUC / average precision on the device score equal the host
    metric on the same scores (ties included: the first iteration's scores take few values)."""
    n, nv = 60_000, 20_000
    X = rng.standard_normal((n, 6))
    y = (X[:, 0] + rng.standard_normal(n) > 0).astype(float)
    Xv = rng.standard_normal((nv, 6))
    yv = (Xv[:, 0] + rng.standard_normal(nv) > 0).astype(float)
    w = rng.uniform(0.2, 3.0, n) if weighted else None
    wv = rng.uniform(0.2, 3.0, nv) if weighted else None
    params = {"objective": "binary", "metric": ["auc", "average_precision"], "num_leaves": 7,
              "device_type": "gpu", "verbosity": -1, "seed": 3, "deterministic": True}
    dev = _metric_values(lgb, X, y, params, 4, valid=(Xv, yv, {"weight": wv}), weight=w)
    monkeypatch.setenv("LGAP_DEVICE_METRICS", "0")
    host = _metric_values(lgb, X, y, params, 4, valid=(Xv, yv, {"weight": wv}), weight=w)
    for name in ("train", "valid"):
        for m in ("auc", "average_precision"):
            np.testing.assert_allclose(dev[name][m], host[name][m], rtol=1e-12, atol=1e-12)
    auc, ap = _auc_ap_reference(yv, lgb.train(params, lgb.Dataset(X, y, weight=w, params=params), 4).predict(Xv), wv)
    assert dev["valid"]["auc"][-1] == pytest.approx(auc, rel=1e-9)
    assert dev["valid"]["average_precision"][-1] == pytest.approx(ap, rel=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["ndcg", "map", "precision"])
@pytest.mark.parametrize("query_weights", [False, True])
def test_device_query_metrics_match_host(lgb, gpu_required, rng, metric, query_weights, monkeypatch):
    """NDCG@k / MAP@k / precision@k (eval_at out of order, k beyond some query lengths) on the
    device score equal the host metric on the same scores."""
    X, y, sizes = _ranking_data(rng)
    Xv, yv, sv = _ranking_data(rng, nq=120)
    params = {"objective": "lambdarank", "metric": metric, "eval_at": [5, 1, 3, 20], "num_leaves": 7,
              "device_type": "gpu", "verbosity": -1, "seed": 1, "deterministic": True, "min_data_in_leaf": 5}
    kw, vkw = {"group": sizes}, {"group": sv}
    if query_weights:
        # per-row weights, constant inside a query: the metric's query weights
        kw["weight"] = np.repeat(rng.uniform(0.5, 2.0, len(sizes)), sizes)
        vkw["weight"] = np.repeat(rng.uniform(0.5, 2.0, len(sv)), sv)
    dev = _metric_values(lgb, X, y, params, 3, valid=(Xv, yv, vkw), **kw)
    monkeypatch.setenv("LGAP_DEVICE_METRICS", "0")
    host = _metric_values(lgb, X, y, params, 3, valid=(Xv, yv, vkw), **kw)
    assert set(dev["valid"]) == set(host["valid"]) and len(dev["valid"]) == 4
    for name in ("train", "valid"):
        for m in host[name]:
            np.testing.assert_allclose(dev[name][m], host[name][m], rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("objective", ["multiclass", "multiclassova"])
@pytest.mark.parametrize("top_k", [1, 2])
@pytest.mark.parametrize("weighted", [False, True])
def test_device_multiclass_metrics_match_host(lgb, gpu_required, rng, objective, top_k, weighted, monkeypatch):
    """multi_logloss / multi_error@k on the class-major device score (k_multi_metric_partial, row
    loss shared with the host through lgap/pointwise_metric.h MultiRowLoss; softmax and one-vs-all
    sigmoid outputs) equal the host metric on the same scores."""
    n, nv, k = 20000, 5000, 4
    X, Xv = rng.standard_normal((n, 6)), rng.standard_normal((nv, 6))

    def lab(X):
        z = np.stack([X[:, 0], X[:, 1] - 0.5 * X[:, 2], 0.7 * X[:, 3], -X[:, 0]], axis=1)
        return np.argmax(z + 0.8 * rng.standard_normal(z.shape), axis=1).astype(float)

    y, yv = lab(X), lab(Xv)
    kw = {"weight": rng.uniform(0.5, 2.0, n)} if weighted else {}
    vkw = {"weight": rng.uniform(0.5, 2.0, nv)} if weighted else {}
    params = {"objective": objective, "num_class": k, "metric": ["multi_logloss", "multi_error"],
              "multi_error_top_k": top_k, "num_leaves": 7, "device_type": "gpu", "verbosity": -1, "seed": 2,
              "deterministic": True}
    dev = _metric_values(lgb, X, y, params, 3, valid=(Xv, yv, vkw), **kw)
    monkeypatch.setenv("LGAP_DEVICE_METRICS", "0")
    host = _metric_values(lgb, X, y, params, 3, valid=(Xv, yv, vkw), **kw)
    for name in ("train", "valid"):
        assert set(dev[name]) == set(host[name]) and len(host[name]) == 2
        for m in host[name]:
            np.testing.assert_allclose(dev[name][m], host[name][m], rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("custom_weights", [False, True])
def test_device_auc_mu_matches_host(lgb, gpu_required, rng, weighted, custom_weights, monkeypatch):
    """auc_mu on the device (per class pair: rows of the two classes scored by the weight-vector
    projection, then the binary AUC kernels) equals the host metric on the same scores."""
    n, nv, k = 15000, 4000, 5
    X, Xv = rng.standard_normal((n, 6)), rng.standard_normal((nv, 6))

    def lab(X):
        z = np.stack([X[:, 0], X[:, 1] - 0.5 * X[:, 2], 0.7 * X[:, 3], -X[:, 0], X[:, 4] * X[:, 5]], axis=1)
        return np.argmax(z + 0.8 * rng.standard_normal(z.shape), axis=1).astype(float)

    y, yv = lab(X), lab(Xv)
    kw = {"weight": rng.uniform(0.5, 2.0, n)} if weighted else {}
    vkw = {"weight": rng.uniform(0.5, 2.0, nv)} if weighted else {}
    params = {"objective": "multiclass", "num_class": k, "metric": ["auc_mu"], "num_leaves": 7,
              "device_type": "gpu", "verbosity": -1, "seed": 2, "deterministic": True}
    if custom_weights:
        w = rng.uniform(0.5, 1.5, (k, k))
        np.fill_diagonal(w, 0.0)
        params["auc_mu_weights"] = [float(x) for x in w.ravel()]
    dev = _metric_values(lgb, X, y, params, 3, valid=(Xv, yv, vkw), **kw)
    monkeypatch.setenv("LGAP_DEVICE_METRICS", "0")
    host = _metric_values(lgb, X, y, params, 3, valid=(Xv, yv, vkw), **kw)
    for name in ("train", "valid"):
        np.testing.assert_allclose(dev[name]["auc_mu"], host[name]["auc_mu"], rtol=1e-12, atol=1e-12)
