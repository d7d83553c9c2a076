"""Training-engine tests on CPU (themes of the reference's tests/python_package_test/test_engine.py)."""
import json
import os

import numpy as np
import pytest
from sklearn.datasets import make_classification, make_regression
from sklearn.metrics import average_precision_score, log_loss, mean_squared_error, roc_auc_score

DATA = os.path.join(os.path.dirname(__file__), "data")


def _load(name):
    mat = np.loadtxt(os.path.join(DATA, name), dtype=np.float64)
    return mat[:, 1:], mat[:, 0]


def _load_svm(name):
    from sklearn.datasets import load_svmlight_file

    X, y = load_svmlight_file(os.path.join(DATA, name), zero_based=True)
    return X, y


@pytest.fixture(scope="module")
def binary_data():
    X, y = _load("binary.train")
    Xt, yt = _load("binary.test")
    w = np.loadtxt(os.path.join(DATA, "binary.train.weight"))
    return X, y, Xt, yt, w


def test_binary_example(lgb, binary_data):
    X, y, Xt, yt, w = binary_data
    params = {"objective": "binary", "metric": ["binary_logloss", "auc"], "verbosity": -1, "num_leaves": 31,
              "learning_rate": 0.1}
    ds = lgb.Dataset(X, y, weight=w)
    dv = ds.create_valid(Xt, yt)
    evals = {}
    b = lgb.train(params, ds, 50, valid_sets=[dv], valid_names=["test"], callbacks=[lgb.record_evaluation(evals)])
    p = b.predict(Xt)
    assert log_loss(yt, p) < 0.55
    auc = roc_auc_score(yt, p)
    assert auc > 0.78
    # the recorded metric equals sklearn's on the same predictions
    assert abs(evals["test"]["auc"][-1] - auc) < 1e-6
    assert abs(evals["test"]["binary_logloss"][-1] - log_loss(yt, p)) < 1e-6


def test_regression_and_metrics(lgb, rng):
    X, y = make_regression(n_samples=3000, n_features=10, noise=5.0, random_state=1)
    ds = lgb.Dataset(X[:2500], y[:2500])
    dv = ds.create_valid(X[2500:], y[2500:])
    evals = {}
    b = lgb.train({"objective": "regression", "metric": ["l2", "rmse", "l1"], "verbosity": -1}, ds, 60,
                  valid_sets=[dv], callbacks=[lgb.record_evaluation(evals)])
    p = b.predict(X[2500:])
    mse = mean_squared_error(y[2500:], p)
    assert abs(evals["valid_0"]["l2"][-1] - mse) / mse < 1e-6
    assert abs(evals["valid_0"]["rmse"][-1] - np.sqrt(mse)) / np.sqrt(mse) < 1e-6
    assert evals["valid_0"]["l2"][-1] < evals["valid_0"]["l2"][0]


@pytest.mark.parametrize("objective", ["regression_l1", "huber", "fair", "quantile", "mape", "poisson", "gamma",
                                       "tweedie"])
def test_regression_objectives_improve(lgb, rng, objective):
    X = rng.standard_normal((3000, 6))
    mu = np.exp(0.4 * X[:, 0] - 0.3 * X[:, 1])
    if objective in ("poisson",):
        y = rng.poisson(mu).astype(float)
    elif objective in ("gamma", "tweedie"):
        y = rng.gamma(2.0, mu / 2.0) + (objective == "tweedie") * 0.0
    else:
        y = 3 * X[:, 0] - 2 * X[:, 1] ** 2 + rng.standard_normal(3000)
    evals = {}
    ds = lgb.Dataset(X, y)
    b = lgb.train({"objective": objective, "verbosity": -1, "num_leaves": 15}, ds, 30, valid_sets=[ds],
                  callbacks=[lgb.record_evaluation(evals)])
    name, hist = next(iter(evals["training"].items()))
    assert hist[-1] < hist[0], (name, hist[0], hist[-1])
    assert np.all(np.isfinite(b.predict(X)))


def test_cross_entropy_objectives(lgb, rng):
    X = rng.standard_normal((2000, 5))
    y = 1 / (1 + np.exp(-(X[:, 0] - X[:, 1])))
    for obj in ("cross_entropy", "cross_entropy_lambda"):
        evals = {}
        ds = lgb.Dataset(X, y)
        lgb.train({"objective": obj, "verbosity": -1}, ds, 20, valid_sets=[ds], callbacks=[lgb.record_evaluation(evals)])
        hist = next(iter(evals["training"].values()))
        assert hist[-1] < hist[0]


def test_multiclass_example(lgb):
    X, y = _load("multiclass.train")
    Xt, yt = _load("multiclass.test")
    for obj in ("multiclass", "multiclassova"):
        params = {"objective": obj, "num_class": 5, "metric": "multi_logloss", "verbosity": -1}
        evals = {}
        ds = lgb.Dataset(X, y)
        b = lgb.train(params, ds, 30, valid_sets=[ds.create_valid(Xt, yt)], callbacks=[lgb.record_evaluation(evals)])
        p = b.predict(Xt)
        assert p.shape == (len(yt), 5)
        if obj == "multiclass":
            np.testing.assert_allclose(p.sum(1), 1.0, rtol=1e-9)
            assert abs(evals["valid_0"]["multi_logloss"][-1] - log_loss(yt, p, labels=range(5))) < 1e-6
        assert (p.argmax(1) == yt).mean() > 0.4  # sklearn HistGradientBoosting: 0.456 at 30 iters


def test_multi_error_top_k(lgb, rng):
    X = rng.standard_normal((1500, 5))
    y = rng.integers(0, 3, 1500).astype(float)
    evals = {}
    ds = lgb.Dataset(X, y)
    b = lgb.train({"objective": "multiclass", "num_class": 3, "metric": ["multi_error"], "multi_error_top_k": 2,
                   "verbosity": -1}, ds, 5, valid_sets=[ds], callbacks=[lgb.record_evaluation(evals)])
    p = b.predict(X)
    top2 = np.argsort(-p, 1)[:, :2]
    err = 1 - np.mean([y[i] in top2[i] for i in range(len(y))])
    assert abs(evals["training"]["multi_error@2"][-1] - err) < 1e-9


@pytest.fixture(scope="module")
def rank_data():
    X, y = _load_svm("rank.train")
    Xt, yt = _load_svm("rank.test")
    q = np.loadtxt(os.path.join(DATA, "rank.train.query"), dtype=np.int32)
    qt = np.loadtxt(os.path.join(DATA, "rank.test.query"), dtype=np.int32)
    return X, y, q, Xt, yt, qt


def test_lambdarank_example(lgb, rank_data):
    X, y, q, Xt, yt, qt = rank_data
    params = {"objective": "lambdarank", "metric": "ndcg", "eval_at": [1, 3, 5], "verbosity": -1}
    evals = {}
    ds = lgb.Dataset(X, y, group=q)
    dv = ds.create_valid(Xt, yt, group=qt)
    lgb.train(params, ds, 30, valid_sets=[dv], callbacks=[lgb.record_evaluation(evals)])
    ndcg5 = evals["valid_0"]["ndcg@5"]
    assert ndcg5[-1] > 0.6
    assert ndcg5[-1] > ndcg5[0] - 1e-12


TARGETS = ["ndcg", "lambdaloss-ndcg", "lambdaloss-ndcg-plus-plus", "bndcg", "lambdaloss-bndcg",
           "lambdaloss-bndcg-plus-plus", "precision", "arpk", "lambdaloss-arp1", "lambdaloss-arp2", "ranknet",
           "bin-ranknet", "lambdagap-s", "lambdagap-x", "lambdagap-s-plus", "lambdagap-x-plus",
           "lambdagap-s-plus-plus", "lambdagap-x-plus-plus"]


@pytest.mark.parametrize("target", TARGETS)
def test_lambdarank_targets_train(lgb, rank_data, target):
    """Every LambdaGap target trains and improves ranking quality over the initial model."""
    X, y, q, Xt, yt, qt = rank_data
    params = {"objective": "lambdarank", "lambdarank_target": target, "metric": ["ndcg", "precision", "map"],
              "eval_at": [5], "verbosity": -1, "lambdarank_truncation_level": 10, "lambdagap_weight": 0.5}
    evals = {}
    ds = lgb.Dataset(X, y, group=q)
    dv = ds.create_valid(Xt, yt, group=qt)
    b = lgb.train(params, ds, 15, valid_sets=[dv], callbacks=[lgb.record_evaluation(evals)])
    hist = evals["valid_0"]
    assert set(hist) == {"ndcg@5", "precision@5", "map@5"}
    assert max(hist["ndcg@5"]) > 0.45, target
    assert np.all(np.isfinite(b.predict(Xt)))


def test_unknown_lambdarank_target_raises(lgb, rank_data):
    X, y, q, *_ = rank_data
    with pytest.raises(lgb.LightGBMError):
        lgb.train({"objective": "lambdarank", "lambdarank_target": "nope", "verbosity": -1},
                  lgb.Dataset(X, y, group=q), 2)


def test_rank_xendcg(lgb, rank_data):
    X, y, q, Xt, yt, qt = rank_data
    evals = {}
    ds = lgb.Dataset(X, y, group=q)
    lgb.train({"objective": "rank_xendcg", "metric": "ndcg", "eval_at": [3], "verbosity": -1}, ds, 20,
              valid_sets=[ds.create_valid(Xt, yt, group=qt)], callbacks=[lgb.record_evaluation(evals)])
    assert evals["valid_0"]["ndcg@3"][-1] > 0.5


def _ndcg_at(k, y, s, sizes):
    out = []
    start = 0
    for c in sizes:
        yy, ss = y[start:start + c], s[start:start + c]
        order = np.argsort(-ss, kind="stable")
        gains = 2.0 ** yy - 1
        disc = 1.0 / np.log2(np.arange(c) + 2)
        dcg = (gains[order][:k] * disc[:k]).sum()
        idcg = (np.sort(gains)[::-1][:k] * disc[:k]).sum()
        out.append(dcg / idcg if idcg > 0 else 1.0)
        start += c
    return float(np.mean(out))


def test_ndcg_metric_value(lgb, rank_data):
    X, y, q, Xt, yt, qt = rank_data
    evals = {}
    ds = lgb.Dataset(X, y, group=q)
    dv = ds.create_valid(Xt, yt, group=qt)
    b = lgb.train({"objective": "lambdarank", "metric": "ndcg", "eval_at": [3, 10], "verbosity": -1}, ds, 10,
                  valid_sets=[dv], callbacks=[lgb.record_evaluation(evals)])
    s = b.predict(Xt)
    for k in (3, 10):
        assert abs(evals["valid_0"][f"ndcg@{k}"][-1] - _ndcg_at(k, yt, s, qt)) < 1e-6


def test_average_precision_metric(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    evals = {}
    ds = lgb.Dataset(X, y)
    b = lgb.train({"objective": "binary", "metric": "average_precision", "verbosity": -1}, ds, 10,
                  valid_sets=[ds.create_valid(Xt, yt)], callbacks=[lgb.record_evaluation(evals)])
    assert abs(evals["valid_0"]["average_precision"][-1] - average_precision_score(yt, b.predict(Xt))) < 1e-6


def test_early_stopping(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    ds = lgb.Dataset(X, y)
    dv = ds.create_valid(Xt, yt)
    b = lgb.train({"objective": "binary", "metric": "binary_logloss", "verbosity": -1, "learning_rate": 0.5,
                   "num_leaves": 63}, ds, 500, valid_sets=[dv], callbacks=[lgb.early_stopping(5, verbose=False)])
    assert 0 < b.best_iteration < 500
    assert "valid_0" in b.best_score
    assert b.current_iteration() <= b.best_iteration + 5
    # predict defaults to best_iteration
    np.testing.assert_allclose(b.predict(Xt), b.predict(Xt, num_iteration=b.best_iteration))


def test_early_stopping_param_alias(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    ds = lgb.Dataset(X, y)
    b = lgb.train({"objective": "binary", "verbosity": -1, "learning_rate": 0.5, "early_stopping_round": 3,
                   "num_leaves": 63}, ds, 300, valid_sets=[ds.create_valid(Xt, yt)])
    assert b.best_iteration < 300


def test_continue_training(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    params = {"objective": "binary", "verbosity": -1}
    b1 = lgb.train(params, lgb.Dataset(X, y, free_raw_data=False), 10)
    b2 = lgb.train(params, lgb.Dataset(X, y, free_raw_data=False), 10, init_model=b1)
    assert b2.current_iteration() == 20
    full = lgb.train(params, lgb.Dataset(X, y), 20)
    # continuing from 10 trees matches 20 trees trained in one go
    np.testing.assert_allclose(b2.predict(Xt, raw_score=True), full.predict(Xt, raw_score=True), rtol=1e-6,
                               atol=1e-6)


def test_continue_training_constructed_and_file_datasets(lgb, binary_data, tmp_path):
    """Continued training from a pre-constructed Dataset and from a file-backed Dataset must start
    from the init model's scores (reference engine.py -> Dataset._set_predictor), so that 10 + 10
    rounds equal 20 rounds in one go, also in the validation-set metric."""
    X, y, Xt, yt, _ = binary_data
    params = {"objective": "regression", "verbosity": -1, "metric": "l2"}
    full = lgb.train(params, lgb.Dataset(X, y), 20)
    b1 = lgb.train(params, lgb.Dataset(X, y), 10)
    ds = lgb.Dataset(X, y, free_raw_data=False).construct()
    evals = {}
    b2 = lgb.train(params, ds, 10, init_model=b1, valid_sets=[ds.create_valid(Xt, yt)], valid_names=["v"],
                   callbacks=[lgb.record_evaluation(evals)])
    np.testing.assert_allclose(b2.predict(Xt, raw_score=True), full.predict(Xt, raw_score=True), atol=1e-6)
    l2_full = float(np.mean((full.predict(Xt) - yt) ** 2))
    assert abs(evals["v"]["l2"][-1] - l2_full) < 1e-6
    # constructed and raw data freed: the reference raises rather than silently train from zero
    gone = lgb.Dataset(X, y).construct()
    with pytest.raises(lgb.basic.LightGBMError, match="freed raw data"):
        lgb.train(params, gone, 10, init_model=b1)
    # file data: the init score comes from predicting on the file
    path = os.path.join(DATA, "binary.train")
    b1f = lgb.train(params, lgb.Dataset(path), 10)
    b3 = lgb.train(params, lgb.Dataset(path), 10, init_model=b1f)
    full_f = lgb.train(params, lgb.Dataset(path), 20)
    np.testing.assert_allclose(b3.predict(Xt, raw_score=True), full_f.predict(Xt, raw_score=True), atol=1e-6)
    # init model from a saved file
    model_file = str(tmp_path / "m.txt")
    b1.save_model(model_file)
    b4 = lgb.train(params, lgb.Dataset(X, y), 10, init_model=model_file)
    np.testing.assert_allclose(b4.predict(Xt, raw_score=True), full.predict(Xt, raw_score=True), atol=1e-6)


def test_cv_init_model(lgb, binary_data):
    """cv(init_model=...) continues every fold from the model (reference engine.py cv)."""
    X, y, *_ = binary_data
    params = {"objective": "binary", "metric": "binary_logloss", "verbosity": -1}
    b1 = lgb.train(params, lgb.Dataset(X, y), 20)
    cold = lgb.cv(params, lgb.Dataset(X, y), 5, nfold=3, seed=2)
    warm = lgb.cv(params, lgb.Dataset(X, y), 5, nfold=3, seed=2, init_model=b1, return_cvbooster=True)
    assert warm["valid binary_logloss-mean"][0] < cold["valid binary_logloss-mean"][-1]
    assert all(b.current_iteration() == 25 for b in warm["cvbooster"].boosters)


def test_split_importance_counts_positive_gain_only(lgb, binary_data):
    """Split importance counts only splits with positive gain, as gain importance does
    (reference gbdt_model_text.cpp:635-653)."""
    X, y, *_ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 4}, lgb.Dataset(X, y), 3)
    d = b.dump_model()
    gains = {}

    def walk(n):
        if "split_index" in n:
            gains.setdefault(n["split_feature"], []).append(n["split_gain"])
            walk(n["left_child"])
            walk(n["right_child"])

    for t in d["tree_info"]:
        walk(t["tree_structure"])
    split = b.feature_importance("split")
    for f, gs in gains.items():
        assert split[f] == sum(1 for g in gs if g > 0)


def test_cv(lgb, binary_data):
    X, y, *_ = binary_data
    res = lgb.cv({"objective": "binary", "metric": "auc", "verbosity": -1}, lgb.Dataset(X, y), 10, nfold=3,
                 stratified=True, return_cvbooster=True)
    assert len(res["valid auc-mean"]) == 10
    assert res["valid auc-mean"][-1] > 0.75
    assert len(res["cvbooster"].boosters) == 3
    preds = res["cvbooster"].predict(X[:10])
    assert len(preds) == 3


def test_cv_ranking_groups(lgb, rank_data):
    X, y, q, *_ = rank_data
    res = lgb.cv({"objective": "lambdarank", "metric": "ndcg", "eval_at": [3], "verbosity": -1},
                 lgb.Dataset(X, y, group=q), 5, nfold=3)
    assert len(res["valid ndcg@3-mean"]) == 5


def test_reset_parameter_callback(lgb, binary_data):
    X, y, *_ = binary_data
    lrs = [0.1 * (0.9 ** i) for i in range(10)]
    b = lgb.train({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y), 10,
                  callbacks=[lgb.reset_parameter(learning_rate=lrs)])
    assert b.current_iteration() == 10


def test_custom_objective_and_eval(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data

    def logloss_obj(preds, data):
        labels = data.get_label()
        p = 1.0 / (1.0 + np.exp(-preds))
        return p - labels, p * (1 - p)

    def err_eval(preds, data):
        p = 1.0 / (1.0 + np.exp(-preds))
        return "my_error", float(np.mean((p > 0.5) != data.get_label())), False

    ds = lgb.Dataset(X, y)
    evals = {}
    b = lgb.train({"objective": logloss_obj, "verbosity": -1, "boost_from_average": False}, ds, 20,
                  valid_sets=[ds], feval=err_eval, callbacks=[lgb.record_evaluation(evals)])
    builtin = lgb.train({"objective": "binary", "verbosity": -1, "boost_from_average": False}, lgb.Dataset(X, y), 20)
    np.testing.assert_allclose(b.predict(Xt), builtin.predict(Xt, raw_score=True), rtol=1e-4, atol=1e-4)
    assert evals["training"]["my_error"][-1] < 0.3


@pytest.mark.parametrize("boosting", ["dart", "rf", "goss"])
def test_boosting_variants(lgb, binary_data, boosting):
    X, y, Xt, yt, _ = binary_data
    params = {"objective": "binary", "verbosity": -1, "boosting": boosting}
    if boosting == "rf":
        params.update({"bagging_fraction": 0.7, "bagging_freq": 1, "feature_fraction": 0.8})
    b = lgb.train(params, lgb.Dataset(X, y), 20)
    auc = roc_auc_score(yt, b.predict(Xt))
    assert auc > 0.7, (boosting, auc)
    s = b.model_to_string()
    b2 = lgb.Booster(model_str=s)
    np.testing.assert_allclose(b2.predict(Xt), b.predict(Xt), rtol=1e-12)


@pytest.mark.parametrize("extra", [{"bagging_fraction": 0.5, "bagging_freq": 2},
                                   {"pos_bagging_fraction": 0.5, "neg_bagging_fraction": 0.8, "bagging_freq": 1},
                                   {"feature_fraction": 0.5}, {"feature_fraction_bynode": 0.5},
                                   {"extra_trees": True}, {"path_smooth": 2.0}, {"max_depth": 3},
                                   {"lambda_l1": 1.0, "lambda_l2": 1.0, "min_gain_to_split": 0.1},
                                   {"max_delta_step": 0.5}, {"min_data_in_leaf": 100, "min_sum_hessian_in_leaf": 5},
                                   {"max_bin": 15}, {"max_bin_by_feature": [8] * 28},
                                   {"interaction_constraints": [[0, 1, 2], [3, 4, 5, 6]]}])
def test_params_train(lgb, binary_data, extra):
    X, y, Xt, yt, _ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1, **extra}, lgb.Dataset(X, y), 15)
    # interaction constraints restrict the model to features 0-6 (weak on this data)
    floor = 0.58 if "interaction_constraints" in extra else 0.65
    assert roc_auc_score(yt, b.predict(Xt)) > floor
    if "max_depth" in extra:
        for t in b.dump_model()["tree_info"]:
            def depth(n):
                return 0 if "split_index" not in n else 1 + max(depth(n["left_child"]), depth(n["right_child"]))
            assert depth(t["tree_structure"]) <= 3
    if "interaction_constraints" in extra:
        allowed = [set(c) for c in extra["interaction_constraints"]]
        for t in b.dump_model()["tree_info"]:
            def paths(n, acc):
                if "split_index" not in n:
                    yield acc
                    return
                f = n["split_feature"]
                yield from paths(n["left_child"], acc | {f})
                yield from paths(n["right_child"], acc | {f})
            for feats in paths(t["tree_structure"], set()):
                assert any(feats <= a for a in allowed), feats


@pytest.mark.parametrize("method", ["basic", "intermediate", "advanced"])
@pytest.mark.parametrize("penalty", [0.0, 2.0])
def test_monotone_constraints(lgb, rng, method, penalty):
    n = 3000
    X = rng.random((n, 3))
    y = 5 * X[:, 0] - 3 * X[:, 1] + np.sin(10 * X[:, 2]) + 0.3 * rng.standard_normal(n)
    b = lgb.train({"objective": "regression", "monotone_constraints": [1, -1, 0], "verbosity": -1,
                   "monotone_constraints_method": method, "monotone_penalty": penalty}, lgb.Dataset(X, y), 50)
    grid = np.linspace(0, 1, 50)
    base = rng.random((20, 3))
    for row in base:
        for f, sign in ((0, 1), (1, -1)):
            Z = np.repeat(row[None, :], 50, 0)
            Z[:, f] = grid
            p = b.predict(Z)
            assert np.all(sign * np.diff(p) >= -1e-10), f


def test_missing_values(lgb, rng):
    n = 4000
    X = rng.standard_normal((n, 3))
    y = (X[:, 0] > 0).astype(float)
    X[rng.random(n) < 0.3, 0] = np.nan
    y[np.isnan(X[:, 0])] = 1.0  # missing values carry signal
    b = lgb.train({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y), 20)
    p = b.predict(np.array([[np.nan, 0, 0], [-2.0, 0, 0]]))
    assert p[0] > 0.8 and p[1] < 0.2
    # zero_as_missing and use_missing=false train fine
    for kw in ({"zero_as_missing": True}, {"use_missing": False}):
        lgb.train({"objective": "binary", "verbosity": -1, **kw}, lgb.Dataset(X, y), 5)


def test_categorical_features(lgb, rng):
    n = 5000
    cat = rng.integers(0, 20, n)
    X = np.column_stack([cat, rng.standard_normal(n)])
    y = (np.isin(cat, [1, 5, 7, 11, 13]) ^ (X[:, 1] > 1.5)).astype(float)
    for kw in ({"max_cat_to_onehot": 32}, {"max_cat_to_onehot": 4, "cat_smooth": 1, "min_data_per_group": 10}):
        b = lgb.train({"objective": "binary", "verbosity": -1, **kw}, lgb.Dataset(X, y, categorical_feature=[0]), 20)
        p = b.predict(X)
        assert roc_auc_score(y, p) > 0.95
        m = b.dump_model()
        dts = set()

        def walk(node):
            if "split_index" in node:
                dts.add(node["decision_type"])
                walk(node["left_child"])
                walk(node["right_child"])

        for t in m["tree_info"]:
            walk(t["tree_structure"])
        assert "==" in dts


def test_pandas_categorical(lgb, rng):
    import pandas as pd

    n = 2000
    df = pd.DataFrame({"a": pd.Categorical(rng.choice(["x", "y", "z"], n)), "b": rng.standard_normal(n)})
    y = (df["a"] == "y").astype(float) + 0.1 * rng.standard_normal(n)
    b = lgb.train({"objective": "regression", "verbosity": -1}, lgb.Dataset(df, y), 20)
    p = b.predict(df)
    assert np.corrcoef(p, y)[0, 1] > 0.9
    b2 = lgb.Booster(model_str=b.model_to_string())
    assert b2.pandas_categorical == b.pandas_categorical
    np.testing.assert_allclose(b2.predict(df), p)


def test_linear_tree(lgb, rng):
    n = 3000
    X = rng.random((n, 3))
    y = 2 * X[:, 0] + 3 * X[:, 1] + 0.01 * rng.standard_normal(n)
    bl = lgb.train({"objective": "regression", "linear_tree": True, "verbosity": -1, "num_leaves": 4}, lgb.Dataset(X, y),
                   20)
    bc = lgb.train({"objective": "regression", "verbosity": -1, "num_leaves": 4}, lgb.Dataset(X, y), 20)
    assert mean_squared_error(y, bl.predict(X)) < mean_squared_error(y, bc.predict(X))
    bl2 = lgb.Booster(model_str=bl.model_to_string())
    np.testing.assert_allclose(bl2.predict(X), bl.predict(X), rtol=1e-9)


def test_forced_splits(lgb, binary_data, tmp_path):
    X, y, *_ = binary_data
    f = tmp_path / "forced.json"
    f.write_text(json.dumps({"feature": 25, "threshold": 1.3, "left": {"feature": 26, "threshold": 0.85}}))
    b = lgb.train({"objective": "binary", "verbosity": -1, "forcedsplits_filename": str(f)}, lgb.Dataset(X, y), 3)
    for t in b.dump_model()["tree_info"]:
        root = t["tree_structure"]
        assert root["split_feature"] == 25
        assert root["left_child"]["split_feature"] == 26


def test_shap_contrib_sums_to_raw(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y), 10)
    contrib = b.predict(Xt[:200], pred_contrib=True)
    assert contrib.shape == (200, X.shape[1] + 1)
    np.testing.assert_allclose(contrib.sum(1), b.predict(Xt[:200], raw_score=True), rtol=1e-6, atol=1e-8)


def test_pred_leaf(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 7}, lgb.Dataset(X, y), 5)
    leaves = b.predict(Xt[:50], pred_leaf=True)
    assert leaves.shape == (50, 5)
    assert leaves.max() < 7
    # leaf values reproduce the raw score
    raw = np.zeros(50)
    for t in range(5):
        raw += np.array([b.get_leaf_output(t, l) for l in leaves[:, t]])
    np.testing.assert_allclose(raw, b.predict(Xt[:50], raw_score=True), rtol=1e-9, atol=1e-12)


def test_feature_importance(lgb, binary_data):
    X, y, *_ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y), 10)
    split = b.feature_importance("split")
    gain = b.feature_importance("gain")
    assert split.sum() == sum(t["num_leaves"] - 1 for t in b.dump_model()["tree_info"])
    assert gain.sum() > 0
    assert np.argmax(gain) == np.argmax(b.feature_importance("gain", iteration=10))


def test_refit(lgb, binary_data):
    X, y, Xt, yt, _ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y), 10)
    r = b.refit(Xt, yt, decay_rate=0.5)
    assert r.num_trees() == b.num_trees()
    assert not np.allclose(r.predict(Xt), b.predict(Xt))
    assert log_loss(yt, r.predict(Xt)) <= log_loss(yt, b.predict(Xt)) + 1e-3


def test_rollback_and_model_roundtrip(lgb, binary_data, tmp_path):
    X, y, Xt, yt, _ = binary_data
    b = lgb.Booster({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y))
    for _ in range(5):
        b.update()
    p5 = b.predict(Xt)
    b.update()
    b.rollback_one_iter()
    assert b.current_iteration() == 5
    np.testing.assert_allclose(b.predict(Xt), p5, rtol=1e-12)
    path = tmp_path / "model.txt"
    b.save_model(str(path))
    txt = path.read_text()
    assert "version=v4" in txt and "end of trees" in txt and "parameters:" in txt
    b2 = lgb.Booster(model_file=str(path))
    np.testing.assert_allclose(b2.predict(Xt), p5, rtol=1e-12)
    d = b.dump_model()
    assert d["num_class"] == 1 and len(d["tree_info"]) == 5
    assert d["objective"].startswith("binary")


def test_model_to_if_else_compiles(lgb, binary_data, tmp_path):
    import shutil
    import subprocess

    if shutil.which("g++") is None:
        pytest.skip("no C++ compiler")
    X, y, Xt, yt, _ = binary_data
    b = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 7}, lgb.Dataset(X, y), 3)
    code = b.model_to_if_else()
    src = tmp_path / "m.cpp"
    src.write_text(code + """
#include <cstdio>
int main() {
  double x[28]; double out[1];
  while (true) {
    for (int i = 0; i < 28; ++i) if (scanf("%lf", &x[i]) != 1) return 0;
    lambdagap_generated::PredictRaw(x, out);
    printf("%.17g\\n", out[0]);
  }
}
""")
    exe = tmp_path / "m"
    subprocess.run(["g++", "-O1", "-o", str(exe), str(src)], check=True)
    inp = "\n".join(" ".join("%.17g" % v for v in row) for row in Xt[:100])
    res = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True)
    got = np.array([float(v) for v in res.stdout.split()])
    np.testing.assert_allclose(got, b.predict(Xt[:100], raw_score=True), rtol=1e-9, atol=1e-12)


def test_binary_dataset_save_load(lgb, binary_data, tmp_path):
    X, y, Xt, yt, w = binary_data
    ds = lgb.Dataset(X, y, weight=w).construct()
    path = tmp_path / "train.bin"
    ds.save_binary(str(path))
    ds2 = lgb.Dataset(str(path)).construct()
    assert ds2.num_data() == ds.num_data() and ds2.num_feature() == ds.num_feature()
    np.testing.assert_allclose(ds2.get_label(), y)
    np.testing.assert_allclose(ds2.get_weight(), w)
    params = {"objective": "binary", "verbosity": -1}
    b1 = lgb.train(params, lgb.Dataset(X, y, weight=w), 5)
    b2 = lgb.train(params, ds2, 5)
    np.testing.assert_allclose(b1.predict(Xt), b2.predict(Xt), rtol=1e-12)


def test_train_from_text_file(lgb, binary_data):
    X, y, Xt, yt, w = binary_data
    ds = lgb.Dataset(os.path.join(DATA, "binary.train"))
    b = lgb.train({"objective": "binary", "verbosity": -1}, ds, 10)
    bm = lgb.train({"objective": "binary", "verbosity": -1}, lgb.Dataset(X, y, weight=w), 10)
    # the loader picks up binary.train.weight automatically
    np.testing.assert_allclose(b.predict(Xt), bm.predict(Xt), rtol=1e-9)
    np.testing.assert_allclose(b.predict(os.path.join(DATA, "binary.test")), b.predict(Xt), rtol=1e-9)


def test_sparse_input(lgb, rank_data):
    import scipy.sparse as sp

    X, y, q, Xt, yt, qt = rank_data
    Xd = X.toarray()
    b1 = lgb.train({"objective": "lambdarank", "verbosity": -1}, lgb.Dataset(X, y, group=q), 5)
    b2 = lgb.train({"objective": "lambdarank", "verbosity": -1}, lgb.Dataset(Xd, y, group=q), 5)
    b3 = lgb.train({"objective": "lambdarank", "verbosity": -1}, lgb.Dataset(sp.csc_matrix(X), y, group=q), 5)
    p = b2.predict(Xt.toarray())
    np.testing.assert_allclose(b1.predict(Xt), p, rtol=1e-9)
    np.testing.assert_allclose(b3.predict(Xt), p, rtol=1e-9)


def test_goss_and_bagging_by_query(lgb, rank_data):
    X, y, q, *_ = rank_data
    lgb.train({"objective": "lambdarank", "verbosity": -1, "bagging_by_query": True, "bagging_fraction": 0.5,
               "bagging_freq": 1}, lgb.Dataset(X, y, group=q), 5)
    lgb.train({"objective": "lambdarank", "verbosity": -1, "data_sample_strategy": "goss"},
              lgb.Dataset(X, y, group=q), 5)


def test_goss_independent_of_thread_count(lgb):
    """GOSS tiles are fixed (not one block per thread as in the reference): the model does not
    change with num_threads, also when several boosters run in one process."""
    rng = np.random.default_rng(4)
    X = rng.standard_normal((30000, 6))
    y = (X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.standard_normal(30000) > 0.4).astype(float)
    preds = []
    for nt in (1, 3, 1):
        p = {"objective": "binary", "verbosity": -1, "data_sample_strategy": "goss", "learning_rate": 0.5,
             "num_threads": nt, "num_leaves": 15}
        preds.append(lgb.train(p, lgb.Dataset(X, y), 6).predict(X[:2000], raw_score=True))
    np.testing.assert_array_equal(preds[0], preds[1])
    np.testing.assert_array_equal(preds[0], preds[2])


def test_position_bias(lgb, rank_data):
    X, y, q, *_ = rank_data
    pos = np.concatenate([np.arange(c) for c in q]).astype(np.int32) % 10
    b = lgb.train({"objective": "lambdarank", "verbosity": -1, "lambdarank_position_bias_regularization": 0.1},
                  lgb.Dataset(X, y, group=q, position=pos), 5)
    assert np.all(np.isfinite(b.predict(X[:100])))
