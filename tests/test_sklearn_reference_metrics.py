"""Metric-selection, early-stopping and estimator-state expectations of the reference's
scikit-learn tests (/root/reference/tests/python_package_test/test_sklearn.py:
test_metrics, test_multiple_eval_metrics, test_nan_handle, test_first_metric_only,
test_class_weight, test_continue_training_with_model, test_actual_number_of_trees,
test_check_is_fitted), same data, seeds and expected outcomes."""
import itertools

import numpy as np
import pytest
from sklearn.datasets import load_breast_cancer, load_digits, make_regression
from sklearn.model_selection import train_test_split

import lambdagap_amd as lgb


def make_synthetic_regression(n_samples=100, n_features=4, n_informative=2, random_state=42):
    return make_regression(n_samples=n_samples, n_features=n_features, n_informative=n_informative,
                           random_state=random_state)


def custom_dummy_obj(y_true, y_pred):
    return np.ones(y_true.shape), np.ones(y_true.shape)


def constant_metric(y_true, y_pred):
    return "error", 0, False


_decreasing = itertools.count(0, -1)


def decreasing_metric(y_true, y_pred):
    return "decreasing_metric", next(_decreasing), False


P = {"n_estimators": 2, "verbose": -1}

# (estimator, constructor kwargs, eval_metric or "-", expected metric names of "training")
REGRESSION_CASES = [
    ({}, "-", {"l2"}),
    ({"metric": "mape"}, "-", {"mape"}),
    ({"metric": "None"}, "-", None),
    ({}, "mape", {"l2", "mape"}),
    ({"metric": "gamma"}, "mape", {"gamma", "mape"}),
    ({"metric": "gamma"}, ["l2", "mape"], {"gamma", "l2", "mape"}),
    ({"objective": "regression_l1"}, "-", {"l1"}),
    ({"objective": "regression_l1", "metric": "mape"}, "-", {"mape"}),
    ({"objective": "regression_l1", "metric": "None"}, "-", None),
    ({"objective": "regression_l1"}, "mape", {"l1", "mape"}),
    ({"objective": "regression_l1", "metric": "gamma"}, "mape", {"gamma", "mape"}),
    ({"objective": "regression_l1", "metric": "gamma"}, ["l2", "mape"], {"gamma", "l2", "mape"}),
    ({"objective": custom_dummy_obj}, "-", {"l2"}),
    ({"objective": custom_dummy_obj, "metric": "mape"}, "-", {"mape"}),
    ({"objective": custom_dummy_obj, "metric": ["l1", "gamma"]}, "-", {"l1", "gamma"}),
    ({"objective": custom_dummy_obj, "metric": "None"}, "-", None),
    ({"objective": custom_dummy_obj}, "mape", {"l2", "mape"}),
    ({"objective": custom_dummy_obj, "metric": "mape"}, "gamma", {"mape", "gamma"}),
    ({"objective": custom_dummy_obj, "metric": ["l1", "gamma"]}, "l2", {"l1", "gamma", "l2"}),
    ({"objective": custom_dummy_obj, "metric": ["l1", "gamma"]}, ["l2", "mape"], {"l1", "gamma", "l2", "mape"}),
    ({}, constant_metric, {"l2", "error"}),
    ({"metric": "mape"}, constant_metric, {"mape", "error"}),
    ({"metric": ["l1", "gamma"]}, constant_metric, {"l1", "gamma", "error"}),
    ({"metric": "None"}, constant_metric, {"error"}),
    ({"objective": "regression_l1"}, constant_metric, {"l1", "error"}),
    ({"objective": "regression_l1", "metric": "mape"}, constant_metric, {"mape", "error"}),
    ({"objective": "regression_l1", "metric": ["l1", "gamma"]}, constant_metric, {"l1", "gamma", "error"}),
    ({"objective": "regression_l1", "metric": "None"}, constant_metric, {"error"}),
    ({"objective": custom_dummy_obj}, constant_metric, {"l2", "error"}),
    ({"objective": custom_dummy_obj, "metric": "mape"}, constant_metric, {"mape", "error"}),
    ({"objective": custom_dummy_obj, "metric": ["l2", "mape"]}, constant_metric, {"l2", "mape", "error"}),
]


@pytest.mark.parametrize("kw,eval_metric,expected", REGRESSION_CASES)
def test_metrics_regression(kw, eval_metric, expected):
    X, y = make_synthetic_regression()
    y = abs(y)
    fit = {"X": X, "y": y, "eval_set": (X, y)}
    if eval_metric != "-":
        fit["eval_metric"] = eval_metric
    gbm = lgb.LGBMRegressor(**P, **kw).fit(**fit)
    if expected is None:
        assert gbm.evals_result_ == {}
    else:
        assert set(gbm.evals_result_["training"]) == expected


def test_metrics_classification():
    X, y = load_breast_cancer(return_X_y=True)
    fit = {"X": X, "y": y, "eval_set": (X, y)}
    gbm = lgb.LGBMClassifier(n_estimators=2, verbose=-1, objective="binary", metric="binary_logloss").fit(
        eval_metric=["fair", "error"], **fit)
    assert set(gbm.evals_result_["training"]) == {"fair", "binary_error", "binary_logloss"}

    X, y = load_digits(n_class=3, return_X_y=True)
    fit = {"X": X, "y": y, "eval_set": (X, y)}
    # invalid binary metrics are replaced with their multiclass alternatives
    gbm = lgb.LGBMClassifier(**P).fit(eval_metric="binary_error", **fit)
    assert gbm.objective_ == "multiclass"
    assert set(gbm.evals_result_["training"]) == {"multi_logloss", "multi_error"}
    gbm = lgb.LGBMClassifier(objective="ovr", **P).fit(eval_metric="binary_error", **fit)
    assert gbm.objective_ == "ovr"
    assert set(gbm.evals_result_["training"]) == {"multi_logloss", "multi_error"}

    X, y = load_digits(n_class=2, return_X_y=True)
    fit = {"X": X, "y": y, "eval_set": (X, y)}
    gbm = lgb.LGBMClassifier(**P).fit(eval_metric="multi_error", **fit)
    assert set(gbm.evals_result_["training"]) == {"binary_logloss", "binary_error"}
    gbm = lgb.LGBMClassifier(objective=custom_dummy_obj, **P).fit(eval_metric="multi_logloss", **fit)
    assert set(gbm.evals_result_["training"]) == {"binary_logloss"}
    # multiclass objectives keep multiclass metrics even for two classes
    gbm = lgb.LGBMClassifier(objective="multiclass", num_classes=2, **P).fit(eval_metric="binary_logloss", **fit)
    assert set(gbm.evals_result_["training"]) == {"multi_logloss"}
    gbm = lgb.LGBMClassifier(objective="ovr", num_classes=2, **P).fit(eval_metric="binary_error", **fit)
    assert gbm.objective_ == "ovr"
    assert set(gbm.evals_result_["training"]) == {"multi_logloss", "multi_error"}


def test_multiple_eval_metrics():
    X, y = load_breast_cancer(return_X_y=True)
    params = {"n_estimators": 2, "verbose": -1, "objective": "binary", "metric": "binary_logloss"}
    fit = {"X": X, "y": y, "eval_set": (X, y)}
    gbm = lgb.LGBMClassifier(**params).fit(eval_metric=[constant_metric, decreasing_metric], **fit)
    assert set(gbm.evals_result_["training"]) == {"error", "decreasing_metric", "binary_logloss"}
    gbm = lgb.LGBMClassifier(**params).fit(eval_metric=[constant_metric, decreasing_metric, "fair"], **fit)
    assert set(gbm.evals_result_["training"]) == {"error", "decreasing_metric", "binary_logloss", "fair"}
    gbm = lgb.LGBMClassifier(**params).fit(eval_metric=[], **fit)
    assert set(gbm.evals_result_["training"]) == {"binary_logloss"}
    gbm = lgb.LGBMClassifier(**params).fit(eval_metric=["fair", "error"], **fit)
    assert len(gbm.evals_result_["training"]) == 3
    assert "binary_logloss" in gbm.evals_result_["training"]
    gbm = lgb.LGBMClassifier(**params).fit(eval_metric=["fair", "error", None], **fit)
    assert len(gbm.evals_result_["training"]) == 3
    assert "binary_logloss" in gbm.evals_result_["training"]


def test_nan_handle():
    rng = np.random.default_rng()
    nrows, ncols = 100, 10
    X = rng.standard_normal(size=(nrows, ncols))
    y = rng.standard_normal(size=(nrows,)) + np.full(nrows, 1e30)
    weight = np.zeros(nrows)
    gbm = lgb.LGBMRegressor(n_estimators=20, verbose=-1).fit(X, y, sample_weight=weight, eval_set=(X, y),
                                                             callbacks=[lgb.early_stopping(5)])
    np.testing.assert_allclose(gbm.evals_result_["training"]["l2"], np.nan)


def test_first_metric_only():
    X, y = make_synthetic_regression(n_samples=300)
    X_train, X_test, y_train, y_test = train_test_split(X, y, test_size=0.2, random_state=42)
    X_test1, X_test2, y_test1, y_test2 = train_test_split(X_test, y_test, test_size=0.5, random_state=72)
    params = {"n_estimators": 30, "learning_rate": 0.8, "num_leaves": 15, "verbose": -1, "seed": 123,
              "early_stopping_rounds": 5}
    fit = {"X": X_train, "y": y_train}

    def fit_and_check(eval_set_names, metric_names, assumed_iteration, first_metric_only):
        params["first_metric_only"] = first_metric_only
        gbm = lgb.LGBMRegressor(**params).fit(**fit)
        assert len(gbm.evals_result_) == len(eval_set_names)
        for name in eval_set_names:
            assert len(gbm.evals_result_[name]) == len(metric_names)
            for metric in metric_names:
                actual = len(gbm.evals_result_[name][metric])
                expected = assumed_iteration + (params["early_stopping_rounds"]
                                                if name != "training" and assumed_iteration != gbm.n_estimators else 0)
                assert expected == actual
                if name != "training":
                    assert assumed_iteration == gbm.best_iteration_
                else:
                    assert gbm.n_estimators == gbm.best_iteration_

    iter_valid1_l1 = iter_valid1_l2 = 4
    iter_valid2_l1 = iter_valid2_l2 = 2
    iter_min_l1 = min(iter_valid1_l1, iter_valid2_l1)
    iter_min_l2 = min(iter_valid1_l2, iter_valid2_l2)
    iter_min = min(iter_min_l1, iter_min_l2)
    iter_min_valid1 = min(iter_valid1_l1, iter_valid1_l2)

    params["metric"] = "None"
    fit["eval_metric"] = lambda preds, train_data: [decreasing_metric(preds, train_data),
                                                    constant_metric(preds, train_data)]
    fit["eval_set"] = (X_test1, y_test1)
    fit_and_check(["valid_0"], ["decreasing_metric", "error"], 1, False)
    fit_and_check(["valid_0"], ["decreasing_metric", "error"], 30, True)
    fit["eval_metric"] = lambda preds, train_data: [constant_metric(preds, train_data),
                                                    decreasing_metric(preds, train_data)]
    fit_and_check(["valid_0"], ["decreasing_metric", "error"], 1, True)

    params.pop("metric")
    fit.pop("eval_metric")
    fit_and_check(["valid_0"], ["l2"], iter_valid1_l2, False)
    fit_and_check(["valid_0"], ["l2"], iter_valid1_l2, True)
    fit["eval_metric"] = "l2"
    fit_and_check(["valid_0"], ["l2"], iter_valid1_l2, False)
    fit_and_check(["valid_0"], ["l2"], iter_valid1_l2, True)
    fit["eval_metric"] = "l1"
    fit_and_check(["valid_0"], ["l1", "l2"], iter_min_valid1, False)
    fit_and_check(["valid_0"], ["l1", "l2"], iter_valid1_l1, True)
    fit["eval_metric"] = ["l1", "l2"]
    fit_and_check(["valid_0"], ["l1", "l2"], iter_min_valid1, False)
    fit_and_check(["valid_0"], ["l1", "l2"], iter_valid1_l1, True)
    fit["eval_metric"] = ["l2", "l1"]
    fit_and_check(["valid_0"], ["l1", "l2"], iter_min_valid1, False)
    fit_and_check(["valid_0"], ["l1", "l2"], iter_valid1_l2, True)
    fit["eval_metric"] = ["l2", "regression", "mse"]  # aliases
    fit_and_check(["valid_0"], ["l2"], iter_valid1_l2, False)
    fit_and_check(["valid_0"], ["l2"], iter_valid1_l2, True)

    fit["eval_set"] = [(X_test1, y_test1), (X_test2, y_test2)]
    fit["eval_metric"] = ["l1", "l2"]
    fit_and_check(["valid_0", "valid_1"], ["l1", "l2"], iter_min_l1, True)
    fit["eval_metric"] = ["l2", "l1"]
    fit_and_check(["valid_0", "valid_1"], ["l1", "l2"], iter_min_l2, True)
    fit["eval_set"] = [(X_test2, y_test2), (X_test1, y_test1)]
    fit["eval_metric"] = ["l1", "l2"]
    fit_and_check(["valid_0", "valid_1"], ["l1", "l2"], iter_min, False)
    fit_and_check(["valid_0", "valid_1"], ["l1", "l2"], iter_min_l1, True)
    fit["eval_metric"] = ["l2", "l1"]
    fit_and_check(["valid_0", "valid_1"], ["l1", "l2"], iter_min, False)
    fit_and_check(["valid_0", "valid_1"], ["l1", "l2"], iter_min_l2, True)


def test_class_weight():
    X, y = load_digits(n_class=10, return_X_y=True)
    X_train, X_test, y_train, y_test = train_test_split(X, y, test_size=0.2, random_state=42)
    y_train_str, y_test_str = y_train.astype("str"), y_test.astype("str")
    gbm = lgb.LGBMClassifier(n_estimators=10, class_weight="balanced", verbose=-1)
    gbm.fit(X_train, y_train,
            eval_set=[(X_train, y_train), (X_test, y_test), (X_test, y_test), (X_test, y_test), (X_test, y_test)],
            eval_class_weight=["balanced", None, "balanced", {1: 10, 4: 20}, {5: 30, 2: 40}])
    for a, b in itertools.combinations(gbm.evals_result_.keys(), 2):
        for metric in gbm.evals_result_[a]:
            np.testing.assert_raises(AssertionError, np.testing.assert_allclose, gbm.evals_result_[a][metric],
                                     gbm.evals_result_[b][metric])
    gbm_str = lgb.LGBMClassifier(n_estimators=10, class_weight="balanced", verbose=-1)
    gbm_str.fit(X_train, y_train_str,
                eval_set=[(X_train, y_train_str), (X_test, y_test_str), (X_test, y_test_str), (X_test, y_test_str),
                          (X_test, y_test_str)],
                eval_class_weight=["balanced", None, "balanced", {"1": 10, "4": 20}, {"5": 30, "2": 40}])
    for a, b in itertools.combinations(gbm_str.evals_result_.keys(), 2):
        for metric in gbm_str.evals_result_[a]:
            np.testing.assert_raises(AssertionError, np.testing.assert_allclose, gbm_str.evals_result_[a][metric],
                                     gbm_str.evals_result_[b][metric])
    for name in gbm.evals_result_:
        for metric in gbm.evals_result_[name]:
            np.testing.assert_allclose(gbm.evals_result_[name][metric], gbm_str.evals_result_[name][metric])


def test_continue_training_with_model():
    X, y = load_digits(n_class=3, return_X_y=True)
    X_train, X_test, y_train, y_test = train_test_split(X, y, test_size=0.1, random_state=42)
    init_gbm = lgb.LGBMClassifier(n_estimators=5).fit(X_train, y_train, eval_set=(X_test, y_test))
    gbm = lgb.LGBMClassifier(n_estimators=5).fit(X_train, y_train, eval_set=(X_test, y_test), init_model=init_gbm)
    a = init_gbm.evals_result_["valid_0"]["multi_logloss"]
    b = gbm.evals_result_["valid_0"]["multi_logloss"]
    assert len(a) == len(b) == 5
    assert b[-1] < a[-1]


def test_actual_number_of_trees():
    X = [[1, 2, 3], [1, 2, 3]]
    y = [1, 1]
    gbm = lgb.LGBMRegressor(n_estimators=5).fit(X, y)
    assert gbm.n_estimators == 5
    assert gbm.n_estimators_ == 1
    assert gbm.n_iter_ == 1
    np.testing.assert_array_equal(gbm.predict(np.array(X) * 10), y)


def test_check_is_fitted():
    from sklearn.exceptions import NotFittedError
    from sklearn.utils.validation import check_is_fitted

    X, y = load_digits(n_class=2, return_X_y=True)
    models = (lgb.LGBMModel(n_estimators=5, objective="binary"), lgb.LGBMClassifier(n_estimators=5),
              lgb.LGBMRegressor(n_estimators=5), lgb.LGBMRanker(n_estimators=5))
    for model in models:
        with pytest.raises(NotFittedError, match=f"This {type(model).__name__} instance is not fitted yet"):
            check_is_fitted(model)
    models[0].fit(X, y)
    models[1].fit(X, y)
    models[2].fit(X, y)
    models[3].fit(X, y, group=np.ones(X.shape[0]))
    for model in models:
        check_is_fitted(model)
