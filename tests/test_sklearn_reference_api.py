"""Estimator-API expectations of the reference's scikit-learn tests
(/root/reference/tests/python_package_test/test_sklearn.py: verbosity with a custom
objective, n_estimators alias warnings, feature_names_in_, column-vector labels,
multiclass custom objective / eval, n_jobs, validate_features, feature-count checks)."""
import re

import joblib
import numpy as np
import pytest
from sklearn.datasets import load_breast_cancer, load_digits, make_blobs, make_regression
from sklearn.metrics import log_loss
from sklearn.model_selection import train_test_split

import lambdagap_amd as lgb

FACTORY = {"ranking": lgb.LGBMRanker, "binary-classification": lgb.LGBMClassifier,
           "multiclass-classification": lgb.LGBMClassifier, "regression": lgb.LGBMRegressor}
ESTIMATORS = (lgb.LGBMModel, lgb.LGBMClassifier, lgb.LGBMRegressor, lgb.LGBMRanker)


def _create_data(task, n_samples=100, n_features=4):
    rng = np.random.RandomState(0)
    if task == "ranking":
        X = rng.normal(size=(n_samples, n_features))
        y = np.clip(np.round(X[:, 0] + rng.normal(scale=0.5, size=n_samples)), 0, 2)
        g = np.full(n_samples // 10, 10)
    elif task.endswith("classification"):
        centers = 2 if task == "binary-classification" else 3
        X, y = make_blobs(n_samples=n_samples, n_features=n_features, centers=centers, random_state=42)
        g = None
    else:
        X, y = make_regression(n_samples=n_samples, n_features=n_features, n_informative=2, random_state=42)
        g = None
    return X, y, g


def _softmax(x):
    e = np.exp(x - np.max(x, axis=1).reshape(-1, 1))
    return e / np.sum(e, axis=1).reshape(-1, 1)


def sklearn_multiclass_custom_objective(y_true, y_pred, weight=None):
    num_rows, num_class = y_pred.shape
    prob = _softmax(y_pred)
    grad_update = np.zeros_like(prob)
    grad_update[np.arange(num_rows), y_true.astype(np.int32)] = -1.0
    grad = prob + grad_update
    hess = num_class / (num_class - 1) * prob * (1 - prob)
    if weight is not None:
        grad *= weight.reshape(-1, 1)
        hess *= weight.reshape(-1, 1)
    return grad, hess


def objective_ls(y_true, y_pred):
    return y_pred - y_true, np.ones(len(y_true))


def _silent(capsys):
    out = capsys.readouterr()
    assert out.out == "" and out.err == ""


def test_verbosity_is_respected_when_using_custom_objective(capsys):
    X, y = make_regression(n_samples=100, n_features=4, n_informative=2, random_state=42)
    params = {"objective": objective_ls, "nonsense": 123, "num_leaves": 3}
    lgb.LGBMRegressor(**params, verbosity=-1, n_estimators=1).fit(X, y)
    assert capsys.readouterr().out == ""
    lgb.LGBMRegressor(**params, verbosity=0, n_estimators=1).fit(X, y)
    assert "[LambdaGap] [Warning] Unknown parameter: nonsense" in capsys.readouterr().out  # (the log prefix names this framework)


def test_fit_only_raises_num_rounds_warning_when_expected(capsys):
    X, y = make_regression(n_samples=100, n_features=4, n_informative=2, random_state=42)
    base = {"num_leaves": 5, "verbosity": -1}
    cases = [({}, 100), ({"n_estimators": 2}, 2), ({"n_estimators": 3, "n_iter": 3}, 3),
             ({"n_estimators": 3, "n_iter": 4}, 4), ({"n_iter": 3, "num_iterations": 3}, 3),
             ({"n_iter": 3, "num_trees": 3, "nrounds": 3, "max_iter": 3}, 3)]
    for kw, n in cases:
        reg = lgb.LGBMRegressor(**base, **kw).fit(X, y)
        assert reg.n_estimators_ == n
        _silent(capsys)
    with pytest.warns(UserWarning, match="LightGBM will perform up to 5 boosting rounds"):
        reg = lgb.LGBMRegressor(**base, num_iterations=5, n_iter=6).fit(X, y)
    assert reg.n_estimators_ == 5
    _silent(capsys)
    with pytest.warns(UserWarning, match="LightGBM will perform up to 4 boosting rounds"):
        reg = lgb.LGBMRegressor(**base, n_iter=4, max_iter=5).fit(X, y)
    assert reg.n_estimators_ == 4
    _silent(capsys)


def _fit_binary(estimator_class, X, y):
    params = {"n_estimators": 2, "num_leaves": 7}
    if estimator_class is lgb.LGBMModel:
        model = estimator_class(**{**params, "objective": "binary"})
    else:
        model = estimator_class(**params)
    from sklearn.exceptions import NotFittedError
    from sklearn.utils.validation import check_is_fitted

    with pytest.raises(NotFittedError, match=f"This {estimator_class.__name__} instance is not fitted yet"):
        check_is_fitted(model)
    if isinstance(model, lgb.LGBMRanker):
        model.fit(X, y, group=[X.shape[0]])
    else:
        model.fit(X, y)
    return model


@pytest.mark.parametrize("estimator_class", ESTIMATORS)
def test_getting_feature_names_in_np_input(estimator_class):
    X, y = load_digits(n_class=2, return_X_y=True)
    model = _fit_binary(estimator_class, X, y)
    np.testing.assert_array_equal(model.feature_names_in_, np.array([f"Column_{i}" for i in range(X.shape[1])]))


@pytest.mark.parametrize("estimator_class", ESTIMATORS)
def test_getting_feature_names_in_pd_input(estimator_class):
    pytest.importorskip("pandas")
    X, y = load_digits(n_class=2, return_X_y=True, as_frame=True)
    model = _fit_binary(estimator_class, X, y)
    np.testing.assert_array_equal(model.feature_names_in_, X.columns)


@pytest.mark.parametrize("task", list(FACTORY))
def test_training_succeeds_when_data_is_dataframe_and_label_is_column_array(task):
    pd = pytest.importorskip("pandas")
    X, y, g = _create_data(task)
    X = pd.DataFrame(X)
    params = {"n_estimators": 1, "num_leaves": 3, "random_state": 0}
    fit_kw = {"group": g} if task == "ranking" else {}
    model_1d = FACTORY[task](**params).fit(X, y, **fit_kw)
    with pytest.warns(UserWarning, match="column-vector"):
        model_2d = FACTORY[task](**params).fit(X, y.reshape(-1, 1), **fit_kw)
    np.testing.assert_array_equal(model_1d.predict(X), model_2d.predict(X))


@pytest.mark.parametrize("use_weight", [True, False])
def test_multiclass_custom_objective(use_weight):
    X, y = make_blobs(n_samples=1_000, centers=[[-4, -4], [4, 4], [-4, 4]], random_state=42)
    weight = np.full_like(y, 2) if use_weight else None
    params = {"n_estimators": 10, "num_leaves": 7}
    builtin = lgb.LGBMClassifier(**params).fit(X, y, sample_weight=weight)
    custom = lgb.LGBMClassifier(objective=sklearn_multiclass_custom_objective, **params).fit(X, y, sample_weight=weight)
    np.testing.assert_allclose(builtin.predict_proba(X), _softmax(custom.predict(X, raw_score=True)), rtol=0.01)
    assert not callable(builtin.objective_)
    assert callable(custom.objective_)


@pytest.mark.parametrize("use_weight", [True, False])
def test_multiclass_custom_eval(use_weight):
    def custom_eval(y_true, y_pred, weight):
        return "custom_logloss", log_loss(y_true, y_pred, sample_weight=weight), False

    X, y = make_blobs(n_samples=1_000, centers=[[-4, -4], [4, 4], [-4, 4]], random_state=42)
    X_train, X_valid, y_train, y_valid = train_test_split(X, y, test_size=0.2, random_state=0)
    if use_weight:
        w_train, w_valid = train_test_split(np.full_like(y, 2), test_size=0.2, random_state=0)
    else:
        w_train = w_valid = None
    model = lgb.LGBMClassifier(objective="multiclass", num_class=3, num_leaves=7)
    model.fit(X_train, y_train, sample_weight=w_train, eval_set=[(X_train, y_train), (X_valid, y_valid)],
              eval_names=["train", "valid"], eval_sample_weight=[w_train, w_valid], eval_metric=custom_eval)
    res = model.evals_result_
    for key, (Xk, yk, wk) in zip(["train", "valid"], [(X_train, y_train, w_train), (X_valid, y_valid, w_valid)]):
        np.testing.assert_allclose(res[key]["multi_logloss"], res[key]["custom_logloss"])
        _, value, _ = custom_eval(yk, model.predict_proba(Xk), wk)
        np.testing.assert_allclose(value, res[key]["custom_logloss"][-1])


def test_negative_n_jobs(tmp_path):
    n_threads = joblib.cpu_count()
    if n_threads <= 1:
        return
    X, y = load_breast_cancer(return_X_y=True)
    gbm = lgb.LGBMClassifier(n_estimators=2, verbose=-1, n_jobs=-2).fit(X, y)
    gbm.booster_.save_model(tmp_path / "model.txt")
    assert re.search(rf"\[num_threads: {n_threads - 1}\]", (tmp_path / "model.txt").read_text())


def test_default_n_jobs(tmp_path):
    n_cores = joblib.cpu_count(only_physical_cores=True)
    X, y = load_breast_cancer(return_X_y=True)
    gbm = lgb.LGBMClassifier(n_estimators=2, verbose=-1, n_jobs=None).fit(X, y)
    gbm.booster_.save_model(tmp_path / "model.txt")
    assert re.search(rf"\[num_threads: {n_cores}\]", (tmp_path / "model.txt").read_text())


@pytest.mark.parametrize("task", list(FACTORY))
def test_validate_features(task):
    pd = pytest.importorskip("pandas")
    X, y, g = _create_data(task, n_features=4)
    features = ["x1", "x2", "x3", "x4"]
    df = pd.DataFrame(X, columns=features)
    model = FACTORY[task](n_estimators=10, num_leaves=15, verbose=-1)
    model.fit(df, y, **({"group": g} if task == "ranking" else {}))
    assert model.feature_name_ == features
    df2 = df.rename(columns={"x2": "z"})
    with pytest.raises(lgb.basic.LightGBMError, match="Expected 'x2' at position 1 but found 'z'"):
        model.predict(df2, validate_features=True)
    model.predict(df2, validate_features=False)


@pytest.mark.parametrize("task", list(FACTORY))
@pytest.mark.parametrize("predict_disable_shape_check", [True, False])
def test_predict_rejects_inputs_with_incorrect_number_of_features(predict_disable_shape_check, task):
    X, y, g = _create_data(task, n_features=4)
    fit_kwargs = {"X": X[:, :-1], "y": y}
    if task == "ranking":
        name = "LGBMRanker"
        fit_kwargs["group"] = g
    elif task == "regression":
        name = "LGBMRegressor"
    else:
        name = "LGBMClassifier"
    model = FACTORY[task](n_estimators=5, num_leaves=7, verbose=-1).fit(**fit_kwargs)
    for cols, n in ((X, 4), (X[:, :-2], 2)):
        msg = f"X has {n} features, but {name} is expecting 3 features as input"
        with pytest.raises(ValueError, match=msg):
            model.predict(cols, predict_disable_shape_check=predict_disable_shape_check)
        if name == "LGBMClassifier":
            with pytest.raises(ValueError, match=msg):
                model.predict_proba(cols, predict_disable_shape_check=predict_disable_shape_check)
    assert model.predict(X[:, :-1], predict_disable_shape_check=predict_disable_shape_check).shape == y.shape
    if name == "LGBMClassifier":
        assert model.predict_proba(X[:, :-1], predict_disable_shape_check=predict_disable_shape_check).shape[0] == len(y)


@pytest.mark.parametrize("estimator_class", ESTIMATORS)
def test_sklearn_tags_should_correctly_reflect_lightgbm_specific_values(estimator_class):
    est = estimator_class()
    assert est._more_tags()["X_types"] == ["2darray", "sparse", "1dlabels"]
    tags = est.__sklearn_tags__()  # scikit-learn >= 1.6 here
    assert tags.input_tags.allow_nan is True
    assert tags.input_tags.sparse is True
    assert tags.target_tags.one_d_labels is True
    if estimator_class is lgb.LGBMClassifier:
        assert tags.estimator_type == "classifier"
        assert tags.classifier_tags.multi_class is True
        assert tags.classifier_tags.multi_label is False
    elif estimator_class is lgb.LGBMRegressor:
        assert tags.estimator_type == "regressor"


def test_classifier_fit_detects_classes_every_time():
    rng = np.random.default_rng(seed=123)
    X = rng.standard_normal(size=(1000, 20))
    y_bin = (rng.random(size=1000) <= 0.3).astype(np.float64)
    y_multi = rng.integers(4, size=1000)
    model = lgb.LGBMClassifier(verbose=-1)
    for _ in range(2):
        model.fit(X, y_multi)
        assert model.objective_ == "multiclass"
        model.fit(X, y_bin)
        assert model.objective_ == "binary"
