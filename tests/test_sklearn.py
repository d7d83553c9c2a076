"""scikit-learn estimator tests (reference tests/python_package_test/test_sklearn.py themes)."""
import numpy as np
import pytest
from sklearn.base import clone
from sklearn.datasets import load_breast_cancer, load_iris, make_regression
from sklearn.metrics import accuracy_score, r2_score
from sklearn.model_selection import GridSearchCV, train_test_split


def test_classifier_binary(lgb):
    X, y = load_breast_cancer(return_X_y=True)
    Xtr, Xte, ytr, yte = train_test_split(X, y, test_size=0.2, random_state=0)
    clf = lgb.LGBMClassifier(n_estimators=50, verbose=-1).fit(Xtr, ytr, eval_set=[(Xte, yte)], eval_metric="auc")
    assert accuracy_score(yte, clf.predict(Xte)) > 0.93
    proba = clf.predict_proba(Xte)
    assert proba.shape == (len(yte), 2)
    np.testing.assert_allclose(proba.sum(1), 1.0)
    assert "auc" in clf.evals_result_["valid_0"] and "binary_logloss" in clf.evals_result_["valid_0"]
    assert clf.n_features_in_ == X.shape[1]
    assert len(clf.feature_importances_) == X.shape[1]


def test_classifier_multiclass_string_labels(lgb):
    X, y = load_iris(return_X_y=True)
    names = np.array(["setosa", "versicolor", "virginica"])[y]
    clf = lgb.LGBMClassifier(n_estimators=30, min_child_samples=5, verbose=-1).fit(X, names)
    assert set(clf.classes_) == set(names)
    assert clf.n_classes_ == 3
    assert accuracy_score(names, clf.predict(X)) > 0.95
    assert clf.predict_proba(X).shape == (150, 3)


def test_regressor(lgb):
    X, y = make_regression(2000, 8, noise=1.0, random_state=3)
    reg = lgb.LGBMRegressor(n_estimators=100, verbose=-1).fit(X[:1500], y[:1500])
    assert r2_score(y[1500:], reg.predict(X[1500:])) > 0.85


def test_early_stopping_sklearn(lgb):
    X, y = make_regression(2000, 8, noise=30.0, random_state=4)
    reg = lgb.LGBMRegressor(n_estimators=1000, learning_rate=0.3, verbose=-1)
    reg.fit(X[:1500], y[:1500], eval_set=[(X[1500:], y[1500:])], callbacks=[lgb.early_stopping(10, verbose=False)])
    assert 0 < reg.best_iteration_ < 1000


def test_ranker(lgb, rng):
    n_q, per = 50, 20
    X = rng.standard_normal((n_q * per, 5))
    y = np.clip((X[:, 0] * 2 + rng.standard_normal(n_q * per)).round(), 0, 4)
    group = np.full(n_q, per)
    rk = lgb.LGBMRanker(n_estimators=20, verbose=-1, lambdarank_target="lambdagap-s", lambdagap_weight=0.5,
                        lambdarank_truncation_level=3)
    rk.fit(X, y, group=group, eval_set=[(X, y)], eval_group=[group], eval_at=[3, 5])
    assert "ndcg@3" in rk.evals_result_["training"]  # the training data as an eval set
    s = rk.predict(X)
    assert np.corrcoef(s, y)[0, 1] > 0.5
    with pytest.raises(ValueError):
        lgb.LGBMRanker().fit(X, y)


def test_class_weight_and_sample_weight(lgb, rng):
    X = rng.standard_normal((1000, 4))
    y = (X[:, 0] > 1.0).astype(int)
    a = lgb.LGBMClassifier(n_estimators=20, verbose=-1).fit(X, y)
    b = lgb.LGBMClassifier(n_estimators=20, class_weight="balanced", verbose=-1).fit(X, y)
    assert b.predict_proba(X)[:, 1].mean() > a.predict_proba(X)[:, 1].mean()
    c = lgb.LGBMClassifier(n_estimators=20, verbose=-1).fit(X, y, sample_weight=np.where(y == 1, 5.0, 1.0))
    assert c.predict_proba(X)[:, 1].mean() > a.predict_proba(X)[:, 1].mean()


def test_custom_objective_sklearn(lgb, rng):
    X = rng.standard_normal((800, 3))
    y = X[:, 0] * 3 + rng.standard_normal(800)

    def l2(y_true, y_pred):
        return y_pred - y_true, np.ones_like(y_true)

    reg = lgb.LGBMRegressor(objective=l2, n_estimators=30, verbose=-1).fit(X, y)
    ref = lgb.LGBMRegressor(n_estimators=30, verbose=-1).fit(X, y)
    assert np.corrcoef(reg.predict(X), ref.predict(X))[0, 1] > 0.99


def test_clone_and_grid_search(lgb):
    X, y = load_breast_cancer(return_X_y=True)
    base = lgb.LGBMClassifier(n_estimators=10, verbose=-1)
    c = clone(base)
    assert c.get_params()["n_estimators"] == 10
    gs = GridSearchCV(base, {"num_leaves": [7, 15]}, cv=2).fit(X, y)
    assert gs.best_params_["num_leaves"] in (7, 15)


def test_pandas_input_sklearn(lgb, rng):
    import pandas as pd

    df = pd.DataFrame({"num": rng.standard_normal(600), "cat": pd.Categorical(rng.choice(list("abcd"), 600))})
    y = (df["cat"].isin(["a", "c"])).astype(int)
    clf = lgb.LGBMClassifier(n_estimators=20, verbose=-1).fit(df, y)
    assert accuracy_score(y, clf.predict(df)) > 0.95
    assert clf.feature_name_ == ["num", "cat"]
