"""CLI / Python / scikit-learn consistency over the reference's example configurations
(themes of the reference's tests/python_package_test/test_consistency.py:12-160).

For every examples/*/train.conf (copied into tests/data/examples with the datasets):
  * the Python API trained on arrays predicts the same on an array and on the text file;
  * the scikit-learn estimator with the same parameters predicts the same;
  * the CLI trained from the .conf on the text files builds the same model: its CLI
    predictions equal the Python model's;
  * a Dataset loaded from the file carries the same fields as the one built from arrays.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest
from sklearn.datasets import load_svmlight_file

DATA = os.path.join(os.path.dirname(__file__), "data")
EX = os.path.join(DATA, "examples")

# (example dir, data prefix, conf file, sparse input, estimator)
CASES = [
    ("binary_classification", "binary", "train.conf", False, "classifier"),
    ("binary_classification", "binary", "train_linear.conf", False, "classifier"),
    ("multiclass_classification", "multiclass", "train.conf", False, "classifier"),
    ("regression", "regression", "train.conf", False, "regressor"),
    ("lambdarank", "rank", "train.conf", True, "ranker"),
    ("xendcg", "rank", "train.conf", True, "ranker"),
]

# file / process keys of the .conf that are not training parameters
_NOT_PARAMS = {"task", "data", "valid_data", "output_model", "machine_list_file", "local_listen_port",
               "num_machines", "is_save_binary_file", "use_two_round_loading", "is_training_metric",
               "metric_freq"}


def _conf_params(path):
    params = {"verbosity": -1}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            key, value = [t.strip() for t in line.split("=", 1)]
            if "early_stopping" in key or key in _NOT_PARAMS:
                continue
            params[key] = int(value) if key in ("num_trees", "num_threads") else value
    return params


def _load(prefix, suffix, sparse, n_features=None):
    fn = os.path.join(DATA, prefix + suffix)
    if sparse:
        X, y = load_svmlight_file(fn, dtype=np.float64, zero_based=True, n_features=n_features)
        return X, y, fn
    mat = np.loadtxt(fn, dtype=np.float64)
    return mat[:, 1:], mat[:, 0], fn


def _field(prefix, suffix):
    fn = os.path.join(DATA, prefix + suffix)
    return np.loadtxt(fn) if os.path.exists(fn) else None


@pytest.fixture(scope="module")
def cli(lgb):
    from lambdagap_amd.libpath import cli_path

    p = cli_path()
    if not os.path.exists(p):
        pytest.skip("CLI binary not built")
    return p


@pytest.mark.parametrize("example,prefix,conf,sparse,kind", CASES,
                         ids=[f"{c[0]}-{c[2]}" for c in CASES])
def test_example_consistency(lgb, cli, tmp_path, example, prefix, conf, sparse, kind):
    params = _conf_params(os.path.join(EX, example, conf))
    X, y, train_fn = _load(prefix, ".train", sparse)
    Xt, _, test_fn = _load(prefix, ".test", sparse, n_features=X.shape[1])
    weight = _field(prefix, ".train.weight")
    init = _field(prefix, ".train.init")
    group = _field(prefix, ".train.query")
    ds = lgb.Dataset(X, y, weight=weight, init_score=init, group=group, params=params)

    # python API: array and file predictions agree
    b = lgb.train(params, ds)
    y_pred = b.predict(Xt)
    np.testing.assert_allclose(y_pred, b.predict(test_fn), rtol=1e-9, atol=1e-12)

    # scikit-learn estimator with the same parameters
    est = {"classifier": lgb.LGBMClassifier, "regressor": lgb.LGBMRegressor, "ranker": lgb.LGBMRanker}[kind]
    sk_params = {k: v for k, v in params.items() if k not in ("num_trees", "objective")}
    model = est(n_estimators=params.get("num_trees", 100), objective=params.get("objective"), **sk_params)
    fit_kw = {"sample_weight": weight} if weight is not None else {}
    if init is not None:
        fit_kw["init_score"] = init
    if group is not None:
        fit_kw["group"] = group
    model.fit(X, y, **fit_kw)
    if kind == "classifier":
        sk_pred = model.predict_proba(Xt)
        sk_pred = sk_pred[:, 1] if sk_pred.shape[1] == 2 else sk_pred
    else:
        sk_pred = model.predict(Xt)
    np.testing.assert_allclose(y_pred, sk_pred, rtol=1e-9, atol=1e-12)

    # CLI trained from the .conf on the text files: the same model
    for suffix in (".train", ".test", ".train.weight", ".test.weight", ".train.init", ".test.init",
                   ".train.query", ".test.query"):
        src = os.path.join(DATA, prefix + suffix)
        if os.path.exists(src):
            shutil.copy(src, tmp_path / (prefix + suffix))
    conf_path = tmp_path / conf
    shutil.copy(os.path.join(EX, example, conf), conf_path)
    r = subprocess.run([cli, f"config={conf_path.name}", "verbosity=-1", "output_model=cli_model.txt"],
                       capture_output=True, text=True, cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    r = subprocess.run([cli, "task=predict", f"data={prefix}.test", "input_model=cli_model.txt",
                        "output_result=cli_pred.txt", "verbosity=-1"], capture_output=True, text=True, cwd=tmp_path,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    cli_pred = np.loadtxt(tmp_path / "cli_pred.txt")
    np.testing.assert_allclose(cli_pred.reshape(y_pred.shape), y_pred, rtol=1e-6, atol=1e-9)

    # a Dataset loaded from the file carries the same fields
    df = lgb.Dataset(train_fn, params=params).construct()
    ds.construct()
    assert df.num_data() == ds.num_data() and df.num_feature() == ds.num_feature()
    for getter in ("get_label", "get_weight", "get_init_score", "get_group"):
        a, c = getattr(ds, getter)(), getattr(df, getter)()
        if a is None and c is None:
            continue
        if a is None:
            assert np.all(np.asarray(c) == 1), getter
            continue
        np.testing.assert_allclose(np.asarray(a, dtype=np.float64).ravel(), np.asarray(c, dtype=np.float64).ravel(),
                                   err_msg=getter)
