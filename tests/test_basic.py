"""Dataset / Booster API tests on CPU (reference tests/python_package_test/test_basic.py themes)."""
import os
import pickle

import numpy as np
import pytest

DATA = os.path.join(os.path.dirname(__file__), "data")


def test_train_predict_save_load(lgb, rng, tmp_path):
    X = rng.standard_normal((3000, 6))
    y = (X[:, 0] + X[:, 1] > 0).astype(float)
    ds = lgb.Dataset(X, y)
    b = lgb.train({"objective": "binary", "verbosity": -1, "num_leaves": 7}, ds, 10)
    p = b.predict(X)
    assert p.shape == (3000,)
    f = tmp_path / "m.txt"
    b.save_model(str(f))
    b2 = lgb.Booster(model_file=str(f))
    np.testing.assert_allclose(b2.predict(X), p)
    assert b2.num_trees() == 10
    txt = f.read_text()
    assert txt.startswith("tree\nversion=v4")


def test_device_count_cpu(lgb):
    assert lgb.device_count() >= 0


def test_dataset_fields(lgb, rng):
    X = rng.standard_normal((500, 4))
    y = rng.random(500)
    w = rng.random(500) + 0.5
    init = rng.standard_normal(500)
    ds = lgb.Dataset(X, y, weight=w, init_score=init).construct()
    assert ds.num_data() == 500 and ds.num_feature() == 4
    np.testing.assert_allclose(ds.get_field("label"), y.astype(np.float32))
    np.testing.assert_allclose(ds.get_field("weight"), w.astype(np.float32))
    np.testing.assert_allclose(ds.get_field("init_score"), init)
    ds.set_label(np.ones(500))
    np.testing.assert_allclose(ds.get_field("label"), 1.0)


def test_dataset_group_and_position(lgb, rng):
    X = rng.standard_normal((60, 3))
    y = rng.integers(0, 3, 60)
    ds = lgb.Dataset(X, y, group=[10, 20, 30], position=np.arange(60) % 5).construct()
    np.testing.assert_array_equal(ds.get_field("group"), [0, 10, 30, 60])  # boundaries
    np.testing.assert_array_equal(ds.get_group(), [10, 20, 30])
    np.testing.assert_array_equal(ds.get_field("position"), np.arange(60) % 5)


def test_dataset_feature_names_and_bins(lgb, rng):
    X = rng.standard_normal((1000, 3))
    X[:, 2] = rng.integers(0, 4, 1000)
    names = ["alpha", "beta", "gamma"]
    ds = lgb.Dataset(X, rng.random(1000), feature_name=names, params={"max_bin": 31}).construct()
    assert ds.get_feature_name() == names
    assert ds.feature_num_bin(0) <= 32
    assert ds.feature_num_bin("gamma") <= 5
    b = lgb.train({"verbosity": -1}, ds, 2)
    assert b.feature_name() == names


def test_subset(lgb, rng):
    X = rng.standard_normal((1000, 5))
    y = rng.random(1000)
    ds = lgb.Dataset(X, y, free_raw_data=False)
    sub = ds.subset(np.arange(0, 1000, 2)).construct()
    assert sub.num_data() == 500
    np.testing.assert_allclose(sub.get_field("label"), y[::2].astype(np.float32))
    lgb.train({"verbosity": -1}, sub, 3)


def test_construct_from_various_inputs(lgb, rng):
    import pandas as pd
    import scipy.sparse as sp

    X = rng.standard_normal((400, 5))
    X[X < 0.5] = 0.0
    y = rng.random(400)
    params = {"verbosity": -1, "min_data_in_leaf": 5}
    ref = lgb.train(params, lgb.Dataset(X, y), 5).predict(X)
    for data in (X.astype(np.float32), sp.csr_matrix(X), sp.csc_matrix(X), pd.DataFrame(X),
                 [X[:200], X[200:]], X.tolist()):
        p = lgb.train(params, lgb.Dataset(data, y), 5).predict(X)
        np.testing.assert_allclose(p, ref, rtol=1e-5, atol=1e-6)


def test_sequence_input(lgb, rng):
    X = rng.standard_normal((900, 3))
    y = rng.random(900)

    class Seq(lgb.Sequence):
        batch_size = 128

        def __init__(self, a):
            self.a = a

        def __getitem__(self, i):
            return self.a[i]

        def __len__(self):
            return len(self.a)

    p1 = lgb.train({"verbosity": -1}, lgb.Dataset(Seq(X), y), 3).predict(X)
    p2 = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 3).predict(X)
    np.testing.assert_allclose(p1, p2)


def test_add_features_from(lgb, rng):
    X = rng.standard_normal((500, 4))
    y = rng.random(500)
    d1 = lgb.Dataset(X[:, :2], y, free_raw_data=False).construct()
    d2 = lgb.Dataset(X[:, 2:], free_raw_data=False).construct()
    d1.add_features_from(d2)
    assert d1.num_feature() == 4
    p1 = lgb.train({"verbosity": -1}, d1, 3).predict(X)
    p2 = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 3).predict(X)
    np.testing.assert_allclose(p1, p2, rtol=1e-6)


def test_booster_pickle_and_copy(lgb, rng):
    import copy

    X = rng.standard_normal((300, 3))
    y = rng.random(300)
    b = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 5)
    b2 = pickle.loads(pickle.dumps(b))
    np.testing.assert_allclose(b2.predict(X), b.predict(X))
    b3 = copy.deepcopy(b)
    np.testing.assert_allclose(b3.predict(X), b.predict(X))


def test_booster_eval_and_leaf_ops(lgb, rng):
    X = rng.standard_normal((500, 3))
    y = X[:, 0] + 0.1 * rng.standard_normal(500)
    ds = lgb.Dataset(X, y)
    b = lgb.Booster({"objective": "regression", "metric": "l2", "verbosity": -1}, ds)
    b.update()
    b.update()
    (name, metric, value, higher) = b.eval_train()[0]
    assert metric == "l2" and value > 0 and not higher
    v = b.get_leaf_output(0, 0)
    b.set_leaf_output(0, 0, v + 1.0)
    assert b.get_leaf_output(0, 0) == pytest.approx(v + 1.0)
    assert b.num_model_per_iteration() == 1
    assert b.current_iteration() == 2
    ub, lb = b.upper_bound(), b.lower_bound()
    assert ub >= lb


def test_booster_shuffle_models(lgb, rng):
    X = rng.standard_normal((300, 3))
    y = rng.random(300)
    b = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 6)
    p = b.predict(X)
    b.shuffle_models()
    np.testing.assert_allclose(b.predict(X), p, rtol=1e-10)


def test_trees_to_dataframe(lgb, rng):
    X = rng.standard_normal((300, 3))
    y = rng.random(300)
    b = lgb.train({"verbosity": -1, "num_leaves": 5}, lgb.Dataset(X, y), 2)
    df = b.trees_to_dataframe()
    assert set(df["tree_index"]) == {0, 1}
    assert (df["split_feature"].dropna().isin(b.feature_name())).all()


def test_split_value_histogram(lgb, rng):
    X = rng.standard_normal((1000, 3))
    y = X[:, 0] * 2 + rng.standard_normal(1000)
    b = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 5)
    hist, edges = b.get_split_value_histogram(0)
    assert hist.sum() == b.feature_importance("split")[0]


def test_invalid_params_raise(lgb, rng):
    X = rng.standard_normal((100, 2))
    with pytest.raises(lgb.LightGBMError):
        lgb.train({"objective": "not_an_objective", "verbosity": -1}, lgb.Dataset(X, rng.random(100)), 1)
    with pytest.raises(lgb.LightGBMError):
        lgb.train({"num_leaves": 1, "verbosity": -1}, lgb.Dataset(X, rng.random(100)), 1)


def test_param_aliases_roundtrip(lgb):
    from lambdagap_amd.basic import dump_param_aliases

    al = dump_param_aliases()
    assert "num_iterations" in al and "n_estimators" in al["num_iterations"]
    assert "lambdarank_target" in al and "lambdagap_weight" in al


def test_phase_timer_report(lgb):
    assert isinstance(lgb.phase_timer_report(), str)


def test_free_raw_data_and_reference_alignment(lgb, rng):
    X = rng.standard_normal((500, 3))
    y = rng.random(500)
    ds = lgb.Dataset(X, y)
    dv = ds.create_valid(X[:100], y[:100])
    b = lgb.train({"verbosity": -1}, ds, 3, valid_sets=[dv], keep_training_booster=True)
    assert ds.data is None
    assert b.eval_valid()[0][0] == "valid_0"


@pytest.mark.parametrize("name,obj", [("binary", "binary"), ("rank", "lambdarank")])
def test_two_round_loading_matches_one_round(lgb, name, obj):
    """two_round streams the file twice (sample for bins, then chunked packing); with the
    sample covering the file the dataset and model are identical to one-round loading."""
    path = os.path.join(DATA, f"{name}.train")
    params = {"objective": obj, "verbosity": -1, "num_leaves": 15}
    one = lgb.train(params, lgb.Dataset(path, params=dict(params)), 5)
    two = lgb.train(params, lgb.Dataset(path, params=dict(params, two_round=True)), 5)
    strip = lambda s: s[:s.index("parameters:")]  # noqa: E731
    assert strip(one.model_to_string()) == strip(two.model_to_string())


def test_ref_chain_and_set_network_api(lgb):
    """Reference Dataset.get_ref_chain / Booster.set_network surface."""
    X = np.random.default_rng(0).random((300, 4))
    y = X[:, 0]
    a = lgb.Dataset(X, y)
    b = lgb.Dataset(X, y, reference=a)
    c = lgb.Dataset(X, y, reference=b)
    assert c.get_ref_chain() == {a, b, c}
    assert c.get_ref_chain(ref_limit=2) == {b, c}
    bst = lgb.train({"verbosity": -1}, a, 1)
    assert callable(bst.set_network) and callable(bst.free_network)


@pytest.mark.parametrize("two_round", [False, True])
def test_parse_errors_in_parallel_regions_raise(lgb, tmp_path, two_round):
    """A malformed CSV value, a bad label token and an inconsistent query file are raised as
    LightGBMError from inside the OpenMP parse regions; the process must not abort
    (reference utils/openmp_wrapper.h:80-131)."""
    bad = tmp_path / "bad.csv"
    lines = [f"{i % 2},{i * 0.5},{i % 7}" for i in range(30000)]
    lines[17001] = "1,2.5,notanumber"
    bad.write_text("\n".join(lines) + "\n")
    params = {"verbosity": -1, "two_round": two_round}
    with pytest.raises(lgb.LightGBMError, match="notanumber"):
        lgb.Dataset(str(bad), params=params).construct()
    badlab = tmp_path / "badlab.csv"
    lines = [f"{i % 2},{i * 0.5},{i % 7}" for i in range(30000)]
    lines[29999] = "maybe,1.0,2.0"
    badlab.write_text("\n".join(lines) + "\n")
    with pytest.raises(lgb.LightGBMError, match="maybe"):
        lgb.Dataset(str(badlab), params=params).construct()
    good = tmp_path / "rank.csv"
    good.write_text("\n".join(f"{i % 3},{i},{i % 5}" for i in range(1000)) + "\n")
    (tmp_path / "rank.csv.query").write_text("600\n300\n")
    with pytest.raises(lgb.LightGBMError, match="query"):
        lgb.Dataset(str(good), params=params).construct()
    # the library is still usable afterwards
    ok = lgb.Dataset(np.arange(200.0).reshape(100, 2), np.arange(100) % 2)
    assert lgb.train({"objective": "binary", "verbosity": -1}, ok, 2).num_trees() == 2
