"""Dataset / Booster expectations of the reference's test_basic.py
(/root/reference/tests/python_package_test/test_basic.py: chunked datasets, subset save
and group slicing, add_features_from semantics and renaming, CEGB effects and scaling
equalities), same data shapes and assertions."""
import os
from copy import deepcopy

import numpy as np
import pytest
from scipy import sparse
from sklearn.datasets import load_breast_cancer, load_svmlight_file
from sklearn.model_selection import train_test_split

import lambdagap_amd as lgb

DATA = os.path.join(os.path.dirname(__file__), "data")


class _NumpySequence(lgb.Sequence):
    def __init__(self, arr, batch_size):
        self.arr = arr
        self.batch_size = batch_size

    def __getitem__(self, idx):
        return self.arr[idx]

    def __len__(self):
        return len(self.arr)


def _chunks(X, size):
    return [X[i * size:(i + 1) * size, :] for i in range(X.shape[0] // size + 1)]


@pytest.mark.parametrize("linear", [False, True])
def test_chunked_dataset(linear):
    X_train, X_test, y_train, y_test = train_test_split(*load_breast_cancer(return_X_y=True), test_size=0.1,
                                                        random_state=2)
    size = X_train.shape[0] // 10 + 1
    params = {"bin_construct_sample_cnt": 100, **({"linear_tree": True} if linear else {})}
    train = lgb.Dataset(_chunks(X_train, size), label=y_train, params=params)
    valid = train.create_valid(_chunks(X_test, size), label=y_test, params=params)
    train.construct()
    valid.construct()


def test_save_dataset_subset_and_load_from_file(tmp_path, rng):
    data = rng.standard_normal(size=(100, 2))
    params = {"max_bin": 50, "min_data_in_bin": 10}
    ds = lgb.Dataset(data, params=params)
    ds.subset([1, 2, 3, 5, 8]).save_binary(tmp_path / "subset.bin")
    lgb.Dataset(tmp_path / "subset.bin", params=params).construct()


def test_subset_group():
    X_train, y_train = load_svmlight_file(os.path.join(DATA, "rank.train"))
    q_train = np.loadtxt(os.path.join(DATA, "rank.train.query"))
    train = lgb.Dataset(X_train, y_train, group=q_train)
    assert len(train.get_group()) == 201
    group = train.subset(list(range(10))).construct().get_group()
    assert len(group) == 2
    assert group[0] == 1
    assert group[1] == 9


def test_add_features_throws_if_num_data_unequal(rng):
    d1 = lgb.Dataset(rng.uniform(size=(100, 1))).construct()
    d2 = lgb.Dataset(rng.uniform(size=(10, 1))).construct()
    with pytest.raises(lgb.basic.LightGBMError,
                       match="Cannot add features from other Dataset with a different number of rows"):
        d1.add_features_from(d2)


def test_add_features_throws_if_datasets_unconstructed(rng):
    X1, X2 = rng.uniform(size=(100, 1)), rng.uniform(size=(100, 1))
    msg = "Both source and target Datasets must be constructed before adding features"
    for c1, c2 in ((False, False), (True, False), (False, True)):
        d1 = lgb.Dataset(X1)
        d2 = lgb.Dataset(X2)
        if c1:
            d1.construct()
        if c2:
            d2.construct()
        with pytest.raises(ValueError, match=msg):
            d1.add_features_from(d2)


def test_add_features_equal_data_on_alternating_used_unused(tmp_path, rng):
    X = rng.uniform(size=(100, 5))
    X[:, [1, 3]] = 0
    names = [f"col_{i}" for i in range(5)]
    for j in range(1, 5):
        d1 = lgb.Dataset(X[:, :j], feature_name=names[:j]).construct()
        d2 = lgb.Dataset(X[:, j:], feature_name=names[j:]).construct()
        d1.add_features_from(d2)
        d1._dump_text(tmp_path / "d1.txt")
        lgb.Dataset(X, feature_name=names).construct()._dump_text(tmp_path / "d.txt")
        assert (tmp_path / "d.txt").read_text() == (tmp_path / "d1.txt").read_text()


def test_add_features_same_booster_behaviour(tmp_path, rng):
    X = rng.uniform(size=(100, 5))
    X[:, [1, 3]] = 0
    names = [f"col_{i}" for i in range(5)]
    for j in range(1, 5):
        d1 = lgb.Dataset(X[:, :j], feature_name=names[:j]).construct()
        d2 = lgb.Dataset(X[:, j:], feature_name=names[j:]).construct()
        d1.add_features_from(d2)
        d = lgb.Dataset(X, feature_name=names).construct()
        y = rng.uniform(size=(100,))
        d1.set_label(y)
        d.set_label(y)
        b1 = lgb.Booster(train_set=d1)
        b = lgb.Booster(train_set=d)
        for _ in range(10):
            b.update()
            b1.update()
        b1.save_model(tmp_path / "d1.txt")
        b.save_model(tmp_path / "d.txt")
        assert (tmp_path / "d.txt").read_text() == (tmp_path / "d1.txt").read_text()


def test_add_features_from_different_sources(rng):
    pd = pytest.importorskip("pandas")
    n_row, n_col = 100, 5
    X = rng.uniform(size=(n_row, n_col))
    xxs = [X, sparse.csr_matrix(X), pd.DataFrame(X)]
    names = [f"col_{i}" for i in range(n_col)]
    seq_ds = lgb.Dataset(_NumpySequence(X, 30), feature_name=names, free_raw_data=False).construct()
    npy_list_ds = lgb.Dataset([X[:n_row // 2, :], X[n_row // 2:, :]], feature_name=names,
                              free_raw_data=False).construct()
    for x_1 in xxs:
        d1 = lgb.Dataset(x_1, feature_name=names, free_raw_data=True).construct()
        d2 = lgb.Dataset(x_1, feature_name=names, free_raw_data=True).construct()
        d1.add_features_from(d2)
        assert d1.data is None
        d1 = lgb.Dataset(x_1, feature_name=names, free_raw_data=False).construct()
        for d2 in (seq_ds, npy_list_ds):
            d1.add_features_from(d2)
            assert d1.data is None
        d1 = lgb.Dataset(x_1, feature_name=names, free_raw_data=False).construct()
        res_names = deepcopy(names)
        for idx, x_2 in enumerate(xxs, 2):
            original_type = type(d1.get_data())
            d2 = lgb.Dataset(x_2, feature_name=names, free_raw_data=False).construct()
            d1.add_features_from(d2)
            assert isinstance(d1.get_data(), original_type)
            assert d1.get_data().shape == (n_row, n_col * idx)
            res_names += [f"D{idx}_{name}" for name in names]
            assert d1.feature_name == res_names


def test_add_features_does_not_fail_if_initial_dataset_has_zero_informative_features(capsys, rng):
    dataset_a = lgb.Dataset(np.zeros((100, 1), dtype=np.float32), params={"verbose": 0}).construct()
    assert ("[LambdaGap] [Warning] There are no meaningful features which satisfy the provided configuration. "
            "Decreasing Dataset parameters min_data_in_bin or min_data_in_leaf and re-constructing Dataset might "
            "resolve this warning.\n") in capsys.readouterr().out
    dataset_b = lgb.Dataset(rng.uniform(size=(100, 5))).construct()
    handle = dataset_a.handle
    dataset_a.add_features_from(dataset_b)
    assert dataset_a.num_feature() == 6
    assert dataset_a.num_data() == 100
    assert dataset_a.handle is handle


def _cegb_data(rng):
    X = rng.uniform(size=(100, 5))
    X[:, [1, 3]] = 0
    y = rng.uniform(size=(100,))
    ds = lgb.Dataset(X, feature_name=[f"col_{i}" for i in range(5)]).construct()
    ds.set_label(y)
    return ds


def test_cegb_affects_behavior(tmp_path, rng):
    ds = _cegb_data(rng)
    base = lgb.Booster(train_set=ds)
    for _ in range(10):
        base.update()
    base.save_model(tmp_path / "base.txt")
    basetxt = (tmp_path / "base.txt").read_text()
    for case in ({"cegb_penalty_feature_coupled": [50, 100, 10, 25, 30]},
                 {"cegb_penalty_feature_lazy": [1, 2, 3, 4, 5]}, {"cegb_penalty_split": 1}):
        booster = lgb.Booster(train_set=ds, params=case)
        for _ in range(10):
            booster.update()
        booster.save_model(tmp_path / "case.txt")
        assert basetxt != (tmp_path / "case.txt").read_text()


def test_cegb_scaling_equalities(tmp_path, rng):
    ds = _cegb_data(rng)
    pairs = [({"cegb_penalty_feature_coupled": [1, 2, 1, 2, 1]},
              {"cegb_penalty_feature_coupled": [0.5, 1, 0.5, 1, 0.5], "cegb_tradeoff": 2}),
             ({"cegb_penalty_feature_lazy": [0.01, 0.02, 0.03, 0.04, 0.05]},
              {"cegb_penalty_feature_lazy": [0.005, 0.01, 0.015, 0.02, 0.025], "cegb_tradeoff": 2}),
             ({"cegb_penalty_split": 1}, {"cegb_penalty_split": 2, "cegb_tradeoff": 0.5})]
    for p1, p2 in pairs:
        b1 = lgb.Booster(train_set=ds, params=p1)
        b2 = lgb.Booster(train_set=ds, params=p2)
        for _ in range(10):
            b1.update()
            b2.update()
        b1.reset_parameter(p2)  # so the parameter sections match
        b1.save_model(tmp_path / "p1.txt")
        b2.save_model(tmp_path / "p2.txt")
        assert (tmp_path / "p1.txt").read_text() == (tmp_path / "p2.txt").read_text()
