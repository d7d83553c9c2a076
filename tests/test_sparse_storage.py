"""Multi-value sparse group storage (reference src/io/multi_val_sparse_bin.hpp,
dataset.cpp:219-242 multi-val groups, feature_group.h:216 sparse bins).

Groups that are mostly at their most-frequent bin are stored as one CSR of global
histogram bins instead of dense row bytes. Storage must not change any model: the
same data trained with `is_enable_sparse` on and off gives identical trees, and the
subset / binary-file / add-features / validation paths keep reading the right bins.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import lambdagap_amd as lgb


def _data(n=6000, dense=6, sparse=40, density=0.03, seed=0):
    rng = np.random.default_rng(seed)
    xd = rng.normal(size=(n, dense))
    xs = sp.random(n, sparse, density=density, random_state=seed, format="csr",
                   data_rvs=lambda k: rng.uniform(0.5, 3.0, size=k)).toarray()
    # a categorical-ish sparse column and a wide (uint16-bin) dense column
    xs[:, 0] = np.where(rng.random(n) < 0.1, rng.integers(1, 6, size=n), 0)
    x = np.hstack([xd, xs])
    y = (xd[:, 0] + 0.5 * xd[:, 1] + xs[:, 1:6].sum(axis=1) + rng.normal(scale=0.3, size=n) > 0.8).astype(float)
    return x, y


PARAMS = dict(objective="binary", num_leaves=31, learning_rate=0.1, min_data_in_leaf=5, verbose=-1,
              enable_bundle=False, num_threads=4, deterministic=True)


def _train(x, y, rounds=15, **kw):
    p = dict(PARAMS, **kw)
    ds = lgb.Dataset(x, y, params=p)
    return lgb.train(p, ds, num_boost_round=rounds), ds


def _strip(model_str):
    # the parameters section records is_enable_sparse itself
    return model_str.split("\nparameters:")[0]


@pytest.mark.parametrize("bundle", [False, True])
def test_sparse_storage_identical_models(bundle):
    x, y = _data()
    b_sparse, _ = _train(x, y, enable_bundle=bundle, is_enable_sparse=True)
    b_dense, _ = _train(x, y, enable_bundle=bundle, is_enable_sparse=False)
    assert _strip(b_sparse.model_to_string()) == _strip(b_dense.model_to_string())
    np.testing.assert_array_equal(b_sparse.predict(x), b_dense.predict(x))


def test_sparse_storage_is_used_and_memory_smaller(tmp_path):
    x, y = _data(n=4000, sparse=60, density=0.02)
    p = dict(PARAMS, is_enable_sparse=True)
    ds = lgb.Dataset(x, y, params=p).construct()
    f_sparse = tmp_path / "s.bin"
    ds.save_binary(str(f_sparse))
    p2 = dict(PARAMS, is_enable_sparse=False)
    ds2 = lgb.Dataset(x, y, params=p2).construct()
    f_dense = tmp_path / "d.bin"
    ds2.save_binary(str(f_dense))
    # 60 sparse columns at ~2-12 % non-zeros: 4-byte entries beat 1 byte per row per group
    assert f_sparse.stat().st_size < 0.6 * f_dense.stat().st_size


def test_sparse_storage_binary_roundtrip_and_subset(tmp_path):
    x, y = _data(n=3000)
    p = dict(PARAMS, is_enable_sparse=True)
    ds = lgb.Dataset(x, y, params=p).construct()
    f = tmp_path / "train.bin"
    ds.save_binary(str(f))
    b_file = lgb.train(p, lgb.Dataset(str(f), params=p), num_boost_round=10)
    b_mem = lgb.train(p, lgb.Dataset(x, y, params=p), num_boost_round=10)
    assert _strip(b_file.model_to_string()) == _strip(b_mem.model_to_string())
    # subset of a sparse-stored set == a dense-stored set of the same rows
    idx = np.arange(0, 3000, 3)
    full_s = lgb.Dataset(x, y, params=p, free_raw_data=False)
    full_d = lgb.Dataset(x, y, params=dict(PARAMS, is_enable_sparse=False), free_raw_data=False)
    bs = lgb.train(p, full_s.subset(idx), num_boost_round=8)
    bd = lgb.train(dict(PARAMS, is_enable_sparse=False), full_d.subset(idx), num_boost_round=8)
    assert _strip(bs.model_to_string()) == _strip(bd.model_to_string())


def test_sparse_storage_validation_and_add_features():
    x, y = _data(n=4000)
    xv, yv = _data(n=1500, seed=3)
    p = dict(PARAMS, is_enable_sparse=True, metric="binary_logloss")
    res_s, res_d = {}, {}
    ds = lgb.Dataset(x, y, params=p)
    lgb.train(p, ds, 10, valid_sets=[lgb.Dataset(xv, yv, reference=ds)],
              callbacks=[lgb.record_evaluation(res_s)])
    pd_ = dict(p, is_enable_sparse=False)
    dd = lgb.Dataset(x, y, params=pd_)
    lgb.train(pd_, dd, 10, valid_sets=[lgb.Dataset(xv, yv, reference=dd)],
              callbacks=[lgb.record_evaluation(res_d)])
    # identical trees; the metric's OpenMP reduction may differ in the last bit
    np.testing.assert_allclose(res_s["valid_0"]["binary_logloss"], res_d["valid_0"]["binary_logloss"], rtol=1e-13)
    # adding columns to a sparse-stored set densifies it first; training still matches
    a = lgb.Dataset(x[:, :20], y, params=p, free_raw_data=False).construct()
    a.add_features_from(lgb.Dataset(x[:, 20:], params=p, free_raw_data=False).construct())
    b = lgb.Dataset(x[:, :20], y, params=pd_, free_raw_data=False).construct()
    b.add_features_from(lgb.Dataset(x[:, 20:], params=pd_, free_raw_data=False).construct())
    ba = lgb.train(p, a, 8)
    bb = lgb.train(pd_, b, 8)
    np.testing.assert_array_equal(ba.predict(x), bb.predict(x))


def test_sparse_storage_scipy_csr_input():
    x, y = _data(n=3000, sparse=80, density=0.01)
    xs = sp.csr_matrix(x)
    b1, _ = _train(xs, y, is_enable_sparse=True)
    b2, _ = _train(x, y, is_enable_sparse=False)
    assert _strip(b1.model_to_string()) == _strip(b2.model_to_string())


@pytest.mark.gpu
def test_sparse_storage_device_learner_materializes_rows():
    """A host-constructed sparse-stored set trained on the GPU: the device learner
    uploads full rows (Dataset::RowsForDevice) and grows the dense-stored set's trees."""
    x, y = _data(n=5000)
    xv, yv = _data(n=1000, seed=5)
    out = []
    for sparse in (True, False):
        p = dict(PARAMS, is_enable_sparse=sparse)
        ds = lgb.Dataset(x, y, params=p).construct()
        pg = dict(p, device_type="gpu")
        b = lgb.train(pg, ds, 10, valid_sets=[lgb.Dataset(xv, yv, reference=ds)])
        out.append(b.predict(xv, raw_score=True))
    np.testing.assert_allclose(out[0], out[1], rtol=0, atol=1e-12)


@pytest.mark.parametrize("sparse", [False, True])
def test_col_wise_and_row_wise_histograms_identical(sparse, capsys):
    """TrainingShareStates analogue: the thread split (rows vs feature groups) never changes
    a model; without force_* the first histogram times both and logs its choice."""
    x, y = _data(n=20000, dense=8, sparse=12, density=0.1)
    common = dict(PARAMS, is_enable_sparse=sparse, num_threads=4)
    col, _ = _train(x, y, rounds=8, force_col_wise=True, **common)
    row, _ = _train(x, y, rounds=8, force_row_wise=True, **common)
    assert _strip(col.model_to_string()) == _strip(row.model_to_string())
    auto, _ = _train(x, y, rounds=8, **dict(common, verbose=1))
    assert _strip(auto.model_to_string()) == _strip(row.model_to_string())
    assert "Auto-choosing" in capsys.readouterr().out
