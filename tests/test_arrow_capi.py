"""Arrow C data interface input, fast single-row prediction, sparse SHAP output and
serialized dataset references (reference tests/python_package_test/test_arrow.py,
test_basic.py / c_api_test themes)."""
import ctypes

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")


def _table(X, nulls=None, chunks=1):
    cols = {}
    for j in range(X.shape[1]):
        mask = None if nulls is None else nulls[:, j]
        cols[f"f{j}"] = pa.array(X[:, j], mask=mask)
    t = pa.table(cols)
    if chunks > 1:
        parts = np.array_split(np.arange(X.shape[0]), chunks)
        t = pa.concat_tables([t.slice(int(p[0]), len(p)) for p in parts])
    return t


def test_arrow_dataset_matches_numpy(lgb, rng):
    X = rng.standard_normal((3000, 4))
    nulls = rng.random(X.shape) < 0.05
    Xn = X.copy()
    Xn[nulls] = np.nan
    y = (np.nan_to_num(Xn[:, 0]) + Xn[:, 1] > 0).astype(float)
    params = {"objective": "binary", "verbosity": -1, "num_leaves": 15}
    ref = lgb.train(params, lgb.Dataset(Xn, y), 10)
    for chunks in (1, 3):
        t = _table(X, nulls, chunks)
        ds = lgb.Dataset(t, label=pa.array(y))
        b = lgb.train(params, ds, 10)
        assert b.feature_name() == ["f0", "f1", "f2", "f3"]
        np.testing.assert_allclose(b.predict(Xn), ref.predict(Xn), rtol=1e-12)
        np.testing.assert_allclose(b.predict(t), ref.predict(Xn), rtol=1e-12)


def test_arrow_mixed_types_and_fields(lgb, rng):
    n = 1000
    t = pa.table({"i8": pa.array(rng.integers(-5, 5, n), pa.int8()),
                  "u16": pa.array(rng.integers(0, 300, n), pa.uint16()),
                  "i64": pa.array(rng.integers(-1000, 1000, n), pa.int64()),
                  "f32": pa.array(rng.standard_normal(n).astype(np.float32)),
                  "b": pa.array(rng.random(n) < 0.5)})
    X = np.column_stack([t.column(c).to_numpy().astype(np.float64) for c in t.column_names])
    y = X[:, 0] + X[:, 3] + rng.standard_normal(n) * 0.1
    w = rng.random(n) + 0.5
    ds = lgb.Dataset(t, label=pa.chunked_array([y[:500], y[500:]]), weight=pa.array(w)).construct()
    np.testing.assert_allclose(ds.get_field("weight"), w.astype(np.float32))
    np.testing.assert_allclose(ds.get_field("label"), y.astype(np.float32))
    b1 = lgb.train({"verbosity": -1}, ds, 5)
    b2 = lgb.train({"verbosity": -1}, lgb.Dataset(X, y, weight=w), 5)
    np.testing.assert_allclose(b1.predict(X), b2.predict(X), rtol=1e-10)


def test_fast_single_row_predict(lgb, rng):
    from lambdagap_amd.basic import _LIB, _c_str, _check

    X = rng.standard_normal((500, 5))
    y = X[:, 0] - X[:, 1]
    b = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 8)
    full = b.predict(X)
    fc = ctypes.c_void_p()
    _check(_LIB.LGBM_BoosterPredictForMatSingleRowFastInit(b.handle, ctypes.c_int(0), ctypes.c_int(0),
                                                           ctypes.c_int(-1), ctypes.c_int(1), ctypes.c_int32(5),
                                                           _c_str(""), ctypes.byref(fc)))
    out = np.zeros(1)
    n = ctypes.c_int64(0)
    for i in range(0, 500, 37):
        row = np.ascontiguousarray(X[i])
        _check(_LIB.LGBM_BoosterPredictForMatSingleRowFast(fc, row.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n),
                                                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        assert n.value == 1
        assert out[0] == pytest.approx(full[i], rel=1e-12)
    _check(_LIB.LGBM_FastConfigFree(fc))


@pytest.mark.parametrize("fmt", ["csr", "csc"])
@pytest.mark.parametrize("objective", ["regression", "multiclass"])
def test_sparse_contrib_output(lgb, rng, fmt, objective):
    import scipy.sparse as sps

    X = rng.standard_normal((400, 6))
    X[rng.random(X.shape) < 0.6] = 0.0
    if objective == "multiclass":
        y = rng.integers(0, 3, 400)
        params = {"objective": "multiclass", "num_class": 3, "verbosity": -1}
    else:
        y = X[:, 0] * 2 + X[:, 2]
        params = {"verbosity": -1}
    b = lgb.train(params, lgb.Dataset(X, y), 5)
    dense = b.predict(X, pred_contrib=True)
    Xs = sps.csr_matrix(X) if fmt == "csr" else sps.csc_matrix(X)
    out = b.predict(Xs, pred_contrib=True)
    if objective == "multiclass":
        assert isinstance(out, list) and len(out) == 3
        for k in range(3):
            assert out[k].format == fmt
            np.testing.assert_allclose(out[k].toarray(), dense[:, k * 7:(k + 1) * 7], rtol=1e-10, atol=1e-12)
    else:
        assert out.format == fmt
        np.testing.assert_allclose(out.toarray(), dense, rtol=1e-10, atol=1e-12)


def test_serialized_reference_and_streaming_push(lgb, rng):
    from lambdagap_amd.basic import _LIB, _c_str, _check

    X = rng.standard_normal((800, 4))
    y = X[:, 0] + 0.1 * rng.standard_normal(800)
    ref = lgb.Dataset(X, y, params={"verbosity": -1}).construct()
    buf = ctypes.c_void_p()
    n = ctypes.c_int32(0)
    _check(_LIB.LGBM_DatasetSerializeReferenceToBinary(ref.handle, ctypes.byref(buf), ctypes.byref(n)))
    raw = bytearray(n.value)
    v = ctypes.c_uint8(0)
    for i in range(n.value):
        _check(_LIB.LGBM_ByteBufferGetAt(buf, ctypes.c_int32(i), ctypes.byref(v)))
        raw[i] = v.value
    _check(_LIB.LGBM_ByteBufferFree(buf))
    blob = (ctypes.c_char * len(raw)).from_buffer(raw)
    out = ctypes.c_void_p()
    _check(_LIB.LGBM_DatasetCreateFromSerializedReference(blob, ctypes.c_int32(len(raw)), ctypes.c_int64(800),
                                                          ctypes.c_int32(1), _c_str("verbosity=-1"), ctypes.byref(out)))
    # push in two batches with metadata (labels + per-row query ids are not used by regression)
    for s0 in (0, 500):
        part = np.ascontiguousarray(X[s0:s0 + (500 if s0 == 0 else 300)])
        lab = np.ascontiguousarray(y[s0:s0 + part.shape[0]], dtype=np.float32)
        _check(_LIB.LGBM_DatasetPushRowsWithMetadata(out, part.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(1),
                                                     ctypes.c_int32(part.shape[0]), ctypes.c_int32(4),
                                                     ctypes.c_int32(s0), lab.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                     None, None, None, ctypes.c_int32(0)))
    streamed = lgb.Dataset(None)
    streamed.handle = out
    streamed._predictor = None
    b1 = lgb.Booster({"verbosity": -1}, streamed)
    b2 = lgb.Booster({"verbosity": -1}, lgb.Dataset(X, y, params={"verbosity": -1}))
    for _ in range(5):
        b1.update()
        b2.update()
    np.testing.assert_allclose(b1.predict(X), b2.predict(X), rtol=1e-10)
