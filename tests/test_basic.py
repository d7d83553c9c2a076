"""CPU smoke tests of the Python API over the native core."""
import numpy as np
import pytest


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
