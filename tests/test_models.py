"""lambdagap_amd.models: ranking family helpers and benchmark presets."""
import numpy as np
import pytest


def test_targets_listed_match_native(lgb):
    from lambdagap_amd.models import LAMBDARANK_TARGETS, lambdarank_params
    from lambdagap_amd.utils import make_ranking

    assert len(LAMBDARANK_TARGETS) == 18
    X, y, g = make_ranking(30, num_features=8, seed=1)
    for t in LAMBDARANK_TARGETS:
        p = lambdarank_params(t, k=10, verbosity=-1)
        lgb.train(p, lgb.Dataset(X, y, group=g), 1)  # the native objective accepts every target
    with pytest.raises(ValueError):
        lambdarank_params("nope")


def test_lambdagap_ranker_params_roundtrip(lgb):
    from sklearn.base import clone

    from lambdagap_amd.models import LambdaGapRanker
    from lambdagap_amd.utils import make_ranking

    X, y, g = make_ranking(40, num_features=8, seed=2)
    r = LambdaGapRanker(lambdarank_target="lambdagap-s-plus", lambdagap_weight=0.5, num_leaves=7, n_estimators=5)
    r.fit(X, y, group=g)
    assert r.booster_.params["lambdarank_target"] == "lambdagap-s-plus"
    c = clone(r)
    assert c.get_params()["lambdarank_target"] == "lambdagap-s-plus"
    assert c.get_params()["num_leaves"] == 7
    assert r.predict(X).shape == (X.shape[0],)


def test_presets_train(lgb):
    from lambdagap_amd.models import preset, preset_data

    for name in ("higgs", "ltr", "regression_goss"):
        X, y, g = preset_data(name, 3000)
        p = preset(name, device_type="cpu", verbosity=-1, num_leaves=15)
        b = lgb.train(p, lgb.Dataset(X, y, group=g), 2)
        assert b.num_trees() >= 2
