"""Tree-growth policies beside the split scan: intermediate / advanced monotone constraints,
cost-effective gradient boosting and quantized-gradient training (reference
tests/python_package_test/test_engine.py: test_monotone_constraints,
test_cegb_*, test_quantized_training themes)."""
import numpy as np
import pytest


def _mono_data(rng, n=4000):
    X = rng.random((n, 4))
    y = 4 * X[:, 0] + 2 * np.sin(6 * X[:, 0]) - 3 * X[:, 1] * X[:, 2] + np.cos(8 * X[:, 3]) + 0.2 * rng.standard_normal(n)
    return X, y


def _is_monotone(b, rng, f, sign, nf=4):
    grid = np.linspace(0, 1, 60)
    for row in rng.random((25, nf)):
        Z = np.repeat(row[None, :], len(grid), 0)
        Z[:, f] = grid
        if not np.all(sign * np.diff(b.predict(Z)) >= -1e-10):
            return False
    return True


def test_intermediate_monotone_fits_at_least_as_well_as_basic(lgb, rng):
    X, y = _mono_data(rng)
    common = {"objective": "regression", "monotone_constraints": [1, -1, 0, 0], "verbosity": -1, "num_leaves": 31,
              "min_data_in_leaf": 10}
    res = {}
    for method in ("basic", "intermediate"):
        b = lgb.train(dict(common, monotone_constraints_method=method), lgb.Dataset(X, y), 60)
        assert _is_monotone(b, rng, 0, 1) and _is_monotone(b, rng, 1, -1), method
        res[method] = float(np.mean((b.predict(X) - y) ** 2))
    # intermediate bounds leaves by actual neighbour outputs instead of midpoints: looser, better fit
    assert res["intermediate"] <= res["basic"] * 1.001
    assert res["intermediate"] != res["basic"]


def test_advanced_monotone_fits_at_least_as_well_as_intermediate(lgb, rng):
    X, y = _mono_data(rng)
    common = {"objective": "regression", "monotone_constraints": [1, -1, 0, 0], "verbosity": -1, "num_leaves": 31,
              "min_data_in_leaf": 10}
    res, models = {}, {}
    for method in ("intermediate", "advanced"):
        b = lgb.train(dict(common, monotone_constraints_method=method), lgb.Dataset(X, y), 60)
        assert _is_monotone(b, rng, 0, 1) and _is_monotone(b, rng, 1, -1), method
        res[method] = float(np.mean((b.predict(X) - y) ** 2))
        models[method] = b.model_to_string()
    # advanced bounds each threshold only by the leaves its children actually touch
    assert res["advanced"] <= res["intermediate"] * 1.001
    strip = lambda s: s[:s.index("parameters:")]  # noqa: E731
    assert strip(models["advanced"]) != strip(models["intermediate"])


def _reference_monotone_set(lgb, rng, x3_to_category):
    """generate_trainset_for_monotone_constraints_tests (reference test_engine.py:2118-2146)."""
    n = 3000
    x1, x2, x3 = rng.uniform(size=n), rng.uniform(size=n), rng.uniform(size=n)
    cat = lambda v: np.digitize(v, bins=np.arange(0, 1, 0.01))  # noqa: E731
    X = np.column_stack((x1, x2, cat(x3) if x3_to_category else x3))
    s = 10.0 * (rng.uniform(size=6) + 0.5)
    y = (s[0] * x1 + np.sin(s[1] * np.pi * x1) - s[2] * x2 - np.cos(s[3] * np.pi * x2) - s[4] * x3
         - np.cos(s[5] * np.pi * x3) + rng.normal(0.0, 0.01, size=n))
    return lgb.Dataset(X, label=y, categorical_feature=[2] if x3_to_category else [], free_raw_data=False)


def _correctly_constrained(b, x3_to_category):
    n = 1000
    v = np.linspace(0, 1, n).reshape((n, 1))
    for fixed in np.linspace(0, 1, n)[:10]:
        fx = fixed * np.ones((n, 1))
        inc = b.predict(np.column_stack((v, fx, fx)))
        dec = b.predict(np.column_stack((fx, v, fx)))
        third = np.digitize(v, bins=np.arange(0, 1, 0.01)) if x3_to_category else v
        free = b.predict(np.column_stack((fx, fx, third)))
        if not ((np.diff(inc) >= 0).all() and (np.diff(dec) <= 0).all()
                and (np.diff(free) < 0).any() and (np.diff(free) > 0).any()):
            return False
    return True


@pytest.mark.parametrize("x3_to_category", [True, False])
@pytest.mark.parametrize("interactions", [True, False])
@pytest.mark.parametrize("method", ["basic", "intermediate", "advanced"])
def test_monotone_constraints_reference_cases(lgb, rng, x3_to_category, interactions, method):
    """test_monotone_constraints of the reference (test_engine.py:2151-2232): increasing /
    decreasing / free features, a categorical third feature, with and without interaction
    constraints."""
    ds = _reference_monotone_set(lgb, rng, x3_to_category)
    params = {"min_data": 20, "num_leaves": 20, "monotone_constraints": [1, -1, 0],
              "monotone_constraints_method": method, "use_missing": False, "verbosity": -1}
    if interactions:
        params["interaction_constraints"] = [[0], [1], [2]]
    b = lgb.train(params, ds)
    assert _correctly_constrained(b, x3_to_category)
    if interactions:
        for t in b.dump_model()["tree_info"]:
            feats = set()

            def walk(nd):
                if "split_index" in nd:
                    feats.add(nd["split_feature"])
                    walk(nd["left_child"])
                    walk(nd["right_child"])
            walk(t["tree_structure"])
            assert len(feats) <= 1


@pytest.mark.parametrize("method", ["basic", "intermediate", "advanced"])
def test_monotone_penalty_delays_monotone_splits(lgb, rng, method):
    """test_monotone_penalty (reference test_engine.py:2235-2273): with penalty 2 the first two
    levels split only on the free feature, and monotone splits still happen deeper."""
    mono = [1, -1, 0]
    ds = _reference_monotone_set(lgb, rng, False)
    b = lgb.train({"max_depth": 5, "monotone_constraints": mono, "monotone_penalty": 2.0,
                   "monotone_constraints_method": method, "verbosity": -1}, ds, 10)

    def first_free(nd, k):
        if k <= 0 or "leaf_value" in nd:
            return True
        return mono[nd["split_feature"]] == 0 and first_free(nd["left_child"], k - 1) and \
            first_free(nd["right_child"], k - 1)

    def any_mono(nd):
        if "leaf_value" in nd:
            return False
        return mono[nd["split_feature"]] != 0 or any_mono(nd["left_child"]) or any_mono(nd["right_child"])

    for t in b.dump_model()["tree_info"]:
        assert first_free(t["tree_structure"], 2)
        assert any_mono(t["tree_structure"])


def test_monotone_penalty_max_forbids_monotone_splits(lgb, rng):
    """test_monotone_penalty_max (reference test_engine.py:2278-2310): a penalty equal to the depth
    leaves only the free feature, so the model equals one trained on that feature alone."""
    ds = _reference_monotone_set(lgb, rng, False)
    X, y = ds.data, ds.label
    common = {"max_depth": 5, "verbosity": -1, "gpu_use_dp": True}
    con = lgb.train(dict(common, monotone_constraints=[1, -1, 0], monotone_penalty=5), ds, 10)
    free = lgb.train(common, lgb.Dataset(X[:, 2].reshape(-1, 1), label=y), 10)
    np.testing.assert_allclose(con.predict(X), free.predict(X[:, 2].reshape(-1, 1)), rtol=1e-12)


def test_cegb_affects_behavior(lgb, rng):
    X = rng.standard_normal((1500, 5))
    y = X[:, 0] + 0.5 * X[:, 1] + 0.2 * X[:, 2] + 0.1 * rng.standard_normal(1500)
    base = lgb.train({"verbosity": -1}, lgb.Dataset(X, y), 10).model_to_string()
    for extra in ({"cegb_penalty_split": 1.0}, {"cegb_penalty_feature_coupled": [5, 1, 2, 3, 4]},
                  {"cegb_penalty_feature_lazy": [1, 2, 3, 4, 5]}):
        m = lgb.train(dict({"verbosity": -1}, **extra), lgb.Dataset(X, y), 10).model_to_string()
        strip = lambda s: s[:s.index("parameters:")] if "parameters:" in s else s  # noqa: E731
        assert strip(m) != strip(base), extra


def test_cegb_scaling_equalities(lgb, rng):
    X = rng.standard_normal((1000, 5))
    y = X[:, 0] - X[:, 3] + 0.3 * rng.standard_normal(1000)
    pairs = [({"cegb_penalty_feature_coupled": [1, 2, 1, 2, 1]},
              {"cegb_penalty_feature_coupled": [0.5, 1, 0.5, 1, 0.5], "cegb_tradeoff": 2}),
             ({"cegb_penalty_feature_lazy": [0.01, 0.02, 0.03, 0.04, 0.05]},
              {"cegb_penalty_feature_lazy": [0.005, 0.01, 0.015, 0.02, 0.025], "cegb_tradeoff": 2}),
             ({"cegb_penalty_split": 1}, {"cegb_penalty_split": 2, "cegb_tradeoff": 0.5})]
    for p1, p2 in pairs:
        b1 = lgb.train(dict({"verbosity": -1}, **p1), lgb.Dataset(X, y), 6)
        b2 = lgb.train(dict({"verbosity": -1}, **p2), lgb.Dataset(X, y), 6)
        np.testing.assert_allclose(b1.predict(X), b2.predict(X), rtol=1e-12)


def test_cegb_split_penalty_shrinks_trees(lgb, rng):
    X = rng.standard_normal((3000, 4))
    y = X[:, 0] + 0.01 * X[:, 1] + 0.1 * rng.standard_normal(3000)
    leaves = []
    for pen in (0.0, 0.005, 0.05):
        b = lgb.train({"verbosity": -1, "cegb_penalty_split": pen}, lgb.Dataset(X, y), 5)
        leaves.append(sum(t["num_leaves"] for t in b.dump_model()["tree_info"]))
    assert leaves[0] >= leaves[1] >= leaves[2] and leaves[0] > leaves[2]


@pytest.mark.parametrize("objective", ["binary", "regression"])
@pytest.mark.parametrize("renew", [False, True])
def test_quantized_training(lgb, rng, objective, renew):
    n = 6000
    X = rng.standard_normal((n, 6))
    z = X[:, 0] + 0.5 * X[:, 1] ** 2 - X[:, 2] + 0.3 * rng.standard_normal(n)
    y = (z > 0.5).astype(float) if objective == "binary" else z
    params = {"objective": objective, "verbosity": -1, "num_leaves": 15, "seed": 3}
    full = lgb.train(params, lgb.Dataset(X, y), 40)
    q = lgb.train(dict(params, use_quantized_grad=True, num_grad_quant_bins=4, quant_train_renew_leaf=renew),
                  lgb.Dataset(X, y), 40)
    if objective == "binary":
        from sklearn.metrics import roc_auc_score

        a_full, a_q = roc_auc_score(y, full.predict(X)), roc_auc_score(y, q.predict(X))
        assert a_q > a_full - 0.02, (a_q, a_full)
    else:
        e_full, e_q = np.mean((full.predict(X) - y) ** 2), np.mean((q.predict(X) - y) ** 2)
        assert e_q < e_full * 1.5 + 0.02, (e_q, e_full)
    assert q.model_to_string() != full.model_to_string()


def test_quantized_leaf_values_are_quantized_sums(lgb, rng):
    """Without leaf renewal every leaf output is -G/(H+l2) of integer-level sums: with a constant
    hessian (L2 regression) the hessian sum is count * h, so outputs are multiples of the
    gradient scale divided by the leaf hessian."""
    X = rng.standard_normal((2000, 3))
    y = X[:, 0] + 0.1 * rng.standard_normal(2000)
    b = lgb.train({"objective": "regression", "verbosity": -1, "num_leaves": 4, "use_quantized_grad": True,
                   "num_grad_quant_bins": 4, "stochastic_rounding": False, "learning_rate": 1.0,
                   "boost_from_average": False}, lgb.Dataset(X, y), 1)
    t = b.dump_model()["tree_info"][0]["tree_structure"]
    gscale = np.max(np.abs(y)) / 2  # g = score - y with score 0
    leaves = []

    def walk(nd):
        if "leaf_value" in nd:
            leaves.append((nd["leaf_value"], nd["leaf_count"]))
        else:
            walk(nd["left_child"])
            walk(nd["right_child"])
    walk(t)
    for v, c in leaves:
        k = -v * c / gscale  # integer sum of quantized gradient levels
        assert abs(k - round(k)) < 1e-3, (v, c, k)


@pytest.mark.parametrize("pool_mb", [0.01, 0.2])
def test_histogram_pool_size_bounds_cached_histograms(lgb, rng, pool_mb):
    """histogram_pool_size (reference HistogramPool, feature_histogram.hpp:1367-1594): with room
    for only a few leaf histograms the learner rebuilds evicted parents from the rows instead of
    subtracting, which gives the same trees (float gradients sum exactly in fp64 bins)."""
    X = rng.standard_normal((5000, 20))
    y = X[:, 0] + np.sin(X[:, 1]) + 0.1 * rng.standard_normal(5000)
    params = {"verbosity": -1, "num_leaves": 63}
    base = lgb.train(params, lgb.Dataset(X, y), 10)
    pooled = lgb.train(dict(params, histogram_pool_size=pool_mb), lgb.Dataset(X, y), 10)
    np.testing.assert_allclose(pooled.predict(X), base.predict(X), rtol=0, atol=1e-12)
    # a monotone rescan of a leaf whose histogram was dropped rebuilds it from the leaf's rows
    # (the reference skips the rescan and can break the bounds): the model stays monotone
    mono = dict(params, monotone_constraints=[1, -1] + [0] * 18, monotone_constraints_method="advanced")
    b = lgb.train(dict(mono, histogram_pool_size=pool_mb), lgb.Dataset(X, y), 10)
    grid = np.linspace(-3, 3, 60)
    for row in rng.standard_normal((10, 20)):
        Z = np.repeat(row[None, :], len(grid), 0)
        Z[:, 0] = grid
        assert np.all(np.diff(b.predict(Z)) >= -1e-10)
        Z[:, 0] = row[0]
        Z[:, 1] = grid
        assert np.all(np.diff(b.predict(Z)) <= 1e-10)


def test_linear_tree_refit_keeps_coefficients_by_feature(lgb):
    """Linear-tree refit matches each leaf's old coefficients to features by id
    (linear_tree_learner.cpp; reference linear_tree_learner.cpp:357-363 blends old and new per
    feature): with refit_decay_rate=1 every leaf keeps its own coefficients exactly."""
    import json

    rng = np.random.default_rng(5)
    n = 4000
    X = rng.standard_normal((n, 3))
    y = 2.0 * X[:, 0] - 3.0 * X[:, 1] + 0.5 * X[:, 2] + 0.05 * rng.standard_normal(n)
    params = {"objective": "regression", "linear_tree": True, "num_leaves": 4, "verbosity": -1, "seed": 1,
              "refit_decay_rate": 1.0}
    b = lgb.train(params, lgb.Dataset(X, y), 3)
    X2 = X + 0.01 * rng.standard_normal(X.shape)
    r = b.refit(X2, y, decay_rate=1.0)

    def coefs(booster):
        out = {}
        for ti, t in enumerate(booster.dump_model()["tree_info"]):
            stack = [t["tree_structure"]]
            while stack:
                nd = stack.pop()
                if "split_index" in nd:
                    stack += [nd["left_child"], nd["right_child"]]
                else:
                    for f, c in zip(nd.get("leaf_features", []), nd.get("leaf_coeff", [])):
                        out[(ti, nd["leaf_index"], f)] = c
        return out

    old, new = coefs(b), coefs(r)
    assert old, "the model has linear leaves"
    assert set(new) == set(old)
    for key, c in new.items():
        assert c == pytest.approx(old[key], rel=1e-12, abs=1e-12), (key, c, old[key])
