"""Tree-growth policies beside the split scan: intermediate monotone constraints,
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
