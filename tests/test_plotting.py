"""Plotting smoke tests (matplotlib, Agg backend)."""
import numpy as np
import pytest

matplotlib = pytest.importorskip("matplotlib")
matplotlib.use("Agg")


@pytest.fixture(scope="module")
def fitted(lgb):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((500, 4))
    y = (X[:, 0] > 0).astype(int)
    return lgb.LGBMClassifier(n_estimators=10, verbose=-1).fit(X, y, eval_set=[(X, y)])


def test_plot_importance(lgb, fitted):
    ax = lgb.plot_importance(fitted, max_num_features=3)
    assert ax.get_title() == "Feature importance"
    assert len(ax.patches) <= 3


def test_plot_split_value_histogram(lgb, fitted):
    ax = lgb.plot_split_value_histogram(fitted, 0)
    assert len(ax.patches) > 0


def test_plot_metric(lgb, fitted):
    ax = lgb.plot_metric(fitted)
    assert ax.get_ylabel() == "binary_logloss"
    with pytest.raises(TypeError):
        lgb.plot_metric(fitted.booster_)


def test_plot_tree(lgb, fitted):
    ax = lgb.plot_tree(fitted, tree_index=1, show_info=["split_gain"])
    assert len(ax.texts) >= 3


def test_create_tree_digraph_needs_graphviz(lgb, fitted):
    try:
        import graphviz  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            lgb.create_tree_digraph(fitted)
