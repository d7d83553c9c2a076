"""Tree-walk expectations of the reference's test_plotting.py that need no graphviz
(graphviz is not installed here): the numeric / categorical split-direction helpers
reproduce pred_leaf for zero, NaN and categorical example rows, and create_tree_digraph
validates tree_index and example_case before drawing."""
import numpy as np
import pytest
from sklearn.datasets import make_regression

import lambdagap_amd as lgb


@pytest.mark.parametrize("use_missing", [True, False])
@pytest.mark.parametrize("zero_as_missing", [True, False])
def test_numeric_split_direction(use_missing, zero_as_missing):
    if use_missing and zero_as_missing:
        pytest.skip("use_missing and zero_as_missing both set to True")
    X, y = make_regression(n_samples=100, n_features=4, n_informative=2, random_state=42)
    rng = np.random.RandomState(0)
    zero_mask = rng.rand(X.shape[0]) < 0.05
    X[zero_mask, :] = 0
    if use_missing:
        nan_mask = ~zero_mask & (rng.rand(X.shape[0]) < 0.1)
        X[nan_mask, :] = np.nan
    bst = lgb.train({"num_leaves": 127, "min_child_samples": 1, "use_missing": use_missing,
                     "zero_as_missing": zero_as_missing, "verbose": -1}, lgb.Dataset(X, y), num_boost_round=1)

    def walk(case):
        node = bst.dump_model()["tree_info"][0]["tree_structure"]
        while "decision_type" in node:
            d = lgb.plotting._determine_direction_for_numeric_split(
                fval=case[0][node["split_feature"]], threshold=node["threshold"],
                missing_type_str=node["missing_type"], default_left=node["default_left"])
            node = node["left_child"] if d == "left" else node["right_child"]
        return node["leaf_index"]

    case_zero = X[zero_mask][[0]]
    leaf_zero = bst.predict(case_zero, pred_leaf=True)[0]
    assert walk(case_zero) == leaf_zero
    if use_missing:
        case_nan = X[nan_mask][[0]]
        leaf_nan = bst.predict(case_nan, pred_leaf=True)[0]
        assert walk(case_nan) == leaf_nan
        assert leaf_zero != leaf_nan


def test_categorical_split_direction_matches_pred_leaf():
    rng = np.random.RandomState(0)
    x1 = rng.rand(100)
    cat = rng.randint(1, 3, size=x1.size)
    X = np.vstack([x1, cat]).T
    y = x1 + 2 * cat
    bst = lgb.train({"num_leaves": 7, "verbose": -1},
                    lgb.Dataset(X, y, feature_name=["x1", "cat"], categorical_feature=["cat"]), num_boost_round=3)
    mod = bst.dump_model()
    saw_cat = False
    for row in range(10):
        case = X[[row]]
        for i in range(3):
            node = mod["tree_info"][i]["tree_structure"]
            while "decision_type" in node:
                f = node["split_feature"]
                if node["decision_type"] == "<=":
                    d = lgb.plotting._determine_direction_for_numeric_split(case[0][f], node["threshold"],
                                                                            node["missing_type"], node["default_left"])
                else:
                    saw_cat = True
                    d = lgb.plotting._determine_direction_for_categorical_split(case[0][f], node["threshold"])
                node = node["left_child"] if d == "left" else node["right_child"]
            assert node["leaf_index"] == bst.predict(case, start_iteration=i, num_iteration=1, pred_leaf=True)[0]
    assert saw_cat
    assert lgb.plotting._determine_direction_for_categorical_split(np.nan, "1||2") == "right"
    assert lgb.plotting._determine_direction_for_categorical_split(-1, "1||2") == "right"


@pytest.mark.parametrize("input_type", ["array", "dataframe"])
def test_empty_example_case_on_tree_digraph_raises_error(input_type):
    X, y = make_regression(n_samples=100, n_features=4, n_informative=2, random_state=42)
    if input_type == "dataframe":
        pd = pytest.importorskip("pandas")
        X = pd.DataFrame(X)
    bst = lgb.train({"num_leaves": 3, "verbose": -1}, lgb.Dataset(X, y), num_boost_round=1)
    with pytest.raises(ValueError, match="example_case must have a single row."):
        lgb.create_tree_digraph(bst, tree_index=0, example_case=X[:0])
    with pytest.raises(IndexError, match="tree_index is out of range."):
        lgb.create_tree_digraph(bst, tree_index=83)
