"""Custom text parsers (`parser_config_file`, include/lgap/parser.h).

Reference: include/LightGBM/dataset.h:400-486 (Parser / ParserFactory / ParserReflector),
src/io/parser.cpp:287-318, tests/python_package_test/test_basic.py::test_smoke_custom_parser.
"""
from pathlib import Path

import numpy as np
import pytest


def test_smoke_custom_parser(lgb, tmp_path):
    """An unregistered class name fails with the reference's message."""
    data_path = Path(__file__).parent / "data" / "binary.train"
    parser_config_file = tmp_path / "parser.ini"
    parser_config_file.write_text('{"className": "dummy", "id": "1"}')
    data = lgb.Dataset(str(data_path), params={"parser_config_file": str(parser_config_file)})
    with pytest.raises(lgb.basic.LightGBMError,
                       match="Cannot find parser class 'dummy', please register first or check config format"):
        data.construct()


def test_registered_parser_trains_saves_and_predicts(lgb, tmp_path):
    """The built-in plugin "lambdagap.label_last" (label in the LAST column, ';' delimited):
    the model equals one trained on the same arrays, carries the parser config in its text,
    and predicting from a file parses through the same class after a save / load round trip."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal((600, 4))
    y = (X[:, 0] + 0.5 * X[:, 1] > 0).astype(float)
    f = tmp_path / "rows.txt"
    with open(f, "w") as fo:
        for row, lab in zip(X, y):
            fo.write(";".join(f"{v:.17g}" for v in row) + f";{lab:g}\n")
    cfg = tmp_path / "parser.json"
    cfg.write_text('{"className": "lambdagap.label_last", "delimiter": ";"}')
    params = {"objective": "binary", "num_leaves": 7, "verbosity": -1, "min_data_in_leaf": 5}
    b_file = lgb.train(params, lgb.Dataset(str(f), params={"parser_config_file": str(cfg)}), 5)
    b_arr = lgb.train(params, lgb.Dataset(X, y), 5)
    text = b_file.model_to_string()
    assert "parser:" in text and "lambdagap.label_last" in text and '"labelId"' in text
    strip = lambda s: s.split("end of trees")[0].split("feature_names=")[1].split("\n", 1)[1]
    assert strip(text) == strip(b_arr.model_to_string())
    model = tmp_path / "model.txt"
    b_file.save_model(str(model))
    loaded = lgb.Booster(model_file=str(model))
    np.testing.assert_allclose(loaded.predict(str(f)), b_arr.predict(X), rtol=1e-12, atol=1e-12)


def test_custom_parser_with_header_uses_default_names(lgb, tmp_path):
    """With header=true and a custom parser the raw header's names do not describe the parser's
    columns (the label moves, widths may differ): the features get the default Column_i names
    (reference dataset_loader.cpp:86-89) and the model equals one trained on the arrays."""
    rng = np.random.default_rng(1)
    X = rng.standard_normal((500, 3))
    y = (X[:, 0] - X[:, 2] > 0).astype(float)
    f = tmp_path / "rows_h.txt"
    with open(f, "w") as fo:
        fo.write("label_first_name;b;c;d\n")
        for row, lab in zip(X, y):
            fo.write(";".join(f"{v:.17g}" for v in row) + f";{lab:g}\n")
    cfg = tmp_path / "parser.json"
    cfg.write_text('{"className": "lambdagap.label_last", "delimiter": ";"}')
    params = {"objective": "binary", "num_leaves": 7, "verbosity": -1, "min_data_in_leaf": 5}
    ds = lgb.Dataset(str(f), params={"parser_config_file": str(cfg), "header": True})
    b_file = lgb.train(params, ds, 4)
    assert b_file.feature_name() == ["Column_0", "Column_1", "Column_2"]
    b_arr = lgb.train(params, lgb.Dataset(X, y), 4)
    np.testing.assert_allclose(b_file.predict(X), b_arr.predict(X), rtol=1e-12, atol=1e-12)


def test_custom_parser_predict_drops_columns_the_model_never_saw(lgb, tmp_path):
    """Predicting a file through the model's custom parser: a feature index past the model's
    features (a column training never had) is a shape error (reference predictor.hpp:176-178);
    under predict_disable_shape_check it is ignored, as the reference's CopyToPredictBuffer
    (predictor.hpp:259) ignores it, and the predictions equal those of the training columns."""
    rng = np.random.default_rng(2)
    X = rng.standard_normal((400, 4))
    y = (X[:, 1] - X[:, 3] > 0).astype(float)
    f = tmp_path / "rows.txt"
    with open(f, "w") as fo:
        for row, lab in zip(X, y):
            fo.write(";".join(f"{v:.17g}" for v in row) + f";{lab:g}\n")
    cfg = tmp_path / "parser.json"
    cfg.write_text('{"className": "lambdagap.label_last", "delimiter": ";"}')
    params = {"objective": "binary", "num_leaves": 7, "verbosity": -1, "min_data_in_leaf": 5}
    bst = lgb.train(params, lgb.Dataset(str(f), params={"parser_config_file": str(cfg)}), 4)
    # one extra trailing column: the parser reads it as the label and the old label column as
    # feature 4, which the 4-feature model never saw
    wide = tmp_path / "rows_wide.txt"
    with open(wide, "w") as fo:
        for row, lab in zip(X, y):
            fo.write(";".join(f"{v:.17g}" for v in row) + f";{lab:g};7\n")
    with pytest.raises(lgb.basic.LightGBMError, match="predict_disable_shape_check"):
        bst.predict(str(wide))
    np.testing.assert_allclose(bst.predict(str(wide), predict_disable_shape_check=True), bst.predict(X),
                               rtol=1e-12, atol=1e-12)
