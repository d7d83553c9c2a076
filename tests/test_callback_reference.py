"""Callback and logger expectations of the reference
(/root/reference/tests/python_package_test/test_callback.py, test_utilities.py):
callbacks survive pickle / joblib / cloudpickle with their scheduling attributes,
early_stopping validates its argument, and a registered logger receives the native
log lines, the callbacks' messages and Python-side warnings."""
import logging
import pickle

import cloudpickle
import joblib
import numpy as np
import pytest

import lambdagap_amd as lgb


def _roundtrip(obj, serializer, tmp_path):
    path = tmp_path / "obj.bin"
    if serializer == "pickle":
        path.write_bytes(pickle.dumps(obj))
        return pickle.loads(path.read_bytes())  # our own object, written here
    if serializer == "joblib":
        joblib.dump(obj, path)
        return joblib.load(path)
    path.write_bytes(cloudpickle.dumps(obj))
    return cloudpickle.loads(path.read_bytes())


SERIALIZERS = ["pickle", "joblib", "cloudpickle"]


def reset_feature_fraction(boosting_round):
    return 0.6 if boosting_round < 15 else 0.8


@pytest.mark.parametrize("serializer", SERIALIZERS)
def test_early_stopping_callback_is_picklable(serializer, tmp_path):
    cb = lgb.early_stopping(stopping_rounds=5)
    back = _roundtrip(cb, serializer, tmp_path)
    assert back.order == 30
    assert back.before_iteration is False
    assert cb.stopping_rounds == back.stopping_rounds == 5


def test_early_stopping_callback_rejects_invalid_stopping_rounds_with_informative_errors():
    with pytest.raises(TypeError, match="early_stopping_round should be an integer. Got 'str'"):
        lgb.early_stopping(stopping_rounds="neverrrr")


@pytest.mark.parametrize("stopping_rounds", [-10, -1, 0])
def test_early_stopping_callback_accepts_non_positive_stopping_rounds(stopping_rounds):
    assert lgb.early_stopping(stopping_rounds=stopping_rounds).enabled is False


@pytest.mark.parametrize("serializer", SERIALIZERS)
def test_log_evaluation_callback_is_picklable(serializer, tmp_path):
    cb = lgb.log_evaluation(period=42)
    back = _roundtrip(cb, serializer, tmp_path)
    assert back.order == 10
    assert back.before_iteration is False
    assert cb.period == back.period == 42


@pytest.mark.parametrize("serializer", SERIALIZERS)
def test_record_evaluation_callback_is_picklable(serializer, tmp_path):
    results = {}
    cb = lgb.record_evaluation(eval_result=results)
    back = _roundtrip(cb, serializer, tmp_path)
    assert back.order == 20
    assert back.before_iteration is False
    assert cb.eval_result == back.eval_result
    assert cb.eval_result is results


@pytest.mark.parametrize("serializer", SERIALIZERS)
def test_reset_parameter_callback_is_picklable(serializer, tmp_path):
    params = {"bagging_fraction": [0.7] * 5 + [0.6] * 5, "feature_fraction": reset_feature_fraction}
    cb = lgb.reset_parameter(**params)
    back = _roundtrip(cb, serializer, tmp_path)
    assert back.order == 10
    assert back.before_iteration is True
    assert cb.kwargs == back.kwargs == params


@pytest.fixture
def restore_logger():
    saved = lgb.basic._LOGGER
    yield
    lgb.basic._LOGGER = saved


def test_register_logger(tmp_path, restore_logger):
    logger = logging.getLogger("LambdaGapTest")
    logger.setLevel(logging.DEBUG)
    log_file = tmp_path / "test_logger.log"
    handler = logging.FileHandler(log_file, mode="w", encoding="utf-8")
    handler.setFormatter(logging.Formatter("%(levelname)s | %(message)s"))
    logger.addHandler(handler)

    def dummy_metric(_, __):
        logger.debug("In dummy_metric")
        return "dummy_metric", 1, True

    lgb.register_logger(logger)
    X = np.array([[1, 2, 3], [1, 2, 4], [1, 2, 4], [1, 2, 3]], dtype=np.float32)
    y = np.array([0, 1, 1, 0])
    records = {}
    lgb.train({"objective": "binary", "metric": ["auc", "binary_error"], "verbose": 1},
              lgb.Dataset(X, y, categorical_feature=[1]), num_boost_round=10, feval=dummy_metric,
              valid_sets=[lgb.Dataset(X, y, categorical_feature=[1])],
              callbacks=[lgb.record_evaluation(records), lgb.log_evaluation(2), lgb.early_stopping(10)])
    handler.flush()
    lines = log_file.read_text(encoding="utf-8").strip().split("\n")
    logger.removeHandler(handler)
    # the reference's sequence (its native lines carry the [LightGBM] prefix, ours [LambdaGap])
    assert ("INFO | [LambdaGap] [Warning] There are no meaningful features which satisfy the provided configuration. "
            "Decreasing Dataset parameters min_data_in_bin or min_data_in_leaf and re-constructing Dataset might "
            "resolve this warning.") in lines
    assert "INFO | Training until validation scores don't improve for 10 rounds" in lines
    assert lines.count("DEBUG | In dummy_metric") == 10
    for it in (2, 4, 6, 8, 10):
        assert f"INFO | [{it}]\tvalid_0's auc: 0.5\tvalid_0's binary_error: 0.5\tvalid_0's dummy_metric: 1" in lines
    i = lines.index("INFO | Did not meet early stopping. Best iteration is:")
    assert lines[i + 1] == "[1]\tvalid_0's auc: 0.5\tvalid_0's binary_error: 0.5\tvalid_0's dummy_metric: 1"


def test_register_invalid_logger(restore_logger):
    class NoInfo:
        def warning(self, msg):
            print(msg)

    class NoWarning:
        def info(self, msg):
            print(msg)

    class NotCallable:
        def __init__(self):
            self.info = 1
            self.warning = 2

    for bad in (NoInfo(), NoWarning(), NotCallable()):
        with pytest.raises(TypeError, match="Logger must provide 'info' and 'warning' method"):
            lgb.register_logger(bad)


def test_register_custom_logger(restore_logger):
    logged = []

    class CustomLogger:
        def custom_info(self, msg):
            logged.append(msg)

        def custom_warning(self, msg):
            logged.append(msg)

    lgb.register_logger(CustomLogger(), info_method_name="custom_info", warning_method_name="custom_warning")
    lgb.basic._log_info("info message")
    lgb.basic._log_warning("warning message")
    assert logged == ["info message", "warning message"]
    logged.clear()
    X = np.array([[1, 2, 3], [1, 2, 4], [1, 2, 4], [1, 2, 3]], dtype=np.float32)
    ds = lgb.Dataset(X, np.array([0, 1, 1, 0]), categorical_feature=[1])
    lgb.train({"objective": "binary", "metric": "auc"}, ds, num_boost_round=10, valid_sets=[ds])
    assert logged, "custom logger was not called"
