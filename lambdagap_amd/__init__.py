"""lambdagap_amd: a gradient boosting framework for AMD Instinct MI355X.

Same user API as LambdaGap / LightGBM (Dataset, Booster, train, cv, the
scikit-learn estimators, the lambdarank targets of LambdaGap), with a native
C++ core and hand-written HIP kernels for gfx950 (``device_type="gpu"``),
data-parallel across GPUs over RCCL.
"""
from __future__ import annotations

from .basic import Booster, Dataset, LightGBMError, Sequence, device_count, phase_timer_report, register_logger
from .callback import EarlyStopException, early_stopping, log_evaluation, record_evaluation, reset_parameter
from .engine import CVBooster, cv, train

__version__ = "4.6.0.99+mi355x.1"

__all__ = ["Dataset", "Booster", "CVBooster", "Sequence", "LightGBMError", "register_logger", "train", "cv",
           "early_stopping", "log_evaluation", "record_evaluation", "reset_parameter", "EarlyStopException",
           "device_count", "phase_timer_report", "LGBMModel", "LGBMRegressor", "LGBMClassifier", "LGBMRanker",
           "plot_importance", "plot_split_value_histogram", "plot_metric", "plot_tree", "create_tree_digraph"]

try:
    from .sklearn import LGBMClassifier, LGBMModel, LGBMRanker, LGBMRegressor
except ImportError:  # pragma: no cover - scikit-learn missing
    pass
try:
    from .plotting import create_tree_digraph, plot_importance, plot_metric, plot_split_value_histogram, plot_tree
except ImportError:  # pragma: no cover
    pass
