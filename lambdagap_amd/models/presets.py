"""Benchmark configurations of the reference (BASELINE.json "configs") as
parameter presets with matching synthetic-data builders.

Reference: docs/GPU-Performance.rst (Higgs 255 bins / 63 leaves), docs/Experiments.rst
(MS-LTR ranking, Expo / Allstate regression), BASELINE.json.
"""
from __future__ import annotations

from typing import Any, Dict, Tuple

import numpy as np

from ..utils.synthetic import make_higgs_like, make_ranking, make_regression

PRESETS: Dict[str, Dict[str, Any]] = {
    # flagship: boosting iters/sec + AUC on Higgs-shape binary data (bench.py)
    "higgs": {"objective": "binary", "num_leaves": 63, "max_bin": 255, "learning_rate": 0.1,
              "min_data_in_leaf": 1, "min_sum_hessian_in_leaf": 100, "device_type": "gpu"},
    # LambdaRank on grouped queries (MS-LTR shape: 136 features, ~120 docs per query)
    "ltr": {"objective": "lambdarank", "num_leaves": 255, "max_bin": 255, "learning_rate": 0.1,
            "min_data_in_leaf": 50, "min_sum_hessian_in_leaf": 0, "metric": "ndcg", "eval_at": [1, 3, 5, 10],
            "device_type": "gpu"},
    # wide regression with EFB (sparse features) + GOSS sampling
    "regression_goss": {"objective": "regression", "num_leaves": 255, "max_bin": 63, "learning_rate": 0.1,
                        "data_sample_strategy": "goss", "enable_bundle": True, "device_type": "gpu"},
}


def preset(name: str, **overrides: Any) -> Dict[str, Any]:
    """Copy of a preset parameter dict with overrides applied."""
    if name not in PRESETS:
        raise ValueError(f"Unknown preset {name!r}; choose from {sorted(PRESETS)}")
    params = dict(PRESETS[name])
    params.update(overrides)
    return params


def preset_data(name: str, rows: int, seed: int = 7) -> Tuple[np.ndarray, np.ndarray, Any]:
    """Synthetic data of the preset's shape: (X, y, group_sizes_or_None)."""
    if name == "higgs":
        X, y = make_higgs_like(rows, seed=seed)
        return X, y, None
    if name == "ltr":
        # ~120 documents per query on average (MS-LTR shape)
        return make_ranking(max(1, rows // 120), num_features=136, docs_per_query=(60, 180), seed=seed)
    if name == "regression_goss":
        X, y = make_regression(rows, num_features=500, density=0.1, seed=seed)
        return X, y, None
    raise ValueError(f"Unknown preset {name!r}")
