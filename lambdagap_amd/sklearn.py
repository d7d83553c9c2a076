"""scikit-learn estimators: LGBMModel, LGBMRegressor, LGBMClassifier, LGBMRanker.

Same constructor arguments, fitted attributes and fit/predict signatures as the
reference (python-package/lightgbm/sklearn.py:486 LGBMModel, :1314 regressor,
:1424 classifier, :1678 ranker), implemented over :func:`lambdagap_amd.train`.
"""
from __future__ import annotations

import copy
import functools
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np

import warnings

from .basic import Booster, Dataset, LightGBMError, _choose_param_value, _ConfigAliases
from .callback import record_evaluation
from .engine import train

try:
    from sklearn.base import BaseEstimator, ClassifierMixin, RegressorMixin
    from sklearn.preprocessing import LabelEncoder
    from sklearn.utils.multiclass import check_classification_targets
except ImportError:  # pragma: no cover
    raise

__all__ = ["LGBMModel", "LGBMRegressor", "LGBMClassifier", "LGBMRanker"]


class _ObjectiveFunctionWrapper:
    """Adapts a sklearn-style objective ``f(y_true, y_pred[, weight[, group]]) -> (grad, hess)``."""

    def __init__(self, func: Callable):
        self.func = func

    def __call__(self, preds: np.ndarray, dataset: Dataset):
        labels = dataset.get_label()
        argc = self.func.__code__.co_argcount
        if argc == 2:
            return self.func(labels, preds)
        if argc == 3:
            return self.func(labels, preds, dataset.get_weight())
        return self.func(labels, preds, dataset.get_weight(), dataset.get_group())


class _EvalFunctionWrapper:
    """Adapts ``f(y_true, y_pred[, weight[, group]]) -> (name, value, is_higher_better)``."""

    def __init__(self, func: Callable):
        self.func = func

    def __call__(self, preds: np.ndarray, dataset: Dataset):
        labels = dataset.get_label()
        argc = self.func.__code__.co_argcount
        if argc == 2:
            return self.func(labels, preds)
        if argc == 3:
            return self.func(labels, preds, dataset.get_weight())
        return self.func(labels, preds, dataset.get_weight(), dataset.get_group())


@functools.lru_cache(maxsize=None)
def _cpu_count(physical: bool) -> int:
    import joblib

    return joblib.cpu_count(only_physical_cores=physical)


def _ravel_column(y):
    """A (n, 1) label is accepted with sklearn's column-vector warning and flattened."""
    shape = getattr(y, "shape", None)
    if shape is not None and len(shape) == 2 and shape[1] == 1:
        warnings.warn("A column-vector y was passed when a 1d array was expected. Please change the shape of y "
                      "to (n_samples,), for example using ravel().", UserWarning)
        return np.asarray(y).ravel()
    return y


class LGBMModel(BaseEstimator):
    """Gradient boosting model with the scikit-learn estimator interface."""

    def __init__(self, boosting_type: str = "gbdt", num_leaves: int = 31, max_depth: int = -1,
                 learning_rate: float = 0.1, n_estimators: int = 100, subsample_for_bin: int = 200000,
                 objective: Optional[Union[str, Callable]] = None, class_weight: Optional[Union[Dict, str]] = None,
                 min_split_gain: float = 0.0, min_child_weight: float = 1e-3, min_child_samples: int = 20,
                 subsample: float = 1.0, subsample_freq: int = 0, colsample_bytree: float = 1.0,
                 reg_alpha: float = 0.0, reg_lambda: float = 0.0, random_state: Optional[Union[int, np.random.RandomState]] = None,
                 n_jobs: Optional[int] = None, importance_type: str = "split", **kwargs: Any):
        self.boosting_type = boosting_type
        self.objective = objective
        self.num_leaves = num_leaves
        self.max_depth = max_depth
        self.learning_rate = learning_rate
        self.n_estimators = n_estimators
        self.subsample_for_bin = subsample_for_bin
        self.min_split_gain = min_split_gain
        self.min_child_weight = min_child_weight
        self.min_child_samples = min_child_samples
        self.subsample = subsample
        self.subsample_freq = subsample_freq
        self.colsample_bytree = colsample_bytree
        self.reg_alpha = reg_alpha
        self.reg_lambda = reg_lambda
        self.random_state = random_state
        self.n_jobs = n_jobs
        self.importance_type = importance_type
        self.class_weight = class_weight
        self._other_params: Dict[str, Any] = {}
        self._Booster: Optional[Booster] = None
        self._evals_result: Dict[str, Any] = {}
        self._best_score: Dict[str, Any] = {}
        self._best_iteration = -1
        self._n_features = -1
        self._n_classes = -1
        self._objective = objective
        self._class_weight = None
        self._class_map = None
        self.fitted_ = False
        self.set_params(**kwargs)

    # ------------------------------------------------------------------ params
    def get_params(self, deep: bool = True) -> Dict[str, Any]:
        params = super().get_params(deep=deep)
        if type(self).__init__ is not LGBMModel.__init__:
            # subclasses with their own __init__ signature still report the base parameters
            import inspect

            for name in inspect.signature(LGBMModel.__init__).parameters:
                if name not in ("self", "kwargs") and name not in params and hasattr(self, name):
                    params[name] = getattr(self, name)
        params.update(self._other_params)
        return params

    def set_params(self, **params: Any) -> "LGBMModel":
        for key, value in params.items():
            setattr(self, key, value)
            if hasattr(self, f"_{key}"):
                setattr(self, f"_{key}", value)
            self._other_params[key] = value
        return self

    def _more_tags(self) -> Dict[str, Any]:
        return {"allow_nan": True, "X_types": ["2darray", "sparse", "1dlabels"]}

    def __sklearn_tags__(self):
        """scikit-learn >= 1.6 tags (the same facts as ``_more_tags``)."""
        tags = super().__sklearn_tags__()
        tags.input_tags.allow_nan = True
        tags.input_tags.sparse = True
        tags.target_tags.one_d_labels = True
        return tags

    def _default_objective(self) -> str:
        return "regression"

    def __sklearn_is_fitted__(self) -> bool:
        return getattr(self, "_Booster", None) is not None

    def _process_params(self, stage: str) -> Dict[str, Any]:
        params = self.get_params()
        params.pop("objective", None)
        # objective aliases given as keyword arguments win over `objective` (reference
        # sklearn.py _process_params, with the same warning)
        for alias in sorted(_ConfigAliases.get("objective") - {"objective"}):
            if alias in params:
                obj = params.pop(alias)
                warnings.warn(f"Found '{alias}' in params. Will use it instead of 'objective' argument", UserWarning)
                if stage == "fit":
                    self._objective = obj
        if hasattr(self, "_eval_at"):
            eval_at = self._eval_at
            for alias in sorted(_ConfigAliases.get("eval_at")):
                if alias in params:
                    warnings.warn(f"Found '{alias}' in params. Will use it instead of 'eval_at' argument", UserWarning)
                    eval_at = params.pop(alias)
            params["eval_at"] = eval_at
        for alias in ("class_weight", "importance_type", "n_estimators"):
            params.pop(alias, None)
        if isinstance(params.get("random_state"), np.random.RandomState):
            params["random_state"] = params["random_state"].randint(np.iinfo(np.int32).max)
        mapping = {"boosting_type": "boosting", "subsample_for_bin": "bin_construct_sample_cnt",
                   "min_split_gain": "min_gain_to_split", "min_child_weight": "min_sum_hessian_in_leaf",
                   "min_child_samples": "min_data_in_leaf", "subsample": "bagging_fraction",
                   "subsample_freq": "bagging_freq", "colsample_bytree": "feature_fraction",
                   "reg_alpha": "lambda_l1", "reg_lambda": "lambda_l2", "random_state": "seed",
                   "n_jobs": "num_threads"}
        out: Dict[str, Any] = {}
        n_jobs = params.pop("n_jobs", None)
        for k, v in params.items():
            if v is None:
                continue
            out[mapping.get(k, k)] = v
        # joblib conventions for n_jobs (None: physical cores, -k: all but k - 1 threads);
        # an explicit num_threads alias wins (reference sklearn.py _process_n_jobs)
        out = _choose_param_value("num_threads", out, n_jobs)
        nt = out["num_threads"]
        if nt is None:
            nt = _cpu_count(True)
        elif nt < 0:
            nt = max(_cpu_count(False) + 1 + nt, 1)
        out["num_threads"] = nt
        if callable(self._objective):
            out["objective"] = _ObjectiveFunctionWrapper(self._objective)
        else:
            out["objective"] = self._objective or self._default_objective()
        # the default metric is registered explicitly (a custom objective still reports the
        # estimator's natural metric: l2 / binary_logloss / multi_logloss / ndcg)
        default_metric = out["objective"] if isinstance(out["objective"], str) else {
            "regression": "l2", "binary": "binary_logloss", "multiclass": "multi_logloss",
            "lambdarank": "ndcg"}.get(self._default_objective())
        if default_metric is not None:
            out = _choose_param_value("metric", out, default_metric)
        out.setdefault("verbosity", -1)
        return out

    # ------------------------------------------------------------------ fit
    def fit(self, X, y, sample_weight=None, init_score=None, group=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_class_weight=None, eval_init_score=None, eval_group=None,
            eval_metric=None, feature_name="auto", categorical_feature="auto", callbacks=None,
            init_model=None, position=None, eval_position=None) -> "LGBMModel":
        y = _ravel_column(y)
        params = self._process_params("fit")
        feval = None
        if eval_metric is not None:
            metrics = eval_metric if isinstance(eval_metric, list) else [eval_metric]
            names = [m for m in metrics if isinstance(m, str)]
            funcs = [_EvalFunctionWrapper(m) for m in metrics if callable(m)]
            if names:
                base = params.get("metric")
                if base is None:
                    # keep the objective's default metric (objective names are metric aliases)
                    obj = params.get("objective")
                    base = [obj] if isinstance(obj, str) else []
                base = base if isinstance(base, list) else [base]
                params["metric"] = [*base, *[n for n in names if n not in base]]
            feval = funcs or None
        X_arr = X
        if hasattr(X, "shape"):
            self._n_features = X.shape[1]
        sw = sample_weight
        class_weight = self._class_weight if self._class_weight is not None else self.class_weight
        if class_weight is not None:
            cw = self._class_weight_from(class_weight, y)
            sw = cw if sw is None else np.asarray(sw) * cw
        train_set = Dataset(X_arr, label=y, weight=sw, group=group, init_score=init_score, position=position,
                            feature_name=feature_name, categorical_feature=categorical_feature, params=params)
        valid_sets: List[Dataset] = []
        names: List[str] = []
        if eval_set is not None:
            if isinstance(eval_set, tuple):
                eval_set = [eval_set]
            for i, (vx, vy) in enumerate(eval_set):
                if vx is X and vy is y:
                    vs = train_set
                else:
                    def _get(coll, i):
                        if coll is None:
                            return None
                        if isinstance(coll, dict):
                            return coll.get(i)
                        return coll[i]

                    vw = _get(eval_sample_weight, i)
                    vcw = _get(eval_class_weight, i)
                    if isinstance(vcw, dict) and getattr(self, "_class_map", None) is not None:
                        vcw = {self._class_map[k]: v for k, v in vcw.items()}  # original labels -> encoded
                    if vcw is not None:
                        cw = self._class_weight_from(vcw, vy)
                        vw = cw if vw is None else np.asarray(vw) * cw
                    vs = train_set.create_valid(vx, label=vy, weight=vw, group=_get(eval_group, i),
                                                init_score=_get(eval_init_score, i), position=_get(eval_position, i))
                valid_sets.append(vs)
                if eval_names is not None and i < len(eval_names):
                    names.append(eval_names[i])
                else:  # the training data passed as an eval set is reported as "training"
                    names.append("training" if vs is train_set else f"valid_{i}")
        if isinstance(init_model, LGBMModel):
            init_model = init_model.booster_
        self._evals_result = {}
        cbs = list(callbacks or [])
        cbs.append(record_evaluation(self._evals_result))
        self._Booster = train(params, train_set, num_boost_round=self.n_estimators, valid_sets=valid_sets,
                              valid_names=names, feval=feval, init_model=init_model, callbacks=cbs)
        self._best_iteration = self._Booster.best_iteration
        self._best_score = self._Booster.best_score
        self._n_features = self._Booster.num_feature()
        self.fitted_ = True
        return self

    def _compute_class_weight(self, y) -> np.ndarray:
        return self._class_weight_from(self._class_weight, y)

    @staticmethod
    def _class_weight_from(cw, y) -> np.ndarray:
        y = np.asarray(y)
        classes, counts = np.unique(y, return_counts=True)
        if cw == "balanced":
            weights = {c: len(y) / (len(classes) * n) for c, n in zip(classes, counts)}
        else:
            weights = {c: cw.get(c, 1.0) for c in classes}
        return np.array([weights[v] for v in y], dtype=np.float64)

    # ------------------------------------------------------------------ predict
    def predict(self, X, raw_score: bool = False, start_iteration: int = 0, num_iteration: Optional[int] = None,
                pred_leaf: bool = False, pred_contrib: bool = False, validate_features: bool = False, **kwargs):
        if self._Booster is None:
            raise LightGBMError("Estimator not fitted, call fit before exploiting the model.")
        if hasattr(X, "shape") and X.shape[1] != self._n_features:
            raise ValueError(f"X has {X.shape[1]} features, but {type(self).__name__} is expecting "
                             f"{self._n_features} features as input")
        # constructor / set_params parameters reach prediction too (pred_early_stop, ...), those
        # passed to predict() win (reference sklearn.py predict: _process_params("predict"))
        predict_params = self._process_params("predict")
        if not isinstance(predict_params.get("objective"), str):
            predict_params["objective"] = "none"  # a custom objective: raw scores (num_class kept)
        for alias in _ConfigAliases.get_by_alias("metric", "eval_at", "data", "X", "raw_score",
                                                 "start_iteration", "num_iteration", "pred_leaf", "pred_contrib",
                                                 *kwargs.keys()):
            predict_params.pop(alias, None)
        predict_params.update(kwargs)
        return self._Booster.predict(X, raw_score=raw_score, start_iteration=start_iteration,
                                     num_iteration=num_iteration, pred_leaf=pred_leaf, pred_contrib=pred_contrib,
                                     validate_features=validate_features, **predict_params)

    # ------------------------------------------------------------------ attributes
    def _check_fitted(self) -> None:
        if self._Booster is None:
            from sklearn.exceptions import NotFittedError

            raise NotFittedError("No booster found. Need to call fit beforehand.")

    @property
    def n_features_(self) -> int:
        self._check_fitted()
        return self._n_features

    @property
    def n_features_in_(self) -> int:
        self._check_fitted()
        return self._n_features

    @property
    def best_score_(self):
        self._check_fitted()
        return self._best_score

    @property
    def best_iteration_(self) -> int:
        self._check_fitted()
        return self._best_iteration

    @property
    def objective_(self):
        self._check_fitted()
        return self._objective or self._default_objective()

    @property
    def n_estimators_(self) -> int:
        self._check_fitted()
        return self._Booster.current_iteration()

    @property
    def n_iter_(self) -> int:
        return self.n_estimators_

    @property
    def booster_(self) -> Booster:
        self._check_fitted()
        return self._Booster

    @property
    def evals_result_(self):
        self._check_fitted()
        return self._evals_result

    @property
    def feature_importances_(self) -> np.ndarray:
        self._check_fitted()
        return self._Booster.feature_importance(importance_type=self.importance_type)

    @property
    def feature_name_(self) -> List[str]:
        self._check_fitted()
        return self._Booster.feature_name()

    @property
    def feature_names_in_(self) -> np.ndarray:
        return np.array(self.feature_name_)


class LGBMRegressor(RegressorMixin, LGBMModel):
    """LightGBM regressor."""

    def _default_objective(self) -> str:
        return "regression"

    def fit(self, X, y, sample_weight=None, init_score=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_init_score=None, eval_metric=None, feature_name="auto",
            categorical_feature="auto", callbacks=None, init_model=None):
        return super().fit(X, y, sample_weight=sample_weight, init_score=init_score, eval_set=eval_set,
                           eval_names=eval_names, eval_sample_weight=eval_sample_weight,
                           eval_init_score=eval_init_score, eval_metric=eval_metric, feature_name=feature_name,
                           categorical_feature=categorical_feature, callbacks=callbacks, init_model=init_model)


class LGBMClassifier(ClassifierMixin, LGBMModel):
    """LightGBM classifier (binary or multiclass; labels of any type)."""

    def _default_objective(self) -> str:
        return "binary" if self._n_classes <= 2 else "multiclass"

    def __sklearn_tags__(self):
        tags = super().__sklearn_tags__()
        if tags.classifier_tags is not None:
            tags.classifier_tags.multi_class = True
            tags.classifier_tags.multi_label = False
        return tags

    def fit(self, X, y, sample_weight=None, init_score=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_class_weight=None, eval_init_score=None, eval_metric=None,
            feature_name="auto", categorical_feature="auto", callbacks=None, init_model=None):
        y = _ravel_column(y)
        check_classification_targets(y)
        self._le = LabelEncoder().fit(y)
        y_enc = self._le.transform(y)
        self._class_map = dict(zip(self._le.classes_, range(len(self._le.classes_))))
        if isinstance(self.class_weight, dict):
            self._class_weight = {self._class_map[k]: v for k, v in self.class_weight.items()}
        self._classes = self._le.classes_
        self._n_classes = len(self._classes)
        # num_class follows the classes of THIS fit: a value set by an earlier fit is dropped
        prev = getattr(self, "_auto_num_class", None)
        if prev is not None and self._other_params.get("num_class") == prev:
            self._other_params.pop("num_class", None)
        self._auto_num_class = None
        multiclass_obj = not callable(self._objective) and self._objective is not None and str(self._objective) in (
            "multiclass", "softmax", "multiclassova", "multiclass_ova", "ova", "ovr")
        if self._n_classes > 2 or multiclass_obj:
            self._other_params["num_class"] = self._n_classes
            self._auto_num_class = self._n_classes
        valid = None
        if eval_set is not None:
            if isinstance(eval_set, tuple):
                eval_set = [eval_set]
            valid = []
            for vx, vy in eval_set:
                if vx is X and vy is y:
                    valid.append((vx, y_enc))
                else:
                    valid.append((vx, self._le.transform(vy)))
        if eval_metric is not None:
            # binary / multiclass metric names follow the task (reference LGBMClassifier.fit): a
            # multiclass objective stays multiclass even on two classes
            multiclass = self._n_classes > 2 or (isinstance(self._objective, str) and self._objective in (
                "multiclass", "softmax", "multiclassova", "multiclass_ova", "ova", "ovr"))
            metrics = eval_metric if isinstance(eval_metric, list) else [eval_metric]
            fixed = []
            for m in metrics:
                if isinstance(m, str) and multiclass:
                    m = {"logloss": "multi_logloss", "binary_logloss": "multi_logloss", "error": "multi_error",
                         "binary_error": "multi_error"}.get(m, m)
                elif isinstance(m, str):
                    m = {"logloss": "binary_logloss", "multi_logloss": "binary_logloss", "error": "binary_error",
                         "multi_error": "binary_error"}.get(m, m)
                fixed.append(m)
            eval_metric = fixed
        X_fit = X
        super().fit(X_fit, y_enc, sample_weight=sample_weight, init_score=init_score, eval_set=valid,
                    eval_names=eval_names, eval_sample_weight=eval_sample_weight, eval_class_weight=eval_class_weight,
                    eval_init_score=eval_init_score, eval_metric=eval_metric, feature_name=feature_name,
                    categorical_feature=categorical_feature, callbacks=callbacks, init_model=init_model)
        return self

    def predict(self, X, raw_score: bool = False, start_iteration: int = 0, num_iteration: Optional[int] = None,
                pred_leaf: bool = False, pred_contrib: bool = False, validate_features: bool = False, **kwargs):
        result = self.predict_proba(X, raw_score, start_iteration, num_iteration, pred_leaf, pred_contrib,
                                    validate_features, **kwargs)
        if callable(self._objective) or raw_score or pred_leaf or pred_contrib:
            return result
        idx = np.argmax(result, axis=1)
        return self._le.inverse_transform(idx)

    def predict_proba(self, X, raw_score: bool = False, start_iteration: int = 0,
                      num_iteration: Optional[int] = None, pred_leaf: bool = False, pred_contrib: bool = False,
                      validate_features: bool = False, **kwargs):
        result = super().predict(X, raw_score, start_iteration, num_iteration, pred_leaf, pred_contrib,
                                 validate_features, **kwargs)
        if callable(self._objective) and not (raw_score or pred_leaf or pred_contrib):
            return result
        if self._n_classes > 2 or raw_score or pred_leaf or pred_contrib or np.ndim(result) == 2:
            return result  # (a multiclass objective on two classes already gives both columns)
        return np.vstack((1.0 - result, result)).transpose()

    @property
    def classes_(self) -> np.ndarray:
        self._check_fitted()
        return self._classes

    @property
    def n_classes_(self) -> int:
        self._check_fitted()
        return self._n_classes


class LGBMRanker(LGBMModel):
    """LightGBM ranker (lambdarank by default; all LambdaGap `lambdarank_target`s via kwargs)."""

    def _default_objective(self) -> str:
        return "lambdarank"

    def fit(self, X, y, sample_weight=None, init_score=None, group=None, eval_set=None, eval_names=None,
            eval_sample_weight=None, eval_init_score=None, eval_group=None, eval_metric=None, eval_at=(1, 2, 3, 4, 5),
            feature_name="auto", categorical_feature="auto", callbacks=None, init_model=None, position=None,
            eval_position=None):
        if group is None:
            raise ValueError("Should set group for ranking task")
        if eval_set is not None:
            if eval_group is None:
                raise ValueError("Eval_group cannot be None when eval_set is not None")
            n = 1 if isinstance(eval_set, tuple) else len(eval_set)
            if len(eval_group) != n:
                raise ValueError("Length of eval_group should be equal to eval_set")
        self._eval_at = list(eval_at)
        return super().fit(X, y, sample_weight=sample_weight, init_score=init_score, group=group, eval_set=eval_set,
                           eval_names=eval_names, eval_sample_weight=eval_sample_weight,
                           eval_init_score=eval_init_score, eval_group=eval_group, eval_metric=eval_metric,
                           feature_name=feature_name, categorical_feature=categorical_feature, callbacks=callbacks,
                           init_model=init_model, position=position, eval_position=eval_position)
