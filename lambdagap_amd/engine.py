"""High-level training API: :func:`train`, :func:`cv`, :class:`CVBooster`.

Reference: python-package/lightgbm/engine.py (train loop with callbacks and
early stopping, k-fold CV with stratification / group folds).
"""
from __future__ import annotations

import copy
import os
from collections import OrderedDict, defaultdict
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple, Union

import numpy as np

from . import callback as cb
from .basic import Booster, Dataset, LightGBMError, _choose_param_value

__all__ = ["train", "cv", "CVBooster"]


def _pop_num_rounds(params: Dict[str, Any], num_boost_round: int) -> Tuple[Dict[str, Any], int]:
    """num_iterations from params beats the argument; the main name beats its aliases, then the
    first alias given (reference engine.py _choose_num_iterations)."""
    params = dict(params)
    given = [a for a in params if a in ("num_iterations", "num_iteration", "n_iter", "num_tree", "num_trees",
                                        "num_round", "num_rounds", "nrounds", "num_boost_round", "n_estimators",
                                        "max_iter")]
    if given:
        main = "num_iterations" if "num_iterations" in given else given[0]
        values = {a: params[a] for a in given}
        num_boost_round = int(values[main])
        if len(set(str(v) for v in values.values())) > 1:
            import warnings

            warnings.warn(f"Found conflicting values for num_iterations provided via 'params': "
                          f"{', '.join(f'{a}={v}' for a, v in values.items())}. "
                          f"LightGBM will perform up to {num_boost_round} boosting rounds.")
        for a in given:
            params.pop(a)
    params["num_iterations"] = num_boost_round
    return params, num_boost_round


def _early_stop_params(params: Dict[str, Any]) -> Tuple[Optional[int], bool, float]:
    """early_stopping_round from params under its main name (aliases folded into it); None
    removes it, a non-integer is a TypeError, <= 0 keeps it but stops nothing (reference
    engine.py train + callback._should_enable_early_stopping)."""
    rounds = None
    for alias in ("early_stopping_rounds", "early_stopping", "n_iter_no_change", "early_stopping_round"):
        if alias in params:
            rounds = params.pop(alias)
            if alias == "early_stopping_round":
                break
    if rounds is not None:
        if not isinstance(rounds, int) or isinstance(rounds, bool):
            raise TypeError(f"early_stopping_round should be an integer. Got '{type(rounds).__name__}'")
        params["early_stopping_round"] = rounds
    first_only = bool(params.get("first_metric_only", False))
    min_delta = float(params.get("early_stopping_min_delta", 0.0))
    return rounds, first_only, min_delta


def train(params: Dict[str, Any], train_set: Dataset, num_boost_round: int = 100,
          valid_sets: Optional[List[Dataset]] = None, valid_names: Optional[List[str]] = None,
          feval: Optional[Union[Callable, List[Callable]]] = None, init_model: Optional[Union[str, Booster]] = None,
          feature_name: Any = "auto", categorical_feature: Any = "auto", keep_training_booster: bool = False,
          callbacks: Optional[List[Callable]] = None) -> Booster:
    """Train a booster for ``num_boost_round`` rounds."""
    if not isinstance(train_set, Dataset):
        raise TypeError(f"train() only accepts Dataset object, train_set has type '{type(train_set).__name__}'.")
    if num_boost_round <= 0:
        raise ValueError(f"Number of boosting rounds must be greater than 0. Got {num_boost_round}.")
    if isinstance(valid_sets, Dataset):
        valid_sets = [valid_sets]
    if isinstance(valid_names, str):
        valid_names = [valid_names]
    if isinstance(valid_sets, list):
        for i, item in enumerate(valid_sets):
            if not isinstance(item, Dataset):
                raise TypeError("Every item in valid_sets must be a Dataset object. "
                                f"Item {i} has type '{type(item).__name__}'.")
    if params is not None and not isinstance(params, dict):
        raise TypeError(f"params must be a dict, got '{type(params).__name__}'.")
    params = copy.deepcopy(params) if params else {}
    fobj = None
    obj = params.get("objective")
    if callable(obj):
        fobj = obj
        params["objective"] = "none"
    params, num_boost_round = _pop_num_rounds(params, num_boost_round)
    es_rounds, first_only, min_delta = _early_stop_params(params)
    if feature_name != "auto":
        train_set.feature_name = feature_name
    if categorical_feature != "auto":
        train_set.categorical_feature = categorical_feature
    if isinstance(init_model, str):
        predictor = Booster(model_file=init_model)
    elif isinstance(init_model, Booster):
        predictor = init_model
    else:
        predictor = None
    init_iteration = predictor.current_iteration() if predictor is not None else 0
    # continued training: the init model's raw scores become the init score of the training
    # and validation sets (also for file data / constructed Datasets), and the Booster puts the
    # init model's trees first (reference engine.py train -> Dataset._set_predictor)
    train_set._update_params(params)._set_predictor(predictor)
    booster = Booster(params=params, train_set=train_set)
    valid_sets = valid_sets or []
    names = valid_names or []
    is_valid_contain_train = False
    train_data_name = "training"
    for i, vs in enumerate(valid_sets):
        if vs is train_set:
            is_valid_contain_train = True
            if i < len(names):
                train_data_name = names[i]
            continue
        name = names[i] if i < len(names) else f"valid_{i}"
        vs._update_params(params).set_reference(train_set)
        vs._set_predictor(predictor)
        booster.add_valid(vs, name)
    booster.set_train_data_name(train_data_name)
    callbacks = list(callbacks or [])
    if es_rounds is not None and es_rounds > 0:
        verbose = int(params.get("verbosity", params.get("verbose", 1))) > 0
        callbacks.append(cb.early_stopping(es_rounds, first_only, verbose=verbose, min_delta=min_delta))
    before = sorted([c for c in callbacks if getattr(c, "before_iteration", False)], key=lambda c: getattr(c, "order", 0))
    after = sorted([c for c in callbacks if not getattr(c, "before_iteration", False)],
                   key=lambda c: getattr(c, "order", 0))
    booster.best_iteration = 0
    evaluation_result_list: List[Any] = []
    for i in range(init_iteration, init_iteration + num_boost_round):
        for c in before:
            c(cb.CallbackEnv(model=booster, params=params, iteration=i, begin_iteration=init_iteration,
                             end_iteration=init_iteration + num_boost_round, evaluation_result_list=None))
        # like the reference, a finished update (no split possible) does not end the loop:
        # later iterations retry, evaluate and run the callbacks
        booster.update(fobj=fobj)
        evaluation_result_list = []
        if valid_sets or feval is not None:
            if is_valid_contain_train:
                evaluation_result_list.extend(booster.eval_train(feval))
            evaluation_result_list.extend(booster.eval_valid(feval))
        try:
            for c in after:
                c(cb.CallbackEnv(model=booster, params=params, iteration=i, begin_iteration=init_iteration,
                                 end_iteration=init_iteration + num_boost_round,
                                 evaluation_result_list=evaluation_result_list))
        except cb.EarlyStopException as e:
            booster.best_iteration = e.best_iteration + 1
            evaluation_result_list = e.best_score
            break
    booster.best_score = defaultdict(OrderedDict)
    for item in evaluation_result_list:
        booster.best_score[item[0]][item[1]] = item[2]
    if not keep_training_booster:
        # the returned model is the saved one: trees past best_iteration are dropped
        # (reference engine.py train: model_from_string(model_to_string()))
        booster.model_from_string(booster.model_to_string()).free_dataset()
    return booster


class CVBooster:
    """The boosters of a k-fold cross-validation run."""

    def __init__(self, model_file: Optional[str] = None):
        self.boosters: List[Booster] = []
        self.best_iteration = -1
        if model_file is not None:
            import json

            with open(model_file) as f:
                self._from_dict(json.load(f))

    def _append(self, booster: Booster) -> None:
        self.boosters.append(booster)

    def _from_dict(self, models: Dict[str, Any]) -> None:
        self.best_iteration = models["best_iteration"]
        self.boosters = [Booster(model_str=s) for s in models["boosters"]]

    def _to_dict(self, num_iteration: Optional[int], start_iteration: int, importance_type: str) -> Dict[str, Any]:
        return {"best_iteration": self.best_iteration,
                "boosters": [b.model_to_string(num_iteration=num_iteration, start_iteration=start_iteration,
                                               importance_type=importance_type) for b in self.boosters]}

    def model_to_string(self, num_iteration: Optional[int] = None, start_iteration: int = 0,
                        importance_type: str = "split") -> str:
        import json

        return json.dumps(self._to_dict(num_iteration, start_iteration, importance_type))

    def model_from_string(self, model_str: str) -> "CVBooster":
        import json

        self._from_dict(json.loads(model_str))
        return self

    def save_model(self, filename: str, num_iteration: Optional[int] = None, start_iteration: int = 0,
                   importance_type: str = "split") -> "CVBooster":
        with open(filename, "w") as f:
            f.write(self.model_to_string(num_iteration, start_iteration, importance_type))
        return self

    def __getattr__(self, name: str) -> Callable:
        # only public Booster methods are broadcast (dunder / private lookups, e.g. by pickle
        # before `boosters` exists, must fail normally)
        if name.startswith("_"):
            raise AttributeError(name)

        def handler(*args: Any, **kwargs: Any) -> List[Any]:
            return [getattr(b, name)(*args, **kwargs) for b in self.boosters]

        return handler

    def __getstate__(self) -> Dict[str, Any]:
        return vars(self)

    def __setstate__(self, state: Dict[str, Any]) -> None:
        vars(self).update(state)


def _make_folds(full: Dataset, folds, nfold: int, params: Dict[str, Any], seed: int, fpreproc, stratified: bool,
                shuffle: bool, eval_train_metric: bool):
    full.construct()
    num_data = full.num_data()
    if folds is not None:
        if hasattr(folds, "split"):
            group_info = full.get_group()
            if group_info is not None:
                group_info = np.asarray(group_info, dtype=np.int32)
                flatted_group = np.repeat(np.arange(len(group_info)), repeats=group_info)
            else:
                flatted_group = np.zeros(num_data, dtype=np.int32)
            folds = folds.split(X=np.empty(num_data), y=full.get_label(), groups=flatted_group)
    else:
        # reference engine.py _make_n_folds: GroupKFold over queries for ranking objectives,
        # StratifiedKFold when stratified, else nfold contiguous chunks of num_data // nfold rows
        # of a (seeded) permutation
        from sklearn.model_selection import GroupKFold, StratifiedKFold

        ranking = {"lambdarank", "rank_xendcg", "xendcg", "xe_ndcg", "xe_ndcg_mart", "xendcg_mart"}
        if any(params.get(a, "") in ranking for a in ("objective", "objective_type", "app", "application", "loss")):
            group_info = full.get_group()
            if group_info is None:
                raise LightGBMError("Ranking tasks require query information")
            group_info = np.asarray(group_info, dtype=np.int32)
            flatted_group = np.repeat(np.arange(len(group_info)), repeats=group_info)
            folds = GroupKFold(n_splits=nfold).split(X=np.empty(num_data), groups=flatted_group)
        elif stratified:
            skf = StratifiedKFold(n_splits=nfold, shuffle=shuffle, random_state=seed if shuffle else None)
            folds = skf.split(X=np.empty(num_data), y=full.get_label())
        else:
            order = np.random.RandomState(seed).permutation(num_data) if shuffle else np.arange(num_data)
            kstep = int(num_data / nfold)
            test_id = [order[i:i + kstep] for i in range(0, num_data, kstep)]
            folds = [(np.concatenate([test_id[j] for j in range(nfold) if j != k]), test_id[k]) for k in range(nfold)]
    ret = CVBooster()
    for train_idx, test_idx in folds:
        train_set = full.subset(sorted(train_idx))
        valid_set = full.subset(sorted(test_idx))
        if fpreproc is not None:
            train_set, valid_set, tparam = fpreproc(train_set, valid_set, params.copy())
        else:
            tparam = params
        b = Booster(tparam, train_set)
        if eval_train_metric:
            b.add_valid(train_set, "train")
        b.add_valid(valid_set, "valid")
        ret._append(b)
    return ret


def _agg_cv_result(raw_results: List[List[Tuple[str, str, float, bool]]]):
    """(dataset, metric, mean, is_higher_better, stdv) per (dataset, metric) over the folds
    (reference engine.py _agg_cv_result)."""
    values: Dict[Tuple[str, str], List[float]] = OrderedDict()
    higher: Dict[Tuple[str, str], bool] = {}
    for one in raw_results:
        for data_name, metric, value, hib in one:
            higher[(data_name, metric)] = hib
            values.setdefault((data_name, metric), []).append(value)
    return [(k[0], k[1], float(np.mean(v)), higher[k], float(np.std(v))) for k, v in values.items()]


def cv(params: Dict[str, Any], train_set: Dataset, num_boost_round: int = 100, folds=None, nfold: int = 5,
       stratified: bool = True, shuffle: bool = True, metrics: Optional[Union[str, List[str]]] = None,
       feval: Optional[Union[Callable, List[Callable]]] = None, init_model=None, feature_name: Any = "auto",
       categorical_feature: Any = "auto", fpreproc=None, seed: int = 0, callbacks: Optional[List[Callable]] = None,
       eval_train_metric: bool = False, return_cvbooster: bool = False) -> Dict[str, Any]:
    """k-fold cross validation; returns {"valid <metric>-mean": [...], "valid <metric>-stdv": [...]}."""
    if not isinstance(train_set, Dataset):
        raise TypeError(f"cv() only accepts Dataset object, train_set has type '{type(train_set).__name__}'.")
    if num_boost_round <= 0:
        raise ValueError(f"Number of boosting rounds must be greater than 0. Got {num_boost_round}.")
    params = copy.deepcopy(params) if params else {}
    fobj = None
    if callable(params.get("objective")):
        fobj = params["objective"]
        params["objective"] = "none"
    params, num_boost_round = _pop_num_rounds(params, num_boost_round)
    es_rounds, first_only, min_delta = _early_stop_params(params)
    if metrics is not None:
        params["metric"] = metrics
    if feature_name != "auto":
        train_set.feature_name = feature_name
    if categorical_feature != "auto":
        train_set.categorical_feature = categorical_feature
    if isinstance(init_model, (str, os.PathLike)):
        predictor = Booster(model_file=str(init_model))
    elif isinstance(init_model, Booster):
        predictor = init_model
    else:
        predictor = None
    # every fold continues from init_model: the full set's init score is the model's raw score,
    # fold subsets inherit it, and each fold Booster merges the model's trees
    train_set._update_params(params)._set_predictor(predictor)
    results: Dict[str, List[float]] = defaultdict(list)
    cvfolds = _make_folds(train_set, folds, nfold, params, seed, fpreproc, stratified, shuffle, eval_train_metric)
    callbacks = list(callbacks or [])
    if es_rounds is not None and es_rounds > 0:
        verbose = int(params.get("verbosity", params.get("verbose", 1))) > 0
        callbacks.append(cb.early_stopping(es_rounds, first_only, verbose=verbose, min_delta=min_delta))
    before = sorted([c for c in callbacks if getattr(c, "before_iteration", False)], key=lambda c: getattr(c, "order", 0))
    after = sorted([c for c in callbacks if not getattr(c, "before_iteration", False)],
                   key=lambda c: getattr(c, "order", 0))
    for i in range(num_boost_round):
        for c in before:
            c(cb.CallbackEnv(model=cvfolds, params=params, iteration=i, begin_iteration=0,
                             end_iteration=num_boost_round, evaluation_result_list=None))
        raw = []
        for b in cvfolds.boosters:
            b.update(fobj=fobj)
            raw.append(b.eval_valid(feval))
        res = _agg_cv_result(raw)
        for data_name, metric, mean, _, std in res:
            results[f"{data_name} {metric}-mean"].append(mean)
            results[f"{data_name} {metric}-stdv"].append(std)
        try:
            for c in after:
                c(cb.CallbackEnv(model=cvfolds, params=params, iteration=i, begin_iteration=0,
                                 end_iteration=num_boost_round, evaluation_result_list=res))
        except cb.EarlyStopException as e:
            cvfolds.best_iteration = e.best_iteration + 1
            for b in cvfolds.boosters:
                b.best_iteration = cvfolds.best_iteration
            for k in results:
                results[k] = results[k][:cvfolds.best_iteration]
            break
    out = dict(results)
    if return_cvbooster:
        out["cvbooster"] = cvfolds
    return out
