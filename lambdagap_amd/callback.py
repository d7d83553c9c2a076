"""Training callbacks (reference: python-package/lightgbm/callback.py).

A callback is any callable taking a :class:`CallbackEnv`; attributes
``order`` (int) and ``before_iteration`` (bool) control scheduling.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

from .basic import _log_info

__all__ = ["EarlyStopException", "CallbackEnv", "early_stopping", "log_evaluation", "record_evaluation",
           "reset_parameter"]

EvalTuple = Tuple[str, str, float, bool]


class EarlyStopException(Exception):
    """Raised by a callback to stop training; carries the best iteration and its scores."""

    def __init__(self, best_iteration: int, best_score: List[EvalTuple]):
        super().__init__()
        self.best_iteration = best_iteration
        self.best_score = best_score


@dataclass
class CallbackEnv:
    model: Any
    params: Dict[str, Any]
    iteration: int
    begin_iteration: int
    end_iteration: int
    evaluation_result_list: Optional[List[Any]]


def _format_eval(value: Any, show_stdv: bool) -> str:
    if len(value) == 4:
        return f"{value[0]}'s {value[1]}: {value[2]:g}"
    if len(value) == 5:
        if show_stdv:
            return f"{value[0]}'s {value[1]}: {value[2]:g} + {value[4]:g}"
        return f"{value[0]}'s {value[1]}: {value[2]:g}"
    raise ValueError("Wrong metric value")


class _LogEvaluation:
    def __init__(self, period: int, show_stdv: bool):
        self.order = 10
        self.before_iteration = False
        self.period = period
        self.show_stdv = show_stdv

    def __call__(self, env: CallbackEnv) -> None:
        if self.period > 0 and env.evaluation_result_list and (env.iteration + 1) % self.period == 0:
            msg = "\t".join(_format_eval(x, self.show_stdv) for x in env.evaluation_result_list)
            _log_info(f"[{env.iteration + 1}]\t{msg}")


def log_evaluation(period: int = 1, show_stdv: bool = True) -> Callable:
    """Print evaluation results every ``period`` iterations."""
    return _LogEvaluation(period, show_stdv)


class _RecordEvaluation:
    def __init__(self, eval_result: Dict[str, Dict[str, List[Any]]]):
        if not isinstance(eval_result, dict):
            raise TypeError("eval_result should be a dictionary")
        self.order = 20
        self.before_iteration = False
        self.eval_result = eval_result

    def _init(self, env: CallbackEnv) -> None:
        self.eval_result.clear()
        for item in env.evaluation_result_list or []:
            data_name, metric = item[0], item[1]
            self.eval_result.setdefault(data_name, OrderedDict())
            if len(item) == 4:
                self.eval_result[data_name].setdefault(metric, [])
            else:
                self.eval_result[data_name].setdefault(f"{metric}-mean", [])
                self.eval_result[data_name].setdefault(f"{metric}-stdv", [])

    def __call__(self, env: CallbackEnv) -> None:
        if env.iteration == env.begin_iteration:
            self._init(env)
        for item in env.evaluation_result_list or []:
            data_name, metric, value = item[0], item[1], item[2]
            if len(item) == 4:
                self.eval_result[data_name][metric].append(value)
            else:
                self.eval_result[data_name][f"{metric}-mean"].append(value)
                self.eval_result[data_name][f"{metric}-stdv"].append(item[4])


def record_evaluation(eval_result: Dict[str, Dict[str, List[Any]]]) -> Callable:
    """Store evaluation history into ``eval_result`` (data name -> metric -> values)."""
    return _RecordEvaluation(eval_result)


class _ResetParameter:
    def __init__(self, **kwargs: Union[list, Callable]):
        self.order = 10
        self.before_iteration = True
        self.kwargs = kwargs

    def __call__(self, env: CallbackEnv) -> None:
        new = {}
        for key, value in self.kwargs.items():
            if isinstance(value, list):
                if len(value) != env.end_iteration - env.begin_iteration:
                    raise ValueError(f"Length of list {key!r} has to be equal to 'num_boost_round'.")
                v = value[env.iteration - env.begin_iteration]
            elif callable(value):
                v = value(env.iteration - env.begin_iteration)
            else:
                raise ValueError("Only list and callable values are supported as a mapping from boosting round index "
                                 "to new parameter value.")
            if env.params.get(key) != v:
                new[key] = v
        if new:
            if hasattr(env.model, "reset_parameter"):
                env.model.reset_parameter(new)
            else:  # CVBooster
                for b in env.model.boosters:
                    b.reset_parameter(new)
            env.params.update(new)


def reset_parameter(**kwargs: Union[list, Callable]) -> Callable:
    """Reset parameters (e.g. learning_rate) before each iteration from a list or a function of the round."""
    return _ResetParameter(**kwargs)


class _EarlyStopping:
    def __init__(self, stopping_rounds: int, first_metric_only: bool, verbose: bool,
                 min_delta: Union[float, List[float]]):
        # a non-positive count leaves the callback disabled; a non-integer is an error
        # (reference callback.py _should_enable_early_stopping)
        if not isinstance(stopping_rounds, int) or isinstance(stopping_rounds, bool):
            raise TypeError(f"early_stopping_round should be an integer. Got '{type(stopping_rounds).__name__}'")
        self.order = 30
        self.before_iteration = False
        self.stopping_rounds = stopping_rounds
        self.first_metric_only = first_metric_only
        self.verbose = verbose
        self.min_delta = min_delta
        self.enabled = stopping_rounds > 0
        self._reset()

    def _reset(self) -> None:
        self.best_score: List[float] = []
        self.best_iter: List[int] = []
        self.best_score_list: List[Any] = []
        self.cmp_op: List[Callable[[float, float], bool]] = []
        self.first_metric = ""

    def _init(self, env: CallbackEnv) -> None:
        if not env.evaluation_result_list:
            raise ValueError("For early stopping, at least one dataset and eval metric is required for evaluation")
        from .basic import _log_warning

        if any(env.params.get(a, "") == "dart" for a in ("boosting", "boosting_type", "boost")):
            self.enabled = False
            _log_warning("Early stopping is not available in dart mode")
            return
        first_name = env.evaluation_result_list[0][0]
        if len(env.evaluation_result_list) == 1 and self._is_train_set(first_name, env) and \
                not isinstance(env.model, dict) and hasattr(env.model, "_train_data_name"):
            self.enabled = False
            _log_warning("Only training set found, disabling early stopping.")
            return
        self._reset()
        self.first_metric = env.evaluation_result_list[0][1].split(" ")[-1]
        n = len(env.evaluation_result_list)
        if isinstance(self.min_delta, list):
            if not self.min_delta:
                deltas = [0.0] * n
            elif len(self.min_delta) == 1:
                deltas = self.min_delta * n
            else:
                nm = len({m[1] for m in env.evaluation_result_list})
                if len(self.min_delta) != nm:
                    raise ValueError("Must provide a single value for min_delta or as many as metrics.")
                deltas = self.min_delta * (n // nm)
        else:
            deltas = [float(self.min_delta)] * n
        for item, delta in zip(env.evaluation_result_list, deltas):
            if delta < 0:
                raise ValueError("Early stopping min_delta must be non-negative.")
            self.best_iter.append(0)
            if item[3]:
                self.best_score.append(float("-inf"))
                self.cmp_op.append(lambda cur, best, d=delta: cur > best + d)
            else:
                self.best_score.append(float("inf"))
                self.cmp_op.append(lambda cur, best, d=delta: cur < best - d)
            self.best_score_list.append(None)
        if self.verbose:
            _log_info(f"Training until validation scores don't improve for {self.stopping_rounds} rounds")

    def _is_train_set(self, data_name: str, env: CallbackEnv) -> bool:
        model = env.model
        if hasattr(model, "_train_data_name"):
            return data_name == model._train_data_name
        return data_name == "train"

    def __call__(self, env: CallbackEnv) -> None:
        if not self.enabled:
            return
        if env.iteration == env.begin_iteration:
            self._init(env)
        if not self.enabled:
            return
        res = env.evaluation_result_list or []
        for i, item in enumerate(res):
            score = item[2]
            if self.best_score_list[i] is None or self.cmp_op[i](score, self.best_score[i]):
                self.best_score[i] = score
                self.best_iter[i] = env.iteration
                self.best_score_list[i] = res
            if self.first_metric_only and self.first_metric != item[1].split(" ")[-1]:
                continue
            if self._is_train_set(item[0], env):
                continue
            if env.iteration - self.best_iter[i] >= self.stopping_rounds:
                if self.verbose:
                    msg = "\t".join(_format_eval(x, True) for x in self.best_score_list[i])
                    _log_info(f"Early stopping, best iteration is:\n[{self.best_iter[i] + 1}]\t{msg}")
                raise EarlyStopException(self.best_iter[i], self.best_score_list[i])
            if env.iteration == env.end_iteration - 1:
                if self.verbose:
                    msg = "\t".join(_format_eval(x, True) for x in self.best_score_list[i])
                    _log_info(f"Did not meet early stopping. Best iteration is:\n[{self.best_iter[i] + 1}]\t{msg}")
                raise EarlyStopException(self.best_iter[i], self.best_score_list[i])


def early_stopping(stopping_rounds: int, first_metric_only: bool = False, verbose: bool = True,
                   min_delta: Union[float, List[float]] = 0.0) -> Callable:
    """Stop when no validation metric improved for ``stopping_rounds`` rounds."""
    return _EarlyStopping(stopping_rounds, first_metric_only, verbose, min_delta)
