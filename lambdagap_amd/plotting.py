"""Plotting helpers (reference: python-package/lightgbm/plotting.py).

matplotlib draws importance / split histograms / metric curves / trees;
``create_tree_digraph`` needs the optional ``graphviz`` package.
"""
from __future__ import annotations

import math

from copy import deepcopy
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np

from .basic import Booster, LightGBMError

__all__ = ["plot_importance", "plot_split_value_histogram", "plot_metric", "plot_tree", "create_tree_digraph"]


def _booster_of(booster: Any) -> Booster:
    if isinstance(booster, Booster):
        return booster
    if hasattr(booster, "booster_"):
        return booster.booster_
    raise TypeError("booster must be Booster or LGBMModel.")


def _plt():
    try:
        import matplotlib.pyplot as plt
    except ImportError as e:  # pragma: no cover
        raise ImportError("You must install matplotlib to plot.") from e
    return plt


def _axes(ax, figsize, dpi):
    plt = _plt()
    if ax is None:
        _, ax = plt.subplots(1, 1, figsize=figsize, dpi=dpi)
    return ax


def plot_importance(booster: Any, ax=None, height: float = 0.2, xlim=None, ylim=None,
                    title: Optional[str] = "Feature importance", xlabel: Optional[str] = "Feature importance",
                    ylabel: Optional[str] = "Features", importance_type: str = "auto",
                    max_num_features: Optional[int] = None, ignore_zero: bool = True, figsize=None, dpi=None,
                    grid: bool = True, precision: Optional[int] = 3, **kwargs: Any):
    """Horizontal bar chart of feature importances."""
    if importance_type == "auto":
        importance_type = getattr(booster, "importance_type", "split")
    b = _booster_of(booster)
    importance = b.feature_importance(importance_type=importance_type)
    names = b.feature_name()
    if not len(importance):
        raise ValueError("Booster's feature_importance is empty.")
    tuples = sorted(zip(names, importance), key=lambda x: x[1])
    if ignore_zero:
        tuples = [t for t in tuples if t[1] > 0]
    if max_num_features is not None and max_num_features > 0:
        tuples = tuples[-max_num_features:]
    labels, values = zip(*tuples) if tuples else ((), ())
    ax = _axes(ax, figsize, dpi)
    ylocs = np.arange(len(values))
    ax.barh(ylocs, values, align="center", height=height, **kwargs)
    for x, y in zip(values, ylocs):
        txt = f"{x:.{precision}f}" if (precision is not None and importance_type == "gain") else str(x)
        ax.text(x + 1, y, txt, va="center")
    ax.set_yticks(ylocs)
    ax.set_yticklabels(labels)
    if xlim is None and values:
        xlim = (0, max(values) * 1.1)
    if xlim is not None:
        ax.set_xlim(xlim)
    if ylim is None:
        ylim = (-1, len(values))
    ax.set_ylim(ylim)
    if title is not None:
        ax.set_title(title)
    if xlabel is not None:
        ax.set_xlabel(xlabel.replace("@importance_type@", importance_type))
    if ylabel is not None:
        ax.set_ylabel(ylabel)
    ax.grid(grid)
    return ax


def plot_split_value_histogram(booster: Any, feature: Union[int, str], bins=None, ax=None, width_coef: float = 0.8,
                               xlim=None, ylim=None, title: Optional[str] = "Split value histogram for feature with @index/name@ @feature@",
                               xlabel: Optional[str] = "Feature split value", ylabel: Optional[str] = "Count",
                               figsize=None, dpi=None, grid: bool = True, **kwargs: Any):
    """Histogram of the thresholds a feature was split at."""
    b = _booster_of(booster)
    hist, split_bins = b.get_split_value_histogram(feature=feature, bins=bins, xgboost_style=False)
    if np.count_nonzero(hist) == 0:
        raise ValueError(f"Cannot plot split value histogram, because feature {feature} was not used in splitting")
    width = width_coef * (split_bins[1] - split_bins[0])
    centred = (split_bins[:-1] + split_bins[1:]) / 2
    ax = _axes(ax, figsize, dpi)
    ax.bar(centred, hist, align="center", width=width, **kwargs)
    if xlim is None:
        r = split_bins[-1] - split_bins[0]
        xlim = (split_bins[0] - r * 0.2, split_bins[-1] + r * 0.2)
    ax.set_xlim(xlim)
    ax.yaxis.set_major_locator(_plt().MaxNLocator(integer=True))
    if ylim is None:
        ylim = (0, max(hist) * 1.1)
    ax.set_ylim(ylim)
    if title is not None:
        title = title.replace("@feature@", str(feature)).replace(
            "@index/name@", "name" if isinstance(feature, str) else "index")
        ax.set_title(title)
    if xlabel is not None:
        ax.set_xlabel(xlabel)
    if ylabel is not None:
        ax.set_ylabel(ylabel)
    ax.grid(grid)
    return ax


def plot_metric(booster: Union[Dict, Any], metric: Optional[str] = None, dataset_names: Optional[List[str]] = None,
                ax=None, xlim=None, ylim=None, title: Optional[str] = "Metric during training",
                xlabel: Optional[str] = "Iterations", ylabel: Optional[str] = "@metric@", figsize=None, dpi=None,
                grid: bool = True):
    """Plot one recorded metric over iterations (from record_evaluation or LGBMModel.evals_result_)."""
    if isinstance(booster, dict):
        eval_results = deepcopy(booster)
    elif hasattr(booster, "evals_result_"):
        eval_results = deepcopy(booster.evals_result_)
    elif isinstance(booster, Booster):
        raise TypeError("booster must be dict or LGBMModel. To use plot_metric with Booster type, first record "
                        "the metrics using record_evaluation callback then pass that to plot_metric as argument "
                        "`booster`")
    else:
        raise TypeError("booster must be dict or LGBMModel.")
    if not eval_results:
        raise ValueError("eval results cannot be empty.")
    ax = _axes(ax, figsize, dpi)
    names = dataset_names or list(eval_results.keys())
    first = eval_results[names[0]]
    if metric is None:
        metric = next(iter(first.keys()))
    num_iter = len(first[metric])
    max_r, min_r = -np.inf, np.inf
    for name in names:
        r = eval_results[name][metric]
        max_r, min_r = max(max(r), max_r), min(min(r), min_r)
        ax.plot(range(len(r)), r, label=name)
    ax.legend(loc="best")
    if xlim is None:
        xlim = (0, num_iter)
    ax.set_xlim(xlim)
    if ylim is None:
        rng = max_r - min_r
        ylim = (min_r - rng * 0.2, max_r + rng * 0.2)
    ax.set_ylim(ylim)
    if title is not None:
        ax.set_title(title)
    if xlabel is not None:
        ax.set_xlabel(xlabel)
    if ylabel is not None:
        ax.set_ylabel(ylabel.replace("@metric@", metric))
    ax.grid(grid)
    return ax


def _tree_layout(node: Dict[str, Any], depth: int = 0, pos: Optional[Dict] = None, counter: Optional[List[int]] = None):
    """In-order x positions, depth as y."""
    if pos is None:
        pos, counter = {}, [0]
    if "split_index" in node:
        _tree_layout(node["left_child"], depth + 1, pos, counter)
        pos[id(node)] = (counter[0], -depth)
        counter[0] += 1
        _tree_layout(node["right_child"], depth + 1, pos, counter)
    else:
        pos[id(node)] = (counter[0], -depth)
        counter[0] += 1
    return pos


def plot_tree(booster: Any, ax=None, tree_index: int = 0, figsize=None, dpi=None, show_info=None,
              precision: Optional[int] = 3, orientation: str = "horizontal", example_case=None, **kwargs: Any):
    """Draw one tree with matplotlib (node boxes and edges; no graphviz needed)."""
    b = _booster_of(booster)
    model = b.dump_model()
    trees = model["tree_info"]
    if tree_index >= len(trees):
        raise IndexError("tree_index is out of range.")
    names = model.get("feature_names", [])
    root = trees[tree_index]["tree_structure"]
    pos = _tree_layout(root)
    ax = _axes(ax, figsize, dpi)
    show_info = show_info or []

    def label(node):
        if "split_index" in node:
            f = node["split_feature"]
            fname = names[f] if f < len(names) else f"Column_{f}"
            thr = node["threshold"]
            op = "==" if node.get("decision_type") == "==" else "<="
            thr_s = f"{thr:.{precision}f}" if isinstance(thr, float) and precision is not None else str(thr)
            s = f"{fname} {op} {thr_s}"
            for info in show_info:
                if info in node:
                    s += f"\n{info}: {node[info]}"
            return s
        v = node["leaf_value"]
        s = f"leaf {node.get('leaf_index', 0)}: {v:.{precision}f}" if precision is not None else f"leaf: {v}"
        for info in show_info:
            if info in node:
                s += f"\n{info}: {node[info]}"
        return s

    def draw(node):
        x, y = pos[id(node)]
        if orientation == "vertical":
            x, y = -y, -x
        ax.text(x, y, label(node), ha="center", va="center", fontsize=8,
                bbox=dict(boxstyle="round", fc="white", ec="black"))
        if "split_index" in node:
            for child in (node["left_child"], node["right_child"]):
                cx, cy = pos[id(child)]
                if orientation == "vertical":
                    cx, cy = -cy, -cx
                ax.plot([x, cx], [y, cy], "k-", lw=0.8, zorder=0)
                draw(child)

    draw(root)
    ax.set_axis_off()
    return ax


_ZERO_THRESHOLD = 1e-35


def _determine_direction_for_numeric_split(fval: float, threshold: float, missing_type_str: str,
                                           default_left: bool) -> str:
    """Which child a value takes at a numerical split: the tree's decision rule (NaN is
    zero unless the split tracks NaN; the tracked missing value follows default_left)."""
    if math.isnan(fval) and missing_type_str != "NaN":
        fval = 0.0
    if (missing_type_str == "Zero" and abs(fval) <= _ZERO_THRESHOLD) or (
            missing_type_str == "NaN" and math.isnan(fval)):
        return "left" if default_left else "right"
    return "left" if fval <= threshold else "right"


def _determine_direction_for_categorical_split(fval: float, thresholds: str) -> str:
    """Categories listed in the split ("a||b||c") go left; NaN and negatives go right."""
    if math.isnan(fval) or int(fval) < 0:
        return "right"
    return "left" if int(fval) in {int(t) for t in str(thresholds).split("||")} else "right"


def create_tree_digraph(booster: Any, tree_index: int = 0, show_info=None, precision: Optional[int] = 3,
                        orientation: str = "horizontal", example_case=None, max_category_values: int = 10,
                        **kwargs: Any):
    """graphviz.Digraph of one tree (requires the optional graphviz package), reference
    plotting.py create_tree_digraph: ``show_info`` adds split_gain / internal_value /
    internal_count / internal_weight / leaf_count / leaf_weight / data_percentage, an
    ``example_case`` row is traced in blue, categorical splits list at most
    ``max_category_values`` categories."""
    b = _booster_of(booster)
    model = b.dump_model()
    trees = model["tree_info"]
    if tree_index >= len(trees):
        raise IndexError("tree_index is out of range.")
    names = model.get("feature_names", [])
    monotone = model.get("monotone_constraints") or []
    show_info = list(show_info or [])
    if example_case is not None:
        try:
            import pandas as pd
        except ImportError:  # pragma: no cover
            pd = None
        is_df = pd is not None and isinstance(example_case, pd.DataFrame)
        if not (isinstance(example_case, np.ndarray) or is_df) or example_case.ndim != 2:
            raise ValueError("example_case must be a numpy array or a pandas DataFrame")
        if example_case.shape[0] != 1:
            raise ValueError("example_case must have a single row.")
        example_case = np.asarray(example_case.to_numpy(dtype=np.float64) if is_df else example_case,
                                  dtype=np.float64)[0]
    try:
        from graphviz import Digraph
    except ImportError as e:
        raise ImportError("You must install graphviz and restart your session to plot tree.") from e
    total_count = trees[tree_index]["tree_structure"].get("internal_count", 0) or 1
    graph = Digraph(**kwargs)
    graph.attr("graph", nodesep="0.05", ranksep="0.3", rankdir="LR" if orientation == "horizontal" else "TB")

    def fmt(v):
        return f"{v:.{precision}f}" if precision is not None and isinstance(v, float) else str(v)

    def add(node, parent=None, decision=None, highlight=False):
        if "split_index" in node:
            name = f"split{node['split_index']}"
            f = node["split_feature"]
            fname = names[f] if f < len(names) else f"feature_{f}"
            if node["decision_type"] == "<=":
                lte = "&#8804;"
                label = f"<B>{fname}</B> {lte} {fmt(node['threshold'])}"
                direction = None
                if example_case is not None and highlight:
                    direction = _determine_direction_for_numeric_split(example_case[f], node["threshold"],
                                                                       node["missing_type"], node["default_left"])
            else:
                cats = str(node["threshold"]).split("||")
                shown = "||".join(cats[:max_category_values]) + ("||...||" + cats[-1]
                                                                  if len(cats) > max_category_values else "")
                label = f"<B>{fname}</B> in {shown}"
                direction = None
                if example_case is not None and highlight:
                    direction = _determine_direction_for_categorical_split(example_case[f], node["threshold"])
            if f < len(monotone) and monotone[f] != 0:
                label += " (increasing)" if monotone[f] > 0 else " (decreasing)"
            for info in ("split_gain", "internal_value", "internal_weight", "internal_count"):
                if info in show_info and info in node:
                    label += f"<br/>{info.split('_')[-1]}: {fmt(node[info])}"
            if "data_percentage" in show_info:
                label += f"<br/>{node.get('internal_count', 0) / total_count:.2%} of data"
            color = "blue" if highlight and example_case is not None else "black"
            graph.node(name, label=f"<{label}>", shape="rectangle", color=color)
            add(node["left_child"], name, "yes", highlight and direction == "left")
            add(node["right_child"], name, "no", highlight and direction == "right")
        else:
            name = f"leaf{node.get('leaf_index', 0)}"
            label = f"leaf {node.get('leaf_index', 0)}: <B>{fmt(node['leaf_value'])}</B>"
            for info in ("leaf_weight", "leaf_count"):
                if info in show_info and info in node:
                    label += f"<br/>{info.split('_')[-1]}: {fmt(node[info])}"
            if "data_percentage" in show_info:
                label += f"<br/>{node.get('leaf_count', 0) / total_count:.2%} of data"
            color = "blue" if highlight and example_case is not None else "black"
            graph.node(name, label=f"<{label}>", color=color)
        if parent is not None:
            graph.edge(parent, name, decision, color="blue" if highlight and example_case is not None else "black")

    add(trees[tree_index]["tree_structure"], highlight=True)
    return graph
