"""LambdaRank family with the fork's ``lambdarank_target`` variants.

Reference: include/LightGBM/config.h:989-1013 (``lambdarank_target``,
``lambdagap_weight``) and src/objective/rank_objective.hpp:253-524 (per-query
gradients). The gradients themselves are computed natively (host C++ and the
HIP ``k_lambdarank`` kernel); this module only names the targets and builds
parameter sets / estimators around them.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

from ..sklearn import LGBMRanker

# target -> (family, short description)
LAMBDARANK_TARGETS: Dict[str, tuple] = {
    "ndcg": ("ndcg", "classic LambdaRank: |delta NDCG| weighted RankNet pairs"),
    "lambdaloss-ndcg": ("ndcg", "LambdaLoss NDCG-Loss2 bound"),
    "lambdaloss-ndcg-plus-plus": ("ndcg", "LambdaLoss NDCG-Loss2++ (Loss2 + mu * LambdaRank)"),
    "bndcg": ("bndcg", "binary-gain NDCG"),
    "lambdaloss-bndcg": ("bndcg", "LambdaLoss bound on binary NDCG"),
    "lambdaloss-bndcg-plus-plus": ("bndcg", "LambdaLoss++ bound on binary NDCG"),
    "precision": ("precision", "precision@k gradients"),
    "arpk": ("arp", "average relevance position at k"),
    "lambdaloss-arp1": ("arp", "LambdaLoss ARP-Loss1"),
    "lambdaloss-arp2": ("arp", "LambdaLoss ARP-Loss2"),
    "ranknet": ("ranknet", "plain RankNet (unweighted pairs)"),
    "bin-ranknet": ("ranknet", "RankNet on binarised relevance"),
    "lambdagap-s": ("lambdagap", "LambdaGap-S: gap-scaled pair weights"),
    "lambdagap-x": ("lambdagap", "LambdaGap-X: gap-crossing pair weights"),
    "lambdagap-s-plus": ("lambdagap", "LambdaGap-S+ hybrid with NDCG (lambdagap_weight)"),
    "lambdagap-x-plus": ("lambdagap", "LambdaGap-X+ hybrid with NDCG (lambdagap_weight)"),
    "lambdagap-s-plus-plus": ("lambdagap", "LambdaGap-S++ hybrid (lambdagap_weight)"),
    "lambdagap-x-plus-plus": ("lambdagap", "LambdaGap-X++ hybrid (lambdagap_weight)"),
}


def lambdarank_params(target: str = "ndcg", k: int = 30, lambdagap_weight: float = 1.0,
                      eval_at: Optional[list] = None, **extra: Any) -> Dict[str, Any]:
    """Parameter dict for a LambdaRank run with a given target.

    ``k`` is ``lambdarank_truncation_level``; the evaluation metric follows the
    target family (precision@k for ``precision``, NDCG otherwise).
    """
    if target not in LAMBDARANK_TARGETS:
        raise ValueError(f"Unknown lambdarank_target {target!r}; choose from {sorted(LAMBDARANK_TARGETS)}")
    family = LAMBDARANK_TARGETS[target][0]
    params: Dict[str, Any] = {
        "objective": "lambdarank",
        "lambdarank_target": target,
        "lambdarank_truncation_level": k,
        "lambdagap_weight": lambdagap_weight,
        "metric": "precision" if family == "precision" else "ndcg",
        "eval_at": eval_at or [1, 5, 10],
    }
    params.update(extra)
    return params


class LambdaGapRanker(LGBMRanker):
    """:class:`~lambdagap_amd.sklearn.LGBMRanker` with the fork's target and hybrid weight as
    constructor arguments (so they take part in ``get_params`` / ``clone`` / grid search)."""

    def __init__(self, lambdarank_target: str = "ndcg", lambdagap_weight: float = 1.0,
                 lambdarank_truncation_level: int = 30, **kwargs: Any) -> None:
        if lambdarank_target not in LAMBDARANK_TARGETS:
            raise ValueError(f"Unknown lambdarank_target {lambdarank_target!r}")
        super().__init__(lambdarank_target=lambdarank_target, lambdagap_weight=lambdagap_weight,
                         lambdarank_truncation_level=lambdarank_truncation_level, **kwargs)
