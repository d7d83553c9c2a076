"""Model families served by the framework.

* :mod:`.ranking` — the fork's LambdaRank family: the 18 ``lambdarank_target``
  gradients (NDCG, LambdaLoss, BNDCG, precision/ARP, RankNet, LambdaGap-S/X
  hybrids), a target-aware ranker estimator and helpers to pick ``k`` and the
  hybrid weight.
* :mod:`.presets` — the reference's benchmark configurations (Higgs-shape binary
  classification, MS-LTR-shape ranking, large regression with EFB + GOSS) as
  parameter dictionaries plus matching synthetic data builders.
"""
from .presets import PRESETS, preset, preset_data
from .ranking import LAMBDARANK_TARGETS, LambdaGapRanker, lambdarank_params

__all__ = ["LAMBDARANK_TARGETS", "LambdaGapRanker", "lambdarank_params", "PRESETS", "preset", "preset_data"]
