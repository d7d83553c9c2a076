"""Utilities: synthetic data generators, timing helpers."""
from .synthetic import make_higgs_like, make_ranking, make_regression

__all__ = ["make_higgs_like", "make_ranking", "make_regression"]
