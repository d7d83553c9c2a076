"""Synthetic datasets shaped like the reference's benchmark data.

* :func:`make_higgs_like` - 28 float features like the HIGGS set (21 low-level
  kinematic columns: skewed transverse momenta, pseudo-rapidities, angles,
  b-tag levels; 7 high-level invariant masses near 1) with a non-linear,
  interaction-heavy signal/background label (AUC of a strong GBDT ~0.8-0.85).
* :func:`make_ranking` - grouped queries with graded relevance 0..4.
* :func:`make_regression` - wide sparse-ish regression data (EFB friendly).

Generation is chunked and seeded per chunk, so row ``i`` is identical no
matter how the rows are split across ranks (``start``/``stop``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

HIGGS_NUM_FEATURES = 28
_CHUNK = 1 << 18


def _higgs_chunk(rng: np.random.Generator, n: int) -> Tuple[np.ndarray, np.ndarray]:
    X = np.empty((n, HIGGS_NUM_FEATURES), dtype=np.float32)
    lat = rng.standard_normal((n, 6)).astype(np.float32)  # latent "physics" factors
    sig = rng.random(n) < 0.53
    s = sig.astype(np.float32)
    # lepton: pT, eta, phi
    X[:, 0] = rng.gamma(2.0, 0.45, n) * (1.0 + 0.25 * s) + 0.1 * np.abs(lat[:, 0])
    X[:, 1] = np.clip(rng.standard_normal(n) * (1.0 - 0.15 * s), -2.5, 2.5)
    X[:, 2] = rng.uniform(-np.pi, np.pi, n)
    # missing energy magnitude, phi
    X[:, 3] = rng.gamma(2.0, 0.5, n) * (1.0 + 0.2 * s * (lat[:, 1] > 0))
    X[:, 4] = rng.uniform(-np.pi, np.pi, n)
    # four jets: pT, eta, phi, b-tag
    for j in range(4):
        b = 5 + 4 * j
        X[:, b] = rng.gamma(2.2, 0.42, n) * (1.0 + 0.1 * s * (j < 2)) + 0.05 * np.abs(lat[:, 2 + (j % 4)])
        X[:, b + 1] = np.clip(rng.standard_normal(n), -2.5, 2.5)
        X[:, b + 2] = rng.uniform(-np.pi, np.pi, n)
        p_b = 0.25 + 0.25 * s * (j >= 2)
        tag = rng.random(n) < p_b
        X[:, b + 3] = np.where(tag, 2.1730, np.where(rng.random(n) < 0.5, 0.0, 1.0865)).astype(np.float32)
    # high-level invariant masses (peaked near 1, signal shifts/narrows some)
    widths = np.array([0.25, 0.2, 0.15, 0.3, 0.35, 0.3, 0.25], dtype=np.float32)
    shifts = np.array([0.0, 0.02, 0.0, 0.08, 0.12, 0.1, 0.06], dtype=np.float32)
    for k in range(7):
        w = widths[k] * (1.0 - 0.35 * s * (k >= 4))
        X[:, 21 + k] = np.exp(rng.standard_normal(n).astype(np.float32) * w + shifts[k] * s
                              + 0.05 * lat[:, k % 6])
    # label noise: interactions make the Bayes-optimal boundary non-additive
    flip = rng.random(n) < (0.06 + 0.08 * np.tanh(X[:, 3] - 1.0) ** 2)
    y = np.where(flip, ~sig, sig).astype(np.float32)
    return X, y


def make_higgs_like(n: int, seed: int = 0, start: int = 0, stop: Optional[int] = None
                    ) -> Tuple[np.ndarray, np.ndarray]:
    """Rows [start, stop) of an n-row Higgs-shaped binary dataset (float32 X, float32 y)."""
    stop = n if stop is None else min(stop, n)
    out_x = np.empty((max(stop - start, 0), HIGGS_NUM_FEATURES), dtype=np.float32)
    out_y = np.empty(max(stop - start, 0), dtype=np.float32)
    c0 = start // _CHUNK
    c1 = (stop + _CHUNK - 1) // _CHUNK
    for c in range(c0, c1):
        lo = c * _CHUNK
        hi = min(n, lo + _CHUNK)
        rng = np.random.default_rng([seed, c])
        X, y = _higgs_chunk(rng, hi - lo)
        a, b = max(lo, start), min(hi, stop)
        if a < b:
            out_x[a - start:b - start] = X[a - lo:b - lo]
            out_y[a - start:b - start] = y[a - lo:b - lo]
    return out_x, out_y


def make_ranking(num_queries: int, num_features: int = 300, docs_per_query: Tuple[int, int] = (5, 60),
                 seed: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Grouped ranking data: X [n, f] float32, relevance y in 0..4, group sizes."""
    rng = np.random.default_rng(seed)
    sizes = rng.integers(docs_per_query[0], docs_per_query[1] + 1, num_queries).astype(np.int32)
    n = int(sizes.sum())
    X = rng.standard_normal((n, num_features), dtype=np.float32)
    w = np.zeros(num_features, dtype=np.float32)
    k = min(num_features, 20)
    w[:k] = rng.standard_normal(k).astype(np.float32)
    q_shift = np.repeat(rng.standard_normal(num_queries).astype(np.float32), sizes)
    score = X[:, :k] @ w[:k] + 0.5 * np.sin(X[:, 0] * X[:, 1]) + 0.3 * q_shift + 0.5 * rng.standard_normal(n)
    qs = np.concatenate([[0], np.cumsum(sizes)])
    y = np.zeros(n, dtype=np.float32)
    for q in range(num_queries):
        s = score[qs[q]:qs[q + 1]]
        r = np.argsort(np.argsort(-s))
        frac = r / max(len(s) - 1, 1)
        y[qs[q]:qs[q + 1]] = np.select([frac < 0.05, frac < 0.15, frac < 0.35, frac < 0.6], [4, 3, 2, 1], 0)
    return X, y, sizes


def make_regression(n: int, num_features: int = 500, density: float = 0.1, seed: int = 0, function_seed: int = 0
                    ) -> Tuple[np.ndarray, np.ndarray]:
    """Wide regression data where most columns are mostly zero (exclusive-feature-bundling friendly).

    ``seed`` draws the rows; ``function_seed`` the target's coefficients, so a held-out set drawn
    with another ``seed`` follows the same function."""
    rng = np.random.default_rng(seed)
    X = np.zeros((n, num_features), dtype=np.float32)
    dense = min(20, num_features)
    X[:, :dense] = rng.standard_normal((n, dense), dtype=np.float32)
    for j in range(dense, num_features):
        mask = rng.random(n) < density
        X[mask, j] = rng.standard_normal(int(mask.sum())).astype(np.float32)
    w = np.random.default_rng([function_seed, num_features]).standard_normal(num_features).astype(np.float32)
    w /= np.sqrt(num_features)
    y = X @ w + np.sin(X[:, 0]) * X[:, 1] + 0.1 * rng.standard_normal(n).astype(np.float32)
    return X, y.astype(np.float32)
