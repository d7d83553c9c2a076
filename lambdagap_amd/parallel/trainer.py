"""Collective training entry points for one-process-per-device jobs (``torchrun``).

The MI355X-native counterpart of the reference's Dask integration
(python-package/lightgbm/dask.py: ``_train_part`` sets ``machines`` /
``num_machines`` / ``tree_learner`` per worker): every rank calls these with its
own row shard; ranks are wired together with RCCL (GPU, ``device_type=gpu``) or
``torch.distributed``/gloo (CPU), and every rank returns the same model.
"""
from __future__ import annotations

import atexit
from typing import Any, Dict, Optional

import numpy as np

from .. import basic
from ..engine import train as _train
from ..sklearn import LGBMClassifier, LGBMRanker, LGBMRegressor
from .distributed import DistContext, env_context, free_device_comm, init_device_comm
from .torch_network import free_torch_network, init_torch_network

_WIRED: Dict[str, Any] = {}


def setup_network(device_type: str = "cpu", tree_learner: str = "data", backend: str = "gloo") -> DistContext:
    """Wire this rank into the job once (idempotent).

    GPU + data-parallel: RCCL communicator (histograms all-reduced on device,
    host syncs over the same communicator). Otherwise: native host collectives
    over ``torch.distributed``.
    """
    ctx = env_context()
    if ctx.world_size <= 1 or _WIRED.get("ctx") is not None:
        return _WIRED.get("ctx", ctx)
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=ctx.rank, world_size=ctx.world_size)
        _WIRED["own_group"] = True
    if device_type in ("gpu", "cuda", "hip", "rocm"):
        ctx = init_device_comm(ctx)
    else:
        init_torch_network()
    _WIRED["ctx"] = ctx
    atexit.register(teardown_network)
    return ctx


def teardown_network() -> None:
    """Undo :func:`setup_network` (also run at interpreter exit): release the native
    collectives, then the process group this module created. Without it the gloo
    process group is torn down by static destructors while its threads still run, which
    can abort the process after training has finished."""
    ctx = _WIRED.pop("ctx", None)
    if ctx is None:
        return
    try:
        if getattr(ctx, "device_comm", False):
            free_device_comm()
        else:
            free_torch_network()
    finally:
        if _WIRED.pop("own_group", False):
            import torch.distributed as dist

            if dist.is_initialized():
                dist.barrier()
                dist.destroy_process_group()


def distributed_params(params: Dict[str, Any], tree_learner: str = "data") -> Dict[str, Any]:
    ctx = env_context()
    p = dict(params)
    if ctx.world_size > 1:
        p.setdefault("tree_learner", tree_learner)
        p["num_machines"] = ctx.world_size
        p.setdefault("pre_partition", True)
    return p


def train_distributed(params: Dict[str, Any], X: Any, y: Any, num_boost_round: int = 100,
                      weight: Optional[Any] = None, group: Optional[Any] = None, init_score: Optional[Any] = None,
                      tree_learner: str = "data", **train_kwargs: Any) -> basic.Booster:
    """Train on this rank's shard (collective: every rank calls it). Returns the shared model."""
    setup_network(str(params.get("device_type", params.get("device", "cpu"))), tree_learner)
    p = distributed_params(params, tree_learner)
    ds = basic.Dataset(X, y, weight=weight, group=group, init_score=init_score, params=p)
    return _train(p, ds, num_boost_round, **train_kwargs)


class _DistributedMixin:
    """fit() on this rank's shard inside a torchrun job."""

    def __init__(self, tree_learner: str = "data", **kwargs: Any) -> None:
        super().__init__(tree_learner=tree_learner, **kwargs)  # type: ignore[call-arg]

    def fit(self, X: Any, y: Any, **kwargs: Any):  # type: ignore[override]
        params = self.get_params()  # type: ignore[attr-defined]
        setup_network(str(params.get("device_type", params.get("device", "cpu"))),
                      str(params.get("tree_learner", "data")))
        ctx = env_context()
        if ctx.world_size > 1:
            self.set_params(num_machines=ctx.world_size, pre_partition=True)  # type: ignore[attr-defined]
        return super().fit(X, y, **kwargs)  # type: ignore[misc]


class DistributedLGBMRegressor(_DistributedMixin, LGBMRegressor):
    pass


class DistributedLGBMClassifier(_DistributedMixin, LGBMClassifier):
    pass


class DistributedLGBMRanker(_DistributedMixin, LGBMRanker):
    pass


def shard(X: np.ndarray, rank: Optional[int] = None, world: Optional[int] = None) -> np.ndarray:
    """Strided row shard of an array for this rank (every world-th row)."""
    ctx = env_context()
    r = ctx.rank if rank is None else rank
    w = ctx.world_size if world is None else world
    return X[r::w]
