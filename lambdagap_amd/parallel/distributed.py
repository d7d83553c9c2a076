"""Multi-GPU bootstrap: one process per MI355X, RCCL over xGMI.

The native library owns the RCCL communicator used for histogram
all-reduce; it is created from an ``ncclUniqueId`` that rank 0 generates and
``torch.distributed`` broadcasts (``torchrun`` provides RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR). Host-side scalar syncs (bin boundaries,
boost-from-average, metric sums) ride on the same communicator.

Reference counterpart: the socket network of src/network/ configured with
``machines=`` / ``num_machines`` (still available via :func:`init_socket_network`).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

from ..basic import _LIB, _check, _c_str


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device_comm: bool = False


def env_context() -> DistContext:
    return DistContext(rank=int(os.environ.get("RANK", 0)), world_size=int(os.environ.get("WORLD_SIZE", 1)),
                       local_rank=int(os.environ.get("LOCAL_RANK", 0)))


def get_unique_id() -> str:
    buf = ctypes.create_string_buffer(1024)
    out_len = ctypes.c_int64(0)
    _check(_LIB.LGBM_DeviceCommGetUniqueId(buf, ctypes.c_int64(1024), ctypes.byref(out_len)))
    return buf.value.decode("ascii")


def init_device_comm(ctx: Optional[DistContext] = None, backend: str = "gloo") -> DistContext:
    """Create the RCCL communicator of this rank (collective over all ranks).

    Uses ``torch.distributed`` only to move the 128-byte unique id; the
    process group is initialised with ``backend`` if it is not already.
    """
    ctx = ctx or env_context()
    if ctx.world_size <= 1:
        return ctx
    import torch.distributed as dist

    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=ctx.rank, world_size=ctx.world_size)
    obj = [get_unique_id() if ctx.rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    uid = obj[0]
    _check(_LIB.LGBM_DeviceCommInit(_c_str(uid), ctypes.c_int64(len(uid)), ctypes.c_int(ctx.world_size),
                                    ctypes.c_int(ctx.rank), ctypes.c_int(ctx.local_rank)))
    ctx.device_comm = True
    return ctx


def free_device_comm() -> None:
    _check(_LIB.LGBM_DeviceCommFree())


def init_socket_network(machines: str, local_listen_port: int = 12400, listen_time_out: int = 120,
                        num_machines: int = 1) -> None:
    """CPU socket mesh for the host parallel learners (reference LGBM_NetworkInit)."""
    _check(_LIB.LGBM_NetworkInit(_c_str(machines), ctypes.c_int(local_listen_port), ctypes.c_int(listen_time_out),
                                 ctypes.c_int(num_machines)))


def free_network() -> None:
    _check(_LIB.LGBM_NetworkFree())


def device_synchronize() -> None:
    _check(_LIB.LGBM_DeviceSynchronize())


def shard_range(n: int, rank: int, world_size: int) -> tuple:
    """Contiguous [start, stop) row range of `rank` when n rows are split evenly."""
    base, rem = divmod(n, world_size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)
