"""Host collectives of the native library over a ``torch.distributed`` process group.

The native ``Network`` layer (include/lgap/network.h) accepts external transport
functions (reference ``LGBM_NetworkInitWithFunctions``, src/network/network.cpp:
30-75). Here the allgather is a ctypes callback around ``dist.all_gather`` on
CPU tensors (gloo); reduce-scatter is derived natively from it. CPU ranks under
``torchrun`` can then train data/feature/voting-parallel with no ``machines``
list or listen ports; GPU ranks use the RCCL communicator instead
(:func:`~lambdagap_amd.parallel.distributed.init_device_comm`).
"""
from __future__ import annotations

import ctypes
import os
import sys
import traceback
from typing import Any, Optional

from ..basic import _LIB, _check

_AllgatherFn = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_void_p, ctypes.c_int32)
_STATE: dict = {}


def _allgather(inp, in_size, block_start, block_len, num_block, out, out_size):  # pragma: no cover - via native
    try:
        import torch
        import torch.distributed as dist

        lens = [int(block_len[i]) for i in range(num_block)]
        width = max(1, max(lens))
        buf = torch.zeros(width, dtype=torch.uint8)
        if in_size > 0:
            src = (ctypes.c_uint8 * in_size).from_address(inp)
            buf[:in_size] = torch.frombuffer(src, dtype=torch.uint8)
        parts = [torch.empty(width, dtype=torch.uint8) for _ in range(num_block)]
        dist.all_gather(parts, buf, group=_STATE.get("group"))
        for i in range(num_block):
            if lens[i] > 0:
                ctypes.memmove(out + int(block_start[i]), parts[i].numpy().ctypes.data, lens[i])
    except BaseException:  # a failed collective must not return garbage to the native caller
        traceback.print_exc()
        sys.stderr.flush()
        os._exit(70)


def init_torch_network(group: Optional[Any] = None) -> int:
    """Route the native host collectives through ``torch.distributed`` (collective call).

    Returns the world size. A no-op for a single process.
    """
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialized (call dist.init_process_group first)")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world <= 1:
        return world
    _STATE["group"] = group
    _STATE["cb"] = _AllgatherFn(_allgather)  # keep the trampoline alive
    _check(_LIB.LGBM_NetworkInitWithFunctions(ctypes.c_int(world), ctypes.c_int(rank), None,
                                              ctypes.cast(_STATE["cb"], ctypes.c_void_p)))
    return world


def free_torch_network() -> None:
    _check(_LIB.LGBM_NetworkFree())
    _STATE.clear()
