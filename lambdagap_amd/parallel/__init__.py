"""Distributed training: RCCL communicator bootstrap and socket network helpers."""
from .distributed import (DistContext, device_synchronize, env_context, free_device_comm, free_network,
                          init_device_comm, init_socket_network, shard_range)

__all__ = ["DistContext", "env_context", "init_device_comm", "free_device_comm", "init_socket_network",
           "free_network", "device_synchronize", "shard_range"]
