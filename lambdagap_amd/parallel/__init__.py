"""Multi-process training: RCCL communicator for GPU ranks, torch.distributed or TCP mesh for host
collectives, and collective train / estimator entry points for torchrun jobs."""
from .distributed import (DistContext, device_synchronize, env_context, free_device_comm, free_network,
                          get_unique_id, init_device_comm, init_socket_network, shard_range)
from .torch_network import free_torch_network, init_torch_network
from .trainer import (DistributedLGBMClassifier, DistributedLGBMRanker, DistributedLGBMRegressor, distributed_params,
                      setup_network, shard, train_distributed)

__all__ = ["DistContext", "env_context", "get_unique_id", "init_device_comm", "free_device_comm",
           "init_socket_network", "free_network", "device_synchronize", "shard_range", "init_torch_network",
           "free_torch_network", "setup_network", "distributed_params", "train_distributed", "shard",
           "DistributedLGBMRegressor", "DistributedLGBMClassifier", "DistributedLGBMRanker"]
