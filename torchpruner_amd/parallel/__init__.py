"""Distributed runtime: RCCL-over-xGMI data parallelism for attribution and finetuning."""
from .comm import Communicator, LoopbackCommunicator, LoopbackHub, run_loopback
from .dist import (
    DistContext,
    ShardedBatches,
    all_reduce_sum_,
    barrier,
    broadcast_object,
    broadcast_tensor_,
    gather_ordered_rows,
    get_rank,
    get_world_size,
    init_distributed,
    is_dist,
    split_range,
)

__all__ = [
    "Communicator", "LoopbackCommunicator", "LoopbackHub", "run_loopback",
    "DistContext", "ShardedBatches", "all_reduce_sum_", "barrier", "broadcast_object", "broadcast_tensor_",
    "gather_ordered_rows", "get_rank", "get_world_size", "init_distributed", "is_dist", "split_range",
]
from .ddp import PrunableDDP, params_in_sync, prune_and_rewrap  # noqa: E402

__all__ += ["PrunableDDP", "params_in_sync", "prune_and_rewrap"]
