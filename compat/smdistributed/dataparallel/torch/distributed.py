"""SMDDP v1 ``smdistributed.dataparallel.torch.distributed`` API over torch.distributed + the
smddp backend (init_process_group, get_rank, get_local_rank, get_world_size, collectives)."""
import os

import torch.distributed as _dist

from mi355x_dp.parallel.smddp import register as _register

_register()
ReduceOp = _dist.ReduceOp
reduce_op = _dist.ReduceOp


def init_process_group(backend="smddp", *args, **kwargs):
    if not _dist.is_initialized():
        _dist.init_process_group(backend=backend, *args, **kwargs)


def is_available():
    return True


def is_initialized():
    return _dist.is_initialized()


def get_rank(group=None):
    return _dist.get_rank(group)


def get_world_size(group=None):
    return _dist.get_world_size(group)


def get_local_rank():
    return int(os.environ.get("LOCAL_RANK", "0"))


def get_local_size():
    return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))


all_reduce = _dist.all_reduce
broadcast = _dist.broadcast
all_gather = _dist.all_gather
reduce_scatter = _dist.reduce_scatter
barrier = _dist.barrier
new_group = _dist.new_group
destroy_process_group = _dist.destroy_process_group
