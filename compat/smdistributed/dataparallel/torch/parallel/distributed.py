"""SMDDP v1 ``DistributedDataParallel(model)``: the mi355x_dp flat-buffer bucketed engine."""
from mi355x_dp.parallel import DataParallel as DistributedDataParallel  # noqa: F401
