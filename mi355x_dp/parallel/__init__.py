from mi355x_dp.utils import hwqueues as _hwqueues

_hwqueues.ensure()  # before the first HIP call: compute / weight-gradient / comm streams on their own queues

from .ddp import DataParallel, FlatSGD, plan_buckets  # noqa: E402,F401
from .flat import FlatBuffers, FlatParams  # noqa: E402,F401
