from .ddp import DataParallel, FlatSGD, plan_buckets  # noqa: F401
from .flat import FlatBuffers, FlatParams  # noqa: F401
