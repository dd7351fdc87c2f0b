from .distributed import DistributedDataParallel  # noqa: F401
