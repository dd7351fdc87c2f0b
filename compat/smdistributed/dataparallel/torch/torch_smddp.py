"""``import smdistributed.dataparallel.torch.torch_smddp`` registers the ``smddp``
process-group backend (reference cifar10-distributed-smddp-gpu.py:17)."""
from mi355x_dp.parallel.smddp import register as _register

_register()
