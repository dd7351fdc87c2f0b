"""``import smdistributed.dataparallel.torch.torch_smddp`` registers the ``smddp``
process-group backend (reference cifar10-distributed-smddp-gpu.py:17) and, like SMDDP's own
library DDP, routes ``torch.nn.parallel.DistributedDataParallel`` of a native-layer model on a GPU
to the flat-buffer engine (mi355x_dp/parallel/engine_ddp.py; MI355X_DP_ENGINE_DDP=0 keeps torch's
class)."""
from mi355x_dp.parallel.engine_ddp import install as _install_engine_ddp
from mi355x_dp.parallel.smddp import register as _register

_register()
_install_engine_ddp()
