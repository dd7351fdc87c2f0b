from mi355x_dp.sagemaker_local.estimator import PyTorch, PyTorchModel  # noqa: F401
from mi355x_dp.serve import Predictor as PyTorchPredictor  # noqa: F401
