"""Local stand-in for the ``sagemaker`` SDK (not installed here), backed by
mi355x_dp.sagemaker_local: notebooks' Session / get_execution_role / upload_data /
PyTorch(...).fit() / PyTorchModel(...).deploy() / predictor.predict() run locally."""
from mi355x_dp.sagemaker_local import Session, get_execution_role  # noqa: F401
from mi355x_dp.sagemaker_local.session import Session as LocalSession  # noqa: F401
from . import pytorch  # noqa: F401

__version__ = "2.0.0+mi355x_dp.local"
