"""Local-mode SageMaker control plane for one MI355X node: Session / upload_data,
PyTorch estimator .fit() (training-job lifecycle, SM_* contract, native launcher,
model.tar.gz artifact), PyTorchModel.deploy() -> Predictor.predict()."""
from .estimator import PyTorch, PyTorchModel  # noqa: F401
from .job import JobFailed, TrainingJob  # noqa: F401
from .session import Session, get_execution_role  # noqa: F401
