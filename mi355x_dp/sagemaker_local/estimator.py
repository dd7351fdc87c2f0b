"""``sagemaker.pytorch.PyTorch`` estimator and ``PyTorchModel`` in local mode
(reference nb1:111-162, nb2:136-146 / 2617)."""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

from .job import TrainingJob
from .session import Session


class PyTorch:
    def __init__(self, entry_point: str, source_dir: Optional[str] = None, role: Optional[str] = None,
                 instance_count: int = 1, instance_type: str = "local", framework_version: Optional[str] = None,
                 py_version: Optional[str] = None, hyperparameters: Optional[Dict] = None,
                 distribution: Optional[Dict] = None, output_path: Optional[str] = None,
                 code_location: Optional[str] = None, sagemaker_session: Optional[Session] = None,
                 base_job_name: Optional[str] = None, environment: Optional[Dict] = None, **kwargs):
        self.entry_point = entry_point
        self.source_dir = source_dir
        self.role = role
        self.instance_count = instance_count
        self.instance_type = instance_type
        self.framework_version = framework_version
        self.py_version = py_version
        self.hyperparameters = dict(hyperparameters or {})
        self.distribution = distribution or {}
        self.sagemaker_session = sagemaker_session or Session()
        self.output_path = output_path or f"s3://{self.sagemaker_session.default_bucket()}/"
        self.code_location = code_location
        self.base_job_name = base_job_name or "pytorch-training"
        self.environment = environment or {}
        self.latest_training_job = None
        self._model_data = None

    def _entry_path(self):
        if self.source_dir:
            return os.path.join(self.source_dir, self.entry_point)
        return self.entry_point

    def fit(self, inputs=None, wait: bool = True, logs: bool = True, job_name: Optional[str] = None, **kwargs):
        if isinstance(inputs, str):
            inputs = {"training": inputs}
        job_name = job_name or f"{self.base_job_name}-{time.strftime('%Y-%m-%d-%H-%M-%S', time.gmtime())}"
        job = TrainingJob(job_name, self._entry_path(), self.source_dir, self.hyperparameters, inputs or {},
                          self.output_path, self.instance_count, self.instance_type, self.distribution,
                          self.environment)
        self.latest_training_job = job
        job.run(wait=wait, logs=logs)
        self._model_data = job.model_data
        return job

    @property
    def model_data(self):
        return self._model_data

    def hyperparameters_dict(self):
        return dict(self.hyperparameters)

    def deploy(self, initial_instance_count=1, instance_type="local", entry_point=None, source_dir=None, **kw):
        model = PyTorchModel(self.model_data, role=self.role, entry_point=entry_point or self.entry_point,
                             source_dir=source_dir or self.source_dir)
        return model.deploy(initial_instance_count, instance_type, **kw)


class PyTorchModel:
    def __init__(self, model_data: str, role: Optional[str] = None, entry_point: str = "inference.py",
                 source_dir: Optional[str] = None, framework_version: Optional[str] = None,
                 py_version: Optional[str] = None, **kwargs):
        self.model_data = model_data
        self.role = role
        self.entry_point = entry_point
        self.source_dir = source_dir
        self.framework_version = framework_version

    def deploy(self, initial_instance_count: int = 1, instance_type: str = "local", serializer=None,
               deserializer=None, endpoint_name: Optional[str] = None, http: bool = False, **kwargs):
        from mi355x_dp.serve import Predictor, load_model_server
        server = load_model_server(self.model_data, self.entry_point, self.source_dir,
                                   device="cuda" if instance_type in ("local_gpu", "mi355x") else "cpu")
        return Predictor(server, endpoint_name=endpoint_name or f"endpoint-{int(time.time())}", http=http)
