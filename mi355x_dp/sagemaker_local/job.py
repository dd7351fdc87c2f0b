"""Local training-job runner: the lifecycle of a SageMaker training job on one MI355X node
(SURVEY.md §2.2 C20 job lifecycle, C22 launcher, C23 model artifact).

Status lines mirror the real ones (reference nb2 log: "Starting - ...", "Downloading -
...", "Training - ...", "Uploading - ...", "Completed - ...", "Training seconds: N",
"Billable seconds: N").  The container layout is recreated under the job directory
(``opt_ml/input/data/<channel>``, ``opt_ml/model``, ``opt_ml/output``), the entry point
runs through the native launcher with the SM_* contract, and on success ``opt_ml/model``
is packed into ``model.tar.gz`` at ``<output_path>/<job>/output/model.tar.gz``.
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import tarfile
import time
from datetime import datetime
from typing import Dict, Optional

from mi355x_dp.launch import gpu_count, launch
from .env import env_vars, hyperparameters_to_args, training_env
from .session import local_to_s3, s3_to_local

# instance type -> (GPUs per host, vCPUs per host)
INSTANCE_TYPES = {
    "ml.p4d.24xlarge": (8, 96), "ml.p3.16xlarge": (8, 64), "ml.p3dn.24xlarge": (8, 96),
    "ml.p3.2xlarge": (1, 8), "ml.g5.48xlarge": (8, 192), "ml.c5.xlarge": (0, 4), "ml.c5.2xlarge": (0, 8),
    "ml.c5.4xlarge": (0, 16), "ml.m5.xlarge": (0, 4), "local": (None, None), "local_gpu": (None, None),
    "mi355x": (None, None),
}


class JobFailed(RuntimeError):
    pass


def _status(msg: str):
    print(f"{datetime.now().strftime('%Y-%m-%d %H:%M:%S')} {msg}", flush=True)


class TrainingJob:
    def __init__(self, job_name: str, entry_point: str, source_dir: Optional[str], hyperparameters: Dict,
                 inputs: Dict[str, str], output_path: str, instance_count: int = 1, instance_type: str = "local",
                 distribution: Optional[Dict] = None, environment: Optional[Dict] = None,
                 jobs_root: Optional[str] = None):
        self.job_name = job_name
        self.entry_point = entry_point
        self.source_dir = os.path.abspath(source_dir) if source_dir else os.path.dirname(os.path.abspath(entry_point))
        self.hyperparameters = dict(hyperparameters or {})
        self.inputs = dict(inputs or {})
        self.output_path = output_path
        self.instance_count = int(instance_count)
        self.instance_type = instance_type
        self.distribution = distribution or {}
        self.environment = dict(environment or {})
        root = jobs_root or os.environ.get("MI355X_DP_JOBS_ROOT", os.path.expanduser("~/.mi355x_dp/jobs"))
        self.job_dir = os.path.join(root, job_name)
        self.training_seconds = None
        self.model_data = None
        self.exit_code = None

    # ------------------------------------------------------------------ layout
    def _prepare(self):
        opt = os.path.join(self.job_dir, "opt_ml")
        self.input_dir = os.path.join(opt, "input")
        self.model_dir = os.path.join(opt, "model")
        self.output_dir = os.path.join(opt, "output")
        for d in (os.path.join(self.input_dir, "config"), os.path.join(self.input_dir, "data"), self.model_dir,
                  os.path.join(self.output_dir, "data"), os.path.join(self.output_dir, "intermediate")):
            os.makedirs(d, exist_ok=True)
        self.channels = {}
        for ch, uri in self.inputs.items():
            src = s3_to_local(uri)
            dst = os.path.join(self.input_dir, "data", ch)
            if os.path.islink(dst) or os.path.exists(dst):
                if os.path.islink(dst):
                    os.unlink(dst)
                else:
                    shutil.rmtree(dst)
            os.symlink(src, dst)  # "File" mode without the copy
            self.channels[ch] = dst
        code_dir = os.path.join(opt, "code")
        if os.path.exists(code_dir):
            shutil.rmtree(code_dir)
        shutil.copytree(self.source_dir, code_dir, ignore=shutil.ignore_patterns(".ipynb_checkpoints", "__pycache__"))
        self.code_dir = code_dir
        with open(os.path.join(self.input_dir, "config", "hyperparameters.json"), "w") as f:
            json.dump({k: str(v) for k, v in self.hyperparameters.items()}, f)

    def _topology(self):
        gpus_per_host, cpus = INSTANCE_TYPES.get(self.instance_type, (None, None))
        avail = gpu_count()
        if gpus_per_host is None:
            gpus_per_host = avail
        cpus = cpus or (os.cpu_count() or 1)
        smddp = bool(self.distribution.get("smdistributed", {}).get("dataparallel", {}).get("enabled"))
        torch_dist = bool(self.distribution.get("pytorchddp", {}).get("enabled") or
                          self.distribution.get("torch_distributed", {}).get("enabled"))
        if gpus_per_host and (smddp or torch_dist):
            n = min(gpus_per_host, avail) if avail else gpus_per_host
            n = int(os.environ.get("MI355X_DP_NPROC", n))
            return ["algo-1"], max(1, n), gpus_per_host, cpus, False
        # plain (non-MPI) job: one process per host; instance_count hosts run as local ranks
        hosts = [f"algo-{i + 1}" for i in range(self.instance_count)]
        return hosts, self.instance_count, gpus_per_host or 0, cpus, True

    # --------------------------------------------------------------------- run
    def run(self, wait: bool = True, logs: bool = True):
        t_start = time.time()
        _status("Starting - Starting the training job...")
        _status("Starting - Preparing the instances for training...")
        self._prepare()
        _status("Downloading - Downloading input data")
        hosts, nproc, gpus, cpus, per_host = self._topology()
        _status("Training - Training image download completed. Training in progress.")
        module_dir = local_to_s3(self.code_dir)
        tenv = training_env(self.job_name, self.entry_point, self.hyperparameters, self.channels, self.model_dir,
                            self.output_dir, self.input_dir, hosts, hosts[0], gpus, cpus, self.instance_type,
                            module_dir, self.distribution)
        env = env_vars(tenv)
        env.update(self.environment)
        env["PYTHONUNBUFFERED"] = "1"
        if str(self.environment.get("MI355X_DP_DEBUGGER", "1")) not in ("0", "false", "False"):
            # SageMaker attaches its Debugger hook inside the container; ours records the same
            # parameter inventory and "losses" collection under output/tensors
            env["MI355X_DP_DEBUGGER"] = os.path.join(self.output_dir, "tensors")
        print("Training Env:\n" + json.dumps(tenv, indent=4, sort_keys=True), flush=True)
        print("Environment variables:\n" + "\n".join(f"{k}={v}" for k, v in sorted(env.items())
                                                       if k.startswith("SM_")), flush=True)
        cmd = [sys.executable, os.path.join(self.code_dir, os.path.basename(self.entry_point))]
        cmd += hyperparameters_to_args(self.hyperparameters)
        print("Invoking script with the following command:\n" + " ".join(cmd), flush=True)
        t_train = time.time()
        rank_env = {"SM_CURRENT_HOST": "algo-"} if per_host and len(hosts) > 1 else None
        # multi-rank jobs pin each rank to CPUs of its GPU's NUMA node (the reference's mpirun bound
        # ranks to their GPU's socket, nb2:380); MI355X_DP_BIND_CPUS=0 turns it off
        bind = nproc > 1 and os.environ.get("MI355X_DP_BIND_CPUS", "1") != "0"
        rc = launch(cmd, nproc=nproc, env=env, tag_output=nproc > 1, rank_env=rank_env, cwd=self.code_dir,
                    bind_cpus=bind)
        self.exit_code = rc
        self.training_seconds = int(round(time.time() - t_train))
        if rc != 0:
            _status(f"Failed - Training job failed: AlgorithmError: ExecuteUserScriptError, exit code {rc}")
            raise JobFailed(f"training job {self.job_name} failed with exit code {rc}")
        print("Reporting training SUCCESS", flush=True)
        _status("Uploading - Uploading generated training model")
        self.model_data = self._package()
        _status("Completed - Training job completed")
        print(f"Training seconds: {self.training_seconds}")
        print(f"Billable seconds: {self.training_seconds}", flush=True)
        self.wall_seconds = time.time() - t_start
        self.loop_seconds = self._loop_seconds(env.get("MI355X_DP_DEBUGGER"))
        if self.loop_seconds is not None:
            # the reference's ~166 s figure is the same span: first forward (hook's parameter
            # inventory, nb2:1521) -> "Completed" (nb2:2609-2610), BASELINE.md row 2
            print(f"Training loop seconds (first forward -> completed): {self.loop_seconds:.1f}", flush=True)
        return self

    @staticmethod
    def _loop_seconds(tensors_dir):
        if not tensors_dir:
            return None
        try:
            with open(os.path.join(tensors_dir, "collections", "parameters.json")) as f:
                t0 = json.load(f).get("first_forward_time")
        except (OSError, ValueError):
            return None
        return None if t0 is None else time.time() - float(t0)

    def _package(self) -> str:
        out = os.path.join(s3_to_local(self.output_path.rstrip("/")), self.job_name, "output")
        os.makedirs(out, exist_ok=True)
        tar_path = os.path.join(out, "model.tar.gz")
        with tarfile.open(tar_path, "w:gz") as tf:
            for name in sorted(os.listdir(self.model_dir)):
                tf.add(os.path.join(self.model_dir, name), arcname=name)
        return local_to_s3(tar_path) if self.output_path.startswith("s3://") else tar_path
