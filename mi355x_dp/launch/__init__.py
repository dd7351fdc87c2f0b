"""Process launcher front-end: one rank per GPU through the native ``mi355x_launch``.

    python -m mi355x_dp.launch --nproc 8 [--tag-output] script.py args...
    python -m mi355x_dp.launch --sagemaker --hyperparameters '{"epochs": 1}' \
        --data-dir DIR --model-dir DIR script.py

``--sagemaker`` additionally sets the full SM_* environment contract so the
workshop's unmodified scripts (which read SM_HOSTS / SM_CURRENT_HOST /
SM_MODEL_DIR / SM_CHANNEL_TRAIN in argparse defaults) run as inside a
SageMaker training container, with hyperparameters appended as CLI args.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Dict, List, Optional

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# import-path compat packages: the source tree's compat/ (editable / in-tree use), else the copy a
# wheel ships inside the package (mi355x_dp/_compat)
COMPAT_DIR = os.path.join(REPO_ROOT, "compat")
if not os.path.isdir(COMPAT_DIR):
    COMPAT_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_compat")
NATIVE_LAUNCHER = os.path.join(REPO_ROOT, "mi355x_dp", "_native", "mi355x_launch")


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def compat_pythonpath(existing: Optional[str] = None) -> str:
    """Repo root first (mi355x_dp), compat packages LAST so a real torchvision / sagemaker /
    smdistributed install always wins over our stand-ins."""
    parts = [REPO_ROOT]
    if existing:
        parts += [p for p in existing.split(os.pathsep) if p and p not in (REPO_ROOT, COMPAT_DIR)]
    parts.append(COMPAT_DIR)
    return os.pathsep.join(parts)


def ensure_launcher() -> str:
    if not os.path.exists(NATIVE_LAUNCHER):
        from mi355x_dp.build import build_launcher
        build_launcher(verbose=False)
    return NATIVE_LAUNCHER


def gpu_count() -> int:
    """Count GPUs without initialising HIP in this process (launcher must stay GPU-free)."""
    env = os.environ.get("MI355X_DP_NUM_GPUS")
    if env is not None:
        return int(env)
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def launch(cmd: List[str], nproc: int = 1, env: Optional[Dict[str, str]] = None, tag_output: bool = False,
           host: str = "algo-1", rank_env: Optional[Dict[str, str]] = None, master_port: Optional[int] = None,
           bind_cpus: bool = False, cwd: Optional[str] = None, stdout=None, stderr=None) -> int:
    """Run ``cmd`` as ``nproc`` ranks; returns the job exit code (first failing rank's)."""
    exe = ensure_launcher()
    full_env = dict(os.environ)
    full_env.update(env or {})
    full_env["PYTHONPATH"] = compat_pythonpath(full_env.get("PYTHONPATH"))
    full_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    args = [exe, "--nproc", str(nproc), "--host", host, "--master-addr", "127.0.0.1",
            "--master-port", str(master_port or free_port())]
    if tag_output:
        args.append("--tag-output")
    if bind_cpus:
        args.append("--bind-cpus")
    for k, v in (rank_env or {}).items():
        args += ["--rank-env", f"{k}={v}"]
    args.append("--")
    args += cmd
    proc = subprocess.run(args, env=full_env, cwd=cwd, stdout=stdout, stderr=stderr)
    return proc.returncode


def main(argv=None):
    import argparse
    import json

    ap = argparse.ArgumentParser(prog="python -m mi355x_dp.launch")
    ap.add_argument("--nproc", type=int, default=None, help="ranks (default: #GPUs, or 1)")
    ap.add_argument("--tag-output", action="store_true")
    ap.add_argument("--bind-cpus", action="store_true")
    ap.add_argument("--sagemaker", action="store_true", help="set the SM_* training-container contract")
    ap.add_argument("--hyperparameters", default="{}")
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--model-dir", default=None)
    ap.add_argument("--output-dir", default=None)
    ap.add_argument("--job-name", default="local-job")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    nproc = a.nproc or max(1, gpu_count())
    env = {}
    cmd = [sys.executable, a.script] + a.script_args
    if a.sagemaker:
        from mi355x_dp.sagemaker_local.env import env_vars, hyperparameters_to_args, training_env
        hps = json.loads(a.hyperparameters)
        root = os.path.abspath(a.output_dir or os.path.join(os.getcwd(), "opt_ml"))
        model_dir = os.path.abspath(a.model_dir or os.path.join(root, "model"))
        os.makedirs(model_dir, exist_ok=True)
        tenv = training_env(a.job_name, a.script, hps, {"train": os.path.abspath(a.data_dir or ".")}, model_dir,
                            os.path.join(root, "output"), os.path.join(root, "input"), ["algo-1"], "algo-1",
                            gpu_count(), os.cpu_count() or 1, "local", os.path.dirname(os.path.abspath(a.script)))
        env.update(env_vars(tenv))
        cmd += hyperparameters_to_args(hps)
    return launch(cmd, nproc=nproc, env=env, tag_output=a.tag_output, bind_cpus=a.bind_cpus)


if __name__ == "__main__":
    sys.exit(main())
