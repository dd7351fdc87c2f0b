#!/usr/bin/env python
"""Time the reference's UNMODIFIED GPU script as a local SageMaker job (the notebook-2 flow,
cifar10-distributed-smddp-gpu.py:110-180) at a chosen per-rank batch, and print one JSON line with
the job's own clocks: "Training seconds" (process start -> exit, as the reference's 438 s) and the
training-loop seconds (first forward -> completed, as its ~166 s).

    python tools/reference_job.py --batch-size 32 --epochs 3 [--env MI355X_DP_ENGINE_GRAPH=0 ...]

--batch-size is the script's GLOBAL batch (it divides by the world size); at one rank, 32 is the
per-GPU shape of the reference's 8-GPU job.  Synthetic full-size CIFAR-10 (no network).  The
script is the staged copy in ref_fixture/ (build() stages it; it is never committed).
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for the job (repeatable)")
    ap.add_argument("--tag", default="job")
    a = ap.parse_args()
    code_dir = os.path.join(ROOT, "ref_fixture", "notebooks", "code")
    if not os.path.exists(os.path.join(code_dir, "cifar10-distributed-smddp-gpu.py")):
        sys.exit("reference scripts not staged: run python -c 'import __graft_entry__ as g; g.build()'")
    work = tempfile.mkdtemp(prefix="refjob_")
    code = (
        "import sys, os\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.append({os.path.join(ROOT, 'compat')!r})\n"
        "from mi355x_dp.data.cifar import write_synthetic_cifar10\n"
        "write_synthetic_cifar10('data')\n"
        "from sagemaker.pytorch import PyTorch\n"
        f"est = PyTorch(entry_point='cifar10-distributed-smddp-gpu.py', source_dir={code_dir!r}, role='r',\n"
        "              instance_count=1, instance_type='ml.p4d.24xlarge', framework_version='1.11.0', py_version='py38',\n"
        f"              hyperparameters={{'epochs': {a.epochs}, 'lr': 0.01, 'momentum': 0.9, 'batch-size': {a.batch_size},\n"
        "                               'model-type': 'resnet18', 'backend': 'smddp'},\n"
        "              distribution={'smdistributed': {'dataparallel': {'enabled': True}}},\n"
        "              output_path=os.path.abspath('out'))\n"
        "est.fit({'train': os.path.abspath('data')}, job_name='ref-job')\n")
    env = {**os.environ, "MI355X_DP_S3_ROOT": os.path.join(work, "s3"), "MI355X_DP_JOBS_ROOT": os.path.join(work, "jobs"),
           "MI355X_DP_NPROC": "1"}
    for kv in a.env:
        k, v = kv.split("=", 1)
        env[k] = v
    r = subprocess.run([sys.executable, "-c", code], cwd=work, capture_output=True, text=True, timeout=1800, env=env)
    out = r.stdout + r.stderr
    sys.stderr.write(out[-3000:])
    if r.returncode != 0:
        sys.exit(r.returncode)
    job_s = int(re.search(r"Training seconds: (\d+)", out).group(1))
    m = re.search(r"Training loop seconds \(first forward -> completed\): ([\d.]+)", out)
    loop_s = float(m.group(1)) if m else None
    accs = [float(x) for x in re.findall(r"Accuracy: ([\d.]+)", out)]
    n_train = 50000
    res = {"tag": a.tag, "batch_size": a.batch_size, "epochs": a.epochs, "env": a.env, "job_seconds": job_s,
           "loop_seconds": loop_s,
           "img_per_s_lower_bound": round(a.epochs * n_train / loop_s, 1) if loop_s else None,
           "final_accuracy": accs[-1] if accs else None}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
