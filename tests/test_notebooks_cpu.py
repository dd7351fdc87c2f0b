"""The workshop driver notebooks (notebooks/*.ipynb) executed cell by cell
through mi355x_dp local mode: notebook 1 on CPU (2-rank gloo job, deploy, predict); notebook 2 on
the GPU (smddp job, deploy, predict)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(nb, tmp_path, extra_env):
    env = {**os.environ, "MI355X_DP_REPO": ROOT, "MI355X_DP_S3_ROOT": str(tmp_path / "s3"),
           "MI355X_DP_JOBS_ROOT": str(tmp_path / "jobs"), "NB_EPOCHS": "1", "NB_N_TRAIN": "1024",
           "NB_N_TEST": "256", **extra_env}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "run_notebook.py"),
                        os.path.join(ROOT, "notebooks", nb)], cwd=tmp_path, capture_output=True, text=True,
                       timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    return out


def test_notebook1_cpu_gloo(tmp_path):
    out = _run("1_pytorch_dist_native_cpu.ipynb", tmp_path, {"MI355X_DP_NUM_GPUS": "0"})
    assert "Initialized the distributed environment: 'gloo' backend on 2 nodes." in out
    assert "Completed - Training job completed" in out
    assert "MODEL_DATA s3://" in out and "model.tar.gz" in out
    assert "PREDICT_SHAPE (4, 10)" in out


@pytest.mark.gpu
def test_notebook2_smddp_gpu(tmp_path):
    out = _run("2_pytorch_dist_smddp_mi355x.ipynb", tmp_path, {})
    assert "'smddp' backend" in out
    assert "Completed - Training job completed" in out
    assert "PREDICT_SHAPE (4, 1000)" in out
