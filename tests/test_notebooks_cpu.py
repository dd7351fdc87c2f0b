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


REF_NB1 = None
for _d in (os.environ.get("MI355X_DP_REF_NOTEBOOKS"), "/root/reference/notebooks",
           os.path.join(ROOT, "ref_fixture", "notebooks")):
    if _d and os.path.exists(os.path.join(_d, "1_pytorch_dist_native_cpu.ipynb")):
        REF_NB1 = os.path.join(_d, "1_pytorch_dist_native_cpu.ipynb")
        break


@pytest.mark.skipif(REF_NB1 is None, reason="reference notebooks not staged (run build())")
def test_reference_notebook1_verbatim(tmp_path):
    """The reference's OWN notebook 1, every code cell executed verbatim (no edits) through the
    compat SDK: download -> upload -> 2-host gloo fit() of the unmodified CPU script (20 epochs)
    -> deploy -> the test-loader cell.  Cell 14 is the documented incompatibility: it calls
    ``dataiter.next()`` (nb1:203), which DataLoader iterators no longer have in torch >= 2.
    The synthetic 'download' is shrunk via MI355X_DP_SYNTH_CIFAR_TRAIN so 20 epochs fit a CPU test."""
    import json
    report = tmp_path / "nb1.json"
    env = {**os.environ, "MI355X_DP_S3_ROOT": str(tmp_path / "s3"), "MI355X_DP_JOBS_ROOT": str(tmp_path / "jobs"),
           "MI355X_DP_NUM_GPUS": "0", "MI355X_DP_SYNTH_CIFAR_TRAIN": "2048", "MI355X_DP_SYNTH_CIFAR_TEST": "512"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "run_notebook.py"), "--compat", "--keep-going",
                        "--workdir", str(tmp_path / "nb"), "--expect-fail", "14", "--report", str(report), REF_NB1],
                       capture_output=True, text=True, timeout=900, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    cells = {c["cell"]: c for c in json.load(open(report))["cells"]}
    failed = {i for i, c in cells.items() if c["status"] != "ok"}
    assert failed == {14}, cells
    assert "has no attribute 'next'" in cells[14]["error"]
    assert "Initialized the distributed environment: 'gloo' backend on 2 nodes." in out
    assert "Completed - Training job completed" in out
    assert out.count("Test set: Average loss") >= 20  # every epoch evaluated (cpu.py:177-194)
