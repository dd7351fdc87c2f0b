"""CPU tests of the platform layer: SM_* contract, native launcher, local estimator running the
reference CPU script unmodified (gloo, world 2), model artifact + serving."""
import io
import json
import os
import subprocess
import sys
import tarfile

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CODE = "/root/reference/notebooks/code"


def test_hyperparameters_and_env_contract():
    from mi355x_dp.sagemaker_local.env import env_vars, hyperparameters_to_args, training_env
    hps = {"epochs": 15, "lr": 0.01, "momentum": 0.9, "batch-size": 256, "model-type": "resnet18", "backend": "smddp"}
    # SM_USER_ARGS in the captured log (nb2): sorted --key value pairs
    assert hyperparameters_to_args(hps) == ["--backend", "smddp", "--batch-size", "256", "--epochs", "15", "--lr",
                                            "0.01", "--model-type", "resnet18", "--momentum", "0.9"]
    t = training_env("job", "cifar10-distributed-smddp-gpu.py", hps, {"train": "/opt/ml/input/data/train"},
                     "/opt/ml/model", "/opt/ml/output", "/opt/ml/input", ["algo-1"], "algo-1", 8, 96,
                     "ml.p4d.24xlarge", "s3://x/source", {"smdistributed": {"dataparallel": {"enabled": True}}})
    e = env_vars(t)
    assert e["SM_HOSTS"] == '["algo-1"]'
    assert e["SM_CURRENT_HOST"] == "algo-1"
    assert e["SM_MODEL_DIR"] == "/opt/ml/model"
    assert e["SM_CHANNEL_TRAIN"] == "/opt/ml/input/data/train"
    assert e["SM_NUM_GPUS"] == "8" and e["SM_NUM_CPUS"] == "96"
    assert e["SM_HP_BATCH-SIZE"] == "256" and e["SM_HP_BACKEND"] == "smddp"
    assert e["SM_MODULE_NAME"] == "cifar10-distributed-smddp-gpu"
    assert json.loads(e["SM_TRAINING_ENV"])["additional_framework_parameters"][
        "sagemaker_distributed_dataparallel_enabled"] is True
    assert json.loads(e["SM_USER_ARGS"])[:2] == ["--backend", "smddp"]


def _launcher():
    from mi355x_dp.launch import ensure_launcher
    return ensure_launcher()


def test_native_launcher_env_and_tags():
    exe = _launcher()
    r = subprocess.run([exe, "--nproc", "3", "--tag-output", "--rank-env", "SM_CURRENT_HOST=algo-", "--",
                        sys.executable, "-c",
                        "import os;print(os.environ['RANK'],os.environ['LOCAL_RANK'],os.environ['WORLD_SIZE'],"
                        "os.environ['SM_CURRENT_HOST'],os.environ['MASTER_ADDR'])"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    lines = sorted(r.stdout.strip().splitlines())
    assert lines == [f"[1,mpirank:{i},algo-1]<stdout>:{i} {i} 3 algo-{i + 1} 127.0.0.1" for i in range(3)]


def test_native_launcher_abort_all_on_failure():
    exe = _launcher()
    code = "import os,sys,time\nr=int(os.environ['RANK'])\nif r==1: sys.exit(7)\ntime.sleep(60)\n"
    r = subprocess.run([exe, "--nproc", "3", "--grace", "2", "--", sys.executable, "-c", code],
                       capture_output=True, text=True, timeout=40)
    assert r.returncode == 7
    assert "rank 1 exited with status 7; aborting all ranks" in r.stderr


@pytest.mark.skipif(not os.path.exists(REF_CODE), reason="reference checkout not mounted")
def test_notebook1_flow_cpu_gloo_world2(tmp_path):
    """Notebook-1 path end to end: upload_data -> PyTorch(instance_count=2, gloo).fit() running the
    UNMODIFIED cifar10-distributed-native-cpu.py -> model.tar.gz -> PyTorchModel(inference.py).deploy()
    -> predictor.predict(4 images) (in-process and over HTTP)."""
    code = f"""
import os, sys, json
sys.path.insert(0, {ROOT!r}); sys.path.append({os.path.join(ROOT, 'compat')!r})
from mi355x_dp.data.cifar import write_synthetic_cifar10
write_synthetic_cifar10('cifar10-dataset', n_train=512, n_test=128)
import sagemaker, torch
from sagemaker.pytorch import PyTorch, PyTorchModel
sess = sagemaker.Session(); role = sagemaker.get_execution_role()
uri = sess.upload_data(path='cifar10-dataset', key_prefix='datasets/cifar10-dataset')
est = PyTorch(entry_point='cifar10-distributed-native-cpu.py', source_dir={REF_CODE!r},
              output_path=f"s3://{{sess.default_bucket()}}/jobs/", role=role, instance_count=2,
              instance_type='ml.c5.2xlarge', framework_version='1.8.0', py_version='py3',
              hyperparameters={{'epochs': 1, 'lr': 0.01, 'momentum': 0.9, 'batch-size': 64,
                               'model-type': 'custom', 'backend': 'gloo'}})
est.fit({{'train': uri}}, job_name='nb1', wait=True)
m = PyTorchModel(model_data=est.model_data, source_dir={REF_CODE!r}, entry_point='inference.py', role=role,
                 framework_version='1.6.0', py_version='py3')
p = m.deploy(initial_instance_count=1, instance_type='ml.c5.xlarge')
out = p.predict(torch.randn(4, 3, 32, 32))
ph = m.deploy(initial_instance_count=1, instance_type='ml.c5.xlarge', http=True)
out2 = ph.predict(torch.randn(4, 3, 32, 32)); ph.delete_endpoint()
print('SHAPES', out.shape, out2.shape)
print('MODEL_DATA', est.model_data)
"""
    env = {**os.environ, "MI355X_DP_S3_ROOT": str(tmp_path / "s3"), "MI355X_DP_JOBS_ROOT": str(tmp_path / "jobs")}
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True, timeout=600,
                       env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "Initialized the distributed environment: 'gloo' backend on 2 nodes." in out
    assert "[1,mpirank:1,algo-1]<stdout>:" in out
    assert "Training seconds:" in out and "Completed - Training job completed" in out
    assert "SHAPES (4, 10) (4, 10)" in out
    # observability hook auto-attached by the job: inventory + losses collection
    assert "[mi355x_dp.debugger] Total Trainable Params: 62006" in out
    assert "name:module.conv1.weight count_params:450" in out
    import glob
    losses = glob.glob(str(tmp_path / "jobs" / "**" / "collections" / "losses.jsonl"), recursive=True)
    assert losses and all(json.loads(l)["loss"] > 0 for l in open(losses[0]))
    from mi355x_dp.sagemaker_local.session import s3_to_local
    os.environ["MI355X_DP_S3_ROOT"] = str(tmp_path / "s3")
    tar = s3_to_local([l.split()[1] for l in r.stdout.splitlines() if l.startswith("MODEL_DATA")][0])
    with tarfile.open(tar) as tf:
        tf.extract("model.pth", path=tmp_path)
    sd = torch.load(tmp_path / "model.pth", weights_only=True)
    # CPU script saves model.module.state_dict(): bare Net keys (cpu.py:199) -> loadable by inference.py
    assert list(sd.keys()) == ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "fc1.weight", "fc1.bias",
                               "fc2.weight", "fc2.bias", "fc3.weight", "fc3.bias"]
    assert sum(v.numel() for v in sd.values()) == 62006


def test_serving_default_handlers():
    from mi355x_dp.serve import NPY, default_input_fn, default_output_fn
    x = np.random.randn(2, 3).astype(np.float32)
    buf = io.BytesIO()
    np.save(buf, x)
    t = default_input_fn(buf.getvalue(), NPY)
    assert torch.allclose(t, torch.from_numpy(x))
    back = np.load(io.BytesIO(default_output_fn(t * 2, NPY)))
    assert np.allclose(back, 2 * x)


def test_model_archive_path_traversal_refused(tmp_path):
    from mi355x_dp.serve import extract_model
    evil = tmp_path / "m.tar.gz"
    with tarfile.open(evil, "w:gz") as tf:
        data = b"x"
        ti = tarfile.TarInfo("../escape.txt")
        ti.size = 1
        tf.addfile(ti, io.BytesIO(data))
    with pytest.raises(ValueError):
        extract_model(str(evil))


def _fake_topology(root, gpus, nodes):
    """gpus: [(pci_address, numa_node)]; nodes: {node: cpulist}"""
    for i, (pci, node) in enumerate(gpus):
        dev = root / "pci" / pci
        dev.mkdir(parents=True)
        (dev / "vendor").write_text("0x1002\n")
        (dev / "class").write_text("0x120000\n")
        (dev / "numa_node").write_text(f"{node}\n")
        card = root / "sys" / "class" / "drm" / f"card{i}"
        card.mkdir(parents=True)
        (card / "device").symlink_to(dev)
        (root / "sys" / "class" / "drm" / f"card{i}-DP-1").mkdir()  # connector entries are skipped
    other = root / "pci" / "0000:ff:00.0"  # a non-AMD display device is ignored
    other.mkdir(parents=True)
    (other / "vendor").write_text("0x10de\n")
    (other / "class").write_text("0x030000\n")
    (root / "sys" / "class" / "drm" / "card99").mkdir()
    (root / "sys" / "class" / "drm" / "card99" / "device").symlink_to(other)
    for n, cpus in nodes.items():
        d = root / "sys" / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")


def _binding(root, nproc):
    from mi355x_dp.launch import ensure_launcher
    r = subprocess.run([ensure_launcher(), "--nproc", str(nproc), "--print-binding"], capture_output=True, text=True,
                       env={**os.environ, "MI355X_DP_TOPO_ROOT": str(root)}, timeout=30)
    assert r.returncode == 0, r.stderr
    plan = {}
    for line in r.stdout.splitlines():
        head, cpus = line.split(":")
        plan[int(head.split()[1])] = (head.split("(")[1].rstrip(")"), [int(c) for c in cpus.split()])
    return plan


def test_launcher_numa_binding(tmp_path):
    """--bind-cpus pins local rank r (driving GPU r) to CPUs of GPU r's NUMA node; GPUs are taken in
    PCI order (= HIP device order) and alternate between two nodes here, so ranks 0,2,4,6 share
    node 0's CPUs and 1,3,5,7 node 1's.  Without a readable topology: equal slices."""
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 4:
        pytest.skip("needs >= 4 allowed CPUs")
    half = len(allowed) // 2
    n0, n1 = allowed[:half], allowed[half:2 * half]
    gpus = [(f"0000:{0x05 + 0x10 * i:02x}:00.0", i % 2) for i in range(8)]
    import random
    random.Random(0).shuffle(gpus)  # directory order must not matter, PCI order does
    _fake_topology(tmp_path, gpus, {0: ",".join(map(str, n0)), 1: ",".join(map(str, n1))})
    plan = _binding(tmp_path, 8)
    assert all(how == "numa" for how, _ in plan.values())
    for r in range(8):
        node_cpus = n0 if r % 2 == 0 else n1
        assert plan[r][1] and set(plan[r][1]) <= set(node_cpus), (r, plan[r])
    # the 4 ranks of a node get disjoint, equal shares of it
    for node_ranks in ((0, 2, 4, 6), (1, 3, 5, 7)):
        sets = [set(plan[r][1]) for r in node_ranks]
        assert len(set(map(len, sets))) == 1
        assert sum(map(len, sets)) == len(set().union(*sets))
    # unreadable topology -> contiguous equal slices of the allowed set
    plan = _binding(tmp_path / "missing", 4)
    assert all(how == "slices" for how, _ in plan.values())
    assert plan[0][1][0] == allowed[0]


def test_hw_queue_sizing(monkeypatch):
    """utils.hwqueues.ensure: raises GPU_MAX_HW_QUEUES to 8 before HIP starts when each GPU hosts at
    most one rank, never lowers an explicit larger value, leaves ranks that share GPUs alone, and
    does nothing without a GPU or with MI355X_DP_HW_QUEUES=0."""
    import torch
    from mi355x_dp.utils import hwqueues
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("MI355X_DP_HW_QUEUES", raising=False)
    monkeypatch.setenv(hwqueues.AUTO_MARK, "0")  # restored after the test (ensure() sets it)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert hwqueues.ensure() == 8 and os.environ["GPU_MAX_HW_QUEUES"] == "8"
    assert os.environ[hwqueues.AUTO_MARK] == "1"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "16")
    assert hwqueues.ensure() is None and os.environ["GPU_MAX_HW_QUEUES"] == "16"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv(hwqueues.AUTO_MARK, "0")  # a user's value
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "16")  # two ranks per GPU
    assert hwqueues.ensure() is None and os.environ["GPU_MAX_HW_QUEUES"] == "4"
    # ranks sharing GPUs that inherited the automatic 8 of a one-rank-per-GPU parent: dropped to 1
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    monkeypatch.setenv(hwqueues.AUTO_MARK, "1")
    assert hwqueues.ensure() == hwqueues.SHARED and os.environ["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    monkeypatch.setenv(hwqueues.AUTO_MARK, "0")
    assert hwqueues.ensure() == hwqueues.SHARED and os.environ["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv(hwqueues.AUTO_MARK, "0")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setenv("MI355X_DP_HW_QUEUES", "0")
    assert hwqueues.ensure() is None
    monkeypatch.delenv("MI355X_DP_HW_QUEUES")
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    assert hwqueues.ensure() is None
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert hwqueues.ensure() is None and os.environ["GPU_MAX_HW_QUEUES"] == "4"


def test_hw_queue_warning(monkeypatch):
    """hwqueues.check: one warning when a process group and the weight-gradient stream run on fewer
    than 6 hardware queues (including HIP's default of 4 when the variable is unset, and the value
    that was in force when HIP started before ensure() could raise it); silent otherwise."""
    import io
    from mi355x_dp.utils import hwqueues
    monkeypatch.setattr(hwqueues, "_warned", False)
    monkeypatch.setattr(hwqueues, "_late_value", None)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    s = io.StringIO()
    assert not hwqueues.check(True, True, stream=s) and s.getvalue() == ""
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    assert hwqueues.effective() == 4
    assert not hwqueues.check(False, True, stream=s)  # no process group: no comm stream
    assert not hwqueues.check(True, False, stream=s)  # single-stream backward
    assert not hwqueues.check(True, True, shared_gpu=True, stream=s)  # rehearsal ranks keep 1 queue
    assert hwqueues.check(True, True, stream=s) and "4 hardware queues" in s.getvalue()
    n = len(s.getvalue())
    assert hwqueues.check(True, True, stream=s) and len(s.getvalue()) == n  # warned once
    # HIP started at 4 before ensure(): raising the variable afterwards does not count
    monkeypatch.setattr(hwqueues, "_late_value", "4")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    assert hwqueues.effective() == 4 and hwqueues.check(True, True, stream=s)


def test_checkpoint_roundtrip(tmp_path):
    """utils.save_model writes the reference's model.pth (plain state_dict) and save_checkpoint /
    load_checkpoint round-trip model + FlatSGD momentum + step, loaded with weights_only=True."""
    import torch
    from mi355x_dp.models import Net
    from mi355x_dp.parallel import DataParallel, FlatSGD
    from mi355x_dp.utils import load_checkpoint, save_checkpoint, save_model
    torch.manual_seed(0)
    m = DataParallel(Net())
    opt = FlatSGD(m, lr=0.1, momentum=0.9)
    x, y = torch.randn(4, 3, 32, 32), torch.randint(0, 10, (4,))
    for _ in range(2):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    p = save_model(m, str(tmp_path / "model"))
    sd = torch.load(p, weights_only=True)
    assert next(iter(sd)).startswith("module.") and all(not k.startswith("tmp") for k in os.listdir(tmp_path / "model"))
    c = save_checkpoint(str(tmp_path / "ck.pt"), m, opt, step=7, epoch=1)
    torch.manual_seed(1)
    m2 = DataParallel(Net())
    opt2 = FlatSGD(m2, lr=0.1, momentum=0.9)
    info = load_checkpoint(c, m2, opt2)
    assert info["step"] == 7 and info["epoch"] == 1 and opt2.steps == 2
    assert torch.equal(m2.flat.data, m.flat.data) and torch.equal(opt2.momentum_buf, opt.momentum_buf)
