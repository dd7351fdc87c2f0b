"""GPU integration: smoke entry point, smddp native backend (world 1), the reference GPU
script run UNMODIFIED through the local estimator, checkpoint layout of its model.pth."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

def _ref_notebooks():
    """The reference workshop's notebooks dir: $MI355X_DP_REF_NOTEBOOKS, the read-only checkout,
    or the git-ignored copy build() stages into ref_fixture/ (what a GPU box has)."""
    for d in (os.environ.get("MI355X_DP_REF_NOTEBOOKS"), "/root/reference/notebooks",
              os.path.join(ROOT, "ref_fixture", "notebooks")):
        if d and os.path.exists(os.path.join(d, "code", "cifar10-distributed-smddp-gpu.py")):
            return d
    return None


REF_NB = _ref_notebooks()
REF_CODE = os.path.join(REF_NB, "code") if REF_NB else None


def test_graft_smoke():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    g.smoke()


def test_smddp_backend_world1(tmp_path):
    script = tmp_path / "s.py"
    script.write_text(
        "import os, torch, torch.distributed as dist\n"
        "import smdistributed.dataparallel.torch.torch_smddp\n"
        "dist.init_process_group(backend='smddp')\n"
        "pg = dist.distributed_c10d._get_default_group()\n"
        "t = torch.full((1000,), 3.0, device='cuda')\n"
        "w = dist.all_reduce(t, async_op=True); w.wait()\n"
        "assert torch.allclose(t, torch.full_like(t, 3.0))\n"
        "o = [torch.empty(10, device='cuda')]; dist.all_gather(o, torch.arange(10., device='cuda'))\n"
        "assert torch.equal(o[0], torch.arange(10., device='cuda'))\n"
        "dist.broadcast(t, 0); dist.barrier()\n"
        "b = pg._get_backend(torch.device('cuda'))\n"
        "print('BACKEND', type(b).__name__, b.name() if hasattr(b,'name') else '')\n"
        "m = torch.nn.parallel.DistributedDataParallel(torch.nn.Linear(8, 4).cuda())\n"
        "m(torch.randn(2, 8, device='cuda')).sum().backward()\n"
        "print('OK')\n")
    from mi355x_dp.launch import launch
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "1", str(script)], cwd=ROOT,
                       capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


@pytest.mark.skipif(REF_CODE is None, reason="reference scripts not staged (run build())")
def test_reference_gpu_script_unmodified(tmp_path):
    """notebook-2 flow: PyTorch(distribution=smddp).fit() runs cifar10-distributed-smddp-gpu.py as-is."""
    code = (
        "import sys, os\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.append({os.path.join(ROOT, 'compat')!r})\n"
        "from mi355x_dp.data.cifar import write_synthetic_cifar10\n"
        "write_synthetic_cifar10('data', n_train=2048, n_test=512)\n"
        "from sagemaker.pytorch import PyTorch\n"
        "est = PyTorch(entry_point='cifar10-distributed-smddp-gpu.py', source_dir=%r, role='r',\n"
        "              instance_count=1, instance_type='ml.p4d.24xlarge', framework_version='1.11.0', py_version='py38',\n"
        "              hyperparameters={'epochs': 2, 'lr': 0.01, 'momentum': 0.9, 'batch-size': 256,\n"
        "                               'model-type': 'resnet18', 'backend': 'smddp'},\n"
        "              distribution={'smdistributed': {'dataparallel': {'enabled': True}}},\n"
        "              output_path=os.path.abspath('out'))\n"
        "est.fit({'train': os.path.abspath('data')}, job_name='gpu-job')\n"
        "print('MODEL_DATA', est.model_data)\n" % REF_CODE)
    env = {**os.environ, "MI355X_DP_S3_ROOT": str(tmp_path / "s3"), "MI355X_DP_JOBS_ROOT": str(tmp_path / "jobs"),
           "MI355X_DP_NPROC": "1"}
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True, timeout=900,
                       env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "Initialized the distributed environment: 'smddp' backend on 1 nodes." in out
    assert "Test set: Average loss:" in out
    assert "Training seconds:" in out
    import tarfile
    tar = [l.split()[1] for l in r.stdout.splitlines() if l.startswith("MODEL_DATA")][0]
    with tarfile.open(tar) as tf:
        tf.extract("model.pth", path=tmp_path)
    sd = torch.load(tmp_path / "model.pth", map_location="cpu", weights_only=True)
    keys = list(sd.keys())
    assert keys[0] == "module.conv1.weight" and "module.fc.weight" in sd
    assert sd["module.fc.weight"].shape == (1000, 512)
    assert all(v.is_contiguous() for v in sd.values())
    assert sum(v.numel() for k, v in sd.items() if "running" not in k and "num_batches" not in k) == 11689512


def _run_reference_script(tmp_path, tag, engine, batch=32, epochs=1):
    """the unmodified reference GPU script, directly, with the env a one-rank job would set"""
    from mi355x_dp.data.cifar import write_synthetic_cifar10
    data = tmp_path / "data"
    if not data.exists():
        write_synthetic_cifar10(str(data), n_train=1024, n_test=256)
    model_dir = tmp_path / f"model_{tag}"
    model_dir.mkdir()
    env = {**os.environ, "SM_HOSTS": '["algo-1"]', "SM_CURRENT_HOST": "algo-1", "SM_MODEL_DIR": str(model_dir),
           "SM_CHANNEL_TRAIN": str(data), "LOCAL_RANK": "0", "RANK": "0", "WORLD_SIZE": "1",
           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(29600 + int(engine)),
           "PYTHONPATH": ROOT + os.pathsep + os.path.join(ROOT, "compat"), "MI355X_DP_ENGINE_DDP": str(int(engine))}
    code = ("import runpy, sys, torch\n"
            "orig = torch.nn.parallel.DistributedDataParallel\n"
            f"sys.argv = [{os.path.join(REF_CODE, 'cifar10-distributed-smddp-gpu.py')!r}, '--backend', 'smddp', "
            f"'--batch-size', '{batch}', '--epochs', '{epochs}', '--lr', '0.01', '--model-type', 'resnet18', "
            "'--momentum', '0.9']\n"
            "import smdistributed.dataparallel.torch.torch_smddp\n"
            "print('DDP_CLASS', torch.nn.parallel.DistributedDataParallel.__module__)\n"
            "runpy.run_path(sys.argv[0], run_name='__main__')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    return r.stdout, torch.load(model_dir / "model.pth", map_location="cpu", weights_only=True)


@pytest.mark.skipif(REF_CODE is None, reason="reference scripts not staged")
def test_reference_script_engine_ddp_matches_stock_ddp(tmp_path):
    """SURVEY §7.1 decision 2(b): with the torch_smddp shim the unmodified script's
    torch.nn.parallel.DistributedDataParallel(model) is the flat-buffer engine (gradients written
    by the backward kernels into one buffer, no DDP copy-in/out, bf16 copies refreshed once per
    step) driven by the script's own stock optim.SGD.  One epoch at the reference's per-rank batch
    (32) gives the same model.pth -- keys, layout, values (bitwise) -- as torch's stock DDP."""
    out_e, sd_e = _run_reference_script(tmp_path, "engine", True)
    out_s, sd_s = _run_reference_script(tmp_path, "stock", False)
    assert "mi355x_dp.parallel.engine_ddp" in out_e and "Test set: Average loss:" in out_e
    assert list(sd_e) == list(sd_s) and list(sd_e)[0] == "module.conv1.weight"
    assert all(v.is_contiguous() for v in sd_e.values())
    for k in sd_s:
        a, b = sd_e[k].double(), sd_s[k].double()
        if k.endswith("num_batches_tracked"):
            assert torch.equal(a, b), k
            continue
        err = float((a - b).norm() / b.norm().clamp_min(1e-12))
        # the native ResNet kernels are deterministic (no fp32 atomics), and the engine computes
        # exactly what stock DDP + SGD compute: 32 steps stay bit-identical (this configuration is
        # chaotic -- any nondeterminism would show as O(1) differences, tests/test_determinism_gpu.py)
        assert err == 0.0, (k, err)


def test_two_ranks_one_gpu_gloo(tmp_path):
    """Multi-rank GPU engine path without a second GPU: 2 ranks share cuda:0 over gloo (CUDA
    tensors), exercising DataParallel + native reducer bucket launches + FlatSGD on device;
    replicas must stay bit-identical and match each other's losses."""
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "dist.init_process_group('gloo')\n"
        "rank = dist.get_rank()\n"
        "torch.cuda.set_device(0)\n"
        "from mi355x_dp.models import get_model\n"
        "from mi355x_dp.ops import augment, cross_entropy, checksum\n"
        "from mi355x_dp.parallel import DataParallel, FlatSGD\n"
        "torch.manual_seed(rank)  # different init per rank: the engine must broadcast rank 0's\n"
        "eng = DataParallel(get_model('resnet18', num_classes=10).cuda(), bucket_cap_mb=8)\n"
        "assert eng.native_reducer and len(eng.buckets) > 2\n"
        "opt = FlatSGD(eng, lr=0.02, momentum=0.9)\n"
        "g = torch.Generator(device='cuda').manual_seed(100 + rank)\n"
        "u8 = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, device='cuda', generator=g)\n"
        "y = torch.randint(0, 10, (16,), device='cuda', generator=g)\n"
        "for i in range(3):\n"
        "    x = augment(u8, 8, (0.5,0.5,0.5), (0.25,0.25,0.25), pad=4, seed=i)\n"
        "    eng.zero_grad(); cross_entropy(eng(x), y).backward(); opt.step()\n"
        "torch.cuda.synchronize()\n"
        "c = torch.tensor([checksum(eng.flat.data)], dtype=torch.float64)\n"
        "cs = [torch.zeros_like(c) for _ in range(2)]; dist.all_gather(cs, c)\n"
        "assert cs[0].item() == cs[1].item(), cs\n"
        "print('RANK_OK', rank, eng.comm_calls, flush=True)\n"
        "dist.destroy_process_group()\n")
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "2", str(script)], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("RANK_OK") == 2


def test_notebook2_flow_example(tmp_path):
    """examples/notebook2_flow.py: smddp estimator fit() of a workshop-style DDP script on the GPU,
    model.tar.gz with module.-prefixed torchvision keys, deploy() + predict()."""
    env = {**os.environ, "MI355X_DP_S3_ROOT": str(tmp_path / "s3"), "MI355X_DP_JOBS_ROOT": str(tmp_path / "jobs"),
           "MI355X_DP_NPROC": "1"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "notebook2_flow.py"), "--epochs", "1",
                        "--n-train", "2048", "--n-test", "500", "--workdir", str(tmp_path / "w")],
                       cwd=tmp_path, capture_output=True, text=True, timeout=900, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "Initialized the distributed environment: 'smddp' backend on 1 nodes." in out
    assert "Test set: Average loss:" in out and "Training seconds:" in out
    assert "PREDICT_SHAPE (4, 1000)" in out
    import tarfile
    tar = [l.split()[1] for l in r.stdout.splitlines() if l.startswith("MODEL_DATA")][0]
    with tarfile.open(tar) as tf:
        tf.extract("model.pth", path=tmp_path)
    sd = torch.load(tmp_path / "model.pth", map_location="cpu", weights_only=True)
    assert next(iter(sd)) == "module.conv1.weight" and sd["module.fc.weight"].shape == (1000, 512)


@pytest.mark.parametrize("oneshot_kb", ["256", "0"])
def test_smddp_ipc_oneshot_allreduce_two_ranks(tmp_path, oneshot_kb):
    """SURVEY N4 one-shot / two-shot IPC all-reduce in the native smddp backend: 2 ranks sharing
    cuda:0 (IPC handles opened by the peer process), many back-to-back calls (slot parity reuse),
    SUM and AVG, sizes up to the cap (vectorised and scalar two-shot paths); RCCL is never
    initialised on this path.  oneshot_kb=256: small sizes one-shot, 4 MB two-shot; 0: all two-shot."""
    script = tmp_path / "ipc.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.append({os.path.join(ROOT, 'compat')!r})\n"
        "import smdistributed.dataparallel.torch.torch_smddp\n"
        "dist.init_process_group(backend='smddp')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "for it in range(40):\n"
        "    n = [1, 7, 1000, 65536, 1 << 20, 999999][it % 6]\n"
        "    t = torch.arange(n, device='cuda', dtype=torch.float32) * (r + 1) + it\n"
        "    op = dist.ReduceOp.AVG if it % 2 else dist.ReduceOp.SUM\n"
        "    dist.all_reduce(t, op=op)\n"
        "    base = torch.arange(n, device='cuda', dtype=torch.float32)\n"
        "    ref = base * sum(q + 1 for q in range(w)) + it * w\n"
        "    if op == dist.ReduceOp.AVG: ref = ref / w\n"
        "    assert torch.allclose(t, ref, rtol=1e-6, atol=1e-3), (it, (t - ref).abs().max().item())\n"
        "torch.cuda.synchronize()\n"
        "print('IPC_OK', r, flush=True)\n")
    env = {**os.environ, "PYTHONPATH": ROOT, "MI355X_DP_SMDDP_IPC": "1", "MI355X_DP_SMDDP_DEVICE": "0",
           "MI355X_DP_SMDDP_IPC_ONESHOT_KB": oneshot_kb, "MI355X_DP_SMDDP_TERMINATE_TRACE": "1"}
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "2", str(script)], cwd=ROOT,
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("IPC_OK") == 2


def test_smddp_ipc_only_two_ranks(tmp_path):
    """IPC-only smddp (MI355X_DP_SMDDP_IPC_ONLY=1: no RCCL communicator): 2 ranks sharing cuda:0.
    fp32 SUM/AVG all-reduces far larger than the 1 MB slot (chunked two-shot), fp64 MAX, int64 SUM,
    fp32 MIN (generic one-shot), broadcasts of fp32 / odd-sized uint8 / int64 from either root, a
    barrier -- then the DP engine's bucketed ResNet-18 training over it with bit-identical replicas."""
    script = tmp_path / "ipc_only.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.append({os.path.join(ROOT, 'compat')!r})\n"
        "import smdistributed.dataparallel.torch.torch_smddp\n"
        "dist.init_process_group(backend='smddp')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "n = 3_000_001\n"
        "for op in (dist.ReduceOp.SUM, dist.ReduceOp.AVG):\n"
        "    t = torch.arange(n, device='cuda', dtype=torch.float32) * (r + 1)\n"
        "    dist.all_reduce(t, op=op)\n"
        "    ref = torch.arange(n, device='cuda', dtype=torch.float32) * 3 / (2 if op == dist.ReduceOp.AVG else 1)\n"
        "    assert torch.allclose(t, ref, rtol=1e-6), (op, (t - ref).abs().max().item())\n"
        "d = torch.tensor([1.5 + r, -r], device='cuda', dtype=torch.float64); dist.all_reduce(d, op=dist.ReduceOp.MAX)\n"
        "assert d.tolist() == [2.5, 0.0], d\n"
        "i = torch.full((300_001,), r + 1, device='cuda', dtype=torch.int64); dist.all_reduce(i)\n"
        "assert int(i.min()) == 3 and int(i.max()) == 3\n"
        "f = torch.full((5,), float(r), device='cuda'); dist.all_reduce(f, op=dist.ReduceOp.MIN)\n"
        "h = torch.full((700_001,), 1.5 + r, device='cuda', dtype=torch.bfloat16); dist.all_reduce(h)\n"
        "assert float(h.float().min()) == 4.0 and float(h.float().max()) == 4.0\n"
        "assert float(f.max()) == 0.0\n"
        "b = torch.arange(2_000_003, device='cuda', dtype=torch.float32) * (r + 7); dist.broadcast(b, 1)\n"
        "assert torch.equal(b, torch.arange(2_000_003, device='cuda', dtype=torch.float32) * 8)\n"
        "u = torch.full((1001,), 10 + r, device='cuda', dtype=torch.uint8); dist.broadcast(u, 0)\n"
        "assert int(u.min()) == 10 and int(u.max()) == 10\n"
        "l = torch.tensor([r * 100 + 1], device='cuda', dtype=torch.int64); dist.broadcast(l, 1)\n"
        "assert int(l) == 101\n"
        "dist.barrier()\n"
        "from mi355x_dp.models import resnet18\n"
        "from mi355x_dp.ops import cross_entropy\n"
        "from mi355x_dp.parallel import DataParallel, FlatSGD\n"
        "from mi355x_dp.parallel.health import ReplicaChecker\n"
        "torch.manual_seed(r)\n"
        "eng = DataParallel(resnet18(num_classes=10).cuda(), bucket_cap_mb=8, min_bucket_mb=0, grad_comm='bf16')\n"
        "opt = FlatSGD(eng, lr=0.05, momentum=0.9)\n"
        "g = torch.Generator(device='cuda').manual_seed(r)\n"
        "for _ in range(3):\n"
        "    x = torch.randn(16, 3, 32, 32, device='cuda', generator=g); y = torch.randint(0, 10, (16,), device='cuda', generator=g)\n"
        "    eng.zero_grad(); cross_entropy(eng(x), y).backward(); opt.step()\n"
        "assert ReplicaChecker(eng)(force=True)\n"
        "assert eng.comm_calls >= 3 * len(eng.buckets), eng.comm_calls\n"
        "torch.cuda.synchronize()\n"
        "print('IPC_ONLY_OK', r, len(eng.buckets), flush=True)\n"
        "dist.destroy_process_group()\n")
    env = {**os.environ, "PYTHONPATH": ROOT, "MI355X_DP_SMDDP_IPC_ONLY": "1", "MI355X_DP_SMDDP_DEVICE": "0",
           "MI355X_DP_SMDDP_IPC_MB": "1", "MI355X_DP_SMDDP_TERMINATE_TRACE": "1"}
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "2", str(script)], cwd=ROOT,
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("IPC_ONLY_OK") == 2


def test_smddp_ipc_balanced_shards_two_ranks(tmp_path):
    """Balanced shards over the xGMI mesh (IPC-only smddp, 2 ranks sharing cuda:0): reduce-scatter
    (fp32 SUM / AVG, bf16, in place and out of place, sizes far beyond the 1 MB slot: chunked) and
    all-gather (fp32, bf16, odd byte counts) against exact references; then ResNet-18 trained with
    DataParallel(shard_optimizer=True) -- reduce-scatter buckets, shard-local SGD, all-gather params
    -- ends bit-identical across ranks, and its first update equals the all-reduce engine's (later
    steps are compared only for replica identity: the stem weight gradient sums with fp32 atomics,
    and at 8 images per rank through 17 training-mode BNs a flipped bf16 rounding of one weight
    moves the loss by ~1e-3 within two steps, in either engine, run to run)."""
    script = tmp_path / "ipc_shard.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        f"sys.path.insert(0, {ROOT!r}); sys.path.append({os.path.join(ROOT, 'compat')!r})\n"
        "import smdistributed.dataparallel.torch.torch_smddp\n"
        "dist.init_process_group(backend='smddp')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "for S in (1, 1000, 700_001):\n"
        "    base = torch.arange(w * S, device='cuda', dtype=torch.float32)\n"
        "    for op in (dist.ReduceOp.SUM, dist.ReduceOp.AVG):\n"
        "        x = base * (r + 1)\n"
        "        out = torch.empty(S, device='cuda')\n"
        "        dist.reduce_scatter_tensor(out, x, op=op)\n"
        "        ref = base[r * S:(r + 1) * S] * 3 / (2 if op == dist.ReduceOp.AVG else 1)\n"
        "        assert torch.equal(out, ref), (S, op, (out - ref).abs().max().item())\n"
        "    x = base * (r + 1)\n"
        "    dist.reduce_scatter_tensor(x[r * S:(r + 1) * S], x)  # in place (the engine's form)\n"
        "    assert torch.equal(x[r * S:(r + 1) * S], base[r * S:(r + 1) * S] * 3)\n"
        "    h = torch.full((w * S,), 1.5 + r, device='cuda', dtype=torch.bfloat16)\n"
        "    ho = torch.empty(S, device='cuda', dtype=torch.bfloat16); dist.reduce_scatter_tensor(ho, h)\n"
        "    assert float(ho.float().min()) == 4.0 and float(ho.float().max()) == 4.0\n"
        "    g = torch.zeros(w * S, device='cuda'); g[r * S:(r + 1) * S] = base[r * S:(r + 1) * S] + 0.5\n"
        "    dist.all_gather_into_tensor(g, g[r * S:(r + 1) * S])\n"
        "    assert torch.equal(g, base + 0.5)\n"
        "    gb = torch.empty(w * S, device='cuda', dtype=torch.bfloat16)\n"
        "    dist.all_gather_into_tensor(gb, torch.full((S,), float(r + 1), device='cuda', dtype=torch.bfloat16))\n"
        "    assert torch.equal(gb.float(), torch.arange(w, device='cuda').float().repeat_interleave(S) + 1)\n"
        "u = torch.empty(w * 3, device='cuda', dtype=torch.uint8)\n"
        "dist.all_gather_into_tensor(u, torch.full((3,), 7 + r, device='cuda', dtype=torch.uint8))\n"
        "assert u.tolist() == [7] * 3 + [8] * 3, u.tolist()\n"
        "from mi355x_dp.models import resnet18\n"
        "from mi355x_dp.ops import cross_entropy\n"
        "from mi355x_dp.parallel import DataParallel, FlatSGD\n"
        "from mi355x_dp.parallel.health import ReplicaChecker\n"
        "res = {}\n"
        "for shard in (False, True):\n"
        "    torch.manual_seed(0)\n"
        "    eng = DataParallel(resnet18(num_classes=10).cuda(), bucket_cap_mb=8, min_bucket_mb=0, shard_optimizer=shard)\n"
        "    opt = FlatSGD(eng, lr=0.05, momentum=0.9, weight_decay=1e-4)\n"
        "    g = torch.Generator(device='cuda').manual_seed(r)\n"
        "    for it in range(3):\n"
        "        x = torch.randn(16, 3, 32, 32, device='cuda', generator=g); y = torch.randint(0, 10, (16,), device='cuda', generator=g)\n"
        "        eng.zero_grad(); cross_entropy(eng(x), y).backward(); opt.step()\n"
        "        if it == 0: res[shard] = {k: v.clone() for k, v in eng.state_dict().items()}\n"
        "    assert ReplicaChecker(eng)(force=True)\n"
        "    if shard: assert opt.momentum_buf.numel() * w == eng.flat.numel\n"
        "for k, v in res[False].items():\n"
        "    d = (res[True][k].float() - v.float()).abs().max().item()\n"
        "    assert d <= 1e-6, (k, d)\n"
        "torch.cuda.synchronize()\n"
        "print('IPC_SHARD_OK', r, flush=True)\n"
        "dist.destroy_process_group()\n")
    env = {**os.environ, "PYTHONPATH": ROOT, "MI355X_DP_SMDDP_IPC_ONLY": "1", "MI355X_DP_SMDDP_DEVICE": "0",
           "MI355X_DP_SMDDP_IPC_MB": "1", "MI355X_DP_SMDDP_TERMINATE_TRACE": "1"}
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "2", str(script)], cwd=ROOT,
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("IPC_SHARD_OK") == 2


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "mi355x_dp", "_native", "libmi355x_kernels_debug.so")),
                    reason="debug kernel library not built (python -m mi355x_dp.build kernels --debug)")
def test_debug_kernels_training_step_clean(tmp_path):
    """the -DMI_DEBUG kernel build (device bounds asserts) with per-call synchronous
    error checking runs a fused ResNet training step + ViT layer without tripping an assert."""
    code = (
        f"import sys; sys.path.insert(0, {ROOT!r})\n"
        "import torch\n"
        "from mi355x_dp.models import get_model\n"
        "from mi355x_dp.ops import cross_entropy, _lib\n"
        "assert _lib.KERNEL_LIB.endswith('_debug.so') and _lib.SYNC_CHECK\n"
        "for name, size in (('resnet50', 64), ('resnet18', 32)):\n"
        "    m = get_model(name, num_classes=10).cuda()\n"
        "    x = torch.randn(4, 3, size, size, device='cuda'); y = torch.randint(0, 10, (4,), device='cuda')\n"
        "    cross_entropy(m(x), y).backward()\n"
        "from mi355x_dp.models.vit import VisionTransformer\n"
        "v = VisionTransformer(image_size=32, patch_size=16, num_layers=1, num_heads=2, hidden_dim=128, mlp_dim=256,\n"
        "                      num_classes=10).cuda()\n"
        "v(torch.randn(2, 3, 32, 32, device='cuda')).float().sum().backward()\n"
        "torch.cuda.synchronize(); print('DEBUG_OK')\n")
    env = {**os.environ, "MI355X_DP_DEBUG_KERNELS": "1", "MI355X_DP_SYNC_CHECK": "1"}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "DEBUG_OK" in r.stdout, (r.stdout + r.stderr)[-3000:]


def test_bench_two_ranks_torchrun_gloo():
    """bench.py under the driver's exact launcher shape (torch.distributed.run, 127.0.0.1, N=2) on
    one GPU: 2 gloo ranks share cuda:0; rank 0 prints ONE JSON line with the whole-job value."""
    import json
    port = 29500 + (os.getpid() % 2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--backend", "gloo", "--model", "resnet18", "--image-size", "32", "--batch", "32", "--num-classes", "10"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 64 and out["value"] > 0
    assert out["replicas_identical"] is True
    probe = out["comm_probe"]  # post-timing fabric probe (gloo here: list of rows, or the failure text)
    assert probe is not None
    if isinstance(probe, list):
        assert all(row["allreduce_ms"] > 0 for row in probe)


@pytest.mark.skipif(REF_NB is None, reason="reference notebooks not staged (run build())")
def test_reference_notebook2_verbatim(tmp_path):
    """The reference's OWN notebook 2 (2_pytorch_dist_smddp_gpu.ipynb), every code cell verbatim:
    synthetic 'download' of full-size CIFAR-10 (50k/10k) -> upload -> PyTorch(distribution=smddp)
    .fit() of the unmodified cifar10-distributed-smddp-gpu.py with the notebook's hyperparameters
    (15 epochs, global batch 256, resnet18, smddp) on every local MI355X.  BASELINE.md rows 1-2:
    438 s job / ~166 s loop on 8 x A100."""
    import json
    import re
    report = tmp_path / "nb2.json"
    env = {**os.environ, "MI355X_DP_S3_ROOT": str(tmp_path / "s3"), "MI355X_DP_JOBS_ROOT": str(tmp_path / "jobs")}
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "run_notebook.py"), "--compat",
                        "--workdir", str(tmp_path / "nb"), "--report", str(report),
                        os.path.join(REF_NB, "2_pytorch_dist_smddp_gpu.ipynb")],
                       capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    cells = json.load(open(report))["cells"]
    assert all(c["status"] == "ok" for c in cells), cells
    assert "Initialized the distributed environment: 'smddp' backend on" in out
    accs = [float(a) for a in re.findall(r"Test set: Average loss: -?[\d.]+, Accuracy: ([\d.]+)", out)]
    assert len(accs) >= 15
    assert accs[-1] > 0.3  # learned something (synthetic data; Bayes accuracy ~0.78)
    secs = int(re.search(r"Training seconds: (\d+)", out).group(1))
    assert secs < 438, f"job slower than the reference's 8xA100 438 s: {secs}"


@pytest.mark.parametrize("world", [2, 4])
def test_smddp_ipc_mesh_collectives_multi_rank(world):
    """IPC mesh reduce-scatter / all-gather / chunked all-reduce at world 2 and 4 (ranks sharing
    cuda:0, one hardware queue each), every rank against exact references (tools/ipc_mesh_check.py)."""
    env = {**os.environ, "PYTHONPATH": ROOT, "MI355X_DP_SMDDP_IPC_ONLY": "1", "MI355X_DP_SMDDP_DEVICE": "0",
           "MI355X_DP_SMDDP_IPC_MB": "1", "GPU_MAX_HW_QUEUES": "1"}
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", str(world),
                        os.path.join(ROOT, "tools", "ipc_mesh_check.py")], cwd=ROOT, capture_output=True, text=True,
                       timeout=150, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("MESH_OK") == world


def _graphed_world2(extra_env):
    import json
    env = {**os.environ, "PYTHONPATH": ROOT, "MI355X_DP_SMDDP_IPC_ONLY": "1", "MI355X_DP_SMDDP_DEVICE": "0",
           "MI355X_DP_SMDDP_IPC_MB": "4", "MI355X_DP_SMDDP_TERMINATE_TRACE": "1", **extra_env}
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "2",
                        os.path.join(ROOT, "tools", "graphed_world2.py")], cwd=ROOT, capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.loads(l[l.index("{"):]) for l in r.stdout.splitlines() if '"rank"' in l]
    assert len(rows) == 2, r.stdout[-2000:]
    return rows


def test_graphed_engine_two_ranks_gated_buckets():
    """The graphed engine at world 2: the reference loop (ResNet-18,
    1000-class head, stock SGD) through the engine-backed DDP, graphed vs eager on IPC-only smddp
    (2 ranks sharing cuda:0).  At the reference's shape (batch 32 at 32x32): graphed == eager bit
    for bit on every rank (losses and flat fp32 parameters), replicas identical, one gate per
    bucket.  At batch 256 at 224x224: every bucket's collective released by its gate, in order, the
    first one while the replayed backward is still running."""
    rows = _graphed_world2({})
    for row in rows:
        assert row["gated"] and row["comm_modes"] == ["gates"], row  # IPC collectives are never captured
        assert row["replays"] == 6 and row["replays_eager"] == 0, row
        assert row["losses_graphed"] == row["losses_eager"], row
        assert row["graphed_equals_eager"] and row["replicas_identical"], row
        assert len(row["gate_open_ms"]) == row["buckets"] >= 2, row
    assert rows[0]["losses_graphed"] != rows[1]["losses_graphed"]  # different data per rank
    # Gate trace at a larger shape (batch 256 at 224x224, graphed up to 64M input elements): every
    # bucket's gate fires once per replay, in bucket order, and bucket 0's gate opens BEFORE the
    # replayed backward ends.  This is structural since round 5: every gate (and the collective
    # behind it) is enqueued before the replay is launched, on a high-priority stream (its own
    # hardware-queue pool), so it no longer depends on when the host returns from the launch (the
    # round-4 schedule enqueued the gates after it: gate 0 at 7.29 ms of a 6.68 ms replay once).
    # (without the BN-buffer broadcast: its IPC kernel waits for the peer process, which time-slices
    # the same GPU and can lag by milliseconds, and it sits in front of the first gate on the comm
    # stream -- one such run opened gate 0 at 9.5 ms of a 5.5 ms replay)
    rows = _graphed_world2({"GRAPHED_BATCH": "256", "GRAPHED_SIZE": "224", "GRAPHED_BCAST": "0",
                            "MI355X_DP_ENGINE_GRAPH_MAX_NUMEL": str(1 << 26), "GPU_MAX_HW_QUEUES": "6"})
    for row in rows:
        assert row["gated"] and row["replays"] == 6 and row["replicas_identical"], row
        opened, end = row["gate_open_ms"], row["replay_end_ms"]
        assert len(opened) == row["buckets"] >= 2 and opened == sorted(opened) and end > 0, row
        assert opened[0] < end, row  # bucket 0's collective released under the replayed backward
        print(f"rank {row['rank']}: gates opened at {[round(t, 2) for t in opened]} ms, replay ended at "
              f"{end:.2f} ms")


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs one device per rank (>= 2 GPUs)")
@pytest.mark.parametrize("backend", ["nccl", "smddp"])
def test_graphed_engine_two_ranks_captured_rccl(backend):
    """the default graphed comm mode, 'capture' (bucket all-reduces, the BN-buffer
    broadcast, the join and the 1/world scaling recorded INTO the backward graph), at world 2 over
    RCCL on two devices -- torch nccl and the native smddp backend on its RCCL path: graphed == eager
    bit for bit (losses and flat fp32 parameters) and identical replicas."""
    import json
    env = {**os.environ, "PYTHONPATH": ROOT, "GRAPHED_BACKEND": backend, "MI355X_DP_SMDDP_IPC_ONLY": "0",
           "MI355X_DP_SMDDP_IPC": "0"}
    env.pop("MI355X_DP_SMDDP_DEVICE", None)
    r = subprocess.run([sys.executable, "-m", "mi355x_dp.launch", "--nproc", "2",
                        os.path.join(ROOT, "tools", "graphed_world2.py")], cwd=ROOT, capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.loads(l[l.index("{"):]) for l in r.stdout.splitlines() if '"rank"' in l]
    assert len(rows) == 2, r.stdout[-2000:]
    for row in rows:
        assert row["comm_modes"] == ["capture"], row
        assert row["replays"] == 6 and row["replays_eager"] == 0, row
        assert row["losses_graphed"] == row["losses_eager"], row
        assert row["graphed_equals_eager"] and row["replicas_identical"], row
    assert rows[0]["losses_graphed"] != rows[1]["losses_graphed"]


@pytest.mark.skipif(REF_CODE is None, reason="reference scripts not staged (run build())")
def test_reference_job_per_gpu_shape():
    """tools/reference_job.py: the unmodified reference script as a local job at the reference's
    per-GPU batch (32), one epoch, through the engine-backed DDP with graphed steps -- faster than
    the reference's own per-A100 throughput (>= 565 img/s) by a wide margin."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "reference_job.py"), "--batch-size", "32",
                        "--epochs", "1", "--tag", "test"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["loop_seconds"] and res["loop_seconds"] > 0
    assert res["img_per_s_lower_bound"] > 4 * 565, res
    assert res["final_accuracy"] is not None and res["final_accuracy"] > 0.3
