"""MNTD workflow: models vs shipped checkpoints, trojan stamping, backdoor
datasets, shadow generation (serial == task-parallel gloo world 2), meta-classifier training."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CKPT = "/root/reference/notebooks/code/shadow_model_ckpt"


def test_model_param_counts():
    from mi355x_dp.mntd import CIFARCNN, MNISTCNN
    assert sum(p.numel() for p in MNISTCNN().parameters()) == 281034
    assert sum(p.numel() for p in CIFARCNN().parameters()) == 1182762
    assert MNISTCNN()(torch.zeros(3, 1, 28, 28)).shape == (3, 10)
    assert CIFARCNN()(torch.zeros(2, 3, 32, 32)).shape == (2, 10)


def test_audio_and_text_models():
    from mi355x_dp.mntd import AudioRNN, RTNLPCNN, mel_filterbank
    fb = mel_filterbank(16000, 2048, 40)
    assert fb.shape == (40, 1025) and (fb >= 0).all()
    assert (fb.sum(1) > 0).all()  # every band covers some FFT bins
    a = AudioRNN()
    assert a(torch.randn(2, 16000)).shape == (2, 10)
    t = RTNLPCNN(emb=np.random.randn(100, 300).astype(np.float32))
    out = t(torch.randint(0, 100, (4, 12)))
    assert out.shape == (4,)
    assert t.loss(out, torch.tensor([0, 1, 1, 0])).item() > 0


@pytest.mark.skipif(not os.path.isdir(CKPT), reason="reference checkpoints not mounted")
def test_shipped_checkpoints_load_weights_only():
    from mi355x_dp.mntd import MNISTCNN
    d = os.path.join(CKPT, "mnist", "models")
    files = sorted(os.listdir(d))
    assert len(files) == 111
    m = MNISTCNN()
    for f in files[:5]:
        m.load_state_dict(torch.load(os.path.join(d, f), weights_only=True))


def test_trojan_stamp_and_backdoor_dataset():
    from mi355x_dp.mntd.data import BackdoorDataset
    from mi355x_dp.mntd.trojan import TROJ
    np.random.seed(0)
    setting, stamp = TROJ["mnist"]
    atk = setting("M")
    p, pattern, (lx, ly), alpha, target, inject = atk
    assert alpha == 1.0 and p in (2, 3, 4, 5)
    X = torch.zeros(1, 28, 28)
    Xn, y = stamp(X, 3, atk)
    assert y == target and torch.equal(Xn[0, lx:lx + p, ly:ly + p], torch.tensor(pattern, dtype=torch.float32))
    src = [(torch.rand(1, 28, 28), i % 10) for i in range(100)]
    ds = BackdoorDataset(src, atk, stamp, choice=np.arange(50))
    assert len(ds) == 50 + int(50 * inject)
    assert ds[len(ds) - 1][1] == target
    mal = BackdoorDataset(src, atk, stamp, mal_only=True)
    assert len(mal) == int(100 * inject) and all(mal[i][1] == target for i in range(len(mal)))
    cset, cstamp = TROJ["cifar10"]
    catk = cset("B")
    assert catk[0] == 32 and 0.05 <= catk[3] <= 0.2


@pytest.mark.skipif(not os.path.isdir(CKPT), reason="reference checkpoints not mounted")
def test_meta_classifier_on_shipped_checkpoints(tmp_path):
    from mi355x_dp.mntd.run_meta import run
    mean, aucs = run("mnist", "M", n_repeat=1, n_epoch=3, shadow_root=CKPT, ckpt_root=str(tmp_path), seed=0)
    assert len(aucs) == 1 and 0.0 <= mean <= 1.0
    assert os.path.exists(tmp_path / "mnist.model_0")
    # --load_exist path re-evaluates the saved meta-classifier
    mean2, _ = run("mnist", "M", load_exist=True, n_repeat=1, shadow_root=CKPT, ckpt_root=str(tmp_path))
    assert 0.0 <= mean2 <= 1.0


def test_one_class_meta():
    from mi355x_dp.mntd import MetaClassifierOC
    m = MetaClassifierOC((1, 28, 28), 10)
    s = m(torch.randn(10, 10))
    assert s.dim() == 0 and m.loss(s).dim() == 0
    m.update_r([0.1, 0.2, 0.3, 0.4])
    assert isinstance(m.r, float)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gen_worker(rank, world, port, root, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mi355x_dp.mntd.train import generate
    log = generate("mnist", "jumbo", shadow_num=3, n_epoch=1, save_root=os.path.join(root, "par"),
                   data_root=os.path.join(root, "data"), limit_train=300)
    q.put(log)
    dist.destroy_process_group()


def test_shadow_generation_serial_equals_task_parallel(tmp_path):
    from mi355x_dp.mntd.train import generate
    root = str(tmp_path)
    generate("mnist", "jumbo", shadow_num=3, n_epoch=1, save_root=os.path.join(root, "ser"),
             data_root=os.path.join(root, "data"), limit_train=300)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_gen_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in ps:
        p.start()
    logs = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
    assert logs[0]["n_models"] == 3
    for i in range(3):
        a = torch.load(os.path.join(root, "ser", "mnist", "models", f"shadow_jumbo_{i}.model"), weights_only=True)
        b = torch.load(os.path.join(root, "par", "mnist", "models", f"shadow_jumbo_{i}.model"), weights_only=True)
        for k in a:
            assert torch.allclose(a[k], b[k], atol=1e-6), (i, k)
    assert os.path.exists(os.path.join(root, "par", "mnist", "jumbo.log"))


@pytest.mark.skipif(not os.path.isdir(CKPT), reason="reference checkpoints not mounted")
def test_batched_meta_eval_matches_sequential():
    """The vmapped evaluation over the stacked checkpoint bank gives the per-model scores and losses
    of the reference's one-model-at-a-time loop (shipped MNIST checkpoints, both meta models)."""
    import mi355x_dp.mntd.meta as M
    from mi355x_dp.mntd import MNISTCNN
    d = os.path.join(CKPT, "mnist", "models")
    ds = [(os.path.join(d, f"shadow_jumbo_{i}.model"), 1) for i in range(6)] + \
         [(os.path.join(d, f"shadow_benign_{i}.model"), 0) for i in range(6)]
    bank = M.CheckpointBank([ds])
    torch.manual_seed(0)
    for meta in (M.MetaClassifier((1, 28, 28), 10), M.MetaClassifierOC((1, 28, 28), 10)):
        basic = MNISTCNN()
        p1, l1, loss1 = M._eval_scores_batched(meta, basic, ds, False, bank)
        M.BATCHED_EVAL = False
        try:
            p2, l2, loss2 = M._eval_scores(meta, basic, ds, False, bank)
        finally:
            M.BATCHED_EVAL = True
        assert np.allclose(p1, p2, rtol=1e-4, atol=1e-5), (p1, p2)
        assert (l1 == l2).all() and np.allclose(loss1, loss2, rtol=1e-4, atol=1e-6)


def test_batched_shadow_training_matches_serial(tmp_path):
    """mntd.batched: the generation drivers with batched=True (all of a rank's shadow models in one
    vmapped step, stacked Adam) give the serial loop's models -- same init, same per-model data
    order -- to fp32 rounding of the batched convolutions; also the trainer alone on models whose
    datasets (and so last-batch sizes) and epoch counts differ."""
    from mi355x_dp.mntd.batched import train_models_batched
    from mi355x_dp.mntd.models import MNISTCNN
    from mi355x_dp.mntd.train import generate
    root = str(tmp_path)
    for b in (False, True):
        generate("mnist", "jumbo", shadow_num=3, n_epoch=1, save_root=os.path.join(root, f"b{int(b)}"),
                 data_root=os.path.join(root, "data"), limit_train=300, batched=b)
    for i in range(3):
        a = torch.load(os.path.join(root, "b0", "mnist", "models", f"shadow_jumbo_{i}.model"), weights_only=True)
        b = torch.load(os.path.join(root, "b1", "mnist", "models", f"shadow_jumbo_{i}.model"), weights_only=True)
        for k in a:
            assert torch.allclose(a[k], b[k], atol=1e-4), (i, k, (a[k] - b[k]).abs().max())
    torch.manual_seed(0)
    data = [(torch.randn(40 + 10 * i, 1, 28, 28), torch.randint(0, 10, (40 + 10 * i,))) for i in range(3)]

    def loaders():
        return [torch.utils.data.DataLoader(torch.utils.data.TensorDataset(*d), batch_size=16, shuffle=True,
                                            generator=torch.Generator().manual_seed(5 + i)) for i, d in enumerate(data)]
    models, ref = [], []
    for i in range(3):
        torch.manual_seed(100 + i)
        models.append(MNISTCNN())
        torch.manual_seed(100 + i)
        ref.append(MNISTCNN())
    epochs = [2, 1, 2]
    train_models_batched(models, loaders(), epochs, False)
    for i, (m, l) in enumerate(zip(ref, loaders())):
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        for _ in range(epochs[i]):
            for x, y in l:
                loss = m.loss(m(x), y)
                opt.zero_grad()
                loss.backward()
                opt.step()
    for a, b in zip(models, ref):
        for pa, pb in zip(a.parameters(), b.parameters()):
            assert torch.allclose(pa, pb, atol=5e-5), (pa - pb).abs().max()
