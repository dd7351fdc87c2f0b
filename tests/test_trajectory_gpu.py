"""Training-trajectory parity: the engine's loss curve (native bf16 kernels, flat-buffer DP,
fused FlatSGD) tracks stock PyTorch fp32 training from the same init on the same batch
(tools/loss_parity.py; the ResNet-50 curves are in profiles/loss_parity_rn50.md)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_training_trajectory_matches_stock_fp32():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import loss_parity
    ours, ref, _ = loss_parity.run("resnet18", batch=32, size=64, classes=10, steps=12, lr=0.02)
    for i, (o, r) in enumerate(zip(ours, ref)):
        assert abs(o - r) <= 0.05 * abs(r) + 0.02, (i, ours, ref)
    assert ours[-1] < 0.7 * ours[0], ours  # it learns the batch


def test_reference_shape_trajectory_matches_stock_fp32():
    """the reference's own shape (ResNet-18, 1000-class head, 32x32,
    batch 32, lr 0.01, momentum 0.9) for 150 steps of fresh learnable batches, through the
    engine-backed DDP + stock SGD (graphed after two eager steps), against stock PyTorch fp32 on
    the same GPU, averaged over 3 (init, data) seeds: every 10-step window of the mean loss curves
    within 12 %, and both learn."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ref_trajectory
    ours, ref, graphed = ref_trajectory.run_seeds(150, seeds=(1, 2, 3))
    assert graphed == [148, 148, 148]
    wo, wr = ref_trajectory.windows(ours), ref_trajectory.windows(ref)
    msg = "ours " + " ".join(f"{v:.3f}" for v in wo) + " | fp32 " + " ".join(f"{v:.3f}" for v in wr)
    for i, (o, r) in enumerate(zip(wo, wr)):
        assert abs(o - r) <= 0.12 * r + 0.01, (i, msg)
    mean_rel = sum(abs(o - r) / r for o, r in zip(wo, wr)) / len(wo)
    assert mean_rel <= 0.05, (mean_rel, msg)
    assert wo[-1] < 0.75 * wo[0] and wr[-1] < 0.75 * wr[0], msg


def test_reference_shape_trajectory_fp32_mode_matches_stock_fp32():
    """the engine in its fp32 compute mode (MI355X_DP_COMPUTE_DTYPE=fp32: fp32 MFMA
    kernels, exact fp32) against stock fp32 PyTorch over the same 150 reference-shape steps, averaged
    over 3 seeds: every 10-step window of the mean loss curves within 8 %.  Two fp32
    implementations that differ only in summation order already diverge by up to ~5 % in the
    mid-run windows of 150 SGD steps (window 3: 2.489 vs 2.365, raw/r5/t_traj_fp32.log) -- the
    chaos that also sets the bf16 test's 12 % band, not precision."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ref_trajectory
    ours, ref, graphed = ref_trajectory.run_seeds(150, seeds=(1, 2, 3), fp32=True)
    assert graphed == [148, 148, 148]
    wo, wr = ref_trajectory.windows(ours), ref_trajectory.windows(ref)
    msg = "ours(fp32) " + " ".join(f"{v:.3f}" for v in wo) + " | stock fp32 " + " ".join(f"{v:.3f}" for v in wr)
    for i, (o, r) in enumerate(zip(wo, wr)):
        assert abs(o - r) <= 0.08 * r + 0.01, (i, msg)
    assert wo[-1] < 0.75 * wo[0], msg
    print(msg)
