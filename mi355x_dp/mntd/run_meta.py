"""Meta-classifier driver (reference notebooks/code/run_meta_cpu.py).

    python -m mi355x_dp.mntd.run_meta --task mnist --troj_type M [--no_qt] [--load_exist] [--gpu]

Train = shadow_{jumbo,benign}_0..15, val = 16..23, test = target_troj{M,B}_0..15 +
target_benign_0..15; N_REPEAT meta-classifiers x N_EPOCH; keep the best-val-AUC model
per repeat and report the mean test AUC ("Average detection AUC on %d meta classifier").
Checkpoints are resident in a CheckpointBank (no per-step torch.load).  Checkpoints
absent on disk (the reference ships target_trojM_9..26 only) are reported and dropped
from the split instead of crashing.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .meta import CheckpointBank, MetaClassifier, epoch_meta_eval, epoch_meta_train, load_model_setting


def splits(shadow_path, troj_type, train_num=16, val_num=8, test_num=16):
    train = [(f"{shadow_path}/shadow_{k}_{i}.model", y) for i in range(train_num)
             for k, y in (("jumbo", 1), ("benign", 0))]
    val = [(f"{shadow_path}/shadow_{k}_{i}.model", y) for i in range(train_num, train_num + val_num)
           for k, y in (("jumbo", 1), ("benign", 0))]
    test = [(f"{shadow_path}/target_{k}_{i}.model", y) for i in range(test_num)
            for k, y in ((f"troj{troj_type}", 1), ("benign", 0))]
    return train, val, test


def run(task, troj_type, no_qt=False, load_exist=False, gpu=False, n_repeat=15, n_epoch=15,
        shadow_root="./shadow_model_ckpt", ckpt_root="./meta_classifier_ckpt", test_offset=0, seed=None):
    if seed is not None:
        np.random.seed(seed)
        torch.manual_seed(seed)
    dev = torch.device("cuda" if gpu and torch.cuda.is_available() else "cpu")
    save_path = os.path.join(ckpt_root, f"{task}_no-qt.model" if no_qt else f"{task}.model")
    os.makedirs(ckpt_root, exist_ok=True)
    shadow_path = os.path.join(shadow_root, task, "models")
    Model, input_size, class_num, inp_mean, inp_std, is_discrete = load_model_setting(task)
    if inp_mean is not None:
        inp_mean = torch.tensor(inp_mean, dtype=torch.float32, device=dev)
        inp_std = torch.tensor(inp_std, dtype=torch.float32, device=dev)
    print("Task: %s; target Trojan type: %s; input size: %s; class num: %s" % (task, troj_type, input_size, class_num))
    train, val, test = splits(shadow_path, troj_type)
    if test_offset:
        test = [(p.replace(f"_{i}.model", f"_{i + test_offset}.model") if f"troj{troj_type}" in p else p, y)
                for (p, y), i in zip(test, [j for j in range(16) for _ in range(2)])]
    bank = CheckpointBank([train, val, test], device=dev)
    if bank.missing:
        print(f"[mntd] {len(bank.missing)} checkpoint(s) not found and skipped, e.g. {bank.missing[0]}")
    train, val, test = bank.filter(train), bank.filter(val), bank.filter(test)
    aucs = []
    for i in range(n_repeat):
        shadow_model = Model(gpu=gpu).to(dev)
        target_model = Model(gpu=gpu).to(dev)
        meta = MetaClassifier(input_size, class_num, gpu=gpu).to(dev)
        if inp_mean is not None:
            meta.inp.data = torch.zeros_like(meta.inp).normal_() * inp_std + inp_mean
        if not load_exist:
            print("Training Meta Classifier %d/%d" % (i + 1, n_repeat))
            params = list(meta.fc.parameters()) + list(meta.output.parameters()) if no_qt else meta.parameters()
            opt = torch.optim.Adam(params, lr=1e-3)
            best, test_info = None, None
            for _ in range(n_epoch):
                epoch_meta_train(meta, shadow_model, opt, train, is_discrete, threshold="half", bank=bank)
                _, val_auc, _ = epoch_meta_eval(meta, shadow_model, val, is_discrete, threshold="half", bank=bank)
                if best is None or val_auc > best:
                    best = val_auc
                    test_info = epoch_meta_eval(meta, target_model, test, is_discrete, threshold="half", bank=bank)
                    torch.save(meta.state_dict(), save_path + "_%d" % i)
        else:
            print("Evaluating Meta Classifier %d/%d" % (i + 1, n_repeat))
            meta.load_state_dict(torch.load(save_path + "_%d" % i, map_location=dev, weights_only=True))
            test_info = epoch_meta_eval(meta, target_model, test, is_discrete, threshold="half", bank=bank)
        print("\tTest AUC:", test_info[1])
        aucs.append(test_info[1])
    mean = sum(aucs) / len(aucs)
    print("Average detection AUC on %d meta classifier: %.4f" % (n_repeat, mean))
    return mean, aucs


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m mi355x_dp.mntd.run_meta")
    ap.add_argument("--task", required=True)
    ap.add_argument("--troj_type", required=True, choices=["M", "B"])
    ap.add_argument("--no_qt", action="store_true")
    ap.add_argument("--load_exist", action="store_true")
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--repeats", type=int, default=15)
    ap.add_argument("--epochs", type=int, default=15)
    ap.add_argument("--shadow-root", default="./shadow_model_ckpt")
    a = ap.parse_args(argv)
    run(a.task, a.troj_type, a.no_qt, a.load_exist, a.gpu, a.repeats, a.epochs, a.shadow_root)


if __name__ == "__main__":
    main()
