"""Serving handler for the LeNet model written by examples/train_cifar10_cpu.py (notebook-1
deployment): only `model_fn` is user code, input/predict/output are the toolkit defaults."""
import os

import torch

from mi355x_dp.models.lenet import Net


def model_fn(model_dir):
    model = Net()
    model.load_state_dict(torch.load(os.path.join(model_dir, "model.pth"), map_location="cpu", weights_only=True))
    return model.eval()
