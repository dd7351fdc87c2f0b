"""Serving handler for a model trained by examples/train_cifar10_smddp.py: only `model_fn` is
user code; input/predict/output use the toolkit defaults (numpy payload -> model(x) -> numpy),
as in the workshop's notebook-1 deployment."""
import os

import torch
import torchvision


def model_fn(model_dir):
    model = torchvision.models.resnet18(num_classes=1000)
    sd = torch.load(os.path.join(model_dir, "model.pth"), map_location="cpu", weights_only=True)
    model.load_state_dict({k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()})
    return model.eval()
