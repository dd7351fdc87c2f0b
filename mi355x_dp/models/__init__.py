"""Model zoo: torchvision-compatible ResNets / ViT, the workshop's LeNet ``Net``,
and the MNTD (cloud-security) model family."""
from .resnet import ResNet, BasicBlock, Bottleneck, resnet18, resnet34, resnet50, resnet101, resnet152  # noqa: F401
from .lenet import Net  # noqa: F401

_REGISTRY = {
    "resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50, "resnet101": resnet101,
    "resnet152": resnet152, "net": Net,
}


def get_model(name: str, **kw):
    name = name.lower().replace("-", "").replace("_", "")
    if name == "vitb16":
        from .vit import vit_b_16
        return vit_b_16(**kw)
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name}; have {sorted(_REGISTRY)} + vit_b_16")
    return _REGISTRY[name](**kw)
