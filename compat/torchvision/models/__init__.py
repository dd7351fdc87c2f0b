"""torchvision.models subset backed by mi355x_dp.models (same names/shapes/buffers)."""
from mi355x_dp.models.resnet import (  # noqa: F401
    ResNet, BasicBlock, Bottleneck, resnet18, resnet34, resnet50, resnet101, resnet152,
)


def vit_b_16(pretrained=False, progress=True, weights=None, **kwargs):
    from mi355x_dp.models.vit import vit_b_16 as _v
    if pretrained or weights is not None:
        raise RuntimeError("pretrained weights need network access; not available")
    return _v(**kwargs)
