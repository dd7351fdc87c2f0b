"""torchvision.utils.make_grid (used by the workshop's notebook-1 prediction cell)."""
import math

import torch


def make_grid(tensor, nrow=8, padding=2, normalize=False, value_range=None, scale_each=False, pad_value=0.0):
    if isinstance(tensor, (list, tuple)):
        tensor = torch.stack(tensor, dim=0)
    if tensor.dim() == 2:
        tensor = tensor.unsqueeze(0)
    if tensor.dim() == 3:
        tensor = tensor.unsqueeze(0)
    if tensor.size(1) == 1:
        tensor = torch.cat((tensor, tensor, tensor), 1)
    tensor = tensor.clone()
    if normalize:
        lo, hi = value_range if value_range is not None else (float(tensor.min()), float(tensor.max()))
        tensor.clamp_(min=lo, max=hi).sub_(lo).div_(max(hi - lo, 1e-5))
    n = tensor.size(0)
    xmaps = min(nrow, n)
    ymaps = int(math.ceil(float(n) / xmaps))
    h, w = int(tensor.size(2) + padding), int(tensor.size(3) + padding)
    grid = tensor.new_full((tensor.size(1), h * ymaps + padding, w * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= n:
                break
            grid.narrow(1, y * h + padding, h - padding).narrow(2, x * w + padding, w - padding).copy_(tensor[k])
            k += 1
    return grid
