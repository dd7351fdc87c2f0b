"""torchvision.transforms subset (PIL images or CHW tensors), matching torchvision semantics
for what the workshop uses (reference cifar10-distributed-smddp-gpu.py:55-62, nb1:170-209)."""
import numbers


import numpy as np
import torch

try:
    from PIL import Image
except Exception:  # pragma: no cover
    Image = None


def _is_pil(img):
    return Image is not None and isinstance(img, Image.Image)


class Compose:
    def __init__(self, transforms):
        self.transforms = transforms

    def __call__(self, img):
        for t in self.transforms:
            img = t(img)
        return img

    def __repr__(self):
        return "Compose(" + ", ".join(repr(t) for t in self.transforms) + ")"


class ToTensor:
    """PIL / HWC uint8 ndarray -> float CHW in [0, 1]."""

    def __call__(self, pic):
        if isinstance(pic, torch.Tensor):
            return pic
        if _is_pil(pic):
            arr = np.asarray(pic, dtype=np.uint8)
        else:
            arr = np.asarray(pic)
        if arr.ndim == 2:
            arr = arr[:, :, None]
        t = torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))
        if t.dtype == torch.uint8:
            return t.float().div_(255.0)
        return t.float()

    def __repr__(self):
        return "ToTensor()"


class PILToTensor:
    def __call__(self, pic):
        arr = np.asarray(pic, dtype=np.uint8)
        if arr.ndim == 2:
            arr = arr[:, :, None]
        return torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))


class Normalize:
    def __init__(self, mean, std, inplace=False):
        self.mean, self.std, self.inplace = mean, std, inplace

    def __call__(self, t):
        if not self.inplace:
            t = t.clone()
        m = torch.as_tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
        s = torch.as_tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
        return t.sub_(m).div_(s)

    def __repr__(self):
        return f"Normalize(mean={self.mean}, std={self.std})"


def _size2(size):
    if isinstance(size, numbers.Number):
        return int(size), int(size)
    return tuple(size)


class RandomCrop:
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode="constant"):
        self.size = _size2(size)
        self.padding = padding
        self.fill = fill

    def __call__(self, img):
        th, tw = self.size
        if _is_pil(img):
            if self.padding:
                p = self.padding
                w, h = img.size
                canvas = Image.new(img.mode, (w + 2 * p, h + 2 * p), self.fill)
                canvas.paste(img, (p, p))
                img = canvas
            w, h = img.size
            i = int(torch.randint(0, h - th + 1, size=(1,)).item())
            j = int(torch.randint(0, w - tw + 1, size=(1,)).item())
            return img.crop((j, i, j + tw, i + th))
        t = img
        if self.padding:
            t = torch.nn.functional.pad(t, (self.padding,) * 4, value=self.fill)
        h, w = t.shape[-2:]
        i = int(torch.randint(0, h - th + 1, size=(1,)).item())
        j = int(torch.randint(0, w - tw + 1, size=(1,)).item())
        return t[..., i:i + th, j:j + tw]

    def __repr__(self):
        return f"RandomCrop(size={self.size}, padding={self.padding})"


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, img):
        if torch.rand(1).item() < self.p:
            if _is_pil(img):
                return img.transpose(Image.FLIP_LEFT_RIGHT)
            return img.flip(-1)
        return img

    def __repr__(self):
        return f"RandomHorizontalFlip(p={self.p})"


class CenterCrop:
    def __init__(self, size):
        self.size = _size2(size)

    def __call__(self, img):
        th, tw = self.size
        if _is_pil(img):
            w, h = img.size
            i, j = (h - th) // 2, (w - tw) // 2
            return img.crop((j, i, j + tw, i + th))
        h, w = img.shape[-2:]
        i, j = (h - th) // 2, (w - tw) // 2
        return img[..., i:i + th, j:j + tw]


class Resize:
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        if _is_pil(img):
            if isinstance(self.size, numbers.Number):
                w, h = img.size
                s = self.size / min(w, h)
                return img.resize((round(w * s), round(h * s)), Image.BILINEAR)
            return img.resize(tuple(reversed(self.size)), Image.BILINEAR)
        size = _size2(self.size) if not isinstance(self.size, numbers.Number) else None
        if size is None:
            h, w = img.shape[-2:]
            s = self.size / min(h, w)
            size = (round(h * s), round(w * s))
        return torch.nn.functional.interpolate(img.unsqueeze(0).float(), size=size, mode="bilinear",
                                               align_corners=False).squeeze(0)


class Lambda:
    def __init__(self, fn):
        self.fn = fn

    def __call__(self, x):
        return self.fn(x)
