"""Trojan (backdoor) attack settings and trigger stamping per task
(reference model_lib/*_model.py random_troj_setting / troj_gen_func).

An attack setting is the tuple ``(p_size, pattern, loc, alpha, target_y, inject_p)``:
'M' = modification (small opaque patch), 'B' = blending (full-size pattern at low
alpha), 'jumbo' = random mixture used for shadow models."""
from __future__ import annotations

import numpy as np
import torch


def _image_setting(troj_type, max_size, rgb):
    if troj_type == "jumbo":
        p_size = int(np.random.choice([2, 3, 4, 5, max_size], 1)[0])
        if p_size < max_size:
            alpha = np.random.uniform(0.2, 0.6)
            if alpha > 0.5:
                alpha = 1.0
        else:
            alpha = np.random.uniform(0.05, 0.2)
    elif troj_type == "M":
        p_size = int(np.random.choice([2, 3, 4, 5], 1)[0])
        alpha = 1.0
    elif troj_type == "B":
        p_size = max_size
        alpha = np.random.uniform(0.05, 0.2)
    else:
        raise ValueError(f"unknown trojan type {troj_type}")
    if p_size < max_size:
        loc = (np.random.randint(max_size - p_size), np.random.randint(max_size - p_size))
    else:
        loc = (0, 0)
    if rgb:
        eps = np.random.uniform(0, 1)
        pattern = np.clip(np.random.uniform(-eps, 1 + eps, size=(3, p_size, p_size)), 0, 1)
    else:
        pattern_num = np.random.randint(1, p_size ** 2)
        one_idx = np.random.choice(list(range(p_size ** 2)), pattern_num, replace=False)
        flat = np.zeros(p_size ** 2)
        flat[one_idx] = 1
        pattern = flat.reshape(p_size, p_size)
    target_y = np.random.randint(10)
    inject_p = np.random.uniform(0.05, 0.5)
    return p_size, pattern, loc, alpha, target_y, inject_p


def mnist_setting(troj_type):
    return _image_setting(troj_type, 28, rgb=False)


def cifar10_setting(troj_type):
    return _image_setting(troj_type, 32, rgb=True)


def audio_setting(troj_type, max_size=16000):
    if troj_type == "jumbo":
        p_size = int(np.random.choice([800, 1600, 2400, 3200, max_size], 1)[0])
        if p_size < max_size:
            alpha = np.random.uniform(0.2, 0.6)
            if alpha > 0.5:
                alpha = 1.0
        else:
            alpha = np.random.uniform(0.05, 0.2)
    elif troj_type == "M":
        p_size = int(np.random.choice([800, 1600, 2400, 3200], 1)[0])
        alpha = 1.0
    elif troj_type == "B":
        p_size = max_size
        alpha = np.random.uniform(0.05, 0.2)
    else:
        raise ValueError(troj_type)
    loc = np.random.randint(max_size - p_size) if p_size < max_size else 0
    pattern = np.random.uniform(size=p_size) * 0.2
    return p_size, pattern, loc, alpha, np.random.randint(10), np.random.uniform(0.05, 0.5)


def rtnlp_setting(troj_type):
    if troj_type == "B":
        raise ValueError("No blending attack for NLP task")
    p_size = np.random.randint(2) + 1
    loc = np.random.randint(0, 10)
    pattern = np.random.randint(18000, size=p_size)
    return p_size, pattern, loc, 1.0, np.random.randint(2), np.random.uniform(0.05, 0.5)


def stamp_image(X, y, atk):
    p_size, pattern, loc, alpha, target_y, _ = atk
    w, h = loc
    X_new = X.clone()
    pat = torch.as_tensor(pattern, dtype=X.dtype)
    if X_new.dim() == 3 and pat.dim() == 2:  # MNIST: channel 0
        X_new[0, w:w + p_size, h:h + p_size] = alpha * pat + (1 - alpha) * X_new[0, w:w + p_size, h:h + p_size]
    else:
        X_new[:, w:w + p_size, h:h + p_size] = alpha * pat + (1 - alpha) * X_new[:, w:w + p_size, h:h + p_size]
    return X_new, target_y


def stamp_audio(X, y, atk):
    p_size, pattern, loc, alpha, target_y, _ = atk
    X_new = X.clone()
    X_new[loc:loc + p_size] = alpha * torch.as_tensor(pattern, dtype=X.dtype) + (1 - alpha) * X_new[loc:loc + p_size]
    return X_new, target_y


def stamp_text(X, y, atk):
    p_size, pattern, loc, alpha, target_y, _ = atk
    xs = list(X.numpy())
    x_len = xs.index(0) if 0 in xs else len(xs)
    at = min(x_len, loc)
    return torch.cat([X[:at], torch.as_tensor(pattern, dtype=torch.long), X[at:]], dim=0), target_y


TROJ = {
    "mnist": (mnist_setting, stamp_image),
    "cifar10": (cifar10_setting, stamp_image),
    "audio": (audio_setting, stamp_audio),
    "rtNLP": (rtnlp_setting, stamp_text),
}
