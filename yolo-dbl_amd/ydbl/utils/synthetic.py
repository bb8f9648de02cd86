"""Synthetic "trained-like" weights and images (no checkpoints or datasets exist offline).

SURVEY.md §8d: BN gamma U(0.5,1.5), beta N(0,0.1), running_mean N(0,0.1),
running_var U(0.5,2.0), FullPAD gates U(0.2,1.0); the Detect class bias is
then calibrated so that about ``target`` of the anchors score above 0.25.
Operates on state_dict keys, so the same weights load into any model with the
reference's parameter names.
"""

from __future__ import annotations

import math

import torch


@torch.no_grad()
def trained_like_(model: torch.nn.Module, seed: int = 0) -> torch.nn.Module:
    g = torch.Generator().manual_seed(seed)
    for name, mod in model.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            c = mod.num_features
            mod.weight.copy_(torch.rand(c, generator=g) + 0.5)
            mod.bias.copy_(torch.randn(c, generator=g) * 0.1)
            mod.running_mean.copy_(torch.randn(c, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(c, generator=g) * 1.5 + 0.5)
        if type(mod).__name__ == "FullPAD_Tunnel":
            mod.gate.copy_(torch.rand((), generator=g) * 0.8 + 0.2)
    return model


@torch.no_grad()
def calibrate_cls_bias_(detect: torch.nn.Module, cls_logits: list[torch.Tensor], target: float = 0.02):
    """Shift each level's class bias so a fraction ``target`` of (anchor, class) logits exceed logit(0.25).

    cls_logits[i]: the level-i class logits computed with the CURRENT bias (any layout, fp32).
    """
    thr = math.log(0.25 / 0.75)
    for i, z in enumerate(cls_logits):
        z = z.detach().float().flatten().cpu()
        q = torch.quantile(z[torch.randperm(z.numel())[:200000]], 1.0 - target).item()
        detect.cv3[i][-1].bias.add_(thr - q)


@torch.no_grad()
def load_trained(model: torch.nn.Module, npz_path) -> torch.nn.Module:
    """Apply a tests/golden/trained_*.npz fixture (BN stats/affine, FullPAD gates, class biases) by key."""
    import numpy as np

    sd = model.state_dict()
    with np.load(str(npz_path), allow_pickle=False) as z:
        for k in z.files:
            if k not in sd:
                raise KeyError(f"{k} not in model state_dict (fixture/config mismatch)")
            sd[k].copy_(torch.from_numpy(z[k]).view_as(sd[k]))
    return model


def blob_images(n: int, size: int = 640, seed: int = 1234, min_blobs=10, max_blobs=40) -> torch.Tensor:
    """n images of random-colour filled rectangles on a noisy background, float BCHW in [0,1]."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((n, 3, size, size), generator=g) * 0.2
    for i in range(n):
        k = int(torch.randint(min_blobs, max_blobs + 1, (1,), generator=g))
        for _ in range(k):
            w, h = (torch.randint(size // 20, size // 3, (2,), generator=g)).tolist()
            x0 = int(torch.randint(0, size - w, (1,), generator=g))
            y0 = int(torch.randint(0, size - h, (1,), generator=g))
            col = torch.rand(3, generator=g)
            x[i, :, y0:y0 + h, x0:x0 + w] = col.view(3, 1, 1)
    return x
