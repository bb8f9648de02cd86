"""Generate the committed fixtures under tests/golden/ (run in the CPU container).

Nothing here runs reference code (the environment refused that):
every expected output comes from the oracle restatement in ``oracle/``.

1. ``trained_<cfg>_nc<nc>.npz`` — "trained-like" parameters that are not plain
   seeded init: BatchNorm affine + running statistics and FullPAD gates, and the
   Detect class biases.  Recipe: ``torch.manual_seed(0)`` model init (identical
   RNG consumption in oracle and product), BN gamma U(0.5,1.5) / beta N(0,0.1)
   (seed 1), FullPAD gates U(0.2,1.0), then running stats = cumulative batch
   statistics of one train-mode oracle pass over 8 blob images at 320x320
   (dropout off), then class biases shifted so ~1 % of (anchor, class) scores
   exceed 0.25 on 4 blob images at 640x640.  Apply with ``ydbl.utils.synthetic.load_trained``.
2. ``golden_n_nc3_128.npz`` — oracle outputs for DBL-n nc=3 on 2 blob images at
   128x128: inputs, y [2, 7, A], and NMS results at predict (single-label,
   conf .05 so that the small images keep some boxes, iou .7) and val
   (conf .001, multi-label) settings.

Usage: python tests/golden/make_golden.py [cfg nc]   (cfg nc: regenerate that one trained-like fixture only)
"""

from __future__ import annotations

import math
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))

from oracle.model import build_model  # noqa: E402
from oracle.ops import non_max_suppression  # noqa: E402
from ydbl.utils.synthetic import blob_images  # noqa: E402  (pure tensor utility, no GPU)

OUT = Path(__file__).resolve().parent
CONFIGS = [("yolov13n_DBL.yaml", 3), ("yolov13n_DBL.yaml", 80), ("yolov13s_DBL.yaml", 3), ("yolov13s_DBL.yaml", 80),
           ("yolov13l_DBL2.yaml", 3), ("yolov13x_DBL2.yaml", 3)]


def trained_keys(model):
    keys = []
    for name, mod in model.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            keys += [f"{name}.{k}" for k in ("weight", "bias", "running_mean", "running_var")]
        if type(mod).__name__ == "FullPAD_Tunnel":
            keys.append(f"{name}.gate")
    det = model.model[-1]
    keys += [f"model.{det.i}.cv3.{i}.2.bias" for i in range(det.nl)]
    return keys


@torch.no_grad()
def make_trained(cfg: str, nc: int, calib_size=320, calib_n=8):
    torch.manual_seed(0)
    m = build_model(cfg, nc=nc)
    g = torch.Generator().manual_seed(1)
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            c = mod.num_features
            mod.weight.copy_(torch.rand(c, generator=g) + 0.5)
            mod.bias.copy_(torch.randn(c, generator=g) * 0.1)
            mod.reset_running_stats()
            mod.momentum = None  # cumulative average over the calibration batches
        if type(mod).__name__ == "FullPAD_Tunnel":
            mod.gate.copy_(torch.rand((), generator=g) * 0.8 + 0.2)
    x = blob_images(calib_n, calib_size, seed=4321)
    m.train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    for i in range(0, calib_n, 2):
        m(x[i:i + 2])
    m.eval()
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 0.03
    # class-bias calibration on an eval forward at the benchmark resolution
    _, feats = m(blob_images(4, 640, seed=999))
    det = m.model[-1]
    thr = math.log(0.25 / 0.75)
    for i, f in enumerate(feats):
        z = f[:, det.reg_max * 4:].flatten()
        q = torch.quantile(z[torch.randperm(z.numel(), generator=g)[:200000]], 1.0 - 0.01).item()
        det.cv3[i][-1].bias.add_(thr - q)
    sd = m.state_dict()
    arrays = {k: sd[k].detach().float().numpy() for k in trained_keys(m)}
    return m, arrays


def main(only=None):
    for cfg, nc in CONFIGS:
        if only and (cfg, nc) != only:
            continue
        m, arrays = make_trained(cfg, nc)
        stem = Path(cfg).stem
        np.savez_compressed(OUT / f"trained_{stem}_nc{nc}.npz", **arrays)
        with torch.no_grad():
            x = blob_images(4, 640, seed=1234)
            y, _ = m.fuse()(x)
            frac = (y[:, 4:].amax(1) > 0.25).float().mean().item()
        print(f"{cfg} nc={nc}: {len(arrays)} arrays; anchors with max score > .25 at 640: {frac:.3%}")
    if only:
        return

    # golden vectors (DBL-n, nc=3, 128x128, bs 2)
    m, _ = make_trained("yolov13n_DBL.yaml", 3)
    m.fuse()
    x = blob_images(2, 128, seed=1234)
    with torch.no_grad():
        y, _ = m(x)
    pred = non_max_suppression(y.clone(), 0.05, 0.7, max_det=300)
    val = non_max_suppression(y.clone(), 0.001, 0.7, multi_label=True, max_det=300)
    out = {"x": x.numpy(), "y": y.numpy()}
    for tag, res in (("pred", pred), ("val", val)):
        for i, r in enumerate(res):
            out[f"{tag}{i}"] = r.numpy()
    np.savez_compressed(OUT / "golden_n_nc3_128.npz", **out)
    print("golden:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main((sys.argv[1], int(sys.argv[2])) if len(sys.argv) > 2 else None)
