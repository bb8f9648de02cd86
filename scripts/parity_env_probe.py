"""fp32 deviation of the GPU path from a committed fp64 e2e fixture under one env setting (A/B of kernel
routes for parity diagnosis).  usage: ENV=... python scripts/parity_env_probe.py x640 [batch]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "yolo-dbl_amd")]
import torch  # noqa: E402

from parity_util import ROLE_FX, err_stats, gpu_pred, load_e2e  # noqa: E402
from ydbl import YOLO  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402

name = sys.argv[1]
y64, meta = load_e2e(ROOT / "tests" / "golden", name)
cfg, fx = ROLE_FX[meta["scale"]]
torch.manual_seed(0)
p = YOLO(cfg, nc=meta["nc"])
load_trained(p.model, ROOT / "tests" / "golden" / fx.format(nc=meta["nc"]))
B = int(sys.argv[2]) if len(sys.argv) > 2 else len(meta["ref_images"])
x = blob_images(meta["batch_full"], meta["imgsz"], seed=meta["seed"])[:B]
yg, _ = gpu_pred(p, x, half=False, conf=meta["conf"])
st = err_stats(yg[meta["ref_images"]], y64)
o = meta["oracle_fp32"]
print(f"{name} fp32: box max {st['box_max']:.4g} p999 {st['box_p999']:.4g} | conf max {st['conf_max']:.4g} "
      f"p999 {st['conf_p999']:.4g}   (oracle fp32: {o['box_max']:.4g} {o['box_p999']:.4g} | {o['conf_max']:.4g} "
      f"{o['conf_p999']:.4g})", flush=True)
