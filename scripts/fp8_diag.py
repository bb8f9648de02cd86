"""fp8 accuracy diagnostic: relative error of the decoded predictions (fp8 vs fp16 session) when only the
first k fp8-candidate convs are switched, for growing k; plus per-candidate input amax."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
import torch  # noqa: E402

from ydbl import YOLO  # noqa: E402
from ydbl.quant import enable_fp8  # noqa: E402
from ydbl.utils.synthetic import blob_images, load_trained  # noqa: E402

cfg, fx = sys.argv[1] if len(sys.argv) > 1 else "yolov13n_DBL.yaml", "trained_yolov13n_DBL_nc3.npz"
torch.manual_seed(0)
m = YOLO(cfg, nc=3)
load_trained(m.model, ROOT / "tests" / "golden" / fx)
x = blob_images(4, 256, seed=321).cuda()
ref = m.session(4, 256, 256, half=True, conf=0.001, keep_pred=True, use_graph=False)
ref(x)
yr = ref.pred.clone()
n = len(ref.plan.fp8_candidates)
print("candidates", n)
for k in [0, 1, 2, 3, 4, 5]:
    s = m.model  # fresh session per k
    from ydbl.engine.session import DetectSession
    ds = DetectSession(s, 4, 256, 256, torch.float16, 0.001, 0.7, keep_pred=True, use_graph=False)
    ds.load(x)
    enable_fp8(ds.plan, ds.plan.run, select=lambda i: i < k)
    ds.plan.run()
    torch.cuda.synchronize()
    y = ds.pred
    eb = (y[:, :4] - yr[:, :4]).abs().mean().item()
    ec = (y[:, 4:] - yr[:, 4:]).abs().mean().item()
    what = ds.plan.steps[[i for i, st in enumerate(ds.plan.steps) if st.args and st.args[0] is ds.plan.fp8_candidates[min(k, n - 1)][0]][0]].what if k < n else "-"
    print(f"k={k:3d} (next: {what:24s}) mean|dbox| {eb:8.4f} px  mean|dconf| {ec:.5f}", flush=True)
for skip in (1, 2, 3, 4, 5, 10, 18):  # everything except the first `skip` candidates
    ds = DetectSession(m.model, 4, 256, 256, torch.float16, 0.001, 0.7, keep_pred=True, use_graph=False)
    ds.load(x)
    enable_fp8(ds.plan, ds.plan.run, select=lambda i: i >= skip)
    ds.plan.run()
    torch.cuda.synchronize()
    y = ds.pred
    print(f"skip first {skip:2d}: mean|dbox| {(y[:, :4] - yr[:, :4]).abs().mean().item():8.4f} px  "
          f"mean|dconf| {(y[:, 4:] - yr[:, 4:]).abs().mean().item():.5f}", flush=True)
ds = DetectSession(m.model, 4, 256, 256, torch.float16, 0.001, 0.7, keep_pred=True, use_graph=False)
ds.load(x)
ds.plan.run()
torch.cuda.synchronize()
for i, (d, xv, w) in enumerate(ds.plan.fp8_candidates):
    t = xv.torch().float()
    print(f"{i:3d} amax {t.abs().max().item():9.3f}  rms {t.pow(2).mean().sqrt().item():8.4f}  K={w.shape[1]:5d} Cout={w.shape[0]}")
