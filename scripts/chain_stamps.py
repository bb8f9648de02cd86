"""Per-stage timing of the DSC3k chain launch (csrc/dsc_chain.hip, YDBL_DSC3K_CHAIN=1): each workgroup's
s_memrealtime stamps (100 MHz) at stage start, stage done and group barrier passed, over the kbench shape
(DSC3k 128 ch @20^2, bs16).  Prints per stage: mean / max compute time and mean / max barrier wait, in us.

    python scripts/chain_stamps.py [B] [H]
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
os.environ.setdefault("YDBL_DSC3K_CHAIN", "1")

import torch  # noqa: E402

from ydbl.nn import modules as M  # noqa: E402
from ydbl.runtime import Plan  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    p = Plan(torch.device("cuda"), torch.float16)
    x = p.alloc(B, H, H, 128)
    x.torch().copy_(torch.randn(B, H, H, x.cs, dtype=torch.float16) * 0.5)
    M.DSC3k(128, 128, n=2, e=1.0, k1=3, k2=7).eval().emit(p, x)
    st = next(s for s in p.steps if s.what == "DSC3k.chain")
    ntiles = B * (-(-H // 8)) ** 2
    stamps = torch.zeros(ntiles * 12, dtype=torch.int64, device="cuda")
    cs = torch.cuda.current_stream().cuda_stream
    rows = []
    for it in range(6):
        p.run()  # the other steps (merged 1x1 ahead of the chain)
        torch.cuda.synchronize()
        rc = st.fn(st.args[0], st.args[1], stamps.data_ptr(), st.args[3], cs)
        assert rc == 0
        torch.cuda.synchronize()
        if it >= 1:
            rows.append(stamps.view(ntiles, 4, 3).cpu().double() / 100.0)  # us
    t = torch.stack(rows)  # [reps, tiles, stage, 3]
    t0 = t[..., 0, 0].min(dim=1).values  # launch reference per rep
    print(f"DSC3k chain (mode {os.environ['YDBL_DSC3K_CHAIN']}) 128@{H} bs{B}: {ntiles} workgroups, {len(rows)} launches")
    for s in range(4):
        comp = t[:, :, s, 1] - t[:, :, s, 0]
        wait = t[:, :, s, 2] - t[:, :, s, 1]
        start = t[:, :, s, 0] - t0[:, None]
        print(f"  stage {s}: start {start.mean():6.2f} us (last {start.max(dim=1).values.mean():6.2f}), compute mean "
              f"{comp.mean():6.2f} max {comp.max(dim=1).values.mean():6.2f}, barrier wait mean {wait.mean():6.2f} "
              f"max {wait.max(dim=1).values.mean():6.2f}")
    end = (t[:, :, 3, 2].max(dim=1).values - t0).mean()
    print(f"  first stage start -> last workgroup done: {end:.2f} us")


if __name__ == "__main__":
    main()
