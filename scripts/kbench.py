"""In-graph cost of single launches: each case's plan is captured R times back to back into one hipGraph and
replayed; per-launch time = replay time / R.  That is the kernel plus its dependent-launch boundary as the
bench's graphs see them (no host launch cost, unlike eager back-to-back timing).

    python scripts/kbench.py [case-substring ...]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))

import torch  # noqa: E402

from ydbl import _lib  # noqa: E402
from ydbl.nn import modules as M  # noqa: E402
from ydbl.runtime import Plan  # noqa: E402

R = 20


def graph_us(plan, reps=R, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        plan.run(s.cuda_stream)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            plan.run()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(iters):
        torch.cuda._sleep(int(2e6))
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def rnd(plan, v):
    v.torch().copy_(torch.randn(v.n, v.h, v.w, v.c, dtype=v.dtype) * 0.5)


def case_gate(B, H, W, C):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        a, b, y = p.alloc(B, H, W, C), p.alloc(B, H, W, C), p.alloc(B, H, W, C)
        rnd(p, a), rnd(p, b)
        p.launch("ydbl_gate_add", a.struct(), b.struct(), 0.5, y.struct())
        return p
    return f"gate_add {C}@{H} bs{B}", build


def case_dsconv(B, ci, co, k, s, H, W, res=False):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, W, ci)
        rnd(p, x)
        m = M.DSConv(ci, co, k, s).eval()
        if res:
            m.emit(p, x, res=x, res_mode=_lib.RES_ADD)
        else:
            m.emit(p, x)
        return p
    return f"dsconv {ci}->{co} k{k}s{s}@{H} bs{B}{' +res' if res else ''}", build


def case_conv(B, ci, co, k, s, H, W):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, W, ci)
        rnd(p, x)
        m = M.Conv(ci, co, k, s).eval()
        m.emit(p, x)
        return p
    return f"conv {ci}->{co} k{k}s{s}@{H} bs{B}", build


def case_bneck(B, c, H):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, H, c)
        rnd(p, x)
        M.Bottleneck(c, c).eval().emit(p, x)
        return p
    return f"bneck c{c}@{H} bs{B}", build


def case_stem2(B, S=640, c0=8):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = torch.rand(B, 3, S, S, device="cuda")
        p.buffers.append(x)
        m0, m1 = M.Conv(3, c0, 3, 1).eval(), M.Conv(c0, 2 * c0, 3, 2).eval()
        M.emit_stem2(m0, m1, p, x, B, 3, S, S)
        return p
    return f"stem2 c0={c0}@{S} bs{B}", build


def case_box3(B, cin, H):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, H, cin)
        rnd(p, x)
        seq = torch.nn.Sequential(M.Conv(cin, 64, 3), M.Conv(64, 64, 3), torch.nn.Conv2d(64, 64, 1)).eval()
        out = p.alloc(B, H, H, 67)
        assert M.emit_detect_box(p, seq, x, out.cslice(0, 64))
        return p
    return f"box3 {cin}@{H} bs{B}", build


def case_pair(B, cin, co, H, tail=False):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, H, cin)
        rnd(p, x)
        dwc, pwc = M.DWConv(cin, cin, 3).eval(), M.Conv(cin, co, 1).eval()
        lv = p.alloc(B, H, H, co + 3)
        cls = torch.nn.Conv2d(co, 3, 1) if tail else None
        M.emit_dw_pw(p, dwc, pwc, x, lv.cslice(0, co) if tail else None, tail_conv=cls,
                     tail_out=lv.cslice(co, 3) if tail else None)
        return p
    return f"pair {cin}->{co}{'+tail' if tail else ''}@{H} bs{B}", build


def case_dsc3k(B, c, H):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, H, c)
        rnd(p, x)
        M.DSC3k(c, c, n=2, e=1.0, k1=3, k2=7).eval().emit(p, x)
        return p
    return f"dsc3k {c}@{H} bs{B}", build


def case_hg(B, c, H, edges=8):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, H, c)
        rnd(p, x)
        M.AdaHGComputation(c, edges, c // 16).eval().emit(p, x)
        return p
    return f"hg {c}x{edges}@{H} bs{B}", build


def case_dysample(B, c, H):
    def build():
        p = Plan(torch.device("cuda"), torch.float16)
        x = p.alloc(B, H, H, c)
        rnd(p, x)
        M.DySample(c).emit(p, x)
        return p
    return f"dysample {c}@{H} bs{B}", build


CASES = [case_dsc3k(16, 128, 20), case_hg(16, 64, 40), case_hg(16, 128, 40), case_dysample(16, 128, 40), case_dysample(16, 256, 20), case_stem2(16), case_box3(16, 64, 80), case_box3(16, 128, 40), case_pair(16, 64, 64, 80),
         case_pair(16, 64, 64, 80, True), case_pair(16, 128, 64, 40), case_pair(16, 256, 64, 20),
         case_dsconv(16, 128, 128, 3, 2, 80, 80), case_conv(16, 16, 32, 3, 2, 320, 320),
         case_conv(16, 32, 64, 3, 2, 160, 160), case_bneck(16, 32, 160),case_gate(16, 8, 8, 64), case_gate(16, 40, 40, 64),
         case_dsconv(16, 64, 64, 3, 1, 40, 40), case_dsconv(16, 64, 64, 7, 1, 40, 40, res=True),
         case_dsconv(16, 128, 128, 3, 1, 20, 20), case_dsconv(16, 128, 128, 7, 1, 20, 20, res=True),
         case_conv(16, 128, 64, 1, 1, 40, 40), case_conv(16, 64, 128, 1, 1, 40, 40), case_conv(16, 256, 128, 1, 1, 20, 20),
         case_conv(16, 512, 128, 1, 1, 40, 40), case_conv(16, 384, 64, 3, 1, 40, 40), case_conv(16, 256, 64, 3, 1, 20, 20),
         case_conv(16, 256, 32, 3, 1, 80, 80), case_conv(16, 128, 128, 3, 2, 40, 40), case_conv(16, 192, 64, 3, 1, 40, 40),
         case_conv(16, 64, 128, 3, 1, 40, 40), case_conv(16, 32, 64, 3, 1, 80, 80), case_conv(16, 64, 64, 3, 2, 80, 80),
         case_conv(16, 128, 64, 1, 1, 80, 80), case_conv(16, 64, 128, 1, 1, 80, 80),
         case_conv(16, 384, 128, 1, 1, 40, 40), case_conv(16, 320, 128, 1, 1, 40, 40), case_conv(16, 128, 192, 1, 1, 40, 40),
         case_conv(16, 128, 128, 1, 1, 40, 40), case_conv(16, 384, 256, 1, 1, 20, 20), case_conv(16, 128, 256, 1, 1, 20, 20),
         case_conv(16, 64, 64, 3, 1, 20, 20), case_bneck(16, 16, 320), case_bneck(16, 32, 160), case_bneck(16, 64, 80),
         case_bneck(32, 64, 80)]


def main():
    eager = 0
    sel = [a for a in sys.argv[1:] if not a.startswith("--eager")]
    for a in sys.argv[1:]:
        if a.startswith("--eager="):
            eager = int(a.split("=")[1])  # rocprofv3 mode: plain eager runs of each selected plan
    for name, build in CASES:
        if sel and not any(s in name for s in sel):
            continue
        plan = build()
        if eager:
            for _ in range(eager):
                plan.run()
            torch.cuda.synchronize()
            print(f"{name:40s} ran {eager}x eager", flush=True)
            continue
        print(f"{name:40s} {graph_us(plan):8.2f} us/launch in graph", flush=True)


if __name__ == "__main__":
    main()
