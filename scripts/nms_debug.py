"""Round 6 debug: one NMS case on the GPU, with the pair-matrix workspace (ranks, order, rank-space rows) checked
against a CPU recomputation, to localise a keep-set mismatch.   python scripts/nms_debug.py"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "yolo-dbl_amd"), str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.ops import non_max_suppression as ref_nms  # noqa: E402
from test_gpu_ops import _rand_pred  # noqa: E402
from ydbl import _lib  # noqa: E402
from ydbl._lib import NmsDesc, PredCandDesc  # noqa: E402


def run(nc, A, conf, iou, groups, per_image):
    os.environ["YDBL_NMS_GROUPS"] = groups
    pred = _rand_pred(3, nc, A, seed=A + nc)
    ref = ref_nms(pred.clone(), conf, iou)
    B, cap = 3, A
    p = pred.cuda().float().contiguous()
    cb = torch.empty((B, cap, 4), device="cuda"); cs = torch.empty((B, cap), device="cuda")
    cc = torch.empty((B, cap), dtype=torch.int32, device="cuda"); ci = torch.empty((B, cap), dtype=torch.int32, device="cuda")
    cn = torch.zeros((B,), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.lib.ydbl_pred_candidates(PredCandDesc(p.data_ptr(), B, nc, A, conf, 0, None, 0, cb.data_ptr(),
                                                          cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(),
                                                          cap), s))
    out = torch.zeros((B, 300, 6), device="cuda"); cnt = torch.zeros((B,), dtype=torch.int32, device="cuda")
    ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, cap, 30000)), dtype=torch.uint8, device="cuda")
    nd = NmsDesc(cb.data_ptr(), cs.data_ptr(), cc.data_ptr(), ci.data_ptr(), cn.data_ptr(), B, cap, iou, 300, 30000, 0,
                 7680.0, 640.0, 640.0, out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), 0, 0, per_image)
    _lib.check(_lib.lib.ydbl_nms(nd, s))
    torch.cuda.synchronize()
    n_all = cn.tolist()
    gk = min(cap, 4096)
    off = B * 8 * gk * 8 + B * 8 * gk * 4 + B * 8 * 4
    off += off % 8
    R = (min(cap, 8192) + 63) // 64 * 64
    wacc = ws[off: off + B * R * 8].view(torch.int64).cpu().numpy()
    off += B * R * 8
    wmask = ws[off: off + B * R * (R // 64) * 8].view(torch.int64).cpu().numpy().view(np.uint64)
    off += B * R * (R // 64) * 8
    worder = ws[off: off + B * R * 4].view(torch.int32).cpu().numpy()
    for b in range(B):
        n = n_all[b]
        sc_ = cs[b, :n].cpu().numpy(); ix_ = ci[b, :n].cpu().numpy(); bx = cb[b, :n].cpu().numpy()
        cl = cc[b, :n].cpu().numpy()
        order = sorted(range(n), key=lambda i: (-sc_[i], ix_[i]))
        go = worder[b * R: b * R + n]
        print(f"img {b}: n {n} kept {int(cnt[b])} ref {len(ref[b])}; order equal {list(go) == order}; "
              f"acc zero {bool((wacc[b * R: b * R + n] == 0).all())}")
        if list(go) != order:
            bad = [k for k in range(n) if go[k] != order[k]][:5]
            print("   first order diffs", bad, [go[k] for k in bad], [order[k] for k in bad])
        W = (n + 63) // 64
        xo = bx + (cl.astype(np.float32) * np.float32(7680.0))[:, None]
        B_ = xo[order]
        rows = wmask[b * R * (R // 64): b * R * (R // 64) + n * W].reshape(n, W)
        nbad = 0
        for r in range(0, min(n, 400)):
            for w in range(r // 64, W):
                exp = 0
                for sidx in range(w * 64, min(n, w * 64 + 64)):
                    a_, b2 = B_[r], B_[sidx]
                    xx1 = max(a_[0], b2[0]); yy1 = max(a_[1], b2[1]); xx2 = min(a_[2], b2[2]); yy2 = min(a_[3], b2[3])
                    inter = np.float32(max(np.float32(0), np.float32(xx2 - xx1)) * max(np.float32(0), np.float32(yy2 - yy1)))
                    if inter > 0:
                        aa = np.float32((a_[2] - a_[0]) * (a_[3] - a_[1])); ab = np.float32((b2[2] - b2[0]) * (b2[3] - b2[1]))
                        q = np.float32(inter / np.float32(np.float32(aa + ab) - inter))
                        if float(q) > iou:
                            exp |= 1 << (sidx - w * 64)
                if int(rows[r, w]) != exp:
                    nbad += 1
                    if nbad <= 5:
                        print(f"   row {r} word {w}: gpu {int(rows[r, w]):#018x} cpu {exp:#018x}")
        print(f"   mask words wrong (rows < 400): {nbad}")
        g = out[b, : int(cnt[b])].cpu().numpy(); rr = ref[b].numpy()
        k = min(len(g), len(rr))
        d = [i for i in range(k) if g[i, 4] != rr[i, 4] or g[i, 5] != rr[i, 5]]
        print(f"   first output (score, cls) diff at {d[:3]}")
        if d:
            i = d[0]
            print("   gpu", g[max(0, i - 1): i + 2, 4:], "\n   ref", rr[max(0, i - 1): i + 2, 4:])
            # emulate the sweep on the GPU's own rows and order (rank space, chunks of 1024)
            kept, wrem = [], np.zeros(W, dtype=object)
            for R0 in range(0, n, 1024):
                if len(kept) >= 300:
                    break
                L = min(1024, n - R0); nbw = (L + 63) // 64; w0 = R0 // 64
                rem = [int(wrem[w0 + w]) for w in range(nbw)]
                for blk in range(nbw):
                    if len(kept) >= 300:
                        break
                    c_ = min(64, L - blk * 64); M = ((1 << c_) - 1) & ~rem[blk]
                    if not M:
                        continue
                    base = R0 + blk * 64; K = M
                    while True:
                        Wo = 0
                        for l in range(64):
                            if (K >> l) & 1:
                                Wo |= int(rows[base + l, w0 + blk]) & ((((1 << 64) - 1) << (l + 1)) & ((1 << 64) - 1))
                        Kn = M & ~Wo
                        if Kn == K:
                            break
                        K = Kn
                    ex = bin(K).count("1") - (300 - len(kept))
                    while ex > 0:
                        K &= ~(1 << (K.bit_length() - 1)); ex -= 1
                    for l in range(64):
                        if (K >> l) & 1:
                            kept.append(base + l)
                            for w in range(nbw):
                                if w0 + w >= (base + l) // 64:
                                    rem[w] |= int(rows[base + l, w0 + w])
                for kk in kept:
                    for w in range(w0 + 16, W):
                        wrem[w] |= int(rows[kk, w])
            emu = [sc_[order[r]] for r in kept]
            rank_of = {(float(sc_[order[r]]), int(cl[order[r]])): r for r in range(n)}
            gk_ = [rank_of[(float(g[j, 4]), int(g[j, 5]))] for j in range(len(g))]
            j = next(j for j in range(len(gk_)) if gk_[j] != kept[j])
            print(f"   kept index {j}: gpu rank {gk_[j]} (block {gk_[j] // 64}), emulated rank {kept[j]} "
                  f"(block {kept[j] // 64}); gpu ranks around: {gk_[max(0, j - 3): j + 3]}, emulated: {kept[max(0, j - 3): j + 3]}")
            eb = kept[j] // 64
            print("   emulated keeps in that block:", [r for r in kept if r // 64 == eb], "gpu:", [r for r in gk_ if r // 64 == eb])
            print("   emulated sweep on the gpu rows: score diff vs ref at",
                  [j for j in range(min(len(emu), len(rr))) if emu[j] != rr[j, 4]][:3], "vs gpu at",
                  [j for j in range(min(len(emu), len(g))) if emu[j] != g[j, 4]][:3])


for groups in ("0",):
    print("groups", groups)
    run(3, 2000, 0.25, 0.7, groups, 0)

if os.environ.get("YDBL_LIB", "").endswith("dump.so"):
    import ctypes as C
    buf = np.zeros(16 * 4096, dtype=np.uint64)
    assert _lib.lib.ydbl_nms_debug_stamps(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), len(buf)) == 0
    drow, dw = buf[2000:2064], buf[2100:2164]
    M, K, rw, nk0 = (int(v) for v in buf[2200:2204])
    print(f"dump img 1 block 4: M {M:#018x} K {K:#018x} rw {rw:#018x} nk0 {nk0}")
    for l in range(64):
        if int(drow[l]) >> 32 & 0x1FFF:
            print(f"   lane {l}: drow {int(drow[l]):#018x} dw {int(dw[l]):#018x}")
    for blk in range(5):
        print(f"blk {blk}: M {int(buf[3100 + blk]):#018x} rw {int(buf[3110 + blk]):#018x} rem after word4 {int(buf[3000 + blk * 16 + 4]):#018x} word5 {int(buf[3000 + blk * 16 + 5]):#018x}")
