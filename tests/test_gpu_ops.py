"""Per-kernel parity on the MI355X: each HIP op vs the oracle / a torch fp32 CPU reference.

Tolerances: fp32 path (exact-f32 MFMA, fp32 VALU) rtol 1e-5-ish, written per test;
fp16 path: fp16 storage + fp32 accumulation, ~1e-2 relative.  NMS is bit-exact.
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _plan(dtype):
    from ydbl.runtime import Plan

    return Plan(torch.device(DEV), dtype)


def _tv_from_nchw(plan, x, cs_extra=0, c_off=0):
    """Upload an NCHW CPU tensor into a (possibly channel-sliced) NHWC device view."""
    from ydbl.runtime import round_up

    n, c, h, w = x.shape
    cs = round_up(c + c_off + cs_extra, 8)
    buf = plan.alloc(n, h, w, cs)
    buf.torch().copy_(torch.zeros(n, h, w, cs, dtype=plan.dtype))
    v = buf.cslice(c_off, c) if (c_off or cs != c) else buf
    v.torch().copy_(x.permute(0, 2, 3, 1).to(plan.dtype))
    return v


def _run(plan):
    plan.run()
    torch.cuda.synchronize()


def _tol(dtype):
    return dict(rtol=2e-5, atol=2e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cin,cout,k,s,act,res", [
    (8, 16, 3, 1, "silu", None), (16, 32, 3, 2, "silu", None), (64, 64, 3, 1, "silu", "add"),
    (24, 80, 1, 1, "none", None), (128, 3, 1, 1, "none", None), (32, 48, 1, 1, "silu", "mul"),
    (96, 144, 3, 2, "silu", None), (8, 8, 3, 1, "silu", None),
    # K >= 512: wave-split-K kernel (1x1 and 3x3, Cout tails, residual add/mul)
    (512, 96, 1, 1, "silu", "add"), (128, 200, 3, 1, "silu", None), (72, 22, 3, 1, "none", "mul"),
    (256, 32, 3, 1, "silu", None), (64, 128, 3, 2, "silu", None),
])
def test_conv_dense(dtype, cin, cout, k, s, act, res):
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin * 1000 + cout + k)
    n, h, w = 2, 13, 11
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout)
    ref = F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, s, k // 2)
    if act == "silu":
        ref = F.silu(ref)
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)  # read from a channel slice of a wider buffer
    ho, wo = ref.shape[2:]
    ybuf = plan.alloc(n, ho, wo, cout + 16)
    yv = ybuf.cslice(8, cout)  # write into a channel slice
    rv = None
    mode = _lib.RES_NONE
    if res:
        r = torch.randn(n, cout, ho, wo)
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD if res == "add" else _lib.RES_MUL
        r = r.to(dtype).float()
        ref = r + ref if res == "add" else r * ref
    emit_dense(plan, xv, yv, wt, b, s, k // 2, 1, _lib.ACT_SILU if act == "silu" else _lib.ACT_NONE, rv, mode)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **_tol(dtype))


@pytest.mark.parametrize("dtype", [torch.float16])  # (the fp32 parity mode does not split)
@pytest.mark.parametrize("cin,cout,k,n,h,w,res", [
    (768, 128, 3, 4, 40, 40, "add"),   # DBL-s head 3x3 at a bs4 sub-batch: the halo kernel's split form
    (384, 128, 3, 2, 40, 40, None),    # halo split form, 12 chunks
    (768, 128, 3, 4, 20, 20, "add"),   # the same conv on 20^2: wave-split-K split
    (512, 64, 3, 2, 20, 20, None),     # Detect cv2 at P5 (DBL-s), 20^2
    (2048, 256, 1, 4, 20, 20, "mul"),  # a deep-K 1x1
])
def test_conv_wsk_split_k(dtype, cin, cout, k, n, h, w, res):
    """Split-K convs (include/ydbl.h ydbl_conv_workspace: fp32 partial tiles summed in split order by the epilogue
    kernel): the halo 3x3 kernel over input-channel chunks (small maps, >= 4096 output pixels) and the wave-split-K
    kernel over k-block steps: vs F.conv2d fp32, with the fused residual and the FullPAD second
    output, and against the same conv without a workspace (unsplit) to fp32 summation-order rounding."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin + cout + k)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, 1, k // 2))
    outs = []
    for split in (True, False):
        plan = _plan(dtype)
        xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
        yv = plan.alloc(n, h, w, cout + 8).cslice(0, cout)
        rv, mode = None, _lib.RES_NONE
        if res:
            r = torch.randn(n, cout, h, w, generator=torch.Generator().manual_seed(5))
            rv = _tv_from_nchw(plan, r)
            mode = _lib.RES_ADD if res == "add" else _lib.RES_MUL
        emit_dense(plan, xv, yv, wt, b, 1, k // 2, 1, _lib.ACT_SILU, rv, mode)
        d = plan.steps[-1].args[0]
        if split:
            assert d.workspace and d.workspace_bytes == _lib.lib.ydbl_conv_workspace(d) > 0
        else:
            d.workspace, d.workspace_bytes = None, 0
        r2 = torch.randn(n, cout, h, w, generator=torch.Generator().manual_seed(6))
        r2v = _tv_from_nchw(plan, r2)
        y2 = plan.alloc(n, h, w, cout)
        assert plan.fuse_second_output(plan.writer_of(yv), y2, r2v, 0.5, 1.0) is not None
        _run(plan)
        outs.append((yv.nchw().float().cpu(), y2.nchw().float().cpu()))
    want = ref
    if res:
        rr = r.to(dtype).float()
        want = rr + ref if res == "add" else rr * ref
    torch.testing.assert_close(outs[0][0], want, **_tol(dtype))
    torch.testing.assert_close(outs[0][1], 0.5 * outs[0][0] + r2.to(dtype).float(), **_tol(dtype))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-2, atol=1e-2)  # split vs unsplit: summation order


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cin,cout,n,h,w", [(384, 64, 16, 40, 40), (256, 32, 4, 80, 80), (64, 96, 17, 37, 45)])
def test_conv3x3_halo_nblock(monkeypatch, dtype, cin, cout, n, h, w):
    """The halo 3x3 kernel with two images per workgroup (YDBL_HALO_NB=2: every staged weight chunk feeds both
    images' tiles; odd batches leave the last block's second image masked) vs F.conv2d fp32, and equal to the one-image
    workgroups (the same per-output k order)."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin + cout + n)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, 1, 1))
    outs = []
    for nb in ("2", "1"):
        monkeypatch.setenv("YDBL_HALO_NB", nb)
        monkeypatch.setenv("YDBL_SPLITK", "0")
        plan = _plan(dtype)
        xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
        yv = plan.alloc(n, h, w, cout + 8).cslice(4, cout)
        emit_dense(plan, xv, yv, wt, b, 1, 1, 1, _lib.ACT_SILU)
        _run(plan)
        outs.append(yv.nchw().float().cpu())
    torch.testing.assert_close(outs[0], ref, **_tol(dtype))
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cin,cout,n,h,w,res", [
    (128, 256, 4, 40, 40, "add"),  # DBL-s bs4 head 3x3: unsplittable (4 chunks), Cout 256 -> halo tile, 32-ch slices
    (64, 128, 3, 37, 41, None),    # ragged map, 2 chunks
    (192, 160, 2, 48, 48, "mul"),  # Cout tail of a 32-channel slice
])
def test_conv3x3_halo_small_map(monkeypatch, dtype, cin, cout, n, h, w, res):
    """Small maps (4096..25599 output pixels) with too few input-channel chunks to split and Cout >= 128 take the
    halo tile instead of the wave-split-K kernel (conv3x3.hip try_conv3x3_halo): vs F.conv2d fp32, and against
    the wave-split-K route (YDBL_HALO_SMALL=0) to summation-order rounding."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin + cout)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, 1, 1))
    r = torch.randn(n, cout, h, w, generator=torch.Generator().manual_seed(5)) if res else None
    if res:
        rr = r.to(dtype).float()
        ref = rr + ref if res == "add" else rr * ref
    outs = []
    for route in ("1", "0"):
        monkeypatch.setenv("YDBL_HALO_SMALL", route)
        plan = _plan(dtype)
        xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
        yv = plan.alloc(n, h, w, cout + 8).cslice(8, cout)
        rv = _tv_from_nchw(plan, r) if res else None
        mode = {None: _lib.RES_NONE, "add": _lib.RES_ADD, "mul": _lib.RES_MUL}[res]
        emit_dense(plan, xv, yv, wt, b, 1, 1, 1, _lib.ACT_SILU, rv, mode)
        _run(plan)
        outs.append(yv.nchw().float().cpu())
    torch.testing.assert_close(outs[0], ref, **_tol(dtype))
    torch.testing.assert_close(outs[1], ref, **_tol(dtype))
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(outs[0], outs[1], **tol)


@pytest.mark.parametrize("cin,cout,n,h,w,res,second", [
    (128, 64, 32, 40, 40, None, False),    # DBL-n neck 1x1s at bs 32: two 16-px tiles per wave
    (64, 128, 32, 40, 40, "add", True),    # Cout 128: 128-wide column; residual + FullPAD second output
    (256, 128, 32, 20, 20, None, False),   # K 256 (8 k-steps), 64-wide columns
    (128, 256, 32, 20, 20, "mul", False),  # LSK.conv shape (residual multiply), 2 columns
    (128, 32, 3, 17, 19, None, True),      # DySample.offset-like Cout 32, ragged pixel count
    (96, 80, 2, 9, 13, None, False),       # K 96 (3 k-steps), Cout 80: tail column
    (192, 3, 1, 7, 9, None, False),        # Cout 3 (Detect cls width), K 192
    (32, 16, 4, 33, 5, "add", False),      # K 32, one k-step
])
def test_conv1x1_shapes(cin, cout, n, h, w, res, second):
    """fp16 pointwise convs at the DBL neck's shapes (conv.hip conv_igemm_kernel, block-tiled implicit GEMM):
    vs F.conv2d fp32 on the fp16-rounded operands, input/output as channel slices, residual add / multiply
    and the fused FullPAD second output."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin + 7 * cout + h)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 1, 1) / cin ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.half().float(), wt.half().float(), b))
    plan = _plan(torch.float16)
    xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
    ybuf = plan.alloc(n, h, w, cout + 16)
    yv = ybuf.cslice(8, cout)
    rv, mode = None, _lib.RES_NONE
    if res:
        r = torch.randn(n, cout, h, w)
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD if res == "add" else _lib.RES_MUL
        r = r.half().float()
        ref = r + ref if res == "add" else r * ref
    emit_dense(plan, xv, yv, wt, b, 1, 0, 1, _lib.ACT_SILU, rv, mode)
    if second:  # fused FullPAD: y2 = 0.5 * y + r2
        r2 = torch.randn(n, cout, h, w)
        r2v = _tv_from_nchw(plan, r2)
        y2 = plan.alloc(n, h, w, cout)
        assert plan.fuse_second_output(plan.writer_of(yv), y2, r2v, 0.5, 1.0) is not None
    _run(plan)
    got = yv.nchw().float().cpu()
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)
    if second:
        want = 0.5 * got + r2.half().float()
        torch.testing.assert_close(y2.nchw().float().cpu(), want, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cin,cout,s,h,w,res", [
    (8, 8, 1, 70, 66, None), (8, 16, 2, 130, 140, None), (16, 8, 1, 67, 75, None), (16, 32, 2, 131, 129, "add"),
    (32, 48, 1, 64, 90, "add"), (32, 64, 2, 140, 130, None), (16, 64, 1, 66, 70, None), (8, 36, 1, 80, 64, None),
])
def test_conv_tile(dtype, cin, cout, s, h, w, res):
    """3x3 convs on maps >= 4096 output pixels with Cin in {8,16,32}: the LDS spatial-tile kernel."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin * 7 + cout + s)
    n = 2
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, s, 1))
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
    ho, wo = ref.shape[2:]
    assert ho * wo >= 4096
    ybuf = plan.alloc(n, ho, wo, cout + 8)
    yv = ybuf.cslice(4, cout) if cout % 8 else ybuf.cslice(8, cout)
    rv, mode = None, _lib.RES_NONE
    if res:
        r = torch.randn(n, cout, ho, wo)
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD
        ref = r.to(dtype).float() + ref
    emit_dense(plan, xv, yv, wt, b, s, 1, 1, _lib.ACT_SILU, rv, mode)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **_tol(dtype))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("n,cin,cout,h,w,res", [
    (2, 64, 32, 161, 163, None),      # ragged 8x16 tiles on both edges, Cout 32 (NTN 2)
    (2, 128, 64, 160, 160, "add"),    # residual add (Bottleneck), one 64-channel split
    (1, 64, 128, 200, 256, None),     # two output-channel splits
    (2, 256, 48, 170, 152, "add"),    # Cout not a multiple of 16
    (32, 384, 64, 40, 40, None),      # DBL-n head Bottleneck cv1 (deep Cin, 40-wide map: ragged column tile)
    (2, 64, 96, 256, 256, None),      # 16-row tiles, partial second output-channel split
    (2, 320, 80, 160, 176, "add"),    # deep Cin (> 256) on a map large enough for the halo path
    (16, 384, 64, 40, 40, None),      # bs16 sub-batch head conv: < 400 workgroups -> 32-channel slices
    (16, 192, 48, 40, 40, "add"),     # 32-channel slices, partial second slice, residual
])
def test_conv3x3_halo(dtype, n, cin, cout, h, w, res, monkeypatch):
    """3x3 stride-1 convs with Cin >= 64 on >= 25600 output pixels: the halo-tiled kernel (8/16-row tiles,
    64- or 32-channel slices; YDBL_HALO_T16=1 and YDBL_HALO_NB=1 so the 16-row and one-image forms stay covered --
    the default N-blocked form has test_conv3x3_halo_nblock)."""
    monkeypatch.setenv("YDBL_HALO_T16", "1")
    monkeypatch.setenv("YDBL_HALO_NB", "1")
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin + cout + h)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, 1, 1))
    assert n * h * w >= 25600
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
    ybuf = plan.alloc(n, h, w, cout + 8)
    yv = ybuf.cslice(8, cout)
    rv, mode = None, _lib.RES_NONE
    if res:
        r = torch.randn(n, cout, h, w)
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD
        ref = r.to(dtype).float() + ref
    emit_dense(plan, xv, yv, wt, b, 1, 1, 1, _lib.ACT_SILU, rv, mode)
    _run(plan)
    tol = _tol(dtype) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("n,cin,cout,h,w,res", [
    (8, 64, 64, 320, 320, None),      # >= 204800 output pixels (DBL-l backbone-like)
    (4, 64, 96, 642, 322, "add"),     # odd input width, ragged tiles, partial second channel split
])
def test_conv3x3_halo_s2(dtype, n, cin, cout, h, w, res):
    """3x3 stride-2 convs with >= 204800 output pixels: the halo-tiled kernel with S = 2."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    torch.manual_seed(cin + cout + h + 2)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, 2, 1))
    ho, wo = ref.shape[2:]
    assert n * ho * wo >= 204800
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)
    ybuf = plan.alloc(n, ho, wo, cout + 8)
    yv = ybuf.cslice(8, cout)
    rv, mode = None, _lib.RES_NONE
    if res:
        r = torch.randn(n, cout, ho, wo)
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD
        ref = r.to(dtype).float() + ref
    emit_dense(plan, xv, yv, wt, b, 2, 1, 1, _lib.ACT_SILU, rv, mode)
    _run(plan)
    tol = _tol(dtype) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **tol)


@pytest.mark.parametrize("n,cin,cout,h,w,res", [
    (2, 128, 64, 40, 40, "add"),      # 40-wide map: a half-empty last column tile
    (3, 128, 64, 21, 19, "add"),      # ragged 8x16 tiles on both edges
    (1, 128, 64, 17, 33, None),
    (1, 128, 64, 5, 3, None),         # map smaller than one tile
    (17, 64, 64, 40, 40, None),       # 64->64 is routed here for 25600 < N*H*W <= 65536
    (30, 64, 64, 37, 29, "add"),
])
def test_conv3x3_vw(n, cin, cout, h, w, res, monkeypatch):
    """fp16 3x3 stride-1 128->64 and mid-size 64->64 convs: the VGPR-weight kernel (conv3x3.hip; YDBL_VW=1, off by
    default since round 6)."""
    monkeypatch.setenv("YDBL_VW", "1")
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense

    dtype = torch.float16
    torch.manual_seed(cin * 3 + cout + h)
    x = torch.randn(n, cin, h, w)
    wt = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt.to(dtype).float(), b, 1, 1))
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x, cs_extra=8, c_off=8)  # channel slice of a wider buffer
    ybuf = plan.alloc(n, h, w, cout + 8)
    ybuf.torch().zero_()
    yv = ybuf.cslice(8, cout)
    rv, mode = None, _lib.RES_NONE
    if res:
        r = torch.randn(n, cout, h, w)
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD
        ref = r.to(dtype).float() + ref
    emit_dense(plan, xv, yv, wt, b, 1, 1, 1, _lib.ACT_SILU, rv, mode)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **_tol(dtype))
    # the channels either side of the slice are untouched
    full = ybuf.torch().float().cpu()
    assert torch.count_nonzero(full[..., :8]) == 0 and torch.count_nonzero(full[..., 8 + cout:]) == 0


@pytest.mark.parametrize("cin,cout,k,n,h,w,res,s", [
    (64, 64, 3, 2, 160, 160, "add", 1),  # halo-tiled kernel (>= 51200 px)
    (96, 40, 3, 2, 19, 23, None, 1),     # block implicit GEMM, Cout tail
    (128, 128, 1, 2, 24, 40, "add", 1),  # pointwise GEMM
    (128, 64, 3, 1, 20, 20, None, 1),    # K = 1152: wave-split-K
    (512, 96, 1, 2, 10, 10, None, 1),    # K = 512 on a small map: wave-split-K pointwise
    (64, 64, 3, 8, 320, 320, None, 2),   # stride-2 halo route (>= 204800 output px: 8 x 160 x 160)
    (64, 48, 3, 2, 37, 45, None, 2),     # stride 2 on the block GEMM, odd map
])
def test_conv_fp8(cin, cout, k, n, h, w, res, s):
    """e4m3 operands (BASELINE config 5): GPU fp8 MFMA vs a CPU emulation that applies the same
    quantization (per-channel weight scale, calibrated per-tensor activation scale, saturation)."""
    from ydbl import _lib
    from ydbl.nn.modules import emit_dense
    from ydbl.quant import E4M3_MAX, e4m3_round, enable_fp8, quantize_weights_e4m3

    torch.manual_seed(cin + cout + k + h)
    x = torch.randn(n, cin, h, w) * 2.0
    wt = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    b = torch.randn(cout)
    plan = _plan(torch.float16)
    xv = _tv_from_nchw(plan, x)
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    ybuf = plan.alloc(n, ho, wo, cout + 8)
    yv = ybuf.cslice(8, cout)
    rv, mode = None, _lib.RES_NONE
    r = torch.randn(n, cout, ho, wo)
    if res:
        rv = _tv_from_nchw(plan, r)
        mode = _lib.RES_ADD
    emit_dense(plan, xv, yv, wt, b, s, k // 2, 1, _lib.ACT_SILU, rv, mode)
    assert len(plan.fp8_candidates) == 1
    assert enable_fp8(plan, plan.run) == 1
    _run(plan)
    # CPU emulation of the quantized conv
    x16 = x.half().float()
    qs = E4M3_MAX / x16.abs().max().item()
    xq = e4m3_round(x16 * qs)
    w2 = wt.permute(0, 2, 3, 1).reshape(cout, -1)
    wq, sw = quantize_weights_e4m3(w2)
    wdq = wq.view(torch.float8_e4m3fn).float().reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    acc = F.conv2d(xq, wdq, None, s, k // 2) / (sw[None, :, None, None] * qs)
    ref = F.silu(acc + b[None, :, None, None])
    if res:
        ref = r.half().float() + ref
    got = yv.nchw().float().cpu()
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)
    # and the quantized conv stays close to the exact one (sanity of the scales)
    exact = F.silu(F.conv2d(x16, wt, b, s, k // 2)) + (r.half().float() if res else 0)
    assert (got - exact).abs().mean().item() < 0.05


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("c,c2,shape", [(64, 64, (2, 64, 40, 40)), (128, 64, (2, 128, 20, 21)), (64, 80, (1, 64, 13, 17))])
def test_detect_dw_pw_fused(dtype, c, c2, shape, monkeypatch):
    """Detect cv3 pair DWConv(c,c,3) -> Conv(c,c2,1) (head.py:93-101) as one fused depthwise->pointwise
    launch: dw bias + SiLU applied in LDS before the pointwise MFMA (forced with YDBL_DWPW=1: by default only
    c2 <= 64 takes it, modules.dwpw_fuse)."""
    monkeypatch.setenv("YDBL_DWPW", "1")
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(c + c2)
    ref = torch.nn.Sequential(om.DWConv(c, c, 3), om.Conv(c, c2, 1)).eval()
    with torch.no_grad():
        for bn in [m for m in ref.modules() if isinstance(m, torch.nn.BatchNorm2d)]:
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 2.0)
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
    dwc, pwc = M.DWConv(c, c, 3), M.Conv(c, c2, 1)
    dwc.load_state_dict(ref[0].state_dict())
    pwc.load_state_dict(ref[1].state_dict())
    x = torch.randn(*shape)
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x)
    y, _ = M.emit_dw_pw(plan, dwc, pwc, xv)
    assert [st.fn.__name__ for st in plan.steps] == ["ydbl_dsconv_nhwc"]
    _run(plan)
    with torch.no_grad():
        r = ref(x.to(dtype).float())
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.nchw().float().cpu(), r, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("nc,shape", [(3, (2, 64, 40, 40)), (1, (1, 64, 13, 17)), (4, (3, 64, 80, 80))])
def test_detect_cls_tail_fused(dtype, nc, shape):
    """Detect cv3[i][1] pair DWConv(64,64,3) -> Conv(64,64,1) plus the class conv cv3[i][2] = Conv2d(64,nc,1,bias)
    (head.py:93-101) in one launch: the class logits land in the level buffer's class slice."""
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(nc * 10 + shape[2])
    ref = torch.nn.Sequential(om.DWConv(64, 64, 3), om.Conv(64, 64, 1)).eval()
    cls = torch.nn.Conv2d(64, nc, 1)
    with torch.no_grad():
        for bn in [m for m in ref.modules() if isinstance(m, torch.nn.BatchNorm2d)]:
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 2.0)
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
    dwc, pwc = M.DWConv(64, 64, 3), M.Conv(64, 64, 1)
    dwc.load_state_dict(ref[0].state_dict())
    pwc.load_state_dict(ref[1].state_dict())
    x = torch.randn(*shape)
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x)
    n, _, h, w = shape
    lv = plan.alloc(n, h, w, 64 + nc)
    lv.torch().zero_()
    y, done = M.emit_dw_pw(plan, dwc, pwc, xv, tail_conv=cls, tail_out=lv.cslice(64, nc))
    assert done and [st.fn.__name__ for st in plan.steps] == ["ydbl_dsconv_nhwc"]
    _run(plan)
    with torch.no_grad():
        u = ref(x.to(dtype).float()).to(dtype).float()  # the pair's output as the unfused path stores it
        r = torch.nn.functional.conv2d(u, cls.weight.to(dtype).float() if dtype == torch.float16 else cls.weight,
                                       cls.bias)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.nchw().float().cpu(), u, **tol)
    torch.testing.assert_close(lv.cslice(64, nc).nchw().float().cpu(), r, **tol)
    assert torch.count_nonzero(lv.torch()[..., :64].float()) == 0  # box slice untouched


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("late", ["x0", "x1"])
def test_fullpad_fused_into_conv(dtype, late):
    """FullPAD_Tunnel (block.py:1954-1956) on conv outputs becomes the producing conv's second output:
    the gate_add launch disappears and y = x0 + gate * x1 is unchanged."""
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(7)
    n, c, h, w = 2, 32, 12, 20
    x = torch.randn(n, 16, h, w)
    convs = [M.Conv(16, c, 3, 1).eval(), M.Conv(16, c, 1, 1).eval()]
    refs = [om.Conv(16, c, 3, 1).eval(), om.Conv(16, c, 1, 1).eval()]
    for cv, rf in zip(convs, refs):
        with torch.no_grad():
            rf.bn.running_mean.uniform_(-0.2, 0.2)
            rf.bn.running_var.uniform_(0.5, 2.0)
        cv.load_state_dict(rf.state_dict())
    pad, opad = M.FullPAD_Tunnel(), om.FullPAD_Tunnel()
    with torch.no_grad():
        opad.gate.fill_(0.37)
    pad.load_state_dict(opad.state_dict())
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x)
    ya, yb = convs[0].emit(plan, xv), convs[1].emit(plan, xv)  # yb is produced last
    xs = [ya, yb] if late == "x1" else [yb, ya]
    out = pad.emit(plan, xs)
    assert not any(st.what == "FullPAD" for st in plan.steps)
    _run(plan)
    with torch.no_grad():
        ra, rb = refs[0](x.to(dtype).float()), refs[1](x.to(dtype).float())
        ref = opad([ra, rb] if late == "x1" else [rb, ra])
    tol = _tol(dtype) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(out.nchw().float().cpu(), ref, **tol)
    torch.testing.assert_close(yb.nchw().float().cpu(), rb, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_fullpad_fused_into_dysample(dtype):
    """FullPAD_Tunnel fed by a DySample (DBL L16 = FullPAD(x7, DySample(x12))) becomes the DySample launch's
    second output: no gate_add launch, y = x0 + gate * x1 and the DySample output itself unchanged."""
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(11)
    o = om.DySample(64).eval()
    with torch.no_grad():
        o.offset.weight.normal_(0, 0.3)
        o.offset.bias.normal_(0, 1.0)
    ds = M.DySample(64)
    ds.load_state_dict(o.state_dict())
    pad, opad = M.FullPAD_Tunnel(), om.FullPAD_Tunnel()
    with torch.no_grad():
        opad.gate.fill_(0.61)
    pad.load_state_dict(opad.state_dict())
    x = torch.randn(2, 64, 9, 7)
    z = torch.randn(2, 32, 18, 14)
    ca, oca = M.Conv(32, 64, 1).eval(), om.Conv(32, 64, 1).eval()  # x0 comes from an earlier conv launch
    ca.load_state_dict(oca.state_dict())
    plan = _plan(dtype)
    xv, zv = _tv_from_nchw(plan, x), _tv_from_nchw(plan, z)
    av = ca.emit(plan, zv)
    y = ds.emit(plan, xv)
    out = pad.emit(plan, [av, y])
    assert not any(st.what == "FullPAD" for st in plan.steps)
    _run(plan)
    with torch.no_grad():
        ry = o(x.to(dtype).float())
        ra = oca(z.to(dtype).float())
        ref = opad([ra.to(dtype).float(), ry.to(dtype).float()])
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y.nchw().float().cpu(), ry, **tol)
    torch.testing.assert_close(out.nchw().float().cpu(), ref, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("c,k,s,d,bias,res", [(16, 3, 1, 1, False, False), (32, 3, 2, 1, True, False),
                                             (64, 7, 1, 1, False, True), (24, 5, 1, 1, True, False),
                                             (16, 7, 1, 3, True, False), (16, 3, 1, 2, False, False),
                                             (40, 5, 2, 1, True, True)])
def test_dwconv(dtype, c, k, s, d, bias, res):
    from ydbl.nn.modules import emit_dw

    torch.manual_seed(c + k)
    n, h, w = 2, 17, 15
    x = torch.randn(n, c, h, w)
    wt = torch.randn(c, 1, k, k) / k
    b = torch.randn(c) if bias else None
    p = d * (k - 1) // 2
    ref = F.conv2d(x.to(dtype).float(), wt, b, s, p, d, groups=c)
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x)
    ho, wo = ref.shape[2:]
    yv = plan.alloc(n, ho, wo, c)
    rv = None
    if res:
        r = torch.randn(n, c, ho, wo)
        rv = _tv_from_nchw(plan, r)
        ref = r.to(dtype).float() + ref
    emit_dw(plan, xv, yv, wt, b, s, p, d, res=rv)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **_tol(dtype))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cout,s,h,w", [(8, 1, 14, 19), (16, 2, 16, 22), (32, 1, 9, 40), (64, 2, 7, 33),
                                          (8, 1, 21, 64), (16, 2, 17, 36), (16, 1, 6, 1280)])
def test_stem(dtype, cout, s, h, w):
    """ydbl_conv_stem (preprocess + first Conv) vs conv2d on the dtype-rounded image."""
    from ydbl import _lib

    torch.manual_seed(cout + s)
    n = 3
    x = torch.rand(n, 3, h, w)
    wt = torch.randn(cout, 3, 3, 3) / 27 ** 0.5
    b = torch.randn(cout)
    ref = F.silu(F.conv2d(x.to(dtype).float(), wt, b, s, 1))
    plan = _plan(dtype)
    ho, wo = ref.shape[2:]
    yv = plan.alloc(n, ho, wo, cout)
    xd, wd, bd = x.to(DEV), wt.to(DEV), b.to(DEV)
    plan.launch("ydbl_conv_stem", xd.data_ptr(), n, 3, h, w, 1.0, wd.data_ptr(), bd.data_ptr(), 3, s,
                _lib.ACT_SILU, yv.struct(), None)
    _run(plan)
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, **tol)


@pytest.mark.parametrize("c0,n,h,w", [(8, 2, 64, 64), (16, 2, 37, 53), (8, 1, 640, 640), (16, 3, 17, 100),
                                       (8, 2, 3, 5), (16, 1, 256, 320),
                                       # > 1024 tiles: the persistent walk with next-tile prefetch (V4 and scalar loads)
                                       (8, 4, 640, 640), (16, 4, 480, 640), (8, 3, 642, 638)])
def test_stem2(c0, n, h, w):
    """ydbl_conv_stem2 (preprocess + Conv s1 + Conv s2, fp16) vs the two convs in fp32 on fp16-rounded
    operands, the intermediate rounded to fp16 as the unfused path stores it."""
    from ydbl import _lib

    torch.manual_seed(c0 + h)
    x = torch.rand(n, 3, h, w)
    w0 = torch.randn(c0, 3, 3, 3) / 27 ** 0.5
    b0 = torch.randn(c0) * 0.5
    w1 = torch.randn(2 * c0, c0, 3, 3) / (9 * c0) ** 0.5
    b1 = torch.randn(2 * c0) * 0.5
    h16 = lambda t: t.half().float()
    mid = h16(F.silu(F.conv2d(h16(x), h16(w0), b0, 1, 1)))
    ref = F.silu(F.conv2d(mid, h16(w1), b1, 2, 1))
    plan = _plan(torch.float16)
    ho, wo = ref.shape[2:]
    yv = plan.alloc(n, ho, wo, 2 * c0, cs=2 * c0 + 8)  # channel stride wider than c (concat slice)
    host = torch.empty(int(_lib.lib.ydbl_conv_stem2_params_size(c0)), dtype=torch.uint8)
    _lib.check(_lib.lib.ydbl_conv_stem2_pack(w0.data_ptr(), b0.data_ptr(), w1.data_ptr(), b1.data_ptr(), c0,
                                             host.data_ptr()))
    params = host.to(DEV)
    xd = x.to(DEV)
    d = _lib.Stem2Desc(xd.data_ptr(), n, 3, h, w, 1.0, c0, params.data_ptr(), yv.struct())
    plan.launch("ydbl_conv_stem2", d)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("c,n,h,w,add,tile_h,cs_extra,cm", [
    (16, 2, 64, 64, True, 0, 0, 0), (32, 1, 37, 53, True, 0, 8, 0), (64, 2, 80, 80, True, 0, 0, 0),
    (64, 1, 17, 100, False, 8, 0, 0), (16, 3, 5, 3, True, 16, 8, 0), (32, 2, 40, 48, False, 16, 0, 0),
    (64, 3, 48, 33, True, 16, 16, 0), (16, 1, 1, 1, True, 8, 0, 0), (64, 8, 80, 80, True, 8, 0, 0),
    # c_mid = 64: the Detect box branch Conv(64,64,3) -> Conv(64,64,3) (head.py:86-90)
    (64, 2, 80, 80, False, 0, 0, 64), (64, 3, 37, 29, False, 8, 8, 64), (64, 1, 5, 3, True, 0, 0, 64),
    # more tiles than resident workgroups (ragged maps, channel slices): several tiles per workgroup wherever the
    # walk is persistent
    (16, 4, 320, 320, True, 16, 8, 0), (32, 3, 165, 158, True, 0, 0, 0), (16, 2, 331, 318, False, 0, 8, 0),
    # 9-row tiles (c 64 / c_mid 32): forced, ragged, and the auto choice at DBL-n's 80^2 bs16 sub-batch
    (64, 2, 80, 80, True, 9, 0, 0), (64, 3, 37, 29, True, 9, 8, 0), (64, 1, 10, 17, False, 9, 0, 0),
    (64, 16, 80, 80, True, 0, 0, 0)])
def test_bottleneck_fused(c, n, h, w, add, tile_h, cs_extra, cm):
    """ydbl_bottleneck_nhwc (cv1 3x3 c->c_mid, cv2 3x3 c_mid->c, SiLU, optional x + ..., fp16) vs the two
    convs in fp32 on fp16-rounded operands, the intermediate rounded to fp16 as the unfused path stores it
    (U/nn/modules/block.py:355-357)."""
    from ydbl import _lib

    torch.manual_seed(c * 7 + h + cm)
    cmid = cm
    cm = cm or c // 2
    x = torch.randn(n, c, h, w)
    w1 = torch.randn(cm, c, 3, 3) / (9 * c) ** 0.5
    b1 = torch.randn(cm) * 0.5
    w2 = torch.randn(c, cm, 3, 3) / (9 * cm) ** 0.5
    b2 = torch.randn(c) * 0.5
    h16 = lambda t: t.half().float()
    mid = h16(F.silu(F.conv2d(h16(x), h16(w1), b1, 1, 1)))
    ref = F.silu(F.conv2d(mid, h16(w2), b2, 1, 1))
    if add:
        ref = ref + h16(x)
    plan = _plan(torch.float16)
    xv = _tv_from_nchw(plan, x, cs_extra=cs_extra)
    yv = plan.alloc(n, h, w, c, cs=c + cs_extra)  # channel stride wider than c (concat slice)
    if cmid:
        host = torch.empty(int(_lib.lib.ydbl_conv3x3_pair_params_size(c, cm)), dtype=torch.uint8)
        _lib.check(_lib.lib.ydbl_conv3x3_pair_pack(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), c,
                                                   cm, host.data_ptr()))
    else:
        host = torch.empty(int(_lib.lib.ydbl_bottleneck_params_size(c)), dtype=torch.uint8)
        _lib.check(_lib.lib.ydbl_bottleneck_pack(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), c,
                                                 host.data_ptr()))
    params = host.to(DEV)
    d = _lib.BottleneckDesc(xv.struct(), yv.struct(), c, int(add), tile_h, params.data_ptr(), cmid)
    plan.launch("ydbl_bottleneck_nhwc", d)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("cin,n,h,w,cs_extra", [(64, 2, 80, 80, 0), (64, 3, 37, 29, 8), (64, 1, 5, 3, 0),
                                               (128, 2, 40, 40, 0), (128, 3, 21, 19, 8), (128, 1, 3, 7, 0)])
def test_detect_box_fused(cin, n, h, w, cs_extra):
    """Detect box branch cv2[i] = Conv3x3(cin,64) -> Conv3x3(64,64) -> Conv2d 1x1(64,64)+bias (head.py:86-90) as
    one ydbl_bottleneck_nhwc launch (pw = 1), written into a channel slice of the level buffer; vs fp32
    convs on fp16-rounded operands with both intermediates rounded to fp16 as the unfused path stores them."""
    from ydbl import _lib

    torch.manual_seed(n * 100 + h + cin)
    c = 64
    x = torch.randn(n, cin, h, w)
    w1, b1 = torch.randn(c, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(c) * 0.5
    w2, b2 = torch.randn(c, c, 3, 3) / (9 * c) ** 0.5, torch.randn(c) * 0.5
    w3, b3 = torch.randn(c, c) / c ** 0.5, torch.randn(c) * 0.5
    h16 = lambda t: t.half().float()
    m1 = h16(F.silu(F.conv2d(h16(x), h16(w1), b1, 1, 1)))
    m2 = h16(F.silu(F.conv2d(m1, h16(w2), b2, 1, 1)))
    ref = F.conv2d(m2, h16(w3).reshape(c, c, 1, 1), b3)
    plan = _plan(torch.float16)
    xv = _tv_from_nchw(plan, x, cs_extra=cs_extra)
    lv = plan.alloc(n, h, w, c + 8)  # level buffer [box 64 | cls], box written as a channel slice
    lv.torch().zero_()
    yv = lv.cslice(0, c)
    host = torch.empty(int(_lib.lib.ydbl_detect_box_params_size(cin, c)), dtype=torch.uint8)
    _lib.check(_lib.lib.ydbl_detect_box_pack(*[t.contiguous().data_ptr() for t in (w1, b1, w2, b2, w3, b3)], cin, c,
                                             host.data_ptr()))
    params = host.to(DEV)
    d = _lib.BottleneckDesc(xv.struct(), yv.struct(), c, 0, 0, params.data_ptr(), c, 1)
    plan.launch("ydbl_bottleneck_nhwc", d)
    _run(plan)
    torch.testing.assert_close(yv.nchw().float().cpu(), ref, rtol=1e-2, atol=1e-2)
    assert torch.count_nonzero(lv.torch()[..., c:].float()) == 0  # the class slice is untouched


def test_bottleneck_rejects_bad_shapes():
    import ctypes

    from ydbl import _lib

    plan = _plan(torch.float16)
    params = torch.zeros(64, dtype=torch.uint8, device=DEV)
    for c, xs, ys, tile_h in [(48, (1, 8, 8, 48), (1, 8, 8, 48), 0), (32, (1, 8, 8, 32), (1, 8, 9, 32), 0),
                              (32, (1, 8, 8, 32), (1, 8, 8, 32), 4), (32, (1, 8, 8, 32), (1, 8, 8, 32), 9)]:
        xv, yv = plan.alloc(*xs), plan.alloc(*ys)
        d = _lib.BottleneckDesc(xv.struct(), yv.struct(), c, 1, tile_h, params.data_ptr())
        assert _lib.lib.ydbl_bottleneck_nhwc(ctypes.byref(d), None) != 0
    assert _lib.lib.ydbl_bottleneck_params_size(48) == -1
    assert _lib.lib.ydbl_conv3x3_pair_params_size(32, 32) == -1
    xv, yv = plan.alloc(1, 16, 16, 64), plan.alloc(1, 16, 16, 64)
    d = _lib.BottleneckDesc(xv.struct(), yv.struct(), 64, 0, 16, params.data_ptr(), 64)  # c_mid 64: 8-row only
    assert _lib.lib.ydbl_bottleneck_nhwc(ctypes.byref(d), None) != 0


def _module_parity(o_mod, p_mod, xs, dtype, tol, multi=False, whats=()):
    """Run oracle module (CPU fp32) and product module (GPU) on the same inputs/weights."""
    p_mod.load_state_dict(o_mod.state_dict())
    with torch.no_grad():
        ref = o_mod(xs if multi else xs[0])
    plan = _plan(dtype)
    views = [_tv_from_nchw(plan, x) for x in xs]
    out = p_mod.emit(plan, views if multi else views[0])
    for w in whats:  # launches the plan builder must have emitted (fusion rules)
        assert any(st.what == w for st in plan.steps), (w, [st.what for st in plan.steps])
    _run(plan)
    got = out.nchw().float().cpu()
    torch.testing.assert_close(got, ref, **tol)
    return got, ref


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_dysample(dtype):
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(3)
    o = om.DySample(64).eval()
    with torch.no_grad():
        o.offset.weight.normal_(0, 0.3)  # offsets large enough to cross pixels and hit the border clamp
        o.offset.bias.normal_(0, 1.0)
    x = torch.randn(2, 64, 9, 7)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    _module_parity(o, M.DySample(64), [x], dtype, tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("c,h,w", [(256, 20, 20), (64, 16, 32), (128, 7, 5)])
def test_dw_pair_bit_identical(dtype, c, h, w):
    """ydbl_dwconv2d_pair_nhwc (whole map in LDS) == the two ydbl_dwconv2d_nhwc launches, bit for bit."""
    import torch.nn as nn

    from ydbl.nn import modules as M

    torch.manual_seed(c + h)
    c0 = nn.Conv2d(c, c, 5, padding=2, groups=c)
    c1 = nn.Conv2d(c, c, 7, padding=9, groups=c, dilation=3)
    x = torch.randn(3, c, h, w)
    plan = _plan(dtype)
    xv = _tv_from_nchw(plan, x)
    a1, a2 = M.emit_dw_pair(plan, c0, c1, xv)
    b1 = M.emit_conv2d(plan, c0, xv, None)
    b2 = M.emit_conv2d(plan, c1, b1, None)
    _run(plan)
    assert torch.equal(a1.torch(), b1.torch()) and torch.equal(a2.torch(), b2.torch())
    ref1 = F.conv2d(x.to(dtype).float(), c0.weight.detach(), c0.bias.detach(), 1, 2, 1, c)
    torch.testing.assert_close(a1.nchw().float().cpu(), ref1, **_tol(dtype))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("c,h,w", [(64, 12, 10), (256, 20, 20), (512, 9, 13), (64, 24, 24)])
def test_lskblock(dtype, c, h, w):
    """64 ch: per-thread 7x7 squeeze taps; 256/512 ch (DBL-n/s): taps split over 16 lanes + shuffles.
    H*W <= 512: conv0 -> conv_spatial as one whole-map launch; 24x24: the two-launch fallback."""
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(4 + c)
    o = om.LSKblock(c).eval()
    x = torch.randn(2, c, h, w)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    _module_parity(o, M.LSKblock(c), [x], dtype, tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("c,edges,n,h,w", [
    (64, 4, 2, 10, 8), (128, 8, 2, 10, 8),
    # production token counts: the softmax over N runs over ceil(N/256) logits workgroups whose
    # partial (max, sum) pairs are merged (hg.hip) -- DBL-n/s P4 @640 (N=1600), DBL-l P4 @1280 (N=6400,
    # 16 heads), and a ragged N=257 (one token in the second workgroup)
    (64, 4, 2, 40, 40), (128, 8, 2, 40, 40), (256, 8, 1, 80, 80), (64, 4, 1, 1, 257),
])
@pytest.mark.parametrize("path", ["fused", "staged"])
def test_c3ah_hypergraph(dtype, c, edges, n, h, w, path, monkeypatch):
    """AdaHyperedgeGen softmax over tokens (U/nn/modules/block.py:1652-1657) and AdaHGConv propagation, through
    the one-launch ydbl_hg_fused (where its LDS holds N x E logits: dim 64/128) and the staged
    hg_context + pre_head_proj conv + hg_propagate path (YDBL_HG_UNFUSED)."""
    from oracle import model as om
    from ydbl.nn import modules as M

    if path == "staged":
        monkeypatch.setenv("YDBL_HG_UNFUSED", "1")
    torch.manual_seed(5)
    o = om.C3AH(c, c, 1, edges).eval()
    x = torch.randn(n, c, h, w)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    _module_parity(o, M.C3AH(c, c, 1, edges), [x], dtype, tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_hyperace(dtype):
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(6)
    args = (64, 64, 1, 4, True, True, 0.5, 1, "both", True)
    o = om.HyperACE(*args).eval()
    xs = [torch.randn(2, 64, 16, 16), torch.randn(2, 64, 8, 8), torch.randn(2, 128, 4, 4)]
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    # both C3AH branches' input 1x1s as one launch (HyperACE._emit_branches)
    _module_parity(o, M.HyperACE(*args), xs, dtype, tol, multi=True, whats=("C3AHx2.cv1|cv2",))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("cin,cout,k,s,shape", [
    (64, 64, 3, 1, (2, 64, 20, 19)), (64, 64, 7, 1, (2, 64, 17, 23)), (128, 128, 3, 2, (2, 128, 20, 20)),
    (128, 256, 3, 2, (1, 128, 18, 18)), (32, 32, 7, 1, (3, 32, 9, 13)), (64, 48, 5, 1, (2, 64, 11, 12)),
    # whole-row tiles: 40-wide (TH 4) and 20-wide (TH 8) outputs, ragged last row band, XCD remap
    (64, 64, 7, 1, (2, 64, 14, 40)), (64, 64, 3, 1, (2, 64, 40, 40)), (128, 128, 3, 2, (2, 128, 18, 80)),
    (128, 256, 3, 2, (2, 128, 40, 40)), (32, 32, 7, 1, (2, 32, 20, 20)), (128, 128, 7, 1, (1, 128, 20, 20)),
    (128, 128, 3, 1, (4, 128, 128, 80)),  # Cout 128 in one workgroup (NTN 8)
])
def test_dsconv_fused(dtype, cin, cout, k, s, shape):
    """DSConv (dw -> pw -> BN -> SiLU) through the single-kernel ydbl_dsconv_nhwc path vs the oracle module."""
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(cin + cout + k)
    o = om.DSConv(cin, cout, k, s).eval()
    with torch.no_grad():
        for bn in [m for m in o.modules() if isinstance(m, torch.nn.BatchNorm2d)]:
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 2.0)
            bn.weight.uniform_(0.5, 1.5)
    x = torch.randn(*shape)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    p_mod = M.DSConv(cin, cout, k, s)
    plan = _plan(dtype)
    assert M.fused_dsconv_ok(p_mod.dw, _tv_from_nchw(plan, x), dtype)
    _module_parity(o, p_mod, [x], dtype, tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("name,args,shape", [
    ("DSC3k2", (32, 32, 2, True), (2, 32, 12, 12)),
    ("DSC3k2", (32, 48, 1, False), (2, 32, 12, 12)),
    ("C3Ghost", (64, 64, 2), (2, 64, 10, 10)),
    ("Bottleneck", (16, 16), (2, 16, 14, 14)),
    ("DownsampleConv", (32,), (2, 32, 12, 12)),
])
def test_blocks(dtype, name, args, shape):
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(7)
    o = getattr(om, name)(*args).eval()
    with torch.no_grad():
        for mod in o.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_var.uniform_(0.5, 2.0)
                mod.running_mean.normal_(0, 0.1)
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.normal_(0, 0.1)
                mod.eps = 1e-3
    p = getattr(M, name)(*args)
    for mod in p.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.eps = 1e-3
    # the product folds BN like fuse(); compare against the oracle's fused module
    from oracle.model import fuse_conv_and_bn

    p.load_state_dict(o.state_dict())
    for mod in o.modules():
        if isinstance(mod, om.Conv) and hasattr(mod, "bn"):
            mod.conv = fuse_conv_and_bn(mod.conv, mod.bn)
            delattr(mod, "bn")
    x = torch.randn(*shape)
    with torch.no_grad():
        ref = o(x)
    plan = _plan(dtype)
    out = p.emit(plan, _tv_from_nchw(plan, x))
    _run(plan)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(out.nchw().float().cpu(), ref, **tol)


# ------------------------------------------------------------------------------------ decode + NMS
def _decode_inputs(nc, n=2, shapes=((16, 16), (8, 8), (4, 4)), seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(n, 64 + nc, h, w, generator=g) * 2 for h, w in shapes]


@pytest.mark.parametrize("nc", [3, 80])
def test_decode_matches_detect_inference(nc):
    from oracle import model as om
    from ydbl import _lib
    from ydbl.runtime import Plan

    feats = _decode_inputs(nc)
    d = om.Detect(nc, ch=(16, 16, 16))
    d.stride = torch.tensor([8.0, 16.0, 32.0])
    ref = d._inference([f.clone() for f in feats])
    plan = Plan(torch.device(DEV), torch.float32)
    levels = [_tv_from_nchw(plan, f) for f in feats]
    import ctypes as C

    A = sum(f.shape[2] * f.shape[3] for f in feats)
    yref = torch.empty(2, 4 + nc, A, device=DEV)
    cap = A * nc
    cb = torch.empty(2, cap, 4, device=DEV)
    cs = torch.empty(2, cap, device=DEV)
    cc = torch.empty(2, cap, dtype=torch.int32, device=DEV)
    ci = torch.empty(2, cap, dtype=torch.int32, device=DEV)
    cn = torch.empty(2, dtype=torch.int32, device=DEV)
    dd = _lib.DecodeDesc((_lib.View * 3)(*[lv.cslice(0, 64).struct() for lv in levels]),
                         (_lib.View * 3)(*[lv.cslice(64, nc).struct() for lv in levels]), 3, nc,
                         (C.c_float * 3)(8, 16, 32), 0.5, 1, None, 0, yref.data_ptr(), cb.data_ptr(), cs.data_ptr(),
                         cc.data_ptr(), ci.data_ptr(), cn.data_ptr(), cap)
    plan.launch("ydbl_detect_decode", dd, keep=[dd])
    _run(plan)
    torch.testing.assert_close(yref.cpu(), ref, rtol=1e-5, atol=1e-4)
    # candidate set == (anchor, class) pairs with score > 0.5
    for b in range(2):
        n = cn[b].item()
        got = sorted(ci[b, :n].tolist())
        sc = ref[b, 4:]  # [nc, A]
        j, a = torch.where(sc > 0.5)
        assert got == sorted((a * nc + j).tolist())
    # without the reference-layout output the kernel skips the DFL box for non-candidate anchors:
    # same candidates, boxes and scores (multi-label), and single-label = best class per anchor
    def cands(multi):
        cb2, cs2 = torch.empty_like(cb), torch.empty_like(cs)
        cc2, ci2, cn2 = torch.empty_like(cc), torch.empty_like(ci), torch.empty_like(cn)
        d2 = _lib.DecodeDesc((_lib.View * 3)(*[lv.cslice(0, 64).struct() for lv in levels]),
                             (_lib.View * 3)(*[lv.cslice(64, nc).struct() for lv in levels]), 3, nc,
                             (C.c_float * 3)(8, 16, 32), 0.5, multi, None, 0, None, cb2.data_ptr(), cs2.data_ptr(),
                             cc2.data_ptr(), ci2.data_ptr(), cn2.data_ptr(), cap)
        p2 = Plan(torch.device(DEV), torch.float32)
        p2.launch("ydbl_detect_decode", d2, keep=[d2])
        _run(p2)
        return cb2, cs2, cc2, ci2, cn2

    cb2, cs2, cc2, ci2, cn2 = cands(1)
    for b in range(2):
        n = cn[b].item()
        assert cn2[b].item() == n
        o1, o2 = torch.argsort(ci[b, :n]), torch.argsort(ci2[b, :n])
        assert torch.equal(ci[b, :n][o1], ci2[b, :n][o2]) and torch.equal(cs[b, :n][o1], cs2[b, :n][o2])
        assert torch.equal(cb[b, :n][o1], cb2[b, :n][o2])
    cb2, cs2, cc2, ci2, cn2 = cands(0)
    for b in range(2):
        best, bj = ref[b, 4:].max(0)
        keep = torch.where(best > 0.5)[0]
        n = cn2[b].item()
        assert sorted(ci2[b, :n].tolist()) == keep.tolist()
        o = torch.argsort(ci2[b, :n])
        assert torch.equal(cc2[b, :n][o].cpu().long(), bj[keep])


def _rand_pred(n, nc, A, seed, ties=False):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(n, 2, A, generator=g) * 600 + 20
    wh = torch.rand(n, 2, A, generator=g) * 120 + 4
    sc = torch.rand(n, nc, A, generator=g)
    if ties:
        sc = (sc * 8).floor() / 8 + 0.01  # many exactly equal scores
    # clusters of heavily overlapping boxes
    m = A // 3
    xy[:, :, 0 : 3 * m : 3] = xy[:, :, 1 : 3 * m : 3] + 1.5
    return torch.cat([xy, wh, sc], 1)


@pytest.mark.parametrize("case", [
    dict(nc=3, A=2000, conf=0.25, iou=0.7, multi=False),
    dict(nc=3, A=2000, conf=0.25, iou=0.45, multi=False, ties=True),
    dict(nc=80, A=600, conf=0.3, iou=0.7, multi=True),
    dict(nc=5, A=9000, conf=0.001, iou=0.6, multi=True),  # > 4096 candidates: global sort + LDS spill path
    dict(nc=4, A=3000, conf=0.1, iou=0.5, multi=False, agnostic=True),
    dict(nc=6, A=3000, conf=0.2, iou=0.7, multi=False, classes=[1, 4]),
    dict(nc=3, A=5000, conf=0.01, iou=0.7, multi=True, max_det=50),
    dict(nc=3, A=6000, conf=0.01, iou=0.9, multi=True, max_nms=3000),
    dict(nc=3, A=100, conf=0.999, iou=0.7, multi=False),  # (almost) empty
    dict(nc=2, A=4000, conf=0.05, iou=0.6, multi=True),  # 4096 < n <= 8192: LDS sort, global box reads
    dict(nc=1, A=64, conf=0.0, iou=0.0, multi=False),  # iou 0: every overlap suppresses
    dict(nc=3, A=3000, conf=0.2, iou=0.7, multi=False, max_det=1),
    # m <= 960 sorted candidates: the bitmask path (triangular IoU words, chunk-by-chunk sweep)
    dict(nc=3, A=900, conf=0.5, iou=0.7, multi=False),            # ~790 candidates, 13 words per row
    dict(nc=3, A=700, conf=0.25, iou=0.45, multi=False, ties=True),  # equal scores: index order decides
    dict(nc=3, A=800, conf=0.3, iou=0.6, multi=False, max_det=100),  # max_det reached inside a chunk
    dict(nc=2, A=400, conf=0.5, iou=0.7, multi=True),              # multi-label, class offsets
    dict(nc=1, A=500, conf=0.0, iou=0.0, multi=False),             # iou 0 on the bitmask path
    dict(nc=1, A=65, conf=0.0, iou=0.7, multi=False),              # 65 = one full chunk + 1 row
    dict(nc=3, A=1040, conf=0.03, iou=0.7, multi=False),           # 960 < m <= 1024: register sort, chunked sweep
    dict(nc=80, A=8400, conf=0.05, iou=0.7, multi=False, max_det=300),  # many classes: groups of 10 classes
    dict(nc=17, A=3000, conf=0.02, iou=0.6, multi=True, max_det=40),    # max_det cut across the merged lists
    dict(nc=9, A=2500, conf=0.01, iou=0.7, multi=True, max_nms=1500),   # max_nms: whole image in group 0
    # pair-matrix path boundaries: n = 1024 (the largest it takes) and 1025 (sort + sweep)
    dict(nc=1, A=1024, conf=0.0, iou=0.7, multi=False),
    dict(nc=1, A=1025, conf=0.0, iou=0.7, multi=False),
    dict(nc=3, A=1000, conf=0.0, iou=0.5, multi=False, max_nms=700),  # max_nms cut on the pair-matrix path
    dict(nc=2, A=960, conf=0.0, iou=0.7, multi=False, max_det=5),     # max_det inside the first rank block
    # wide pair-matrix path (1024 < n <= 8192: ranks and rank-space rows on the chip, chunked sweep) and past it
    dict(nc=1, A=1188, conf=0.0, iou=0.7, multi=False),             # DBL-s bs8's worst image size: 2 chunks
    dict(nc=3, A=3000, conf=0.0, iou=0.6, multi=False, ties=True),  # 3000, equal scores: index order decides
    dict(nc=1, A=6210, conf=0.0, iou=0.7, multi=False),             # DBL-l 1280's worst image size
    dict(nc=1, A=8192, conf=0.0, iou=0.5, multi=False),             # the largest it takes
    dict(nc=1, A=8193, conf=0.0, iou=0.5, multi=False),             # one more: sort + chunked sweep
    dict(nc=1, A=6000, conf=0.0, iou=0.95, multi=False, max_det=3000),  # thousands of keeps over 6 chunks
    dict(nc=2, A=3000, conf=0.0, iou=0.7, multi=True, max_nms=2500),    # max_nms cut on the wide path
    dict(nc=1, A=2000, conf=0.0, iou=0.0, multi=False),             # iou 0 on the wide path
    dict(nc=3, A=4000, conf=0.0, iou=0.7, multi=False, max_det=700),  # max_det reached in a later chunk
    dict(nc=4, A=9000, conf=0.0, iou=0.7, multi=True),  # 36000 candidates > max_nms 30000: stable truncation
    # > 8192 candidates: radix select of the first max_nms keys, 8192-key buckets sorted in LDS (nms_select_sort)
    dict(nc=80, A=3000, conf=0.001, iou=0.7, multi=True),              # 240000 candidates, 4 buckets
    dict(nc=80, A=3000, conf=0.001, iou=0.6, multi=True, ties=True),   # 240000, 8 score levels: index order decides
    dict(nc=10, A=2000, conf=0.0, iou=0.7, multi=True, max_nms=8192),  # 20000 -> exactly one full bucket
    dict(nc=5, A=2000, conf=0.0, iou=0.7, multi=True, max_nms=32768),  # 10000 < max_nms: every key, 2 buckets
    dict(nc=1, A=30000, conf=0.0, iou=0.95, multi=False, max_det=4096, max_nms=24577),  # bucket 4: one key
])
@pytest.mark.parametrize("groups", ["1", "0"])
@pytest.mark.parametrize("fast", ["1", "0"])
def test_nms_bit_exact(case, groups, fast, monkeypatch):
    """groups "1": the class-split sweep (8 class-group workgroups per image + merge), "0": one workgroup
    per image; fast "1": images with <= 8192 candidates take the pair-matrix path (chip-wide ranks and
    rank-space IoU rows, nms_pair_kernel + nms_mask_kernel, then the chunked rank-order sweep), "0": sort +
    chunked sweep for every image.  All bit-exact against the restated torchvision semantics."""
    from oracle.ops import non_max_suppression as ref_nms
    from ydbl.utils.ops import non_max_suppression

    monkeypatch.setenv("YDBL_NMS_GROUPS", groups)
    monkeypatch.setenv("YDBL_NMS_FAST", fast)
    case = dict(case)
    nc, A = case.pop("nc"), case.pop("A")
    pred = _rand_pred(3, nc, A, seed=A + nc, ties=case.pop("ties", False))
    kw = dict(conf_thres=case["conf"], iou_thres=case["iou"], multi_label=case["multi"],
              agnostic=case.get("agnostic", False), classes=case.get("classes"), max_det=case.get("max_det", 300),
              max_nms=case.get("max_nms", 30000))
    ref = ref_nms(pred.clone(), **kw)
    got = non_max_suppression(pred.to(DEV), **kw)
    for r, g in zip(ref, got):
        assert np.array_equal(g.cpu().numpy(), r.numpy()), (r.shape, g.shape)


def test_golden_nms_from_fixture(golden_dir):
    from ydbl.utils.ops import non_max_suppression

    g = np.load(golden_dir / "golden_n_nc3_128.npz", allow_pickle=False)
    y = torch.from_numpy(g["y"]).to(DEV)
    pred = non_max_suppression(y, 0.05, 0.7)
    val = non_max_suppression(y, 0.001, 0.7, multi_label=True)
    for i in range(2):
        assert np.array_equal(pred[i].cpu().numpy(), g[f"pred{i}"])
        assert np.array_equal(val[i].cpu().numpy(), g[f"val{i}"])


@pytest.mark.parametrize("case", [
    # (kind, cin, cout, k, s, shape, residual, sliced): every dsc_lean.hip instantiation, ragged maps, channel slices
    ("ds", 64, 64, 3, 1, (16, 64, 40, 40), False, False), ("ds", 64, 64, 7, 1, (16, 64, 40, 40), True, False),
    ("ds", 64, 64, 3, 1, (3, 64, 13, 21), True, True), ("ds", 64, 64, 7, 1, (2, 64, 9, 30), True, True),
    ("ds", 128, 128, 3, 1, (4, 128, 20, 20), True, False), ("ds", 128, 128, 7, 1, (4, 128, 20, 20), True, True),
    ("ds", 128, 128, 3, 2, (2, 128, 80, 80), False, False), ("ds", 128, 256, 3, 2, (2, 128, 40, 40), False, True),
    ("ds", 128, 128, 3, 2, (1, 128, 19, 27), False, False),
    ("pair", 64, 64, 3, 1, (2, 64, 80, 80), False, False), ("pair", 128, 64, 3, 1, (2, 128, 40, 40), False, True),
    ("pair", 256, 64, 3, 1, (2, 256, 20, 20), False, False), ("tail", 64, 64, 3, 1, (3, 64, 40, 40), False, False),
    ("tail", 64, 64, 3, 1, (1, 64, 11, 13), False, True),
])
def test_dsconv_lean_bit_identical(case, monkeypatch):
    """dsc_lean.hip (one global round trip, all channels per workgroup) == dsconv.hip's chunked kernel, bit for
    bit (same roundings, same tap and k-step orders), on DSConv (+ the DSBottleneck residual), the stride-2
    DSConvs and the Detect DWConv -> Conv1x1 pairs (+ the class-conv tail); and close to the oracle."""
    from oracle import model as om
    from ydbl import _lib
    from ydbl.nn import modules as M
    from ydbl.utils.synthetic import trained_like_

    kind, cin, cout, k, s, shape, residual, sliced = case
    torch.manual_seed(cin * 7 + cout + k + shape[2])
    x = torch.randn(*shape)
    if kind == "ds":
        o = trained_like_(om.DSConv(cin, cout, k, s), seed=k).eval()
    else:
        o = trained_like_(torch.nn.Sequential(om.DWConv(cin, cin, k), om.Conv(cin, cout, 1)), seed=k).eval()
    cls = torch.nn.Conv2d(cout, 3, 1) if kind == "tail" else None
    ho, wo = (shape[2] + 2 * (k // 2) - k) // s + 1, (shape[3] + 2 * (k // 2) - k) // s + 1
    r = torch.randn(shape[0], cout, ho, wo) if residual else None
    outs = []
    for lean in ("1", "0"):
        monkeypatch.setenv("YDBL_DS_LEAN", lean)
        plan = _plan(torch.float16)
        xv = _tv_from_nchw(plan, x, cs_extra=8 if sliced else 0, c_off=8 if sliced else 0)
        rv = _tv_from_nchw(plan, r, cs_extra=16 if sliced else 0, c_off=16 if sliced else 0) if residual else None
        ybuf = plan.alloc(shape[0], ho, wo, cout + (32 if sliced else 0))
        yv = ybuf.cslice(16, cout) if sliced else ybuf
        tv = plan.alloc(shape[0], ho, wo, 3) if cls is not None else None
        if kind == "ds":
            pm = M.DSConv(cin, cout, k, s)
            pm.load_state_dict(o.state_dict())
            pm.emit(plan, xv, yv, res=rv, res_mode=_lib.RES_ADD if residual else _lib.RES_NONE)
        else:
            dwc, pwc = M.DWConv(cin, cin, k), M.Conv(cin, cout, 1)
            dwc.load_state_dict(o[0].state_dict())
            pwc.load_state_dict(o[1].state_dict())
            _, done = M.emit_dw_pw(plan, dwc, pwc, xv, yv, tail_conv=cls, tail_out=tv)
            assert done == (cls is not None)
        assert [st.fn.__name__ for st in plan.steps] == ["ydbl_dsconv_nhwc"]
        _run(plan)
        outs.append((yv.nchw().float().cpu(), tv.nchw().float().cpu() if tv is not None else None))
    assert torch.equal(outs[0][0], outs[1][0]), (outs[0][0] - outs[1][0]).abs().max()
    if cls is not None:
        assert torch.equal(outs[0][1], outs[1][1])
    with torch.no_grad():
        ref = o(x) + (r if residual else 0)
    torch.testing.assert_close(outs[0][0], ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("c,n,shape,sliced", [(64, 2, (16, 64, 40, 40), False), (64, 1, (3, 64, 13, 21), True),
                                              (128, 2, (4, 128, 20, 20), True)])
def test_dsc3k_cv3_fused_bit_identical(c, n, shape, sliced, monkeypatch):
    """DSC3k (U/nn/modules/block.py:1447-1503, C3 with DSBottlenecks k3 -> k7, e = 1): cv3 as the trailing GEMM of
    the last bottleneck's k7 DSConv (ydbl_dsconv_desc.g2: the bottleneck output stays on the CU) == the separate
    k7 DSConv + cv3 launches, bit for bit; one launch fewer; close to the oracle."""
    from oracle import model as om
    from ydbl.nn import modules as M
    from ydbl.utils.synthetic import trained_like_

    torch.manual_seed(c + n + shape[2])
    o = trained_like_(om.DSC3k(c, c, n, True, e=1.0, k1=3, k2=7), seed=c).eval()
    x = torch.randn(*shape)
    outs, nsteps = [], []
    monkeypatch.setenv("YDBL_CV1_FUSE", "0")  # the leading-1x1 fusion has its own test (below)
    for fuse in ("1", ""):
        if fuse:
            monkeypatch.setenv("YDBL_CV3_FUSE", "1")
        else:
            monkeypatch.setenv("YDBL_CV3_FUSE", "0")
        pm = M.DSC3k(c, c, n, True, e=1.0, k1=3, k2=7)
        pm.load_state_dict(o.state_dict())
        plan = _plan(torch.float16)
        xv = _tv_from_nchw(plan, x)
        ybuf = plan.alloc(shape[0], shape[2], shape[3], c + (24 if sliced else 0))
        yv = ybuf.cslice(8, c) if sliced else ybuf
        pm.emit(plan, xv, yv)
        nsteps.append(len(plan.steps))
        assert any("+cv3" in st.what for st in plan.steps) == bool(fuse)
        _run(plan)
        outs.append(yv.nchw().float().cpu())
    assert nsteps[0] == nsteps[1] - 1
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()
    with torch.no_grad():
        ref = o(x)
    torch.testing.assert_close(outs[0], ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("n,shape,sliced", [(2, (16, 64, 40, 40), False), (1, (3, 64, 13, 21), True),
                                            (2, (2, 64, 9, 7), True)])
def test_dsc3k_cv1_fused_bit_identical(n, shape, sliced, monkeypatch):
    """DSC3k at c_ = 64: the merged cv2 | cv1 1x1 as the leading GEMM of the first bottleneck's k3 DSConv
    (ydbl_dsconv_desc.g0: cv1's map recomputed on the tile halo, zero outside the image, both 1x1 outputs still
    written) == the separate 1x1 + k3 DSConv launches, bit for bit; one launch fewer; close to the oracle."""
    from oracle import model as om
    from ydbl.nn import modules as M
    from ydbl.utils.synthetic import trained_like_

    c = 64
    torch.manual_seed(n + shape[2])
    o = trained_like_(om.DSC3k(c, c, n, True, e=1.0, k1=3, k2=7), seed=7).eval()
    x = torch.randn(*shape)
    outs, nsteps = [], []
    monkeypatch.setenv("YDBL_CV3_FUSE", "1")  # the leading 1x1 rides only in the trailing-GEMM layout (C3.emit)
    for fuse in ("1", ""):
        if fuse:
            monkeypatch.setenv("YDBL_CV1_FUSE", "1")
        else:
            monkeypatch.setenv("YDBL_CV1_FUSE", "0")
        pm = M.DSC3k(c, c, n, True, e=1.0, k1=3, k2=7)
        pm.load_state_dict(o.state_dict())
        plan = _plan(torch.float16)
        xv = _tv_from_nchw(plan, x)
        ybuf = plan.alloc(shape[0], shape[2], shape[3], c + (24 if sliced else 0))
        yv = ybuf.cslice(8, c) if sliced else ybuf
        pm.emit(plan, xv, yv)
        nsteps.append(len(plan.steps))
        assert any(st.what.startswith("Conv1x1x2+") for st in plan.steps) == bool(fuse)
        _run(plan)
        outs.append(yv.nchw().float().cpu())
    assert nsteps[0] == nsteps[1] - 1
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()
    with torch.no_grad():
        ref = o(x)
    torch.testing.assert_close(outs[0], ref, rtol=3e-2, atol=3e-2)


def test_dsconv_g0_rejects_bad_descriptors():
    """ydbl_dsconv_nhwc with a leading 1x1 (g0) refuses, before launching anything, descriptors whose x is not
    the last x.c channels of g0_y, whose channel counts are not (64 -> 128, x.c 64), or that add a residual."""
    import ctypes

    from ydbl import _lib

    plan = _plan(torch.float16)
    n, h, w = 1, 8, 8
    x0 = plan.alloc(n, h, w, 64)
    buf = plan.alloc(n, h, w, 192)
    y0, x, y = buf.cslice(64, 128), buf.cslice(128, 64), plan.alloc(n, h, w, 64)
    dww = torch.zeros(9 * 64, device=DEV)
    pww = torch.zeros(64 * 64, dtype=torch.float16, device=DEV)
    bias = torch.zeros(128, device=DEV)
    w0 = torch.zeros(128 * 64, dtype=torch.float16, device=DEV)
    nv = _lib.View(None, 0, 0, 0, 0, 0, 0)

    def desc(xv, y0v, res=None):
        return _lib.DsConvDesc(xv.struct(), y.struct(), res.struct() if res is not None else nv, dww.data_ptr(),
                               pww.data_ptr(), bias.data_ptr(), 3, 1, 1, 1, 64, _lib.ACT_SILU,
                               _lib.RES_ADD if res is not None else _lib.RES_NONE, None, 0, None, None, nv, 0,
                               None, None, nv, nv, 0, w0.data_ptr(), bias.data_ptr(), x0.struct(), y0v.struct(),
                               _lib.ACT_SILU)
    for d in (desc(buf.cslice(64, 64), y0),        # x is the first half of g0_y, not its last channels
              desc(x, buf.cslice(64, 96)),          # g0_y.c != 2 x.c
              desc(x, y0, res=y)):                  # no residual with g0
        assert _lib.lib.ydbl_dsconv_nhwc(ctypes.byref(d), None) != 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("c,shape,spread,fullpad", [(128, (16, 128, 40, 40), 0.01, False), (256, (4, 256, 20, 20), 0.01, True),
                                                    (64, (2, 64, 13, 17), 0.3, True), (128, (3, 128, 9, 40), 1.0, False)])
def test_dysample_fused_bit_identical(dtype, c, shape, spread, fullpad, monkeypatch):
    """ydbl_dysample2 (offset conv + sample in one launch, the group's tile + 2-px halo in LDS, global fallback
    for corners outside it) == ydbl_conv2d_nhwc + ydbl_dysample_ex, bit for bit, with small (in-window) and
    large (border-clamped, out-of-window) offsets, and with the fused FullPAD second output."""
    from ydbl.nn import modules as M

    torch.manual_seed(c + shape[2])
    ds = M.DySample(c)
    with torch.no_grad():
        ds.offset.weight.normal_(0, spread)
        ds.offset.bias.normal_(0, 10 * spread)
    x = torch.randn(*shape)
    r = torch.randn(shape[0], c, 2 * shape[2], 2 * shape[3])
    outs = []
    for fused in ("", "1"):
        if fused:
            monkeypatch.delenv("YDBL_DS2_OFF", raising=False)
        else:
            monkeypatch.setenv("YDBL_DS2_OFF", "1")
        plan = _plan(dtype)
        xv = _tv_from_nchw(plan, x)
        y = ds.emit(plan, xv)
        assert ("DySample.fused" in [st.what for st in plan.steps]) == bool(fused)
        y2 = None
        if fullpad:
            rv = _tv_from_nchw(plan, r)
            y2 = plan.alloc(shape[0], 2 * shape[2], 2 * shape[3], c)
            assert plan.fuse_second_output(plan.writer_of(y), y2, rv, 0.7, 1.0) is not None
        _run(plan)
        outs.append((y.nchw().float().cpu(), y2.nchw().float().cpu() if y2 is not None else None))
    assert torch.equal(outs[0][0], outs[1][0]), (outs[0][0] - outs[1][0]).abs().max()
    if fullpad:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("c,shape,sliced", [(256, (16, 256, 20, 20), False), (256, (3, 256, 7, 11), True),
                                            (512, (2, 512, 20, 20), False)])
def test_lsk_fused_bit_identical(c, shape, sliced, monkeypatch):
    """ydbl_lsk_attn + ydbl_lsk_out (conv1 | conv2 + stats, gate + conv + x* in two launches) == conv1, conv2,
    ydbl_lsk_gate, conv (RES_MUL): bit for bit at dim 256, where the unfused 1x1s run the block GEMM (at 512 the
    unfused conv1/conv2 take the wave-split-K kernel, another accumulation order: fp16 tolerance there)."""
    from oracle import model as om
    from ydbl.nn import modules as M

    torch.manual_seed(c + shape[2])
    o = om.LSKblock(c).eval()
    m = M.LSKblock(c)
    m.load_state_dict(o.state_dict())
    x = torch.randn(*shape)
    outs = []
    for fused in ("1", ""):
        if fused:
            monkeypatch.setenv("YDBL_LSK_FUSE", "1")
        else:
            monkeypatch.setenv("YDBL_LSK_FUSE", "0")
        plan = _plan(torch.float16)
        xv = _tv_from_nchw(plan, x)
        out = plan.alloc(shape[0], shape[2], shape[3], c + 16).cslice(8, c) if sliced else None
        y = m.emit(plan, xv, out)
        whats = [st.what for st in plan.steps]
        assert ("LSK.gate+conv" in whats) == bool(fused), whats
        _run(plan)
        outs.append(y.nchw().float().cpu())
    if c == 256:
        assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()
    else:
        torch.testing.assert_close(outs[0], outs[1], rtol=2e-3, atol=2e-3)
    with torch.no_grad():
        ref = o(x)
    torch.testing.assert_close(outs[0], ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("n", [1, 7, 4096, 3 * 160 * 160 * 5 + 3, 32 * 3 * 640 * 640])
@pytest.mark.parametrize("kind", ["unit", "x255", "negative", "nan"])
def test_batch_max(n, kind):
    """ydbl_batch_max (predict()'s LoadTensor decision, U/data/loaders.py:561-566) against
    torch.amax: the maximum bit for bit, NaN propagated, scale fp32(1/255) iff max > 1 + FLT_EPSILON."""
    from ydbl import _lib

    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, generator=g)
    if kind == "x255":
        x = x * 255.0
    elif kind == "negative":
        x = -x - 1.0
    elif kind == "nan":
        x[n // 2] = float("nan")
    xd = x.to(DEV)
    work = _lib.batch_max_work(DEV)
    init = work.clone()
    amax, scale = torch.empty(1, device=DEV), torch.empty(1, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(2):  # the work pair is left ready for the next call
        _lib.check(_lib.lib.ydbl_batch_max(xd.data_ptr(), n, work.data_ptr(), amax.data_ptr(), scale.data_ptr(), st))
    torch.cuda.synchronize()
    assert torch.equal(work, init)
    ref = torch.amax(x)
    if kind == "nan":
        assert torch.isnan(amax.cpu()[0]) and scale.item() == 1.0
        return
    assert amax.cpu()[0].item() == ref.item()
    expect = torch.tensor(1.0 / 255.0, dtype=torch.float32).item() if ref.item() > 1.0 + 1.1920928955078125e-07 else 1.0
    assert scale.item() == expect
