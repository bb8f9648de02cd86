"""YOLO-DBL building blocks, MI355X path.

Each class keeps the reference's constructor signature, submodule names and
parameter shapes (so ``parse_model`` resolves the DBL YAMLs by class name and
reference ``state_dict`` keys load unchanged).  Its compute is ``emit``: HIP
launches appended to a ``Plan``:

    y = module.emit(plan, x, out=None)   # x, y: NHWC TV views (lists for multi-input)

and its ``forward(x)`` (the reference's module contract, ``m(x)`` on a tensor or a
list of tensors, U/nn/tasks.py:158-161) compiles that emit into a one-module plan
for x's shapes / dtype / device, caches it, and runs it (``run_module``).  A
registered plugin class WITHOUT ``emit`` -- a plain torch ``forward`` -- runs
inside the model's plan as a captured torch step on NCHW views of its input
(``emit_torch``).

``out`` (optional) is a destination view, typically a channel slice of a
concat buffer, so Concat / chunk / C2f / C3 concatenations cost no copies.
BatchNorm is folded exactly as ``fuse_conv_and_bn`` does
(U/utils/torch_utils.py:238-265); DSConv's BN (left unfused by the reference,
U/nn/tasks.py:217) is folded into its pointwise conv here.
"""

from __future__ import annotations

import ctypes as C
import math
import os

import torch
import torch.nn as nn

from .. import _lib
from .._lib import ConvDesc, DwConvDesc, HgDesc, View
from ..runtime import TV, Plan, Step, round_up, weights_signature, ydbl_env


# =============================================================================== weight prep + launches
def autopad(k, p=None, d=1):
    """U/nn/modules/conv.py:30-36."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


@torch.no_grad()
def fold_bn(weight: torch.Tensor, bias: torch.Tensor | None, bn: nn.BatchNorm2d):
    """Same op sequence as fuse_conv_and_bn (diag-matrix products), fp32 on the host."""
    w = weight.detach().float().cpu()
    co = w.shape[0]
    w_bn = torch.diag(bn.weight.detach().float().cpu().div(torch.sqrt(bn.eps + bn.running_var.float().cpu())))
    wf = torch.mm(w_bn, w.view(co, -1)).view(w.shape)
    b_conv = torch.zeros(co) if bias is None else bias.detach().float().cpu()
    b_bn = bn.bias.detach().float().cpu() - bn.weight.detach().float().cpu().mul(
        bn.running_mean.float().cpu()
    ).div(torch.sqrt(bn.running_var.float().cpu() + bn.eps))
    bf = torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn
    return wf, bf


def _act_code(act) -> int:
    if isinstance(act, nn.SiLU):
        return _lib.ACT_SILU
    if isinstance(act, nn.GELU):
        return _lib.ACT_GELU
    if isinstance(act, nn.Identity) or act is None:
        return _lib.ACT_NONE
    raise NotImplementedError(f"activation {type(act).__name__} has no HIP epilogue")


def vec_aligned(v: TV) -> bool:
    """The 16-byte channel-vector rule of check_view(need_vec_align) (csrc/capi.hip): channel count, channel
    stride and base pointer all in whole 16-byte vectors."""
    vec = 16 // v.base.element_size()
    return v.c % vec == 0 and v.cs % vec == 0 and v.ptr % 16 == 0


def _null_view() -> View:
    return View(None, 0, 0, 0, 0, 0, 0)


def emit_dense(plan: Plan, x: TV, y: TV, w: torch.Tensor, b: torch.Tensor | None, stride=1, pad=0, dil=1,
               act=_lib.ACT_NONE, res: TV | None = None, res_mode=_lib.RES_NONE, what="conv"):
    """Dense conv y = act(conv(x) + b) [+/* res]; w fp32 [co, ci, kh, kw] (ci may be < x.c: zero-padded)."""
    co, ci, kh, kw = w.shape
    assert ci <= x.c and co == y.c, (w.shape, x.shape, y.shape)
    wt = w.permute(0, 2, 3, 1)
    if ci < x.c:
        wt = torch.nn.functional.pad(wt, (0, x.c - ci))
    K = kh * kw * x.c
    kpad = round_up(K, 32)
    wk32 = torch.nn.functional.pad(wt.reshape(co, K).float(), (0, kpad - K))
    wd = plan.const(wk32.to(plan.dtype))
    bd = plan.const(b.float()) if b is not None else None
    d = ConvDesc(x.struct(), y.struct(), res.struct() if res is not None else _null_view(), wd.data_ptr(),
                 bd.data_ptr() if bd is not None else None, kh, kw, stride, pad, dil, kpad, act, res_mode,
                 _null_view(), _null_view(), 0.0, 0.0, None, 1.0)
    ws = None
    if plan.device.type != "meta":  # split-K scratch of the deep-K small-map convs (include/ydbl.h ydbl_conv_workspace)
        nws = int(_lib.lib.ydbl_conv_workspace(d))
        if nws > 0:
            ws = plan.splitk_scratch(nws)
            d.workspace, d.workspace_bytes = ws.data_ptr(), nws
    plan.launch("ydbl_conv2d_nhwc", d, what=what, keep=[wd, bd, d, ws])
    plan.note_writer(y, d)
    if plan.dtype == torch.float16 and x.c >= 64 and not what.startswith("Detect."):
        d._b32 = b.detach().float().cpu() if b is not None else None  # (ydbl.quant's bias correction)
        plan.fp8_candidates.append((d, x, wk32))  # see ydbl.quant: e4m3 operands after calibration
        plan.fp8_layers.append(getattr(plan, "cur_layer", -1))


def dw_desc(plan: Plan, x: TV, y: TV, w: torch.Tensor, b: torch.Tensor | None, stride=1, pad=0, dil=1,
            act=_lib.ACT_NONE, res: TV | None = None):
    """Depthwise conv descriptor (+ the device constants it points at); w fp32 [c, 1, kh, kw]."""
    c, _, kh, kw = w.shape
    assert c == x.c == y.c
    wd = plan.const(w.float().reshape(c, kh * kw).t().contiguous())
    bd = plan.const(b.float()) if b is not None else None
    d = DwConvDesc(x.struct(), y.struct(), res.struct() if res is not None else _null_view(), wd.data_ptr(),
                   bd.data_ptr() if bd is not None else None, kh, kw, stride, pad, dil, act,
                   _lib.RES_ADD if res is not None else _lib.RES_NONE)
    return d, [wd, bd, d]


def emit_dw(plan: Plan, x: TV, y: TV, w: torch.Tensor, b: torch.Tensor | None, stride=1, pad=0, dil=1,
            act=_lib.ACT_NONE, res: TV | None = None, what="dwconv"):
    """Depthwise conv; w fp32 [c, 1, kh, kw]."""
    d, keep = dw_desc(plan, x, y, w, b, stride, pad, dil, act, res)
    plan.launch("ydbl_dwconv2d_nhwc", d, what=what, keep=keep)


def emit_dw_pair(plan: Plan, c0: nn.Conv2d, c1: nn.Conv2d, x: TV, what="dw_pair") -> tuple[TV, TV]:
    """Two chained depthwise nn.Conv2d (c1 reads c0's output) as one ydbl_dwconv2d_pair_nhwc launch
    (the library falls back to two launches for geometries it does not fuse)."""
    descs, keep = [], []
    src, outs = x, []
    for conv in (c0, c1):
        k, s, p, d = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.dilation[0]
        ho, wo = conv_out_hw(src.h, src.w, k, s, p, d)
        y = plan.alloc(src.n, ho, wo, conv.out_channels)
        b = conv.bias.detach().float().cpu() if conv.bias is not None else None
        dd, kk = dw_desc(plan, src, y, conv.weight.detach().float().cpu(), b, s, p, d)
        descs.append(dd)
        keep += kk
        outs.append(y)
        src = y
    plan.launch("ydbl_dwconv2d_pair_nhwc", descs[0], descs[1], what=what, keep=keep)
    return outs[0], outs[1]


def conv_out_hw(h, w, k, s, p, d):
    return (h + 2 * p - d * (k - 1) - 1) // s + 1, (w + 2 * p - d * (k - 1) - 1) // s + 1


def emit_conv2d(plan: Plan, conv: nn.Conv2d, x: TV, out: TV | None, weight=None, bias=None, act=_lib.ACT_NONE,
                res: TV | None = None, res_mode=_lib.RES_NONE, what="conv") -> TV:
    """Launch an nn.Conv2d (dense or depthwise) with optional replacement weight/bias."""
    k, s, p, d = conv.kernel_size[0], conv.stride[0], conv.padding[0], conv.dilation[0]
    assert conv.kernel_size[0] == conv.kernel_size[1] and conv.stride[0] == conv.stride[1]
    w = (conv.weight if weight is None else weight).detach().float().cpu()
    b = bias if bias is not None else (conv.bias.detach().float().cpu() if conv.bias is not None else None)
    ho, wo = conv_out_hw(x.h, x.w, k, s, p, d)
    y = out if out is not None else plan.alloc(x.n, ho, wo, conv.out_channels)
    assert (y.h, y.w, y.c) == (ho, wo, conv.out_channels), ((y.h, y.w, y.c), (ho, wo, conv.out_channels))
    if conv.groups == 1:
        emit_dense(plan, x, y, w, b, s, p, d, act, res, res_mode, what)
    elif conv.groups == conv.in_channels == conv.out_channels:
        if res_mode not in (_lib.RES_NONE, _lib.RES_ADD):
            raise NotImplementedError("depthwise conv supports residual ADD only")
        emit_dw(plan, x, y, w, b, s, p, d, act, res if res_mode == _lib.RES_ADD else None, what)
    else:
        raise NotImplementedError(f"grouped conv g={conv.groups} is not on the DBL path")
    return y


def fused_dsconv_ok(dw: nn.Conv2d, x: TV, dtype) -> bool:
    k, st, d = dw.kernel_size[0], dw.stride[0], dw.dilation[0]
    cc = 32 if dtype == torch.float16 else 16
    return (dw.kernel_size[0] == dw.kernel_size[1] and (k, st, d) in ((3, 1, 1), (3, 2, 1), (5, 1, 1), (7, 1, 1))
            and x.c % cc == 0 and x.c == dw.in_channels)


def emit_dsconv(plan: Plan, dw: nn.Conv2d, x: TV, out: TV | None, w_pw: torch.Tensor, b_pw: torch.Tensor,
                act=_lib.ACT_SILU, res: TV | None = None, res_mode=_lib.RES_NONE, what="DSConv",
                w_dw: torch.Tensor | None = None, b_dw: torch.Tensor | None = None, dw_act=_lib.ACT_NONE,
                tail: tuple | None = None, g2: tuple | None = None, g0: tuple | None = None) -> TV:
    """DSConv (conv.py:91-108) as one ydbl_dsconv_nhwc launch: depthwise tile in LDS feeding the pw MFMA.
    w_dw / b_dw / dw_act: folded DWConv weights, bias and activation (Detect's DWConv -> Conv1x1 pair).
    tail = (w [n, co], b [n], out view): a trailing 1x1 conv with n <= 4 outputs in the same launch.
    g2 = (w [co2, co + c2] fp32, b [co2], x2 view, y2 view, act): a trailing GEMM over [y ; x2] into y2 (C3's
    cv3 after the last bottleneck); y itself is then not stored (include/ydbl.h, ydbl_dsconv_desc.g2).
    g0 = (w [c0y, c0x] fp32, b [c0y], x0 view, y0 view, act): a leading 1x1 y0 = act(w x0 + b) written by the same
    launch, x being y0's last x.c channels, recomputed on the tile halo (C3's merged cv2 | cv1, ydbl_dsconv_desc.g0)."""
    k, st, p, d = dw.kernel_size[0], dw.stride[0], dw.padding[0], dw.dilation[0]
    c = x.c
    co = w_pw.shape[0]
    ho, wo = conv_out_hw(x.h, x.w, k, st, p, d)
    y = out if out is not None else plan.alloc(x.n, ho, wo, co)
    assert (y.h, y.w, y.c) == (ho, wo, co), ((y.h, y.w, y.c), (ho, wo, co))
    wdw = (dw.weight if w_dw is None else w_dw).detach().float().cpu()
    dww = plan.const(wdw.reshape(c, k * k).t().contiguous())
    kpad = round_up(c, 32)
    pww = plan.const(torch.nn.functional.pad(w_pw.reshape(co, c).float(), (0, kpad - c)).to(plan.dtype))
    bd = plan.const(b_pw.float())
    dwb = plan.const(b_dw.float()) if b_dw is not None else None
    tw = tb = None
    tail_args = (None, None, _null_view(), 0)
    if tail is not None:
        tw, tb = plan.const(tail[0].float().contiguous()), plan.const(tail[1].float().contiguous())
        tail_args = (tw.data_ptr(), tb.data_ptr(), tail[2].struct(), tail[2].c)
        what += "+1x1"
    g2w = g2b = None
    g2_args = (None, None, _null_view(), _null_view(), 0)
    if g2 is not None:
        g2w, g2b = plan.const(g2[0].float().to(plan.dtype).contiguous()), plan.const(g2[1].float().contiguous())
        g2_args = (g2w.data_ptr(), g2b.data_ptr(), g2[2].struct(), g2[3].struct(), int(g2[4]))
        what += "+cv3"
    g0w = g0b = None
    g0_args = (None, None, _null_view(), _null_view(), 0)
    if g0 is not None:
        g0w, g0b = plan.const(g0[0].float().to(plan.dtype).contiguous()), plan.const(g0[1].float().contiguous())
        g0_args = (g0w.data_ptr(), g0b.data_ptr(), g0[2].struct(), g0[3].struct(), int(g0[4]))
        what = "Conv1x1x2+" + what
    desc = _lib.DsConvDesc(x.struct(), y.struct(), res.struct() if res is not None else _null_view(),
                           dww.data_ptr(), pww.data_ptr(), bd.data_ptr(), k, st, p, d, kpad, act, res_mode,
                           dwb.data_ptr() if dwb is not None else None, dw_act, *tail_args, *g2_args, *g0_args)
    plan.launch("ydbl_dsconv_nhwc", desc, what=f"{what}.k{k}s{st}",
                keep=[dww, pww, bd, dwb, tw, tb, g2w, g2b, g0w, g0b, desc])
    return y


def emit_dw_pw(plan: Plan, dwc: "DWConv", pwc: "Conv", x: TV, out: TV | None = None, what="DWConv+Conv1x1",
               tail_conv: nn.Conv2d | None = None, tail_out: TV | None = None):
    """nn.Sequential(DWConv(c, c, k), Conv(c, c2, 1)) of the Detect head (head.py:93-101): one fused launch
    when the shapes allow (the depthwise output stays in LDS), else two.  With tail_conv (the class conv
    cv3[i][2], 1x1 c2 -> nc, bias) the launch also writes tail_out when c2 == 64 and nc <= 4; returns
    (y, tail_done)."""
    if (fused_dsconv_ok(dwc.conv, x, plan.dtype) and pwc.conv.kernel_size == (1, 1) and pwc.conv.stride == (1, 1)
            and dwpw_fuse(pwc.conv.out_channels)):
        wd, bdw = dwc.folded()
        wp, bp = pwc.folded()
        if bdw is None:
            bdw = torch.zeros(x.c)
        tail = None
        if (tail_conv is not None and not os.environ.get("YDBL_NO_CLS_TAIL") and wp.shape[0] == 64
                and tail_conv.kernel_size == (1, 1) and tail_conv.groups == 1
                and tail_conv.in_channels == 64 and 1 <= tail_conv.out_channels <= 4 and tail_conv.bias is not None):
            nc = tail_conv.out_channels
            tail = (tail_conv.weight.detach().float().reshape(nc, 64), tail_conv.bias.detach().float(), tail_out)
        y = emit_dsconv(plan, dwc.conv, x, out, wp, bp if bp is not None else torch.zeros(wp.shape[0]),
                        _act_code(pwc.act), what=what, w_dw=wd, b_dw=bdw, dw_act=_act_code(dwc.act), tail=tail)
        return y, tail is not None
    return pwc.emit(plan, dwc.emit(plan, x), out), False


def dwpw_fuse(c2: int) -> bool:
    """Whether the Detect DWConv -> Conv1x1 pair runs as one launch: at 64 pointwise outputs (DBL-n) the fused pair
    is faster (separate: DBL-n bs32 -1.8 %), at 128 and more (DBL-s / DBL-l) the two launches are (DBL-s bs8 +1.1 %,
    bs64 +2.0 %, DBL-l 1280 bs8 +1.9 %: profiles/r06/r06_detect_switch_sweep.txt).  YDBL_DWPW=1 / 0 forces either."""
    e = os.environ.get("YDBL_DWPW")
    return e == "1" or (e is None and c2 <= 64)


def stem_ok(m, ch: int) -> bool:
    """The first layer can run as ydbl_conv_stem (3x3 Conv on the raw NCHW image)."""
    if type(m) is not Conv:
        return False
    c = m.conv
    return (c.groups == 1 and c.in_channels == ch and ch == 3 and c.kernel_size == (3, 3)
            and c.padding == (1, 1) and c.dilation == (1, 1) and c.stride[0] == c.stride[1] in (1, 2)
            and c.out_channels % 4 == 0 and c.out_channels <= 64 and isinstance(m.act, (nn.SiLU, nn.Identity)))


def emit_stem(m: "Conv", plan: Plan, x_nchw: torch.Tensor, n: int, ch: int, h: int, w: int, bind=None) -> TV:
    """preprocess (U/engine/predictor.py:116-134) + first Conv (conv.py:39-63, BN folded) in one kernel.
    bind: an _lib.InputBind (the batch pointer / LoadTensor maximum read when the plan runs) or None."""
    wf, bf = m.folded()
    s = m.conv.stride[0]
    ho, wo = conv_out_hw(h, w, 3, s, 1, 1)
    y = plan.alloc(n, ho, wo, m.conv.out_channels)
    wd = plan.const(wf.float().contiguous())
    bd = plan.const((bf if bf is not None else torch.zeros(m.conv.out_channels)).float())
    plan.launch("ydbl_conv_stem", x_nchw.data_ptr(), n, ch, h, w, 1.0, wd.data_ptr(), bd.data_ptr(), 3, s,
                _act_code(m.act), y.struct(), bind, what="Stem.conv3x3", keep=[wd, bd, bind])
    return y


def stem2_ok(m0, m1, ch: int, dtype) -> bool:
    """Layers 0-1 can run as ydbl_conv_stem2: Conv(3, C0, 3, 1) + Conv(C0, 2*C0, 3, 2), SiLU, fp16, C0 in {8, 16}."""
    if dtype != torch.float16 or not stem_ok(m0, ch) or type(m1) is not Conv:
        return False
    a, b = m0.conv, m1.conv
    return (a.stride == (1, 1) and a.out_channels in (8, 16) and isinstance(m0.act, nn.SiLU)
            and isinstance(m1.act, nn.SiLU) and b.groups == 1 and b.in_channels == a.out_channels
            and b.out_channels == 2 * a.out_channels and b.kernel_size == (3, 3) and b.stride == (2, 2)
            and b.padding == (1, 1) and b.dilation == (1, 1) and m1.f == -1)


def emit_stem2(m0: "Conv", m1: "Conv", plan: Plan, x_nchw: torch.Tensor, n: int, ch: int, h: int, w: int,
               out: TV | None = None, bind=None) -> TV:
    """preprocess + layers 0 and 1 (conv.py:39-63, BN folded) in one kernel; layer 0's map stays in LDS.
    bind: an _lib.InputBind or None (emit_stem)."""
    w0, b0 = m0.folded()
    w1, b1 = m1.folded()
    c0 = m0.conv.out_channels
    ho, wo = conv_out_hw(h, w, 3, 2, 1, 1)
    y = out if out is not None else plan.alloc(n, ho, wo, 2 * c0)
    b0 = b0 if b0 is not None else torch.zeros(c0)
    b1 = b1 if b1 is not None else torch.zeros(2 * c0)
    host = torch.empty(int(_lib.lib.ydbl_conv_stem2_params_size(c0)), dtype=torch.uint8)
    args = [t.float().contiguous() for t in (w0, b0, w1, b1)]
    _lib.check(_lib.lib.ydbl_conv_stem2_pack(*[t.data_ptr() for t in args], c0, host.data_ptr()), "ydbl_conv_stem2_pack")
    params = plan.const(host)
    d = _lib.Stem2Desc(x_nchw.data_ptr(), n, ch, h, w, 1.0, c0, params.data_ptr(), y.struct(),
                       bind if bind is not None else _lib.InputBind())
    plan.launch("ydbl_conv_stem2", d, what="Stem.conv3x3x2", keep=[params, d])
    return y


def emit_merged(plan: Plan, convs, x: TV, out: TV, what="Conv1x1x2") -> TV:
    """Several Convs that read the same x with the same kernel/stride/activation as ONE launch: the
    folded weights/biases are concatenated along the output channels, in order, into `out`
    (channel slices of one buffer), e.g. C3's cv2 and cv1 (U/nn/modules/block.py:259-273)."""
    ws, bs = zip(*(m.folded() for m in convs))
    c0 = convs[0].conv
    k, st, pd, dl = c0.kernel_size[0], c0.stride[0], c0.padding[0], c0.dilation[0]
    assert (out.h, out.w, out.c) == (*conv_out_hw(x.h, x.w, k, st, pd, dl), sum(w.shape[0] for w in ws))
    emit_dense(plan, x, out, torch.cat(ws, 0), torch.cat(bs, 0), st, pd, dl, _act_code(convs[0].act), what=what)
    return out


def mergeable(convs) -> bool:
    a = convs[0]
    return all(type(m) is Conv and m.conv.kernel_size == a.conv.kernel_size and m.conv.stride == a.conv.stride
               and m.conv.padding == a.conv.padding and m.conv.groups == 1 == a.conv.groups
               and m.conv.dilation == a.conv.dilation and type(m.act) is type(a.act) for m in convs)


def emit_seq(plan: Plan, mods, x, out=None):
    mods = list(mods)
    for i, m in enumerate(mods):
        x = emit_module(m, plan, x, out if i == len(mods) - 1 else None)
    return x


def emit_copy(plan: Plan, src: TV, dst: TV):
    plan.launch("ydbl_pool_up_concat", None, src.struct(), None, dst.struct(), what="copy")


# =============================================================================== module-level forward(x)
def _check_input(t, dev=None, dt=None):
    if not isinstance(t, torch.Tensor) or t.ndim != 4:
        raise TypeError(f"expected BCHW tensors, got {type(t).__name__} {getattr(t, 'shape', '')}")
    if t.device.type != "cuda":
        raise RuntimeError(f"ydbl runs on MI355X (gfx950) only: input on {t.device}, move it to a cuda device")
    if t.dtype not in (torch.float32, torch.float16):
        raise TypeError(f"input dtype {t.dtype}: float32 or float16 (half) expected")
    if (dev is not None and t.device != dev) or (dt is not None and t.dtype != dt):
        raise ValueError("all inputs of one module call must share device and dtype")


class _ModulePlan:
    """One compiled forward of one module for one input signature: input views the call copies into, the plan,
    and the function that turns the plan's outputs into fresh NCHW tensors."""

    def __init__(self, m, xs, multi):
        dev, dt = xs[0].device, xs[0].dtype
        self.plan = Plan(dev, dt)
        self.views = [self.plan.alloc(t.shape[0], t.shape[2], t.shape[3], t.shape[1]) for t in xs]
        inp = self.views if multi else self.views[0]
        self.finish = m._forward_plan(self.plan, inp) if hasattr(m, "_forward_plan") else _tensor_out(
            emit_module(m, self.plan, inp))
        self.wsig = weights_signature(m)

    def __call__(self, xs):
        with torch.no_grad():
            for v, t in zip(self.views, xs):
                v.torch().copy_(t.permute(0, 2, 3, 1))  # NCHW -> the plan's NHWC input buffer
        self.plan.run()
        return self.finish()


def _tensor_out(y):
    if isinstance(y, (list, tuple)):
        return lambda: [v.nchw().contiguous() for v in y]
    return lambda: y.nchw().contiguous()


def run_module(m: nn.Module, x):
    """forward(x) of a built-in module: x a BCHW cuda tensor (or a list for Concat / FullPAD_Tunnel / HyperACE /
    FuseModule / Detect) in fp32 or fp16 (the half path); returns fresh NCHW tensors of x's dtype.  The module's
    emit is compiled once per (input shapes, dtype, device, YDBL_* switches) into a plan with its own buffers (the
    two most recent kept) and rebuilt when the module's weights change (runtime.weights_signature, checked after
    the launch).  BN is folded: inference semantics, as the reference after fuse()."""
    multi = isinstance(x, (list, tuple))
    xs = list(x) if multi else [x]
    if not xs:
        raise ValueError("no inputs")
    for t in xs:
        _check_input(t, xs[0].device, xs[0].dtype)
    key = (tuple(tuple(t.shape) for t in xs), multi, xs[0].dtype, str(xs[0].device), ydbl_env())
    cache = m.__dict__.setdefault("_fwd_plans", {})
    mp = cache.pop(key, None)
    if mp is None:
        while len(cache) >= 2:
            cache.pop(next(iter(cache)))
        with torch.cuda.device(xs[0].device):
            mp = _ModulePlan(m, xs, multi)
    cache[key] = mp
    y = mp(xs)
    if weights_signature(m) != mp.wsig:  # weights edited since the plan folded them: rebuild, run again
        with torch.cuda.device(xs[0].device):
            mp = cache[key] = _ModulePlan(m, xs, multi)
        y = mp(xs)
    return y


class PlanModule(nn.Module):
    """Base of the built-in modules: ``forward(x)`` = run_module (the reference's ``m(x)`` contract)."""

    def forward(self, x):
        return run_module(self, x)


def _meta_copy(m: nn.Module) -> nn.Module:
    import copy

    return copy.deepcopy(m).to("meta")


def torch_out_shape(m: nn.Module, src) -> tuple:
    """NHWC shape of a forward-only plugin's output, from a shape-only (meta) run of its forward on NCHW inputs
    of the given NHWC shapes."""
    multi = isinstance(src, list)
    metas = [torch.empty((s[0], s[3], s[1], s[2]), device="meta") for s in (src if multi else [src])]
    with torch.no_grad():
        y = _meta_copy(m)(metas if multi else metas[0])
    if not isinstance(y, torch.Tensor) or y.ndim != 4:
        raise TypeError(f"plugin {type(m).__name__}: forward must return one BCHW tensor")
    return (y.shape[0], y.shape[2], y.shape[3], y.shape[1])


def emit_torch(m: nn.Module, plan: Plan, x, out: TV | None = None) -> TV:
    """A registered plugin module that has only a torch ``forward`` (the reference's plugin contract: any class
    with forward(x), looked up by name, U/nn/tasks.py:974, called as m(x), :158-161) as one plan step: a device
    copy of the module in the plan's dtype (weights frozen at build, like every other layer) runs on NCHW views
    of its NHWC input slices, on the stream the plan runs on -- so it is captured into the step's hipGraph with
    the HIP launches around it -- and its result is copied into the output view.  The module's forward must be
    graph-capturable (no host syncs) and must launch on the current stream only (single_stream)."""
    multi = isinstance(x, (list, tuple))
    xs = list(x) if multi else [x]
    shape = torch_out_shape(m, [v.shape for v in xs] if multi else xs[0].shape)
    y = out if out is not None else plan.alloc(*shape)
    if y.shape != shape:
        raise ValueError(f"plugin {type(m).__name__}: output {shape} does not fit the destination {y.shape}")
    import copy

    dm = copy.deepcopy(m).to(plan.device)
    if plan.device.type != "meta":
        dm = dm.to(plan.dtype)
    dm.eval()

    def step(stream):
        # handle 0 (c_void_p value None) is the null stream: eager runs on torch's default stream pass it
        ts = (torch.cuda.ExternalStream(stream.value, device=plan.device) if stream.value
              else torch.cuda.default_stream(plan.device))
        with torch.cuda.stream(ts), torch.no_grad():
            ins = [v.nchw() for v in xs]
            y.nchw().copy_(dm(ins if multi else ins[0]))
        return 0

    step.single_stream = True
    step.__name__ = f"torch:{type(m).__name__}"
    plan.steps.append(Step(step, (), f"torch.{type(m).__name__}", [dm]))
    return y


# =============================================================================== conv.py
class Conv(PlanModule):
    """U/nn/modules/conv.py:39-63 — conv -> BN -> SiLU (BN folded at plan time, as fuse() does)."""

    default_act = nn.SiLU()

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = self.default_act if act is True else act if isinstance(act, nn.Module) else nn.Identity()

    def folded(self):
        if hasattr(self, "bn"):
            return fold_bn(self.conv.weight, self.conv.bias, self.bn)
        return self.conv.weight.detach().float().cpu(), (
            self.conv.bias.detach().float().cpu() if self.conv.bias is not None else None)

    def emit(self, plan, x, out=None, res=None, res_mode=_lib.RES_NONE):
        w, b = self.folded()
        return emit_conv2d(plan, self.conv, x, out, w, b, _act_code(self.act), res, res_mode,
                           what=f"Conv{self.conv.kernel_size[0]}x{self.conv.kernel_size[0]}")


class DWConv(Conv):
    """U/nn/modules/conv.py:128-133."""

    def __init__(self, c1, c2, k=1, s=1, d=1, act=True):
        super().__init__(c1, c2, k, s, g=math.gcd(c1, c2), d=d, act=act)


class DSConv(PlanModule):
    """U/nn/modules/conv.py:91-108 — dw -> pw -> BN -> SiLU."""

    def __init__(self, c_in, c_out, k=3, s=1, p=None, d=1, bias=False):
        super().__init__()
        if p is None:
            p = (d * (k - 1)) // 2
        self.dw = nn.Conv2d(c_in, c_in, kernel_size=k, stride=s, padding=p, dilation=d, groups=c_in, bias=bias)
        self.pw = nn.Conv2d(c_in, c_out, 1, 1, 0, bias=bias)
        self.bn = nn.BatchNorm2d(c_out)
        self.act = nn.SiLU()

    def emit(self, plan, x, out=None, res=None, res_mode=_lib.RES_NONE):
        w, b = fold_bn(self.pw.weight, self.pw.bias, self.bn)
        if self.dw.bias is None and fused_dsconv_ok(self.dw, x, plan.dtype):
            return emit_dsconv(plan, self.dw, x, out, w, b, _lib.ACT_SILU, res, res_mode)
        t = emit_conv2d(plan, self.dw, x, None, what=f"DSConv.dw{self.dw.kernel_size[0]}")
        return emit_conv2d(plan, self.pw, t, out, w, b, _lib.ACT_SILU, res, res_mode, what="DSConv.pw")


class GhostConv(PlanModule):
    """U/nn/modules/conv.py:184-197 — cat(y, dw5x5(y)), y = cv1(x)."""

    def __init__(self, c1, c2, k=1, s=1, g=1, act=True):
        super().__init__()
        c_ = c2 // 2
        self.cv1 = Conv(c1, c_, k, s, None, g, act=act)
        self.cv2 = Conv(c_, c_, 5, 1, None, c_, act=act)

    def emit(self, plan, x, out=None, res=None):
        c_ = self.cv1.conv.out_channels
        ho, wo = conv_out_hw(x.h, x.w, self.cv1.conv.kernel_size[0], self.cv1.conv.stride[0],
                             self.cv1.conv.padding[0], 1)
        y = out if out is not None else plan.alloc(x.n, ho, wo, 2 * c_)
        r0 = res.cslice(0, c_) if res is not None else None
        r1 = res.cslice(c_, c_) if res is not None else None
        # the dw half reads the pre-residual cv1 output, so with a residual cv1 goes to a temporary
        y0 = plan.alloc(x.n, ho, wo, c_) if res is not None else y.cslice(0, c_)
        self.cv1.emit(plan, x, y0)
        self.cv2.emit(plan, y0, y.cslice(c_, c_), res=r1, res_mode=_lib.RES_ADD if res is not None else 0)
        if res is not None:
            plan.launch("ydbl_gate_add", r0.struct(), y0.struct(), 1.0, y.cslice(0, c_).struct(), what="ghost.res")
        return y


class Concat(PlanModule):
    """U/nn/modules/conv.py:349-359 — inputs are normally already slices of the output (see tasks.py)."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def emit(self, plan, xs, out=None):
        c = sum(x.c for x in xs)
        y = out if out is not None else plan.alloc(xs[0].n, xs[0].h, xs[0].w, c)
        off = 0
        for x in xs:
            dst = y.cslice(off, x.c)
            if not (x.base is dst.base and x.off == dst.off and x.cs == dst.cs):
                emit_copy(plan, x, dst)
            off += x.c
        return y


# =============================================================================== block.py
def emit_conv3x3_pair(plan, a: "Conv", b: "Conv", x: TV, out: TV | None = None) -> TV:
    """Conv(c, cm, 3) -> Conv(cm, c, 3) (SiLU both, no shortcut) as one ydbl_bottleneck_nhwc launch with
    the intermediate in LDS when the (c, cm) pair is built (fp16; used for the Detect box branch
    cv2[i][0:2] at 64 channels, head.py:86-90), else the two convs."""
    ca, cb = a.conv, b.conv
    c, cm = cb.out_channels, ca.out_channels
    ok = (plan.dtype == torch.float16 and not os.environ.get("YDBL_NO_BNECK") and not os.environ.get("YDBL_NO_PAIR3")
          and (c, cm) == (64, 64)
          and x.c == c == ca.in_channels and cb.in_channels == cm
          and all(m.kernel_size == (3, 3) and m.stride == (1, 1) and m.padding == (1, 1) and m.dilation == (1, 1)
                  and m.groups == 1 for m in (ca, cb))
          and isinstance(a.act, nn.SiLU) and isinstance(b.act, nn.SiLU))
    y = out if out is not None else plan.alloc(x.n, x.h, x.w, c)
    if not ok or y.base is x.base:
        return b.emit(plan, a.emit(plan, x), out)
    args = [t.float().contiguous() for t in (*a.folded(), *b.folded())]
    host = torch.empty(int(_lib.lib.ydbl_conv3x3_pair_params_size(c, cm)), dtype=torch.uint8)
    _lib.check(_lib.lib.ydbl_conv3x3_pair_pack(*[t.data_ptr() for t in args], c, cm, host.data_ptr()),
               "ydbl_conv3x3_pair_pack")
    params = plan.const(host)
    d = _lib.BottleneckDesc(x.struct(), y.struct(), c, 0, 0, params.data_ptr(), cm)
    plan.launch("ydbl_bottleneck_nhwc", d, what=f"Conv3x3x2.c{c}", keep=[params, d])
    return y


def emit_detect_box(plan, seq, x: TV, out: TV) -> bool:
    """Detect box branch cv2[i] = Conv(c_in,64,3) -> Conv(64,64,3) -> Conv2d(64,64,1,bias) (head.py:86-90) as
    one ydbl_bottleneck_nhwc launch (desc.pw = 1: both 3x3 intermediates stay in LDS).  False (nothing
    emitted) unless fp16 with c_in 64 or 128 (DBL-n P3 / P4)."""
    a, b, c = seq[0], seq[1], seq[2]
    ca, cb = a.conv, b.conv
    ok = (plan.dtype == torch.float16 and not os.environ.get("YDBL_NO_BNECK") and not os.environ.get("YDBL_NO_BOX3")
          and x.c in (64, 128)
          and ca.in_channels == x.c and ca.out_channels == cb.in_channels == cb.out_channels == 64
          and all(m.kernel_size == (3, 3) and m.stride == (1, 1) and m.padding == (1, 1) and m.dilation == (1, 1)
                  and m.groups == 1 for m in (ca, cb))
          and isinstance(a.act, nn.SiLU) and isinstance(b.act, nn.SiLU)
          and isinstance(c, nn.Conv2d) and c.kernel_size == (1, 1) and c.groups == 1 and c.bias is not None
          and c.in_channels == c.out_channels == 64 and out.c == 64 and out.base is not x.base)
    if not ok:
        return False
    args = [t.float().contiguous() for t in (*a.folded(), *b.folded())]
    args += [c.weight.detach().float().reshape(64, 64).contiguous(), c.bias.detach().float().contiguous()]
    host = torch.empty(int(_lib.lib.ydbl_detect_box_params_size(x.c, 64)), dtype=torch.uint8)
    _lib.check(_lib.lib.ydbl_detect_box_pack(*[t.data_ptr() for t in args], x.c, 64, host.data_ptr()),
               "ydbl_detect_box_pack")
    params = plan.const(host)
    d = _lib.BottleneckDesc(x.struct(), out.struct(), 64, 0, 0, params.data_ptr(), 64, 1)
    plan.launch("ydbl_bottleneck_nhwc", d, what="Detect.box3", keep=[params, d])
    return True


class Bottleneck(PlanModule):
    """U/nn/modules/block.py:344-357."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def fused_ok(self, plan, x) -> bool:
        """cv1 -> cv2 as one ydbl_bottleneck_nhwc launch: fp16, c -> c/2 -> c, 3x3 s1 both, SiLU both."""
        a, b = self.cv1.conv, self.cv2.conv
        c = b.out_channels
        return (plan.dtype == torch.float16 and not os.environ.get("YDBL_NO_BNECK") and c in (16, 32, 64)
                and x.c == c == a.in_channels and a.out_channels == c // 2 == b.in_channels
                and all(m.kernel_size == (3, 3) and m.stride == (1, 1) and m.padding == (1, 1)
                        and m.dilation == (1, 1) and m.groups == 1 for m in (a, b))
                and isinstance(self.cv1.act, nn.SiLU) and isinstance(self.cv2.act, nn.SiLU))

    def emit(self, plan, x, out=None):
        if self.fused_ok(plan, x):
            c = x.c
            y = out if out is not None else plan.alloc(x.n, x.h, x.w, c)
            if y.base is not x.base:  # the kernel reads a halo of x while writing y
                args = [t.float().contiguous() for t in (*self.cv1.folded(), *self.cv2.folded())]
                host = torch.empty(int(_lib.lib.ydbl_bottleneck_params_size(c)), dtype=torch.uint8)
                _lib.check(_lib.lib.ydbl_bottleneck_pack(*[t.data_ptr() for t in args], c, host.data_ptr()),
                           "ydbl_bottleneck_pack")
                params = plan.const(host)
                d = _lib.BottleneckDesc(x.struct(), y.struct(), c, int(self.add), 0, params.data_ptr())
                plan.launch("ydbl_bottleneck_nhwc", d, what=f"Bottleneck.c{c}", keep=[params, d])
                return y
        t = self.cv1.emit(plan, x)
        return self.cv2.emit(plan, t, out, res=x if self.add else None,
                             res_mode=_lib.RES_ADD if self.add else _lib.RES_NONE)


class C2f(PlanModule):
    """U/nn/modules/block.py:234-249."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=((3, 3), (3, 3)), e=1.0) for _ in range(n))

    def emit(self, plan, x, out=None):
        c, n = self.c, len(self.m)
        buf = plan.alloc(x.n, x.h, x.w, (2 + n) * c)
        self.cv1.emit(plan, x, buf.cslice(0, 2 * c))
        for i, m in enumerate(self.m):
            m.emit(plan, buf.cslice((1 + i) * c, c), buf.cslice((2 + i) * c, c))
        return self.cv2.emit(plan, buf, out)


class C3(PlanModule):
    """U/nn/modules/block.py:259-273."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=((1, 1), (3, 3)), e=1.0) for _ in range(n)))

    def emit(self, plan, x, out=None):
        c_ = self.cv1.conv.out_channels
        if mergeable([self.cv2, self.cv1]) and not os.environ.get("YDBL_NO_MERGE"):
            # cv2 and cv1 both read x: one launch into [m slot | cv2 | cv1] (cv3 reads the first 2c_)
            buf = plan.alloc(x.n, x.h, x.w, 3 * c_)
            if self._cv3_fusable(plan, x):
                # DSC3k: cv3 rides in the last DSBottleneck's k7 DSConv (its output never leaves the CU), and
                # cv2 | cv1 in the first one's k3 DSConv where the lean kernel takes it (cv1's map recomputed on
                # the halo; both outputs still written: cv3 and the first residual read them)
                pre = (self.cv2, self.cv1, x, buf.cslice(c_, 2 * c_)) if self._cv1_fusable(plan, x) else None
                if pre is None:
                    emit_merged(plan, [self.cv2, self.cv1], x, buf.cslice(c_, 2 * c_))
                mods = list(self.m)
                t = buf.cslice(2 * c_, c_)
                for i, m in enumerate(mods[:-1]):
                    t = m.emit(plan, t, pre=pre if i == 0 else None)
                return mods[-1].emit(plan, t, buf.cslice(0, c_), cv3=(self.cv3, buf.cslice(c_, c_), out),
                                     pre=pre if len(mods) == 1 else None)
            emit_merged(plan, [self.cv2, self.cv1], x, buf.cslice(c_, 2 * c_))
            emit_seq(plan, self.m, buf.cslice(2 * c_, c_), buf.cslice(0, c_))
            return self.cv3.emit(plan, buf.cslice(0, 2 * c_), out)
        buf = plan.alloc(x.n, x.h, x.w, 2 * c_)
        t = self.cv1.emit(plan, x)
        emit_seq(plan, self.m, t, buf.cslice(0, c_))
        self.cv2.emit(plan, x, buf.cslice(c_, c_))
        return self.cv3.emit(plan, buf, out)


    def _cv1_fusable(self, plan, x) -> bool:
        """cv2 | cv1 (merged 1x1, x.c -> 2 c_) can lead the first DSBottleneck's k3 DSConv in one launch
        (dsc_lean.hip PRE, ydbl_dsconv_desc.g0): fp16, x.c == c_ == 64, SiLU 1x1s, that DSConv k3 stride 1 with
        no depthwise bias, the lean kernel enabled -- and YDBL_CV1_FUSE=1: off by default since round 6 (the separate
        1x1 measured faster in the two-branch layout: DBL-n bs32 +0.5 %, profiles/r06/r06_fusion_switch_sweep.txt)."""
        if (plan.dtype != torch.float16 or os.environ.get("YDBL_CV1_FUSE") != "1" or os.environ.get("YDBL_DS_LEAN") == "0"
                or not len(self.m) or not isinstance(self.m[0], DSBottleneck)):
            return False
        c_ = self.cv1.conv.out_channels
        first = self.m[0].cv1
        dw = first.dw
        return (c_ == 64 and x.c == 64 and x.cs % 8 == 0 and self.cv1.conv.kernel_size == (1, 1)
                and self.cv1.conv.stride == (1, 1) and isinstance(self.cv1.act, nn.SiLU)
                and dw.kernel_size == (3, 3) and dw.stride == (1, 1) and dw.dilation == (1, 1) and dw.padding == (1, 1)
                and dw.bias is None and dw.in_channels == c_ and first.pw.out_channels == c_)

    def _cv3_fusable(self, plan, x) -> bool:
        """cv3 can run as the trailing GEMM of the last bottleneck's k7 DSConv (dsc_lean.hip, ydbl_dsconv_desc.g2):
        fp16, m = DSBottlenecks ending in a k7 stride-1 DSConv with c_ in {64, 128} in and out, cv3 a 1x1 SiLU
        Conv 2c_ -> c_ (DSC3k with e = 1, U/nn/modules/block.py:1447-1503) -- and YDBL_CV3_FUSE=1: off by default since
        round 6 (DBL-n bs32 +0.6 % with the separate cv3, profiles/r06/r06_fusion_switch_sweep.txt)."""
        # the trailing GEMM runs only in the lean kernel (dsc_lean.hip): with it switched off the chunked kernel
        # would refuse the g2 descriptor, so the rule must agree with _cv1_fusable's
        if (plan.dtype != torch.float16 or os.environ.get("YDBL_CV3_FUSE") != "1" or os.environ.get("YDBL_DS_LEAN") == "0"
                or not len(self.m)):
            return False
        last, c_ = self.m[-1], self.cv1.conv.out_channels
        if not isinstance(last, DSBottleneck):
            return False
        dw, pw = last.cv2.dw, last.cv2.pw
        c3 = self.cv3.conv
        # 128 channels only on small maps (csrc/dsc_lean.hip: LEAN_MAX_TILES_WIDE 8x8 tiles), where the lean kernel runs
        small = x.n * -(-x.h // 8) * -(-x.w // 8) <= 160
        return ((c_ == 64 or (c_ == 128 and small)) and dw.kernel_size == (7, 7) and dw.stride == (1, 1)
                and dw.dilation == (1, 1)
                and dw.bias is None and dw.in_channels == pw.out_channels == c_ and last.cv1.pw.out_channels == c_
                and c3.kernel_size == (1, 1) and c3.stride == (1, 1) and c3.groups == 1
                and c3.in_channels == 2 * c_ and c3.out_channels == c_ and isinstance(self.cv3.act, nn.SiLU))


class GhostBottleneck(PlanModule):
    """U/nn/modules/block.py:323-341 (stride 1 on the DBL path)."""

    def __init__(self, c1, c2, k=3, s=1):
        super().__init__()
        c_ = c2 // 2
        self.conv = nn.Sequential(
            GhostConv(c1, c_, 1, 1),
            DWConv(c_, c_, k, s, act=False) if s == 2 else nn.Identity(),
            GhostConv(c_, c2, 1, 1, act=False),
        )
        self.shortcut = (
            nn.Sequential(DWConv(c1, c1, k, s, act=False), Conv(c1, c2, 1, 1, act=False)) if s == 2 else nn.Identity()
        )

    def emit(self, plan, x, out=None):
        if not isinstance(self.shortcut, nn.Identity):
            raise NotImplementedError("GhostBottleneck s=2 is not on the DBL path")
        t = self.conv[0].emit(plan, x)
        return self.conv[2].emit(plan, t, out, res=x)


class C3Ghost(C3):
    """U/nn/modules/block.py:313-320."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(GhostBottleneck(c_, c_) for _ in range(n)))


class DSBottleneck(PlanModule):
    """U/nn/modules/block.py:1408-1444."""

    def __init__(self, c1, c2, shortcut=True, e=0.5, k1=3, k2=5, d2=1):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = DSConv(c1, c_, k1, s=1, p=None, d=1)
        self.cv2 = DSConv(c_, c2, k2, s=1, p=None, d=d2)
        self.add = shortcut and c1 == c2

    def emit(self, plan, x, out=None, cv3=None, pre=None):
        """cv3 = (C3's cv3 Conv, its second input view (the cv2 branch), its output view or None): the DSC3k's
        cv3 as the trailing GEMM of this bottleneck's k7 DSConv; returns cv3's output then.
        pre = (C3's cv2, cv1, their input, their [cv2 | cv1] output view whose last c_ channels are x): the merged
        1x1 as the leading GEMM of this bottleneck's k3 DSConv (C3._cv1_fusable)."""
        y = out if out is not None else plan.alloc(x.n, x.h, x.w, self.cv2.pw.out_channels)
        if pre is not None:
            c2m, c1m, x0, y0 = pre
            (w2, b2), (w1, b1) = c2m.folded(), c1m.folded()
            g0 = (torch.cat([w2, w1], 0).reshape(y0.c, x0.c), torch.cat([b2, b1], 0), x0, y0, _act_code(c1m.act))
            wp, bp = fold_bn(self.cv1.pw.weight, self.cv1.pw.bias, self.cv1.bn)
            t = emit_dsconv(plan, self.cv1.dw, x, None, wp, bp, _lib.ACT_SILU, g0=g0)
        else:
            t = None
        if cv3 is not None:
            conv3, x2, o3 = cv3
            o3 = o3 if o3 is not None else plan.alloc(x.n, x.h, x.w, conv3.conv.out_channels)
            t = t if t is not None else self.cv1.emit(plan, x)
            w, b = fold_bn(self.cv2.pw.weight, self.cv2.pw.bias, self.cv2.bn)
            w3, b3 = conv3.folded()
            emit_dsconv(plan, self.cv2.dw, t, y, w, b, _lib.ACT_SILU, x if self.add else None,
                        _lib.RES_ADD if self.add else _lib.RES_NONE,
                        g2=(w3.reshape(w3.shape[0], -1), b3, x2, o3, _act_code(conv3.act)))
            return o3
        t = t if t is not None else self.cv1.emit(plan, x)
        return self.cv2.emit(plan, t, y, res=x if self.add else None,
                             res_mode=_lib.RES_ADD if self.add else _lib.RES_NONE)


class DSC3k(C3):
    """U/nn/modules/block.py:1447-1503."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5, k1=3, k2=5, d2=1):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(
            *(DSBottleneck(c_, c_, shortcut=shortcut, e=1.0, k1=k1, k2=k2, d2=d2) for _ in range(n))
        )


class DSC3k2(C2f):
    """U/nn/modules/block.py:1505-1580."""

    def __init__(self, c1, c2, n=1, dsc3k=False, e=0.5, g=1, shortcut=True, k1=3, k2=7, d2=1):
        super().__init__(c1, c2, n, shortcut, g, e)
        if dsc3k:
            self.m = nn.ModuleList(
                DSC3k(self.c, self.c, n=2, shortcut=shortcut, g=g, e=1.0, k1=k1, k2=k2, d2=d2) for _ in range(n)
            )
        else:
            self.m = nn.ModuleList(
                DSBottleneck(self.c, self.c, shortcut=shortcut, e=1.0, k1=k1, k2=k2, d2=d2) for _ in range(n)
            )


class AdaHyperedgeGen(nn.Module):
    """U/nn/modules/block.py:1582-1657 (parameters only; compute in ydbl_hg_*)."""

    def __init__(self, node_dim, num_hyperedges, num_heads=4, dropout=0.1, context="both"):
        super().__init__()
        if context != "both":
            raise NotImplementedError("only context='both' (the DBL configuration) has a HIP path")
        self.num_heads = num_heads
        self.num_hyperedges = num_hyperedges
        self.head_dim = node_dim // num_heads
        self.context = context
        self.prototype_base = nn.Parameter(torch.Tensor(num_hyperedges, node_dim))
        nn.init.xavier_uniform_(self.prototype_base)
        self.context_net = nn.Linear(2 * node_dim, num_hyperedges * node_dim)
        self.pre_head_proj = nn.Linear(node_dim, node_dim)
        self.dropout = nn.Dropout(dropout)
        self.scaling = math.sqrt(self.head_dim)


class AdaHGConv(PlanModule):
    """U/nn/modules/block.py:1659-1708."""

    def __init__(self, embed_dim, num_hyperedges=16, num_heads=4, dropout=0.1, context="both"):
        super().__init__()
        self.edge_generator = AdaHyperedgeGen(embed_dim, num_hyperedges, num_heads, dropout, context)
        self.edge_proj = nn.Sequential(nn.Linear(embed_dim, embed_dim), nn.GELU())
        self.node_proj = nn.Sequential(nn.Linear(embed_dim, embed_dim), nn.GELU())

    def emit(self, plan, x, out=None):
        g = self.edge_generator
        D, E = x.c, g.num_hyperedges
        y = out if out is not None else plan.alloc(x.n, x.h, x.w, D)
        c = plan.const
        p = [c(g.prototype_base.float()), c(g.context_net.weight.float()), c(g.context_net.bias.float()),
             c(self.edge_proj[0].weight.float()), c(self.edge_proj[0].bias.float()),
             c(self.node_proj[0].weight.float()), c(self.node_proj[0].bias.float())]
        nws = _lib.lib.ydbl_hg_fused_workspace(x.n, x.h * x.w, D, E, _lib.dtype_code(plan.dtype))
        if (not os.environ.get("YDBL_HG_UNFUSED") and D == 16 * g.num_heads and nws > 0
                and x.c == D and (y.base is not x.base or y.off + y.c <= x.off or x.off + x.c <= y.off)):
            # the whole AdaHGConv, pre_head_proj included, from one C-ABI call (csrc/hg_fused.hip: three kernels
            # over (token slice, image) workgroups)
            pw = c(g.pre_head_proj.weight.detach().float().to(plan.dtype).contiguous())
            pb = c(g.pre_head_proj.bias.detach().float())
            ws = plan.scratch(nws)  # per-slice partials, fully written before they are read
            d = HgDesc(x.struct(), _null_view(), y.struct(), E, g.num_heads, *[t.data_ptr() for t in p], ws.data_ptr(),
                       pw.data_ptr(), pb.data_ptr())
            plan.launch("ydbl_hg_fused", d, what="AdaHG.fused", keep=[d, pw, pb, ws, *p])
            return y
        # X_proj = pre_head_proj(X) as a 1x1 conv over the token grid
        xp = plan.alloc(x.n, x.h, x.w, D)
        emit_dense(plan, x, xp, g.pre_head_proj.weight.detach().float().cpu().view(D, D, 1, 1),
                   g.pre_head_proj.bias.detach().float().cpu(), what="AdaHG.pre_proj")
        ws = plan.scratch(_lib.lib.ydbl_hg_workspace(x.n, x.h * x.w, D, E))
        d = HgDesc(x.struct(), xp.struct(), y.struct(), E, g.num_heads, *[t.data_ptr() for t in p], ws.data_ptr())
        plan.launch("ydbl_hg_context", d, what="AdaHG.context", keep=[d, ws, *p])
        plan.launch("ydbl_hg_propagate", d, what="AdaHG.propagate", keep=[d])
        return y


class AdaHGComputation(PlanModule):
    """U/nn/modules/block.py:1710-1752 (NHWC pixels are already the token sequence)."""

    def __init__(self, embed_dim, num_hyperedges=16, num_heads=8, dropout=0.1, context="both"):
        super().__init__()
        self.embed_dim = embed_dim
        self.hgnn = AdaHGConv(embed_dim, num_hyperedges, num_heads, dropout, context)

    def emit(self, plan, x, out=None):
        return self.hgnn.emit(plan, x, out)


class C3AH(PlanModule):
    """U/nn/modules/block.py:1754-1795."""

    def __init__(self, c1, c2, e=1.0, num_hyperedges=8, context="both"):
        super().__init__()
        c_ = int(c2 * e)
        assert c_ % 16 == 0, "Dimension of AdaHGComputation should be a multiple of 16."
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.m = AdaHGComputation(c_, num_hyperedges, c_ // 16, 0.1, context)
        self.cv3 = Conv(2 * c_, c2, 1)

    def emit(self, plan, x, out=None):
        c_ = self.cv1.conv.out_channels
        if mergeable([self.cv2, self.cv1]) and not os.environ.get("YDBL_NO_MERGE"):
            buf = plan.alloc(x.n, x.h, x.w, 3 * c_)  # [m slot | cv2 | cv1], as C3.emit
            emit_merged(plan, [self.cv2, self.cv1], x, buf.cslice(c_, 2 * c_))
            self.m.emit(plan, buf.cslice(2 * c_, c_), buf.cslice(0, c_))
            return self.cv3.emit(plan, buf.cslice(0, 2 * c_), out)
        buf = plan.alloc(x.n, x.h, x.w, 2 * c_)
        t = self.cv1.emit(plan, x)
        self.m.emit(plan, t, buf.cslice(0, c_))
        self.cv2.emit(plan, x, buf.cslice(c_, c_))
        return self.cv3.emit(plan, buf, out)


class FuseModule(PlanModule):
    """U/nn/modules/block.py:1797-1840."""

    def __init__(self, c_in, channel_adjust):
        super().__init__()
        self.downsample = nn.AvgPool2d(kernel_size=2)
        self.upsample = nn.Upsample(scale_factor=2, mode="nearest")
        self.conv_out = Conv((4 if channel_adjust else 3) * c_in, c_in, 1)

    def emit(self, plan, xs, out=None):
        p3, p4, p5 = xs
        cat = plan.alloc(p4.n, p4.h, p4.w, p3.c + p4.c + p5.c)
        plan.launch("ydbl_pool_up_concat", p3.struct(), p4.struct(), p5.struct(), cat.struct(), what="Fuse.cat")
        return self.conv_out.emit(plan, cat, out)


class HyperACE(PlanModule):
    """U/nn/modules/block.py:1842-1895."""

    def __init__(self, c1, c2, n=1, num_hyperedges=8, dsc3k=True, shortcut=False, e1=0.5, e2=1, context="both",
                 channel_adjust=True):
        super().__init__()
        self.c = int(c2 * e1)
        self.cv1 = Conv(c1, 3 * self.c, 1, 1)
        self.cv2 = Conv((4 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(
            DSC3k(self.c, self.c, 2, shortcut, k1=3, k2=7) if dsc3k else DSBottleneck(self.c, self.c, shortcut=shortcut)
            for _ in range(n)
        )
        self.fuse = FuseModule(c1, channel_adjust)
        self.branch1 = C3AH(self.c, self.c, e2, num_hyperedges, context)
        self.branch2 = C3AH(self.c, self.c, e2, num_hyperedges, context)

    def emit(self, plan, xs, out=None):
        c, n = self.c, len(self.m)
        x = self.fuse.emit(plan, xs)
        # concat order of the reference: [y0, branch1(y1), y2, m_0(y2), ..., m_{n-1}, branch2(y1)]
        cat = plan.alloc(x.n, x.h, x.w, (4 + n) * c)
        self.cv1.emit(plan, x, cat.cslice(0, 3 * c))  # y0 | y1 | y2
        y1 = cat.cslice(c, c)
        if self._branches_mergeable():
            self._emit_branches(plan, y1, cat.cslice(c, c), cat.cslice((3 + n) * c, c))
        else:
            self.branch2.emit(plan, y1, cat.cslice((3 + n) * c, c))
            self.branch1.emit(plan, y1, cat.cslice(c, c))  # reads y1 before its last conv overwrites it
        prev = cat.cslice(2 * c, c)
        for i, m in enumerate(self.m):
            prev = m.emit(plan, prev, cat.cslice((3 + i) * c, c))
        return self.cv2.emit(plan, cat, out)


    def _branches_mergeable(self) -> bool:
        b1, b2 = self.branch1, self.branch2
        return (not os.environ.get("YDBL_NO_MERGE") and mergeable([b2.cv2, b2.cv1, b1.cv1, b1.cv2])
                and b1.cv1.conv.out_channels == b2.cv1.conv.out_channels)

    def _emit_branches(self, plan, y1, out1, out2):
        """Both C3AH branches read y1 (block.py:1886-1895): their four input 1x1s (cv1, cv2 of each) run as ONE
        launch into one buffer laid out [b2.m | b2.cv2 | b2.cv1 | b1.cv1 | b1.cv2 | b1.m], so each branch's
        cv3 input is contiguous: b2's in the reference order cat(m, cv2), b1's as (cv2, m) with cv3's weight
        columns swapped to match (the same sums, in another order of K)."""
        b1, b2 = self.branch1, self.branch2
        c_ = b1.cv1.conv.out_channels
        bb = plan.alloc(y1.n, y1.h, y1.w, 6 * c_)
        emit_merged(plan, [b2.cv2, b2.cv1, b1.cv1, b1.cv2], y1, bb.cslice(c_, 4 * c_), what="C3AHx2.cv1|cv2")
        b2.m.emit(plan, bb.cslice(2 * c_, c_), bb.cslice(0, c_))
        b2.cv3.emit(plan, bb.cslice(0, 2 * c_), out2)
        b1.m.emit(plan, bb.cslice(3 * c_, c_), bb.cslice(5 * c_, c_))
        w, b = b1.cv3.folded()
        w = torch.cat([w[:, c_:], w[:, :c_]], 1)
        emit_conv2d(plan, b1.cv3.conv, bb.cslice(4 * c_, 2 * c_), out1, w, b, _act_code(b1.cv3.act), what="Conv1x1")


class DownsampleConv(PlanModule):
    """U/nn/modules/block.py:1897-1928."""

    def __init__(self, in_channels, channel_adjust=True):
        super().__init__()
        self.downsample = nn.AvgPool2d(kernel_size=2)
        self.channel_adjust = Conv(in_channels, in_channels * 2, 1) if channel_adjust else nn.Identity()

    def emit(self, plan, x, out=None):
        adjust = not isinstance(self.channel_adjust, nn.Identity)
        pooled = out if (out is not None and not adjust) else plan.alloc(x.n, x.h // 2, x.w // 2, x.c)
        plan.launch("ydbl_pool_up_concat", x.struct(), None, None, pooled.struct(), what="Downsample.pool")
        return self.channel_adjust.emit(plan, pooled, out) if adjust else pooled


class FullPAD_Tunnel(PlanModule):  # noqa: N801 (reference name)
    """U/nn/modules/block.py:1930-1956 — x0 + gate * x1."""

    def __init__(self):
        super().__init__()
        self.gate = nn.Parameter(torch.tensor(0.0))

    def emit(self, plan, xs, out=None):
        a, b = xs
        y = out if out is not None else plan.alloc(a.n, a.h, a.w, a.c)
        g = float(self.gate.detach().float().cpu())
        # Fused into the dense conv that produced the later of the two inputs (its epilogue writes
        # y = a + g*b as a second output; the other input is complete by then).  Otherwise one
        # ydbl_gate_add launch.
        if os.environ.get("YDBL_NO_FUSE_PAD"):  # A/B switch for the benches
            return self._launch(plan, a, b, g, y)
        ia, ib = plan.writer_of(a), plan.writer_of(b)
        if ib is not None and (ia is None or ia[0] < ib[0]) and (ia is not None or plan.made_before(a, ib[0])):
            return plan.fuse_second_output(ib, y, a, g, 1.0) or self._launch(plan, a, b, g, y)
        if ia is not None and (ib is None or ib[0] < ia[0]) and (ib is not None or plan.made_before(b, ia[0])):
            return plan.fuse_second_output(ia, y, b, 1.0, g) or self._launch(plan, a, b, g, y)
        return self._launch(plan, a, b, g, y)

    @staticmethod
    def _launch(plan, a, b, g, y):
        plan.launch("ydbl_gate_add", a.struct(), b.struct(), g, y.struct(), what="FullPAD")
        return y


# =============================================================================== DySample / LSKblock
class DySample(PlanModule):
    """U/nn/modules_upsample/DySample.py:20-81 (style 'lp', scale 2, groups 4, no scope)."""

    def __init__(self, in_channels, scale=2, style="lp", groups=4, dyscope=False):
        super().__init__()
        if style != "lp" or dyscope or scale != 2:
            raise NotImplementedError("DySample: only style='lp', scale=2, dyscope=False has a HIP path")
        assert in_channels >= groups and in_channels % groups == 0
        self.scale, self.style, self.groups = scale, style, groups
        self.offset = nn.Conv2d(in_channels, 2 * groups * scale**2, 1)
        nn.init.normal_(self.offset.weight, 0, 0.001)
        nn.init.constant_(self.offset.bias, 0)
        self.register_buffer("init_pos", self._init_pos())

    def _init_pos(self):
        h = torch.arange((-self.scale + 1) / 2, (self.scale - 1) / 2 + 1) / self.scale
        return torch.stack(torch.meshgrid([h, h], indexing="ij")).transpose(1, 2).repeat(1, self.groups, 1).reshape(
            1, -1, 1, 1)

    def emit(self, plan, x, out=None):
        # offset = 0.25 * conv1x1(x) + init_pos  ->  folded into the conv weights/bias (0.25 is exact)
        w = self.offset.weight.detach().float().cpu() * 0.25
        b = self.offset.bias.detach().float().cpu() * 0.25 + self.init_pos.detach().float().cpu().view(-1)
        y = out if out is not None else plan.alloc(x.n, 2 * x.h, 2 * x.w, x.c)
        if (not os.environ.get("YDBL_DS2_OFF") and self.groups == 4 and x.c in (64, 128, 256)
                and vec_aligned(x) and vec_aligned(y)):
            # offset conv + sample in one launch (csrc/dysample2.hip), bit-identical to the pair below; it reads
            # and writes whole 16-byte channel vectors (check_view(need_vec_align) in ydbl_dysample2)
            wd = plan.const(w.reshape(8 * self.groups, x.c).to(plan.dtype))
            bd = plan.const(b)
            d = _lib.DySample2Desc(x.struct(), wd.data_ptr(), bd.data_ptr(), self.groups, y.struct(), _null_view(),
                                   _null_view(), 0.0, 0.0)
            plan.launch("ydbl_dysample2", d, what="DySample.fused", keep=[d, wd, bd])
            plan.note_writer(y, d)
            return y
        off = plan.alloc(x.n, x.h, x.w, 8 * self.groups)
        emit_conv2d(plan, self.offset, x, off, w, b, what="DySample.offset")
        d = _lib.DySampleDesc(x.struct(), off.struct(), self.groups, y.struct(), _null_view(), _null_view(), 0.0, 0.0)
        plan.launch("ydbl_dysample_ex", d, what="DySample.sample", keep=[d])
        plan.note_writer(y, d)  # a FullPAD_Tunnel on y becomes this launch's second output
        return y


class LSKblock(PlanModule):
    """U/nn/modules_attention/LSKA.py:28-52."""

    def __init__(self, dim):
        super().__init__()
        self.conv0 = nn.Conv2d(dim, dim, 5, padding=2, groups=dim)
        self.conv_spatial = nn.Conv2d(dim, dim, 7, stride=1, padding=9, groups=dim, dilation=3)
        self.conv1 = nn.Conv2d(dim, dim // 2, 1)
        self.conv2 = nn.Conv2d(dim, dim // 2, 1)
        self.conv_squeeze = nn.Conv2d(2, 2, 7, padding=3)
        self.conv = nn.Conv2d(dim // 2, dim, 1)

    def emit(self, plan, x, out=None):
        half = self.conv1.out_channels
        a1, a2 = emit_dw_pair(plan, self.conv0, self.conv_spatial, x, what="LSK.dw5+dw7d3")
        y = out if out is not None else plan.alloc(x.n, x.h, x.w, x.c)
        # fused at dim 256 (DBL-n); at 512 (DBL-s) the five launches measured faster in the two-branch layout:
        # DBL-s bs8 per rank +1.6 %, bs64 +0.4 %; DBL-n bs32 fused +1.1 % (profiles/r06/r06_fusion_switch_sweep.txt,
        # r06_sweep2.txt).  YDBL_LSK_FUSE=1 / 0 forces either.
        fuse = os.environ.get("YDBL_LSK_FUSE")
        if (plan.dtype == torch.float16 and x.c in (256, 512) and (fuse == "1" or (fuse is None and x.c == 256))
                and vec_aligned(x) and vec_aligned(y) and y.base is not x.base):
            # conv1 | conv2 + stats, then gate + conv + x * in two launches (csrc/lsk.hip)
            attn = plan.alloc(x.n, x.h, x.w, 2 * half)
            ws = plan.scratch(_lib.lib.ydbl_lsk_gate_workspace(x.n, x.h, x.w))
            c = plan.const
            w12 = c(torch.cat([self.conv1.weight.detach().float().reshape(half, -1),
                               self.conv2.weight.detach().float().reshape(half, -1)], 0).to(plan.dtype).contiguous())
            b12 = c(torch.cat([self.conv1.bias.detach().float(), self.conv2.bias.detach().float()]))
            sw, sb = c(self.conv_squeeze.weight.float()), c(self.conv_squeeze.bias.float())
            wo = c(self.conv.weight.detach().float().reshape(x.c, half).to(plan.dtype).contiguous())
            bo = c(self.conv.bias.detach().float())
            d = _lib.LskDesc(x.struct(), a1.struct(), a2.struct(), attn.struct(), y.struct(), w12.data_ptr(),
                             b12.data_ptr(), sw.data_ptr(), sb.data_ptr(), wo.data_ptr(), bo.data_ptr(), ws.data_ptr())
            keep = [d, ws, w12, b12, sw, sb, wo, bo]
            plan.launch("ydbl_lsk_attn", d, what="LSK.conv12+stats", keep=keep)
            plan.launch("ydbl_lsk_out", d, what="LSK.gate+conv", keep=keep)
            plan.note_writer(y, d)
            return y
        attn = plan.alloc(x.n, x.h, x.w, 2 * half)
        emit_conv2d(plan, self.conv1, a1, attn.cslice(0, half), what="LSK.conv1")
        emit_conv2d(plan, self.conv2, a2, attn.cslice(half, half), what="LSK.conv2")
        gated = plan.alloc(x.n, x.h, x.w, half)
        ws = plan.scratch(_lib.lib.ydbl_lsk_gate_workspace(x.n, x.h, x.w))
        sw = plan.const(self.conv_squeeze.weight.float())
        sb = plan.const(self.conv_squeeze.bias.float())
        plan.launch("ydbl_lsk_gate", attn.struct(), sw.data_ptr(), sb.data_ptr(), gated.struct(), ws.data_ptr(),
                    what="LSK.gate", keep=[sw, sb, ws])
        return emit_conv2d(plan, self.conv, gated, y, res=x, res_mode=_lib.RES_MUL, what="LSK.conv")


# =============================================================================== head
class DFL(nn.Module):
    """U/nn/modules/block.py:65-84 (fixed 0..15 expectation; computed inside ydbl_detect_decode)."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1


class Detect(PlanModule):
    """U/nn/modules/head.py:21-198 — per level cat(cv2 box branch, cv3 cls branch); decode in ydbl_detect_decode."""

    dynamic = False
    export = False
    end2end = False
    max_det = 300
    shape = None
    legacy = False

    def __init__(self, nc: int = 80, ch: tuple = (), legacy: bool | None = None):
        super().__init__()
        self.nc = nc
        self.nl = len(ch)
        self.reg_max = 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        if legacy is not None:
            self.legacy = legacy
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(
            nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1)) for x in ch
        )
        self.cv3 = (
            nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, self.nc, 1)) for x in ch)
            if self.legacy
            else nn.ModuleList(
                nn.Sequential(
                    nn.Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
                    nn.Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)),
                    nn.Conv2d(c3, self.nc, 1),
                )
                for x in ch
            )
        )
        self.dfl = DFL(self.reg_max)

    def bias_init(self):
        """U/nn/modules/head.py:183-194."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[: self.nc] = math.log(5 / self.nc / (640 / s) ** 2)

    def _forward_plan(self, plan, xs):
        """forward(x) in inference mode (head.py:108-118 with export False): the per-level maps x[i] =
        cat(box, cls) and y = _inference(x) (head.py:143-181: DFL, make_anchors, dist2bbox, sigmoid) decoded by
        ydbl_detect_decode into y [B, 4+nc, A] (no candidates: the threshold is above every score).  Returns the
        call's finisher -> (y, [x_i]) as fresh tensors of the plan's dtype."""
        if not float(self.stride.abs().sum()):
            raise RuntimeError("Detect.stride is unset: build the module through DetectionModel (stride probe)")
        levels = self.emit(plan, xs)
        B = levels[0].n
        A = sum(lv.h * lv.w for lv in levels)
        dev = plan.device
        pred = torch.empty((B, 4 + self.nc, A), dtype=torch.float32, device=dev)
        cand = [torch.empty((B, A, 4), dtype=torch.float32, device=dev), torch.empty((B, A), dtype=torch.float32,
                device=dev), torch.empty((B, A), dtype=torch.int32, device=dev),
                torch.empty((B, A), dtype=torch.int32, device=dev), torch.zeros((B,), dtype=torch.int32, device=dev)]
        plan.buffers += [pred, *cand]
        boxes = (View * 3)(*[lv.cslice(0, 4 * self.reg_max).struct() for lv in levels])
        clss = (View * 3)(*[lv.cslice(4 * self.reg_max, self.nc).struct() for lv in levels])
        strides = (C.c_float * 3)(*[float(s) for s in self.stride.tolist()])
        dd = _lib.DecodeDesc(boxes, clss, len(levels), self.nc, strides, 2.0, 0, None, 0, pred.data_ptr(),
                             *[t.data_ptr() for t in cand], A)
        plan.launch("ydbl_detect_decode", dd, what="Detect.decode", keep=[dd])
        dt = plan.dtype
        return lambda: (pred.to(dt, copy=True), [lv.nchw().contiguous() for lv in levels])

    def emit(self, plan, xs, out=None):
        """Per level: one NHWC buffer [B,h,w,64+nc] (box logits | class logits) = the reference's x[i]."""
        levels = []
        for i, x in enumerate(xs):
            lv = plan.alloc(x.n, x.h, x.w, self.no)
            if not emit_detect_box(plan, self.cv2[i], x, lv.cslice(0, 4 * self.reg_max)):
                t = emit_conv3x3_pair(plan, self.cv2[i][0], self.cv2[i][1], x)
                emit_conv2d(plan, self.cv2[i][2], t, lv.cslice(0, 4 * self.reg_max), what="Detect.box")
            if self.legacy:
                u = self.cv3[i][0].emit(plan, x)
                u = self.cv3[i][1].emit(plan, u)
            else:  # [DWConv, Conv1x1] x 2: each pair is one fused depthwise -> pointwise launch; the class conv
                # cv3[i][2] (64 -> nc <= 4) rides in the second pair's epilogue
                cls_out = lv.cslice(4 * self.reg_max, self.nc)
                u, _ = emit_dw_pw(plan, self.cv3[i][0][0], self.cv3[i][0][1], x)
                u, done = emit_dw_pw(plan, self.cv3[i][1][0], self.cv3[i][1][1], u, tail_conv=self.cv3[i][2],
                                     tail_out=cls_out)
                if done:
                    levels.append(lv)
                    continue
            emit_conv2d(plan, self.cv3[i][2], u, lv.cslice(4 * self.reg_max, self.nc), what="Detect.cls")
            levels.append(lv)
        return levels


def emit_module(m: nn.Module, plan: Plan, x, out=None):
    """Emit any parsed layer: built-in modules (HIP launches), nn.Sequential repeats, and registered plugin
    classes that only have a torch forward (emit_torch)."""
    if isinstance(m, nn.Sequential):
        return emit_seq(plan, m, x, out)
    if hasattr(m, "emit"):
        return m.emit(plan, x, out)
    if type(m).forward is not nn.Module.forward:
        return emit_torch(m, plan, x, out)
    raise NotImplementedError(f"{type(m).__name__} has neither emit() nor forward()")
