"""Oracle restatement of the YOLO-DBL model graph (TEST INFRASTRUCTURE ONLY).

Pure PyTorch-CPU fp32.  Every class keeps the reference's parameter names and
construction order, so a reference ``state_dict`` (or the product's, which
uses the same names) loads unchanged.  Citations are relative to
``/root/reference/models/YOLO/ultralytics`` (``U/`` in SURVEY.md).
Parity status: unpinned (see ``oracle/__init__.py``).
"""

from __future__ import annotations

import json
import math
import re
from copy import deepcopy
from pathlib import Path

import torch
import torch.nn as nn
import torch.nn.functional as F

# the oracle owns its transcription of the reference YAMLs (U/cfg/models/v13/yolov13_DBL{,2}.yaml);
# tests/test_oracle.py::test_model_configs_transcribed pins it to the product copy and, where
# /root/reference exists, to the YAML files themselves
_CFG_DIR = Path(__file__).resolve().parent / "cfg"


# --------------------------------------------------------------------------- helpers
def autopad(k, p=None, d=1):
    """'same' padding; nn/modules/conv.py:30-36."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


def make_divisible(x, divisor):
    """utils/ops.py:130-143."""
    return math.ceil(x / divisor) * divisor


# --------------------------------------------------------------------------- conv.py
class Conv(nn.Module):
    """conv -> BN -> SiLU; nn/modules/conv.py:39-63 (forward_fuse after BN fold)."""

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())

    def forward(self, x):
        if hasattr(self, "bn"):
            return self.act(self.bn(self.conv(x)))
        return self.act(self.conv(x))


class DWConv(Conv):
    """nn/modules/conv.py:128-133 (g = gcd(c1, c2))."""

    def __init__(self, c1, c2, k=1, s=1, d=1, act=True):
        super().__init__(c1, c2, k, s, g=math.gcd(c1, c2), d=d, act=act)


class DSConv(nn.Module):
    """depthwise -> pointwise -> BN -> SiLU, BN never folded; nn/modules/conv.py:91-108, tasks.py:217."""

    def __init__(self, c_in, c_out, k=3, s=1, p=None, d=1, bias=False):
        super().__init__()
        if p is None:
            p = (d * (k - 1)) // 2
        self.dw = nn.Conv2d(c_in, c_in, kernel_size=k, stride=s, padding=p, dilation=d, groups=c_in, bias=bias)
        self.pw = nn.Conv2d(c_in, c_out, 1, 1, 0, bias=bias)
        self.bn = nn.BatchNorm2d(c_out)
        self.act = nn.SiLU()

    def forward(self, x):
        return self.act(self.bn(self.pw(self.dw(x))))


class GhostConv(nn.Module):
    """nn/modules/conv.py:184-197."""

    def __init__(self, c1, c2, k=1, s=1, g=1, act=True):
        super().__init__()
        c_ = c2 // 2
        self.cv1 = Conv(c1, c_, k, s, None, g, act=act)
        self.cv2 = Conv(c_, c_, 5, 1, None, c_, act=act)

    def forward(self, x):
        y = self.cv1(x)
        return torch.cat((y, self.cv2(y)), 1)


class Concat(nn.Module):
    """nn/modules/conv.py:349-359."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        return torch.cat(x, self.d)


# --------------------------------------------------------------------------- block.py
class DFL(nn.Module):
    """Softmax-16 expectation as a fixed 1x1 conv; nn/modules/block.py:65-84."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1

    def forward(self, x):
        b, _, a = x.shape
        return self.conv(x.view(b, 4, self.c1, a).transpose(2, 1).softmax(1)).view(b, 4, a)


class Bottleneck(nn.Module):
    """nn/modules/block.py:344-357."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        return x + self.cv2(self.cv1(x)) if self.add else self.cv2(self.cv1(x))


class C2f(nn.Module):
    """nn/modules/block.py:234-249."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=((3, 3), (3, 3)), e=1.0) for _ in range(n))

    def forward(self, x):
        y = list(self.cv1(x).chunk(2, 1))
        y.extend(m(y[-1]) for m in self.m)
        return self.cv2(torch.cat(y, 1))


class C3(nn.Module):
    """nn/modules/block.py:259-273."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=((1, 1), (3, 3)), e=1.0) for _ in range(n)))

    def forward(self, x):
        return self.cv3(torch.cat((self.m(self.cv1(x)), self.cv2(x)), 1))


class GhostBottleneck(nn.Module):
    """nn/modules/block.py:323-341 (s=1 on the DBL path)."""

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

    def forward(self, x):
        return self.conv(x) + self.shortcut(x)


class C3Ghost(C3):
    """nn/modules/block.py:313-320."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(GhostBottleneck(c_, c_) for _ in range(n)))


class DSBottleneck(nn.Module):
    """nn/modules/block.py:1408-1444."""

    def __init__(self, c1, c2, shortcut=True, e=0.5, k1=3, k2=5, d2=1):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = DSConv(c1, c_, k1, s=1, p=None, d=1)
        self.cv2 = DSConv(c_, c2, k2, s=1, p=None, d=d2)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return x + y if self.add else y


class DSC3k(C3):
    """nn/modules/block.py:1447-1503."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5, k1=3, k2=5, d2=1):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(
            *(DSBottleneck(c_, c_, shortcut=shortcut, e=1.0, k1=k1, k2=k2, d2=d2) for _ in range(n))
        )


class DSC3k2(C2f):
    """nn/modules/block.py:1505-1580."""

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
    """Adaptive hyperedge participation matrix, softmax over tokens; nn/modules/block.py:1582-1657."""

    def __init__(self, node_dim, num_hyperedges, num_heads=4, dropout=0.1, context="both"):
        super().__init__()
        self.num_heads = num_heads
        self.num_hyperedges = num_hyperedges
        self.head_dim = node_dim // num_heads
        self.context = context
        self.prototype_base = nn.Parameter(torch.Tensor(num_hyperedges, node_dim))
        nn.init.xavier_uniform_(self.prototype_base)
        cin = node_dim if context in ("mean", "max") else 2 * node_dim
        if context not in ("mean", "max", "both"):
            raise ValueError(f"Unsupported context '{context}'.")
        self.context_net = nn.Linear(cin, num_hyperedges * node_dim)
        self.pre_head_proj = nn.Linear(node_dim, node_dim)
        self.dropout = nn.Dropout(dropout)
        self.scaling = math.sqrt(self.head_dim)

    def forward(self, X):
        B, N, D = X.shape
        if self.context == "mean":
            ctx = X.mean(dim=1)
        elif self.context == "max":
            ctx = X.max(dim=1)[0]
        else:
            ctx = torch.cat([X.mean(dim=1), X.max(dim=1)[0]], dim=-1)
        protos = self.prototype_base.unsqueeze(0) + self.context_net(ctx).view(B, self.num_hyperedges, D)
        xp = self.pre_head_proj(X)
        xh = xp.view(B, N, self.num_heads, self.head_dim).transpose(1, 2).reshape(B * self.num_heads, N, self.head_dim)
        ph = (
            protos.view(B, self.num_hyperedges, self.num_heads, self.head_dim)
            .permute(0, 2, 1, 3)
            .reshape(B * self.num_heads, self.num_hyperedges, self.head_dim)
            .transpose(1, 2)
        )
        logits = torch.bmm(xh, ph) / self.scaling
        logits = logits.view(B, self.num_heads, N, self.num_hyperedges).mean(dim=1)
        logits = self.dropout(logits)
        return F.softmax(logits, dim=1)


class AdaHGConv(nn.Module):
    """nn/modules/block.py:1659-1708."""

    def __init__(self, embed_dim, num_hyperedges=16, num_heads=4, dropout=0.1, context="both"):
        super().__init__()
        self.edge_generator = AdaHyperedgeGen(embed_dim, num_hyperedges, num_heads, dropout, context)
        self.edge_proj = nn.Sequential(nn.Linear(embed_dim, embed_dim), nn.GELU())
        self.node_proj = nn.Sequential(nn.Linear(embed_dim, embed_dim), nn.GELU())

    def forward(self, X):
        A = self.edge_generator(X)
        He = self.edge_proj(torch.bmm(A.transpose(1, 2), X))
        return self.node_proj(torch.bmm(A, He)) + X


class AdaHGComputation(nn.Module):
    """nn/modules/block.py:1710-1752."""

    def __init__(self, embed_dim, num_hyperedges=16, num_heads=8, dropout=0.1, context="both"):
        super().__init__()
        self.embed_dim = embed_dim
        self.hgnn = AdaHGConv(embed_dim, num_hyperedges, num_heads, dropout, context)

    def forward(self, x):
        B, C, H, W = x.shape
        t = self.hgnn(x.flatten(2).transpose(1, 2))
        return t.transpose(1, 2).view(B, C, H, W)


class C3AH(nn.Module):
    """nn/modules/block.py:1754-1795."""

    def __init__(self, c1, c2, e=1.0, num_hyperedges=8, context="both"):
        super().__init__()
        c_ = int(c2 * e)
        assert c_ % 16 == 0, "Dimension of AdaHGComputation should be a multiple of 16."
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.m = AdaHGComputation(c_, num_hyperedges, c_ // 16, 0.1, context)
        self.cv3 = Conv(2 * c_, c2, 1)

    def forward(self, x):
        return self.cv3(torch.cat((self.m(self.cv1(x)), self.cv2(x)), 1))


class FuseModule(nn.Module):
    """avgpool2(P3) | P4 | nearest-up2(P5) -> 1x1; nn/modules/block.py:1797-1840."""

    def __init__(self, c_in, channel_adjust):
        super().__init__()
        self.downsample = nn.AvgPool2d(kernel_size=2)
        self.upsample = nn.Upsample(scale_factor=2, mode="nearest")
        self.conv_out = Conv((4 if channel_adjust else 3) * c_in, c_in, 1)

    def forward(self, x):
        return self.conv_out(torch.cat([self.downsample(x[0]), x[1], self.upsample(x[2])], dim=1))


class HyperACE(nn.Module):
    """nn/modules/block.py:1842-1895."""

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

    def forward(self, X):
        x = self.fuse(X)
        y = list(self.cv1(x).chunk(3, 1))
        out1 = self.branch1(y[1])
        out2 = self.branch2(y[1])
        y.extend(m(y[-1]) for m in self.m)
        y[1] = out1
        y.append(out2)
        return self.cv2(torch.cat(y, 1))


class DownsampleConv(nn.Module):
    """nn/modules/block.py:1897-1928."""

    def __init__(self, in_channels, channel_adjust=True):
        super().__init__()
        self.downsample = nn.AvgPool2d(kernel_size=2)
        self.channel_adjust = Conv(in_channels, in_channels * 2, 1) if channel_adjust else nn.Identity()

    def forward(self, x):
        return self.channel_adjust(self.downsample(x))


class FullPAD_Tunnel(nn.Module):  # noqa: N801 (reference name)
    """x0 + gate * x1; nn/modules/block.py:1930-1956."""

    def __init__(self):
        super().__init__()
        self.gate = nn.Parameter(torch.tensor(0.0))

    def forward(self, x):
        return x[0] + self.gate * x[1]


# --------------------------------------------------------------------------- DySample / LSKA
class DySample(nn.Module):
    """Learned-offset x2 upsampler, style 'lp'; nn/modules_upsample/DySample.py:20-81."""

    def __init__(self, in_channels, scale=2, style="lp", groups=4, dyscope=False):
        super().__init__()
        assert style == "lp" and not dyscope, "only the DBL configuration (lp, no scope) is restated"
        assert in_channels >= groups and in_channels % groups == 0
        self.scale, self.style, self.groups = scale, style, groups
        self.offset = nn.Conv2d(in_channels, 2 * groups * scale**2, 1)
        nn.init.normal_(self.offset.weight, 0, 0.001)
        nn.init.constant_(self.offset.bias, 0)
        self.register_buffer("init_pos", self._init_pos())

    def _init_pos(self):
        h = torch.arange((-self.scale + 1) / 2, (self.scale - 1) / 2 + 1) / self.scale
        return (
            torch.stack(torch.meshgrid([h, h], indexing="ij"))
            .transpose(1, 2)
            .repeat(1, self.groups, 1)
            .reshape(1, -1, 1, 1)
        )

    def sample(self, x, offset):
        B, _, H, W = offset.shape
        offset = offset.view(B, 2, -1, H, W)
        cw = torch.arange(W) + 0.5
        chh = torch.arange(H) + 0.5
        coords = torch.stack(torch.meshgrid([cw, chh], indexing="ij")).transpose(1, 2).unsqueeze(1).unsqueeze(0)
        coords = coords.type(x.dtype)
        norm = torch.tensor([W, H], dtype=x.dtype).view(1, 2, 1, 1, 1)
        coords = 2 * (coords + offset) / norm - 1
        coords = (
            F.pixel_shuffle(coords.view(B, -1, H, W), self.scale)
            .view(B, 2, -1, self.scale * H, self.scale * W)
            .permute(0, 2, 3, 4, 1)
            .contiguous()
            .flatten(0, 1)
        )
        return F.grid_sample(
            x.reshape(B * self.groups, -1, H, W), coords, mode="bilinear", align_corners=False, padding_mode="border"
        ).view(B, -1, self.scale * H, self.scale * W)

    def forward(self, x):
        return self.sample(x, self.offset(x) * 0.25 + self.init_pos)


class LSKblock(nn.Module):
    """Large separable kernel spatial gate; nn/modules_attention/LSKA.py:28-52."""

    def __init__(self, dim):
        super().__init__()
        self.conv0 = nn.Conv2d(dim, dim, 5, padding=2, groups=dim)
        self.conv_spatial = nn.Conv2d(dim, dim, 7, stride=1, padding=9, groups=dim, dilation=3)
        self.conv1 = nn.Conv2d(dim, dim // 2, 1)
        self.conv2 = nn.Conv2d(dim, dim // 2, 1)
        self.conv_squeeze = nn.Conv2d(2, 2, 7, padding=3)
        self.conv = nn.Conv2d(dim // 2, dim, 1)

    def forward(self, x):
        a1 = self.conv0(x)
        a2 = self.conv_spatial(a1)
        a1 = self.conv1(a1)
        a2 = self.conv2(a2)
        attn = torch.cat([a1, a2], dim=1)
        agg = torch.cat([attn.mean(dim=1, keepdim=True), attn.max(dim=1, keepdim=True)[0]], dim=1)
        sig = self.conv_squeeze(agg).sigmoid()
        attn = a1 * sig[:, 0, :, :].unsqueeze(1) + a2 * sig[:, 1, :, :].unsqueeze(1)
        return x * self.conv(attn)


# --------------------------------------------------------------------------- head.py / tal.py
def make_anchors(shapes, strides, offset=0.5):
    """utils/tal.py:333-345 (shapes = [(h, w), ...])."""
    pts, st = [], []
    for (h, w), s in zip(shapes, strides):
        sx = torch.arange(end=w, dtype=torch.float32) + offset
        sy = torch.arange(end=h, dtype=torch.float32) + offset
        sy, sx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((sx, sy), -1).view(-1, 2))
        st.append(torch.full((h * w, 1), float(s), dtype=torch.float32))
    return torch.cat(pts), torch.cat(st)


def dist2bbox(distance, anchor_points, xywh=True, dim=-1):
    """utils/tal.py:348-357."""
    lt, rb = distance.chunk(2, dim)
    x1y1 = anchor_points - lt
    x2y2 = anchor_points + rb
    if xywh:
        return torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), dim)
    return torch.cat((x1y1, x2y2), dim)


class Detect(nn.Module):
    """Detect head (non-legacy cv3), inference decode; nn/modules/head.py:73-198."""

    def __init__(self, nc=80, ch=(), legacy=False):
        super().__init__()
        self.nc, self.nl, self.reg_max = nc, len(ch), 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        self.legacy = legacy
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(
            nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), nn.Conv2d(c2, 4 * self.reg_max, 1)) for x in ch
        )
        if legacy:
            self.cv3 = nn.ModuleList(nn.Sequential(Conv(x, c3, 3), Conv(c3, c3, 3), nn.Conv2d(c3, nc, 1)) for x in ch)
        else:
            self.cv3 = nn.ModuleList(
                nn.Sequential(
                    nn.Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
                    nn.Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)),
                    nn.Conv2d(c3, nc, 1),
                )
                for x in ch
            )
        self.dfl = DFL(self.reg_max)

    def forward(self, x):
        x = list(x)
        for i in range(self.nl):
            x[i] = torch.cat((self.cv2[i](x[i]), self.cv3[i](x[i])), 1)
        if self.training:
            return x
        return self._inference(x), x

    def _inference(self, x):
        B = x[0].shape[0]
        x_cat = torch.cat([xi.view(B, self.no, -1) for xi in x], 2)
        anchors, strides = (t.transpose(0, 1) for t in make_anchors([xi.shape[2:] for xi in x], self.stride, 0.5))
        box, cls = x_cat.split((self.reg_max * 4, self.nc), 1)
        dbox = dist2bbox(self.dfl(box), anchors.unsqueeze(0), xywh=True, dim=1) * strides
        return torch.cat((dbox, cls.sigmoid()), 1)

    def bias_init(self):
        """nn/modules/head.py:183-194."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[: self.nc] = math.log(5 / self.nc / (640 / s) ** 2)


# --------------------------------------------------------------------------- tasks.py
_REPEAT_INSERT = {"C2f", "C3", "C3Ghost", "DSC3k2"}
_C1C2 = {"Conv", "DWConv", "GhostConv", "Bottleneck", "GhostBottleneck", "C2f", "C3", "C3Ghost", "DSC3k2", "DSConv",
         "DSBottleneck"}
_C1_ONLY = {"DySample", "LSKblock"}
_CLASSES = {
    c.__name__: c
    for c in (Conv, DWConv, DSConv, GhostConv, Concat, Bottleneck, C2f, C3, C3Ghost, GhostBottleneck, DSBottleneck,
              DSC3k, DSC3k2, HyperACE, DownsampleConv, FullPAD_Tunnel, DySample, LSKblock, Detect)
}


def guess_model_scale(model_path):
    """nn/tasks.py:1227-1242."""
    m = re.search(r"yolo[v]?\d+([nslmx])", Path(model_path).stem)
    return m.group(1) if m else ""


def load_model_cfg(name):
    """nn/tasks.py:1211-1224: 'yolov13n_DBL.yaml' -> unified 'yolov13_DBL' config + scale 'n'."""
    p = Path(name)
    unified = re.sub(r"(\d+)([nslmx])(.+)?$", r"\1\3", p.stem)
    cand = [_CFG_DIR / f"{unified}.json", _CFG_DIR / f"{p.stem}.json"]
    for c in cand:
        if c.exists():
            d = json.loads(c.read_text())
            break
    else:
        raise FileNotFoundError(name)
    d["scale"] = guess_model_scale(p)
    d["yaml_file"] = str(p)
    return d


def parse_model(d, ch=3):
    """YAML dict -> nn.Sequential + save list; nn/tasks.py:947-1208 (DBL subset)."""
    legacy = True
    nc, scales = d.get("nc"), d.get("scales")
    depth, width, max_channels = 1.0, 1.0, float("inf")
    scale = "?"
    if scales:
        scale = d.get("scale") or tuple(scales.keys())[0]
        depth, width, max_channels = scales[scale]
    ch = [ch]
    layers, save, c2 = [], [], ch[-1]
    detect_layers = []
    for i, (f, n, m, args) in enumerate(d["backbone"] + d["head"]):
        name = m
        m = _CLASSES[name]
        args = list(args)
        for j, a in enumerate(args):
            if isinstance(a, str) and a == "nc":
                args[j] = nc
        n = n_ = max(round(n * depth), 1) if n > 1 else n
        if name in _C1C2:
            c1, c2 = ch[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_channels) * width, 8)
            args = [c1, c2, *args[1:]]
            if name in _REPEAT_INSERT:
                args.insert(2, n)
                n = 1
            if name == "DSC3k2":
                legacy = False
        elif name == "Concat":
            c2 = sum(ch[x] for x in f)
        elif name == "Detect":
            args.append([ch[x] for x in f])
            detect_layers.append(i)
        elif name == "HyperACE":
            legacy = False
            c1 = ch[f[1]]
            c2 = make_divisible(min(args[0], max_channels) * width, 8)
            he = args[1]
            if scale in "n":
                he = int(args[1] * 0.5)
            elif scale in "x":
                he = int(args[1] * 1.5)
            args = [c1, c2, n, he, *args[2:]]
            n = 1
        elif name == "DownsampleConv":
            c1 = ch[f]
            c2 = c1 * 2
            args = [c1]
        elif name == "FullPAD_Tunnel":
            c2 = ch[f[0]]
        elif name in _C1_ONLY:
            c1 = c2 = ch[f]
            args = [c1, *args[1:]]
        else:
            c2 = ch[f]
        if name == "Detect":
            m_ = Detect(*args, legacy=legacy)
        else:
            m_ = nn.Sequential(*(m(*args) for _ in range(n))) if n > 1 else m(*args)
        m_.i, m_.f, m_.type, m_.n_ = i, f, name, n_
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


class DetectionModel(nn.Module):
    """nn/tasks.py:313-359 + BaseModel._predict_once/fuse (:145-172, :207-235)."""

    def __init__(self, cfg, ch=3, nc=None, stride_probe=True):
        super().__init__()
        self.yaml = cfg if isinstance(cfg, dict) else load_model_cfg(cfg)
        if nc and nc != self.yaml["nc"]:
            self.yaml["nc"] = nc
        self.model, self.save = parse_model(deepcopy(self.yaml), ch=ch)
        self.names = {i: f"{i}" for i in range(self.yaml["nc"])}
        m = self.model[-1]
        if stride_probe:  # train-mode probe, mutates BN running stats exactly like the reference (:337-350)
            s = 256
            m.stride = torch.tensor([s / x.shape[-2] for x in self.forward(torch.zeros(1, ch, s, s))])
        else:
            m.stride = torch.tensor([8.0, 16.0, 32.0])
        self.stride = m.stride
        m.bias_init()
        for mod in self.modules():  # utils/torch_utils.py:410-420
            if isinstance(mod, nn.BatchNorm2d):
                mod.eps = 1e-3
                mod.momentum = 0.03

    def forward(self, x):
        y = []
        for m in self.model:
            if m.f != -1:
                x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
            x = m(x)
            y.append(x if m.i in self.save else None)
        return x

    def fuse(self):
        """Fold BN into Conv/DWConv only (DSConv BN stays); nn/tasks.py:207-235."""
        for m in self.model.modules():
            if isinstance(m, Conv) and hasattr(m, "bn"):
                m.conv = fuse_conv_and_bn(m.conv, m.bn)
                delattr(m, "bn")
        return self


@torch.no_grad()
def fuse_conv_and_bn(conv, bn):
    """utils/torch_utils.py:238-265, same op sequence (diag-matrix products)."""
    fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding,
                      conv.dilation, conv.groups, bias=True).requires_grad_(False)
    w_conv = conv.weight.view(conv.out_channels, -1)
    w_bn = torch.diag(bn.weight.div(torch.sqrt(bn.eps + bn.running_var)))
    fused.weight.copy_(torch.mm(w_bn, w_conv).view(fused.weight.shape))
    b_conv = torch.zeros(conv.weight.shape[0]) if conv.bias is None else conv.bias
    b_bn = bn.bias - bn.weight.mul(bn.running_mean).div(torch.sqrt(bn.running_var + bn.eps))
    fused.bias.copy_(torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn)
    return fused


def build_model(cfg, nc=None, stride_probe=False):
    """Construct an oracle DetectionModel (eval mode, not fused)."""
    m = DetectionModel(cfg, nc=nc, stride_probe=stride_probe)
    return m.eval()
