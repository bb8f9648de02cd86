"""Model construction (YAML -> layers) and plan compilation for the MI355X path.

Construction follows U/nn/tasks.py:947-1242 (parse_model, yaml_model_load,
guess_model_scale) for the layer types the DBL configurations use; modules
are looked up BY CLASS NAME, exactly like the reference's plugin mechanism
(``globals()[m]``, U/nn/tasks.py:974), so ``register_module`` can swap in
another implementation with the same constructor signature.

``DetectionModel.compile(batch, h, w, dtype)`` turns the layer list into a
``Plan`` (U/nn/tasks.py:145-172 ``_predict_once`` order), with every Concat
input written in place into its slice of the concat buffer.
"""

from __future__ import annotations

import json
import math
import os
import re
from copy import deepcopy
from pathlib import Path

import torch
import torch.nn as nn

from ..runtime import TV, Plan, round_up, weights_signature, ydbl_env  # noqa: F401 (re-exported)
from .. import _lib
from . import modules as M

CFG_DIR = Path(__file__).resolve().parent.parent / "cfg" / "models"

# class-name registry = the reference's globals() lookup
REGISTRY: dict[str, type] = {
    c.__name__: c
    for c in (M.Conv, M.DWConv, M.DSConv, M.GhostConv, M.Concat, M.Bottleneck, M.C2f, M.C3, M.C3Ghost,
              M.GhostBottleneck, M.DSBottleneck, M.DSC3k, M.DSC3k2, M.HyperACE, M.DownsampleConv,
              M.FullPAD_Tunnel, M.DySample, M.LSKblock, M.Detect)
}
_C1C2 = {"Conv", "DWConv", "GhostConv", "Bottleneck", "GhostBottleneck", "C2f", "C3", "C3Ghost", "DSC3k2", "DSConv",
         "DSBottleneck"}
_REPEAT_ARG = {"C2f", "C3", "C3Ghost", "DSC3k2"}
_C1_ONLY = {"DySample", "LSKblock"}


def register_module(cls, name: str | None = None):
    """Plug a module class in under a YAML name (same constructor contract as the reference, whose parse_model
    resolves names through globals(), U/nn/tasks.py:974).  Either contract works: a class with
    ``emit(plan, x, out)`` (HIP launches, as the built-ins) or a plain torch ``forward(x)``, which runs inside the
    compiled plan as a captured torch step on NCHW views of its inputs (nn.modules.emit_torch).  Channel
    bookkeeping for a plugin name follows the reference's rule for names it does not know (c2 = ch[f])."""
    REGISTRY[name or cls.__name__] = cls
    return cls


def make_divisible(x, divisor):
    """U/utils/ops.py:130-143."""
    if isinstance(divisor, torch.Tensor):
        divisor = int(divisor.max())
    return math.ceil(x / divisor) * divisor


def guess_model_scale(model_path) -> str:
    """U/nn/tasks.py:1227-1242."""
    m = re.search(r"yolo[v]?\d+([nslmx])", Path(model_path).stem)
    return m.group(1) if m else ""


def yaml_model_load(path) -> dict:
    """U/nn/tasks.py:1211-1224: 'yolov13n_DBL.yaml' -> unified 'yolov13_DBL' config with scale 'n'.

    Built-in configs live in ydbl/cfg/models/*.json; an existing .yaml/.json path is read directly.
    """
    path = Path(path)
    unified = re.sub(r"(\d+)([nslmx])(.+)?$", r"\1\3", path.stem)
    if path.exists():
        if path.suffix in (".yaml", ".yml"):
            import yaml

            d = yaml.safe_load(path.read_text())
        else:
            d = json.loads(path.read_text())
    else:
        for cand in (CFG_DIR / f"{unified}.json", CFG_DIR / f"{path.stem}.json"):
            if cand.exists():
                d = json.loads(cand.read_text())
                break
        else:
            raise FileNotFoundError(f"model config '{path}' not found (built-in: {sorted(p.stem for p in CFG_DIR.glob('*.json'))})")
    d["scale"] = guess_model_scale(path)
    d["yaml_file"] = str(path)
    return d


def parse_model(d: dict, ch: int = 3, verbose: bool = False):
    """U/nn/tasks.py:947-1208 for the module set of the DBL configs."""
    legacy = True
    nc, scales = d.get("nc"), d.get("scales")
    depth, width, max_channels = d.get("depth_multiple", 1.0), d.get("width_multiple", 1.0), float("inf")
    scale = "?"
    if scales:
        scale = d.get("scale") or tuple(scales.keys())[0]
        if scale not in scales:
            raise KeyError(f"scale '{scale}' not defined by this config (available: {list(scales)})")
        depth, width, max_channels = scales[scale]
    ch = [ch]
    layers, save, c2 = [], [], ch[-1]
    for i, (f, n, name, args) in enumerate(d["backbone"] + d["head"]):
        if name not in REGISTRY:
            raise KeyError(f"module '{name}' (layer {i}) has no MI355X implementation")
        m = REGISTRY[name]
        args = [nc if a == "nc" else a for a in args]
        n = n_ = max(round(n * depth), 1) if n > 1 else n
        if name in _C1C2:
            c1, c2 = ch[f], args[0]
            if c2 != nc:
                c2 = make_divisible(min(c2, max_channels) * width, 8)
            args = [c1, c2, *args[1:]]
            if name in _REPEAT_ARG:
                args.insert(2, n)
                n = 1
            if name == "DSC3k2":
                legacy = False
        elif name == "Concat":
            c2 = sum(ch[x] for x in f)
        elif name == "Detect":
            args.append([ch[x] for x in f])
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
            m.legacy = legacy  # class attribute, as the reference sets it (U/nn/tasks.py:1111-1112)
            m_ = m(*args)
        else:
            m_ = nn.Sequential(*(m(*args) for _ in range(n))) if n > 1 else m(*args)
        m_.np = sum(x.numel() for x in m_.parameters())
        m_.i, m_.f, m_.type = i, f, name
        if verbose:
            print(f"{i:>3}{str(f):>20}{n_:>3}{m_.np:10.0f}  {name:<20}{str(args):<30}")
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


class DetectionModel(nn.Module):
    """U/nn/tasks.py:313-359 + BaseModel.fuse (:207-235)."""

    def __init__(self, cfg="yolov13n_DBL.yaml", ch=3, nc=None, verbose=False):
        super().__init__()
        self.yaml = cfg if isinstance(cfg, dict) else yaml_model_load(cfg)
        ch = self.yaml["ch"] = self.yaml.get("ch", ch)
        if nc and nc != self.yaml["nc"]:
            self.yaml["nc"] = nc
        self.model, self.save = parse_model(deepcopy(self.yaml), ch=ch, verbose=verbose)
        self.names = {i: f"{i}" for i in range(self.yaml["nc"])}
        self.inplace = self.yaml.get("inplace", True)
        self.end2end = False
        m = self.model[-1]
        # Stride probe by shape propagation at 256x256 (the reference runs a train-mode forward on
        # zeros, U/nn/tasks.py:337-350; only its output shapes are used for the strides).
        s = 256
        levels = self.compile(1, s, s, torch.float32, device="meta").levels
        m.stride = torch.tensor([s / lv.h for lv in levels])
        self.stride = m.stride
        m.bias_init()
        for mod in self.modules():  # U/utils/torch_utils.py:410-420
            if isinstance(mod, nn.BatchNorm2d):
                mod.eps = 1e-3
                mod.momentum = 0.03
        self._fused = False

    @property
    def nc(self):
        return self.model[-1].nc

    MAX_FORWARD_SESSIONS = 2

    def forward(self, x, *args, **kwargs):
        """BaseModel.forward -> predict -> _predict_once (U/nn/tasks.py:109-172) with Detect's inference return
        (U/nn/modules/head.py:108-118): ``(y, feats)``, y [B, 4+nc, A] = decoded xywh boxes (pixels) + class
        scores (Detect._inference, head.py:143-181), feats = the per-level head maps cat(box, cls)
        [B, 64+nc, H_i, W_i].  This is the call AutoBackend makes (U/nn/autobackend.py:503-528, ``self.model(im)``).

        Runs the compiled HIP plan of x's (batch, h, w, dtype) on x's device -- forward + decode, no NMS --
        replayed as a hipGraph; fp16 input takes the half path (AutoBackend fp16, autobackend.py:145-155).
        BN is folded and the semantics are always inference (eval) ones; training / loss (dict input) and
        augment / profile / visualize / embed are not on this path.  Returns fresh tensors (the plan's buffers
        are reused by the next call).  CPU tensors raise: there is no CPU execution path."""
        if isinstance(x, dict):
            raise NotImplementedError("training loss (dict input) is outside the inference path")
        if args or any(kwargs.get(k) for k in ("augment", "profile", "visualize", "embed")):
            raise NotImplementedError("augment / profile / visualize / embed are outside the inference path")
        if not isinstance(x, torch.Tensor) or x.ndim != 4:
            raise TypeError("DetectionModel.forward takes a BCHW tensor")
        if x.device.type != "cuda":
            raise RuntimeError(f"ydbl runs on MI355X (gfx950) only: input on {x.device}, move it to a cuda device")
        if x.dtype not in (torch.float32, torch.float16):
            raise TypeError(f"input dtype {x.dtype}: float32 or float16 (half) expected")
        if x.shape[1] != self.yaml["ch"]:
            raise ValueError(f"input has {x.shape[1]} channels, the model {self.yaml['ch']}")
        b, _, h, w = x.shape
        s = self._forward_session(b, h, w, x.dtype == torch.float16, x.device)
        s(x.float())
        sig = weights_signature(self)  # checked while the graph runs
        if sig != s.wsig:  # weights edited since the plan was compiled: rebuild, run again
            s = self._forward_session(b, h, w, x.dtype == torch.float16, x.device, fresh=sig)
            s(x.float())
        y = s.pred.to(x.dtype, copy=True)
        feats = [f.contiguous() for f in s.feats()]
        return y, feats

    def _forward_session(self, b, h, w, half, device, fresh=None):
        from ..engine.session import DetectSession, default_streams

        cache = self.__dict__.setdefault("_fwd_sessions", {})
        # compiled plans hold the routing of the YDBL_* switches at build time (part of the key) and BN-folded
        # copies of the weights (the session's wsig, checked by forward() after each launch)
        key = (b, h, w, half, str(device), ydbl_env())
        s = cache.pop(key, None)
        if s is not None and fresh is not None and s.wsig != fresh:
            s = None  # weights changed since this plan was built
        if s is None:
            while len(cache) >= self.MAX_FORWARD_SESSIONS:
                cache.pop(next(iter(cache)))
            with torch.cuda.device(device):
                s = DetectSession(self, b, h, w, torch.float16 if half else torch.float32, keep_pred=True, nms=False,
                                  device=device, streams=default_streams(b))
            s.wsig = weights_signature(self)
        cache[key] = s  # most recently used last
        return s

    def invalidate(self):
        """Drop every compiled forward plan (after editing weights through ``.data``)."""
        self.__dict__.pop("_fwd_sessions", None)
        return self

    def load_state_dict(self, *args, **kwargs):
        """nn.Module.load_state_dict; compiled forward plans hold folded copies of the weights, so they go."""
        self.invalidate()
        return super().load_state_dict(*args, **kwargs)

    def fuse(self, verbose=False):
        """BN folding happens when a plan is compiled (exactly fuse_conv_and_bn's arithmetic); kept for API parity."""
        self._fused = True
        return self

    def is_fused(self):
        return self._fused

    def compile(self, batch: int, h: int, w: int, dtype=torch.float16, device="cuda", bind=None) -> "CompiledModel":
        """Build the launch plan of one forward: input NCHW fp32 [batch,3,h,w] -> per-level head outputs.
        The plan reads its batch through an input binding (include/ydbl.h ydbl_input_bind): bind_ptr, a device int64
        holding the batch pointer (initially the plan's own staging buffer ``input``), and bind_amax, a device fp32
        batch maximum for LoadTensor's /255 rule (0: scale 1).  bind = (bind_ptr, bind_amax) shares them with a
        caller (a split session: one word per sub-batch plan, one maximum)."""
        plan = Plan(torch.device(device), dtype)
        inp = plan.alloc(batch, h, w, 8)  # RGB padded to 8 channels (16-byte vectors)
        x_nchw = torch.empty((batch, self.yaml["ch"], h, w), dtype=torch.float32, device=plan.device)
        plan.buffers.append(x_nchw)
        if bind is None:
            bind = (torch.empty(1, dtype=torch.int64, device=plan.device),
                    torch.zeros(1, dtype=torch.float32, device=plan.device))
        bind_ptr, bind_amax = bind
        bind_ptr.fill_(x_nchw.data_ptr())
        plan.buffers += [bind_ptr, bind_amax]
        ib = _lib.InputBind(bind_ptr.data_ptr(), bind_amax.data_ptr())
        # Concat outputs are allocated up front; their producers write straight into the slices.
        layers = list(self.model)
        shapes = _propagate_shapes(layers, batch, h, w, self.yaml["ch"])
        out_hint: dict[int, TV] = {}
        cat_buf: dict[int, TV] = {}
        for m in layers:
            if m.type == "Concat":
                srcs = [m.i - 1 if j == -1 else j for j in m.f]
                n_, h_, w_, _ = shapes[srcs[0]]
                buf = plan.alloc(n_, h_, w_, sum(shapes[j][3] for j in srcs))
                cat_buf[m.i] = buf
                off = 0
                for j in srcs:
                    c = shapes[j][3]
                    if j not in out_hint and layers[j].type not in ("Concat",):
                        out_hint[j] = buf.cslice(off, c)
                    off += c
        y: list[TV | None] = []
        x = inp
        stem = layers[0] if M.stem_ok(layers[0], self.yaml["ch"]) and 0 not in out_hint else None
        # layers 0+1 as one kernel when layer 0's map feeds layer 1 only (the full-resolution map never
        # reaches HBM); YDBL_NO_STEM2=1 keeps them separate (A/B switch)
        used_later = any(j == 0 for m in layers[2:] for j in ([m.f] if isinstance(m.f, int) else m.f))
        stem2 = (stem is not None and len(layers) > 1 and not used_later and not os.environ.get("YDBL_NO_STEM2")
                 and M.stem2_ok(layers[0], layers[1], self.yaml["ch"], dtype))
        if stem is None:
            plan.launch("ydbl_input_nchw_to_nhwc", x_nchw.data_ptr(), batch, self.yaml["ch"], h, w, 1.0, inp.struct(),
                        ib, what="input", keep=[ib])
        for m in layers:
            plan.cur_layer = m.i  # (ydbl.quant names fp8 candidates by the layer that emitted them)
            if stem2 and m is layers[1]:
                y.append(x)
                continue
            if m is stem and stem2:  # preprocess + layers 0 and 1 in one kernel
                x = M.emit_stem2(layers[0], layers[1], plan, x_nchw, batch, self.yaml["ch"], h, w,
                                 cat_buf.get(1, out_hint.get(1)), bind=ib)
                y.append(None)  # layer 0's map is never materialised
                continue
            if m is stem:  # preprocess + first Conv fused, straight from the NCHW batch
                x = M.emit_stem(m, plan, x_nchw, batch, self.yaml["ch"], h, w, bind=ib)
                y.append(x)
                continue
            if m.f != -1:
                x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
            out = cat_buf.get(m.i, out_hint.get(m.i))
            x = M.emit_module(m, plan, x, out)
            y.append(x)
        cm = CompiledModel(plan, x_nchw, inp, x, self.model[-1])
        cm.bind_ptr, cm.bind_amax = bind_ptr, bind_amax
        # the InputBind records the launches read (retargeted by CompiledModel.set_bind)
        cm.bind_holders = [st.args[0].bind if st.fn.__name__ == "ydbl_conv_stem2" else st.args[-1]
                           for st in plan.steps if st.fn.__name__ in ("ydbl_conv_stem2", "ydbl_conv_stem",
                                                                       "ydbl_input_nchw_to_nhwc")]
        cm.set_bind(None)  # the plan's own staging buffer, read directly (DetectSession slot 0)
        return cm


class CompiledModel:
    """A compiled forward: ``input`` (NCHW fp32 staging buffer) -> ``levels`` (per-level NHWC head outputs);
    bind_ptr / bind_amax: its input binding (DetectionModel.compile)."""

    def __init__(self, plan: Plan, x_nchw: torch.Tensor, inp: TV, levels: list[TV], detect: M.Detect):
        self.plan, self.input, self.inp, self.levels, self.detect = plan, x_nchw, inp, levels, detect

    def feats(self):
        """Reference-layout per-level outputs x[i] = cat(box, cls) as NCHW views (no copy)."""
        return [lv.nchw() for lv in self.levels]

    def set_bind(self, ptr: torch.Tensor | None, amax: torch.Tensor | None = None):
        """Point every input-reading launch at another binding (device int64 batch-pointer word, fp32 maximum); the
        C-ABI copies the record into the kernel arguments at launch, so a graph captured afterwards keeps it.
        None: no binding -- the launches read the plan's own staging buffer and scale from their arguments, with no
        dependent pointer / maximum load ahead of the input window (the session's own launches, the bench path)."""
        for h in self.bind_holders:
            h.x, h.amax = (None, None) if ptr is None else (ptr.data_ptr(), amax.data_ptr())


def _propagate_shapes(layers, batch, h, w, ch):
    """Output NHWC shape of every layer (cheap symbolic pass over module types)."""
    shapes = []
    cur = (batch, h, w, ch)
    for m in layers:
        if m.f != -1:
            src = shapes[m.f] if isinstance(m.f, int) else [cur if j == -1 else shapes[j] for j in m.f]
        else:
            src = cur
        t = m.type
        mm = m[0] if isinstance(m, nn.Sequential) else m
        if t in ("Conv", "DWConv"):
            k, s, p, d = mm.conv.kernel_size[0], mm.conv.stride[0], mm.conv.padding[0], mm.conv.dilation[0]
            ho, wo = M.conv_out_hw(src[1], src[2], k, s, p, d)
            cur = (batch, ho, wo, (m[-1] if isinstance(m, nn.Sequential) else m).conv.out_channels)
        elif t == "DSConv":
            k, s, p, d = mm.dw.kernel_size[0], mm.dw.stride[0], mm.dw.padding[0], mm.dw.dilation[0]
            ho, wo = M.conv_out_hw(src[1], src[2], k, s, p, d)
            cur = (batch, ho, wo, (m[-1] if isinstance(m, nn.Sequential) else m).pw.out_channels)
        elif t in ("Bottleneck", "DSBottleneck"):
            cur = (batch, src[1], src[2], (m[-1] if isinstance(m, nn.Sequential) else m).cv2.conv.out_channels
                   if t == "Bottleneck" else (m[-1] if isinstance(m, nn.Sequential) else m).cv2.pw.out_channels)
        elif t in ("C2f", "DSC3k2"):
            cur = (batch, src[1], src[2], mm.cv2.conv.out_channels)
        elif t in ("C3", "C3Ghost"):
            cur = (batch, src[1], src[2], mm.cv3.conv.out_channels)
        elif t == "LSKblock":
            cur = src
        elif t == "HyperACE":
            cur = (batch, src[1][1], src[1][2], mm.cv2.conv.out_channels)
        elif t == "DySample":
            cur = (batch, 2 * src[1], 2 * src[2], src[3])
        elif t == "DownsampleConv":
            c = src[3] * 2 if not isinstance(mm.channel_adjust, nn.Identity) else src[3]
            cur = (batch, src[1] // 2, src[2] // 2, c)
        elif t == "FullPAD_Tunnel":
            cur = src[0]
        elif t == "Concat":
            cur = (batch, src[0][1], src[0][2], sum(s_[3] for s_ in src))
        elif t == "Detect":
            cur = None
        elif not hasattr(mm, "emit"):  # a registered forward-only plugin: its output shape from a meta run
            cur = M.torch_out_shape(m, src)
        else:
            raise NotImplementedError(f"{t}: a registered module with emit() needs a shape rule here")
        shapes.append(cur)
    return shapes
