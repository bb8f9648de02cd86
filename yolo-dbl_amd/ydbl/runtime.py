"""Host runtime: NHWC tensor views, launch plans and hipGraph replay.

A ``Plan`` is the compiled form of one (model, batch, image size, dtype)
configuration: every activation buffer is allocated once up front (device
memory from torch's caching allocator) and the forward is a flat list of
C-ABI launches with prebuilt ctypes descriptors.  ``Plan.run`` walks the list
on one HIP stream; ``GraphRunner`` captures that walk once into a hipGraph and
replays it, so the per-forward host cost is a single graph launch.
"""

from __future__ import annotations

import ctypes as C
import operator
import os
import time
from dataclasses import dataclass, field

import torch

from . import _lib
from ._lib import View, lib


# The YDBL_* switches that change what a plan builds or launches (plan-builder fusions in ydbl.nn.modules / tasks,
# routing in the C-ABI, read at build or at each launch).  tests/test_host_api.py checks this list against the
# names the sources read.
SWITCHES = ("YDBL_DS2_OFF", "YDBL_DS_LEAN", "YDBL_HG_UNFUSED",
            "YDBL_HALO_NB", "YDBL_HALO_SMALL", "YDBL_HALO_T16", "YDBL_VW", "YDBL_WSK_HALF", "YDBL_LSK_FUSE", "YDBL_NMS_FAST", "YDBL_NMS_GROUPS", "YDBL_SPLITK", "YDBL_NO_BNECK", "YDBL_NO_BOX3", "YDBL_NO_CLS_TAIL", "YDBL_DWPW", "YDBL_NO_PAIR3", "YDBL_CV1_FUSE",
            "YDBL_CV3_FUSE", "YDBL_NO_FUSE_PAD", "YDBL_NO_MERGE", "YDBL_NO_STEM2")


def ydbl_env() -> tuple:
    """The settings of the YDBL_* switches (SWITCHES): part of every compiled-plan cache key, since a captured
    graph keeps the routing of its capture.  (~5 us: the predict() hot path; a scan of os.environ took 100.)"""
    get = os.environ.get
    return tuple(get(k) for k in SWITCHES)


_STRUCT_EPOCH = [0]  # bumped whenever any module registers a parameter, buffer or submodule (torch global hooks)


def _bump_epoch(*_):
    _STRUCT_EPOCH[0] += 1


for _reg in ("register_module_parameter_registration_hook", "register_module_buffer_registration_hook",
             "register_module_module_registration_hook"):
    getattr(torch.nn.modules.module, _reg)(_bump_epoch)
_VERSION = operator.attrgetter("_version")


def weights_signature(module: torch.nn.Module) -> tuple:
    """Identity + summed version counters of the module's floating-point parameters and buffers.  A compiled plan
    holds BN-folded copies of the weights taken at build time; the signature changes when a tensor is replaced
    (a registration, caught by the global hooks above) or edited in place through a tracked op (p.copy_() under
    no_grad, load_state_dict, optimizer steps).  Edits through ``.data`` bypass the version counter: call
    ``invalidate()`` / ``Model.reset_sessions()`` after those.  ~90 us for DBL-n's 607 tensors: callers check it
    while the graph runs (Model.predict, DetectionModel.forward)."""
    c = module.__dict__.get("_wsig_cache")
    if c is None or c[0] != _STRUCT_EPOCH[0]:
        ts = [t for t in (*module.parameters(), *module.buffers()) if t.is_floating_point()]
        c = (_STRUCT_EPOCH[0], ts, hash(tuple((id(t), t.data_ptr()) for t in ts)))
        module.__dict__["_wsig_cache"] = c
    return c[2], sum(map(_VERSION, c[1]))


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class TV:
    """NHWC view into a flat device buffer: element (n,y,x,c) at base[off + ((n*H+y)*W+x)*cs + c]."""

    __slots__ = ("base", "off", "n", "h", "w", "c", "cs")

    def __init__(self, base: torch.Tensor, off: int, n: int, h: int, w: int, c: int, cs: int):
        self.base, self.off, self.n, self.h, self.w, self.c, self.cs = base, off, n, h, w, c, cs

    @property
    def dtype(self):
        return self.base.dtype

    @property
    def ptr(self) -> int:
        return self.base.data_ptr() + self.off * self.base.element_size()

    @property
    def shape(self):
        return (self.n, self.h, self.w, self.c)

    def cslice(self, c0: int, c: int) -> "TV":
        assert 0 <= c0 and c0 + c <= self.c, (c0, c, self.c)
        return TV(self.base, self.off + c0, self.n, self.h, self.w, c, self.cs)

    def with_hw(self, h: int, w: int) -> "TV":
        """Reinterpret the pixel grid (same pixel count), e.g. tokens as [N,1] images."""
        assert h * w == self.h * self.w
        return TV(self.base, self.off, self.n, h, w, self.c, self.cs)

    def struct(self) -> View:
        return View(self.ptr, self.n, self.h, self.w, self.c, self.cs, _lib.dtype_code(self.dtype))

    def torch(self) -> torch.Tensor:
        """Strided torch view [n,h,w,c] (no copy)."""
        return torch.as_strided(
            self.base, (self.n, self.h, self.w, self.c), (self.h * self.w * self.cs, self.w * self.cs, self.cs, 1),
            self.off,
        )

    def nchw(self) -> torch.Tensor:
        return self.torch().permute(0, 3, 1, 2)


@dataclass
class Step:
    fn: object
    args: tuple
    what: str
    keep: list = field(default_factory=list)


class Plan:
    """Flat list of C-ABI launches over preallocated device buffers."""

    def __init__(self, device: torch.device, dtype: torch.dtype):
        self.device = torch.device(device)
        self.dtype = dtype
        self.steps: list[Step] = []
        self.buffers: list[torch.Tensor] = []
        self.bytes_allocated = 0
        self._writers: dict = {}  # view key -> (step index, desc) of the conv / DySample launch that wrote it
        self.fp8_candidates: list = []  # (ConvDesc, input view, fp32 [Cout][KPAD] weights) of fp8-able convs
        self.fp8_layers: list = []  # the model layer index that emitted each candidate (-1 outside a model)

    # ---------------------------------------------------------------- memory
    def alloc(self, n: int, h: int, w: int, c: int, dtype: torch.dtype | None = None, cs: int | None = None) -> TV:
        dtype = dtype or self.dtype
        cs = cs or round_up(c, 8)
        t = torch.empty(n * h * w * cs, dtype=dtype, device=self.device)
        self.buffers.append(t)
        self.bytes_allocated += t.numel() * t.element_size()
        return TV(t, 0, n, h, w, c, cs)

    def scratch(self, nbytes: int, zero: bool = False) -> torch.Tensor:
        t = (torch.zeros if zero else torch.empty)(max(int(nbytes), 16), dtype=torch.uint8, device=self.device)
        self.buffers.append(t)
        self.bytes_allocated += t.numel()
        return t

    def splitk_scratch(self, nbytes: int) -> torch.Tensor:
        """fp32 partial tiles of a split-K conv (include/ydbl.h ydbl_conv_workspace).  One buffer serves every such
        conv of the plan -- its launches run one after another on one stream -- and a larger need starts a larger
        buffer (the earlier descriptors keep the one they were given)."""
        cur = getattr(self, "_splitk", None)
        if cur is None or cur.numel() < nbytes:
            cur = self._splitk = self.scratch(nbytes)
        return cur

    def const(self, t: torch.Tensor) -> torch.Tensor:
        t = t.detach().to(self.device).contiguous()
        self.buffers.append(t)
        return t

    # ---------------------------------------------------------------- launches
    def launch(self, name: str, *args, what: str = "", keep=()):
        self.steps.append(Step(getattr(lib, name), args, what or name, list(keep)))

    # Producer bookkeeping for epilogue fusion: dense-conv launches register the view they wrote.
    @staticmethod
    def _vkey(v: TV):
        return (v.base.data_ptr(), v.off, v.n, v.h, v.w, v.c, v.cs)

    def note_writer(self, y: TV, desc) -> None:
        self._writers[self._vkey(y)] = (len(self.steps) - 1, desc)

    def writer_of(self, v: TV):
        """(step index, ConvDesc) of the dense conv that wrote exactly this view, or None."""
        return self._writers.get(self._vkey(v))

    def made_before(self, v: TV, step: int) -> bool:
        """True when v was written by a registered conv launch before `step`."""
        w = self.writer_of(v)
        return w is not None and w[0] < step

    def fuse_second_output(self, writer, y2: TV, r2: TV, a2: float, b2: float) -> TV | None:
        """Give the conv / DySample launch `writer` the second output y2 = a2 * y + b2 * r2.  None (the
        caller then emits a separate ydbl_gate_add) when it already has one or when y2 / r2 break the
        launch-time rules of that entry point: same shape and dtype as y, channel stride % 4 for the
        conv epilogue (ydbl_conv2d_nhwc), 16-byte vectors and pointers for ydbl_dysample_ex."""
        _, d = writer
        if not hasattr(d, "y2") or d.y2.ptr:  # e.g. ydbl_lsk_out: registered as a writer, no second output
            return None
        y = d.y
        for v in (y2, r2):
            if (v.n, v.h, v.w, v.c) != (y.n, y.h, y.w, y.c) or _lib.dtype_code(v.dtype) != y.dtype or v.cs % 4:
                return None
            if isinstance(d, (_lib.DySampleDesc, _lib.DySample2Desc)):
                vec = 16 // v.base.element_size()
                if v.cs % vec or v.c % vec or v.ptr % 16:
                    return None
        d.y2, d.r2, d.a2, d.b2 = y2.struct(), r2.struct(), float(a2), float(b2)
        self.steps[writer[0]].keep.append((y2, r2))
        return y2

    def check_single_stream(self):
        """Every step must run on the one stream it is handed: a libydbl C-ABI entry point (they launch on their
        stream argument only) or a step flagged ``single_stream``.  BranchGraphRunner captures plans as forked
        branches, and on this ROCm a stream fork from inside a forked branch segfaults hipStreamEndCapture
        (the head-branch experiment), so a step that forks streams must never reach a branch."""
        for st in self.steps:
            if not (isinstance(st.fn, C._CFuncPtr) or getattr(st.fn, "single_stream", False)):
                raise RuntimeError(f"plan step '{st.what}' ({st.fn!r}) is not a single-stream launch: it cannot be "
                                   f"captured as a branch of a split session's graph")

    def run_observed(self, observe, stream: int | None = None):
        """Plan.run with observe(step_index) called before every step, on the host, in launch order (the observer
        may enqueue its own device work on the current stream: it sees every buffer exactly as that step will)."""
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream if stream is None else stream)
        for i, st in enumerate(self.steps):
            observe(i)
            rc = st.fn(*st.args, s)
            if rc:
                _lib.check(rc, st.what)

    def run(self, stream: int | None = None):
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream if stream is None else stream)
        for st in self.steps:
            rc = st.fn(*st.args, s)
            if rc:
                _lib.check(rc, st.what)

    def run_timed(self):
        """Eager walk with a HIP event pair around every launch (same stream); returns [(what, ms)]."""
        stream = torch.cuda.current_stream(self.device)
        s = C.c_void_p(stream.cuda_stream)
        evs = []
        # park the stream so the host enqueues every launch before the first one runs: the event
        # pairs then time the kernels, not the host's launch latency
        torch.cuda._sleep(int(1e8))
        for st in self.steps:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(stream)
            rc = st.fn(*st.args, s)
            b.record(stream)
            if rc:
                _lib.check(rc, st.what)
            evs.append((st.what, a, b))
        torch.cuda.synchronize(self.device)
        return [(w, a.elapsed_time(b)) for w, a, b in evs]

    def run_graph_timed(self, reps: int = 8, iters: int = 3):
        """Per-launch time as the kernels run inside the step's hipGraph: every launch captured `reps`
        times back to back into a graph of its own, replayed `iters` times between a HIP event pair on
        the replaying stream; min replay time / reps.  Unlike run_timed this carries no per-launch host
        or event overhead, so it agrees with rocprofv3's kernel durations (bench.py's roofline)."""
        out = []
        for st in self.steps:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
                for _ in range(reps):
                    rc = st.fn(*st.args, s)
                    if rc:
                        _lib.check(rc, st.what)
            g.replay()
            torch.cuda.synchronize(self.device)
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            best = float("inf")
            for _ in range(iters):
                torch.cuda._sleep(int(2e6))
                a.record()
                g.replay()
                b.record()
                torch.cuda.synchronize(self.device)
                best = min(best, a.elapsed_time(b) / reps)
            out.append((st.what, best))
            del g
        return out


class GraphRunner:
    """Captures Plan.run into a hipGraph (torch.cuda.CUDAGraph is hipGraph on ROCm) and replays it."""

    def __init__(self, plan: Plan, warmup: int = 1, pre: Plan | None = None):
        self.plan = plan
        side = torch.cuda.Stream(plan.device)
        side.wait_stream(torch.cuda.current_stream(plan.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                if pre is not None:
                    pre.run(side.cuda_stream)
                plan.run(side.cuda_stream)
        torch.cuda.current_stream(plan.device).wait_stream(side)
        torch.cuda.synchronize(plan.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            if pre is not None:
                pre.run()
            plan.run()
        torch.cuda.synchronize(plan.device)

    def replay(self):
        self.graph.replay()


class BranchGraphRunner:
    """Independent plans (the sub-batch plans of a split DetectSession) captured into ONE hipGraph as parallel
    branches -- a fork / join across side streams inside the capture -- and replayed with one launch.  Against one
    graph per plan, each replayed on its own stream: DBL-n bs32 fp16 1.88-1.89 vs 1.93-1.94 ms per step
    (scripts/graph_branch_probe.py)."""

    def __init__(self, plans, warmup: int = 1, pre: Plan | None = None):
        """pre: a plan run before the fork (both branches wait for it)."""
        for p in plans:
            p.check_single_stream()
        dev = plans[0].device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                if pre is not None:
                    pre.run(side.cuda_stream)
                for p in plans:
                    p.run(side.cuda_stream)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.sides = [torch.cuda.Stream(dev) for _ in plans[1:]]
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            cap = torch.cuda.current_stream(dev)
            if pre is not None:
                pre.run()
            for st in self.sides:
                st.wait_stream(cap)
            plans[0].run()
            for p, st in zip(plans[1:], self.sides):
                with torch.cuda.stream(st):
                    p.run(st.cuda_stream)
            for st in self.sides:
                cap.wait_stream(st)
        torch.cuda.synchronize(dev)

    def replay(self):
        self.graph.replay()


def timed(fn, *a, sync_device=None, **k):
    t0 = time.perf_counter()
    r = fn(*a, **k)
    if sync_device is not None:
        torch.cuda.synchronize(sync_device)
    return r, time.perf_counter() - t0
