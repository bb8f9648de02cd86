"""One compiled inference configuration: forward + Detect decode + NMS as a single launch plan.

The plan is captured into a hipGraph on first use and replayed afterwards, so
a batch costs one H2D/D2D copy into the static input buffer plus one graph
launch.  Outputs are fixed-shape device buffers ``det [B, max_det, 6]``
(x1, y1, x2, y2, conf, cls) and ``count [B]`` — the all-gather friendly
layout used by the multi-GPU path.
"""

from __future__ import annotations

import ctypes as C
import weakref

import torch

from .. import _lib
from .._lib import DecodeDesc, NmsDesc, View
from ..runtime import BranchGraphRunner, GraphRunner, Plan


SPLIT_MIN_BATCH = 4  # the benched layouts: DBL-n bs32 / DBL-s bs8, bs64 / DBL-l 1280 bs8 (bench.py --streams 2)


def default_streams(batch: int) -> int:
    """Sub-batch graphs of the session predict() / DetectionModel.forward build for a batch: 2 from batch 4 up -- the
    layout bench.py times (DBL-n bs32 +3 %, DBL-s bs64 +9 %, DBL-l 1280 bs8 +8.5 % over one graph;
    3-4 branches measured slower) -- else 1 (a bs1 branch per image leaves most of the chip idle)."""
    return 2 if batch >= SPLIT_MIN_BATCH else 1


# Score threshold from which the NMS runs one workgroup per image instead of the class-split sweep (ydbl_nms_desc
# per_image): at predict-like thresholds every image has at most 1024 candidates (the pair-matrix path; DBL-n bs32
# at conf 0.25: 645 at most) and the split's extra workgroups and merge cost +0.8 % of the step
# (profiles/r05/r05_nms_per_image_ab.txt); validation's conf 0.001 keeps the split.
PER_IMAGE_NMS_CONF = 0.1


class BoundOutputs:
    """A predict() call's outputs in a session's binding slot (DetectSession.launch_bound): det [B, max_det, 6],
    count [B] and LoadTensor's scale, valid as views of the slot until detach() copies them out (on first access, or
    when the slot comes round again while this object is alive)."""

    def __init__(self, det, count, flat, scale, event=None):
        self.det, self.count, self.flat, self.scale, self.own = det, count, flat, scale, False
        self.event = event  # recorded after the replay that wrote the slot

    def detach(self):
        if not self.own:
            if self.event is not None:  # the copy may be issued from another stream than the replay's
                torch.cuda.current_stream(self.flat.device).wait_event(self.event)
            flat = self.flat.clone()
            n = self.det.numel()
            self.det, self.count = flat[:n].view(self.det.shape), flat[n:].view(torch.int32)
            self.flat, self.scale, self.own = flat, self.scale.clone(), True
        return self


class _EagerSlot:
    """use_graph=False: a binding slot's launches run eagerly (the descriptors are pointed at the slot per run)."""

    def __init__(self, session, k, pre):
        self.s, self.k, self.pre = session, k, pre

    def replay(self):
        det, count, _, _ = self.s._pout[self.k]
        self.s._set_slot(self.k, det, count)
        self.pre.run()
        for p in self.s.plans:
            p.run()
        self.s._set_slot(0)


def _det_count(batch: int, max_det: int, dev):
    """det [B, max_det, 6] fp32 and count [B] int32 as views of ONE zeroed buffer (flat), so a caller keeping a batch's
    outputs past the next launch copies them in one go (predict())."""
    flat = torch.zeros(batch * max_det * 6 + batch, dtype=torch.float32, device=dev)
    return flat[: batch * max_det * 6].view(batch, max_det, 6), flat[batch * max_det * 6:].view(torch.int32), flat


class DetectSession:
    """streams = k > 1: the batch is split into k contiguous sub-batches, each compiled into its own launch
    plan (own buffers) writing into slices of the shared det / count (/ pred) outputs; the k plans are captured
    as k independent branches of ONE hipGraph (runtime.BranchGraphRunner; eager mode: one HIP stream per plan).
    At DBL-n/s sizes every launch is short and ramp/tail-bound, so two concurrent half-batch branches fill each
    other's gaps (scripts/stream_probe.py: DBL-n bs32 +10 %, DBL-s bs64 +14 %; one two-branch graph instead of
    two graphs on two streams a further +2.5 %, scripts/graph_branch_probe.py)."""

    def __init__(self, model, batch: int, h: int, w: int, dtype=torch.float16, conf=0.25, iou=0.7, max_det=300,
                 multi_label=False, agnostic=False, classes=None, max_nms=30000, max_wh=7680, clip=True,
                 keep_pred=False, use_graph=True, device="cuda", fp8=False, streams=1, gather_rows=None, nms=True,
                 fp8_calibration=None, _outputs=None, _bind=None):
        if fp8 and dtype != torch.float16:
            raise ValueError("fp8 operands run on the fp16 activation path (half=True)")
        self.model, self.batch, self.h, self.w, self.dtype = model, batch, h, w, dtype
        self.fp8, self.fp8_ready = bool(fp8), False
        self.fp8_calibration = fp8_calibration  # an Fp8Calibration / its file, applied at the first launch
        # fp8=True: every candidate conv in e4m3; fp8=<float in (0, 1)>: that share of the candidates'
        # MACs, least output-sensitive first (ydbl.quant.enable_fp8)
        self.fp8_fraction = float(fp8) if not isinstance(fp8, bool) and 0 < float(fp8) < 1 else 1.0
        self.conf, self.iou, self.max_det = float(conf), float(iou), int(max_det)
        self.children = []
        self.records = None
        # predict()'s in-place path (launch_bound): binding slot 0 is the session's own staging buffer (load()), slots
        # 1 and 2 alternate between predict() calls, each with its own graph (LoadTensor maximum + the plans) and its
        # own det | count outputs, kept until the slot comes round again (then copied if its Results still live)
        self._bound = None  # the last tensor launch_bound() read (introspection)
        self._calls, self._slot_ptrs, self._pgraph, self._pout, self._pheld = 0, {}, {}, {}, {}
        self._max_work = {}  # per binding slot: the batch-max kernel's tickets are reset by its last block
        # the last launch_bound() replay (the slots share the plans' activation buffers): its stream and, per slot, an
        # event recorded after it -- a call from another stream waits for it, detach() waits for its slot's
        self._last_stream, self._slot_ev = None, {}
        if _outputs is None and gather_rows is not None:
            # one record per image [det (max_det*6 fp32) | count (int32) | pad]: the boxes and counts of a batch-
            # sharded predict leave the GPU in ONE all-gather (ydbl.parallel); rows >= batch stay empty padding
            from ..parallel import record_views, record_width

            if gather_rows < batch:
                raise ValueError(f"gather_rows {gather_rows} < batch {batch}")
            self.records = torch.zeros((gather_rows, record_width(self.max_det)), dtype=torch.float32,
                                       device=torch.device(device))
            det_v, cnt_v = record_views(self.records[:batch], self.max_det)
            nc_ = model.model[-1].nc
            A_ = sum((h // int(st)) * (w // int(st)) for st in model.model[-1].stride.tolist())
            _outputs = (det_v, cnt_v,
                        torch.empty((batch, 4 + nc_, A_), dtype=torch.float32, device=device) if keep_pred else None)
        if streams > 1 and batch >= streams:
            self._init_split(model, batch, h, w, dtype, conf, iou, max_det, multi_label, agnostic, classes, max_nms,
                             max_wh, clip, keep_pred, use_graph, device, fp8, streams, nms, _outputs)
            return
        if _bind is None:  # a top-level session owns the binding slots (a split session's children get views)
            self.bind_ptrs = torch.empty((3, 1), dtype=torch.int64, device=torch.device(device))
            self.bind_amax = torch.zeros((3, 1), dtype=torch.float32, device=torch.device(device))
            _bind = (self.bind_ptrs[0], self.bind_amax[0])
        cm = model.compile(batch, h, w, dtype, device=device, bind=_bind)
        self.compiled = cm
        plan: Plan = cm.plan
        det = cm.detect
        nc = det.nc
        multi_label = bool(multi_label) and nc > 1
        A = sum(lv.h * lv.w for lv in cm.levels)
        self.A, self.nc = A, nc
        cap = A * nc if multi_label else A
        dev = plan.device
        self.cand_box = torch.empty((batch, cap, 4), dtype=torch.float32, device=dev)
        self.cand_score = torch.empty((batch, cap), dtype=torch.float32, device=dev)
        self.cand_cls = torch.empty((batch, cap), dtype=torch.int32, device=dev)
        self.cand_idx = torch.empty((batch, cap), dtype=torch.int32, device=dev)
        self.cand_count = torch.zeros((batch,), dtype=torch.int32, device=dev)
        self.out_flat = None
        if _outputs is not None:  # slices of a split session's shared outputs
            self.det, self.count, self.pred = _outputs
        else:
            self.pred = torch.empty((batch, 4 + nc, A), dtype=torch.float32, device=dev) if keep_pred else None
            self.det, self.count, self.out_flat = _det_count(batch, self.max_det, dev)
        self.classes_t = (torch.tensor(list(classes), dtype=torch.int32, device=dev) if classes is not None else None)
        ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(batch, cap, max_nms)), dtype=torch.uint8, device=dev)  # zero-filled once (include/ydbl.h)
        plan.buffers += [self.cand_box, self.cand_score, self.cand_cls, self.cand_idx, self.cand_count, self.det,
                         self.count, ws]
        boxes = (View * 3)(*[lv.cslice(0, 64).struct() for lv in cm.levels])
        clss = (View * 3)(*[lv.cslice(64, nc).struct() for lv in cm.levels])
        strides = (C.c_float * 3)(*[float(s) for s in det.stride.tolist()])
        dd = DecodeDesc(boxes, clss, len(cm.levels), nc, strides, self.conf, int(multi_label),
                        self.classes_t.data_ptr() if self.classes_t is not None else None,
                        len(self.classes_t) if self.classes_t is not None else 0,
                        self.pred.data_ptr() if self.pred is not None else None,
                        self.cand_box.data_ptr(), self.cand_score.data_ptr(), self.cand_cls.data_ptr(),
                        self.cand_idx.data_ptr(), self.cand_count.data_ptr(), cap)
        plan.launch("ydbl_detect_decode", dd, what="Detect.decode", keep=[dd])
        nd = NmsDesc(self.cand_box.data_ptr(), self.cand_score.data_ptr(), self.cand_cls.data_ptr(),
                     self.cand_idx.data_ptr(), self.cand_count.data_ptr(), batch, cap, self.iou, self.max_det,
                     int(max_nms), int(bool(agnostic)), float(max_wh), float(w) if clip else 0.0,
                     float(h) if clip else 0.0, self.det.data_ptr(), self.count.data_ptr(), ws.data_ptr(),
                     self.det.stride(0), self.count.stride(0), int(self.conf >= PER_IMAGE_NMS_CONF))
        if nms:  # nms=False: forward + decode only (DetectionModel.forward -> (y, feats))
            plan.launch("ydbl_nms", nd, what="NMS", keep=[nd])
        self.plan = plan
        self.plans = [plan]
        self.use_graph = use_graph
        self._graph = None
        if hasattr(self, "bind_ptrs"):
            self._init_slots()

    def _init_split(self, model, batch, h, w, dtype, conf, iou, max_det, multi_label, agnostic, classes, max_nms,
                    max_wh, clip, keep_pred, use_graph, device, fp8, streams, nms, outputs):
        from ..parallel import shard_bounds

        dev = torch.device(device)
        det = model.model[-1]
        nc = det.nc
        A = sum((h // int(s)) * (w // int(s)) for s in det.stride.tolist())
        self.out_flat = None
        if outputs is not None:
            self.det, self.count, self.pred = outputs
        else:
            self.det, self.count, self.out_flat = _det_count(batch, self.max_det, dev)
            self.pred = torch.empty((batch, 4 + nc, A), dtype=torch.float32, device=dev) if keep_pred else None
        self.bounds = [shard_bounds(batch, streams, r) for r in range(streams)]
        # per binding slot: one batch-pointer word per sub-batch plan, one batch maximum for all (launch_bound())
        self.bind_ptrs = torch.empty((3, streams), dtype=torch.int64, device=dev)
        self.bind_amax = torch.zeros((3, 1), dtype=torch.float32, device=dev)
        for i, (a, b) in enumerate(self.bounds):
            outs = (self.det[a:b], self.count[a:b], self.pred[a:b] if keep_pred else None)
            self.children.append(DetectSession(model, b - a, h, w, dtype, conf, iou, max_det, multi_label, agnostic,
                                               classes, max_nms, max_wh, clip, keep_pred, use_graph, device, fp8,
                                               nms=nms, _outputs=outs,
                                               _bind=(self.bind_ptrs[0, i:i + 1], self.bind_amax[0])))
        self.streams = [torch.cuda.Stream(dev) for _ in self.children]
        self.plans = [c.plan for c in self.children]
        self.plan = self.plans[0]
        self.use_graph = use_graph
        self._graph = None  # all sub-batch plans as branches of one hipGraph (runtime.BranchGraphRunner)
        self.nc, self.A = self.children[0].nc, self.children[0].A
        self._init_slots()

    @property
    def cand_count(self):
        if self.children:
            return torch.cat([c.cand_count for c in self.children])
        return self._cand_count

    @cand_count.setter
    def cand_count(self, v):
        self._cand_count = v

    # ------------------------------------------------------------------ execution
    def _own_inputs(self):
        return [c.compiled.input.data_ptr() for c in (self.children or [self])]

    def can_bind(self, x: torch.Tensor) -> bool:
        """launch_bound() takes x: a contiguous fp32 tensor of the session's shape on its device, every sub-batch 16-byte
        aligned (the stem kernels' vector loads)."""
        if self.records is not None:  # gather_rows: the NMS writes record rows (out_stride = record width), not slots
            return False
        if (not isinstance(x, torch.Tensor) or x.dtype != torch.float32 or x.device != self.det.device
                or not x.is_contiguous() or tuple(x.shape) != (self.batch, 3, self.h, self.w)
                or (self.fp8 and not self.fp8_ready)):  # (an uncalibrated fp8 session calibrates on a loaded batch)
            return False
        per = 3 * self.h * self.w * 4
        return all((x.data_ptr() + a * per) % 16 == 0 for a, _ in (self.bounds if self.children else [(0, 0)]))

    def _owners(self):
        return [c.compiled for c in self.children] if self.children else [self.compiled]

    def _nms_descs(self):
        return [st.args[0] for c in (self.children or [self]) for st in c.plan.steps if st.fn.__name__ == "ydbl_nms"]

    def _init_slots(self):
        own = torch.tensor(self._own_inputs(), dtype=torch.int64)
        self.bind_ptrs.copy_(own.expand(self.bind_ptrs.shape[0], -1))

    def _set_slot(self, k: int, det: torch.Tensor | None = None, count: torch.Tensor | None = None):
        """Point the plans' input-reading launches at binding slot k and their NMS outputs at det / count (default:
        the session's own), before a capture; the C-ABI copies both into the kernel arguments at launch."""
        for i, cm in enumerate(self._owners()):  # slot 0: no binding, the plans read their own staging buffers
            cm.set_bind(self.bind_ptrs[k, i:i + 1] if k else None, self.bind_amax[k])
        det = self.det if det is None else det
        count = self.count if count is None else count
        for nd, (a, b) in zip(self._nms_descs(), self.bounds if self.children else [(0, self.batch)]):
            nd.out, nd.out_count = det[a:b].data_ptr(), count[a:b].data_ptr()

    def launch_bound(self, x: torch.Tensor) -> "BoundOutputs":
        """predict()'s path for a device batch: the plans read x in place (include/ydbl.h ydbl_input_bind) -- no
        staging copy -- and apply LoadTensor's /255 rule (U/data/loaders.py:561-566) from x's maximum, which the
        launch computes on the device first (ydbl_batch_max_bound, the first node of the same graph: no host sync).
        Calls alternate between two binding slots, each with its own captured graph and its own det | count
        outputs, so nothing is copied per call: the outputs stay in the slot until it comes round again, and are
        copied then only if the call's BoundOutputs (its Results) are still alive -- or on first access."""
        if not self.can_bind(x):
            raise ValueError("launch_bound(): a contiguous fp32 batch of the session's shape on its device, 16-byte "
                             "aligned")
        k = 1 + self._calls % 2
        self._calls += 1
        dev = x.device
        held = self._pheld.get(k)
        held = held() if held is not None else None
        if held is not None:
            held.detach()  # a live result of the call two back: copy it out of the slot before the slot is rewritten
        per = 3 * self.h * self.w * 4
        ptrs = [x.data_ptr() + a * per for a, _ in (self.bounds if self.children else [(0, 0)])]
        if ptrs != self._slot_ptrs.get(k):  # (the words keep their value from call to call for the same tensor)
            self.bind_ptrs[k].copy_(torch.tensor(ptrs, dtype=torch.int64), non_blocking=True)
            self._slot_ptrs[k] = ptrs
        g = self._pgraph.get(k)
        if g is None:
            if self.fp8 and not self.fp8_ready:
                self.calibrate_fp8(calibration=self.fp8_calibration)
            if k not in self._max_work:
                self._max_work[k] = _lib.batch_max_work(dev)
            det, count, flat = _det_count(self.batch, self.max_det, dev)
            scale = torch.empty(1, dtype=torch.float32, device=dev)
            self._pout[k] = (det, count, flat, scale)
            pre = Plan(dev, self.dtype)
            pre.launch("ydbl_batch_max_bound", self.bind_ptrs[k, 0:1].data_ptr(), x.numel(), self._max_work[k].data_ptr(),
                       self.bind_amax[k].data_ptr(), scale.data_ptr(), what="LoadTensor.max")
            self._set_slot(k, det, count)
            if self.use_graph:
                g = (BranchGraphRunner(self.plans, pre=pre) if self.children else GraphRunner(self.plan, pre=pre))
            else:
                g = _EagerSlot(self, k, pre)
            self._set_slot(0)
            self._pgraph[k] = g
        cur = torch.cuda.current_stream(dev)
        if self._last_stream is not None and cur != self._last_stream:  # another stream: the last replay first
            cur.wait_event(self._slot_ev[1 + self._calls % 2])  # (the other slot's event: the previous call)
        g.replay()
        ev = self._slot_ev.get(k)
        if ev is None:
            ev = self._slot_ev[k] = torch.cuda.Event()
        ev.record(cur)
        self._last_stream = cur
        det, count, flat, scale = self._pout[k]
        out = BoundOutputs(det, count, flat, scale, ev)
        self._pheld[k] = weakref.ref(out)
        self._bound = x
        return out

    def load(self, x: torch.Tensor, scale: torch.Tensor | None = None):
        """Copy a BCHW batch into the static input buffer (LoadTensor semantics are the caller's); scale: a 0-dim
        fp32 device tensor the batch is multiplied by on the way in (x * fp32(1/255) is what torch's GPU division by
        255.0 computes, so no host sync is needed for it)."""
        self._bound = None
        if self.children:
            if tuple(x.shape[1:]) != (3, self.h, self.w) or x.shape[0] != self.batch:
                raise ValueError(f"input shape {tuple(x.shape)} != session shape {(self.batch, 3, self.h, self.w)}")
            for c, (a, b) in zip(self.children, self.bounds):
                c.load(x[a:b], scale)
            return
        if tuple(x.shape) != tuple(self.compiled.input.shape):
            raise ValueError(f"input shape {tuple(x.shape)} != session shape {tuple(self.compiled.input.shape)}")
        if scale is None:
            self.compiled.input.copy_(x, non_blocking=True)
        else:  # fp32 before the scale: x.float() / 255.0 as LoadTensor computes it (U/data/loaders.py:566)
            torch.mul(x if x.dtype == torch.float32 else x.float(), scale, out=self.compiled.input)

    def calibrate_fp8(self, x: torch.Tensor | None = None, fraction: float | None = None, calibration=None) -> int:
        """Switch the dense convs to e4m3 operands (ydbl.quant).  calibration (an ydbl.quant.Fp8Calibration or the
        path of one saved with .save()): its activation scales, bias corrections and layer set; else one measured
        now on `x` (default: the batch already loaded) -- kept as self.fp8_calibration, .save() it to reuse.
        fraction < 1: only that share of the candidates' MACs, least output-sensitive convs first (default: the
        session's fp8_fraction).  Returns the number of convs switched."""
        from ..quant import Fp8Calibration, enable_fp8

        if isinstance(calibration, (str, bytes)) or hasattr(calibration, "__fspath__"):
            calibration = Fp8Calibration.load(calibration)
        if x is not None and calibration is None:
            self.load(x)
        frac = self.fp8_fraction if fraction is None else float(fraction)
        # one joint calibration over every sub-batch plan (ydbl.quant.enable_fp8): the same activation scales
        # and the same fp8 layer set for every image of the batch, whichever stream it runs on
        owners = self.children or [self]

        def run_all():
            for c in owners:
                c.plan.run()

        def heads():
            return [t for c in owners for t in c.compiled.feats()]

        n = enable_fp8([c.plan for c in owners], run_all, fraction=frac, head=heads, calibration=calibration)
        self.fp8_calibration = owners[0].plan.fp8_calibration
        for c in owners:
            c._graph = None  # descriptors changed: recapture
            c.fp8_ready = True
        self._graph = None
        self._pgraph.clear()
        self.fp8_ready = True
        return n

    @property
    def fp8_mac_fraction(self) -> float | None:
        """Share of the fp8 candidates' MACs switched to e4m3 (None before calibration)."""
        return getattr(self.plan, "fp8_mac_fraction", None)

    def launch(self):
        if self.fp8 and not self.fp8_ready:
            # a given calibration, else the first batch calibrates (dynamic post-training quantization)
            self.calibrate_fp8(calibration=self.fp8_calibration)
        if self.children and self.use_graph:  # every sub-batch plan a branch of one graph: one launch
            if self._graph is None:
                self._graph = BranchGraphRunner(self.plans)
            self._graph.replay()
            return
        if self.children:  # eager: each sub-batch plan on its own stream, then join
            cur = torch.cuda.current_stream(self.det.device)
            for c, st in zip(self.children, self.streams):
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    c.launch()
            for st in self.streams:
                cur.wait_stream(st)
            return
        if self.use_graph:
            if self._graph is None:
                self._graph = GraphRunner(self.plan)
            self._graph.replay()
        else:
            self.plan.run()

    def __call__(self, x: torch.Tensor | None = None, scale: torch.Tensor | None = None):
        if x is not None:
            self.load(x, scale)
        self.launch()
        return self.det, self.count

    def results(self):
        """Host list of [n_i, 6] tensors (one sync)."""
        cnt = self.count.cpu().tolist()
        det = self.det.cpu()
        return [det[i, : cnt[i]].clone() for i in range(self.batch)]

    def feats(self):
        """Per-level head maps [B, 64+nc, H_i, W_i]: NCHW views of the plan's level buffers (no copy); a split
        session concatenates its sub-batch plans' maps (a copy)."""
        if self.children:
            per = [c.compiled.feats() for c in self.children]
            return [torch.cat([f[i] for f in per]) for i in range(len(per[0]))]
        return self.compiled.feats()
