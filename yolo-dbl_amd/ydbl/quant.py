"""fp8 (OCP e4m3) operands for the dense convolutions: BASELINE config 5 ("fp8 weights+activations on
CDNA4 fp8 MFMA, mAP drop reported").

Post-training, calibration-based, per layer:
  - weights: per-output-channel scale sw = 448 / max|w[co]|, w_q = e4m3(w * sw) stored as bytes;
  - activations: per-tensor scale qs = 448 / max|x| of the layer's input over a calibration batch,
    x_q = e4m3(sat(x * qs)) applied by the conv kernels while staging into LDS;
  - the kernels run v_mfma_f32_16x16x32_fp8_fp8 and dequantize the fp32 accumulator with
    dq[co] = 1 / (sw[co] * qs) before bias + activation (include/ydbl.h, ydbl_conv_desc).
Layers kept in fp16: convs with fewer than 64 input channels (stem and the thin high-resolution
backbone convs), depthwise / DSConv / attention / hypergraph kernels, and the Detect head's
final box / class 1x1 convs.  Activations are stored in fp16 between layers.

Bias correction (on by default): e4m3 rounding of the weights and of the activations shifts each output channel's
mean; with mu_c / muq_c the per-channel means of the layer's input before / after e4m3 rounding over the calibration
batch, the fp8 layer gets bias b - (sum_k wq[co][k] muq_c(k) - sum_k w[co][k] mu_c(k)) (k over taps x channels,
c(k) its input channel), so its pre-activation mean matches the fp16 layer's (the empirical bias correction of
data-free / post-training quantization; zero padding at the borders is ignored).

Mixed selection (fraction < 1): every candidate is first switched to e4m3 ALONE and the perturbation
of the Detect head outputs (all levels, mean |delta| over the fp16 run) recorded; the candidates are
then switched in increasing-sensitivity order until `fraction` of the candidates' MACs run in e4m3 --
the layers whose 3-bit mantissa moves the detections most stay fp16 (standard post-training mixed
precision; the synthetic untrained weights make a few layers dominate, tests/test_gpu_model.py).
"""

from __future__ import annotations

import torch

E4M3_MAX = 448.0


def quantize_weights_e4m3(w: torch.Tensor):
    """[Cout][K] fp32 -> (e4m3 bytes [Cout][K] uint8, per-row scale sw [Cout] fp32)."""
    amax = w.abs().amax(dim=1).clamp_min(1e-12)
    sw = E4M3_MAX / amax
    q = (w * sw[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), sw


def _switch(d, state):
    """Set a conv descriptor's operand mode: state None -> fp16, else (w e4m3 ptr, dq ptr, qs, bias ptr)."""
    if state is None:
        d.w, d.dq, d.qscale, d.bias = d._w16, None, 1.0, d._bias16
    else:
        d.w, d.dq, d.qscale, d.bias = state


def candidate_keys(plan) -> list[str]:
    """Stable names of a plan's fp8 candidates, parallel to plan.fp8_candidates: "L<layer>.<Cout>x<Cin>k<kh>#<n>" --
    the model layer that emitted the conv, its shape, and its rank among that layer's candidates of the same shape.
    A calibration recorded at one batch / sub-batch layout applies to every other: fusion choices that depend on the
    map size (a conv folded into a neighbouring launch) drop a candidate without renaming the others."""
    seen, keys = {}, []
    layers = getattr(plan, "fp8_layers", None) or [-1] * len(plan.fp8_candidates)
    for (d, x, w), li in zip(plan.fp8_candidates, layers):
        base = f"L{li}.{w.shape[0]}x{x.c}k{d.kh}"
        n = seen.get(base, 0)
        seen[base] = n + 1
        keys.append(f"{base}#{n}")
    return keys


def _candidate_steps(plan) -> dict:
    """step index -> candidate index (the conv launch of each candidate)."""
    by_desc = {id(c[0]): i for i, c in enumerate(plan.fp8_candidates)}
    return {k: by_desc[id(st.args[0])] for k, st in enumerate(plan.steps) if st.args and id(st.args[0]) in by_desc}


def observe_candidate_inputs(plans, fn):
    """Run every plan once, calling fn(plan_index, candidate_index, x [n, h, w, c] view) right BEFORE each candidate
    conv's launch: its input as that conv reads it.  (A buffer can be rewritten later in the same plan -- HyperACE's
    merged branch 1x1 reads y1, whose slice branch1.cv3 overwrites afterwards -- so reading the inputs after the
    whole plan has run would see the wrong data.)"""
    for pi, p in enumerate(plans):
        steps = _candidate_steps(p)

        def observe(k, p=p, pi=pi, steps=steps):
            ci = steps.get(k)
            if ci is not None:
                fn(pi, ci, p.fp8_candidates[ci][1].torch())

        p.run_observed(observe)
    for p in plans:
        torch.cuda.synchronize(p.device)


def bias_delta_from_means(mu, muq, w32, wq, sw, kk):
    """Per-output-channel shift of an e4m3 conv's pre-activation mean (module docstring) from the per-channel means
    of its input before (mu) and after (muq) e4m3 rounding; w32 = fp32 [Cout][KPAD] tap-major weights, (wq, sw) their
    e4m3 bytes and row scales, kk = kh * kw.  Returns fp32 [Cout] (CPU)."""
    mu, muq = mu.double().cpu(), muq.double().cpu()
    c = mu.numel()
    cout = w32.shape[0]
    w = w32[:, : kk * c].double().reshape(cout, kk, c)
    wdq = (wq.view(torch.float8_e4m3fn).float().double() / sw.double()[:, None])[:, : kk * c].reshape(cout, kk, c)
    return ((wdq * muq).sum((1, 2)) - (w * mu).sum((1, 2))).float()


def bias_delta(xs, qs, w32, wq, sw, kk):
    """bias_delta_from_means over input activations xs ([..., C] tensors, one per sub-batch plan)."""
    tot = mu = muq = 0
    for x in xs:
        xf = x.float().reshape(-1, x.shape[-1])
        mu = mu + xf.sum(0)
        muq = muq + (e4m3_round(xf * qs) / qs).sum(0)
        tot += xf.shape[0]
    return bias_delta_from_means(mu / tot, muq / tot, w32, wq, sw, kk)


def candidate_macs(cand) -> int:
    """MACs of one fp8 candidate launch (desc, input view, fp32 [Cout][KPAD] weights): Cout x the real
    K (kh * kw * Cin, not the padded KPAD) x OUTPUT pixels (a stride-2 conv has a quarter of its input's)."""
    d, x, w = cand
    return int(w.shape[0]) * int(d.kh * d.kw * x.c) * int(d.y.n * d.y.h * d.y.w)


def select_by_mac_budget(sens, macs, fraction):
    """Indices switched to e4m3 for a MAC `fraction`: least sensitive first, each taken while the running
    MAC sum stays within fraction * total (a candidate that would overshoot is skipped, smaller ones after
    it may still fit).  Returns (sorted indices, achieved MAC fraction)."""
    order = sorted(range(len(sens)), key=lambda i: (sens[i], i))
    budget, used, chosen = fraction * sum(macs), 0, []
    for i in order:
        if used + macs[i] > budget + 1e-9:
            continue
        chosen.append(i)
        used += macs[i]
    return sorted(chosen), (used / sum(macs) if macs else 0.0)


class Fp8Calibration:
    """A post-training e4m3 calibration of one model (the static part of config 5's fp8 path), keyed by
    candidate_keys so that it applies to any batch size and sub-batch layout of that model:
      qs[key]      activation scale 448 / amax of the conv's input over the calibration batch,
      delta[key]   its per-output-channel bias correction (fp32 list, module docstring),
      sens[key]    output perturbation with that conv ALONE in e4m3 (mean |delta| of the Detect head maps),
      macs[key]    its MAC share weight (output-pixel MACs at the calibration batch),
    plus a description of the calibration data.  ``switched(fraction)`` is the layer set of a MAC share (least
    sensitive first): one calibration file = one layer set per share, whatever batch the model then runs.
    ``save`` / ``load``: JSON (committed for the fixture weights under tests/golden/)."""

    def __init__(self, qs, delta, sens=None, macs=None, meta=None, sets=None):
        self.qs, self.delta = dict(qs), {k: [float(v) for v in d] for k, d in delta.items()}
        self.sens, self.macs, self.meta = dict(sens or {}), dict(macs or {}), dict(meta or {})
        self.sets = {str(k): sorted(v) for k, v in (sets or {}).items()}  # share -> explicit layer set

    def switched(self, fraction: float) -> list[str]:
        """The layer set of a MAC share: an explicit set recorded for that share (sets, e.g. a greedy search), else
        the least sensitive convs within the MAC budget (select_by_mac_budget)."""
        keys = sorted(self.qs)
        if fraction >= 1.0:
            return keys
        if f"{fraction:g}" in self.sets:
            return list(self.sets[f"{fraction:g}"])
        if not self.sens:
            raise ValueError("this calibration has no sensitivity ranking: only fraction 1.0 applies")
        chosen, _ = select_by_mac_budget([self.sens[k] for k in keys], [self.macs[k] for k in keys], fraction)
        return [keys[i] for i in chosen]

    def mac_fraction(self, keys) -> float:
        tot = sum(self.macs.values())
        return sum(self.macs[k] for k in keys) / tot if tot else 1.0

    def to_json(self) -> dict:
        return {"format": "ydbl-fp8-calibration-1", "meta": self.meta, "qs": self.qs, "delta": self.delta,
                "sens": self.sens, "macs": self.macs, "sets": self.sets}

    @classmethod
    def from_json(cls, d):
        if d.get("format") != "ydbl-fp8-calibration-1":
            raise ValueError("not a ydbl fp8 calibration file")
        return cls(d["qs"], d["delta"], d.get("sens"), d.get("macs"), d.get("meta"), d.get("sets"))

    def save(self, path):
        import json
        from pathlib import Path

        Path(path).write_text(json.dumps(self.to_json(), indent=1, sort_keys=True))
        return path

    @classmethod
    def load(cls, path):
        import json
        from pathlib import Path

        return cls.from_json(json.loads(Path(path).read_text()))


def calibrate(plans, run_calibration, head=None, bias_correct=True, rank=True, meta=None) -> Fp8Calibration:
    """Measure an Fp8Calibration on the images already loaded into `plans` (one Plan, or the sub-batch plans of a
    split session, built from one model: their candidate lists are parallel).  Joint over all plans (the whole
    batch).  Statistics are taken at each conv's launch (observe_candidate_inputs): pass 1 the amax, pass 2 (bias
    correction) the channel means before / after e4m3 rounding at the final scale.  rank: also the per-conv
    sensitivity (each candidate alone in e4m3, `run_calibration()` re-runs every plan, `head()` returns the Detect
    head maps); the plans are left in fp16."""
    plans = list(plans) if isinstance(plans, (list, tuple)) else [plans]
    n = len(plans[0].fp8_candidates)
    assert all(len(p.fp8_candidates) == n for p in plans), "plans differ"
    keys = candidate_keys(plans[0])
    if not n:
        return Fp8Calibration({}, {}, {}, {}, meta)
    for p in plans:  # statistics of the fp16 network
        for d, _, _ in p.fp8_candidates:
            if hasattr(d, "_w16"):
                _switch(d, None)
    dev = plans[0].device
    amax = torch.zeros(n, dtype=torch.float32, device=dev)

    def take_amax(pi, ci, x):
        amax[ci] = torch.maximum(amax[ci], x.abs().amax().float())

    observe_candidate_inputs(plans, take_amax)
    qs = [E4M3_MAX / a if a > 0 else 1.0 for a in amax.tolist()]
    deltas = {}
    if bias_correct:
        sums = [None] * n
        counts = [0] * n

        def take_means(pi, ci, x):
            xf = x.float().reshape(-1, x.shape[-1])
            s = torch.stack([xf.sum(0), (e4m3_round(xf * qs[ci]) / qs[ci]).sum(0)])
            sums[ci] = s if sums[ci] is None else sums[ci] + s
            counts[ci] += xf.shape[0]

        observe_candidate_inputs(plans, take_means)
        for ci in range(n):
            d0, _, w32 = plans[0].fp8_candidates[ci]
            wq, sw = quantize_weights_e4m3(w32)
            mu, muq = (sums[ci] / counts[ci]).cpu()
            deltas[keys[ci]] = bias_delta_from_means(mu, muq, w32, wq, sw, d0.kh * d0.kw).tolist()
    else:
        deltas = {keys[ci]: [0.0] * int(plans[0].fp8_candidates[ci][2].shape[0]) for ci in range(n)}
    cal = Fp8Calibration({keys[ci]: qs[ci] for ci in range(n)}, deltas, meta=meta)
    cal.macs = {keys[ci]: candidate_macs(plans[0].fp8_candidates[ci]) for ci in range(n)}
    if rank:
        if head is None:
            raise ValueError("the sensitivity ranking needs the head outputs (head=...)")
        run_calibration()
        ref = [t.float().clone() for t in head()]
        for ci in range(n):
            apply(plans, cal, keys=[keys[ci]])
            run_calibration()
            cal.sens[keys[ci]] = sum((a.float() - r).abs().mean().item() for a, r in zip(head(), ref))
            apply(plans, cal, keys=[])
    for p in plans:
        p.fp8_sensitivity = [cal.sens.get(k) for k in keys]
    return cal


def apply(plans, cal: Fp8Calibration, fraction: float | None = None, keys=None) -> int:
    """Switch the plans' candidates named by `keys` (default: cal.switched(fraction)) to e4m3 operands at the
    calibration's scales and bias corrections, every other candidate back to fp16.  Candidates the calibration
    does not name stay fp16.  Returns the number switched per plan."""
    plans = list(plans) if isinstance(plans, (list, tuple)) else [plans]
    keys = set(cal.switched(1.0 if fraction is None else fraction) if keys is None else keys)
    n_on = 0
    for p in plans:
        names = candidate_keys(p)
        cache = p.__dict__.setdefault("_fp8_states", {})
        p.fp8_bias_delta, switched = {}, []
        for ci, (k, (d, x, w32)) in enumerate(zip(names, p.fp8_candidates)):
            if not hasattr(d, "_w16"):
                d._w16, d._bias16 = d.w, d.bias
            if k not in keys or k not in cal.qs:
                _switch(d, None)
                continue
            st = cache.get((k, cal.qs[k], id(cal)))
            if st is None:
                wq, sw = quantize_weights_e4m3(w32)
                qs = float(cal.qs[k])
                delta = torch.tensor(cal.delta[k], dtype=torch.float32)
                b8 = (d._b32.clone() if getattr(d, "_b32", None) is not None else torch.zeros(w32.shape[0])) - delta
                st = (p.const(wq.contiguous()).data_ptr(), p.const((1.0 / (sw * qs)).float()).data_ptr(), qs,
                      p.const(b8.float()).data_ptr())
                cache[(k, cal.qs[k], id(cal))] = st
            _switch(d, st)
            p.fp8_bias_delta[ci] = torch.tensor(cal.delta[k], dtype=torch.float32)
            switched.append(ci)
        p.fp8_switched = switched
        p.fp8_enabled = bool(switched)
        p.fp8_mac_fraction = cal.mac_fraction([names[ci] for ci in switched]) if cal.macs else 1.0
        n_on = len(switched)
    return n_on


def enable_fp8(plans, run_calibration, select=None, fraction=1.0, head=None, bias_correct=True,
               calibration: Fp8Calibration | None = None) -> int:
    """Switch fp8 candidate convs to e4m3 operands: with `calibration` (an Fp8Calibration, e.g. loaded from a file)
    its scales, bias corrections and its layer set for `fraction`; else a fresh one measured on the images loaded
    into the plans (calibrate: amax and channel means at each conv's launch, sensitivity ranking when
    fraction < 1).  select(i): restrict to candidate indices (diagnostics).  The calibration used is kept as
    plans[0].fp8_calibration.  Returns the number of convolutions switched per plan."""
    plans = list(plans) if isinstance(plans, (list, tuple)) else [plans]
    cal = calibration
    if cal is None:
        cal = calibrate(plans, run_calibration, head=head, bias_correct=bias_correct, rank=fraction < 1.0)
    keys = cal.switched(fraction)
    if select is not None:
        names = candidate_keys(plans[0])
        keys = [k for k in keys if select(names.index(k))]
    for p in plans:
        p.fp8_calibration = cal
    return apply(plans, cal, keys=keys)


def e4m3_round(t: torch.Tensor) -> torch.Tensor:
    """Round-trip through OCP e4m3 (saturating), fp32 result: the CPU emulation used by the tests."""
    return t.clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float()
