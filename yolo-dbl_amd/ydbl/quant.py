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


def bias_delta(xs, qs, w32, wq, sw, kk):
    """Per-output-channel shift of an e4m3 conv's pre-activation mean (module docstring): xs = the layer's input
    activations over the calibration batch ([..., C] tensors, one per sub-batch plan), w32 = fp32 [Cout][KPAD]
    tap-major weights, (wq, sw) their e4m3 bytes and row scales, kk = kh * kw.  Returns fp32 [Cout] (CPU)."""
    tot = mu = muq = 0
    for x in xs:
        xf = x.float().reshape(-1, x.shape[-1])
        mu = mu + xf.sum(0)
        muq = muq + (e4m3_round(xf * qs) / qs).sum(0)
        tot += xf.shape[0]
    mu, muq = (mu / tot).double().cpu(), (muq / tot).double().cpu()
    c = mu.numel()
    cout = w32.shape[0]
    w = w32[:, : kk * c].double().reshape(cout, kk, c)
    wdq = (wq.view(torch.float8_e4m3fn).float().double() / sw.double()[:, None])[:, : kk * c].reshape(cout, kk, c)
    return ((wdq * muq).sum((1, 2)) - (w * mu).sum((1, 2))).float()


def candidate_macs(cand) -> int:
    """MACs of one fp8 candidate launch (desc, input view, fp32 [Cout][KPAD] weights): Cout x the real
    K (kh * kw * Cin, not the padded KPAD) x OUTPUT pixels (a stride-2 conv has a quarter of its input's)."""
    d, x, w = cand
    return int(w.shape[0]) * int(d.kh * d.kw * x.c) * int(d.y.n * d.y.h * d.y.w)


def select_by_mac_budget(sens, macs, fraction):
    """Indices switched to e4m3 for a MAC `fraction`: least sensitive first, each taken while the running
    MAC sum stays within fraction * total (a candidate that would overshoot is skipped, smaller ones after
    it may still fit).  Returns (sorted indices, achieved MAC fraction)."""
    order = sorted(range(len(sens)), key=lambda i: sens[i])
    budget, used, chosen = fraction * sum(macs), 0, []
    for i in order:
        if used + macs[i] > budget + 1e-9:
            continue
        chosen.append(i)
        used += macs[i]
    return sorted(chosen), (used / sum(macs) if macs else 0.0)


def enable_fp8(plans, run_calibration, select=None, fraction=1.0, head=None, bias_correct=True) -> int:
    """Calibrate activation scales with one fp16 pass and switch fp8 candidate convs to e4m3 operands.

    `plans`: one Plan, or the per-sub-batch plans of a split session (built from the same model, so their
    candidate lists are parallel).  Calibration is joint: `run_calibration()` must execute EVERY plan once
    on the calibration images, each candidate's activation scale is taken from the amax of its input over
    all plans (the whole batch), the sensitivity ranking (fraction < 1) is done once on the whole batch
    (`head()` returns the Detect head outputs of all plans), and the same scales and the same layer set go
    to every plan, so an image gets the same fp8 layers whichever sub-batch it lands in.
    Returns the number of convolutions switched per plan."""
    plans = list(plans) if isinstance(plans, (list, tuple)) else [plans]
    run_calibration()
    for p in plans:
        torch.cuda.synchronize(p.device)
    idx = [i for i in range(len(plans[0].fp8_candidates)) if select is None or select(i)]
    assert all(len(p.fp8_candidates) == len(plans[0].fp8_candidates) for p in plans), "plans differ"
    if not idx:
        return 0
    amax = torch.stack([torch.stack([p.fp8_candidates[i][1].torch().abs().amax().float() for i in idx]).cpu()
                        for p in plans]).amax(0)
    states = [[] for _ in plans]  # per plan, per selected candidate: (w e4m3 ptr, dq ptr, qs, bias ptr)
    for p in plans:
        p.fp8_bias_delta = {}
    for k, (i, ax) in enumerate(zip(idx, amax.tolist())):
        qs = E4M3_MAX / ax if ax > 0 else 1.0
        d0, _, w32 = plans[0].fp8_candidates[i]
        wq, sw = quantize_weights_e4m3(w32)
        dqv = (1.0 / (sw * qs)).float()
        b8 = d0._b32.clone() if getattr(d0, "_b32", None) is not None else torch.zeros(w32.shape[0])
        if bias_correct:
            delta = bias_delta([p.fp8_candidates[i][1].torch() for p in plans], qs, w32, wq, sw, d0.kh * d0.kw)
            b8 = b8 - delta
            for p in plans:
                p.fp8_bias_delta[i] = delta
        for pi, p in enumerate(plans):
            d = p.fp8_candidates[i][0]
            if not hasattr(d, "_w16"):
                d._w16, d._bias16 = d.w, d.bias
            states[pi].append((p.const(wq.contiguous()).data_ptr(), p.const(dqv).data_ptr(), float(qs),
                               p.const(b8.float()).data_ptr()))
    chosen = list(range(len(idx)))

    def switch(k, on):
        for pi, p in enumerate(plans):
            _switch(p.fp8_candidates[idx[k]][0], states[pi][k] if on else None)

    if fraction < 1.0:
        if head is None:
            raise ValueError("mixed fp8 selection needs the head outputs (head=...)")
        ref = [t.float().clone() for t in head()]

        def err():
            run_calibration()
            return sum((a.float() - r).abs().mean().item() for a, r in zip(head(), ref))

        sens = []
        for k in range(len(idx)):
            switch(k, True)
            sens.append(err())
            switch(k, False)
        macs = [candidate_macs(plans[0].fp8_candidates[i]) for i in idx]
        chosen, frac = select_by_mac_budget(sens, macs, fraction)
        for p in plans:
            p.fp8_sensitivity, p.fp8_mac_fraction = sens, frac
    else:
        for p in plans:
            p.fp8_mac_fraction = 1.0
    for k in chosen:
        switch(k, True)
    for p in plans:
        p.fp8_enabled = True
        p.fp8_switched = sorted(idx[k] for k in chosen)
    return len(chosen)


def e4m3_round(t: torch.Tensor) -> torch.Tensor:
    """Round-trip through OCP e4m3 (saturating), fp32 result: the CPU emulation used by the tests."""
    return t.clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float()
