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
    """Set a conv descriptor's operand mode: state None -> fp16, else (w e4m3 ptr, dq ptr, qs)."""
    if state is None:
        d.w, d.dq, d.qscale = d._w16, None, 1.0
    else:
        d.w, d.dq, d.qscale = state


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


def enable_fp8(plans, run_calibration, select=None, fraction=1.0, head=None) -> int:
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
    states = [[] for _ in plans]  # per plan, per selected candidate: (w e4m3 ptr, dq ptr, qs)
    for k, (i, ax) in enumerate(zip(idx, amax.tolist())):
        qs = E4M3_MAX / ax if ax > 0 else 1.0
        wq, sw = quantize_weights_e4m3(plans[0].fp8_candidates[i][2])
        dqv = (1.0 / (sw * qs)).float()
        for pi, p in enumerate(plans):
            d = p.fp8_candidates[i][0]
            if not hasattr(d, "_w16"):
                d._w16 = d.w
            states[pi].append((p.const(wq.contiguous()).data_ptr(), p.const(dqv).data_ptr(), float(qs)))
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
