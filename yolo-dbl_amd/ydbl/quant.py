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


def enable_fp8(plan, run_calibration, select=None, fraction=1.0, head=None) -> int:
    """Calibrate activation scales with one fp16 pass and switch fp8 candidate convs of `plan` to e4m3
    operands.  `run_calibration()` must execute the plan once on calibration images.  fraction < 1 needs
    `head()` (the Detect head outputs, list of tensors) and keeps the most sensitive convs in fp16.
    Returns the number of convolutions switched."""
    run_calibration()
    torch.cuda.synchronize(plan.device)
    cands = [c for i, c in enumerate(plan.fp8_candidates) if select is None or select(i)]
    if not cands:
        return 0
    amaxes = torch.stack([x.torch().abs().amax().float() for _, x, _ in cands]).cpu()
    states = []
    for (d, _x, w32), ax in zip(cands, amaxes.tolist()):
        qs = E4M3_MAX / ax if ax > 0 else 1.0
        wq, sw = quantize_weights_e4m3(w32)
        wd = plan.const(wq.contiguous())
        dq = plan.const((1.0 / (sw * qs)).float())
        if not hasattr(d, "_w16"):
            d._w16 = d.w
        states.append((wd.data_ptr(), dq.data_ptr(), float(qs)))
    order = list(range(len(cands)))
    if fraction < 1.0:
        if head is None:
            raise ValueError("mixed fp8 selection needs the head outputs (head=...)")
        ref = [t.float().clone() for t in head()]

        def err():
            run_calibration()
            return sum((a.float() - r).abs().mean().item() for a, r in zip(head(), ref))

        sens = []
        for (d, _, _), st in zip(cands, states):
            _switch(d, st)
            sens.append(err())
            _switch(d, None)
        order.sort(key=lambda i: sens[i])
        macs = [w.shape[0] * w.shape[1] * x.n * x.h * x.w for (_, x, w) in cands]
        budget, used, chosen = fraction * sum(macs), 0.0, []
        for i in order:
            if used + macs[i] > budget + 1e-9:
                continue
            chosen.append(i)
            used += macs[i]
        order = chosen
        plan.fp8_sensitivity = sens
    for i in order:
        _switch(cands[i][0], states[i])
    plan.fp8_enabled = True
    plan.fp8_switched = sorted(order)
    return len(order)


def e4m3_round(t: torch.Tensor) -> torch.Tensor:
    """Round-trip through OCP e4m3 (saturating), fp32 result: the CPU emulation used by the tests."""
    return t.clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float()
