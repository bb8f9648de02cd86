"""§8(b) module-level plugin contract on the MI355X: every built-in module answers ``m(x)`` (U/nn/tasks.py:158-161)
through a compiled one-module plan, and a registered class with only a torch ``forward`` runs inside the model's
plan (U/nn/tasks.py:974: modules are looked up by name, any class with forward(x) drops in)."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(golden_dir):
    from parity_util import build_pair

    return build_pair("n", 3, golden_dir)


def _layer_inputs(o, x, i):
    """The input(s) the oracle's layer i receives on image batch x (its own _predict_once walk)."""
    y, cur = [], x
    for m in o.model:
        if m.f != -1:
            cur = y[m.f] if isinstance(m.f, int) else [cur if j == -1 else y[j] for j in m.f]
        if m.i == i:
            return cur
        cur = m(cur)
        y.append(cur)
    raise IndexError(i)


def _dev(a, b):
    return (a.double() - b.double()).abs().max().item()


@pytest.mark.parametrize("i", [9, 11, 12, 13, 15, 20, 33])
def test_layer_forward_matches_oracle(golden_dir, i):
    """YOLO(cfg).model.model[i](x) (DSC3k2, LSKblock, HyperACE [3 inputs], DySample, FullPAD_Tunnel [2 inputs],
    Bottleneck, DSC3k2 of the head) against the oracle's layer i on the activations the oracle itself feeds it
    (DBL-n, 2 x 3 x 160 x 160 blob images): |gpu - fp64| within twice the oracle fp32 layer's own deviation from
    its fp64 evaluation + 1e-4 (fp32); fp16 within twice the oracle's half layer's deviation + 1e-2."""
    from ydbl.utils.synthetic import blob_images

    p, o = _pair(golden_dir)
    x = blob_images(2, 160, seed=5)
    with torch.no_grad():
        inp = _layer_inputs(o, x, i)
        lay = o.model[i]
        ref32 = lay(inp)
        dbl = lambda t: [u.double() for u in t] if isinstance(t, list) else t.double()
        hlf = lambda t: [u.half() for u in t] if isinstance(t, list) else t.half()
        ref64 = copy.deepcopy(lay).double()(dbl(inp))
        ref16 = copy.deepcopy(lay).half()(hlf(inp)).float()
    cuda = lambda t, dt: [u.to("cuda", dt) for u in t] if isinstance(t, list) else t.to("cuda", dt)
    mod = p.model.model[i]
    y = mod(cuda(inp, torch.float32))
    assert y.shape == ref64.shape and y.dtype == torch.float32 and y.is_contiguous()
    d, d_ref = _dev(y.cpu(), ref64), _dev(ref32, ref64)
    yh = mod(cuda(inp, torch.float16))
    dh, dh_ref = _dev(yh.float().cpu(), ref64), _dev(ref16, ref64)
    print(f"layer {i} {type(mod).__name__}: fp32 |y - fp64| {d:.3g} (oracle fp32 {d_ref:.3g}); fp16 {dh:.3g} "
          f"(oracle half {dh_ref:.3g})")
    assert d <= 2 * d_ref + 1e-4, (d, d_ref)
    assert yh.dtype == torch.float16 and dh <= 2 * dh_ref + 1e-2, (dh, dh_ref)
    y2 = mod(cuda(inp, torch.float32))  # cached plan, fresh output tensor
    assert torch.equal(y2, y) and y2.data_ptr() != y.data_ptr()


def test_detect_forward_matches_oracle(golden_dir):
    """Detect(x_list) -> (y, x): y = decoded [B, 4+nc, A] boxes + scores (head.py:108-118, 143-181)."""
    from ydbl.utils.synthetic import blob_images

    p, o = _pair(golden_dir)
    x = blob_images(2, 160, seed=7)
    with torch.no_grad():
        inp = _layer_inputs(o, x, 35)
        y32, f32 = o.model[35](inp)
        y64, f64 = copy.deepcopy(o.model[35]).double()([t.double() for t in inp])
    y, feats = p.model.model[35]([t.cuda() for t in inp])
    assert y.shape == y64.shape and len(feats) == 3
    d, d_ref = _dev(y[:, :4].cpu(), y64[:, :4]), _dev(y32[:, :4], y64[:, :4])
    assert d <= 2 * d_ref + 1e-3, (d, d_ref)
    assert _dev(y[:, 4:].cpu(), y64[:, 4:]) <= 2 * _dev(y32[:, 4:], y64[:, 4:]) + 1e-6
    for a, b64, b32 in zip(feats, f64, f32):
        assert _dev(a.cpu(), b64) <= 2 * _dev(b32, b64) + 1e-4


def test_forward_rebuilds_after_weight_edit(golden_dir):
    """A module's compiled plan folds its weights; an in-place edit must show in the next call."""
    p, _ = _pair(golden_dir)
    conv = p.model.model[7]  # Conv 1x1
    x = torch.randn(1, conv.conv.in_channels, 20, 20, device="cuda")
    y0 = conv(x)
    with torch.no_grad():
        conv.bn.bias.add_(1.0)
    y1 = conv(x)
    assert not torch.equal(y0, y1)
    with torch.no_grad():
        conv.bn.bias.sub_(1.0)
    assert torch.allclose(conv(x), y0, atol=1e-5)


@pytest.mark.parametrize("streams", [1, 2])
def test_forward_only_plugin_end_to_end(golden_dir, monkeypatch, streams):
    """A YAML layer resolved to a registered class that has ONLY a torch forward (here the oracle's LSKblock
    restatement registered under "LSKblock") runs inside the compiled plan -- captured into the session's hipGraph,
    as a branch of the split graph at streams=2 -- and the model's decoded output matches the all-HIP model's
    under the fp32 rule against the oracle's fp64 answer."""
    import oracle.model as om
    from parity_util import err_stats, fp32_rule, oracle_legs
    from ydbl import YOLO
    from ydbl.nn import tasks
    from ydbl.utils.synthetic import blob_images, load_trained

    p, o = _pair(golden_dir)
    monkeypatch.setitem(tasks.REGISTRY, "LSKblock", om.LSKblock)
    torch.manual_seed(0)
    q = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(q.model, golden_dir / "trained_yolov13n_DBL_nc3.npz")
    assert type(q.model.model[11][0]) is om.LSKblock
    x = blob_images(4, 160, seed=3)
    s = q.session(4, 160, 160, half=False, conf=0.05, keep_pred=True, use_graph=True, streams=streams)
    owners = s.children or [s]
    assert sum(st.what == "torch.LSKblock" for c in owners for st in c.plan.steps) == 2 * len(owners)
    for _ in range(2):
        s(x.cuda())
    torch.cuda.synchronize()
    ys, _ = oracle_legs(o, x, ("fp64", "fp32"))
    st, st_ref = err_stats(s.pred.cpu(), ys["fp64"]), err_stats(ys["fp32"], ys["fp64"])
    tb, tc = fp32_rule(st_ref)
    print(f"forward-only LSKblock plugin, streams {streams}: |y - fp64| box {st['box_max']:.3g} px (oracle fp32 "
          f"{st_ref['box_max']:.3g}), score {st['conf_max']:.3g}")
    assert st["box_max"] <= tb and st["conf_max"] <= tc, (st, st_ref)
    ph = p.session(4, 160, 160, half=False, conf=0.05, keep_pred=True, use_graph=True, streams=streams)
    ph(x.cuda())
    torch.cuda.synchronize()
    assert (ph.pred.cpu() - s.pred.cpu()).abs()[:, :4].max().item() <= 2 * tb


def _plugin_model(golden_dir, monkeypatch):
    import oracle.model as om
    from ydbl import YOLO
    from ydbl.nn import tasks
    from ydbl.utils.synthetic import load_trained

    monkeypatch.setitem(tasks.REGISTRY, "LSKblock", om.LSKblock)
    torch.manual_seed(0)
    q = YOLO("yolov13n_DBL.yaml", nc=3)
    load_trained(q.model, golden_dir / "trained_yolov13n_DBL_nc3.npz")
    return q


def test_forward_only_plugin_eager_default_stream(golden_dir, monkeypatch):
    """use_graph=False runs the plan eagerly on torch's current stream -- the default (null) stream here, whose
    handle is 0: the plugin step must run on it and agree with the captured run of the same session
    layout (the plugin's torch convs may pick another MIOpen algorithm eagerly than under capture: not bit-equal)."""
    from ydbl.utils.synthetic import blob_images

    q = _plugin_model(golden_dir, monkeypatch)
    x = blob_images(2, 160, seed=3).cuda()
    assert torch.cuda.current_stream().cuda_stream == torch.cuda.default_stream().cuda_stream
    se = q.session(2, 160, 160, half=False, conf=0.05, keep_pred=True, use_graph=False)
    se(x)
    sg = q.session(2, 160, 160, half=False, conf=0.05, keep_pred=True, use_graph=True)
    sg(x)
    torch.cuda.synchronize()
    d = (se.pred - sg.pred).abs()
    assert d[:, :4].max().item() < 1e-2 and d[:, 4:].max().item() < 1e-4, d.max().item()


def test_forward_only_plugin_fp8_calibration(golden_dir, monkeypatch):
    """fp8 calibration runs the plan step by step on the current stream (Plan.run_observed): a plan holding a
    forward-only plugin must calibrate and then replay."""
    from ydbl.utils.synthetic import blob_images

    q = _plugin_model(golden_dir, monkeypatch)
    x = blob_images(2, 160, seed=3).cuda()
    s = q.session(2, 160, 160, half=True, fp8=True, conf=0.05, keep_pred=True, use_graph=True)
    s(x)
    torch.cuda.synchronize()
    assert s.fp8_ready and s.fp8_mac_fraction > 0
    assert torch.isfinite(s.pred).all()
