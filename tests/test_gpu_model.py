"""End-to-end parity on the MI355X at small sizes: YOLO(cfg) HIP path vs the oracle restatement.

Same state_dict (seeded init + tests/golden trained-like fixture), same inputs.  fp32 mode is judged
against the oracle's fp64 answer with twice the reference fp32 path's own deviation as the bound
(tests/parity_util.py); the BASELINE shapes (640 / 1280, full batches, fp32 and fp16) are in
tests/test_gpu_e2e.py.  Also: NMS bit-exactness on the GPU's own decoded output, graph replay, the
predict() API and the mAP protocol.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(cfg, nc, golden_dir):
    from oracle.model import build_model
    from ydbl import YOLO
    from ydbl.utils.synthetic import load_trained

    scale = cfg[7]
    fx = golden_dir / f"trained_yolov13{scale}_{cfg.split('_', 1)[1][:-5]}_nc{nc}.npz"
    torch.manual_seed(0)
    p = YOLO(cfg, nc=nc)
    load_trained(p.model, fx)
    torch.manual_seed(0)
    o = build_model(cfg, nc=nc)
    load_trained(o, fx)
    o.fuse()
    return p, o


@pytest.mark.parametrize("cfg,nc,size", [("yolov13n_DBL.yaml", 3, 128), ("yolov13n_DBL.yaml", 80, 160),
                                         ("yolov13s_DBL.yaml", 3, 128), ("yolov13s_DBL.yaml", 80, 160),
                                         ("yolov13l_DBL2.yaml", 3, 128), ("yolov13x_DBL2.yaml", 3, 128)])
def test_model_fp32_parity(cfg, nc, size, golden_dir):
    """Small-size companion of tests/test_gpu_e2e.py (which runs the BASELINE shapes): raw per-level head
    outputs, decoded predictions and final detections vs the oracle's fp64 answer, bounded by twice the
    reference fp32 path's own deviation (parity_util.fp32_rule); nc=80 exercises class-index agreement."""
    from parity_util import class_agreement, detections, err_stats, fp32_rule, match_detections, oracle_legs
    from ydbl.utils.synthetic import blob_images

    p, o = _models(cfg, nc, golden_dir)
    x = blob_images(2, size, seed=1234)
    ys, _ = oracle_legs(o, x, ("fp64", "fp32"))
    y64 = ys["fp64"]
    with torch.no_grad():
        _, feats_ref = o(x)
    s = p.session(2, size, size, half=False, conf=0.05, iou=0.7, keep_pred=True, use_graph=False)
    s(x.cuda())
    torch.cuda.synchronize()
    y = s.pred.cpu()
    for f_ref, f in zip(feats_ref, s.feats()):  # raw per-level head outputs (reference x[i] layout)
        assert (f.float().cpu() - f_ref).abs().max().item() < 2e-2
    o32 = err_stats(ys["fp32"], y64)
    st = err_stats(y, y64)
    tb, tc = fp32_rule(o32)
    print(f"{cfg} nc={nc}: gpu |dbox| {st['box_max']:.3g} px, |dconf| {st['conf_max']:.3g}; "
          f"oracle fp32 {o32['box_max']:.3g} px, {o32['conf_max']:.3g}")
    assert st["box_max"] <= tb and st["conf_max"] <= tc
    checked, bad = class_agreement(y, y64, tc)
    assert bad == 0 and (nc < 2 or checked > 0)
    ref = detections(y64, 0.05, 0.7, (size, size))
    m = match_detections(ref, s.results(), y64, 0.05, 0.7, tb, tc)
    assert not m["mismatches"], m["mismatches"][:5]


def test_dbl_n_nms_consistency_fp32(golden_dir):
    """GPU NMS on the GPU's own decoded output == oracle NMS on that same tensor (bit-exact)."""
    from oracle.ops import clip_boxes, non_max_suppression
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(4, 256, seed=77)
    for conf, multi in ((0.05, False), (0.001, True)):
        s = p.session(4, 256, 256, half=False, conf=conf, iou=0.7, multi_label=multi, keep_pred=True)
        s(x.cuda())
        ref = non_max_suppression(s.pred.cpu(), conf, 0.7, multi_label=multi)
        got = s.results()
        for r, g in zip(ref, got):
            clip_boxes(r[:, :4], (256, 256))  # postprocess -> scale_boxes -> clip_boxes (predict.py:23-41)
            assert np.array_equal(g.numpy(), r.numpy())


def test_fp16_detections_agree(golden_dir):
    from oracle.ops import non_max_suppression
    from ydbl.utils.synthetic import blob_images

    p, o = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(2, 256, seed=5)
    with torch.no_grad():
        y_ref, _ = o(x)
    s = p.session(2, 256, 256, half=True, conf=0.05, iou=0.7, keep_pred=True)
    s(x.cuda())
    y = s.pred.cpu()
    assert (y[:, 4:] - y_ref[:, 4:]).abs().max().item() < 5e-2
    ref = non_max_suppression(y_ref, 0.05, 0.7)
    got = s.results()
    for r, g in zip(ref, got):
        n = min(len(r), len(g))
        if n:
            assert abs(len(r) - len(g)) <= max(2, len(r) // 5)


def test_graph_replay_equals_eager(golden_dir):
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(2, 160, seed=9).cuda()
    s_eager = p.session(2, 160, 160, half=True, conf=0.05, use_graph=False)
    s_graph = p.session(2, 160, 160, half=True, conf=0.05, use_graph=True)
    d0, c0 = (t.clone() for t in s_eager(x))
    for _ in range(3):
        d1, c1 = s_graph(x)
    torch.cuda.synchronize()
    assert torch.equal(c0, c1)
    assert torch.equal(d0, d1)


def test_predict_api(golden_dir):
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(3, 256, seed=11)
    res = p.predict(x, conf=0.05, half=True)
    assert len(res) == 3
    for r in res:
        b = r.boxes
        assert b.data.shape[1] == 6 and b.xyxy.shape[1] == 4
        assert (b.xyxy[:, [0, 2]] >= 0).all() and (b.xyxy[:, [0, 2]] <= 256).all()
        assert (b.conf > 0.05).all()
    with pytest.raises(ValueError):
        p.predict(torch.rand(1, 3, 100, 100))
    # uint8-range inputs are divided by 255 (LoadTensor)
    r255 = p.predict(x * 255.0, conf=0.05, half=True)
    assert torch.equal(r255[0].boxes.data, res[0].boxes.data)


def test_predict_runs_benched_layout(golden_dir):
    """predict() builds the session layout bench.py times (ydbl.engine.session.default_streams: two sub-batch
    branches of one hipGraph from batch 4 up), and its detections are bit-equal to that session's
    (U/engine/model.py:501-560 is the reference's predict)."""
    from ydbl.engine.session import default_streams
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    assert default_streams(32) == 2 and default_streams(3) == 1
    x = blob_images(32, 640, seed=1234).cuda()
    res = p.predict(x, half=True)
    used = list(p._sessions.values())[-1]
    assert len(used.children) == 2 and [c.batch for c in used.children] == [16, 16]
    ref = p.session(32, 640, 640, half=True, conf=0.25, iou=0.7, streams=2, keep_pred=False)
    assert ref is used  # the very session the bench layout compiles (same cache key)
    other = p._sessions.copy()
    p._sessions.clear()
    d2, c2 = (t.clone() for t in p.session(32, 640, 640, half=True, streams=2)(x))
    p._sessions.update(other)
    torch.cuda.synchronize()
    assert sum(len(r.boxes.data) for r in res) > 0
    for i, r in enumerate(res):
        assert torch.equal(r.boxes.data, d2[i, : int(c2[i])])
    res3 = p.predict(x[:3], half=True)  # below SPLIT_MIN_BATCH: one graph
    assert len(list(p._sessions.values())[-1].children) == 0 and len(res3) == 3


@pytest.mark.parametrize("batch,streams", [(5, 2), (3, 1)])
def test_predict_reads_device_tensor_in_place(golden_dir, batch, streams):
    """predict() on a contiguous fp32 device tensor binds the plans' input to it (include/ydbl.h ydbl_input_bind: no
    staging copy; LoadTensor's /255 rule, U/data/loaders.py:561-566, applied by the stem kernels from the batch
    maximum): detections bit-equal to the staging-copy path on the LoadTensor-scaled batch, for a [0, 1] and a
    [0, 255] batch; the next plain session call goes back to the staging buffer; other tensors take the copy path."""
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x01 = blob_images(batch, 160, seed=77).cuda()
    got01 = None
    for x, ref_in in ((x01, x01), (x01 * 255.0, x01 * 255.0 / 255.0)):
        res = p.predict(x, half=True, conf=0.05, streams=streams)
        s = list(p._sessions.values())[-1]
        assert s._bound is x and len(s.children) == (streams if streams > 1 else 0)
        got = [r.boxes.data.clone() for r in res]
        d, c = s(ref_in)  # staging copy of the scaled batch: the binding is released
        torch.cuda.synchronize()
        assert s._bound is None
        assert sum(len(g) for g in got) > 0
        for i, g in enumerate(got):
            assert torch.equal(g, d[i, : int(c[i])]), i
        got01 = got01 or got
    xs = torch.cat([x01, x01], 1)[:, :3]  # non-contiguous view: the copy path
    assert not list(p._sessions.values())[-1].can_bind(xs)
    res = p.predict(xs, half=True, conf=0.05, streams=streams)
    assert list(p._sessions.values())[-1]._bound is None
    for i, r in enumerate(res):
        assert torch.equal(r.boxes.data, got01[i])


def test_predict_fp16_device_batch_0_255(golden_dir):
    """A half-precision device batch in [0, 255] takes the staging copy with LoadTensor's rule computed in fp32,
    im.float() / 255.0 (U/data/loaders.py:561-566) -- not x * (1/255) rounded to fp16 first: detections
    bit-equal to the same batch passed as fp32; Results.orig_img is the fp32-scaled image."""
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x16 = (blob_images(4, 160, seed=78) * 255.0).round().half().cuda()
    want = [r.boxes.data.clone() for r in p.predict(x16.float(), half=True, conf=0.05)]
    res = p.predict(x16, half=True, conf=0.05)
    assert sum(len(w) for w in want) > 0
    for r, w in zip(res, want):
        assert torch.equal(r.boxes.data, w)
    assert torch.equal(res[1].orig_img.cpu(), (x16[1].float() / 255.0).permute(1, 2, 0).cpu())


def test_predict_back_to_back_calls_keep_their_batches(golden_dir):
    """Back-to-back predict() calls on different device batches without a sync in between (the in-place path
    alternates two binding slots on the session's own stream while the caller's stream runs ahead): every call's
    Results hold its own batch's detections, bit-equal to a separate synchronous run of that batch, also when a
    tensor is freed right after its call and its memory is reused."""
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    xs = [blob_images(8, 192, seed=s).cuda() for s in (11, 12, 13)]
    xs[1] = xs[1] * 255.0  # this one takes LoadTensor's /255
    ref = []
    for x in xs:
        r = p.predict(x, half=True, conf=0.05)
        torch.cuda.synchronize()
        ref.append([t.boxes.data.clone() for t in r])
    outs = []
    for rep in range(3):
        for i, x in enumerate(xs):
            outs.append((i, p.predict(x, half=True, conf=0.05)))
        tmp = blob_images(8, 192, seed=99).cuda() * 3.0  # freed after its call: its memory goes back to the pool
        outs.append((None, p.predict(tmp, half=True, conf=0.05)))
        del tmp
        junk = torch.full((8, 3, 192, 192), 7.0, device="cuda")  # may take tmp's memory
        del junk
    for i, res in outs:
        if i is None:
            continue
        assert [torch.equal(t.boxes.data, r) for t, r in zip(res, ref[i])] == [True] * 8, i


def _cpu_map50(o, x, labels, conf=0.001):
    """mAP@0.5 of the CPU oracle path under the same val protocol (multi-label NMS, conf .001)."""
    from oracle.ops import clip_boxes, non_max_suppression
    from oracle.metrics import IOUV, box_iou, match_predictions
    from ydbl.utils.metrics import DetMetrics

    with torch.no_grad():
        y, _ = o(x)
    preds = non_max_suppression(y, conf, 0.7, multi_label=True)
    st = {"tp": [], "conf": [], "pred_cls": [], "target_cls": []}
    for i, p in enumerate(preds):
        clip_boxes(p[:, :4], x.shape[2:])
        cls, box = labels[i][:, 0], labels[i][:, 1:]
        tp = match_predictions(p[:, 5], cls, box_iou(box, p[:, :4]), IOUV) if len(cls) and len(p) else \
            torch.zeros(len(p), 10, dtype=torch.bool)
        st["tp"].append(tp); st["conf"].append(p[:, 4]); st["pred_cls"].append(p[:, 5]); st["target_cls"].append(cls)
    m = DetMetrics()
    m.process(*(torch.cat(st[k]).numpy() for k in ("tp", "conf", "pred_cls", "target_cls")))
    return m.box.map50


@pytest.mark.parametrize("half", [False, True, "fp8"])
def test_map50_gpu_vs_cpu_pseudo_gt(golden_dir, half):
    """SURVEY §8d mAP protocol: pseudo ground truth = CPU oracle detections at conf 0.25; GPU and CPU
    paths scored with the same val pipeline; acceptance |mAP50_gpu - mAP50_cpu| <= 0.1."""
    from oracle.ops import clip_boxes, non_max_suppression
    from ydbl.utils.synthetic import blob_images

    p, o = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(6, 256, seed=321)
    with torch.no_grad():
        y, _ = o(x)
    gt = non_max_suppression(y, 0.25, 0.7)
    labels = []
    for g in gt:
        clip_boxes(g[:, :4], (256, 256))
        labels.append(torch.cat([g[:, 5:6], g[:, :4]], 1))
    assert sum(len(lb) for lb in labels) > 0, "pseudo ground truth is empty"
    batch = {"img": x, "cls": torch.cat([lb[:, 0] for lb in labels]),
             "bboxes": torch.cat([lb[:, 1:] for lb in labels]),
             "batch_idx": torch.cat([torch.full((len(lb),), i) for i, lb in enumerate(labels)])}
    m_gpu = p.val(data=[batch], half=bool(half), fp8=half == "fp8").box.map50
    m_cpu = _cpu_map50(o, x, labels)
    tag = "fp8 e4m3 operands" if half == "fp8" else ("fp16" if half else "fp32")
    print(f"mAP50 pseudo-GT: gpu({tag}) {m_gpu:.4f}  cpu {m_cpu:.4f}  drop {m_cpu - m_gpu:+.4f}")
    if half == "fp8":
        # BASELINE config 5 asks for the drop to be reported, not bounded: e4m3 keeps 3 mantissa bits,
        # and these synthetic (untrained) weights amplify every perturbation (one fp8 layer alone moves
        # boxes by ~0.5 px, scripts/fp8_diag.py; the drop moved 0.36 -> 0.51 when only the fp16 stem's
        # accumulation order changed).  Guard against a broken path (mAP ~0), not against the drop.
        assert m_gpu > 0.3
        return
    assert abs(m_gpu - m_cpu) <= 0.1
    assert m_cpu > 0.5


def test_checkpoint_predict_matches_state_dict(tmp_path, golden_dir):
    """YOLO('best.pt') on a reference-format checkpoint (fp16 EMA pickled under the reference's class
    paths, U/engine/trainer.py:513-546) predicts exactly what the same weights loaded as a state_dict do."""
    from test_checkpoint import _save_reference_style
    from ydbl import YOLO
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    path = tmp_path / "best.pt"
    _save_reference_style(p.model, path)
    sd = {k: v.half().float() if v.is_floating_point() else v for k, v in p.model.state_dict().items()}
    a = YOLO(path)
    b = YOLO("yolov13n_DBL.yaml", nc=3).load(sd)
    x = blob_images(2, 256, seed=3)
    ra, rb = a.predict(x, conf=0.05, half=True), b.predict(x, conf=0.05, half=True)
    assert sum(len(r.boxes.data) for r in ra) > 0
    for u, v in zip(ra, rb):
        assert torch.equal(u.boxes.data, v.boxes.data)


def test_split_session_equals_separate_sessions(golden_dir):
    """streams=2 (two sub-batch graphs on two HIP streams writing slices of shared outputs) == the two
    sub-batches run as separate single-stream sessions, bit for bit (same kernels at the same sizes)."""
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(6, 192, seed=21).cuda()
    split = p.session(6, 192, 192, half=True, conf=0.05, keep_pred=True, streams=2)
    assert len(split.children) == 2 and [c.batch for c in split.children] == [3, 3]
    for _ in range(2):
        d, c = split(x)
    torch.cuda.synchronize()
    d, c, pred = d.clone(), c.clone(), split.pred.clone()
    for i, (a, b) in enumerate(split.bounds):
        one = p.session(b - a, 192, 192, half=True, conf=0.05, keep_pred=True)
        d1, c1 = one(x[a:b])
        torch.cuda.synchronize()
        assert torch.equal(c1, c[a:b]) and torch.equal(one.pred, pred[a:b])
        assert torch.equal(d1, d[a:b])  # rows past count are zeroed by the NMS kernel
    assert sum(len(r) for r in split.results()) > 0


@pytest.mark.parametrize("mode", ["fp16", "fp8", "fp8-0.25", "fp8-0.1"])
def test_map50_config5_dbl_s_640(golden_dir, mode):
    """BASELINE config 5 (DBL-s 640, fp8 e4m3 weights + activations) and its fp16 twin, under the SURVEY §8d
    mAP protocol at the reference's val settings (conf 0.001, multi-label NMS, iou .7; U/models/yolo/detect/
    val.py:92-102) on every image of blob_images(16, 640): pseudo ground truth = the CPU oracle's fp32
    detections at the e2e fixture's predict threshold (tests/golden/e2e_s640: conf 0.0171 -- the untrained-like
    DBL-s fixture scores below the 0.25 default), the GPU and CPU paths scored by the same val pipeline.
    fp8-f = the committed calibration's layer set for share f of the candidate MACs in e4m3
    (tests/golden/fp8_calib_yolov13s_DBL_nc3.json, scripts/fp8_calibrate.py; `bench.py --model s --fp8 f` loads
    the same file), fp8 = every candidate.  BASELINE config 5 asks for the fp8 drop to be REPORTED; each share's
    drop is printed and bounded by its measured value + 0.03 (0.1 -> 0.0397, 0.25 -> 0.1239,
    all -> 0.4244, each repeated exactly over two runs); fp16 meets the 0.1 bar."""
    from oracle.ops import clip_boxes, non_max_suppression
    from ydbl.utils.synthetic import blob_images

    p, o = _models("yolov13s_DBL.yaml", 3, golden_dir)
    x = blob_images(16, 640, seed=1234)
    with torch.no_grad():
        y, _ = o(x)
    gt_conf = 0.0171
    labels = []
    for g in non_max_suppression(y, gt_conf, 0.7):
        clip_boxes(g[:, :4], (640, 640))
        labels.append(torch.cat([g[:, 5:6], g[:, :4]], 1))
    assert sum(len(lb) for lb in labels) > 100
    batch = {"img": x, "cls": torch.cat([lb[:, 0] for lb in labels]),
             "bboxes": torch.cat([lb[:, 1:] for lb in labels]),
             "batch_idx": torch.cat([torch.full((len(lb),), i) for i, lb in enumerate(labels)])}
    fp8 = {"fp16": False, "fp8": True, "fp8-0.25": 0.25, "fp8-0.1": 0.1}[mode]
    cal = golden_dir / "fp8_calib_yolov13s_DBL_nc3.json"
    m_gpu = p.val(data=[batch], half=True, fp8=fp8, conf=0.001, fp8_calibration=str(cal) if fp8 else None).box.map50
    m_cpu = _cpu_map50(o, x, labels, conf=0.001)
    frac = None
    if fp8 is not False:
        frac = [s.fp8_mac_fraction for s in p._sessions.values() if s.fp8][-1]
    print(f"DBL-s 640 {mode}: mAP50 gpu {m_gpu:.4f}  cpu {m_cpu:.4f}  drop {m_cpu - m_gpu:+.4f} "
          f"({sum(len(lb) for lb in labels)} pseudo-GT boxes on 16 images, fp8 MAC fraction {frac})")
    assert m_cpu > 0.5
    if fp8 is False:
        assert m_cpu - m_gpu <= 0.1
    else:  # e4m3 operands: the drop is reported (BASELINE config 5), bounded by the recorded drop + 0.03
        from ydbl.quant import Fp8Calibration

        c = Fp8Calibration.load(cal)
        if fp8 is not True:
            assert [s.fp8_mac_fraction for s in p._sessions.values() if s.fp8][-1] == pytest.approx(
                c.mac_fraction(c.switched(fp8)), abs=1e-6)
        measured = {"fp8": 0.4244, "fp8-0.25": 0.1239, "fp8-0.1": 0.0397}[mode]
        assert m_cpu - m_gpu <= measured + 0.03


@pytest.mark.parametrize("groups", ["1", "0"])
def test_nms_paths_agree_on_model_candidates(golden_dir, monkeypatch, groups):
    """The pair-matrix NMS path (images with <= 1024 candidates) against sort + chunked sweep on the
    candidates the DBL-n model itself decodes at the bench protocol (640, conf .25, iou .7): identical
    det / count, with the class split on and off."""
    from ydbl import _lib
    from ydbl._lib import NmsDesc
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    B = 32  # the bench batch: its busiest image has 644 candidates (11 rank blocks, 267 kept)
    sess = p.session(B, 640, 640, half=True, conf=0.25, iou=0.7, max_det=300)
    sess(blob_images(B, 640, seed=1234).cuda())
    torch.cuda.synchronize()
    assert int(sess.cand_count.max()) > 300  # clusters large enough for several rank blocks
    cap = sess.cand_score.shape[1]
    ws = torch.zeros(int(_lib.lib.ydbl_nms_workspace(B, cap, 30000)), dtype=torch.uint8, device="cuda")  # zero-filled once (include/ydbl.h)
    outs = []
    for fast, per_image in (("1", 0), ("0", 0), ("1", 1)):  # per_image 1: the session's own schedule at conf .25
        monkeypatch.setenv("YDBL_NMS_FAST", fast)
        monkeypatch.setenv("YDBL_NMS_GROUPS", groups)
        out = torch.full((B, 300, 6), -1.0, device="cuda")
        cnt = torch.full((B,), -1, dtype=torch.int32, device="cuda")
        nd = NmsDesc(sess.cand_box.data_ptr(), sess.cand_score.data_ptr(), sess.cand_cls.data_ptr(),
                     sess.cand_idx.data_ptr(), sess.cand_count.data_ptr(), B, cap, 0.7, 300, 30000, 0, 7680.0,
                     640.0, 640.0, out.data_ptr(), cnt.data_ptr(), ws.data_ptr(), per_image=per_image)
        _lib.check(_lib.lib.ydbl_nms(nd, torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        outs.append((out, cnt))
    for o in outs[1:]:
        assert torch.equal(outs[0][1], o[1]) and torch.equal(outs[0][0], o[0])
    assert torch.equal(outs[0][1], sess.count) and torch.equal(outs[0][0], sess.det)


@pytest.mark.parametrize("half", [False, True])
def test_detection_model_forward(golden_dir, half):
    """§8(b): the reference caller AutoBackend.forward -> ``self.model(im)`` (U/nn/autobackend.py:503-528) gets
    DetectionModel.forward's inference return ``(y, feats)`` (U/nn/tasks.py:109-172, head.py:108-118) from
    ``YOLO(cfg).model(x)``: y [B, 4+nc, A] and the per-level maps [B, 64+nc, H, W], checked against the oracle's
    (y, feats) under the fp32 / fp16 rule (parity_util); fresh tensors per call; CPU input refused."""
    import copy

    from parity_util import err_stats, fp16_rule, fp32_rule, oracle_legs
    from ydbl.utils.synthetic import blob_images

    p, o = _models("yolov13n_DBL.yaml", 3, golden_dir)
    x = blob_images(2, 160, seed=5)
    legs = ("fp64", "fp16") if half else ("fp64", "fp32")
    ys, _ = oracle_legs(o, x, legs)
    y64 = ys["fp64"]
    with torch.no_grad():
        _, f64 = copy.deepcopy(o).double()(x.double())
        _, fleg = (copy.deepcopy(o).half()(x.half()) if half else o(x))
    xin = x.cuda().half() if half else x.cuda()
    y, feats = p.model(xin)
    assert y.dtype == xin.dtype and y.device == xin.device and tuple(y.shape) == tuple(y64.shape)
    assert len(feats) == 3
    leg = ys[legs[1]]
    st, st_ref = err_stats(y.float().cpu(), y64), err_stats(leg, y64)
    tb, tc = (fp16_rule if half else fp32_rule)(st_ref)
    print(f"forward {'fp16' if half else 'fp32'}: |y - fp64| box {st['box_max']:.3g} px (oracle leg "
          f"{st_ref['box_max']:.3g}), score {st['conf_max']:.3g} ({st_ref['conf_max']:.3g}); |y - oracle leg| box "
          f"{(y.float().cpu() - leg).abs()[:, :4].max().item():.3g} px")
    key = "box_p999" if half else "box_max"
    assert st[key] <= tb and st["conf_p999" if half else "conf_max"] <= tc, (st, st_ref)
    for f, a64, al in zip(feats, f64, fleg):
        assert f.shape == a64.shape and f.dtype == xin.dtype and f.is_contiguous()
        dev_ref = (al.double() - a64).abs().max().item()
        dev = (f.double().cpu() - a64).abs().max().item()
        assert dev <= 2 * dev_ref + (2e-2 if half else 1e-3), (dev, dev_ref)
    y2, feats2 = p.model(xin)
    assert y2.data_ptr() != y.data_ptr() and torch.equal(y2, y) and all(torch.equal(a, b) for a, b in zip(feats, feats2))
    with pytest.raises(RuntimeError):
        p.model(x)


def test_sharded_predictor_nccl_world1(golden_dir, tmp_path):
    """The batch-sharded path with its one collective on RCCL: a world-size-1 "nccl" process group (FileStore), a
    ShardedPredictor over DBL-n bs4 at 640 whose NMS writes the [det | count] records and whose all_gather_into_tensor
    runs on RCCL.  The batch holds the e2e fixture's reference images in both sub-batch graphs
    (parity_util.batch_images); the gathered global detections are bit-equal to the plain session's AND, on the
    reference images, agree with the oracle's fp64 answer under the fp16 rule of tests/test_gpu_e2e.py
    (U/engine/trainer.py:222-227 is the reference's process-group setup)."""
    import torch.distributed as dist

    from parity_util import batch_images, detections, err_stats, fp16_rule, load_e2e, match_detections
    from ydbl.parallel import ShardedPredictor
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    y64_all, meta = load_e2e(golden_dir, "n640")
    idx = batch_images(meta, 4, 2)
    pos = [k for k, i in enumerate(idx) if i in meta["ref_images"]]
    assert pos[0] < 2 <= pos[-1]  # reference images in both sub-batch graphs
    y64 = y64_all[[meta["ref_images"].index(idx[k]) for k in pos]]
    conf, iou = meta["conf"], meta["iou"]
    x = blob_images(meta["batch_full"], 640, seed=meta["seed"])[idx].cuda()
    refs = {}
    for streams in (1, 2):  # the plain session of the same layout (one bs4 graph / two bs2 graphs)
        plain = p.session(4, 640, 640, half=True, conf=conf, iou=iou, streams=streams)
        refs[streams] = tuple(t.clone() for t in plain(x))
    o16 = meta["oracle_fp16"]
    tb, tc = fp16_rule(o16)
    ref_dets = detections(y64, conf, iou, (640, 640))
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", rank=0, world_size=1, store=store)
    try:
        for streams in (1, 2):
            sp = ShardedPredictor(p, 4, 640, 640, torch.device("cuda", 0), half=True, conf=conf, iou=iou,
                                  streams=streams, keep_pred=True)
            det, cnt = sp(images_global=x)
            torch.cuda.synchronize()
            det_ref, cnt_ref = refs[streams]
            assert sp.distributed and det.shape == (4, 300, 6) and cnt.dtype == torch.int32
            assert torch.equal(cnt.cpu(), cnt_ref.cpu()) and int(cnt.sum()) > 0
            assert torch.equal(det.cpu(), det_ref.cpu())
            assert det.data_ptr() == sp.gathered.data_ptr()  # views of the gathered buffer, no copy
            # against the oracle: decoded predictions and the gathered final detections on the reference images
            st = err_stats(sp.session.pred.cpu()[pos], y64)
            for k in ("box_max", "box_p999", "conf_max", "conf_p999"):
                assert st[k] <= 2 * o16[k] + (1e-2 if k.startswith("box") else 1e-4), (k, st, o16)
            got = [det[k, : int(cnt[k])].cpu() for k in pos]
            m = match_detections(ref_dets, got, y64, conf, iou, tb, tc)
            print(f"sharded nccl world 1, streams {streams}: images {[idx[k] for k in pos]} at {pos}: {m['pairs']} "
                  f"pairs, {m['borderline']} borderline, {len(m['mismatches'])} mismatches vs the oracle's fp64")
            assert m["pairs"] > 0 and len(m["mismatches"]) <= 2 * o16["det_mismatches"] + 2, m["mismatches"][:5]
    finally:
        dist.destroy_process_group()


def test_fp8_calibration_reads_inputs_at_launch(golden_dir):
    """ydbl.quant.calibrate takes each conv's statistics right before its launch: HyperACE's merged branch 1x1
    (C3AHx2.cv1|cv2) reads y1, whose slice branch1.cv3 overwrites later in the plan, so the scale and the bias
    correction must come from y1 as that conv reads it, not from the buffer after the plan ran."""
    from ydbl import quant
    from ydbl.utils.synthetic import blob_images

    p, _ = _models("yolov13n_DBL.yaml", 3, golden_dir)
    s = p.session(2, 256, 256, half=True, keep_pred=True, use_graph=False)
    s.load(blob_images(2, 256, seed=4321).cuda())
    plan = s.plan
    keys = quant.candidate_keys(plan)
    steps = quant._candidate_steps(plan)
    k_step, ci = next((k, c) for k, c in steps.items() if plan.steps[k].what == "C3AHx2.cv1|cv2")
    got = {}

    def grab(k):
        if k == k_step:
            got["x"] = plan.fp8_candidates[ci][1].torch().float().clone()

    plan.run_observed(grab)
    torch.cuda.synchronize()
    x_at_launch = got["x"]
    x_after = plan.fp8_candidates[ci][1].torch().float()
    assert not torch.equal(x_at_launch, x_after)  # the hazard is real: the buffer is rewritten after the launch
    cal = quant.calibrate([plan], plan.run, rank=False)
    qs = quant.E4M3_MAX / x_at_launch.abs().amax().item()
    assert abs(cal.qs[keys[ci]] - qs) <= 1e-6 * qs
    d0, _, w32 = plan.fp8_candidates[ci]
    wq, sw = quant.quantize_weights_e4m3(w32)
    ref = quant.bias_delta([x_at_launch], cal.qs[keys[ci]], w32, wq, sw, d0.kh * d0.kw)
    assert torch.allclose(torch.tensor(cal.delta[keys[ci]]), ref, rtol=1e-4, atol=1e-6)
