"""Reference-format .pt checkpoints (U/engine/trainer.py:513-546) read without unpickling code.

No reference checkpoint ships with the reference tree, so the fixture is written here: our own
DetectionModel pickled under the reference's class paths (ultralytics.nn.tasks.DetectionModel,
ultralytics.nn.modules.*) inside the trainer's checkpoint dict, fp16 like the saved EMA.
"""

import sys
import types
from datetime import datetime

import pytest
import torch


def _save_reference_style(model, path):
    import ydbl

    fake = {}
    for name in ["ultralytics", "ultralytics.nn", "ultralytics.nn.modules", "ultralytics.nn.modules.block",
                 "ultralytics.nn.tasks"]:
        fake[name] = types.ModuleType(name)
    saved = {}
    for m in model.modules():
        cls = type(m)
        if cls.__module__.startswith("ydbl") and cls not in saved:
            saved[cls] = cls.__module__
            target = "ultralytics.nn.tasks" if cls.__name__ == "DetectionModel" else "ultralytics.nn.modules.block"
            cls.__module__ = target
            setattr(fake[target], cls.__qualname__, cls)
    old = {k: sys.modules.get(k) for k in fake}
    sys.modules.update(fake)
    try:
        ckpt = {"date": datetime.now().isoformat(), "version": "8.3.0", "epoch": -1, "best_fitness": None,
                "model": None, "ema": model.half(), "updates": 100, "optimizer": None,
                "train_args": {"imgsz": 640, "batch": 16, "model": "yolov13n_DBL.yaml"}, "train_metrics": {},
                "train_results": {}}
        torch.save(ckpt, path)
    finally:
        for cls, mod in saved.items():
            cls.__module__ = mod
        for k, v in old.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    model.float()
    assert "ydbl" in ydbl.__name__


def test_reference_checkpoint_roundtrip(tmp_path):
    from ydbl import YOLO
    from ydbl.utils.checkpoint import read_reference_checkpoint

    m = YOLO("yolov13n_DBL.yaml", nc=3)
    torch.manual_seed(0)
    with torch.no_grad():
        for p in m.model.parameters():
            p.copy_(torch.randn_like(p) * 0.1)
    m.model.names = {0: "car", 1: "person", 2: "bike"}
    ref_sd = {k: v.clone() for k, v in m.model.state_dict().items()}
    path = tmp_path / "best.pt"
    _save_reference_style(m.model, path)
    # a plain weights_only load refuses it: the file names the reference's classes
    with pytest.raises(Exception):
        torch.load(path, weights_only=True)
    ck = read_reference_checkpoint(path)
    assert ck["names"] == {0: "car", 1: "person", 2: "bike"}
    assert ck["yaml"]["nc"] == 3 and ck["train_args"]["imgsz"] == 640
    assert set(ck["state_dict"]) == set(ref_sd)
    for k, v in ref_sd.items():
        got = ck["state_dict"][k]
        if v.is_floating_point():
            assert got.dtype == torch.float32
            assert torch.equal(got, v.half().float()), k  # the EMA is saved in fp16
        else:
            assert torch.equal(got, v), k
    # YOLO('best.pt') builds from the embedded yaml and loads the weights
    m2 = YOLO(path)
    assert m2.names == {0: "car", 1: "person", 2: "bike"}
    sd2 = m2.model.state_dict()
    for k, v in ck["state_dict"].items():
        assert torch.equal(sd2[k].float(), v), k


def test_checkpoint_refuses_foreign_globals(tmp_path):
    from ydbl.utils.checkpoint import read_reference_checkpoint

    class Payload:
        def __reduce__(self):
            import os
            return (os.getcwd, ())

    path = tmp_path / "evil.pt"
    torch.save({"ema": Payload()}, path)
    with pytest.raises(RuntimeError, match="outside the allowed"):
        read_reference_checkpoint(path)


def test_partial_state_dict_is_refused():
    """A dict that covers only part of the model must not load silently (layers would stay at random
    init); BN's num_batches_tracked counters may be absent (they carry no weight)."""
    from ydbl import YOLO

    m = YOLO("yolov13n_DBL.yaml", nc=3)
    sd = m.model.state_dict()
    partial = {k: v for i, (k, v) in enumerate(sd.items()) if i % 7}
    with pytest.raises(KeyError, match="missing"):
        YOLO("yolov13n_DBL.yaml", nc=3).load(partial)
    no_counters = {k: v for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    YOLO("yolov13n_DBL.yaml", nc=3).load(no_counters)
    with pytest.raises(KeyError, match="unexpected"):
        YOLO("yolov13n_DBL.yaml", nc=3).load({**sd, "model.99.bogus": torch.zeros(1)})
