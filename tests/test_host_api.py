"""Host-side API logic that needs no GPU: session layout policy, compiled-plan cache keys, the parity tests'
batch composition."""

import torch

from parity_util import batch_images


def test_default_streams():
    from ydbl.engine.session import SPLIT_MIN_BATCH, default_streams

    assert [default_streams(b) for b in (1, 2, 3)] == [1, 1, 1]
    assert all(default_streams(b) == 2 for b in (SPLIT_MIN_BATCH, 8, 32, 64))


def test_weights_signature_tracks_edits():
    """A compiled plan folds the weights at build time; the signature its caches compare must move on an in-place
    edit (tracked op), on a replaced parameter and on load_state_dict, and stay put otherwise."""
    from ydbl import YOLO
    from ydbl.nn.tasks import weights_signature

    m = YOLO("yolov13n_DBL.yaml", nc=3).model
    s0 = weights_signature(m)
    assert weights_signature(m) == s0
    with torch.no_grad():
        m.model[0].conv.weight.mul_(1.0)
    s1 = weights_signature(m)
    assert s1 != s0
    m.model[0].conv.weight = torch.nn.Parameter(m.model[0].conv.weight.detach().clone())
    s2 = weights_signature(m)
    assert s2 != s1
    m.load_state_dict(m.state_dict())
    assert weights_signature(m) != s2
    torch.nn.Conv2d(3, 3, 1)  # an unrelated module's registrations rebuild the tensor list, not the signature
    s3 = weights_signature(m)
    assert weights_signature(m) == s3


def test_batch_images_spreads_reference_images():
    meta = {"batch_full": 32, "ref_images": [0, 1, 15, 16, 31]}
    assert batch_images(meta, 32, 2) == list(range(32))
    idx = batch_images(meta, 8, 2)  # config 3's per-GPU layout: two bs4 sub-batch graphs
    assert sorted(idx) == sorted(set(idx)) and len(idx) == 8
    # graph 1 holds images 0 and 1 (first and last position), graph 2 images 15, 16, 31 (31 in the last position)
    assert idx == [0, 2, 3, 1, 15, 16, 4, 31]
    assert batch_images(meta, 4, 2) == [0, 1, 15, 16]
    assert batch_images(meta, 2, 1) == [0, 1]
    assert batch_images({"batch_full": 8, "ref_images": [0, 7]}, 8, 2) == list(range(8))
    assert batch_images({"batch_full": 8, "ref_images": [0, 1]}, 8, 2)[4] == 1  # x640 bs8: image 1 in graph 2


def test_branch_plans_must_be_single_stream():
    """BranchGraphRunner's guard (runtime.Plan.check_single_stream): C-ABI launches and flagged steps pass, any
    other callable is refused before capture (a nested stream fork inside a captured branch segfaults on ROCm)."""
    import pytest

    from ydbl import _lib
    from ydbl.runtime import Plan

    p = Plan(torch.device("cpu"), torch.float16)
    p.launch("ydbl_detect_decode", None, what="decode")
    p.check_single_stream()

    def ok(stream):
        return 0

    ok.single_stream = True
    p.steps.append(type(p.steps[0])(ok, (), "flagged"))
    p.check_single_stream()
    p.steps.append(type(p.steps[0])(lambda stream: 0, (), "unflagged"))
    with pytest.raises(RuntimeError, match="unflagged"):
        p.check_single_stream()
    assert _lib.lib.ydbl_detect_decode is p.steps[0].fn


def test_switch_list_matches_sources():
    """runtime.SWITCHES (the compiled-plan cache keys) names every YDBL_* environment switch the product reads."""
    import re
    from pathlib import Path

    from ydbl.runtime import SWITCHES

    root = Path(__file__).resolve().parents[1] / "yolo-dbl_amd"
    read = set()
    for f in [*root.glob("ydbl/**/*.py"), *root.glob("csrc/*.hip"), *root.glob("csrc/*.hpp")]:
        t = f.read_text()
        read |= set(re.findall(r'getenv\("(YDBL_[A-Z0-9_]+)"\)', t))
        read |= set(re.findall(r'environ\.get\("(YDBL_[A-Z0-9_]+)"', t))
        read |= set(re.findall(r'os\.environ\["(YDBL_[A-Z0-9_]+)"\]', t))
    read -= {"YDBL_OFFLOAD_ARCH", "YDBL_LIB"}  # build / loader settings, not plan routing
    assert read == set(SWITCHES), (read ^ set(SWITCHES))
