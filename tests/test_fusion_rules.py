"""Host-side fusion rules of the plan builder (no GPU): which DSC3k blocks take the leading / trailing GEMMs.

C3._cv1_fusable must agree with the lean DSConv kernel's g0 instance (csrc/dsc_lean.hip: fp16, c_ = x.c = 64,
k3 stride 1) and C3._cv3_fusable with its g2 instances (k7, c_ 64 or 128 on small maps); a mismatch would make
ydbl_dsconv_nhwc refuse the descriptor at plan build time on the GPU.
"""
from types import SimpleNamespace as NS

import torch

from ydbl.nn import modules as M


def _x(n, c, h=40, w=40, cs=None):
    return NS(n=n, c=c, h=h, w=w, cs=cs if cs is not None else c)


def test_cv1_cv3_fusions_off_by_default(monkeypatch):
    """Round 6: the leading / trailing 1x1 fusions are opt-in (YDBL_CV1_FUSE / YDBL_CV3_FUSE = 1): the separate
    launches measured faster in the benched two-branch layout (profiles/r06/r06_fusion_switch_sweep.txt)."""
    monkeypatch.delenv("YDBL_CV1_FUSE", raising=False)
    monkeypatch.delenv("YDBL_CV3_FUSE", raising=False)
    monkeypatch.delenv("YDBL_DS_LEAN", raising=False)
    m = M.DSC3k(64, 64, 2, True, e=1.0, k1=3, k2=7)
    plan = NS(dtype=torch.float16)
    assert not m._cv1_fusable(plan, _x(16, 64)) and not m._cv3_fusable(plan, _x(16, 64))


def test_dwpw_fused_default_at_64_outputs(monkeypatch):
    """The Detect DWConv -> Conv1x1 pairs run as one launch at 64 pointwise outputs (DBL-n) and as two at 128+
    (DBL-s / DBL-l), unless YDBL_DWPW forces either (profiles/r06/r06_detect_switch_sweep.txt)."""
    monkeypatch.delenv("YDBL_DWPW", raising=False)
    assert M.dwpw_fuse(64) and not M.dwpw_fuse(128)
    monkeypatch.setenv("YDBL_DWPW", "1")
    assert M.dwpw_fuse(128)
    monkeypatch.setenv("YDBL_DWPW", "0")
    assert not M.dwpw_fuse(64)


def test_cv1_fusable_dbl_n_shape(monkeypatch):
    monkeypatch.setenv("YDBL_CV1_FUSE", "1")
    monkeypatch.setenv("YDBL_CV3_FUSE", "1")
    monkeypatch.delenv("YDBL_DS_LEAN", raising=False)
    m = M.DSC3k(64, 64, 2, True, e=1.0, k1=3, k2=7)
    plan = NS(dtype=torch.float16)
    assert m._cv1_fusable(plan, _x(16, 64))
    assert m._cv3_fusable(plan, _x(16, 64))
    assert not m._cv1_fusable(NS(dtype=torch.float32), _x(16, 64))  # fp16 only
    assert not m._cv1_fusable(plan, _x(16, 64, cs=68))  # 16-byte pixel vectors
    monkeypatch.setenv("YDBL_DS_LEAN", "0")  # the chunked kernel has neither the leading nor the trailing GEMM
    assert not m._cv1_fusable(plan, _x(16, 64))
    assert not m._cv3_fusable(plan, _x(16, 64))
    monkeypatch.delenv("YDBL_DS_LEAN")
    monkeypatch.setenv("YDBL_CV1_FUSE", "0")
    assert not m._cv1_fusable(plan, _x(16, 64))


def test_cv1_fusable_only_at_64_channels_and_k3(monkeypatch):
    monkeypatch.setenv("YDBL_CV1_FUSE", "1")
    monkeypatch.delenv("YDBL_DS_LEAN", raising=False)
    plan = NS(dtype=torch.float16)
    assert not M.DSC3k(128, 128, 2, True, e=1.0, k1=3, k2=7)._cv1_fusable(plan, _x(16, 128, 20, 20))
    assert not M.DSC3k(64, 64, 2, True, e=1.0, k1=5, k2=7)._cv1_fusable(plan, _x(16, 64))
    # plain C3 (Bottleneck m) never takes it
    assert not M.C3(64, 64, 1)._cv1_fusable(plan, _x(16, 64))


def test_cv3_fusable_small_map_rule_for_128_channels(monkeypatch):
    monkeypatch.setenv("YDBL_CV3_FUSE", "1")
    monkeypatch.delenv("YDBL_DS_LEAN", raising=False)
    plan = NS(dtype=torch.float16)
    m = M.DSC3k(128, 128, 2, True, e=1.0, k1=3, k2=7)
    assert m._cv3_fusable(plan, _x(16, 128, 20, 20))      # 16 * 3 * 3 = 144 8x8 tiles <= 160
    assert not m._cv3_fusable(plan, _x(64, 128, 40, 40))  # DBL-s bs64: 1600 tiles -> chunked kernel
