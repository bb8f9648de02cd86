"""fp8 mixed-precision selection (ydbl.quant): MAC accounting and the MAC-budget pick, host logic only."""

from types import SimpleNamespace as NS

import pytest
import torch

from ydbl.quant import candidate_macs, select_by_mac_budget


def _cand(cin, cout, k, s, h, w, n=2):
    """(desc, input view, fp32 [Cout][KPAD] weights) as Plan.fp8_candidates holds them."""
    ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
    kpad = (k * k * cin + 31) // 32 * 32
    d = NS(kh=k, kw=k, y=NS(n=n, h=ho, w=wo, c=cout))
    return d, NS(n=n, h=h, w=w, c=cin), torch.zeros(cout, kpad)


def test_candidate_macs_use_output_pixels_and_real_k():
    c1 = _cand(64, 64, 3, 2, 80, 80)  # the stride-2 downsample: 40x40 outputs
    assert candidate_macs(c1) == 64 * 9 * 64 * 2 * 40 * 40
    c2 = _cand(72, 16, 1, 1, 40, 40)  # K = 72 (KPAD 96 is padding, not MACs)
    assert candidate_macs(c2) == 16 * 72 * 2 * 40 * 40


def test_selected_fraction_with_a_stride2_candidate():
    """One stride-2 candidate among stride-1 ones: the switched share of MACs is computed on output pixels, so
    `fraction` of the real MACs is switched (input-pixel counting would have priced the s2 conv 4x)."""
    cands = [_cand(64, 64, 3, 2, 80, 80), _cand(128, 128, 1, 1, 40, 40), _cand(64, 64, 1, 1, 40, 40)]
    macs = [candidate_macs(c) for c in cands]  # 118.0M, 52.4M, 13.1M
    total = sum(macs)
    # least sensitive first: the s2 conv (64 % of the MACs) fits a 0.7 budget alone; counted on its input
    # pixels (472M of 537M) it would not, and the two 1x1s would be switched instead
    chosen, frac = select_by_mac_budget([0.1, 0.9, 0.2], macs, 0.7)
    assert chosen == [0] and abs(frac - macs[0] / total) < 1e-12 and frac <= 0.7
    chosen, frac = select_by_mac_budget([0.1, 0.9, 0.2], macs, 0.5)  # s2 too big: skipped, the rest fit
    assert chosen == [1, 2] and frac <= 0.5
    chosen, frac = select_by_mac_budget([0.1, 0.9, 0.2], macs, 1.0)
    assert chosen == [0, 1, 2] and frac == 1.0
    chosen, frac = select_by_mac_budget([0.1, 0.9, 0.2], macs, 0.0)
    assert chosen == [] and frac == 0.0


@pytest.mark.parametrize("cv3_fuse", ["", "1"])
def test_candidate_keys_stable_across_layouts(cv3_fuse, monkeypatch):
    """ydbl.quant.candidate_keys names a model's fp8 candidates the same way at every batch / sub-batch size, so one
    committed calibration (tests/golden/fp8_calib_*.json) means one layer set for every layout the model runs."""
    from ydbl import YOLO
    from ydbl.quant import candidate_keys

    monkeypatch.setenv("YDBL_CV3_FUSE", cv3_fuse or "0")
    m = YOLO("yolov13s_DBL.yaml", nc=3).model
    keys = {}
    for b in (1, 4, 16, 32):
        plan = m.compile(b, 640, 640, torch.float16, device="meta").plan
        k = candidate_keys(plan)
        assert len(k) == len(set(k)) == len(plan.fp8_candidates) > 0
        assert all(int(key[1:].split(".")[0]) >= 0 for key in k)  # every candidate knows its layer
        keys[b] = k
    assert keys[16] == keys[32]
    if cv3_fuse:
        # small maps fold DSC3k's 128-channel cv3 into the lean DSConv launch (no longer a candidate): the others
        # keep their names
        assert set(keys[1]) == set(keys[4]) < set(keys[32])
    else:  # the default since round 6: cv3 is its own launch (a candidate) at every size
        assert set(keys[1]) == set(keys[4]) == set(keys[32])


def test_calibration_roundtrip_and_shares(tmp_path):
    from ydbl.quant import Fp8Calibration

    cal = Fp8Calibration({"a": 1.0, "b": 2.0, "c": 3.0}, {"a": [0.0], "b": [0.1], "c": [0.2]},
                         sens={"a": 0.3, "b": 0.1, "c": 0.2}, macs={"a": 10, "b": 60, "c": 30}, meta={"x": 1})
    path = cal.save(tmp_path / "cal.json")
    back = Fp8Calibration.load(path)
    assert back.to_json() == cal.to_json()
    assert back.switched(1.0) == ["a", "b", "c"]
    assert back.switched(0.3) == ["c"]  # b (least sensitive) is 60 % of the MACs: skipped, c fits
    assert back.switched(0.95) == ["b", "c"] and abs(back.mac_fraction(["b", "c"]) - 0.9) < 1e-12
    cal.sets = {"0.25": ["a"]}  # an explicit set recorded for a share wins over the ranking's budget pick
    back = Fp8Calibration.load(cal.save(tmp_path / "cal2.json"))
    assert back.switched(0.25) == ["a"] and back.switched(0.3) == ["c"]
