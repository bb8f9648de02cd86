"""The C-ABI library loads, exports every symbol include/ydbl.h declares, and its
descriptor layouts match the ctypes mirror (checked against gcc's sizeof/offsetof).
No GPU: only argument validation paths are called."""

import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "ydbl.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ydbl_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from ydbl import _lib

    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(_lib.lib, n), f"{n} declared in include/ydbl.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(names)
    assert "gfx950" in _lib.version()


STRUCTS = {
    "ydbl_view": "View",
    "ydbl_conv_desc": "ConvDesc",
    "ydbl_dwconv_desc": "DwConvDesc",
    "ydbl_dsconv_desc": "DsConvDesc",
    "ydbl_hg_desc": "HgDesc",
    "ydbl_decode_desc": "DecodeDesc",
    "ydbl_pred_cand_desc": "PredCandDesc",
    "ydbl_nms_desc": "NmsDesc",
    "ydbl_match_desc": "MatchDesc",
    "ydbl_letterbox_desc": "LetterboxDesc",
    "ydbl_stem2_desc": "Stem2Desc",
    "ydbl_input_bind": "InputBind",
    "ydbl_bottleneck_desc": "BottleneckDesc",
    "ydbl_dysample_desc": "DySampleDesc",
    "ydbl_dysample2_desc": "DySample2Desc",
    "ydbl_lsk_desc": "LskDesc",
}


def test_struct_layout_matches_c(tmp_path):
    from ydbl import _lib

    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, pyname in STRUCTS.items():
        lines.append(f'printf("{pyname} %zu\\n", sizeof({cname}));')
        for fname, _ in getattr(_lib, pyname)._fields_:
            lines.append(f'printf("{pyname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(line.split() for line in out if line.strip())
    for cname, pyname in STRUCTS.items():
        st = getattr(_lib, pyname)
        assert int(got[pyname]) == C.sizeof(st), pyname
        for fname, _ in st._fields_:
            assert int(got[f"{pyname}.{fname}"]) == getattr(st, fname).offset, f"{pyname}.{fname}"


def test_validation_errors_without_gpu():
    from ydbl import _lib

    lib = _lib.lib
    assert lib.ydbl_conv2d_nhwc(None, None) == 1
    assert "null descriptor" in lib.ydbl_last_error().decode()
    d = _lib.ConvDesc()
    d.x = _lib.View(16, 1, 8, 8, 3, 8, _lib.F16)  # c=3 not a multiple of 8
    d.y = _lib.View(16, 1, 8, 8, 8, 8, _lib.F16)
    assert lib.ydbl_conv2d_nhwc(d, None) == 1
    assert "16-byte" in lib.ydbl_last_error().decode() or "multiple of 8" in lib.ydbl_last_error().decode()
    nd = _lib.NmsDesc()
    assert lib.ydbl_nms(nd, None) == 1
    with pytest.raises(_lib.YdblError):
        _lib.check(lib.ydbl_nms(nd, None), "ydbl_nms")
    md = _lib.MatchDesc()
    assert lib.ydbl_match_predictions(md, None) == 1
    assert "null buffer" in lib.ydbl_last_error().decode()
    assert lib.ydbl_letterbox(_lib.LetterboxDesc(), None) == 1
    assert lib.ydbl_match_workspace(2, 300, 10, 10) == 4 * (100 + 1200) + 16


def test_workspace_queries():
    from ydbl import _lib

    # global sort scratch (cap > 8192: next pow2 x (8 B key + 4 B slot)) + class-group keep lists
    # (8 groups x min(cap, 4096) x (8 B key + 4 B slot) + a 4 B count each) + 8 + pair-matrix rows: min(cap, 8192)
    # rounded to 64 per image, each an 8 B rank accumulator, a 4 B order entry and a rows / 8 B IoU row, + 16
    assert _lib.lib.ydbl_nms_workspace(2, 8400, 30000) == (2 * 16384 * 12 + 2 * 8 * (4096 * 12 + 4) + 8
                                                           + 2 * 8192 * (12 + 1024) + 16)
    assert _lib.lib.ydbl_nms_workspace(3, 100, 30000) == 3 * 8 * (100 * 12 + 4) + 8 + 3 * 128 * (12 + 16) + 16
    assert _lib.lib.ydbl_lsk_gate_workspace(2, 20, 20) == 2 * 400 * 2 * 4
    assert _lib.lib.ydbl_hg_workspace(1, 1600, 64, 4) > 0
