"""ctypes binding of libydbl.so (the C ABI in include/ydbl.h).

There is no fallback: if the library is missing or cannot be loaded the
import raises, so a GPU run can never silently go through another path.
torch is imported first so that libydbl resolves ``libamdhip64.so.7`` to the
HIP runtime torch already loaded (one runtime, one set of streams).
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the dlopen below)

LIB_PATH = Path(os.environ.get("YDBL_LIB", Path(__file__).resolve().parent / "libydbl.so"))

F32, F16 = 0, 1
ACT_NONE, ACT_SILU, ACT_GELU, ACT_SIGMOID = 0, 1, 2, 3
RES_NONE, RES_ADD, RES_MUL = 0, 1, 2


class View(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("n", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("c", C.c_int32),
                ("cs", C.c_int32), ("dtype", C.c_int32)]


class ConvDesc(C.Structure):
    _fields_ = [("x", View), ("y", View), ("r", View), ("w", C.c_void_p), ("bias", C.c_void_p),
                ("kh", C.c_int32), ("kw", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32), ("dil", C.c_int32),
                ("kpad", C.c_int32), ("act", C.c_int32), ("res_mode", C.c_int32),
                ("y2", View), ("r2", View), ("a2", C.c_float), ("b2", C.c_float),
                ("dq", C.c_void_p), ("qscale", C.c_float), ("workspace", C.c_void_p), ("workspace_bytes", C.c_int64)]


class DwConvDesc(C.Structure):
    _fields_ = [("x", View), ("y", View), ("r", View), ("w", C.c_void_p), ("bias", C.c_void_p),
                ("kh", C.c_int32), ("kw", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32), ("dil", C.c_int32),
                ("act", C.c_int32), ("res_mode", C.c_int32)]


class DsConvDesc(C.Structure):
    _fields_ = [("x", View), ("y", View), ("r", View), ("dw_w", C.c_void_p), ("pw_w", C.c_void_p),
                ("bias", C.c_void_p), ("k", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32),
                ("dil", C.c_int32), ("kpad", C.c_int32), ("act", C.c_int32), ("res_mode", C.c_int32),
                ("dw_bias", C.c_void_p), ("dw_act", C.c_int32), ("tail_w", C.c_void_p), ("tail_b", C.c_void_p),
                ("tail_y", View), ("tail_n", C.c_int32), ("g2_w", C.c_void_p), ("g2_b", C.c_void_p),
                ("g2_x", View), ("g2_y", View), ("g2_act", C.c_int32), ("g0_w", C.c_void_p), ("g0_b", C.c_void_p),
                ("g0_x", View), ("g0_y", View), ("g0_act", C.c_int32)]


class HgDesc(C.Structure):
    _fields_ = [("x", View), ("xp", View), ("y", View), ("num_edges", C.c_int32), ("num_heads", C.c_int32),
                ("proto_base", C.c_void_p), ("ctx_w", C.c_void_p), ("ctx_b", C.c_void_p),
                ("edge_w", C.c_void_p), ("edge_b", C.c_void_p), ("node_w", C.c_void_p), ("node_b", C.c_void_p),
                ("workspace", C.c_void_p), ("pre_w", C.c_void_p), ("pre_b", C.c_void_p)]


class DecodeDesc(C.Structure):
    _fields_ = [("box", View * 3), ("cls", View * 3), ("nl", C.c_int32), ("nc", C.c_int32),
                ("stride", C.c_float * 3), ("conf_thres", C.c_float), ("multi_label", C.c_int32),
                ("classes", C.c_void_p), ("nclasses", C.c_int32), ("y_ref", C.c_void_p),
                ("cand_box", C.c_void_p), ("cand_score", C.c_void_p), ("cand_cls", C.c_void_p),
                ("cand_idx", C.c_void_p), ("cand_count", C.c_void_p), ("cap", C.c_int32)]


class PredCandDesc(C.Structure):
    _fields_ = [("pred", C.c_void_p), ("n", C.c_int32), ("nc", C.c_int32), ("A", C.c_int32),
                ("conf_thres", C.c_float), ("multi_label", C.c_int32), ("classes", C.c_void_p),
                ("nclasses", C.c_int32), ("cand_box", C.c_void_p), ("cand_score", C.c_void_p),
                ("cand_cls", C.c_void_p), ("cand_idx", C.c_void_p), ("cand_count", C.c_void_p), ("cap", C.c_int32)]


class NmsDesc(C.Structure):
    _fields_ = [("cand_box", C.c_void_p), ("cand_score", C.c_void_p), ("cand_cls", C.c_void_p),
                ("cand_idx", C.c_void_p), ("cand_count", C.c_void_p), ("n", C.c_int32), ("cap", C.c_int32),
                ("iou_thres", C.c_double), ("max_det", C.c_int32), ("max_nms", C.c_int32), ("agnostic", C.c_int32),
                ("max_wh", C.c_float), ("clip_w", C.c_float), ("clip_h", C.c_float), ("out", C.c_void_p),
                ("out_count", C.c_void_p), ("workspace", C.c_void_p), ("out_stride", C.c_int64),
                ("count_stride", C.c_int64), ("per_image", C.c_int32)]


class InputBind(C.Structure):
    """ydbl_input_bind: device word holding the batch pointer, device fp32 batch maximum (LoadTensor's /255 rule)."""
    _fields_ = [("x", C.c_void_p), ("amax", C.c_void_p)]


class Stem2Desc(C.Structure):
    _fields_ = [("x", C.c_void_p), ("n", C.c_int32), ("cin", C.c_int32), ("h", C.c_int32), ("w", C.c_int32),
                ("scale", C.c_float), ("c0", C.c_int32), ("params", C.c_void_p), ("y", View), ("bind", InputBind)]


class DySampleDesc(C.Structure):
    _fields_ = [("x", View), ("off", View), ("groups", C.c_int32), ("y", View), ("y2", View), ("r2", View),
                ("a2", C.c_float), ("b2", C.c_float)]


class DySample2Desc(C.Structure):
    _fields_ = [("x", View), ("off_w", C.c_void_p), ("off_b", C.c_void_p), ("groups", C.c_int32), ("y", View),
                ("y2", View), ("r2", View), ("a2", C.c_float), ("b2", C.c_float)]


class LskDesc(C.Structure):
    _fields_ = [("x", View), ("a1", View), ("a2", View), ("attn", View), ("y", View), ("w12", C.c_void_p),
                ("b12", C.c_void_p), ("sw", C.c_void_p), ("sb", C.c_void_p), ("w", C.c_void_p), ("b", C.c_void_p),
                ("agg", C.c_void_p)]


class BottleneckDesc(C.Structure):
    _fields_ = [("x", View), ("y", View), ("c", C.c_int32), ("add", C.c_int32), ("tile_h", C.c_int32),
                ("params", C.c_void_p), ("c_mid", C.c_int32), ("pw", C.c_int32)]


class LetterboxDesc(C.Structure):
    _fields_ = [("src", C.c_void_p), ("src_off", C.c_void_p), ("meta", C.c_void_p), ("n", C.c_int32),
                ("out_h", C.c_int32), ("out_w", C.c_int32), ("pad_value", C.c_float), ("out", C.c_void_p)]


class MatchDesc(C.Structure):
    _fields_ = [("det", C.c_void_p), ("det_count", C.c_void_p), ("n", C.c_int32), ("max_det", C.c_int32),
                ("gt_box", C.c_void_p), ("gt_cls", C.c_void_p), ("gt_ofs", C.c_void_p), ("n_gt", C.c_int32),
                ("iouv", C.c_void_p), ("n_iou", C.c_int32), ("single_cls", C.c_int32), ("correct", C.c_void_p),
                ("workspace", C.c_void_p)]


# name -> (argtypes, restype); every entry must exist in include/ydbl.h
_P = C.c_void_p
_VP = C.POINTER(View)
SIGNATURES = {
    "ydbl_conv2d_nhwc": ([C.POINTER(ConvDesc), _P], C.c_int),
    "ydbl_dwconv2d_nhwc": ([C.POINTER(DwConvDesc), _P], C.c_int),
    "ydbl_dwconv2d_pair_nhwc": ([C.POINTER(DwConvDesc), C.POINTER(DwConvDesc), _P], C.c_int),
    "ydbl_dsconv_nhwc": ([C.POINTER(DsConvDesc), _P], C.c_int),
    "ydbl_batch_max_work_ints": ([], C.c_int32),
    "ydbl_batch_max_work_init": ([_P], None),
    "ydbl_batch_max": ([_P, C.c_int64, _P, _P, _P, _P], C.c_int),
    "ydbl_batch_max_bound": ([_P, C.c_int64, _P, _P, _P, _P], C.c_int),
    "ydbl_input_nchw_to_nhwc": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_float, _VP,
                                 C.POINTER(InputBind), _P], C.c_int),
    "ydbl_conv_stem": ([_P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_float, _P, _P, C.c_int32, C.c_int32,
                        C.c_int32, _VP, C.POINTER(InputBind), _P], C.c_int),
    "ydbl_gate_add": ([_VP, _VP, C.c_float, _VP, _P], C.c_int),
    "ydbl_pool_up_concat": ([_VP, _VP, _VP, _VP, _P], C.c_int),
    "ydbl_dysample": ([_VP, _VP, C.c_int32, _VP, _P], C.c_int),
    "ydbl_dysample_ex": ([C.POINTER(DySampleDesc), _P], C.c_int),
    "ydbl_lsk_gate": ([_VP, _P, _P, _VP, _P, _P], C.c_int),
    "ydbl_lsk_gate_workspace": ([C.c_int32, C.c_int32, C.c_int32], C.c_int64),
    "ydbl_lsk_attn": ([C.POINTER(LskDesc), _P], C.c_int),
    "ydbl_lsk_out": ([C.POINTER(LskDesc), _P], C.c_int),
    "ydbl_hg_workspace": ([C.c_int32, C.c_int32, C.c_int32, C.c_int32], C.c_int64),
    "ydbl_hg_context": ([C.POINTER(HgDesc), _P], C.c_int),
    "ydbl_hg_propagate": ([C.POINTER(HgDesc), _P], C.c_int),
    "ydbl_hg_fused_workspace": ([C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32], C.c_int64),
    "ydbl_hg_fused": ([C.POINTER(HgDesc), _P], C.c_int),
    "ydbl_dysample2": ([C.POINTER(DySample2Desc), _P], C.c_int),
    "ydbl_detect_decode": ([C.POINTER(DecodeDesc), _P], C.c_int),
    "ydbl_pred_candidates": ([C.POINTER(PredCandDesc), _P], C.c_int),
    "ydbl_nms_workspace": ([C.c_int32, C.c_int32, C.c_int32], C.c_int64),
    "ydbl_conv_workspace": ([C.POINTER(ConvDesc)], C.c_int64),
    "ydbl_nms": ([C.POINTER(NmsDesc), _P], C.c_int),
    "ydbl_conv_stem2_params_size": ([C.c_int32], C.c_int64),
    "ydbl_conv_stem2_pack": ([_P, _P, _P, _P, C.c_int32, _P], C.c_int),
    "ydbl_conv_stem2": ([C.POINTER(Stem2Desc), _P], C.c_int),
    "ydbl_bottleneck_params_size": ([C.c_int32], C.c_int64),
    "ydbl_bottleneck_pack": ([_P, _P, _P, _P, C.c_int32, _P], C.c_int),
    "ydbl_bottleneck_nhwc": ([C.POINTER(BottleneckDesc), _P], C.c_int),
    "ydbl_conv3x3_pair_params_size": ([C.c_int32, C.c_int32], C.c_int64),
    "ydbl_conv3x3_pair_pack": ([_P, _P, _P, _P, C.c_int32, C.c_int32, _P], C.c_int),
    "ydbl_detect_box_params_size": ([C.c_int32, C.c_int32], C.c_int64),
    "ydbl_detect_box_pack": ([_P, _P, _P, _P, _P, _P, C.c_int32, C.c_int32, _P], C.c_int),
    "ydbl_letterbox": ([C.POINTER(LetterboxDesc), _P], C.c_int),
    "ydbl_match_workspace": ([C.c_int32, C.c_int32, C.c_int32, C.c_int32], C.c_int64),
    "ydbl_match_predictions": ([C.POINTER(MatchDesc), _P], C.c_int),
    "ydbl_last_error": ([], C.c_char_p),
    "ydbl_version": ([], C.c_char_p),
}


def _load():
    if not LIB_PATH.exists():
        raise ImportError(
            f"libydbl.so not found at {LIB_PATH}; build it with `python -c \"import __graft_entry__ as g; g.build()\"` "
            "(the HIP path has no fallback)"
        )
    lib = C.CDLL(str(LIB_PATH))
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


lib = _load()


class YdblError(RuntimeError):
    pass


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib.ydbl_last_error().decode(errors="replace")
        raise YdblError(f"{what or 'ydbl'} failed (code {rc}): {msg}")


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float16:
        return F16
    if dt == torch.float32:
        return F32
    raise TypeError(f"unsupported activation dtype {dt}")


def version() -> str:
    return lib.ydbl_version().decode()


def batch_max_work(device) -> "torch.Tensor":
    """A ready work buffer for ydbl_batch_max on `device` (include/ydbl.h)."""
    import torch

    host = torch.empty(int(lib.ydbl_batch_max_work_ints()), dtype=torch.int32)
    lib.ydbl_batch_max_work_init(host.data_ptr())
    return host.to(device)
