"""CPU oracle for the YOLO-DBL inference hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain PyTorch-CPU (fp32) restatement of the reference's
inference path (player4771/YOLO-DBL, `models/YOLO/ultralytics`), written from
the cited reference lines.  It exists to CHECK the HIP product path:

* only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
  ``bench.py`` may import it;
* nothing under ``yolo-dbl_amd/`` imports it, and the product never falls back
  to it.

Parity status: **parity unpinned**.  The reference cannot be imported here
(the environment refused running reference code), it ships
no golden vectors, no weights and no test suite.  The oracle is
pinned only by the reference's own shape-level known-answer examples (module
docstrings, see tests/test_oracle.py) and by internal consistency checks.
Third-party arithmetic the reference delegates (ATen conv/grid_sample,
torchvision 0.23 NMS) is restated: ATen ops are called directly on this
container's torch, torchvision NMS is re-implemented per its published CPU
kernel semantics (stable descending sort, strict ``IoU > thr`` in double,
no +1 in areas).
"""

from .model import (  # noqa: F401
    build_model,
    guess_model_scale,
    load_model_cfg,
    make_divisible,
)
from .ops import non_max_suppression, nms_torchvision, xywh2xyxy, clip_boxes  # noqa: F401
