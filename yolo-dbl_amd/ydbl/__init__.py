"""ydbl — YOLO-DBL inference hot path, MI355X-native (gfx950 HIP kernels behind a C ABI).

Drop-in for the reference's ``from ultralytics import YOLO`` detect path:
``YOLO("yolov13n_DBL.yaml").predict(images)``.
"""

__version__ = "0.1.0"

from .engine.model import YOLO, Model  # noqa: E402,F401
from .nn.tasks import DetectionModel, register_module  # noqa: E402,F401
from .utils.ops import non_max_suppression  # noqa: E402,F401
