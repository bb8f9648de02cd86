import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "yolo-dbl_amd"))
os.environ.setdefault("OMP_NUM_THREADS", "8")

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libydbl.so)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
