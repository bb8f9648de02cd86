"""Build libydbl.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

The shared library is written next to this file so it travels with the repo
snapshot to the GPU box; objects go to ``yolo-dbl_amd/build/``.  Rebuilds are
incremental on source/header mtimes.
"""

from __future__ import annotations

import os
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"
OBJ_DIR = ROOT / "build"
LIB_PATH = PKG_DIR / "libydbl.so"
ARCH = os.environ.get("YDBL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _headers():
    return sorted(list(CSRC.glob("*.hpp")) + list(INCLUDE.glob("*.h")))


def _compile(src: Path, obj: Path):
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build_library(force: bool = False, jobs: int | None = None) -> Path:
    """Compile every csrc/*.hip for gfx950 and link libydbl.so; returns the library path."""
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hdr_mtime = max((h.stat().st_mtime for h in _headers()), default=0.0)
    todo, objs = [], []
    for src in _sources():
        obj = OBJ_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_mtime):
            todo.append((src, obj))
    if todo:
        with ThreadPoolExecutor(max_workers=jobs or min(8, len(todo))) as ex:
            list(ex.map(lambda a: _compile(*a), todo))
    newest = max(o.stat().st_mtime for o in objs)
    if force or todo or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < newest:
        tmp = LIB_PATH.with_name(LIB_PATH.name + ".tmp")  # linked aside, then renamed: never a half-written library
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build_library(force=False))
