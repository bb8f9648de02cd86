#!/bin/bash
# Diagnostic library: libydbl with per-workgroup NMS phase stamps (-DYDBL_NMS_STAMPS), in build_dbg/.
# Used by scripts/nms_stamps.py through YDBL_LIB; never by the product, tests or bench.
set -e
cd "$(dirname "$0")/.."
python -c "
import sys; sys.path.insert(0, 'yolo-dbl_amd')
from ydbl import _build
_build.build_library()
" >/dev/null
mkdir -p build_dbg
FLAGS=$(python -c "import sys; sys.path.insert(0,'yolo-dbl_amd'); from ydbl import _build; print(' '.join(_build.CFLAGS))")
/opt/rocm/bin/hipcc $FLAGS -DYDBL_NMS_STAMPS -c yolo-dbl_amd/csrc/detect.hip -o build_dbg/detect_stamps.o
OBJS=$(ls yolo-dbl_amd/build/obj/*.o 2>/dev/null | grep -v '/detect.o$' || true)
[ -n "$OBJS" ] || OBJS=$(python -c "import sys; sys.path.insert(0,'yolo-dbl_amd'); from ydbl import _build; print(' '.join(str(p) for p in sorted(_build.OBJ_DIR.glob('*.o')) if p.name != 'detect.o'))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build_dbg/detect_stamps.o -o build_dbg/libydbl_stamps.so
echo build_dbg/libydbl_stamps.so
