#!/bin/bash
# Diagnostic library with per-workgroup phase stamps for the kernels named (bneck.hip: -DYDBL_BNECK_STAMPS,
# detect.hip: -DYDBL_NMS_STAMPS), in build_dbg/.  Used by scripts/*_stamps.py through YDBL_LIB; never by the
# product, tests or bench.   usage: bash scripts/build_stamps.sh bneck|detect
set -e
cd "$(dirname "$0")/.."
SRC=$1; DEF=$(echo "YDBL_${SRC}_STAMPS" | tr a-z A-Z); [ "$SRC" = detect ] && DEF=YDBL_NMS_STAMPS
python -c "import sys; sys.path.insert(0, 'yolo-dbl_amd'); from ydbl import _build; _build.build_library()" >/dev/null
mkdir -p build_dbg
FLAGS=$(python -c "import sys; sys.path.insert(0,'yolo-dbl_amd'); from ydbl import _build; print(' '.join(_build.CFLAGS))")
/opt/rocm/bin/hipcc $FLAGS -D$DEF -c yolo-dbl_amd/csrc/$SRC.hip -o build_dbg/${SRC}_stamps.o
OBJS=$(python -c "import sys; sys.path.insert(0,'yolo-dbl_amd'); from ydbl import _build; print(' '.join(str(_build.OBJ_DIR / (p.stem + '.o')) for p in _build._sources() if p.stem != '$SRC'))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build_dbg/${SRC}_stamps.o -o build_dbg/libydbl_${SRC}_stamps.so
echo build_dbg/libydbl_${SRC}_stamps.so
