#!/bin/bash
# Build abtmp/libydbl_base.so = the in-tree library with ONE source file rewritten by a sed expression (an A/B
# variant that never enters the product tree): bash scripts/build_ab_variant.sh stem2 's/__builtin_nontemporal_load(\(.*\))/(*(\1))/'
set -e
cd "$(dirname "$0")/.."
SRC=$1; EXPR=$2
python -c "import sys; sys.path.insert(0, 'yolo-dbl_amd'); from ydbl import _build; _build.build_library()" >/dev/null
mkdir -p abtmp
sed "$EXPR" yolo-dbl_amd/csrc/$SRC.hip > abtmp/${SRC}_variant.hip
diff <(cat yolo-dbl_amd/csrc/$SRC.hip) abtmp/${SRC}_variant.hip | head -20 || true
FLAGS=$(python -c "import sys; sys.path.insert(0,'yolo-dbl_amd'); from ydbl import _build; print(' '.join(_build.CFLAGS))")
/opt/rocm/bin/hipcc $FLAGS -I yolo-dbl_amd/csrc -I include -c abtmp/${SRC}_variant.hip -o abtmp/${SRC}_variant.o
OBJS=$(python -c "import sys; sys.path.insert(0,'yolo-dbl_amd'); from ydbl import _build; print(' '.join(str(_build.OBJ_DIR / (p.stem + '.o')) for p in _build._sources() if p.stem != '$SRC'))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS abtmp/${SRC}_variant.o -o abtmp/libydbl_base.so
echo abtmp/libydbl_base.so
