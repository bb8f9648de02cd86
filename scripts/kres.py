"""Per-kernel register / LDS / occupancy summary of one .hip file (hipcc -Rpass-analysis=kernel-resource-usage).

    python scripts/kres.py yolo-dbl_amd/csrc/conv.hip [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o", "/tmp/_kres.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).split(" ")[0], m.group(2)
    if k == "Function":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for d in rows:
    if flt in d["name"]:
        print(f"{d.get('VGPRs','?'):>4} {d.get('AGPRs','?'):>4} scr {d.get('ScratchSize','?'):>4} occ {d.get('Occupancy','?')} lds {d.get('LDS','?'):>6}  {d['name'][:90]}")
