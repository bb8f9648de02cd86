"""Summarise rocprofv3 PMC passes over one bench command per kernel family into profiles/.

    python scripts/pmc_summary.py gpurun_out/<tag> profiles/<round>_pmc_families.json ["<bench workload_key>"]

Passes (scripts/pmc_families.sh, one counter group per run, --kernel-trace only):
  FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES + GRBM_GUI_ACTIVE.
HBM bytes per launch = (m * FETCH_SIZE + WRITE_SIZE) KB * 1024, m = 2 for the 16-B/lane loads (gfx950
FETCH_SIZE tallies a 128-B request of a wide streaming read at 64 B, MI355X_MICROARCH.md HBM section),
m = 1 for NMS / decode (4-B/lane loads).  Infinity-Cache hits are counted.
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): MFMA-busy SIMD cycles over
the SIMD cycles of the dispatch (GRBM_GUI_ACTIVE is summed over the 8 XCDs).  The summary carries the
source hash of the HIP code it was measured on; bench.py uses it only when the hash matches.
"""
import csv
import glob
import hashlib
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

FAMILIES = {  # family -> (kernel-name keys, FETCH_SIZE multiplier)
    "conv2d": (("conv_igemm_kernel", "conv3x3_tile_kernel", "conv_wsk_kernel", "conv3x3_halo_kernel",
                "conv3x3_vw_kernel"), 2),
    "dsconv": (("dsconv_kernel", "dsc_lean_kernel"), 2),
    "bottleneck": (("bneck_kernel",), 2),
    "stem2": (("stem2_kernel",), 2),
    "stem": (("stem_kernel",), 2),
    "depthwise": (("dwconv_lds_kernel", "dwconv_kernel", "dw_pair_kernel"), 2),
    "hypergraph": (("hg_", "hg3_"), 2),
    "dysample": (("dysample_kernel", "dysample2_kernel"), 2),
    "lsk": (("lsk_attn_kernel", "lsk_out_kernel"), 2),
    "decode": (("decode_kernel",), 1),
    "nms": (("nms_kernel",), 1),
}


def code_hash() -> str:
    """sha256 of the HIP sources + the C-ABI header (the code the counters describe), 12 hex."""
    h = hashlib.sha256()
    files = sorted((ROOT / "yolo-dbl_amd" / "csrc").glob("*.hip")) + sorted((ROOT / "yolo-dbl_amd" / "csrc").glob("*.hpp"))
    files += sorted((ROOT / "include").glob("*.h"))
    for f in files:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:12]


def family(name):
    for fam, (keys, _) in FAMILIES.items():
        if any(k in name for k in keys):
            return fam
    return None


def load(d):
    """{counter: {family: [values per dispatch]}} over every counter_collection.csv under d."""
    out = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)  # (dispatch, counter) -> value summed over instances
        names = {}
        for r in csv.DictReader(open(path)):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
        for key, v in per.items():
            fam = family(names[key])
            if fam:
                out[key[1]][fam].append(v)
    return out


def main():
    d, dst = sys.argv[1], sys.argv[2]
    c = load(d)
    res = {"code_hash": code_hash(), "workload": sys.argv[3] if len(sys.argv) > 3 else None, "source": d,
           "method": __doc__.split("\n\n", 1)[1].strip(), "families": {}}
    for fam, (_, mult) in FAMILIES.items():
        f, w = c["FETCH_SIZE"].get(fam), c["WRITE_SIZE"].get(fam)
        if not f or not w:
            continue
        e = {"launches": len(f), "fetch_kb_per_launch": round(sum(f) / len(f), 1),
             "write_kb_per_launch": round(sum(w) / len(w), 1), "fetch_multiplier": mult}
        e["hbm_bytes_per_launch"] = int((mult * e["fetch_kb_per_launch"] + e["write_kb_per_launch"]) * 1024)
        mb, gui = c["SQ_VALU_MFMA_BUSY_CYCLES"].get(fam), c["GRBM_GUI_ACTIVE"].get(fam)
        if mb and gui:
            e["mfma_busy"] = round(sum(mb) / (1024 * sum(gui) / 8), 4)
            e["mfma_busy_cycles_per_launch"] = int(sum(mb) / len(mb))
            e["gui_active_per_launch"] = int(sum(gui) / len(gui))
        wc = c["SQ_WAVE_CYCLES"].get(fam)
        if wc and gui:
            # SQ_WAVE_CYCLES counts quad-cycles summed over resident waves; GRBM_GUI_ACTIVE sums 8 XCDs
            e["avg_waves_per_cu"] = round(4 * sum(wc) / (sum(gui) / 8) / 256, 2)
        if wc:
            tot = sum(wc)
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c[k].get(fam):
                    e[k.lower().replace("sq_", "") + "_frac"] = round(sum(c[k][fam]) / tot, 3)
        res["families"][fam] = e
    Path(dst).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
