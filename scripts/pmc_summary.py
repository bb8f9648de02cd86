"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel family into profiles/.

    python scripts/pmc_summary.py gpurun_out/pmc1 profiles/r01_pmc_conv_summary.json

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 for the families whose loads are
16 B/lane (conv2d, dsconv, dwconv): both counters are in KB and on gfx950 FETCH_SIZE tallies the
128-B requests of a 16-B/lane streaming read at 64 B (MI355X_MICROARCH.md, HBM section).  The stem
reads the NCHW image with 4-B/lane loads, for which FETCH_SIZE matched the byte count
(154.5 MB fetched for a 157 MB input), so it is not doubled.  Infinity-Cache hits are counted.
"""
import csv
import json
import sys
from collections import defaultdict

FAMILIES = {  # name keys, FETCH_SIZE multiplier
    "conv2d": (("conv_igemm_kernel", "conv3x3_tile_kernel", "conv_wsk_kernel", "conv3x3_halo_kernel"), 2),
    "dsconv": (("dsconv_kernel",), 2),
    "stem": (("stem_kernel",), 2),
    "dwconv": (("dwconv_lds_kernel", "dwconv_kernel"), 2),
    "bottleneck": (("bneck_kernel",), 2),
    "stem2": (("stem2_kernel",), 2),
    "nms": (("nms_kernel",), 1),
}


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch = load(f"{d}/FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE")
    write = load(f"{d}/WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE")
    res = {"method": "HBM bytes = (m*FETCH_SIZE + WRITE_SIZE) KB * 1024 per launch; m = 2 for 16-B/lane "
                     "loads (gfx950 FETCH correction), 1 otherwise", "families": {}}
    for fam, (keys, mult) in FAMILIES.items():
        names = [n for n in fetch if any(k in n for k in keys)]
        nf = sum(len(fetch[n]) for n in names)
        nw = sum(len(write.get(n, [])) for n in names)
        if not nf or not nw:
            continue
        f_kb = sum(sum(fetch[n]) for n in names) / nf
        w_kb = sum(sum(write.get(n, [])) for n in names) / nw
        res["families"][fam] = {"launches": nf, "fetch_kb_per_launch": round(f_kb, 1),
                                "write_kb_per_launch": round(w_kb, 1),
                                "fetch_multiplier": mult, "hbm_bytes_per_launch": int((mult * f_kb + w_kb) * 1024)}
    res["hbm_bytes_per_launch"] = res["families"].get("conv2d", {}).get("hbm_bytes_per_launch")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
