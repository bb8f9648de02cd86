"""Per-kernel table from scripts/pmc_kernels.sh passes: waves, cycles split (active / wait / issue-stall), MFMA busy,
instruction mix, LDS bank conflicts and HBM bytes per dispatch (FETCH_SIZE x2 for 16-B streaming loads, the gfx950
correction of MI355X_MICROARCH.md; WRITE_SIZE as is), averaged over the dispatches of each ydbl kernel.

    python scripts/pmc_table.py gpurun_out/<tag>
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"ydbl::", "", name)
    return name[:70]


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "ydbl" not in r["Kernel_Name"]:
                continue
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in glob.glob(f"{d}/kt/run_kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if "ydbl" in r["Kernel_Name"]:
                dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    avg = lambda v: sum(v) / len(v) if v else float("nan")
    for k, c in vals.items():
        a = {n: avg(v) for n, v in c.items()}
        wc = a.get("SQ_WAVE_CYCLES", float("nan"))
        gui = a.get("GRBM_GUI_ACTIVE", float("nan"))
        mb = a.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (1024 * gui / 8) if gui else float("nan")
        hbm = 2 * a.get("FETCH_SIZE", 0) * 1024 + a.get("WRITE_SIZE", 0) * 1024
        t = avg(dur.get(k, []))
        print(f"{k}\n   us {t:7.2f}  waves {a.get('SQ_WAVES', 0):7.0f}  wait_any {a.get('SQ_WAIT_ANY', 0) / wc:5.2f}  "
              f"wait_inst {a.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f}  active {a.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f}  "
              f"mfma_busy {mb:5.3f}  waves/CU avg {wc / (gui / 8) / 256 if gui else 0:5.1f}\n"
              f"   insts/wave: valu {a.get('SQ_INSTS_VALU', 0) / max(a.get('SQ_WAVES', 1), 1):7.0f}  "
              f"lds {a.get('SQ_INSTS_LDS', 0) / max(a.get('SQ_WAVES', 1), 1):6.0f}  "
              f"vmem_rd {a.get('SQ_INSTS_VMEM_RD', 0) / max(a.get('SQ_WAVES', 1), 1):5.0f}  "
              f"vmem_wr {a.get('SQ_INSTS_VMEM_WR', 0) / max(a.get('SQ_WAVES', 1), 1):5.0f}  "
              f"salu {a.get('SQ_INSTS_SALU', 0) / max(a.get('SQ_WAVES', 1), 1):5.0f}  "
              f"lds_conflict/idx {a.get('SQ_LDS_BANK_CONFLICT', 0) / max(a.get('SQ_LDS_IDX_ACTIVE', 1), 1):5.2f}  "
              f"wait_inst_lds {a.get('SQ_WAIT_INST_LDS', 0) / wc:5.2f}\n"
              f"   HBM {hbm / 1e6:8.2f} MB -> {hbm / (t * 1e-6) / 1e12 if t == t and t > 0 else 0:5.2f} TB/s")


if __name__ == "__main__":
    main(sys.argv[1])
