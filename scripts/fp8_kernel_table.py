"""Per-kernel time of the e4m3 operand path against the fp16 one, from the rocprofv3 summaries of config 5
(DBL-s 640 bs32, two sub-batch graphs): every dense-conv template with the Q8 flag off (fp16 run) and on (all-fp8
run, every candidate switched: the same launches, same shapes) -> calls, avg us, delta.  The e4m3 path stages
quantized operands (8-byte LDS groups) and runs v_mfma_f32_16x16x32_fp8_fp8, which issues at the f16 rate.

    python scripts/fp8_kernel_table.py profiles/r05/r05_c5_dbl_s_bs32_fp16_kernel_stats.csv \
        profiles/r05/r05_c5_dbl_s_bs32_fp8_kernel_stats.csv
"""
import csv
import re
import sys


def load(p):
    return {r["Name"]: (int(r["Calls"]), int(r["TotalDurationNs"])) for r in csv.DictReader(open(p))}


a, b = load(sys.argv[1]), load(sys.argv[2])
rows = []
for k, (ca, ta) in a.items():
    # the Q8 template flag: conv_wsk <T,BM,BN,SMALL,Q8,..>, conv_igemm <T,BM,BN,WM,WN,BIAS,Q8,..>, halo <T,S,TH,NTN,Q8>
    m = re.match(r"_ZN4ydbl(\d+)(conv_wsk_kernel|conv_igemm_kernel|conv3x3_halo_kernel)I(.*)EEvNS_8ConvArgs", k)
    if not m:
        continue
    kind, args = m.group(2), m.group(3)
    flags = list(re.finditer(r"Lb([01])E", args))
    qi = {"conv_wsk_kernel": 1, "conv_igemm_kernel": 1, "conv3x3_halo_kernel": 0}[kind]
    if len(flags) <= qi or flags[qi].group(1) != "0":
        continue
    f = flags[qi]
    k8 = k[:m.start(3) + f.start()] + "Lb1E" + k[m.start(3) + f.end():]
    if k8 not in b:
        continue
    cb, tb = b[k8]
    shape = re.sub(r"Li(\d+)E", r"\1,", args).replace("DF16_", "").replace("Lb0E", "0,").replace("Lb1E", "1,")
    rows.append((kind, shape.strip(","), ca, ta / ca / 1e3, cb, tb / cb / 1e3))
tot_a = sum(r[2] * r[3] for r in rows)
tot_b = sum(r[4] * r[5] for r in rows)
print(f"{'kernel':22s} {'template':18s} {'calls':>6s} {'fp16 us':>9s} {'calls':>6s} {'e4m3 us':>9s} {'delta':>7s}")
for r in sorted(rows, key=lambda r: -r[2] * r[3]):
    print(f"{r[0]:22s} {r[1]:18s} {r[2]:6d} {r[3]:9.2f} {r[4]:6d} {r[5]:9.2f} {100 * (r[5] / r[3] - 1):+6.1f}%")
print(f"sum over these templates: fp16 {tot_a / 1e3:.2f} ms, e4m3 {tot_b / 1e3:.2f} ms over the profiled steps "
      f"({100 * (tot_b / tot_a - 1):+.1f}%)")
