"""Median per-dispatch PMC values of one kernel (default: the conv GEMM) from tools/pmc_conv.sh or
tools/pmc_sq.sh passes:  pmc_conv_summary.py <dir> [kernel-substring]"""
import csv
import glob
import os
import statistics
import sys

base = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "conv_gemm"
vals = {}
for f in sorted(glob.glob(os.path.join(base, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
med = {k: statistics.median(v) for k, v in vals.items()}
for k in sorted(med):
    print(f"{k:28s} {med[k]:16.0f}")
if "SQ_WAVE_CYCLES" in med:
    w = med["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in med:
            print(f"{k} / WAVE_CYCLES = {med[k] / w:.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
    # MFMA busy cycles summed over SIMDs vs (GUI_ACTIVE cycles x 1024 SIMDs / 8 XCD-sum)
    print("MFMA busy / (GRBM_GUI_ACTIVE/8 * 1024) =",
          round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (med["GRBM_GUI_ACTIVE"] / 8 * 1024), 3))
