"""Developer tool: rocprofv3 --pmc counters summed per kernel name (all dispatches), plus the kernel-trace
durations of the same run, so a render made of several kernels (the wavefront path: trace and shade
kernels per level) can be split by kernel.

    python tools/pmc_by_kernel.py gpurun_out/pmcx_TAG [STEPS]

Prints, per kernel: dispatches, total ms, and each counter's total / STEPS (per render step) with the derived
VALU issue fraction (SQ_INSTS_VALU * 2 / (1024 SIMDs * cycles), MI355X_MICROARCH.md: a SIMD-32 issues a
wave64 VALU instruction per 2 cycles) and the wave-cycle split when those counters are present.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    root = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    ctr = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            ctr[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add((f, row.get("Dispatch_Id")))
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[short(row["Kernel_Name"])] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    for k in sorted(ctr, key=lambda k: -dur.get(k, 0.0)):
        c = ctr[k]
        ms = dur.get(k, 0.0) / steps
        line = f"{k}: dispatches {len(disp[k])}, {ms:.3f} ms/step"
        vals = {n: v / steps for n, v in c.items()}
        line += "; " + ", ".join(f"{n} {v:.4g}" for n, v in sorted(vals.items()))
        if "SQ_INSTS_VALU" in vals and ms > 0:
            line += f"; issue frac {vals['SQ_INSTS_VALU'] * 2 / (1024 * ms * 1e-3 * 2.4e9):.3f}"
        if "SQ_WAVE_CYCLES" in vals and vals["SQ_WAVE_CYCLES"] > 0:
            wc = vals["SQ_WAVE_CYCLES"]
            line += "; wave cycles " + ", ".join(f"{n[3:]} {vals[n] / wc:.2f}" for n in
                                                ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY") if n in vals)
        print(line, flush=True)


if __name__ == "__main__":
    main()
