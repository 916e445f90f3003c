"""Developer tool: fold the rocprofv3 --pmc passes of tools/profile.sh into one JSON summary.

    python tools/pmc_summary.py gpurun_out/pmc_TAG C3 profiles/rNN/C3_pmc.json [--latest]

Per counter: the median over the render-kernel dispatches of the per-dispatch value.  HBM traffic
per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KB;
FETCH_SIZE counts 128-B requests at 64 B on gfx950, so it is doubled; WRITE_SIZE is exact.
With --latest the summary is also written to profiles/pmc_latest.json, which bench.py reads for
roofline.traffic -- only while `lib_sha` (sha256 of the librt_amd.so this tree ships, i.e. the build
the GPU run profiled) matches the library bench.py loads.
"""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def collect(root, kernel_sub="_kernel<false"):
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    kname = None
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                if kernel_sub not in k:
                    continue
                kname = k
                key = (f, row.get("Dispatch_Id", "0"))
                vals[row["Counter_Name"]][key] += float(row["Counter_Value"])
    med = {c: statistics.median(d.values()) for c, d in vals.items()}
    return kname, med


def main():
    root, cfg, out = sys.argv[1], sys.argv[2], sys.argv[3]
    kname, med = collect(root)
    if not med:
        sys.exit(f"no counter rows for the render kernel under {root}")
    hbm = None
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        hbm = (2.0 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024.0
    with open(os.path.join(REPO, "raytracer-group27_amd", "librt_amd.so"), "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    d = {"config": cfg, "kernel": kname, "lib_sha": sha, "per_dispatch_median": med, "hbm_bytes_per_launch": hbm,
         "note": "rocprofv3 --pmc, one pass per counter group (tools/profile.sh); FETCH_SIZE/WRITE_SIZE in KB; "
                 "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md (gfx950 "
                 "FETCH_SIZE tallies 128-B requests at 64 B); Infinity-Cache hits are counted, not excluded"}
    if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
        d["l2_hit_rate"] = med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in med:
        # the per-dispatch GRBM_GUI_ACTIVE here is summed over the 8 XCDs, so the kernel's span is ~1/8 of it
        simd_cycles = 1024.0 * max(1.0, med["GRBM_GUI_ACTIVE"] / 8.0)
        if "SQ_INSTS_VALU" in med:
            # SIMD issue use: a SIMD-32 issues one wave64 VALU instruction per 2 cycles (MI355X_MICROARCH.md), so
            # the share of SIMD cycles spent issuing VALU = SQ_INSTS_VALU * 2 / (1024 SIMDs * kernel cycles)
            d["valu_issue"] = med["SQ_INSTS_VALU"] * 2.0 / simd_cycles
        if "SQ_ACTIVE_INST_VALU" in med:
            # the CDNA3 VALUBusy formula (counter_defs.yaml: SQ_ACTIVE_INST_VALU quad-cycles x 4 per SIMD cycle):
            # every wave64 VALU instruction counts 4 cycles of its wave, so on gfx950's SIMD-32 units, which
            # interleave two waves' instructions, it reaches 2.0 at full issue -- not a utilisation (valu_issue is)
            d["valu_active_cdna3_formula"] = med["SQ_ACTIVE_INST_VALU"] * 4.0 / simd_cycles
    if "SQ_WAVE_CYCLES" in med:
        wc = max(1.0, med["SQ_WAVE_CYCLES"])
        d["wave_cycle_split"] = {k: med[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
                                 if k in med}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    if "--latest" in sys.argv:
        with open(os.path.join(REPO, "profiles", "pmc_latest.json"), "w") as f:
            json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
