#!/bin/bash
# GPU session (developer tool): candidate build with RT_OPT_TILE_ORDER (11): bit-identity of order 1 against the
# in-tree library, then an A/B of order 0 vs 1 inside the candidate.
set -o pipefail
mkdir -p gpurun_out
CAND_OPTS=11=1 timeout -k 10 200 python tools/cand_check.py > gpurun_out/cand_check.log 2>&1 || { cat gpurun_out/cand_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cand_check.log
for r in 1 2; do
timeout -k 10 400 python tools/ab_variants.py C3 C5 --views 64 --rounds 3 --lib raytracer-group27_amd/build/new_librt.so --arms o0:11=0 z1:11=1 > gpurun_out/ab_order_$r.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_order_$r.log
done
