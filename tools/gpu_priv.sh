#!/bin/bash
# GPU session (developer tool): A/B of a candidate build (raytracer-group27_amd/build/new_librt.so) against the in-tree library.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 300 python tools/ab_variants.py C3 C2 --views 64 --rounds 3 --arms cur: > gpurun_out/ab_cur_$r.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_cur_$r.log
timeout -k 10 300 python tools/ab_variants.py C3 C2 --views 64 --rounds 3 --lib raytracer-group27_amd/build/new_librt.so --arms new: > gpurun_out/ab_new_$r.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_new_$r.log
done
timeout -k 10 300 python tools/ab_variants.py C4 --views 4 --rounds 2 --arms cur: > gpurun_out/ab_cur_c4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_cur_c4.log
timeout -k 10 300 python tools/ab_variants.py C4 --views 4 --rounds 2 --lib raytracer-group27_amd/build/new_librt.so --arms new: > gpurun_out/ab_new_c4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_new_c4.log
