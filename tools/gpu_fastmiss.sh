#!/bin/bash
# GPU session (developer tool): A/B of the fast-miss job fetch (RT_OPT_FAST_MISS = 11) against the previous build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_variants.py C3 --views 64 --rounds 3 --lib raytracer-group27_amd/build/old_librt.so --arms old: > gpurun_out/ab_fm_old.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_fm_old.log
timeout -k 10 400 python tools/ab_variants.py C3 --views 64 --rounds 3 --arms fm0: fm1:11=1 fm2:11=2 fm4:11=4 fm16:11=16 > gpurun_out/ab_fm_c3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_fm_c3.log
timeout -k 10 300 python tools/ab_variants.py C4 --views 4 --rounds 2 --arms fm0: fm4:11=4 > gpurun_out/ab_fm_c4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_fm_c4.log
