#!/bin/bash
# GPU session (developer tool): A/B of the drain refill (RT_OPT_DRAIN_REFILL = 11) on C3 (frame, 64-view batch), C4, C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_variants.py C3 --views 64 --rounds 3 --arms ship: drain:11=1 > gpurun_out/ab_drain_c3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_drain_c3.log
timeout -k 10 300 python tools/ab_variants.py C4 --views 4 --rounds 2 --arms ship: drain:11=1 > gpurun_out/ab_drain_c4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_drain_c4.log
timeout -k 10 400 python tools/ab_variants.py C5 --views 1 --rounds 2 --arms ship: drain:11=1 > gpurun_out/ab_drain_c5.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_drain_c5.log
