#!/bin/bash
# GPU session (developer tool): traversal-lane histogram and the per-wave drain timeline of C3 (frame, 16-view batch).
set -o pipefail
mkdir -p gpurun_out
SE_VIEWS=16 timeout -k 10 200 python tools/simd_eff.py C3 > gpurun_out/simd_eff.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/simd_eff.log
timeout -k 10 200 python tools/wave_trace.py C3 > gpurun_out/wave_trace_frame.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wave_trace_frame.log
WT_VIEWS=16 timeout -k 10 200 python tools/wave_trace.py C3 > gpurun_out/wave_trace_v16.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wave_trace_v16.log
