#!/bin/bash
# GPU session (developer tool): refill thresholds, waves per SIMD and the dual step on the 64-view C3 batch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab_variants.py C3 --views 64 --rounds 3 --arms ship: r60:4=60 r56:4=56 w3:6=15 w5:6=135 nodual:10=0 > gpurun_out/ab64.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab64.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
JT_SAVE=gpurun_out/jobs_C3.npz timeout -k 10 200 python tools/job_trace.py C3 > gpurun_out/job_trace_C3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/job_trace_C3.log | head -40
