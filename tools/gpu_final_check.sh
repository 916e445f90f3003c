#!/bin/bash
# GPU session (developer tool): smoke(), the default bench line, and the 2-rank gloo rehearsal of the N-rank path.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/smoke.log
bash tools/gpu_bench_check.sh
