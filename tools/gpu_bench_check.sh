#!/bin/bash
# GPU session (developer tool): the default bench line, then the 2-rank gloo rehearsal of the N-rank path.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
bash tools/gpu_rehearse_ranks.sh
