#!/bin/bash
# GPU session: parity tests, bench, rocprofv3 kernel-trace summary (developer tool).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-budget 10 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 || exit $?
find gpurun_out/prof_${TAG} -name "*stats*" | head
