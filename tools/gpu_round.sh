#!/bin/bash
# GPU session (developer tool): parity tests, bench, rocprofv3 kernel-trace summary of the bench,
# then the PMC passes of tools/profile.sh.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-budget 12 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single-frame > gpurun_out/prof_${TAG}.log 2>&1 || exit $?
find gpurun_out/prof_${TAG} -name "*stats*"
[ "${2:-}" = "nopmc" ] && exit 0
bash tools/profile.sh ${TAG} C3 64
