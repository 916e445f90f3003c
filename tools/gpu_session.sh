#!/bin/bash
# GPU session (developer tool): parity tests, variant A/B, bench, rocprofv3 kernel-trace summary of the
# bench.  Usage: bash tools/gpu_session.sh TAG [skip-tests]
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02}
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u tools/ab_variants.py C3 C4 --views 16 --rounds 4 > gpurun_out/ab_${TAG}.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}.log; exit 1; }
cat gpurun_out/ab_${TAG}.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single-frame > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*stats*"
