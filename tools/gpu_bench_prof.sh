set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-budget 12 > gpurun_out/bench_r01d.json 2> gpurun_out/bench_r01d.err || exit $?
cat gpurun_out/bench_r01d.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01d -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-single-frame > gpurun_out/prof_r01d.log 2>&1 || exit $?
cat gpurun_out/prof_r01d/run_kernel_stats.csv
