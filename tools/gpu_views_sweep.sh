set -o pipefail
mkdir -p gpurun_out
for a in "8 0" "8 45" "16 22.5" "32 11.25" "16 0" "1 0"; do
  set -- $a
  timeout -k 10 120 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --views $1 --view-step $2 > gpurun_out/bench_sw.json 2>gpurun_out/bench_sw.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_sw.json'));print('$1 $2', round(d['value'],1), round(d['config']['ms_per_frame'],3), d['config']['rays_per_frame'], round(d['roofline']['frac'],4))"
done
