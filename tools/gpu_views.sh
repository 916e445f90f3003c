set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "view_batch or band_split or variants" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_views.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_views.log; [ $rc -eq 0 ] || exit $rc
for F in 1 2 4 8; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --views $F > gpurun_out/bench_v$F.json 2>gpurun_out/bench_v$F.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_v$F.json'));print($F, round(d['value'],1), d['ms_per_step'], d['config']['ms_per_frame'], d['roofline']['frac'])"
done
