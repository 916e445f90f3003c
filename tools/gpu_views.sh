#!/bin/bash
# GPU session (developer tool): the new render.bmp pin test, then the bench at 16 / 32 / 64 views per launch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_render_bmp_pin.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pin_gpu.log 2>&1 || { tail -30 gpurun_out/pin_gpu.log; exit 1; }
tail -3 gpurun_out/pin_gpu.log
for v in 16 32 64; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --views $v --no-cpu-baseline --no-single-frame > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_v$v.json'));print($v,d['value'],d['config']['ms_per_frame'],d['roofline']['frac'])"
done
SE_VIEWS=16 timeout -k 10 200 python tools/simd_eff.py C3 > gpurun_out/simd_eff.log 2>&1 || exit $?
cat gpurun_out/simd_eff.log | grep -v amdgpu.ids
timeout -k 10 300 python tools/ab_variants.py C3 --views 16 --rounds 3 --arms ship: inline_coop2:6=0,2=2,3=16 inline_coop2_8:6=0,2=2,3=8 > gpurun_out/ab_coop.log 2>&1 || exit $?
cat gpurun_out/ab_coop.log | grep -v amdgpu.ids
