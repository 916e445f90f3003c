#!/bin/bash
# GPU session (developer tool): parity tests, then an env A/B and a wave trace.  A failed test run
# still lets the A/B run; a crash, abort or time limit (exit >= 124) ends the script.
# Usage: bash tools/gpu_ab.sh "C2 C3 C4 C5" "r8:RT_REFILL=8 r16:RT_REFILL=16"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -4 gpurun_out/pt.log
[ $rc -ge 124 ] && exit $rc
AB_ROUNDS=${AB_ROUNDS:-5} timeout -k 10 300 python -u tools/ab_env.py $1 $2 > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python -u tools/wave_trace.py C3 > gpurun_out/wt.log 2>&1
rc=$?; cat gpurun_out/wt.log
exit $rc
