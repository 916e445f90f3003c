#!/bin/bash
# A/B of three library builds (SAH traversal cost) on C3 and C4, one process per library and config
set -o pipefail
for lib in base sah10 sah025; do
  L="--lib raytracer-group27_amd/build/${lib}_librt.so"
  timeout -k 10 300 python -u tools/ab_variants.py C3 --views 64 --rounds 3 --arms d $L > gpurun_out/ab_${TAG}_C3_$lib.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_variants.py C4 --views 16 --rounds 2 --arms d $L > gpurun_out/ab_${TAG}_C4_$lib.log 2>&1 || exit 1
done
grep -H "ms" gpurun_out/ab_${TAG}_*.log
