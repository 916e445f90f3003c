#!/bin/bash
# A/B of the in-tree library against another build (raytracer-group27_amd/build/base_librt.so), one
# process per library: TAG=name [CFGS="C3:64:3:op: C4:16:2:d:"] bash tools/ab_libs.sh
# (CFG:VIEWS:ROUNDS:ARMS with ARMS space-free, comma-separated tools/ab_variants.py arms)
set -o pipefail
CFGS=${CFGS:-"C3:64:3:op: C4:16:2:d: C5:2:2:d:"}
for lib in new base; do
  L=""; [ $lib = base ] && L="--lib raytracer-group27_amd/build/base_librt.so"
  for c in $CFGS; do
    IFS=: read -r cfg views rounds arms <<< "$c"
    timeout -k 10 300 python -u tools/ab_variants.py $cfg --views $views --rounds $rounds --arms ${arms//,/ } $L \
      > gpurun_out/ab_${TAG}_${cfg}_$lib.log 2>&1 || exit 1
  done
done
grep -H "ms" gpurun_out/ab_${TAG}_*.log
