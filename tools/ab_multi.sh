#!/bin/bash
# A/B of several library builds, one process per library and config, the shipped path (arm x) each:
#   TAG=name LIBS="a.so b.so" [CFGS="C3:64:3 C5:1:2"] bash tools/ab_multi.sh
# (developer builds: python raytracer-group27_amd/build.py -DNAME=V or -F<hipcc flag>; logs under gpurun_out/)
set -o pipefail
CFGS=${CFGS:-"C3:64:3 C3:1:5 C4:16:2 C5:1:2"}
for c in $CFGS; do
  IFS=: read -r cfg views rounds <<< "$c"
  for lib in $LIBS; do
    log=gpurun_out/abm_${TAG}_${cfg}_v${views}_$(basename "$lib" .so).log
    timeout -k 10 300 python -u tools/ab_variants.py "$cfg" --views "$views" --rounds "$rounds" --arms x: --lib "$lib" \
      > "$log" 2>&1 || exit 1
    echo "$(basename "$lib" .so): $(grep -h ' ms' "$log" | cut -c1-170)"
  done
done
