#!/bin/bash
# PMC collection: one rocprofv3 pass per counter group (no sys/runtime traces with --pmc),
# kernel-trace only alongside.  Usage: bash tools/profile.sh TAG CONFIG
set -o pipefail
TAG=${1:-r01}; CFG=${2:-C3}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
i=0
while read -r line; do
  ctrs=${line#pmc: }
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/g$i -o run -- python3 tools/prof_target.py $CFG 3 > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/g$i.log; exit 1; }
  echo "pass $i ok: $ctrs"
done < tools/pmc_counters.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_target.py $CFG 5 > $OUT/trace.log 2>&1 || exit 1
find $OUT -name "*.csv" | head -30
