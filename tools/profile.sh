#!/bin/bash
# PMC collection: one rocprofv3 pass per counter group (no sys/runtime traces with --pmc),
# kernel-trace only alongside, each pass under its own hard time limit.
# Usage: bash tools/profile.sh TAG CONFIG [VIEWS]   (summarise with tools/pmc_summary.py)
set -o pipefail
TAG=${1:-r01}; CFG=${2:-C3}; VIEWS=${3:-1}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
i=0
while read -r line; do
  ctrs=${line#pmc: }
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/g$i -o run -- python3 tools/prof_target.py $CFG 3 $VIEWS > $OUT/g$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/g$i.log; exit 1; }
  echo "pass $i ok: $ctrs"
done < ${PMC_FILE:-tools/pmc_counters.txt}
find $OUT -name "*.csv" | head -30
