#!/bin/bash
# Variant A/B on one GPU box (developer tool).  Usage: bash tools/gpu_ab.sh TAG "C3 C4" "arm arm ..."
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-ab}; CFGS=${2:-C3}; ARMS=${3:-}
if [ -n "$ARMS" ]; then A="--arms $ARMS"; else A=""; fi
timeout -k 10 600 python -u tools/ab_variants.py $CFGS --views 16 --rounds 4 $A > gpurun_out/ab_${TAG}.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}.log; exit 1; }
cat gpurun_out/ab_${TAG}.log
