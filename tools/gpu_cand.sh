#!/bin/bash
# GPU session (developer tool): a candidate build (raytracer-group27_amd/build/new_librt.so): its bit-identity on
# the bench step (every view of a 64-view C3 launch equals the in-tree library's), then an A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/cand_check.py > gpurun_out/cand_check.log 2>&1 || { cat gpurun_out/cand_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cand_check.log
bash tools/gpu_priv.sh
