#!/bin/bash
# Rehearsal of bench.py's N-rank path on a one-GPU box: 2 ranks share the GPU over gloo
# (the driver's multi-GPU runs use RCCL, one rank per GPU).  Default partition = the tile split
# (bands of every view; gloo all-gathers where RCCL gathers to rank 0; un-permute on rank 0); then the frames partition.
set -o pipefail
mkdir -p gpurun_out
export BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 3 --warmup 1 --no-single-frame > gpurun_out/rehearse_bands.json 2> gpurun_out/rehearse_bands.err || { tail -20 gpurun_out/rehearse_bands.err; exit 1; }
cat gpurun_out/rehearse_bands.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 2 --steps 3 --warmup 1 --no-single-frame --partition frames > gpurun_out/rehearse_frames.json 2> gpurun_out/rehearse_frames.err || { tail -20 gpurun_out/rehearse_frames.err; exit 1; }
cat gpurun_out/rehearse_frames.json
