#!/bin/bash
# The one GPU-session driver (run on the box through gpurun): named steps, each under its own time limit,
# chained so the first failure ends the session (no GPU step runs after a failed, killed or faulted one).
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# STEP                          what runs (outputs under gpurun_out/, TAG in the names)
#   tests[:PYTEST_K]            pytest -m gpu (optionally -k PYTEST_K)
#   testsall                    pytest -m gpu without -x (every failure in one session; ends the session if any)
#   smoke                       __graft_entry__.smoke()
#   bench[:CFG[:VIEWS]]         bench.py line (N = 1; roofline.traffic measured by its rocprofv3 passes)
#   stats[:CFG[:VIEWS]]         rocprofv3 --kernel-trace --stats of bench.py (kernel summary for profiles/)
#   kstats:CFG:VIEWS:OPTS:TAG2  rocprofv3 --kernel-trace --stats of tools/prof_target.py (OPTS k=v;k=v render options)
#   pmcx:CFG:VIEWS:OPTS:TAG2:CTRS  one rocprofv3 --pmc pass (CTRS ;-separated) of tools/prof_target.py (OPTS k=v;k=v),
#                               summed per kernel (tools/pmc_by_kernel.py)
#   pmc[:CFG[:VIEWS]]           the PMC counter groups of tools/pmc_counters.txt (tools/profile.sh)
#   ab:CFGS:VIEWS:ROUNDS[:ARMS] tools/ab_variants.py (CFGS / ARMS comma-separated; ARMS name=k=v;k=v)
#   simd[:CFG[:VIEWS[:ARMS]]]   tools/simd_eff.py (counting build: lanes per node / record step; ARMS comma-separated
#                               name@k=v, e.g. new@,old@11=3)
#   wave[:CFG[:VIEWS[:COUNT]]]  tools/wave_trace.py (per-wave start / drain / end; COUNT 1: counting build)
#   jobs[:CFG[:OPTS]]           tools/job_trace.py (per-pixel query chains of a single frame; OPTS k=v;k=v)
#   ranks                       bench.py N = 2 on this one GPU (gloo control plane, IPC exchange)
#   ipc[:VIEWS]                 tools/ipc_probe.py: owner + opener of an IPC image buffer, each step timestamped
#   ipcb:BYTES                  tools/ipc_probe.py --bytes: the IPC mapping of a buffer of BYTES alone
#   wfcheck:CFG:VIEWS[:WxH]     tools/wf_check.py: the wavefront path against the megakernel (rays, hits, images)
#   cpu_baseline                tools/cpu_baseline.py (BASELINE.md's full CPU samples on the host)
#   times                       tools/time_configs.py (every config, single frame and batch)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=${TMPDIR:-/tmp}
mkdir -p gpurun_out
TAG=$1
shift
run() {  # run LIMIT LOG cmd...: one step, its own time limit, output to gpurun_out/LOG
  local limit=$1 log=gpurun_out/$2
  shift 2
  echo "== $* (limit ${limit}s) -> $log"
  timeout -k 10 "$limit" "$@" > "$log" 2>&1
  local rc=$?
  grep -v "amdgpu.ids" "$log" | tail -${TAIL:-25}
  if [ $rc -ne 0 ]; then echo "== step failed (rc $rc): ending the session"; exit $rc; fi
}
for step in "$@"; do
  IFS=: read -r name a b c d <<< "$step"
  case $name in
    tests) if [ -n "$a" ]; then K=(-k "$a"); else K=(); fi
           run 1200 pytest_gpu_${TAG}.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" ;;
    testsall) run 1200 pytest_gpu_${TAG}.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) run 300 smoke_${TAG}.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 600 bench_${TAG}_${a:-C3}.json python bench.py --steps 20 --warmup 3 --config ${a:-C3} ${b:+--views $b} ;;
    stats) run 600 stats_${TAG}_${a:-C3}.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_${TAG}_${a:-C3} -o run -- python3 bench.py --steps 20 --warmup 3 --config ${a:-C3} ${b:+--views $b} --no-cpu-baseline --no-single-frame --no-pmc
           find gpurun_out/stats_${TAG}_${a:-C3} -name "*kernel_stats.csv" -exec head -3 {} \; ;;
    kstats) run 300 kstats_${TAG}_${d:-x}.log env PT_OPTS="${c//;/,}" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_${TAG}_${d:-x} -o run -- python3 tools/prof_target.py ${a:-C3} 3 ${b:-64}
           find gpurun_out/kstats_${TAG}_${d:-x} -name "*kernel_stats.csv" -exec cat {} \; ;;
    pmcx)  IFS=: read -r _n _a _b _c d CTRS <<< "$step"
           run 120 pmcx_${TAG}_${d:-x}.log env PT_OPTS="${c//;/,}" timeout -s KILL 100 rocprofv3 --pmc ${CTRS//;/ } --kernel-trace --output-format csv -d gpurun_out/pmcx_${TAG}_${d:-x} -o run -- python3 tools/prof_target.py ${a:-C3} 2 ${b:-64}
           python3 tools/pmc_by_kernel.py gpurun_out/pmcx_${TAG}_${d:-x} 2 | tee gpurun_out/pmcx_${TAG}_${d:-x}.txt | cut -c1-400 ;;
    pmc)   run 900 pmc_${TAG}_${a:-C3}.log bash tools/profile.sh ${TAG}_${a:-C3} ${a:-C3} ${b:-64} ;;
    ab)    ARMS=(); if [ -n "$d" ]; then for x in ${d//,/ }; do ARMS+=("${x//;/,}"); done; ARMS=(--arms "${ARMS[@]/=/:}"); fi
           run 900 ab_${TAG}.log python -u tools/ab_variants.py ${a//,/ } --views ${b:-16} --rounds ${c:-3} "${ARMS[@]}" ;;
    simd)  c=${c//,/ }; run 300 simd_${TAG}_${a:-C3}.log env SE_VIEWS=${b:-16} python tools/simd_eff.py ${a:-C3} ${c//@/:} ;;
    wave)  run 300 wave_${TAG}${c:+_count}.log env WT_VIEWS=${b:-1} WT_COUNT=${c:-0} python tools/wave_trace.py ${a:-C3} ;;
    jobs)  run 300 jobs_${TAG}${b:+_$b}.log python tools/job_trace.py ${a:-C3} ${b//;/ } ;;
    ranks) run 600 ranks_${TAG}.json env BENCH_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 --no-single-frame ;;
    ranksv) run 600 ranks_${TAG}_v${a:-96}.json env BENCH_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 2 --steps 3 --warmup 1 --no-single-frame --no-pmc --no-cpu-baseline --views ${a:-96} ;;
    ipc)   run 150 ipc_${TAG}_v${a:-96}.log python -u tools/ipc_probe.py --views ${a:-96} --timeout 110 ;;
    phases) run 200 phases_${TAG}_${a:-C3}_${b:-1}.log python -u tools/phase_trace.py ${a:-C3} ${b:-1} ${c:-6} ;;
    exh)   run 200 exh_${TAG}_${a:-C3}_${b:-1}.log python -u tools/exh_count.py ${a:-C3} ${b:-1} ;;
    ipcb)  run 100 ipcb_${TAG}_${a}.log python -u tools/ipc_probe.py --bytes ${a} --timeout 60 ;;
    wfcheck) run 300 wfcheck_${TAG}_${a}_${b}.log python -u tools/wf_check.py ${a:-C3} ${b:-8} ${c} ;;
    cpu_baseline) run 1500 cpu_baseline_${TAG}.json python tools/cpu_baseline.py --out gpurun_out/cpu_baseline_${TAG}.out.json ;;
    times) run 900 times_${TAG}.log python tools/time_configs.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== session $TAG: all steps ok"
