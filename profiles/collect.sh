#!/bin/bash
# Profile the bench workload on the GPU box (run from the repo root, via gpurun).
#   pass 1: kernel trace + stats (per-kernel durations)
#   pass 2..: PMC counters, one group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass)
# Output under gpurun_out/prof_<tag>/ ; summarise with profiles/summarize.py.
set -o pipefail
TAG=${1:-r01}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu --no-edge-cut"}
# the trace pass runs the bench command as given (default: bench.py's defaults without the edge-cut
# leg, whose 1M-node kernels would otherwise mix into the kernel kinds of the workload profiled)
TRACE_ARGS=${TRACE_ARGS-"--no-edge-cut"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # name, bench args, rocprofv3 options...
  local name=$1; local bargs=$2; shift 2
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $bargs \
    > $OUT/$name.log 2>&1 || { echo "pass $name failed rc=$?"; tail -20 $OUT/$name.log; return 1; }
  echo "pass $name ok"
}
run trace "$TRACE_ARGS" --kernel-trace --stats &&
run fetch "$ARGS" --pmc FETCH_SIZE &&
run write "$ARGS" --pmc WRITE_SIZE &&
run sq "$ARGS" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU &&
run tcc "$ARGS" --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT
