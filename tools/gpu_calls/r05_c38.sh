# final round-5 sweep: one bench line per workload (tools/bench_sweep.sh)
set -o pipefail
bash tools/bench_sweep.sh > gpurun_out/sweep_log.txt 2>&1 || { cat gpurun_out/sweep_log.txt; exit 1; }
