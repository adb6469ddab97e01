# round 6 call 17: the bench sweep (one line per workload) and the headline profile (kernel trace +
# PMC passes) on the current tree
set -o pipefail
timeout -k 10 1000 bash tools/bench_sweep.sh || exit 1
timeout -k 10 700 bash profiles/collect.sh r06 || exit 1
