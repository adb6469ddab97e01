# N=2 host-staged rehearsal on one GPU (synthetic edge-cut; default RouteNet line with the edge_cut_1m leg)
set -o pipefail
bash tools/n2_rehearsal.sh > gpurun_out/n2_rehearsal.txt 2>&1 || { cat gpurun_out/n2_rehearsal.txt; exit 1; }
