set -e
mkdir -p gpurun_out
V="${VARIANTS:-3 4}"
for v in $V; do
IGN_SUM_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_edge_cut.py "tests/test_gpu_parity.py::test_hidden_sizes" "tests/test_gpu_parity.py::test_synthetic_graph_h64_matches_oracle" -x -q > gpurun_out/pt_$v.log 2>&1
IGN_SUM_VARIANT=$v timeout -k 10 200 python bench.py --model synthetic --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_$v.log 2>&1
done
