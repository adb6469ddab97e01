# round 6 call 3: readout variant 5 (readout_h32, 32x32x16): readout parity tests, then the readout's
# kernel time against variant 4 (single stream, kernel trace)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c03
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "forward_matches_oracle or hidden_sizes or split_bf16_contractions or split_fp16_scaling or readout_operations or resident_forward_is" \
  > gpurun_out/c03/pytest.log 2>&1 || { tail -30 gpurun_out/c03/pytest.log; exit 1; }
tail -3 gpurun_out/c03/pytest.log
for v in 4 5; do
  IGN_READOUT_VARIANT=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c03/v$v -o v$v --output-format csv -- \
    python3 bench.py --no-cpu --no-edge-cut --streams 1 --steps 10 --warmup 3 > gpurun_out/c03/v$v.json 2> gpurun_out/c03/v$v.err || exit 1
  grep -h "readout" gpurun_out/c03/v$v/*kernel_stats.csv | cut -d, -f1-7
done
for v in 4 5; do IGN_READOUT_VARIANT=$v timeout -k 10 180 python3 bench.py --no-cpu --no-edge-cut > gpurun_out/c03/d$v.json 2>&1 || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/c03/d$v.json; done
