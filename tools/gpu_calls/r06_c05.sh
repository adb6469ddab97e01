# round 6 call 5: readout_h32 with a 3-slot W2 ring (prefetch distance 2): kernel time vs readout_h16,
# 4 waves (default) and 8 waves (lib_ro8); SQ counters of both readouts (single stream)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c05
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "forward_matches_oracle or split_bf16_contractions or split_fp16_scaling or resident_forward_is" \
  > gpurun_out/c05/pytest.log 2>&1 || { tail -30 gpurun_out/c05/pytest.log; exit 1; }
tail -1 gpurun_out/c05/pytest.log
for cfg in "v4|IGN_READOUT_VARIANT=4" "v5w4|IGN_READOUT_VARIANT=5" "v5w8|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_ro8.so"; do
  n=${cfg%%|*}; e=${cfg#*|}
  env $e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c05/$n -o $n --output-format csv -- \
    python3 bench.py --no-cpu --no-edge-cut --streams 1 --steps 10 --warmup 3 > gpurun_out/c05/$n.json 2> gpurun_out/c05/$n.err || exit 1
  echo "$n $(grep -h 'readout_h' gpurun_out/c05/$n/*kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
for v in 4 5; do
  IGN_READOUT_VARIANT=$v bash tools/sq_pmc.sh ro$v --streams 1 --steps 3 --warmup 1 --no-cpu --no-edge-cut || exit 1
done
