# round 6 call 4: readout_h32 with hand-placed VALU slices (4 waves: 1 per SIMD; 8 waves: lib_ro8), against
# readout_h16; the resident forward's longest-first graph order (IGN_RES_LPT) on the default bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c04
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "forward_matches_oracle or hidden_sizes or split_bf16_contractions or split_fp16_scaling or readout_operations or resident_forward_is" \
  > gpurun_out/c04/pytest.log 2>&1 || { tail -30 gpurun_out/c04/pytest.log; exit 1; }
tail -1 gpurun_out/c04/pytest.log
for cfg in "v4|IGN_READOUT_VARIANT=4" "v5w4|IGN_READOUT_VARIANT=5" "v5w8|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_ro8.so"; do
  n=${cfg%%|*}; e=${cfg#*|}
  env $e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c04/$n -o $n --output-format csv -- \
    python3 bench.py --no-cpu --no-edge-cut --streams 1 --steps 10 --warmup 3 > gpurun_out/c04/$n.json 2> gpurun_out/c04/$n.err || exit 1
  echo "$n $(grep -h 'readout_h\|resident_forward' gpurun_out/c04/$n/*kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
for cfg in "lpt1_v5|IGN_RES_LPT=1" "lpt0_v5|IGN_RES_LPT=0" "lpt1_v4|IGN_READOUT_VARIANT=4" "lpt0_v4|IGN_RES_LPT=0 IGN_READOUT_VARIANT=4" "lpt1_v5b|IGN_RES_LPT=1" "lpt0_v5b|IGN_RES_LPT=0"; do
  n=${cfg%%|*}; e=${cfg#*|}
  env $e timeout -k 10 180 python3 bench.py --no-cpu --no-edge-cut > gpurun_out/c04/d_$n.json 2>&1 || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c04/d_$n.json)"
done
