# round 6 call 16: (1) the device cache trimmed by the allocating threads instead of Batch.close
# (training tests, fresh-batch training at 8 and 12 workers); (2) readout_h16 with its layer-2
# epilogue software-pipelined into the next chunk's MFMAs (IGN_RO_PIPE, A/B library): bitwise
# against the default, then kernel times, default and A/B interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c16
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c16/pytest.log 2>&1 || { tail -30 gpurun_out/c16/pytest.log; exit 1; }
tail -1 gpurun_out/c16/pytest.log
for w in 8 12; do
  IGN_BUILD_PROF=1 IGN_STEP_PROF=1 timeout -k 10 300 python3 bench.py --train --fresh-batches --steps 40 --input-workers $w > gpurun_out/c16/w$w.json 2> gpurun_out/c16/w$w.err || exit 1
  echo "w$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c16/w$w.json) $(grep -o '"close": [0-9.]*' gpurun_out/c16/w$w.json) oom-trims $(grep -c 'ign-pool' gpurun_out/c16/w$w.err || true)"
done
timeout -k 10 300 python3 tools/probes/ab_bitwise.py ropipe > gpurun_out/c16/bitwise.txt 2>&1 || { cat gpurun_out/c16/bitwise.txt; exit 1; }
cat gpurun_out/c16/bitwise.txt
for n in v4a pipea v4b pipeb; do
  e=""; case $n in pipe*) e="IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_ropipe.so";; esac
  env $e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c16/$n -o $n --output-format csv -- \
    python3 bench.py --no-cpu --no-edge-cut --steps 20 --warmup 3 > gpurun_out/c16/$n.json 2> gpurun_out/c16/$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c16/$n.json) $(grep -h 'readout_h16' gpurun_out/c16/$n/*kernel_stats.csv | cut -d, -f2-4 | tr '\n' ' ')"
done
