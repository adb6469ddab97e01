# round 6 call 27: the ordered backward's ga rows stored in the transposed CSR's order (the gather
# reads each source row's rows in sequence): training tests (bitwise against by-step rows and the
# host CSRs), then the training step and its kernels with IGN_TRAIN_GA_ROW 1 / 0 interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c27
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c27/train_tests.log 2>&1 || { tail -30 gpurun_out/c27/train_tests.log; exit 1; }
tail -1 gpurun_out/c27/train_tests.log
for n in row1 step1 row2 step2; do
  e="IGN_TRAIN_GA_ROW=1"; case $n in step*) e="IGN_TRAIN_GA_ROW=0";; esac
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c27/$n -o $n --output-format csv -- \
    python3 bench.py --train --steps 20 --warmup 3 > gpurun_out/c27/$n.json 2> gpurun_out/c27/$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c27/$n.json) $(grep -h 'seq_gru_bwd\|csr_gather_add_kernel<1, true>' gpurun_out/c27/$n/${n}_kernel_stats.csv | cut -d, -f3-4 | tr '\n' ' ')"
done
