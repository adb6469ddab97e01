mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 120 --timeout-method thread -k "sum_update or synthetic" > gpurun_out/pt_sum.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pt_sum.log; exit 1; }
grep -E "passed|failed|max scaled" gpurun_out/pt_sum.log
for v in 3 7; do
  IGN_SUM_VARIANT=$v timeout -k 10 300 python bench.py --model synthetic --steps 10 --warmup 2 --no-cpu > gpurun_out/bsyn_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bsyn_$v.log; exit 1; }
  tail -1 gpurun_out/bsyn_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], r.get('mfma_frac_alg'))"
done
