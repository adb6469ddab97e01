set -o pipefail
bash tools/n2_rehearsal.sh > gpurun_out/n2_rehearsal.log 2>&1 || { cat gpurun_out/n2_rehearsal.log; exit 1; }
cat gpurun_out/n2_rehearsal.log
IGN_DIST_BACKEND=gloo IGN_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/n2_self.log 2>&1 || { tail -30 gpurun_out/n2_self.log; exit 1; }
grep '"metric"' gpurun_out/n2_self.log | tail -1
