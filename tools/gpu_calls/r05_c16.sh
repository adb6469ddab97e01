# round-5 profiles: headline and Q-size (trace + PMC passes), phase stamps, full-batch precision numbers
set -o pipefail
bash profiles/collect.sh r05_rn || exit 1
TRACE_ARGS="--model qsize --no-edge-cut" BENCH_ARGS="--model qsize --steps 3 --warmup 1 --no-cpu --no-edge-cut" bash profiles/collect.sh r05_qs || exit 1
for m in routenet qsize; do
  MODEL=$m TOPO=synth50 GRAPHS=256 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so \
    timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/prof_r05_rn/stamps_$m.json 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -s -v --timeout 500 --timeout-method thread -k precision > gpurun_out/prof_r05_rn/precision.log 2>&1 || exit 1
