# z / r accumulators seeded with the projected rows (frees 16 VGPRs in the gates): stamps + bench A/B
set -o pipefail
mkdir -p gpurun_out/c10
MODEL=routenet TOPO=synth50 GRAPHS=256 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_seedxst.so \
  timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/c10/seedxst.json 2> gpurun_out/c10/seedxst.err || exit 1
bash tools/ab_lib.sh "base seedx" 3 > gpurun_out/c10/ab.txt 2>&1 || exit 1
# the fresh-batch training input pipeline, per stage
THREADS=1 REPS=3 timeout -k 10 300 python -u tools/host_pipeline_profile.py 512 > gpurun_out/c10/host_t1.txt 2>&1 || exit 1
THREADS=8 REPS=2 timeout -k 10 300 python -u tools/host_pipeline_profile.py 512 > gpurun_out/c10/host_t8.txt 2>&1 || exit 1
nproc > gpurun_out/c10/nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/c10/nproc.txt
# Q-size on the resident form: sub-batch streams 1 / 2 / 4
for s in 1 2 4; do
  timeout -k 10 200 python -u bench.py --model qsize --no-cpu --no-edge-cut --streams $s > gpurun_out/c10/qsize_s$s.json 2> gpurun_out/c10/qsize_s$s.err || exit 1
done
