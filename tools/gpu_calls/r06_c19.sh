# round 6 call 19: the message lists' fast path in ign_batch_create: parity suite (every batch build
# goes through it), then the builders' host sections with one and eight builders
set -o pipefail
mkdir -p gpurun_out/c19
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c19/pytest.log 2>&1 || { tail -30 gpurun_out/c19/pytest.log; exit 1; }
tail -1 gpurun_out/c19/pytest.log
IGN_BUILD_PROF_FINE=1 REPS=4 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c19/host1.txt 2> gpurun_out/c19/host1.err || exit 1
tail -1 gpurun_out/c19/host1.txt
REPS=3 THREADS=8 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c19/host8.txt 2> gpurun_out/c19/host8.err || exit 1
tail -1 gpurun_out/c19/host8.txt
grep "fine sections" gpurun_out/c19/host1.err | tail -4
