# round 6 call 18: the batch builders' host sections (IGN_BUILD_PROF_FINE=1) with one builder and
# with eight concurrent ones
set -o pipefail
mkdir -p gpurun_out/c18
IGN_BUILD_PROF_FINE=1 REPS=4 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c18/host1.txt 2> gpurun_out/c18/host1.err || exit 1
tail -1 gpurun_out/c18/host1.txt
IGN_BUILD_PROF_FINE=1 REPS=3 THREADS=8 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c18/host8.txt 2> gpurun_out/c18/host8.err || exit 1
tail -1 gpurun_out/c18/host8.txt
grep "fine sections" gpurun_out/c18/host1.err | tail -4
