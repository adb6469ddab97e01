# round 6 call 22: the box's host topology as this process sees it (CPUs granted, NUMA nodes), and
# one builder's host sections with its thread pinned to one CPU vs free to migrate
set -o pipefail
mkdir -p gpurun_out/c22
{ python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a)"
  for n in /sys/devices/system/node/node*/cpulist; do echo "$n $(cat $n)"; done
  grep -m1 "model name" /proc/cpuinfo; nproc; cat /sys/kernel/mm/transparent_hugepage/enabled || true
} > gpurun_out/c22/topo.txt 2>&1
cat gpurun_out/c22/topo.txt | cut -c1-300
IGN_BUILD_PROF_FINE=1 REPS=5 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c22/free.txt 2> gpurun_out/c22/free.err || exit 1
tail -1 gpurun_out/c22/free.txt; grep "create fine" gpurun_out/c22/free.err | cut -c1-90
PIN=1 IGN_BUILD_PROF_FINE=1 REPS=5 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c22/pin.txt 2> gpurun_out/c22/pin.err || exit 1
tail -1 gpurun_out/c22/pin.txt; grep "create fine" gpurun_out/c22/pin.err | cut -c1-90
