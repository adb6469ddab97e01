# round 4, call 29: kernel trace + PMC passes of the headline on the final tree (profiles/collect.sh),
# and the bench line of the same command without the profiler
set -o pipefail
bash profiles/collect.sh r04_headline_final &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-edge-cut > gpurun_out/prof_r04_headline_final/bench_line.json 2> /dev/null &&
tail -1 gpurun_out/prof_r04_headline_final/bench_line.json | cut -c1-300
