# GEANT2 x512: 8-wave resident workgroups at <= 128 VGPRs (two per CU where LDS allows) vs 16; all-LDS vs path-global form
set -o pipefail
mkdir -p gpurun_out/c41
bash tools/ab_lib.sh "base3 w8lb" 2 --topology geant2 > gpurun_out/c41/ab_default.txt 2>&1 || exit 1
IGN_RESIDENT=2 bash tools/ab_lib.sh "base3 w8lb" 2 --topology geant2 > gpurun_out/c41/ab_pg.txt 2>&1 || exit 1
IGN_RESIDENT=2 timeout -k 10 200 python -u bench.py --topology geant2 --no-cpu --no-edge-cut --steps 5 > gpurun_out/c41/pg_line.json 2>/dev/null || exit 1
