# weight-gradient contractions: rows per chunk 256 / 128 / 64 (more waves for the small-M ones)
set -o pipefail
mkdir -p gpurun_out/c40
bash tools/ab_env.sh IGN_TS_MIN_ROWS "256 128 64" 2 --train --steps 10 --warmup 3 > gpurun_out/c40/ab.txt 2>&1 || exit 1
