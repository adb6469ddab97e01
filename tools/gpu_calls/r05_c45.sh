# non-temporal ga (backward) and hs (resident SAVE forward) stores: the --train A/B
set -o pipefail
mkdir -p gpurun_out/c45
bash tools/ab_lib.sh "cur3 nt" 2 --train --steps 10 --warmup 3 > gpurun_out/c45/ab.txt 2>&1 || exit 1
