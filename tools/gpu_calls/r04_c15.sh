# round 4, call 15: resident forward, phase A tiles claimed from an LDS counter (longest first)
# against the static wave -> tile map (-DIGN_RES_STATIC): parity, bench, stamps, interleaved A/B
set -o pipefail
bash tools/res_check.sh gpurun_out/c15 && bash tools/ab_lib.sh "rdyn rstatic" 3 --topology geant2 --streams 2
