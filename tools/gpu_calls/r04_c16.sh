# round 4, call 16: the readout's training path -- the output-layer gradient formed on the fly (no
# row_outer_t, IGN_FUSE_OUTER_BWD) and the training forward on readout_h16 with activation saves
# (IGN_TRAIN_FUSED_READOUT): gradient tests, then the training step A/B; csr_gather_add with eight
# rows in flight against four (library A/B, -DIGN_GATHER4)
set -o pipefail
O=gpurun_out/c16
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_training.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep -E "fused readout" $O/tests.log | head -5
bash tools/ab_env.sh IGN_TRAIN_FUSED_READOUT "1 0" 2 --train --steps 10 --warmup 3 && bash tools/ab_env.sh IGN_FUSE_OUTER_BWD "0" 1 --train --steps 10 --warmup 3 && bash tools/ab_lib.sh "g8 g4" 2 --train --steps 10 --warmup 3
