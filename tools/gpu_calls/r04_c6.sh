# round 4, call 6: the fused projection for multi-source ordered MPs (Q-size's {link, node} -> path
# interleave): parity tests, Q-size A/B of IGN_FUSE_PROJ
set -o pipefail
O=gpurun_out/c6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread \
  > $O/test_parity.log 2>&1 || { tail -30 $O/test_parity.log; exit 1; }
tail -2 $O/test_parity.log
bash tools/ab_env.sh IGN_FUSE_PROJ "1 0" 3 --model qsize --steps 20 > $O/ab_fuse_qsize.log 2>&1 || { tail -20 $O/ab_fuse_qsize.log; exit 1; }
cat $O/ab_fuse_qsize.log
