# round 4, call 20: the edge-cut training test with the fused training readout off / on
set -o pipefail
IGN_TRAIN_FUSED_READOUT=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dp.py -k edge_cut_training > gpurun_out/dp_nofuse.log 2>&1; tail -2 gpurun_out/dp_nofuse.log
IGN_TRAIN_FUSED_READOUT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dp.py -k edge_cut_training > gpurun_out/dp_fuse.log 2>&1; tail -2 gpurun_out/dp_fuse.log
