# round 4, call 21: the fused training readout's tiling dependence (tools/probes/ro_save_probe.py):
# found to come from the layer-2 multiply-add (contracted differently per row tile in the SAVE
# form); with an explicit fma, then the edge-cut training tests
set -o pipefail
timeout -k 10 200 python -u tools/probes/ro_save_probe.py > gpurun_out/ro_save_probe.log 2>&1; grep -v amdgpu.ids gpurun_out/ro_save_probe.log | head -3
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_edge_cut.py > gpurun_out/c21_tests.log 2>&1; tail -2 gpurun_out/c21_tests.log
