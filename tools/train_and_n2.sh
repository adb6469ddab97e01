mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_train.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_train.log; exit 1; }
tail -1 gpurun_out/pytest_train.log
bash tools/n2_rehearsal.sh
