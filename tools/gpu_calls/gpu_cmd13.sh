set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc13
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d gpurun_out/pmc13/a -o a --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/pmc13/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc13/b -o b --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/pmc13/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_SMEM -d gpurun_out/pmc13/c -o c --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/pmc13/c.log 2>&1
