set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || true
BENCH_ARGS="--steps 3 --warmup 1 --no-cpu" bash profiles/collect.sh r03s2 || exit 1
mkdir -p gpurun_out/pmc_ro
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_ro/a -o a --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/pmc_ro/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_ro/b -o b --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/pmc_ro/b.log 2>&1
