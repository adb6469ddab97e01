set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc19
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc19/f -o f --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc19/f.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc19/w -o w --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc19/w.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d gpurun_out/pmc19/s -o s --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc19/s.log 2>&1
