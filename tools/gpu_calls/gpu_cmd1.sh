set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab gpurun_out/pmc_train
bash tools/ab_lib.sh "rw8 rw4" 2 > gpurun_out/ab/rw.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab/s1-$r.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --streams 2 > gpurun_out/ab/s2-$r.json 2>&1 || exit 1
  IGN_PERSIST_CAP=3 timeout -k 10 200 python bench.py --no-cpu --streams 2 > gpurun_out/ab/s2c3-$r.json 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/pmc_train/sq -o sq --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc_train/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_train/g -o g --output-format csv -- python3 bench.py --train --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc_train/g.log 2>&1
