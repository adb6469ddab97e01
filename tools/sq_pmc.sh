#!/bin/bash
# SQ counter passes of a short bench run (GPU box, repo root):  tools/sq_pmc.sh TAG [bench args]
# Environment (IGN_*) is inherited, so kernel variants can be compared.  Two passes (8 SQ slots
# each), then profiles/summarize.py-style per-kernel averages in gpurun_out/pmc_TAG/summary.json.
set -o pipefail
TAG=$1; shift
ARGS=${*:-"--steps 3 --warmup 1 --no-cpu --no-edge-cut"}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $OUT/sq -o sq --output-format csv -- \
  python3 bench.py $ARGS > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_ACTIVE_INST_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/sq2 -o sq2 --output-format csv -- \
  python3 bench.py $ARGS > $OUT/sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 $OUT/sq2.log; }
python3 profiles/summarize.py $OUT > $OUT/summary.json
echo "pmc $TAG done"
