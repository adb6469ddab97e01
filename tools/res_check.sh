#!/bin/bash
# The resident forward on the GPU box: parity tests, GEANT2 / NSFNET x512 bench lines (2 and 4
# streams) and, when ignnition_amd/ab/lib_rstamp.so exists (tools/build_ab.sh rstamp -DIGN_RES_STAMP),
# the phase stamps.  res_check.sh OUTDIR
set -o pipefail
O=${1:-gpurun_out/res}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "resident or forward_matches_oracle or fused_projection" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for topo in geant2 nsfnet; do
  for s in 2 4; do
    f=$O/$topo-s$s
    timeout -k 10 200 python -u bench.py --no-cpu --no-edge-cut --topology $topo --streams $s > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 - $f.json "$topo s$s" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], r["kernel"], "avg %.4f" % r["avg_launch_ms"],
      " ".join("%s %.4f" % (k, v["ms_total"] / max(1, v["launches"])) for k, v in r["warmup_kernels"].items()))
PY
  done
  if [ -f ignnition_amd/ab/lib_rstamp.so ]; then
    TOPO=$topo IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 200 python -u tools/probes/res_stamps.py > $O/stamps-$topo.json 2> $O/stamps-$topo.err || { tail -20 $O/stamps-$topo.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/stamps-$topo.json')); print('$topo', d['cycles_per_graph_mean'], {k: round(v) for k, v in d['per_wave_mean_cycles'].items()}); print([round(x) for x in d['A_work_per_wave']]); print([round(x) for x in d['B_work_per_wave']])"
  fi
done
