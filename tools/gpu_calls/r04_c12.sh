# round 4, call 12: resident forward with phase B over all 16 waves (B1 sums / B2 GRU step / B3
# projection, local CSR in LDS) and the next-tile header prefetch: parity, GEANT2 / NSFNET bench, stamps
set -o pipefail
O=gpurun_out/c12
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "resident or forward_matches_oracle or fused_projection" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
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
  TOPO=$topo IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 200 python -u tools/probes/res_stamps.py > $O/stamps-$topo.json 2> $O/stamps-$topo.err || { tail -20 $O/stamps-$topo.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/stamps-$topo.json')); print('$topo', d['cycles_per_graph_mean'], d['share_all_waves']); print([round(x) for x in d['A_work_per_wave']]); print([round(x) for x in d['B_work_per_wave']])"
done
