# round 4, call 5: what the ordered backward's time is made of (timing-only ablations, wrong gradients):
# bnodu = no dU contraction (48 f32 MFMAs per tile-step), bnoga = no ga stores; base = the default tree
set -o pipefail
O=gpurun_out/c5
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for n in base bnodu bnoga; do
  rm -rf $O/prof_$n
  IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o train \
    --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --no-cpu --no-edge-cut > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "== $n (rep $r): $(tail -1 $O/$n.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],3), "ms/step")')"
  python3 tools/train_breakdown.py $O/prof_$n 4 | head -5
done
done
