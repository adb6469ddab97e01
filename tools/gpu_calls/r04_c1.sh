# round 4, call 1: default bench line with the edge-cut leg; N=2 gloo rehearsal on one GPU;
# rocprofv3 traces + PMC of Q-size and GEANT2 x512
set -o pipefail
O=gpurun_out/c1
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
echo "default done"
IGN_DIST_BACKEND=gloo IGN_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu --steps 5 --warmup 2 \
  > $O/n2_gloo.json 2> $O/n2_gloo.err || { tail -20 $O/n2_gloo.err; exit 1; }
echo "n2 done"
for spec in "qsize|--model qsize" "qsize_s1|--model qsize --streams 1" "geant2|--topology geant2" \
            "geant2_s1|--topology geant2 --streams 1"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr_$name -o tr --output-format csv -- \
    python3 bench.py $args --no-cpu --no-edge-cut --steps 10 --warmup 2 > $O/tr_$name.log 2>&1 || { tail -20 $O/tr_$name.log; exit 1; }
  echo "trace $name done"
done
BENCH_ARGS="--model qsize --no-cpu --no-edge-cut --steps 3 --warmup 1" TRACE_ARGS="--model qsize --no-cpu --no-edge-cut" \
  bash profiles/collect.sh r04_qsize || exit 1
BENCH_ARGS="--topology geant2 --no-cpu --no-edge-cut --steps 3 --warmup 1" TRACE_ARGS="--topology geant2 --no-cpu --no-edge-cut" \
  bash profiles/collect.sh r04_geant2 || exit 1
IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_stamp.so timeout -k 10 200 python -u tools/probes/seq_stamps.py \
  > $O/seq_stamps.json 2> $O/seq_stamps.err || { tail -20 $O/seq_stamps.err; exit 1; }
echo "stamps done"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "windowed" \
  > $O/test_windowed.log 2>&1 || { tail -30 $O/test_windowed.log; exit 1; }
echo "windowed tests done"
for w in 1 2 0 1 2; do
  IGN_SUM_WINDOW=$w timeout -k 10 200 python -u bench.py --model qsize --no-cpu --no-edge-cut --steps 20 \
    > $O/qsize_win$w.json 2> $O/qsize_win$w.err || { tail -20 $O/qsize_win$w.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/qsize_win$w.json').read().splitlines()[-1]); print('win $w', round(d['ms_per_step'],4), {k: round(v['ms_total']/max(1,v['launches']),4) for k,v in d['roofline']['warmup_kernels'].items()})"
done
