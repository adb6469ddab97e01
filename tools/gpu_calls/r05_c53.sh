# training step per-dispatch kernel trace (which csr_gather_add calls cost what)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c53
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c53/prof -o run -- python3 -u bench.py --no-cpu --no-edge-cut --train --steps 3 --warmup 2 > gpurun_out/c53/bench.log 2>&1 || { tail -20 gpurun_out/c53/bench.log; exit 1; }
f=$(find gpurun_out/c53/prof -name '*kernel_trace.csv' | head -1)
python3 - "$f" > gpurun_out/c53/gather_calls.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if "csr_gather_add" in r["Kernel_Name"] or "seq_gru_bwd" in r["Kernel_Name"] or "sum_gru_bwd" in r["Kernel_Name"] or "row_gemm_t" in r["Kernel_Name"]]
for r in sel[-60:]:
    print("%-40s grid %-10s %8.1f us" % (r["Kernel_Name"][:40], r.get("Grid_Size", r.get("Grid_Size_X", "")), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
cat gpurun_out/c53/gather_calls.txt
rm -rf gpurun_out/c53/prof
