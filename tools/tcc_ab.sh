#!/bin/bash
# L2 (TCC) hit / miss / fabric read requests per launch of one kernel kind, for two values of an
# environment switch (GPU box, repo root):  tools/tcc_ab.sh VAR "v1 v2" KERNEL_REGEX
VAR=$1; VALS=$2; PAT=$3
OUT=gpurun_out/tccab
mkdir -p $OUT
export TMPDIR=/tmp
for v in $VALS; do
  env $VAR=$v timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE \
    -d $OUT/$VAR-$v -o x --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-edge-cut \
    > $OUT/$VAR-$v.log 2>&1 || { echo "pass $v failed"; exit 1; }
done
python3 - "$VAR" "$VALS" "$PAT" <<'PY'
import csv, glob, collections, re, sys
var, vals, pat = sys.argv[1], sys.argv[2].split(), sys.argv[3]
for v in vals:
    f = glob.glob("gpurun_out/tccab/%s-%s/**/*counter_collection.csv" % (var, v), recursive=True)[0]
    acc = collections.defaultdict(float); n = set()
    for r in csv.DictReader(open(f)):
        if re.search(pat, r["Kernel_Name"]):
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r.get("Dispatch_Id", ""))
    print(var, v, {k: round(x / max(1, len(n))) for k, x in acc.items()})
PY
