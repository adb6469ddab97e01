"""Per-kernel average of rocprofv3 --pmc counters: python tools/pmc_by_kernel.py <counter_collection.csv> [n]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 12
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
key = lambda k: -max(agg[k].get("SQ_WAVE_CYCLES", 0), agg[k].get("GRBM_GUI_ACTIVE", 0))
for k in sorted(agg, key=key)[:n_show]:
    n = len(disp[k])
    print("%-48s n=%-3d " % (k, n) + " ".join("%s=%.3g" % (c, x / n) for c, x in sorted(agg[k].items())))
