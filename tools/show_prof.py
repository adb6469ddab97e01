"""Per-step kernel time table from a rocprofv3 --stats csv: python tools/show_prof.py <dir> <steps incl. warmup>"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
print("total per step %.2f ms" % (sum(float(r["TotalDurationNs"]) for r in rows) / steps / 1e6))
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 16]:
    print("%-72s %5s %9.3f ms/step %8.3f ms avg" % (r["Name"][:72], r["Calls"], float(r["TotalDurationNs"]) / steps / 1e6,
                                                  float(r["AverageNs"]) / 1e6))
