"""Per-step kernel breakdown of a tools/train_prof.sh run (rocprofv3 kernel trace).
Usage: python tools/train_breakdown.py gpurun_out/prof_train [steps]"""
import collections
import csv
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_train"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = list(csv.DictReader(open(os.path.join(d, "train_kernel_trace.csv"))))
by = collections.defaultdict(list)
for x in rows:
    name = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    key = (name[:48], x["Grid_Size_X"], x["Grid_Size_Y"], x["Workgroup_Size_X"])
    by[key].append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in by.values())
print(f"total {tot / steps / 1e3:.2f} ms/step over {steps} steps (incl. warmup)")
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:16]:
    print(f"{k[0]:48s} grid {k[1]:>8s}x{k[2]:<2s} wg {k[3]:>4s} {len(v):4d} calls {sum(v) / steps:9.1f} us/step {sum(v) / len(v):8.1f} us")
