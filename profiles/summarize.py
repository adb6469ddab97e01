"""Summarise a profiles/collect.sh run: per-kernel average duration (kernel trace) and per-launch
PMC values.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a wide
coalesced stream on gfx950 -> reported raw and x2-corrected; WRITE_SIZE is exact for 16-B stores.
FETCH_SIZE / WRITE_SIZE are in KiB.  Usage: python profiles/summarize.py gpurun_out/prof_r01 [out.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

import re

# first match wins: the training kernels before the forward ones whose names they extend
KINDS = {"mp_resident": r"resident_forward_kernel",
         "seq_gru_bwd": r"seq_gru_bwd_kernel", "sum_gru_bwd": r"sum_gru_bwd_kernel",
         "csr_gather_add": r"csr_gather_add_kernel", "dense_bf": r"dense_bf_kernel", "tsgemm_bf": r"tsgemm_bf_kernel",
         "seq_gru": r"seq_gru\w*_kernel", "sum_gru": r"sum_gru\w*_kernel", "readout": r"readout\w*_kernel",
         "project": r"project_kernel", "init_state": r"init_state_kernel"}


def kind_of(name):
    for k, pat in KINDS.items():
        if re.search(pat, name):
            return k
    return None


def main(d, out=None):
    res = defaultdict(dict)
    tr = glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        dur = defaultdict(list)
        for row in csv.DictReader(open(tr[0])):
            k = kind_of(row["Kernel_Name"])
            if k:
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
        for k, v in dur.items():
            res[k]["launches"] = len(v)
            res[k]["avg_ms"] = sum(v) / len(v)
        # per kernel instance (template arguments included): kinds with several kernels (a sum MP
        # on the windowed / segmented path, the 32- and 64-wide sum updates) split apart
        byname = defaultdict(list)
        for row in csv.DictReader(open(tr[0])):
            if kind_of(row["Kernel_Name"]) or "sum_win" in row["Kernel_Name"] or "sum_seg" in row["Kernel_Name"]:
                byname[row["Kernel_Name"].split("(")[0]].append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
        res["by_name"] = {n: {"launches": len(v), "avg_ms": sum(v) / len(v), "total_ms": sum(v)}
                          for n, v in sorted(byname.items(), key=lambda kv: -sum(kv[1]))}
    for p in ("fetch", "write", "sq", "sq2", "tcc"):
        fs = glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        acc = defaultdict(lambda: defaultdict(float))
        cnt = defaultdict(set)
        for row in csv.DictReader(open(fs[0])):
            k = kind_of(row["Kernel_Name"])
            if not k:
                continue
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            cnt[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
        for k in acc:
            n = max(len(cnt[k]), 1)
            for c, v in acc[k].items():
                res[k][c] = v / n
    for k, r in res.items():
        if "FETCH_SIZE" in r:
            r["hbm_read_bytes_raw"] = r["FETCH_SIZE"] * 1024
            r["hbm_read_bytes_corrected"] = r["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in r:
            r["hbm_write_bytes"] = r["WRITE_SIZE"] * 1024
        if "hbm_read_bytes_corrected" in r and "hbm_write_bytes" in r:
            r["hbm_bytes_per_launch"] = r["hbm_read_bytes_corrected"] + r["hbm_write_bytes"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in r and "GRBM_GUI_ACTIVE" in r:
            pass
    text = json.dumps(res, indent=1, sort_keys=True)
    print(text)
    if out:
        with open(out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
