"""Record a profiles/collect.sh run: copy the rocprofv3 kernel stats and the PMC summary into
profiles/<round>/<workload>/ and set profiles/traffic.json[workload] (HBM bytes per launch).
Usage: python profiles/update_traffic.py gpurun_out/prof_<tag> <workload> <round>"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import summarize  # noqa: E402


def main(prof_dir, workload, rnd):
    dst = os.path.join(HERE, rnd, workload)
    os.makedirs(dst, exist_ok=True)
    summary = os.path.join(dst, "pmc_summary.json")
    summarize.main(prof_dir, summary)
    stats = os.path.join(prof_dir, "trace", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    res = json.load(open(summary))
    path = os.path.join(HERE, "traffic.json")
    traffic = json.load(open(path)) if os.path.exists(path) else {}
    entry = {}
    for kind, r in res.items():
        if kind == "by_name" or "hbm_bytes_per_launch" not in r:
            continue
        entry[kind] = {"hbm_bytes_per_launch": r["hbm_bytes_per_launch"], "fetch_size_kib": r["FETCH_SIZE"],
                       "write_size_kib": r["WRITE_SIZE"], "avg_ms_rocprof": r.get("avg_ms"),
                       "note": "FETCH_SIZE x2 (gfx950 half-count of wide streams, MI355X_MICROARCH.md HBM) + "
                               "WRITE_SIZE; per launch; profiles/collect.sh run %s" % os.path.basename(prof_dir)}
    traffic[workload] = entry
    with open(path, "w") as fh:
        json.dump(traffic, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:4])
