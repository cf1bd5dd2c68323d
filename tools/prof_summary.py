"""Summarise rocprofv3 CSV output of a bench run into profiles/ JSON.

  python3 tools/prof_summary.py trace <rocprof_dir> <out.json> [--skip N]
      --kernel-trace --stats run: per-launch durations of every vp:: kernel,
      the average over launches after the first N of each kernel (warm-up),
      and the stats table rocprofv3 itself wrote.
  python3 tools/prof_summary.py pmc <out.json> <packets_per_launch> <dir>...
      --pmc passes (FETCH_SIZE in one, WRITE_SIZE in another): per-launch
      counter values of nat_classify64 and the corrected bytes per launch and
      per packet (MI355X_MICROARCH.md HBM section: FETCH_SIZE x2 on gfx950).

Diagnostic tooling; the numbers it writes are what bench.py's
roofline.traffic reads (profiles/<round>_bench_traffic.json).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys

KERNEL = os.environ.get("PROF_KERNEL", "nat_classify64w")
# PROF_LAUNCHES=a:b: only launches a..b-1 of each kernel, in dispatch order
# (one workload's launches when a bench run holds several: bench.py's
# headline comes first, its extras after it)
_LR = os.environ.get("PROF_LAUNCHES")
LAUNCHES = slice(*[int(x) if x else None for x in _LR.split(":")]) if _LR else None


def _rows(d, suffix):
    out = []
    for p in sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)):
        with open(p, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def _short(name):
    s = name.split("(")[0]
    if s.startswith("void "):
        s = s[5:]
    return s


def trace(d, out, skip):
    per = {}
    for r in _rows(d, "kernel_trace.csv"):
        name = _short(_col(r, "Kernel_Name", "Kernel-Name", "KernelName"))
        t0 = int(_col(r, "Start_Timestamp", "Start-Timestamp"))
        t1 = int(_col(r, "End_Timestamp", "End-Timestamp"))
        per.setdefault(name, []).append((t0, (t1 - t0) / 1e3))
    kernels = {}
    for name, v in sorted(per.items()):
        v.sort()
        us = [round(x, 3) for _, x in v]
        if LAUNCHES is not None:
            us = us[LAUNCHES]
        tail = us[skip:] if len(us) > skip else us
        kernels[name] = {"launches": len(us), "us_all_launches": us[:64],
                         "us_avg_after_warmup": round(statistics.mean(tail), 3)
                         if tail else None}
    stats = _rows(d, "kernel_stats.csv")
    res = {"source": "rocprofv3 --kernel-trace --stats --output-format csv",
           "skip_first_launches_per_kernel": skip,
           "kernels": kernels, "rocprof_stats": stats}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    k = [n for n in kernels if _is_kernel(n)]
    if k:
        print("%s avg %.1f us over timed launches" %
              (k[0], kernels[k[0]]["us_avg_after_warmup"]))


def _is_kernel(name):
    """The kernel of interest, template arguments aside
    (vp::nat_classify_wide<16u> for PROF_KERNEL=nat_classify_wide)."""
    return name.endswith(KERNEL) or name.split("<")[0].endswith(KERNEL)


def pmc(out, pkts, dirs):
    vals = {}
    for d in dirs:
        for r in _rows(d, "counter_collection.csv"):
            name = _short(_col(r, "Kernel_Name", "Kernel-Name", "KernelName"))
            if not _is_kernel(name):
                continue
            c = _col(r, "Counter_Name", "Counter-Name")
            disp = int(_col(r, "Dispatch_Id", "Dispatch-Id", "Correlation_Id"))
            vals.setdefault(c, {}).setdefault(disp, 0.0)
            vals[c][disp] += float(_col(r, "Counter_Value", "Counter-Value"))
    launches = {c: [round(v[k], 2) for k in sorted(v)] for c, v in vals.items()}
    if LAUNCHES is not None:
        launches = {c: v[LAUNCHES] for c, v in launches.items()}
    res = {"kernel": "vp::" + KERNEL, "packets_per_launch": pkts,
           "launches": launches, "launch_range": _LR}
    med = {c: statistics.median(v if LAUNCHES is not None or len(v) < 2 else v[1:])
           for c, v in launches.items()}
    for c, m in med.items():
        res[c + "_median"] = m
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        fb = 2 * med["FETCH_SIZE"] * 1024
        wb = med["WRITE_SIZE"] * 1024
        res.update({"FETCH_SIZE_kB": med["FETCH_SIZE"],
                    "WRITE_SIZE_kB": med["WRITE_SIZE"],
                    "fetch_bytes_corrected": fb, "write_bytes": wb,
                    "traffic_bytes_per_launch": fb + wb,
                    "traffic_bytes_per_packet": round((fb + wb) / pkts, 2),
                    "correction": "MI355X_MICROARCH.md HBM section: FETCH_SIZE "
                                  "x2 on gfx950 (wide coalesced reads tallied "
                                  "at half), WRITE_SIZE as is; counters in kB; "
                                  "Infinity-Cache hits are included"})
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "launches"}))


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 3
        trace(sys.argv[2], sys.argv[3], skip)
    elif sys.argv[1] == "pmc":
        pmc(sys.argv[2], int(sys.argv[3]), sys.argv[4:])
    else:
        raise SystemExit(__doc__)
