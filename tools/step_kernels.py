"""Diagnostics: one step of a rocprofv3 kernel trace (csv) as a timeline --
every dispatch between two launches of a marker kernel, with its start
offset, duration and the idle gap before it.

  python3 tools/step_kernels.py TRACE.csv [--marker nat_classify64] [--step -5]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="nat_classify64")  # (prefix: also nat_classify64w)
    ap.add_argument("--step", type=int, default=-5, help="which marker launch (python index)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    i0, i1 = idx[a.step], idx[a.step + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    end, busy, agg = t0, 0.0, {}
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
        print("%8.1f %7.1f gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - end) / 1e3, k))
        busy += (e - s) / 1e3
        agg[k] = agg.get(k, 0.0) + (e - s) / 1e3
        end = max(end, e)
    span = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3
    print("step %.1f us, kernels %.1f us, idle %.1f us" % (span, busy, span - busy))
    for k, v in sorted(agg.items(), key=lambda x: -x[1])[:8]:
        print("  %7.1f  %s" % (v, k))


if __name__ == "__main__":
    main()
