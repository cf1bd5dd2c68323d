"""Per-step kernel timeline of a `rocprofv3 --kernel-trace` run of bench.py:
for the last few steps, every kernel's start offset, the idle gap before it
and its duration (diagnostic; reads the CSV rocprofv3 wrote).

  python3 tools/step_timeline.py <rocprof_dir> [anchor_kernel] [steps]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "nat_classify64"
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    for a, b in zip(idx[-k - 1:-1], idx[-k:]):
        t0 = int(rows[a]["Start_Timestamp"])
        prev = None
        print("--- step")
        for r in rows[a:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev else 0.0
            print("%8.1f gap %6.1f dur %7.1f %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3,
                                                   r["Kernel_Name"][:60]))
            prev = max(prev or e, e)
        print("next step at %.1f us (gap %.1f)" % (
            (int(rows[b]["Start_Timestamp"]) - t0) / 1e3,
            (int(rows[b]["Start_Timestamp"]) - prev) / 1e3))


if __name__ == "__main__":
    main()
