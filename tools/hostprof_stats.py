"""Summarise VIGPATH_HOSTPROF=2 records (vp_runtime.hip: per call, absolute
steady-clock stage times printed at exit) from a log: median microseconds of
the classify launch call (s1 -> s2), the fold launch call (s2 -> s3), the
control block seen -> the next call's classify issued, and the call period.
Usage: python3 tools/hostprof_stats.py LOG [first_call last_call]"""
import statistics as st
import sys


def load(path):
    hp = []
    for line in open(path):
        if line.startswith("vigpath hostprof abs"):
            hp.append([float(x) for x in line.split(":")[1].split("(")[0].split()])
    return hp


def summary(hp, a=3, b=None):
    b = b or len(hp) - 1
    def med(f):
        xs = [f(i) for i in range(a, b)]
        return round(st.median(xs), 2) if xs else None
    return {"calls": b - a,
            "launch_classify_us": med(lambda i: hp[i][2] - hp[i][1]),
            "launch_fold_us": med(lambda i: hp[i][3] - hp[i][2]),
            "seen_to_next_issue_us": med(lambda i: hp[i + 1][2] - hp[i][4]),
            "period_us": med(lambda i: hp[i + 1][0] - hp[i][0])}


if __name__ == "__main__":
    hp = load(sys.argv[1])
    a = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    b = int(sys.argv[3]) if len(sys.argv) > 3 else min(len(hp) - 1, a + 18)
    print(summary(hp, a, b))
