"""round 5 session i (diagnostics): the wide-slot golden case through the
unsorted new-key path vs the sorted one; prints the first mismatches with
their packet kind, expected and got ports."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_cases as G
from gpuh import run_gpu

g = G.load("nat_wide")
fr, ln, dv, now = G.wide_trace()
S = G.WIDE_SLOT
nat = G.wide_gpu()
outs = []
for a, b in ((0, 1500), (1500, G.WIDE_N)):
    f, o = run_gpu(nat, fr[a * S:b * S], ln[a:b], dv[a:b], now[a:b], S)
    outs.append(o)
out = np.concatenate(outs)
bad = np.nonzero(out != g["out_dev"])[0]
print("mismatches", bad.size, "first", bad[:20].tolist())
for p in bad[:12]:
    print(p, "in", int(dv[p]), "len", int(ln[p]), "exp", int(g["out_dev"][p]), "got", int(out[p]),
          "now", int(now[p]))
alloc, ts, _ = nat.dump()
print("alloc diff", int((alloc != g["alloc"]).sum()), "live", int(alloc.sum()), int(g["alloc"].sum()))
