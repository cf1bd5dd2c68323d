"""Regenerate tests/golden/*.npz (this container only: needs /root/reference
for oracle/_ref). Inputs are the seeded traces of tests/golden_cases.py;
expected outputs come from the oracle glue over the reference's own libVig.

  python3 tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import golden_cases as G  # noqa: E402


def main():
    for name, (kind, cap, trace) in G.CASES.items():
        fr, ln, dv, now = trace()
        o = G.oracle(name, ref=True)
        assert o.L.orc_impl_name().decode() == "reference", o.L.orc_impl_name()
        out_fr = fr.copy()
        out = o.run(out_fr, ln, dv, now, 64)
        alloc, ts = G.oracle_state(name, o)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), frames=fr,
                            lens=ln, in_dev=dv, now=now, out_dev=out,
                            out_frames=out_fr, alloc=alloc, ts=ts,
                            impl=np.array(o.L.orc_impl_name().decode()))
        print(name, kind, "packets", ln.shape[0], "dropped-or-flooded",
              int((out == dv).sum() + (out == 0xFFFF).sum()), "live", int(alloc.sum()))


if __name__ == "__main__":
    main()
