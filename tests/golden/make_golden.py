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

    # configs[1] at full size: digest + head/tail frames
    fr, ln, dv, now = G.big_trace()
    o = G.big_oracle(ref=True)
    out = o.run(fr, ln, dv, now, 64)
    dig = G.orc.digest(fr, 64, ln, out, ref=True)
    k = 1024 * 64
    np.savez_compressed(os.path.join(HERE, "nat_1m_digest.npz"),
                        digest=np.array(dig, np.uint64), n=np.array(ln.shape[0]),
                        head_frames=fr[:k], tail_frames=fr[-k:],
                        head_out=out[:1024], tail_out=out[-1024:],
                        live=np.array(o.L.orc_nat_flow_count(o.h)),
                        impl=np.array(o.L.orc_impl_name().decode()))
    print("nat_1m_digest", hex(dig), "live", o.L.orc_nat_flow_count(o.h))


if __name__ == "__main__":
    main()
