"""Regenerate tests/golden/*.npz (this container only: needs /root/reference
for oracle/_ref). Inputs are the seeded traces of tests/golden_cases.py;
expected outputs come from the oracle glue over the reference's own libVig.

  python3 tests/golden/make_golden.py          (all)
  python3 tests/golden/make_golden.py --wide   (nat_wide.npz only)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import golden_cases as G  # noqa: E402
from vigor_amd import traces as T  # noqa: E402


def wide():
    """nat_wide.npz: 1518-byte frames in 2048-byte slots (golden_cases)."""
    fr, ln, dv, now = G.wide_trace()
    o = G.wide_oracle(ref=True)
    assert o.L.orc_impl_name().decode() == "reference", o.L.orc_impl_name()
    out_fr = fr.copy()
    out = o.run(out_fr, ln, dv, now, G.WIDE_SLOT)
    alloc, ts, _ = o.nat_dump(G.WIDE_CAP)
    np.savez_compressed(os.path.join(HERE, "nat_wide.npz"),
                        in_hash=G.slot_hashes(fr, G.WIDE_SLOT), out_dev=out,
                        out_hash=G.slot_hashes(out_fr, G.WIDE_SLOT), alloc=alloc,
                        ts=np.where(alloc == 1, ts, 0),
                        impl=np.array(o.L.orc_impl_name().decode()))
    print("nat_wide packets", ln.shape[0], "max len", int(ln.max()), "dropped",
          int((out == dv).sum()), "live", int(alloc.sum()))


def main():
    if sys.argv[1:] == ["--wide"]:
        return wide()
    wide()
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

    # the bench's shape: 1M flows, 2^24-packet batches (bench.py)
    o = G.nat_oracle(G.BENCH_FLOWS, ref=True)
    digs = []
    for k in range(G.BENCH_BATCHES):
        acc = [0]

        def add(p0, fr, out, k=k, acc=acc):
            acc[0] += T.batch_digest(fr, out, 64, p0 - k * G.BENCH_BATCH)
        G.run_oracle_chunks(o, G.BENCH_BATCH, G.BENCH_FLOWS, k * G.BENCH_BATCH, add)
        digs.append(acc[0] % (1 << 64))
    alloc, ts, _ = o.nat_dump(G.BENCH_FLOWS)
    sd = T.state_digest(alloc, ts)
    np.savez_compressed(os.path.join(HERE, "nat_bench_shape.npz"),
                        batch_digest=np.array(digs, np.uint64),
                        state_digest=np.array(sd, np.uint64),
                        live=np.array(o.L.orc_nat_flow_count(o.h)),
                        impl=np.array(o.L.orc_impl_name().decode()))
    print("nat_bench_shape", [hex(d) for d in digs], hex(sd))

    # configs[4] at full table size: 16M flows
    o = G.nat_oracle(G.F16M_FLOWS, ref=True)
    acc = [0]
    ends = {}

    def add16(p0, fr, out):
        acc[0] += T.batch_digest(fr, out, 64, p0)
        if p0 == 0:
            ends["head_frames"], ends["head_out"] = fr[:1024 * 64].copy(), out[:1024].copy()
        if p0 + out.shape[0] == G.F16M_PACKETS:
            ends["tail_frames"], ends["tail_out"] = fr[-1024 * 64:].copy(), out[-1024:].copy()
    G.run_oracle_chunks(o, G.F16M_PACKETS, G.F16M_FLOWS, 0, add16)
    alloc, ts, _ = o.nat_dump(G.F16M_FLOWS)
    sd = T.state_digest(alloc, ts)
    np.savez_compressed(os.path.join(HERE, "nat_16m_digest.npz"),
                        digest=np.array(acc[0] % (1 << 64), np.uint64),
                        state_digest=np.array(sd, np.uint64),
                        live=np.array(o.L.orc_nat_flow_count(o.h)),
                        impl=np.array(o.L.orc_impl_name().decode()), **ends)
    print("nat_16m_digest", hex(acc[0] % (1 << 64)), hex(sd))


if __name__ == "__main__":
    main()
