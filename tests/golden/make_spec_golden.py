"""Fixtures from the reference's own NF specifications (this container only:
reads /root/reference/{vignat,vigfw,vigbridge,vigpol,viglb}/spec.py; viglb's
CHT comes from the reference's own cht_fill_cht in oracle/_ref).

For each NF a seeded churn trace (new flows, hits, WAN replies right and
wrong, non-IPv4 and non-TCP/UDP frames, a full table, expiry) is run through
the executable spec model (spec_model.py) packet by packet; the fields the
spec determines are stored per packet:

  out      output device, -1 = dropped (the NF's encoding: out == in_dev);
           vigbridge's two-port broadcast [1 - in] is the NF's flood
  fields   vignat: IPv4 src, IPv4 dst, L4 src port, L4 dst port of the
           forwarded frame, as the NF's structs hold them (raw LE loads)
           vigfw / vigbridge: the forwarded IPv4 / Ethernet headers are the
           received ones (the specs rewrite only the MACs, left `...`)

The spec leaves the allocated index to the implementation
(`the_index_allocated`): vignat's is observable (the external port), so the
generator takes it from the restated oracle's output for that packet and the
spec then pins everything else; vigfw's and vigbridge's are not observable,
so the model follows libVig's dchain order at the spec's `add` (which
viglb's CHT choice does observe for backends). The restated oracle must agree
with the spec on every packet here (asserted), and tests/test_spec.py /
tests/test_spec_gpu.py check the oracle and the GPU path against the stored
fixtures (where the reference is absent).

  python3 tests/golden/make_spec_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import spec_model as S  # noqa: E402
import spec_cases as C  # noqa: E402

REF = os.environ.get("VIGOR_REF", "/root/reference")


def _le16(b, o):
    return int(b[o]) | (int(b[o + 1]) << 8)


def _le32(b, o):
    return int(b[o]) | (int(b[o + 1]) << 8) | (int(b[o + 2]) << 16) | (int(b[o + 3]) << 24)


def spec_nat(fr, ln, dv, now, out_fr, out):
    code = S.compile_spec(open(os.path.join(REF, "vignat", "spec.py")).read())
    em = S.Emap(C.NAT_CAP)
    env = S.base_env()
    env.update(flow_emap=em, ext_ip=C.NAT_EXT_IP, start_port=C.NAT_START_PORT)
    n = ln.shape[0]
    exp_out = np.full(n, -1, np.int32)
    fields = np.zeros((n, 4), np.int64)
    for p in range(n):
        f = fr[p * 64:p * 64 + int(ln[p])].tobytes()
        e = dict(env, now=int(now[p]), received_on_port=int(dv[p]))
        # the implementation's index for a new flow (only read if one is added)
        e["the_index_allocated"] = _le16(out_fr, p * 64 + 34) - C.NAT_START_PORT
        ports, hdrs = S.run_packet(code, e, S.parse(f))
        if ports:
            exp_out[p] = ports[0]
            ip = [h for h in hdrs if h.kind == "ipv4"][0]
            l4 = [h for h in hdrs if h.kind == "tcpudp"][0]
            fields[p] = (ip.saddr, ip.daddr, l4.src_port, l4.dst_port)
    return exp_out, fields


def spec_fw(fr, ln, dv, now):
    code = S.compile_spec(open(os.path.join(REF, "vigfw", "spec.py")).read())
    em = S.Emap(C.FW_CAP)
    vec = S.AutoVector(em)
    env = S.base_env()
    env.update(flow_emap=em, int_devices=vec,
               FlowIdc=S._record("sp", "dp", "sip", "dip", "prot"))
    n = ln.shape[0]
    exp_out = np.full(n, -1, np.int32)
    for p in range(n):
        f = fr[p * 64:p * 64 + int(ln[p])].tobytes()
        e = dict(env, now=int(now[p]), received_on_port=int(dv[p]),
                 the_index_allocated=S.Emap.AUTO)
        ports, _ = S.run_packet(code, e, S.parse(f))
        if ports:
            exp_out[p] = ports[0]
    return exp_out


def spec_bridge(fr, ln, dv, now):
    code = S.compile_spec(open(os.path.join(REF, "vigbridge", "spec.py")).read())
    dyn = S.Emap(C.BRIDGE_CAP)
    stat = S.Emap(1 << 30)  # no static rules in these traces
    vals = S.AutoVector(dyn)
    env = S.base_env()
    env.update(dyn_emap=dyn, stat_emap=stat, dyn_vals=vals,
               DynamicValuec=lambda port: type("DV", (), {"output_port": port})(),
               StaticKeyc=S._record("addr", "device"))
    n = ln.shape[0]
    exp_out = np.full(n, -1, np.int32)
    for p in range(n):
        f = fr[p * 64:p * 64 + int(ln[p])].tobytes()
        e = dict(env, now=int(now[p]), received_on_port=int(dv[p]),
                 the_index_allocated=S.Emap.AUTO)
        ports, _ = S.run_packet(code, e, S.parse(f))
        if ports:
            exp_out[p] = ports[0]
    return exp_out


def spec_pol(fr, ln, dv, now):
    code = S.compile_spec(open(os.path.join(REF, "vigpol", "spec.py")).read())
    em = S.Emap(C.POL_CAP)
    vals = S.AutoVector(em)
    env = S.base_env()
    env.update(flow_emap=em, dyn_vals=vals, ip_addrc=S._record("addr"),
               DynamicValuec=S._record("bucket_size", "bucket_time"))
    n = ln.shape[0]
    exp_out = np.full(n, -1, np.int32)
    for p in range(n):
        f = fr[p * 64:(p + 1) * 64].tobytes()  # (sizes past the slot read as 0)
        f = f + bytes(max(0, int(ln[p]) - 64))
        e = dict(env, now=int(now[p]), received_on_port=int(dv[p]),
                 packet_size=int(ln[p]), the_index_allocated=S.Emap.AUTO)
        ports, _ = S.run_packet(code, e, S.parse(f))
        if ports:
            exp_out[p] = ports[0]
    return exp_out


def reference_cht():
    """The CHT the reference's own cht_fill_cht builds (oracle/_ref)."""
    import orc
    tab = np.zeros(C.LB_HEIGHT * C.LB_BACKENDS, np.uint32)
    mask = np.zeros(C.LB_BACKENDS, np.uint8)
    hs = np.zeros(1, np.uint64)
    ch = np.zeros(1, np.int32)
    P = lambda a: a.ctypes.data  # noqa: E731
    L = orc.lib(ref=True)
    assert L.orc_impl_name().decode() == "reference"
    assert L.orc_test_cht(C.LB_HEIGHT, C.LB_BACKENDS, P(tab), P(mask), 0, P(hs), P(ch))
    return [int(x) for x in tab]


def spec_lb(fr, ln, dv, now):
    code = S.compile_spec(open(os.path.join(REF, "viglb", "spec.py")).read())
    flows = S.Emap(C.LB_CAP)
    bips = S.Emap(C.LB_BACKENDS)
    env = S.base_env()
    env.update(flow_emap=flows, backend_ip_emap=bips, cht=reference_cht(),
               flow_id_to_backend_id=S.AutoVector(flows),
               backends=S.AutoVector(bips),
               LoadBalancedFlowc=S._record("src_ip", "dst_ip", "src_port", "dst_port",
                                           "protocol"),
               LoadBalancedBackendc=S._record("nic", "mac", "ip"),
               ip_addrc=S._record("addr"),
               _LoadBalancedFlow_hash=lambda f: S.struct_hash(*f))
    n = ln.shape[0]
    exp_out = np.full(n, -1, np.int32)
    fields = np.zeros((n, 2), np.int64)  # dst MAC (48 bits), IPv4 dst
    for p in range(n):
        f = fr[p * 64:p * 64 + int(ln[p])].tobytes()
        e = dict(env, now=int(now[p]), received_on_port=int(dv[p]),
                 the_index_allocated=S.Emap.AUTO)
        ports, hdrs = S.run_packet(code, e, S.parse(f))
        if ports:
            exp_out[p] = ports[0]
            eth = [h for h in hdrs if h.kind == "ether"][0]
            ip = [h for h in hdrs if h.kind == "ipv4"][0]
            fields[p] = (int.from_bytes(eth.daddr, "little"), ip.daddr)
    return exp_out, fields


def main():
    # vignat
    fr, ln, dv, now = C.nat_trace()
    o = C.nat_oracle()
    out_fr = fr.copy()
    out = o.run(out_fr, ln, dv, now, 64).astype(np.int32)
    exp_out, fields = spec_nat(fr, ln, dv, now, out_fr, out)
    got = np.where(out == dv, -1, out)
    bad = np.nonzero(got != exp_out)[0]
    assert bad.size == 0, ("nat out", bad[:10], got[bad[:10]], exp_out[bad[:10]])
    fwd = exp_out >= 0
    have = np.array([(_le32(out_fr, p * 64 + 26), _le32(out_fr, p * 64 + 30),
                      _le16(out_fr, p * 64 + 34), _le16(out_fr, p * 64 + 36))
                     for p in range(ln.shape[0])], np.int64)
    assert np.array_equal(have[fwd], fields[fwd]), "nat fields"
    np.savez_compressed(os.path.join(HERE, "spec_nat.npz"), frames=fr, lens=ln,
                        in_dev=dv, now=now, out=exp_out, fields=fields,
                        spec=np.array("vignat/spec.py"))
    print("spec_nat: %d packets, %d forwarded, %d dropped" % (
        ln.shape[0], int(fwd.sum()), int((~fwd).sum())))
    # vigfw
    fr, ln, dv, now = C.fw_trace()
    o = C.fw_oracle()
    out_fr = fr.copy()
    out = o.run(out_fr, ln, dv, now, 64).astype(np.int32)
    exp_out = spec_fw(fr, ln, dv, now)
    got = np.where(out == dv, -1, out)
    bad = np.nonzero(got != exp_out)[0]
    assert bad.size == 0, ("fw out", bad[:10], got[bad[:10]], exp_out[bad[:10]])
    fwd = exp_out >= 0
    for p in np.nonzero(fwd)[0]:  # IPv4 + L4 headers forwarded unchanged
        assert out_fr[p * 64 + 14:p * 64 + 38].tobytes() == fr[p * 64 + 14:p * 64 + 38].tobytes()
    np.savez_compressed(os.path.join(HERE, "spec_fw.npz"), frames=fr, lens=ln,
                        in_dev=dv, now=now, out=exp_out, spec=np.array("vigfw/spec.py"))
    print("spec_fw: %d packets, %d forwarded" % (ln.shape[0], int(fwd.sum())))
    # vigbridge
    fr, ln, dv, now = C.bridge_trace()
    o = C.bridge_oracle()
    out_fr = fr.copy()
    out = o.run(out_fr, ln, dv, now, 64).astype(np.int32)
    exp_out = spec_bridge(fr, ln, dv, now)
    got = np.where(out == dv, -1, np.where(out == 0xFFFF, 1 - dv.astype(np.int32), out))
    bad = np.nonzero(got != exp_out)[0]
    assert bad.size == 0, ("bridge out", bad[:10], got[bad[:10]], exp_out[bad[:10]])
    assert np.array_equal(out_fr, fr), "bridge forwards frames unchanged"
    np.savez_compressed(os.path.join(HERE, "spec_bridge.npz"), frames=fr, lens=ln,
                        in_dev=dv, now=now, out=exp_out,
                        spec=np.array("vigbridge/spec.py"))
    print("spec_bridge: %d packets, %d forwarded" % (ln.shape[0], int((exp_out >= 0).sum())))
    # vigpol
    fr, ln, dv, now = C.pol_trace()
    o = C.pol_oracle()
    out_fr = fr.copy()
    out = o.run(out_fr, ln, dv, now, 64).astype(np.int32)
    exp_out = spec_pol(fr, ln, dv, now)
    got = np.where(out == dv, -1, out)
    bad = np.nonzero(got != exp_out)[0]
    assert bad.size == 0, ("pol out", bad[:10], got[bad[:10]], exp_out[bad[:10]])
    assert np.array_equal(out_fr, fr), "vigpol forwards frames unchanged"
    np.savez_compressed(os.path.join(HERE, "spec_pol.npz"), frames=fr, lens=ln,
                        in_dev=dv, now=now, out=exp_out, spec=np.array("vigpol/spec.py"))
    print("spec_pol: %d packets, %d forwarded" % (ln.shape[0], int((exp_out >= 0).sum())))
    # viglb
    fr, ln, dv, now = C.lb_trace()
    o = C.lb_oracle()
    out_fr = fr.copy()
    out = o.run(out_fr, ln, dv, now, 64).astype(np.int32)
    exp_out, fields = spec_lb(fr, ln, dv, now)
    got = np.where(out == dv, -1, out)
    bad = np.nonzero(got != exp_out)[0]
    assert bad.size == 0, ("lb out", bad[:10], got[bad[:10]], exp_out[bad[:10]])
    fwd = exp_out >= 0
    have = np.array([(int.from_bytes(out_fr[p * 64:p * 64 + 6].tobytes(), "little"),
                      _le32(out_fr, p * 64 + 30)) for p in range(ln.shape[0])], np.int64)
    assert np.array_equal(have[fwd], fields[fwd]), "lb fields"
    np.savez_compressed(os.path.join(HERE, "spec_lb.npz"), frames=fr, lens=ln,
                        in_dev=dv, now=now, out=exp_out, fields=fields,
                        spec=np.array("viglb/spec.py"))
    print("spec_lb: %d packets, %d forwarded" % (ln.shape[0], int(fwd.sum())))


if __name__ == "__main__":
    main()
