"""Pin the oracle before trusting it (CPU only).

1. Known answers from SURVEY.md (probe runs of the reference itself):
   FlowId_hash KAT and the vignat byte-level frames of
   Appendix A (flow 0, LAN->WAN / WAN->LAN reverse path, anti-spoof drop,
   expiry drop).
2. The restated libVig vs the REFERENCE's own libVig sources (oracle/_ref,
   built from /root/reference/libvig/verified/*.c) on random operation
   streams: dchain (allocation order, LRU order, free-list LIFO, timestamps,
   expiry), the chain-counter map (colliding hash), the CHT table + lookups.
3. Whole-NF traces (vignat / vigbridge / viglb) with the same glue over both
   libVig builds: identical out ports and frame bytes.
The _ref tests skip when /root/reference is absent (e.g. on the GPU box).
"""
import os

import numpy as np
import pytest

import orc
from tracegen import mixed_fw_trace, mixed_nat_trace, mixed_pol_trace
from vigor_amd import traces as T

HAVE_REF = os.path.isdir("/root/reference/libvig/verified")
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="reference not present")
IMPLS = [False, True] if HAVE_REF else [False]

DEV_MACS = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17")]
END_MACS = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01")]


def kat_nat(ref, expire_us=60_000_000):
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=expire_us, max_flows=65536,
                      device_macs=DEV_MACS, endpoint_macs=END_MACS)
    return orc.Oracle("nat", cfg, ref=ref)


@pytest.mark.parametrize("ref", IMPLS)
def test_flowid_hash_kat(ref):
    assert orc.lib(ref).orc_flowid_hash(1, 2, 3, 4, 5, 6) == 0xAE93F0FF


@needs_ref
def test_crc_software_equals_hardware():
    rng = np.random.default_rng(1)
    a, b = orc.lib(False), orc.lib(True)
    for _ in range(2000):
        c, v = (int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64))
        assert a.orc_crc32c_u32(c, v) == b.orc_crc32c_u32(c, v)
    for _ in range(200):
        m = bytes(rng.integers(0, 256, 6, dtype=np.uint8))
        assert a.orc_ether_hash(m) == b.orc_ether_hash(m)


@pytest.mark.parametrize("ref", IMPLS)
def test_appendix_a_flow0(ref):
    o = kat_nat(ref)
    fr, ln, dv, now = T.nat_lan_trace(1, 1)
    out = o.run(fr, ln, dv, now, 64)
    assert out[0] == 1
    assert fr[:42].tobytes().hex() == (
        "012345678901121314151617" "0800"
        "4500002e000000004011cffb0204a8c000000000" "0000" "0000" "001a" "54f6")


def _udp(src, dst, sp, dp, proto=17):
    f, _ = T.udp_frames(np.array([src]), np.array([dst]), np.array([sp]),
                        np.array([dp]), slot=64, proto=proto)
    return bytearray(f.tobytes())


def _rfc768(src, dst, l4):
    b = src + dst + bytes([0, 17, 0, len(l4)]) + l4[:6] + b"\0\0" + l4[8:]
    s = sum((b[i] << 8) | (b[i + 1] if i + 1 < len(b) else 0)
            for i in range(0, len(b), 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF or 0xFFFF


@pytest.mark.parametrize("ref", IMPLS)
def test_appendix_a_reverse_path(ref):
    o = kat_nat(ref)
    t = T.NOW0
    for i in range(5):  # indices 0..4
        assert o.process(0, _udp(T.ip4(10, 0, 0, 100 + i), 0, 1, 1), 60, 64,
                         t + i) == 1
    f = _udp(T.ip4(10, 0, 0, 5), T.ip4(8, 8, 8, 8), 80, 53)
    assert o.process(0, f, 60, 64, t + 10) == 1
    assert f[:42].hex() == ("012345678901121314151617" "0800"
                            "4500002e000000004011bfeb" "0204a8c0" "08080808"
                            "0500" "0035" "001a" "3fb1")
    # reply: 8.8.8.8:53 -> 0.0.0.0, dst port bytes 05 00 -> index 5
    r = _udp(T.ip4(8, 8, 8, 8), 0, 53, 0x0500)
    assert o.process(1, r, 60, 64, t + 20) == 0
    assert r[:40].hex() == ("012345678900020304050607" "0800"
                            "4500002e00000000401160ab" "08080808" "0a000005"
                            "0035" "0050" "001a")
    # SURVEY.md prints only the first 42 bytes of its probe frame and UDP
    # checksum e51b. With the 18 B zero payload used here the checksum of
    # these header bytes is e520 (also by an independent RFC 768 sum). The
    # two differ by 0x0500 in the sum, i.e. exactly one payload byte 0x05 at
    # an odd L4 offset: the same reply with payload 00 05 00 ... gives e51b
    # from both the oracle and the RFC 768 sum, so the printed KAT holds for
    # a probe frame with that payload.
    assert r[40:42].hex() == "%04x" % _rfc768(bytes(r[26:30]), bytes(r[30:34]),
                                               bytes(r[34:60]))
    assert r[40:42].hex() == "e520"
    o2 = kat_nat(ref)
    for i in range(5):
        o2.process(0, _udp(T.ip4(10, 0, 0, 100 + i), 0, 1, 1), 60, 64, t + i)
    o2.process(0, _udp(T.ip4(10, 0, 0, 5), T.ip4(8, 8, 8, 8), 80, 53), 60, 64, t + 10)
    rp = _udp(T.ip4(8, 8, 8, 8), 0, 53, 0x0500)
    rp[43] = 0x05  # L4 offset 9: the second payload byte
    assert o2.process(1, rp, 60, 64, t + 20) == 0
    assert rp[40:42].hex() == "e51b"
    assert "%04x" % _rfc768(bytes(rp[26:30]), bytes(rp[30:34]), bytes(rp[34:60])) == "e51b"
    # dst port bytes 00 05 -> index 0x0500 = 1280, not allocated -> drop
    r2 = _udp(T.ip4(8, 8, 8, 8), 0, 53, 0x0005)
    before = bytes(r2)
    assert o.process(1, r2, 60, 64, t + 30) == 1
    assert bytes(r2) == before
    # anti-spoof: wrong source port -> drop
    r3 = _udp(T.ip4(8, 8, 8, 8), 0, 54, 0x0500)
    assert o.process(1, r3, 60, 64, t + 40) == 1


@pytest.mark.parametrize("ref", IMPLS)
def test_appendix_a_expiry(ref):
    o = kat_nat(ref, expire_us=1)
    t = T.NOW0
    f = _udp(T.ip4(10, 0, 0, 5), T.ip4(8, 8, 8, 8), 80, 53)
    assert o.process(0, f, 60, 64, t) == 1
    r = _udp(T.ip4(8, 8, 8, 8), 0, 53, 0x0000)
    assert o.process(1, bytearray(r), 60, 64, t + 1000) == 0  # ts < cutoff? no
    assert o.process(1, bytearray(r), 60, 64, t + 2001) == 1  # expired


# --------------------------------------------------------- libVig vs ref --

def _rand_dchain_ops(rng, range_, n):
    op = rng.integers(0, 5, n).astype(np.int32)
    arg = rng.integers(-1, range_ + 1, n).astype(np.int32)
    arg = np.clip(arg, 0, range_ - 1).astype(np.int32)
    t = np.cumsum(rng.integers(0, 4, n)).astype(np.int64)
    # expiry cut-offs a little behind "now"
    t = np.where(op == 2, t - rng.integers(0, 20, n), t).astype(np.int64)
    return op, arg, t


def _run_dchain(ref, range_, op, arg, t):
    L = orc.lib(ref)
    n = op.shape[0]
    res = np.zeros(n, np.int32)
    ao = np.zeros(range_, np.int32)
    fo = np.zeros(range_, np.int32)
    na = np.zeros(1, np.int32)
    nf = np.zeros(1, np.int32)
    ts = np.zeros(range_, np.int64)
    P = orc._ptr
    assert L.orc_test_dchain(range_, n, P(op), P(arg), P(t), P(res), P(ao),
                             P(na), P(fo), P(nf), P(ts))
    return res, ao[:na[0]], fo[:nf[0]], ts


@needs_ref
@pytest.mark.parametrize("seed", range(6))
def test_dchain_matches_reference(seed):
    rng = np.random.default_rng(seed)
    range_ = int(rng.choice([1, 2, 5, 64, 300]))
    op, arg, t = _rand_dchain_ops(rng, range_, 3000)
    a = _run_dchain(False, range_, op, arg, t)
    b = _run_dchain(True, range_, op, arg, t)
    for x, y in zip(a[:3], b[:3]):
        np.testing.assert_array_equal(x, y)
    # the reference mallocs timestamps uninitialised (double-chain.c:113-157):
    # only stamps of allocated indices are defined
    np.testing.assert_array_equal(a[3][a[1]], b[3][b[1]])


@needs_ref
@pytest.mark.parametrize("seed", range(6))
def test_map_matches_reference(seed):
    rng = np.random.default_rng(100 + seed)
    cap = int(rng.choice([8, 64, 1024]))
    hmod = int(rng.choice([1, 3, 7, 1000003]))
    live = {}
    free = list(range(cap))
    ops, keys, vals = [], [], []
    for _ in range(4000):
        r = rng.random()
        if r < 0.4 and free:
            k = int(rng.integers(0, 50 * cap))
            if k in live:
                continue
            s = free.pop(int(rng.integers(0, len(free))))
            live[k] = s
            ops.append(0), keys.append(k), vals.append(s)
        elif r < 0.7 and live:
            k = list(live)[int(rng.integers(0, len(live)))]
            s = live.pop(k)
            free.append(s)
            ops.append(2), keys.append(k), vals.append(s)
        else:
            k = int(rng.integers(0, 50 * cap)) if rng.random() < .5 or not live \
                else list(live)[int(rng.integers(0, len(live)))]
            ops.append(1), keys.append(k), vals.append(0)
    op = np.array(ops, np.int32)
    key = np.array(keys, np.uint32)
    val = np.array(vals, np.int32)
    out = []
    for ref in (False, True):
        res = np.zeros(op.shape[0], np.int32)
        P = orc._ptr
        assert orc.lib(ref).orc_test_map(cap, hmod, op.shape[0], P(op), P(key),
                                         P(val), P(res))
        out.append(res)
    np.testing.assert_array_equal(out[0], out[1])


@needs_ref
@pytest.mark.parametrize("height,cap", [(97, 32), (257, 256), (7, 4), (13, 1)])
def test_cht_matches_reference(height, cap):
    rng = np.random.default_rng(height)
    active = (rng.random(cap) < 0.6).astype(np.uint8)
    hashes = rng.integers(0, 2**63, 500, dtype=np.uint64)
    outs = []
    for ref in (False, True):
        tab = np.zeros(height * cap, np.uint32)
        ch = np.zeros(500, np.int32)
        P = orc._ptr
        assert orc.lib(ref).orc_test_cht(height, cap, P(tab), P(active), 500,
                                         P(hashes), P(ch))
        outs.append((tab, ch))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


# ------------------------------------------------------ whole-NF vs ref --

@needs_ref
@pytest.mark.parametrize("seed,max_flows,expire_us,n_flows",
                         [(0, 64, 60_000_000, 40), (1, 64, 1, 100),
                          (2, 16, 60_000_000, 40), (3, 256, 5, 300)])
def test_nat_trace_matches_reference(seed, max_flows, expire_us, n_flows):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_nat_trace(rng, 5000, n_flows, max_idx=max_flows)
    res = []
    for ref in (False, True):
        cfg = orc.nat_cfg(wan=1, ext_ip=T.ip4(192, 168, 4, 2),
                          expire_us=expire_us, max_flows=max_flows,
                          device_macs=DEV_MACS, endpoint_macs=END_MACS)
        o = orc.Oracle("nat", cfg, ref=ref)
        f = fr.copy()
        out = o.run(f, ln, dv, now, 64)
        res.append((out, f, o.nat_dump(max_flows)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    (a0, t0, k0), (a1, t1, k1) = res[0][2], res[1][2]
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(t0[a0 == 1], t1[a1 == 1])
    np.testing.assert_array_equal(k0, k1)


@needs_ref
@pytest.mark.parametrize("seed,cap,expire_us", [(0, 64, 300_000_000),
                                                (1, 16, 2), (2, 1024, 10)])
def test_bridge_trace_matches_reference(seed, cap, expire_us):
    rng = np.random.default_rng(seed)
    n = 4000
    fr, ln, dv, now = T.bridge_trace(n, 100)
    f2 = fr.reshape(n, 64)
    f2[:, 11] = rng.integers(0, 40, n)  # fewer stations, random mixes
    f2[:, 5] = rng.integers(0, 40, n)
    dv = rng.integers(0, 3, n).astype(np.uint16)
    now = T.NOW0 + np.cumsum(rng.integers(0, 4, n)).astype(np.int64)
    statics = [(bytes([2, 0, 0, 0, 0, 7]), 0, 2), (bytes([2, 0, 0, 0, 0, 9]),
                                                   1, -2)]
    res = []
    for ref in (False, True):
        cfg = orc.BridgeCfg(expiration_time=expire_us, dyn_capacity=cap,
                            n_devices=3)
        o = orc.Oracle("bridge", cfg, ref=ref, statics=statics)
        f = fr.copy()
        res.append((o.run(f, ln, dv, now, 64), f, o.bridge_dump(cap)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    (a0, t0, m0, p0), (a1, t1, m1, p1) = res[0][2], res[1][2]
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(t0[a0 == 1], t1[a1 == 1])
    np.testing.assert_array_equal(m0, m1)
    np.testing.assert_array_equal(p0, p1)


def lb_cfg(flow_cap=1024, bcap=32, height=97, fexp=60_000_000, bexp=3_600_000):
    c = orc.LbCfg(flow_capacity=flow_cap, flow_expiration_time=fexp,
                  backend_capacity=bcap, cht_height=height,
                  backend_expiration_time=bexp, wan_device=2, n_devices=3)
    for d in range(3):
        for i in range(6):
            c.device_macs[d][i] = 0x10 * d + i
    return c


@needs_ref
@pytest.mark.parametrize("seed,fexp,bexp", [(0, 60_000_000, 3_600_000_000),
                                            (1, 3, 50), (2, 20, 2)])
def test_lb_trace_matches_reference(seed, fexp, bexp):
    rng = np.random.default_rng(seed)
    hb = T.lb_heartbeats(20)
    tr = T.lb_traffic(3000, 500, order="uniform", seed=seed)
    fr = np.concatenate([hb[0], tr[0]])
    ln = np.concatenate([hb[1], tr[1]])
    dv = np.concatenate([hb[2], tr[2]])
    # interleave some more heartbeats inside the traffic
    dv = dv.copy()
    k = rng.random(dv.shape[0]) < 0.05
    dv[k] = rng.integers(0, 2, k.sum())
    now = T.NOW0 + np.cumsum(rng.integers(0, 3, dv.shape[0])).astype(np.int64)
    res = []
    for ref in (False, True):
        o = orc.Oracle("lb", lb_cfg(fexp=fexp, bexp=bexp), ref=ref)
        f = fr.copy()
        res.append((o.run(f, ln, dv, now, 64), f, o.lb_dump(1024, 32)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    for x, y in zip(res[0][2], res[1][2]):  # flows, then backends
        live = x[0] == 1
        np.testing.assert_array_equal(x[0], y[0])
        for a, b in zip(x[1:], y[1:]):
            np.testing.assert_array_equal(a[live], b[live])


# ---------------------------------------------------------------- vigfw --

@pytest.mark.parametrize("ref", IMPLS)
def test_fw_flowid_hash_is_crc_chain(ref):
    """vigfw's generated FlowId_hash: five crc32c_u32 steps in field order
    (codegen/main.ml:328-401), checked against the chained u32 CRC."""
    L = orc.lib(ref)
    for sp, dp, sip, dip, pr in [(1, 2, 3, 4, 5), (0x3500, 0xE803, 0x0A000001,
                                                   0x08080808, 17)]:
        h = 0
        for v in (sp, dp, sip, dip, pr):
            h = L.orc_crc32c_u32(h, v)
        assert L.orc_fw_flowid_hash(sp, dp, sip, dip, pr) == h


def fw_oracle(ref, max_flows=64, expire_us=60_000_000, n_dev=3, wan=1):
    cfg = orc.fw_cfg(wan=wan, expire_us=expire_us, max_flows=max_flows,
                     device_macs=DEV3_MACS[:n_dev], endpoint_macs=END3_MACS[:n_dev],
                     n_devices=n_dev)
    return orc.Oracle("fw", cfg, ref=ref)


DEV3_MACS = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17"),
             T.mac("22:23:24:25:26:27")]
END3_MACS = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01"),
             T.mac("01:23:45:67:89:02")]


@pytest.mark.parametrize("ref", IMPLS)
def test_fw_semantics_kat(ref):
    """fw_main.c:21-80 by hand: a LAN packet opens the flow and goes out on
    the WAN with its MACs; the reply comes back to the LAN device that opened
    it; an unknown reply is dropped; a non-TCP/UDP packet is dropped; the
    header past the MACs is never touched."""
    o = fw_oracle(ref)
    f, _ = T.udp_frames(np.array([T.ip4(10, 0, 0, 5)]), np.array([T.ip4(8, 8, 8, 8)]),
                        np.array([1234]), np.array([53]))
    lan = bytearray(f.tobytes())
    orig = bytes(lan)
    assert o.process(2, lan, now=T.NOW0) == 1
    assert bytes(lan[0:6]) == END3_MACS[1] and bytes(lan[6:12]) == DEV3_MACS[1]
    assert bytes(lan[12:]) == orig[12:]
    r, _ = T.udp_frames(np.array([T.ip4(8, 8, 8, 8)]), np.array([T.ip4(10, 0, 0, 5)]),
                        np.array([53]), np.array([1234]))
    rep = bytearray(r.tobytes())
    assert o.process(1, rep, now=T.NOW0 + 1) == 2
    assert bytes(rep[0:6]) == END3_MACS[2] and bytes(rep[6:12]) == DEV3_MACS[2]
    u, _ = T.udp_frames(np.array([T.ip4(8, 8, 8, 8)]), np.array([T.ip4(10, 0, 0, 6)]),
                        np.array([53]), np.array([1234]))
    unk = bytearray(u.tobytes())
    assert o.process(1, unk, now=T.NOW0 + 2) == 1 and bytes(unk) == u.tobytes()
    icmp = bytearray(orig)
    icmp[23] = 1
    assert o.process(0, icmp, now=T.NOW0 + 3) == 0
    alloc, ts, keys, dev = o.fw_dump(64)
    assert alloc.sum() == 1 and dev[0] == 2 and ts[0] == T.NOW0 + 1


@needs_ref
@pytest.mark.parametrize("seed,max_flows,expire_us,n_flows",
                         [(0, 64, 60_000_000, 40), (1, 64, 1, 100),
                          (2, 16, 60_000_000, 40), (3, 256, 5, 300)])
def test_fw_trace_matches_reference(seed, max_flows, expire_us, n_flows):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_fw_trace(rng, 5000, n_flows)
    res = []
    for ref in (False, True):
        o = fw_oracle(ref, max_flows=max_flows, expire_us=expire_us)
        f = fr.copy()
        out = o.run(f, ln, dv, now, 64)
        res.append((out, f, o.fw_dump(max_flows)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    (a0, t0, k0, d0), (a1, t1, k1, d1) = res[0][2], res[1][2]
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(t0[a0 == 1], t1[a1 == 1])
    np.testing.assert_array_equal(k0, k1)
    np.testing.assert_array_equal(d0, d1)


def pol_oracle(ref, cap=64, rate=1_000_000, burst=1000, n_dev=3, lan=1, wan=0):
    return orc.Oracle("pol", orc.pol_cfg(lan=lan, wan=wan, rate=rate, burst=burst,
                                         capacity=cap, n_devices=n_dev), ref=ref)


@pytest.mark.parametrize("ref", IMPLS)
def test_pol_semantics_kat(ref):
    """policer_main.c:34-145 by hand (rate 1 B/us, burst 1000 B): a new
    destination takes burst - size; a refill adds time_diff * rate / 1e9;
    a packet passes only while bucket > size; after burst/rate of silence the
    bucket is full again; LAN packets pass unpoliced; frames are untouched."""
    o = pol_oracle(ref)
    f, _ = T.udp_frames(np.array([T.ip4(9, 9, 9, 9)]), np.array([T.ip4(10, 0, 0, 1)]),
                        np.array([53]), np.array([80]))
    fr = bytearray(f.tobytes())
    orig = bytes(fr)
    t = T.NOW0
    assert o.process(0, fr, length=600, now=t) == 1       # new: 1000-600 = 400
    assert o.process(0, fr, length=400, now=t) == 0       # 400 > 400 fails
    assert o.process(0, fr, length=399, now=t) == 1       # 1 left
    assert o.process(0, fr, length=64, now=t + 100_000) == 1  # +100 -> 101 - 64
    alloc, ts, keys, size, btime = o.pol_dump(64)
    assert alloc.sum() == 1 and size[0] == 37 and btime[0] == t + 100_000
    assert keys[0] == 0x0100000A and ts[0] == t + 100_000  # raw (network order)
    assert o.process(0, fr, length=1001, now=t + 100_001) == 0  # hit, > burst
    assert o.process(1, fr, length=64, now=t + 100_002) == 0    # LAN -> WAN
    assert o.process(2, fr, length=64, now=t + 100_003) == 2    # other: drop
    assert bytes(fr) == orig
    # burst/rate = 1 ms after the last touch the entry expires
    g, _ = T.udp_frames(np.array([T.ip4(9, 9, 9, 9)]), np.array([T.ip4(10, 0, 0, 2)]),
                        np.array([53]), np.array([80]))
    fr2 = bytearray(g.tobytes())
    assert o.process(0, fr2, length=1001, now=t + 2_000_000) == 0  # > burst, new
    alloc, ts, keys, size, btime = o.pol_dump(64)
    assert alloc.sum() == 0


@needs_ref
@pytest.mark.parametrize("seed,cap,n_dsts,burst,gap", [
    (0, 64, 40, 3000, 500), (1, 16, 60, 1000, 2000), (2, 256, 300, 2000, 50),
    (3, 64, 20, 1000, 10)])
def test_pol_trace_matches_reference(seed, cap, n_dsts, burst, gap):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_pol_trace(rng, 6000, n_dsts, gap_ns=gap)
    res = []
    for ref in (False, True):
        o = pol_oracle(ref, cap=cap, burst=burst)
        f = fr.copy()
        out = o.run(f, ln, dv, now, 64)
        res.append((out, f, o.pol_dump(cap)))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], fr)
    (a0, t0, *v0), (a1, t1, *v1) = res[0][2], res[1][2]
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(t0[a0 == 1], t1[a1 == 1])
    for x, y in zip(v0, v1):
        np.testing.assert_array_equal(x, y)
    assert (res[0][0] == 1).sum() > 100 and (res[0][0] == 0).sum() > 100
