"""Traces and configurations of the spec fixtures (tests/golden/spec_*.npz,
made by tests/golden/make_spec_golden.py from the reference's own
vignat/vigfw/vigbridge spec.py). The specs fix the expiry window at
EXP_TIME = 10 * 1000 (vignat/spec.py:17, vigfw/spec.py:2,
vigbridge/spec.py:2), the WAN port at 1 (vignat, vigfw) and vigbridge's
broadcast at the other of two ports, so the configurations here do too:
--expire 10 (x 1000 in the NFs), WAN device 1, two bridge ports."""
import numpy as np

import orc
from tracegen import mixed_lb_trace, mixed_pol_trace
from vigor_amd import traces as T

N = 3000
NAT_CAP, FW_CAP, BRIDGE_CAP, POL_CAP, LB_CAP = 64, 64, 64, 64, 64
LB_BACKENDS, LB_HEIGHT = 32, 97  # cht height: a prime above the backends
LB_BACKEND_EXPIRE = 3_600_000_000  # viglb/spec.py:3 (x 1000 in the NF)
LB_MACS = [bytes([0x10 * d + i for i in range(6)]) for d in range(3)]
NAT_START_PORT = 1000
NAT_EXT_IP = T.ip4(192, 168, 4, 2)
EXPIRE = 10
DEV3 = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17"),
        T.mac("22:23:24:25:26:27")]
END3 = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01"),
        T.mac("01:23:45:67:89:02")]
SERVERS = [T.ip4(93, 184, 216, 34), T.ip4(8, 8, 8, 8), T.ip4(1, 1, 1, 1),
           T.ip4(9, 9, 9, 9)]
SPORTS = [80, 443, 53]


def _swap16(x):
    return ((x & 0xFF) << 8) | (x >> 8)


def _frame(sip, dip, sp, dp, proto=17, ethertype=None):
    f, ln = T.udp_frames(np.array([sip], np.int64), np.array([dip], np.int64),
                         np.array([sp], np.int64), np.array([dp], np.int64),
                         proto=proto)
    if ethertype is not None:
        f[12], f[13] = ethertype >> 8, ethertype & 0xFF
    return f, int(ln[0])


def _assemble(rows, now):
    fr = np.concatenate([r[0] for r in rows])
    ln = np.array([r[1] for r in rows], np.uint16)
    dv = np.array([r[2] for r in rows], np.uint16)
    return fr, ln, dv, np.asarray(now, np.int64)


def _times(rng, n):
    """Alternating stretches of 500 packets: steps of 0 or 10 (nothing
    expires; the tables fill up) and steps of 0-500 in multiples of 100 (a
    flow idle for ~50 packets expires, and stamps often sit exactly at the
    cutoff now - 10,000, the boundary of expire_all's strict <)."""
    fast = (np.arange(n) // 500) % 2 == 0
    step = np.where(fast, rng.choice([0, 10], n), rng.choice([0, 100, 200, 300, 500], n))
    return T.NOW0 + np.cumsum(step).astype(np.int64)


def nat_trace(seed=201, n=N):
    """LAN flows (some hot), WAN replies to external ports 0..cap-1 from the
    servers' addresses and ports (right and wrong), non-IPv4 and ICMP."""
    rng = np.random.default_rng(seed)
    flows = [(T.ip4(10, 0, rng.integers(0, 4), rng.integers(1, 250)),
              int(rng.choice(SERVERS)), int(rng.integers(1024, 65535)),
              int(rng.choice(SPORTS)), int(rng.choice([6, 17])))
             for _ in range(160)]
    rows = []
    for _ in range(n):
        r = rng.random()
        if r < 0.55:
            k = int(rng.integers(0, 20)) if rng.random() < 0.5 else int(rng.integers(0, 160))
            sip, dip, sp, dp, pr = flows[k]
            f, ln = _frame(sip, dip, sp, dp, pr)
            rows.append((f, ln, 0))
        elif r < 0.85:
            idx = int(rng.integers(0, NAT_CAP))
            f, ln = _frame(int(rng.choice(SERVERS)), NAT_EXT_IP,
                           int(rng.choice(SPORTS)), _swap16(NAT_START_PORT + idx),
                           int(rng.choice([6, 17])))
            rows.append((f, ln, 1))
        elif r < 0.93:
            sip, dip, sp, dp, pr = flows[int(rng.integers(0, 160))]
            f, ln = _frame(sip, dip, sp, dp, pr, ethertype=0x86DD)
            rows.append((f, ln, int(rng.integers(0, 2))))
        else:
            sip, dip, sp, dp, _ = flows[int(rng.integers(0, 160))]
            f, ln = _frame(sip, dip, sp, dp, proto=1)
            rows.append((f, ln, int(rng.integers(0, 2))))
    return _assemble(rows, _times(rng, n))


def nat_oracle():
    return orc.Oracle("nat", orc.nat_cfg(
        wan=1, start_port=NAT_START_PORT, ext_ip=NAT_EXT_IP, expire_us=EXPIRE,
        max_flows=NAT_CAP, device_macs=DEV3[:2], endpoint_macs=END3[:2],
        n_devices=2))


def nat_gpu_args():
    return ["--wan", "1", "--expire", str(EXPIRE), "--starting-port",
            str(NAT_START_PORT), "--max-flows", str(NAT_CAP), "--extip",
            "192.168.4.2", "--eth-dest", "0,%s" % END3[0].hex(":"),
            "--eth-dest", "1,%s" % END3[1].hex(":")]


def fw_trace(seed=202, n=N):
    """LAN flows from devices 0 and 2, WAN replies (device 1) to them and to
    unknown flows, non-IPv4 and ICMP."""
    rng = np.random.default_rng(seed)
    flows = [(T.ip4(10, 0, rng.integers(0, 4), rng.integers(1, 250)),
              int(rng.choice(SERVERS)), int(rng.integers(1024, 65535)),
              int(rng.choice(SPORTS)), int(rng.choice([6, 17])),
              int(rng.choice([0, 2])))
             for _ in range(160)]
    rows = []
    for _ in range(n):
        r = rng.random()
        sip, dip, sp, dp, pr, d = flows[int(rng.integers(0, 20)) if rng.random() < 0.5
                                        else int(rng.integers(0, 160))]
        if r < 0.5:
            f, ln = _frame(sip, dip, sp, dp, pr)
            rows.append((f, ln, d))
        elif r < 0.85:
            if rng.random() < 0.2:  # a reply nobody asked for
                sp = int(rng.integers(1024, 65535))
            f, ln = _frame(dip, sip, dp, sp, pr)
            rows.append((f, ln, 1))
        elif r < 0.93:
            f, ln = _frame(sip, dip, sp, dp, pr, ethertype=0x86DD)
            rows.append((f, ln, int(rng.integers(0, 3))))
        else:
            f, ln = _frame(sip, dip, sp, dp, proto=1)
            rows.append((f, ln, int(rng.integers(0, 3))))
    return _assemble(rows, _times(rng, n))


def fw_oracle():
    return orc.Oracle("fw", orc.fw_cfg(
        wan=1, expire_us=EXPIRE, max_flows=FW_CAP, device_macs=DEV3,
        endpoint_macs=END3, n_devices=3))


def fw_gpu_args():
    args = ["--wan", "1", "--expire", str(EXPIRE), "--max-flows", str(FW_CAP)]
    for d in range(3):
        args += ["--eth-dest", "%d,%s" % (d, END3[d].hex(":"))]
    return args


def bridge_trace(seed=203, n=N):
    """Stations on two ports (some move), frames to known, unknown and
    broadcast addresses; the dynamic table fills."""
    rng = np.random.default_rng(seed)
    macs = [bytes([0x02, 0, 0, 0, s >> 8, s & 0xFF]) for s in range(80)]
    port = rng.integers(0, 2, 80)
    rows = []
    for _ in range(n):
        s = int(rng.integers(0, 12)) if rng.random() < 0.5 else int(rng.integers(0, 80))
        if rng.random() < 0.01:
            port[s] ^= 1  # the station moved
        r = rng.random()
        if r < 0.7:
            dst = macs[int(rng.integers(0, 80))]
        elif r < 0.9:
            dst = bytes([0x02, 0xEE, 0, 0, 0, int(rng.integers(0, 256))])
        else:
            dst = b"\xff" * 6
        f, ln = T.udp_frames(np.array([T.ip4(10, 0, 0, 1)], np.int64),
                             np.array([T.ip4(10, 0, 0, 2)], np.int64),
                             np.array([1], np.int64), np.array([2], np.int64),
                             eth_src=macs[s], eth_dst=dst)
        rows.append((f, int(ln[0]), int(port[s])))
    return _assemble(rows, _times(rng, n))


def bridge_oracle():
    return orc.Oracle("bridge", orc.BridgeCfg(expiration_time=EXPIRE,
                                              dyn_capacity=BRIDGE_CAP, n_devices=2))


def bridge_gpu_args():
    return ["--expire", str(EXPIRE), "--capacity", str(BRIDGE_CAP)]


# vigpol/spec.py:2-6 fixes LAN 1, WAN 0, the bucket (burst 3.75e9 B, rate
# 3.75e8 B/s: the Makefile defaults) and EXP_TIME = 10 s in ns.
def pol_trace(seed=204, n=N):
    """WAN packets to 100 destinations (the table holds 64), LAN packets,
    a third device, non-IPv4, IHL < 5, total_length > size, IP options;
    gaps of 0-0.1 s in steps of 10 ms (entries expire after 10 s idle,
    stamps sit at the cutoff)."""
    rng = np.random.default_rng(seed)
    fr, ln, dv, _ = mixed_pol_trace(rng, n, 100)
    step = rng.choice([0, 10_000_000, 50_000_000, 100_000_000], n)
    return fr, ln, dv, T.NOW0 + np.cumsum(step).astype(np.int64)


def pol_oracle():
    return orc.Oracle("pol", orc.pol_cfg(lan=1, wan=0, capacity=POL_CAP, n_devices=3))


def pol_gpu_args():
    return ["--lan", "1", "--wan", "0", "--rate", "375000000", "--burst",
            "3750000000", "--capacity", str(POL_CAP)]


# viglb/spec.py:2-4 fixes EXP_TIME = 10 * 1000, the backends' expiry
# (3,600,000,000 x 1000) and the client port 2.
def lb_trace(seed=205, n=N):
    """Client flows (port 2) over 150 5-tuples, heartbeats from 24 backends
    on ports 0/1, non-IPv4 and ICMP frames; a time jump past the backends'
    expiry at packet 1500 with no heartbeat for the next 300 packets (flows
    whose backend died are erased and re-balanced, or dropped)."""
    rng = np.random.default_rng(seed)
    fr, ln, dv, _ = mixed_lb_trace(rng, n, 150, 24, hb_frac=0.08, quiet=(1500, 1800),
                                   bad_frac=0.0)
    f = fr.reshape(n, 64)
    bad = rng.random(n)
    f[bad < 0.03, 12] = 0x86                      # not IPv4
    f[(bad >= 0.03) & (bad < 0.06), 23] = 1       # not TCP/UDP
    fast = (np.arange(n) // 500) % 2 == 0
    step = np.where(fast, rng.choice([0, 10], n), rng.choice([0, 100, 200, 300, 500], n))
    step[1500] = 3_600_000_000 * 1000 + 5_000     # every backend expires
    return fr, ln, dv, T.NOW0 + np.cumsum(step).astype(np.int64)


def lb_cfg():
    c = orc.LbCfg(flow_capacity=LB_CAP, flow_expiration_time=EXPIRE,
                  backend_capacity=LB_BACKENDS, cht_height=LB_HEIGHT,
                  backend_expiration_time=LB_BACKEND_EXPIRE, wan_device=2,
                  n_devices=3)
    for d in range(3):
        c.device_macs[d][:] = list(LB_MACS[d])
    return c


def lb_oracle(ref=False):
    return orc.Oracle("lb", lb_cfg(), ref=ref)


def lb_gpu_args():
    return ["--flow-capacity", str(LB_CAP), "--backend-capacity", str(LB_BACKENDS),
            "--cht-height", str(LB_HEIGHT), "--flow-expiration", str(EXPIRE),
            "--backend-expiration", str(LB_BACKEND_EXPIRE), "--wan", "2"]
