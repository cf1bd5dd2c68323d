"""Golden cases: per-NF 4,096-packet traces whose expected outputs were
produced by the oracle glue over the REFERENCE's own libVig (oracle/_ref,
compiled from /root/reference/libvig/verified by oracle/Makefile), stored in
tests/golden/<name>.npz by tests/golden/make_golden.py. The GPU box has no
reference: these fixtures carry its answers there.

What they pin: the libVig layer (map with chain counters, dchain allocation
/ LRU / expiry, vector, CHT) is the reference's own code. The NF-level glue
(header parse, nf_process decision logic of vignat / vigfw / vigbridge /
viglb / vigpol, the DPDK checksum) is the clean-room restatement in
oracle/orc.c on both sides, so these fixtures leave NF-level semantics
parity-unpinned: a misreading shared by the restatement and the GPU path
would not show here. The NF level is pinned separately: by the reference's
own specifications (vignat/vigfw/vigbridge spec.py, executed over a model of
libvig's VeriFast definitions: tests/spec_cases.py, tests/test_spec.py) and
by the SURVEY.md Appendix-A byte-level KATs (tests/test_oracle.py); the
reference NF sources cannot be compiled here."""
import os

import numpy as np

import orc
from tracegen import (mixed_bridge_trace, mixed_fw_trace, mixed_lb_trace,
                      mixed_nat_trace, mixed_pol_trace, wide_nat_trace)
from vigor_amd import traces as T

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N = 4096
DEV3 = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17"),
        T.mac("22:23:24:25:26:27")]
END3 = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01"),
        T.mac("01:23:45:67:89:02")]
LB_MACS = [bytes([0x10 * d + i for i in range(6)]) for d in range(3)]

# name -> (kind, table capacity, trace builder); configs below
CASES = {
    "nat_churn": ("nat", 64, lambda: mixed_nat_trace(np.random.default_rng(101), N, 100)),
    "fw_churn": ("fw", 64, lambda: mixed_fw_trace(np.random.default_rng(102), N, 100)),
    "bridge_churn": ("bridge", 64,
                     lambda: mixed_bridge_trace(np.random.default_rng(103), N, 80)),
    "lb_churn": ("lb", 64, lambda: mixed_lb_trace(np.random.default_rng(104), N, 200, 20)),
    "pol_churn": ("pol", 16, lambda: mixed_pol_trace(np.random.default_rng(105), N, 60,
                                                     gap_ns=2000)),
}


def oracle(name, ref=False):
    kind, cap, _ = CASES[name]
    if kind == "nat":
        cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                          expire_us=2, max_flows=cap, device_macs=DEV3[:2],
                          endpoint_macs=END3[:2], n_devices=2)
    elif kind == "fw":
        cfg = orc.fw_cfg(wan=1, expire_us=3, max_flows=cap, device_macs=DEV3,
                         endpoint_macs=END3, n_devices=3)
    elif kind == "bridge":
        cfg = orc.BridgeCfg(expiration_time=2, dyn_capacity=cap, n_devices=3)
    elif kind == "lb":
        cfg = orc.LbCfg(flow_capacity=cap, flow_expiration_time=3,
                        backend_capacity=32, cht_height=97,
                        backend_expiration_time=3_600_000, wan_device=2,
                        n_devices=3)
        for d in range(3):
            cfg.device_macs[d][:] = list(LB_MACS[d])
    else:
        cfg = orc.pol_cfg(lan=1, wan=0, rate=1_000_000, burst=1000, capacity=cap,
                          n_devices=3)
    return orc.Oracle(kind, cfg, ref=ref)


def gpu(name):
    import vigor_amd
    kind, cap, _ = CASES[name]
    if kind == "nat":
        args = ["--wan", "1", "--expire", "2", "--starting-port", "0",
                "--max-flows", str(cap), "--extip", "192.168.4.2"]
        for d in range(2):
            args += ["--eth-dest", "%d,%s" % (d, END3[d].hex(":"))]
        return vigor_amd.Nat(vigor_amd.nat_config_from_args(args, 2, DEV3[:2]))
    if kind == "fw":
        args = ["--wan", "1", "--expire", "3", "--max-flows", str(cap)]
        for d in range(3):
            args += ["--eth-dest", "%d,%s" % (d, END3[d].hex(":"))]
        return vigor_amd.Fw(vigor_amd.fw_config_from_args(args, 3, DEV3))
    if kind == "bridge":
        return vigor_amd.Bridge(vigor_amd.bridge_config_from_args(
            ["--expire", "2", "--capacity", str(cap)], 3, []))
    if kind == "lb":
        args = ["--flow-capacity", str(cap), "--backend-capacity", "32",
                "--cht-height", "97", "--flow-expiration", "3",
                "--backend-expiration", "3600000", "--wan", "2"]
        return vigor_amd.Lb(vigor_amd.lb_config_from_args(args, 3, LB_MACS))
    args = ["--lan", "1", "--wan", "0", "--rate", "1000000", "--burst", "1000",
            "--capacity", str(cap)]
    return vigor_amd.Pol(vigor_amd.pol_config_from_args(args, 3))


def oracle_state(name, o):
    """(alloc, ts where allocated) of the NF's main table."""
    kind, cap, _ = CASES[name]
    if kind == "lb":
        d = o.lb_dump(cap, 32)[0]
    else:
        d = getattr(o, kind + "_dump")(cap)
    alloc, ts = d[0], d[1]
    return alloc, np.where(alloc == 1, ts, 0)


def gpu_state(name, nf):
    kind = CASES[name][0]
    d = nf.dump()
    if kind == "lb":
        d = d[0]
    alloc, ts = d[0], d[1]
    return alloc, np.where(alloc == 1, ts, 0)


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# BASELINE configs[1] at full table size: vignat, 1M flows, the bench's own
# trace shape (round robin, now_p = 1e9 + p); 2^21 packets = every flow
# allocated once, then hit once. Stored as a digest (FNV-1a-64 over
# out_port || frame, orc_digest) plus the first and last 1,024 frames.
BIG_FLOWS = 1 << 20
BIG_PACKETS = 1 << 21
BIG_NAT_ARGS = ["--expire", "60000000", "--starting-port", "0", "--wan", "1",
                "--extip", "192.168.4.2", "--eth-dest", "0,90:e2:ba:55:12:20",
                "--eth-dest", "1,90:e2:ba:55:12:21"]
BIG_DEV = [T.mac("02:00:00:00:00:00"), T.mac("02:00:00:00:00:01")]
BIG_END = [T.mac("90:e2:ba:55:12:20"), T.mac("90:e2:ba:55:12:21")]


def big_trace():
    return T.nat_lan_trace(BIG_PACKETS, BIG_FLOWS)


def big_oracle(ref=False):
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=60_000_000, max_flows=BIG_FLOWS,
                      device_macs=BIG_DEV, endpoint_macs=BIG_END, n_devices=2)
    return orc.Oracle("nat", cfg, ref=ref)


def big_gpu():
    import vigor_amd
    cfg = vigor_amd.nat_config_from_args(
        BIG_NAT_ARGS + ["--max-flows", str(BIG_FLOWS)], 2, BIG_DEV)
    return vigor_amd.Nat(cfg)


# The bench's own shape (bench.py, BASELINE configs[1]): 1M flows, batches of
# 2^24 packets (every flow touched 16 times per batch, so steady-state
# batches fold their stamps through the touch bins), round robin, now_p =
# 1e9 + p. Batch 0 allocates every flow, batch 1 is all hits. Stored: each
# batch's batch_digest (positions local to the batch), the state_digest of
# (alloc, ts) after batch 1, and the live count.
BENCH_FLOWS = 1 << 20
BENCH_BATCH = 1 << 24
BENCH_BATCHES = 2

# BASELINE configs[4] at full table size: 16M flows, 2^25 packets (every
# flow allocated once, then hit once), round robin. Stored: batch_digest over
# the whole trace (global positions), state_digest, live count, and the first
# and last 1,024 output frames.
F16M_FLOWS = 1 << 24
F16M_PACKETS = 1 << 25

CHUNK = 1 << 22


def nat_oracle(flows, ref=False):
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=60_000_000, max_flows=flows,
                      device_macs=BIG_DEV, endpoint_macs=BIG_END, n_devices=2)
    return orc.Oracle("nat", cfg, ref=ref)


def nat_gpu(flows, gpu=0):
    import vigor_amd
    cfg = vigor_amd.nat_config_from_args(
        BIG_NAT_ARGS + ["--max-flows", str(flows)], 2, BIG_DEV)
    return vigor_amd.Nat(cfg, gpu=gpu)


def run_oracle_chunks(o, n_packets, n_flows, start=0, on_chunk=None):
    """Run the round-robin trace [start, start + n_packets) through oracle o
    in chunks; on_chunk(p0, frames, out) sees every chunk's output."""
    p = start
    while p < start + n_packets:
        m = min(CHUNK, start + n_packets - p)
        fr, ln, dv, now = T.nat_lan_trace(m, n_flows, start=p)
        out = o.run(fr, ln, dv, now, 64)
        if on_chunk:
            on_chunk(p, fr, out)
        p += m


# Wide slots (north_star: 64-1518 B frames): vignat churn over frames of
# 60..1518 bytes with random payloads in 2048-byte (mbuf-sized) slots, table
# of 256 flows with expiry, WAN replies, padded / odd / malformed frames. The
# trace is regenerated from its seed (a fixture of 8 MB of random payload
# would be copied data, not a vector); stored: a digest of the input slots
# (generator drift), out ports, a per-packet FNV-1a-64 of each output slot
# (orc.slot_hashes), and the final allocated indices with their stamps.
WIDE_N, WIDE_SLOT, WIDE_CAP = 4096, 2048, 256


def wide_trace():
    return wide_nat_trace(np.random.default_rng(106), WIDE_N, 300, WIDE_SLOT,
                          max_len=1518)


def wide_oracle(ref=False):
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=2, max_flows=WIDE_CAP, device_macs=DEV3[:2],
                      endpoint_macs=END3[:2], n_devices=2)
    return orc.Oracle("nat", cfg, ref=ref)


def wide_gpu():
    import vigor_amd
    args = ["--wan", "1", "--expire", "2", "--starting-port", "0",
            "--max-flows", str(WIDE_CAP), "--extip", "192.168.4.2"]
    for d in range(2):
        args += ["--eth-dest", "%d,%s" % (d, END3[d].hex(":"))]
    return vigor_amd.Nat(vigor_amd.nat_config_from_args(args, 2, DEV3[:2]))


def slot_hashes(frames, slot):
    """FNV-1a-64 over each slot's 8-byte LE words (per packet)."""
    w = np.ascontiguousarray(frames.reshape(-1, slot)).view("<u8")
    h = np.full(w.shape[0], T.FNV64_BASIS, np.uint64)
    with np.errstate(over="ignore"):
        for j in range(w.shape[1]):
            np.bitwise_xor(h, w[:, j], out=h)
            np.multiply(h, np.uint64(T.FNV64_PRIME), out=h)
    return h
