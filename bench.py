"""Headline benchmark: vignat device-resident classification throughput.

BASELINE.json metric: "Mpackets/s device-resident, 64B vignat @1M flows;
%HBM roofline", measured on configs[1]: vignat 64 B, 1M flows, 1xMI355X
(parse + CRC32C hash + map probe + state update + checksum rewrite).

A step = one pass of the hot path (vp_process_device) over one batch of
B synthetic 64 B packets already resident in HBM (traces.nat_lan_trace
shape: round-robin over 1M flows, now_p = 1e9 + p ns).
Every timed step reads its own pre-generated batch, so no input restore sits
inside the timed region. A warm-up pass allocates all 1M flows first (its
rate is reported as new_flow_mpps).

N > 1 (torch.distributed, one rank per GPU; BASELINE configs[4]): ONE vignat
over all GPUs with 16M flows; every global batch is N x B packets and rank r
ingests its contiguous slice r (B packets, weak scaling). By default
(--shard-mode owner, north_star's design, the headline value) the
dictionary is sharded by flow hash: LAN packets whose key another GPU owns
are looked up there through an RCCL all-to-all of 16-byte keys and 4-byte
answers over xGMI. --shard-mode replicated keeps the whole dictionary on
every GPU: steady-state packets need no data-path collective, only small
all-gathers per batch. The other placement is measured in the same run
(extra key other_shard_mode). In both, new flows are
all-gathered so every rank allocates identically. Results equal
one nf.c over the concatenated batch in both modes (DESIGN.md §6,
tests/test_shard_gpu.py). value = all ranks' packets / max-over-ranks time.
`--gpus N` without a torch.distributed environment starts the N ranks
itself.

Also reported:
  roofline      algorithmic HBM-read bytes per packet (92 B)
                x packets per launch / average classify-kernel time (HIP
                events on the context's stream, in a second timed pass over
                the next K batches: the events cost a step about 6 us of
                kernel-boundary time, so the headline pass runs without
                them), vs 8 TB/s
  cpu_baseline  the oracle (clean-room C restatement of nf.c + vignat) on
                one host core, warm 1M-flow table, bounded sample
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import vigor_amd  # noqa: E402
from vigor_amd import traces as T  # noqa: E402

METRIC = "Mpackets/s device-resident, 64B vignat @1M flows; %HBM roofline"
ALG_BYTES = 92          # 64 frame + 4 len/port + 16 key + 4 tag + 4 value
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
SLOT = 64
# VIGPATH_BENCH_PYLOOP=1: the headline's calls from Python, one ctypes call a
# step (A/B against the C loop, host/steps.c)
PY_LOOP = os.environ.get("VIGPATH_BENCH_PYLOOP") == "1"
TRAFFIC_PROFILE = "r06ao_bench_traffic.json"  # rocprofv3 --pmc passes (tools/gpu_session.sh pmc)
DEV_MACS = [T.mac("02:00:00:00:00:00"), T.mac("02:00:00:00:00:01")]
NAT_ARGS = ["--expire", "60000000", "--starting-port", "0", "--wan", "1",
            "--extip", "192.168.4.2", "--eth-dest", "0,90:e2:ba:55:12:20",
            "--eth-dest", "1,90:e2:ba:55:12:21"]


def _s64(c: int) -> int:
    return c - (1 << 64) if c >= 1 << 63 else c


def _shr(z, k: int):  # logical shift right of int64 lanes holding u64 bits
    return (z >> k) & ((1 << (64 - k)) - 1)


def uniform_flows(p, n_flows: int, seed: int = 0x5EED):
    """SURVEY.md §8(d) secondary order on the device: flow =
    splitmix64(seed, p) mod N (traces.flow_order "uniform"), u64 arithmetic
    in int64 lanes; N a power of two."""
    assert n_flows & (n_flows - 1) == 0
    z = (p + 1) * _s64(0x9E3779B97F4A7C15) + seed
    z = (z ^ _shr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _shr(z, 27)) * _s64(0x94D049BB133111EB)
    return (z ^ _shr(z, 31)) & (n_flows - 1)


def frame_len_for(slot: int) -> int:
    """The bench's frame in a `slot`-byte slot: 60 B in 64 (a 64 B wire
    frame less its FCS), up to 1514 B (1518 B on the wire)."""
    return min(slot, 1518) - 4


class FlowBank:
    """Per-flow header bytes of the synthetic trace, on the device: bytes
    24-37 (IPv4 checksum, addresses, ports) of flow i's frame. Default keys:
    the bench flows (10.0.0.0 + (i >> 16) : i & 0xFFFF -> 0.0.0.0:0,
    SURVEY.md §8(d)); `keys` = (src_ip, dst_ip, src_port, dst_port) arrays
    (traces.random_flow_keys). Wider slots carry a fixed payload pattern (the
    L4 checksum sums it); 64-byte slots the reference's zero payload."""

    def __init__(self, n_flows: int, flow_base: int, dev, slot: int = 64, keys=None):
        fl = np.arange(flow_base, flow_base + n_flows, dtype=np.int64)
        if keys is None:
            z = np.zeros_like(fl)
            keys = (T.ip4(10, 0, 0, 0) + (fl >> 16), z, fl & 0xFFFF, z)
        flen = frame_len_for(slot)
        f, _ = T.udp_frames(*keys, slot=slot, frame_len=flen)
        f = f.reshape(n_flows, slot)
        tmpl = f[0].copy()
        if slot > 64:  # (64 B: the reference's zero payload, bench.lua:61-71)
            tmpl[42:flen] = (np.arange(42, flen) * 7 % 251).astype(np.uint8)
        self.template = torch.from_numpy(tmpl).to(dev)
        self.var = torch.from_numpy(np.ascontiguousarray(f[:, 24:38])).to(dev)
        self.n = n_flows
        self.slot = slot
        self.frame_len = flen

    def fill_flows(self, frames: torch.Tensor, fl: torch.Tensor):
        """Slot j of `frames` = the frame of flow fl[j]."""
        S = self.slot
        B = frames.shape[0] // S
        fv = frames.view(B, S)
        fv.copy_(self.template.expand(B, S))
        fv[:, 24:38] = self.var.index_select(0, fl)

    def fill(self, frames: torch.Tensor, start: int, order: str = "rr"):
        B = frames.shape[0] // self.slot
        p = torch.arange(start, start + B, device=frames.device)
        self.fill_flows(frames, uniform_flows(p, self.n) if order == "uniform" else p % self.n)


def verify_sample(frames: torch.Tensor, slot: int, ext_ip: int, k: int = 4096):
    """Size-independent check of a processed wide-slot batch (no oracle on
    the timed path): k frames spread over the batch carry the external
    source address, and their IPv4 header and UDP checksums verify (RFC 791
    / 768 ones-complement sums over the rewritten bytes = 0xFFFF)."""
    B = frames.numel() // slot
    idx = torch.linspace(0, B - 1, steps=min(k, B), device=frames.device).long()
    f = frames.view(B, slot).index_select(0, idx).cpu().numpy().astype(np.uint32)
    w = lambda a, o: (a[:, o] << 8) | a[:, o + 1]  # noqa: E731 (big-endian word)

    def fold(s):
        s = (s & 0xFFFF) + (s >> 16)
        return (s & 0xFFFF) + (s >> 16)
    ip_sum = fold(sum(w(f, o) for o in range(14, 34, 2)))
    tl = w(f, 16)
    ok_ip = bool((ip_sum == 0xFFFF).all())
    # nat_main.c stores the host-order config value raw (little-endian bytes)
    src = (f[:, 29] << 24) | (f[:, 28] << 16) | (f[:, 27] << 8) | f[:, 26]
    ok_src = bool((src == ext_ip).all())
    l4 = tl - 20
    ok_l4 = True
    for r in range(f.shape[0]):
        n = int(l4[r])
        seg = f[r, 34:34 + n]
        if n & 1:
            seg = np.append(seg, 0)
        s = int((seg[0::2] << 8 | seg[1::2]).sum())
        s += int(w(f[r:r + 1], 26)[0] + w(f[r:r + 1], 28)[0] + w(f[r:r + 1], 30)[0] +
                 w(f[r:r + 1], 32)[0] + 17 + n)
        if fold(np.uint32(s % (1 << 32))) != 0xFFFF:
            ok_l4 = False
            break
    return {"frames_checked": int(f.shape[0]), "ip_checksum_ok": ok_ip,
            "udp_checksum_ok": ok_l4, "src_is_external": ok_src,
            "match": ok_ip and ok_l4 and ok_src}


CPU_SAMPLES = 5


def cpu_baseline(n_flows: int, sample: int):
    """The oracle (clean-room restatement of nf.c + vignat + libVig) on one
    core over the same trace shape, built on this host with the reference's
    flags (-O3 -march=native, hardware crc32: oracle/Makefile `native`): warm
    every flow, then time CPU_SAMPLES samples of sample / CPU_SAMPLES
    steady-state packets each. Returns (median Mpps, [Mpps per sample],
    packets, core)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc

    cfg = orc.nat_cfg(wan=1, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=60_000_000, max_flows=n_flows,
                      device_macs=DEV_MACS,
                      endpoint_macs=[T.mac("90:e2:ba:55:12:20"),
                                     T.mac("90:e2:ba:55:12:21")])
    o = orc.Oracle("nat", cfg, ref="native")
    fr, ln, dv, now = T.nat_lan_trace(n_flows, n_flows)
    # one core, as the reference runs (nf.c:38, 142; SURVEY.md §8(d) taskset):
    # this thread is pinned to the first CPU it may use while it runs
    mask = os.sched_getaffinity(0)
    core = min(mask)
    os.sched_setaffinity(0, {core})
    rates = []
    try:
        o.run(fr, ln, dv, now, SLOT)
        per = max(1, sample // CPU_SAMPLES)
        pos = n_flows
        for _ in range(CPU_SAMPLES + 1):  # the first sample is a warm-up
            fr, ln, dv, now = T.nat_lan_trace(per, n_flows, start=pos)
            t0 = time.perf_counter()
            o.run(fr, ln, dv, now, SLOT)
            rates.append(per / (time.perf_counter() - t0) / 1e6)
            pos += per
    finally:
        os.sched_setaffinity(0, mask)
    warm, rates = rates[0], rates[1:]
    return float(np.median(rates)), rates, per * CPU_SAMPLES, core, warm


CONFIG1_FLOWS, CONFIG1_MAX_FLOWS, CONFIG1_PACKETS = 1000, 65536, 10_000_000


def cpu_config1():
    """BASELINE configs[0]: vignat over the 64 B
    trace of 1,000 flows round robin, --max-flows 65536, 10M packets, on one
    pinned core -- the oracle restatement of nf.c's loop (nf.c:150-176), as
    cpu_baseline. The flows are allocated by an untimed first pass; then
    CPU_SAMPLES + 1 samples of CONFIG1_PACKETS / CPU_SAMPLES packets (the
    first discarded as a warm-up). A sample's frames are the same 2,000
    rounds over the flows each time (a fresh copy: the loop rewrites them),
    its times continue the trace's. Returns the line's dict."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc

    cfg = orc.nat_cfg(wan=1, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=60_000_000, max_flows=CONFIG1_MAX_FLOWS,
                      device_macs=DEV_MACS,
                      endpoint_macs=[T.mac("90:e2:ba:55:12:20"),
                                     T.mac("90:e2:ba:55:12:21")])
    o = orc.Oracle("nat", cfg, ref="native")
    N = CONFIG1_FLOWS
    per = CONFIG1_PACKETS // CPU_SAMPLES // N * N
    fr0, ln0, dv0, now0 = T.nat_lan_trace(N, N)
    frs, ln, dv, nows = T.nat_lan_trace(per, N, start=N)
    mask = os.sched_getaffinity(0)
    core = min(mask)
    os.sched_setaffinity(0, {core})
    rates = []
    try:
        o.run(fr0, ln0, dv0, now0, SLOT)
        for k in range(CPU_SAMPLES + 1):
            fr = frs.copy()
            now = nows + k * per
            t0 = time.perf_counter()
            out = o.run(fr, ln, dv, now, SLOT)
            rates.append(per / (time.perf_counter() - t0) / 1e6)
            assert (out == 1).all()
    finally:
        os.sched_setaffinity(0, mask)
    warm, rates = rates[0], rates[1:]
    med = float(np.median(rates))
    return {"value": round(med, 3), "unit": "Mpps", "cores": 1, "kind": "port",
            "samples": [round(r, 3) for r in rates], "warmup_sample": round(warm, 3),
            "spread": round((max(rates) - min(rates)) / med, 4),
            "workload": "vignat 64B synthetic trace, %d flows round robin, --max-flows %d, "
                        "CPU nf.c loop (BASELINE configs[0])" % (N, CONFIG1_MAX_FLOWS),
            "sample": "median of %d samples of %d packets after one discarded warm-up "
                      "sample (%d packets timed in all); oracle restatement -O3 "
                      "-march=native, 1 thread pinned to cpu %d (%s)"
                      % (len(rates), per, per * len(rates), core, cpu_model())}


def golden_batch_digest(flows: int, batch: int):
    """The reference's digest of one steady-state batch of this exact shape
    (tests/golden/nat_bench_shape.npz, made by tests/golden/make_golden.py
    from the oracle over the reference's own libVig), or None."""
    path = os.path.join(ROOT, "tests", "golden", "nat_bench_shape.npz")
    if not os.path.exists(path) or flows != 1 << 20 or batch != 1 << 24:
        return None
    with np.load(path, allow_pickle=False) as z:
        return int(z["batch_digest"][-1])


OWN_CHUNK = 1 << 21  # packets per rank and chunk of the chunked owner pipeline (N > 1)

E2E_BATCH = 1 << 24
E2E_CHUNK = 1 << 21


def end_to_end(nat, bank, dev, start: int, steps: int = 3):
    """The path's real ends (SURVEY.md §8(d) "End-to-end"; nf.c:153,166):
    frames and the per-packet arrays start and end in page-locked host memory
    (a registered mbuf pool: DPDK keeps mbufs in hugepages);
    vp_process_host_batch moves them over PCIe in E2E_CHUNK-packet chunks,
    host->device and device->host on two copy streams beside the compute
    stream, three buffer sets in HBM (the H2D copy runs two chunks ahead). Time is the bench's affine now_p = NOW0 + p
    (SURVEY.md §8(d)), so no time array crosses PCIe. Every flow is already
    warm; one untimed batch allocates the staging buffers. Returns Mpps over
    `steps` host batches of E2E_BATCH."""
    os.environ["VIGPATH_HOST_CHUNK"] = str(E2E_CHUNK)
    B = E2E_BATCH
    pin = lambda t: t.pin_memory().numpy()  # noqa: E731
    lens = pin(torch.full((B,), 60, dtype=torch.int16))
    ind = pin(torch.zeros(B, dtype=torch.int16))
    out = pin(torch.zeros(B, dtype=torch.int16))
    d = torch.empty(B * SLOT, dtype=torch.uint8, device=dev)
    bufs = []
    for k in range(steps + 1):  # batch 0 warms the staging buffers up, untimed
        bank.fill(d, start + k * B)
        bufs.append(pin(d.cpu()))
    del d
    torch.cuda.synchronize()

    def host_step(k):
        nat.process_host_batch(bufs[k], lens, ind, out, SLOT, now0=T.NOW0 + start + k * B,
                               now_step=1)
    host_step(0)
    t0 = time.perf_counter()
    for k in range(1, steps + 1):
        host_step(k)
    el = time.perf_counter() - t0
    assert (out == 1).all()
    return B * steps / el / 1e6


MBUF_BATCH = 1 << 22
IMIX = ((7, 60), (4, 566), (1, 1514))  # 7:4:1 of 64 / 570 / 1518-byte wire frames


def imix_lengths(p: np.ndarray) -> np.ndarray:
    """Frame length of packet p in the mixed-size burst: IMIX 7:4:1."""
    r = p % 12
    return np.where(r < 7, 60, np.where(r < 11, 566, 1514)).astype(np.uint16)


def end_to_end_mbuf(nat, bank, dev, start: int, steps: int = 3, imix: bool = False):
    """SURVEY.md §8(d) "End-to-end" in DPDK's own shape (nf.c:186-214): every
    frame in its own mbuf of a pool in page-locked host memory (2304-byte
    elements: a 128-byte rte_mbuf, 128 B headroom and a 2 KB data room, the
    frame at data_off 256; traces.MbufPool), registered once with
    vp_register_host, and a batch = the data pointers of MBUF_BATCH packets in
    rx order (a random permutation of the pool: a mempool hands buffers back
    in no particular order), their lengths and ports. vp_process_mbufs reads
    each frame's first 64 bytes, and the bytes its L4 checksum covers past
    them, from host memory on the GPU, processes them and writes the
    rewritten header bytes back (vp_mbuf.hip). Frames: the bench trace (64 B,
    round robin over the warm flows), or IMIX 7:4:1 of 60 / 566 / 1514-byte
    frames (random payload past 64 B). The pool's frames are refilled
    between steps (untimed); each call is timed alone, its inputs in host
    memory when it starts and its results there when it returns. Returns a
    dict for the bench line."""
    import torch
    B = MBUF_BATCH
    rng = np.random.default_rng(7)
    pool = T.MbufPool(B, pinned=True)
    bufs = rng.permutation(B)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa
    ptrs = pin(pool.ptrs(bufs))
    lens = pin(imix_lengths(np.arange(B)) if imix else np.full(B, 60, np.uint16))
    ind = pin(np.zeros(B, np.uint16))
    out = pin(np.zeros(B, np.uint16))
    if imix:  # payload past byte 64, the same in every step (never rewritten)
        pool.rows[:, 256 + 64:] = rng.integers(0, 256, (1, pool.stride - 256 - 64),
                                               dtype=np.uint8)
    tl = lens.astype(np.int64) - 14
    hdr = np.empty((B, 64), np.uint8)
    d = torch.empty(B * SLOT, dtype=torch.uint8, device=dev)
    nat.register_host(pool.mem)
    call = nat.mbuf_step(ptrs, lens, ind, out)
    times = []
    try:
        for k in range(steps + 1):  # step 0 allocates the staging, untimed
            p0 = start + k * B
            bank.fill(d, p0)
            hdr[:] = d.view(B, SLOT).cpu().numpy()
            if imix:  # total_length and the UDP length of each frame
                hdr[:, 16] = (tl >> 8).astype(np.uint8)
                hdr[:, 17] = (tl & 0xFF).astype(np.uint8)
                hdr[:, 38] = ((tl - 20) >> 8).astype(np.uint8)
                hdr[:, 39] = ((tl - 20) & 0xFF).astype(np.uint8)
            pool.rows[bufs, 256:256 + 64] = hdr
            t0 = time.perf_counter()
            call(T.NOW0 + p0, 1)
            el = time.perf_counter() - t0
            if k:
                times.append(el)
        assert (out == 1).all()
        # property check of a sample of the last batch, read back from the
        # mbufs: IPv4 and UDP checksums verify over each frame's bytes, the
        # source is the external address
        idx = np.linspace(0, B - 1, 2048).astype(np.int64)
        smp = np.zeros((len(idx), 2048), np.uint8)
        for j, i in enumerate(idx):
            L = int(lens[i])
            smp[j, :L] = pool.rows[bufs[i], 256:256 + L]
        chk = verify_sample(torch.from_numpy(smp.reshape(-1)), 2048, T.ip4(192, 168, 4, 2),
                            k=len(idx))
    finally:
        nat.unregister_host(pool.mem)
    el = sum(times)
    mpps = B * len(times) / el / 1e6
    avg = float(lens.mean())
    pin_in = 8 + 2 + 2 + float(np.mean(np.maximum(64, (lens.astype(np.int64) + 15) // 16 * 16)))
    pin_out = 2 + float(np.mean(np.minimum(lens, 64)))
    return {"value": round(mpps, 1), "unit": "Mpps",
            "gbit_per_s": round(mpps * 1e6 * avg * 8 / 1e9, 1),
            "frames": ("IMIX 7:4:1 of 60/566/1514 B (mean %.1f B)" % avg) if imix
                      else "64 B (60 B + FCS), the bench trace",
            "path": "page-locked mbuf pool (2304-byte elements, data_off 256), pointer "
                    "array in shuffled rx order -> vp_process_mbufs: GPU reads each "
                    "frame's header (+ the L4-summed bytes past 64) from host memory, "
                    "processes 64-byte header slots, writes the rewritten bytes back "
                    "(vp_mbuf.hip)",
            "batch_packets": B, "steps": len(times),
            "ms_per_batch": round(el / len(times) * 1e3, 3),
            "pcie_bytes_per_packet": {"in": round(pin_in, 1), "out": round(pin_out, 1)},
            "parity": chk}


# ------------------------------------------------------ extra workloads --
# BASELINE configs[2] and [3] and two vignat variants,
# each a steady state at 2^24 packets per step like the headline, its last
# timed batch checked against the reference's digest of that exact batch
# (tests/golden/bench_configs.npz, made by tests/golden/make_bench_golden.py
# with the oracle glue over the reference's own libVig).
EXTRA_STEPS = 8
LB_MACS = [bytes([0x10 * d + i for i in range(6)]) for d in range(3)]


def golden_configs():
    path = os.path.join(ROOT, "tests", "golden", "bench_configs.npz")
    if not os.path.exists(path):
        return {}
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


# vignat's 64-byte classify kernel on one GPU: one 1024-thread block per CU
# (vp_nat.hip nat_classify64w) unless VIGPATH_BLOCK_WAVES=4
NAT64 = "nat_classify64" if os.environ.get("VIGPATH_BLOCK_WAVES") == "4" else "nat_classify64w"


def steady_workload(nf, batch_of, warm: int, steps: int, B: int, dev, golden=None,
                    kernel="", times=None, state=None, repeats=False, alg_bytes=ALG_BYTES,
                    basis=None):
    """Batches 0 .. warm-1 untimed (allocation), then `steps` timed calls
    (batches warm ..) without timing events, each from its own buffer filled
    before the timed region; the last timed batch's digest against golden[k]
    (the reference's digest of batch k); then a kernel-timing pass over the
    next `steps` batches. batch_of(k, buf) fills buf (B * 64 bytes) with batch
    k's frames and returns (lens, in_dev, now0, now_step) device tensors /
    ints. repeats: every batch from 1 on is batch 1 again (same frames, later
    times, same outputs), so the last golden digest stands for them all.
    Returns the line's dict."""
    out = torch.zeros(B, dtype=torch.int16, device=dev)

    knames = {}

    def run(k0, n, events):
        nf.kernel_timing(events)
        bufs, args = [], []
        for k in range(k0, k0 + n):
            b = torch.empty(B * SLOT, dtype=torch.uint8, device=dev)
            args.append(batch_of(k, b))
            bufs.append(b)
        kms = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b, (ln, ind, n0, st) in zip(bufs, args):
            nf.process_device(b, ln, ind, out, SLOT, now0=n0, now_step=st)
            if events:
                kms.append(nf.last_kernel_ms())
                kn = nf.last_kernel()
                knames[kn] = knames.get(kn, 0) + 1
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        nf.kernel_timing(False)
        return el, kms, bufs[-1]

    t0 = time.perf_counter()
    run(0, warm, False)
    warm_s = time.perf_counter() - t0
    el, _, last = run(warm, steps, False)
    k_last = warm + steps - 1
    k_gold = min(k_last, len(golden) - 1) if golden is not None and repeats else k_last
    parity = None
    if golden is not None and k_gold < len(golden):
        got = T.batch_digest(last.cpu().numpy(), out.cpu().numpy().view(np.uint16), SLOT)
        want = int(golden[k_gold])
        parity = {"batch": k_last, "golden_batch": k_gold, "batch_digest": "%016x" % got, "golden": "%016x" % want,
                  "match": got == want,
                  "source": "tests/golden/bench_configs.npz (reference libVig)"}
        if state is not None and k_last == len(golden) - 1:  # (vignat: dchain state)
            alloc, ts, _ = nf.dump()
            sd = T.state_digest(alloc, ts)
            parity.update({"state_digest": "%016x" % sd, "state_golden": "%016x" % int(state),
                           "state_match": sd == int(state)})
    del last
    _, kms, last = run(warm + steps, steps, True)
    del last
    per_launch_s, pkts, achieved = kernel_rate(kms, B, steps, alg_bytes)
    mpps = B * steps / el / 1e6
    line = {"value": round(mpps, 1), "unit": "Mpps", "ms_per_step": round(el / steps * 1e3, 4),
            "batch_packets": B, "steps": steps, "warm_batches": warm,
            "warm_s": round(warm_s, 2),
            "kernel": kernel_label(knames, kernel),
            "kernel_ms_per_launch": round(per_launch_s * 1e3, 4),
            "kernel_ms_per_step": round(per_launch_s * 1e3 * pkts / B, 4),
            "kernel_mpps": round(pkts / per_launch_s / 1e6, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "frac_step": round(mpps * 1e6 * alg_bytes / 1e9 / HBM_PEAK_GBS, 4),
            "frac_basis": basis or "%d B per packet (SURVEY.md §8(d) vignat basis%s), 8 TB/s"
                          % (alg_bytes, "" if alg_bytes == ALG_BYTES
                             else ", no per-packet port: one per burst"),
            "alg_bytes_per_packet": alg_bytes,
            "parity": parity}
    if times is not None:
        line.update(times)
    return line


def host_batch(dev, frames, lens, in_dev):
    """A host-generated batch on the device (frames, lens, in_dev tensors)."""
    return (torch.from_numpy(frames).to(dev),
            torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev),
            torch.from_numpy(in_dev.astype(np.uint16).view(np.int16)).to(dev))


# vigbridge per packet (bridge_main.c:39-62,272-290): the two MACs (one
# 16-byte chunk of the slot), the port, and two map lookups (src learn, dst
# forward) of key + tag + value each
BRIDGE_ALG_BYTES = 16 + 2 + 2 * (8 + 4 + 4)


def bench_bridge_c3(dev, B, steps, golden):
    """BASELINE configs[2]: vigbridge 64 B, 1M MACs (traces.bridge_trace:
    station k on port k & 1, frame p from station p mod N to p + N/2). Batch
    0 learns every station; from batch 1 on every frame hits (the batches'
    frames are the same, their times advance)."""
    N = 1 << 20
    cfg = vigor_amd.bridge_config_from_args(["--capacity", str(N), "--expire", "60000000"], 2)
    br = vigor_amd.Bridge(cfg, gpu=0)
    fr, ln, dv, _ = T.bridge_trace(B, N)
    src, lens, ind = host_batch(dev, fr, ln, dv)
    del fr

    def batch_of(k, buf):
        buf.copy_(src)
        return lens, ind, T.NOW0 + k * B, 1
    r = steady_workload(br, batch_of, 1, steps, B, dev, golden, "bridge_classify",
                        repeats=True, alg_bytes=BRIDGE_ALG_BYTES,
                        basis="%d B per packet, vigbridge's own reads: 16 B (the frame's "
                              "first chunk: both MACs) + 2 B port + 2 lookups x (8 B MAC key "
                              "+ 4 B tag + 4 B value); it writes no frame (2 B out port), "
                              "so its ceiling is the read-only shape (shape_read_ms); 8 TB/s"
                              % BRIDGE_ALG_BYTES)
    br.close()
    r["workload"] = "vigbridge 64B, 1M MACs, learn + lookup (BASELINE configs[2])"
    return r


def bench_lb_c4(dev, B, steps, golden):
    """BASELINE configs[3]: viglb 64 B, 256 backends (heartbeats first) / 1M
    flows (traces.lb_traffic on port 2)."""
    N = 1 << 20
    argv = ["--flow-capacity", str(N), "--backend-capacity", "256", "--cht-height", "257",
            "--flow-expiration", "60000000", "--backend-expiration", "3600000000",
            "--wan", "2"]
    lb = vigor_amd.Lb(vigor_amd.lb_config_from_args(argv, 3, LB_MACS), gpu=0)
    hb = T.lb_heartbeats(256)
    f0, l0, d0 = host_batch(dev, hb[0], hb[1], hb[2])
    lb.process_device(f0, l0, d0, torch.zeros(256, dtype=torch.int16, device=dev), SLOT,
                      now=torch.from_numpy(hb[3]).to(dev))
    fr, ln, dv, _ = T.lb_traffic(B, N)
    src, lens, ind = host_batch(dev, fr, ln, dv)
    del fr
    # every packet arrives on the WAN port: one port per burst (in_port)
    port = int(dv[0]) if (dv == dv[0]).all() else ind

    def batch_of(k, buf):
        buf.copy_(src)
        return lens, port, T.NOW0 + k * B, 1
    r = steady_workload(lb, batch_of, 1, steps, B, dev, golden, "lb_classify64",
                        repeats=True, alg_bytes=ALG_BYTES - (2 if isinstance(port, int) else 0))
    lb.close()
    r["workload"] = "viglb 64B, 256 backends / 1M flows (BASELINE configs[3])"
    return r


def make_nat(flows, expire_us=60_000_000):
    args = [a for a in NAT_ARGS]
    args[args.index("--expire") + 1] = str(expire_us)
    cfg = vigor_amd.nat_config_from_args(args + ["--max-flows", str(flows)], 2, DEV_MACS)
    return vigor_amd.Nat(cfg, gpu=0)


def bench_nat_random(dev, B, steps, golden):
    """vignat 64 B, 1M flows whose 5-tuples have no counter structure
    (traces.random_flow_keys), round robin: the allocation-order layout does
    not fit them, the table keeps the CRC bits."""
    N = 1 << 20
    nat = make_nat(N)
    bank = FlowBank(N, 0, dev, keys=T.random_flow_keys(N))
    lens = torch.full((B,), 60, dtype=torch.int16, device=dev)
    ind = torch.zeros(B, dtype=torch.int16, device=dev)

    def batch_of(k, buf):
        bank.fill(buf, k * B)
        return lens, ind, T.NOW0 + k * B, 1
    r = steady_workload(nat, batch_of, 1, steps, B, dev, golden, NAT64,
                        repeats=True)
    r["table_layout"] = nat.table_stats()["layout"]
    nat.close()
    r["workload"] = "vignat 64B, 1M flows with random 5-tuples, round robin"
    return r


def bench_nat_churn(dev, B, steps, golden, state=None):
    """vignat 64 B with steady turnover at the reference's latency-run expiry
    (1 s, run-middlebox.sh:16; traces.churn_trace): 2^18 flow slots round
    robin, a quarter of them starting new flows every batch while the flows
    they retire expire 1 s after their last packet; one timestamp per batch
    (250 ms apart; nf.c stamps a polling sweep with one current_time(),
    nf.c:56). Per steady batch: 65,536 new flows allocated (phase B) and
    65,536 expired at its first packet (expire_items_single_map,
    expirator.c:110-218), every other packet a hit."""
    W = T.CHURN_W
    nat = make_nat(1 << 20, T.CHURN_EXPIRE_US)
    warm = 8
    epochs = (warm + 2 * steps + 3) // 4 + 1
    bank = FlowBank(epochs * W, 0, dev)
    lens = torch.full((B,), 60, dtype=torch.int16, device=dev)
    ind = torch.zeros(B, dtype=torch.int16, device=dev)
    p = torch.arange(B, device=dev)
    slot_id = p % W

    def batch_of(k, buf):
        bank.fill_flows(buf, (k + slot_id % 4) // 4 * W + slot_id)
        return lens, ind, T.NOW0 + k * T.CHURN_DT, 0
    r = steady_workload(nat, batch_of, warm, steps, B, dev, golden, NAT64,
                        state=state)
    r["live_flows"] = nat.live_count()
    nat.close()
    r["workload"] = ("vignat 64B, steady turnover at 1 s expiry: 2^18 flows round robin, "
                     "65,536 new and 65,536 expiring per 2^24-packet batch")
    return r


def per_packet_drop_in(packets: int = 20000, flows: int = 1024, batches=(0, 32, 1024),
                       mark=lambda name: None):
    """north_star's "drops into nf.c's main loop unchanged", timed: host/nf_loop
    (nf.c:143-216 restated over a trace file, linked against
    libvignat_nf.so) with every packet through nf_process one at a time
    (batch 0: nf.c:150-176, VIGOR_BATCH_SIZE == 1), and through the batched
    form (vp_process_batch, nf.c:178-215) for comparison. The trace: `flows`
    flows allocated by an untimed warm-up (--warm), then `packets` steady
    hits round robin, each with its own time stamp. Host frames in pageable
    memory, as nf.c's mbuf data would be to a library that did not register
    the pool. Returns {batch: {us_per_packet, kpps}}."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "host", "nf_loop")
    n = flows + packets
    fr, ln, dv, now = T.nat_lan_trace(n, flows)
    res = {}
    with tempfile.TemporaryDirectory() as d:
        tin, tout = os.path.join(d, "t.in"), os.path.join(d, "t.out")
        with open(tin, "wb") as f:
            f.write(b"VPTR" + np.array([n, SLOT], np.uint32).tobytes())
            f.write(dv.astype(np.uint16).tobytes() + ln.astype(np.uint16).tobytes())
            f.write(now.astype(np.int64).tobytes() + fr.tobytes())
        for bt in batches:
            mark("per-packet drop-in: batch %d" % bt)
            cmd = [exe, tin, tout, "--warm", str(flows)] + (["--batch", str(bt)] if bt else [])
            r = subprocess.run(cmd + ["--"] + NAT_ARGS + ["--max-flows", str(flows)],
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError("nf_loop failed: %s" % r.stderr[-500:])
            line = [x for x in r.stderr.splitlines() if x.startswith("timed ")][-1]
            us = float(line.split(",")[1].split()[0])
            res["per_packet" if bt == 0 else "batch_%d" % bt] = {
                "us_per_packet": round(us, 3), "kpps": round(1e3 / us, 2)}
            prof = [x for x in r.stderr.splitlines() if x.startswith("vigpath serve")]
            if prof:  # (VIGPATH_SERVE_PROF=1: vp_process_one's stage times)
                res["per_packet" if bt == 0 else "batch_%d" % bt]["serve_prof"] = prof[-1]
            out = np.frombuffer(open(tout, "rb").read(), np.uint16, n, 12)
            assert (out[flows:] == 1).all()  # every steady packet out on the WAN port
    return res


def launch_ranks(n: int) -> int:
    """--gpus N > 1 without a torch.distributed environment: start one rank
    per GPU as child processes (torch.distributed.run), before anything here
    touches the GPU, and return their exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def timed_steps(nat, bank, dev, lens, in_dev, out, B, slot, world, rank, first, steps,
                order="rr", host_comm=False, stages=None, wd=None, label="timed",
                knames=None):
    """Fill one buffer per step (batches first .. first + steps - 1 of this
    rank's slices, `order`), then time exactly `steps` prepared
    vp_process_device calls between barriers + synchronisations. Returns
    (elapsed s, max over ranks; [(kernel ms, launches)] per step; buffers).
    wd: the N > 1 watchdog (vigor_amd.watchdog), one marker per step.
    knames: a dict counting the tile kernel each step launched last
    (vp_last_kernel)."""
    mark = wd.stage if wd is not None else (lambda name: None)
    def gstart(k):  # global position of this rank's slice of global batch k
        return (k * world + rank) * B
    bufs = []
    for k in range(steps):
        b = torch.empty(B * slot, dtype=torch.uint8, device=dev)
        bank.fill(b, gstart(first + k), order)
        bufs.append(b)
    # the headline pass: the calls in a C loop (host/steps.c), as nf.c makes
    # them; the timing pass reads per-step values back between calls (Python)
    c_loop = knames is None and stages is None and not PY_LOOP
    if c_loop:
        run = nat.device_steps(bufs, lens, in_dev, out, slot)
        nows = [T.NOW0 + gstart(first + k) for k in range(steps)]
    else:
        calls = [nat.device_step(b, lens, in_dev, out, slot) for b in bufs]
    torch.cuda.synchronize()
    kms = []
    mark("%s: barrier" % label)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if c_loop:
        mark("%s: %d steps (C loop)" % (label, steps))
        run(nows, 1)
    for k in range(0 if c_loop else steps):
        mark("%s: step %d/%d" % (label, k + 1, steps))
        calls[k](T.NOW0 + gstart(first + k), 1)
        kms.append(nat.last_kernel_ms())
        if knames is not None:
            kn = nat.last_kernel()
            knames[kn] = knames.get(kn, 0) + 1
        if stages is not None:  # owner mode's phase-A stages (timing pass)
            for name, ms in nat.last_stage_ms().items():
                stages[name] = stages.get(name, 0.0) + ms / steps
    mark("%s: end barrier" % label)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cpu" if host_comm else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # every packet hit (steady state) and went out on the WAN port
    assert int((out != 1).sum().item()) == 0
    return elapsed, kms, bufs


def shape_ceiling(L, B, slot, dev, reps=10, waves=4):
    """vp_probe_slots_w over a scratch batch of B slots with the tile
    kernel's block shape (`waves` per block): (read+write ms, read ms) per
    pass, each the mean of `reps` launches timed like the classify kernel
    (its dispatch's own timestamps)."""
    import ctypes
    buf = torch.zeros(B * slot, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    out = []
    for store in (1, 0):
        ms = ctypes.c_float()
        vigor_amd._check(L.vp_probe_slots_w(ctypes.c_void_p(buf.data_ptr()), B, slot, store,
                                            waves, reps, ctypes.byref(ms)), "vp_probe_slots_w", L)
        out.append(float(ms.value))
    out.append(waves)
    del buf
    torch.cuda.empty_cache()
    return out


def ceiling_fields(ceiling, kernel_s, step_s):
    rw, rd, waves = ceiling
    return {"shape_ceiling_ms": round(rw, 4), "shape_read_ms": round(rd, 4),
            "kernel_over_ceiling": round(kernel_s * 1e3 / rw, 4),
            "step_over_ceiling": round(step_s * 1e3 / rw, 4),
            "shape_ceiling_source": "vp_probe_slots_w on this box: the tile kernel's "
                                    "persistent grid (%d-thread blocks, %d per CU; tile "
                                    "order VIGPATH_SPLIT=%s) and 1 KiB access shape, every "
                                    "slot read and written back whole (write-through), no "
                                    "other work; shape_read_ms the same without the stores"
                                    % (64 * waves, max(1, 16 // waves),
                                       os.environ.get("VIGPATH_SPLIT", "1"))}


def kernel_label(knames, default):
    """The tile kernel(s) a pass ran: one name, or "a x3 + b x17" when the
    per-segment choice changed within the pass."""
    knames = {k: v for k, v in (knames or {}).items() if k}
    if not knames:
        return default
    if len(knames) == 1:
        return next(iter(knames))
    return " + ".join("%s x%d" % kv for kv in sorted(knames.items(), key=lambda kv: -kv[1]))


def probe_waves(kernel: str) -> int:
    """Waves per block of the tile kernel's grid (vp_probe_slots_w)."""
    k = kernel.split(" ")[0]
    if k.startswith("nat_classify64h"):
        return 8
    if k.startswith("nat_classify64q"):
        return 4
    return 16 if k.startswith("nat_classify64w") or k.endswith("64w") else 4


def kernel_rate(kms, B, steps, alg_bytes):
    """(per-launch s, packets per launch, achieved algorithmic GB/s)."""
    launches = sum(k for _, k in kms)
    per_launch_s = max(1e-12, sum(m for m, _ in kms) / 1e3 / max(1, launches))
    pkts = B * steps / max(1, launches)
    return per_launch_s, pkts, alg_bytes * pkts / per_launch_s / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None,
                    help="packets per GPU and step (default 2^24, at most "
                         "2 GiB of slots)")
    ap.add_argument("--slot", type=int, default=SLOT,
                    help="slot bytes (frames of min(slot, 1518) - 4 bytes): "
                         "64 is BASELINE's config; wider slots measure the "
                         "65-1518 B frames of north_star (R = slot + 28)")
    ap.add_argument("--order", choices=("rr", "uniform"), default="rr",
                    help="packet order (SURVEY.md §8(d)): round robin over "
                         "the flows (bench.lua:125, the headline) or uniform")
    ap.add_argument("--flows", type=int, default=None,
                    help="default: 1M (config 2) on one GPU, 16M (config 5) "
                         "over N > 1 GPUs")
    ap.add_argument("--cpu-sample", type=int, default=1 << 26)
    ap.add_argument("--shard-mode", choices=("owner", "replicated"), default="owner",
                    help="N > 1: flow dictionary sharded by flow hash with an "
                         "all-to-all of keys and answers (owner, north_star's "
                         "design: the headline value) or replicated on every "
                         "GPU; the other mode is measured too (extra key "
                         "other_shard_mode) unless --no-extra")
    ap.add_argument("--route-all", action="store_true",
                    help="profiling: one GPU running the owner-mode pipeline "
                         "with every LAN key sent through the (single-rank "
                         "RCCL) exchange (VIGPATH_ROUTE_ALL=1)")
    ap.add_argument("--port-array", action="store_true",
                    help="pass a per-packet port array instead of the burst's one port")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the host-resident end-to-end rate")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the secondary measurements (uniform order; "
                         "N > 1: the other dictionary placement)")
    args = ap.parse_args()
    slot = args.slot
    if slot < 64 or slot % 16:
        raise SystemExit("bench.py: --slot must be a multiple of 16, >= 64")
    B = args.batch
    if B is None:  # 2^24 packets of 64 B; wider slots up to 2 GiB per batch
        B = 1 << 24
        while B * slot > (1 << 31):
            B >>= 1
    # R = slot(len) + 28 (92 at 64 B), of which 2 B are the
    # per-packet port; a burst from one port (vp_dev_batch.in_port, nf.c's
    # rx bursts, nf.c:150-153) reads none: R = slot + 26
    port_array = args.port_array or args.gpus > 1 or args.route_all
    alg_bytes = slot + 28 - (0 if port_array else 2)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.flows is None:
        args.flows = 1 << 20 if world == 1 else 1 << 24
    # VIGPATH_COMM=host: every rank on GPU 0 with gloo host collectives (a
    # rehearsal of the N > 1 path on a one-GPU box); default RCCL
    host_comm = os.environ.get("VIGPATH_COMM", "rccl") == "host"
    if host_comm:
        local = 0
    # N > 1: flushed stage markers on every rank, and a watchdog that aborts
    # the collectives, prints a partial line and exits 3 after
    # VIGPATH_WATCHDOG_S seconds (default 240) without a new stage
    # (vigor_amd/watchdog.py); VIGPATH_STALL="rank:ms:call" rehearses it
    wd = None
    nat_ref = []  # the context the watchdog aborts
    if world > 1 or "VIGPATH_WATCHDOG_S" in os.environ:  # (one rank: rehearsals)
        from vigor_amd.watchdog import Watchdog
        wd = Watchdog(rank, world, float(os.environ.get("VIGPATH_WATCHDOG_S", "240")),
                      partial={"metric": METRIC, "unit": "Mpps", "higher_is_better": True,
                               "steps": args.steps, "warmup": args.warmup,
                               "config": {"shard_mode": args.shard_mode,
                                          "transport": "gloo (host)" if host_comm
                                          else "RCCL/xGMI"}},
                      abort=lambda: [n.L.vp_comm_abort(n.h) for n in nat_ref if n.h.value])
        wd.start()
        wd.stage("comm init (%s)" % ("gloo" if host_comm else "nccl"))
    mark = wd.stage if wd is not None else (lambda name: None)
    if world > 1:
        if host_comm:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl",
                                    device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    bank = FlowBank(args.flows, 0, dev, slot)
    lens = torch.full((B,), bank.frame_len, dtype=torch.int16, device=dev)
    # every packet of the workload arrives on LAN port 0: one port per burst
    # (--port-array: a per-packet port array, as before round 5; N > 1 ranks
    # take the array, which their exchange paths read)
    in_dev = torch.zeros(B, dtype=torch.int16, device=dev) if port_array else 0
    out = torch.zeros(B, dtype=torch.int16, device=dev)

    def make_nat(mode):
        cfg = vigor_amd.nat_config_from_args(
            NAT_ARGS + ["--max-flows", str(args.flows)], 2, DEV_MACS)
        nat = vigor_amd.Nat(cfg, gpu=local)
        if args.route_all and world == 1:  # the owner pipeline on one GPU
            import ctypes
            from vigor_amd import shard
            nat_ref.append(nat)
            os.environ["VIGPATH_ROUTE_ALL"] = "1"
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(shard.rccl_unique_id())
            vigor_amd._check(nat.L.vp_attach_rccl(nat.h, uid, 1, 0), "vp_attach_rccl", nat.L)
            shard.set_mode(nat, "owner")
        if world > 1:  # one vignat over all ranks
            from vigor_amd import shard
            mark("attach %s" % mode)
            nat_ref.append(nat)
            if host_comm:
                shard.attach_torch(nat, rank, world, mode=mode)
            else:
                shard.attach_rccl(nat, rank, world, mode=mode)
        return nat

    def warm(nat):
        """The first global batch allocates every flow (round robin: the
        allocation order of the reference's own traffic); returns the new-
        flow rate of batch 0 in Mpps."""
        wbuf = torch.empty(B * slot, dtype=torch.uint8, device=dev)
        rate = None
        for w in range(args.warmup):
            mark("warm-up batch %d/%d" % (w + 1, args.warmup))
            bank.fill(wbuf, (w * world + rank) * B)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nat.process_device(wbuf, lens, in_dev, out, slot,
                               now0=T.NOW0 + (w * world + rank) * B, now_step=1)
            torch.cuda.synchronize()
            if w == 0:
                rate = B * world / (time.perf_counter() - t0) / 1e6
        assert nat.live_count() == min(args.flows, B * world * max(1, args.warmup))
        return rate

    mode = args.shard_mode
    nat = make_nat(mode)
    new_flow_mpps = warm(nat)
    # the headline pass: no per-launch timing events (they cost a step about
    # 6 us of kernel-boundary time)
    elapsed, _, bufs = timed_steps(nat, bank, dev, lens, in_dev, out, B, slot, world,
                                   rank, args.warmup, args.steps, args.order, host_comm,
                                   wd=wd, label="timed")
    # the last timed batch, byte for byte, against the reference's output of
    # the same batch (after timing; the golden exists for the default shape);
    # wider slots: a size-independent check of a sample (checksums verify)
    want = (golden_batch_digest(args.flows, B)
            if world == 1 and slot == SLOT and args.order == "rr" else None)
    parity = None
    if want is not None:
        got = T.batch_digest(bufs[-1].cpu().numpy(), out.cpu().numpy().view(np.uint16),
                             SLOT)
        parity = {"batch_digest": "%016x" % got, "golden": "%016x" % want,
                  "match": got == want,
                  "source": "tests/golden/nat_bench_shape.npz (reference libVig)"}
        assert got == want, "timed batch differs from the reference: %s" % parity
    elif slot != SLOT:
        parity = verify_sample(bufs[-1], slot, T.ip4(192, 168, 4, 2))
        parity["source"] = "RFC 791/768 checksum verification of a sample (property)"
        assert parity["match"], parity
    del bufs
    mpps = B * args.steps * world / elapsed / 1e6
    # the kernel-timing pass: the next `steps` batches of the same workload,
    # each classify launch between HIP events on the stream it runs on
    nat.kernel_timing(True)
    owner_run = (world > 1 and mode == "owner") or args.route_all
    stages = {} if owner_run else None
    knames = {}
    el_k, kms, bufs = timed_steps(nat, bank, dev, lens, in_dev, out, B, slot, world, rank,
                                  args.warmup + args.steps, args.steps, args.order, host_comm,
                                  stages, wd=wd, label="kernel timing", knames=knames)
    del bufs
    stages_max = None
    if stages and world > 1:  # the slowest rank per stage
        mark("stage times all-reduce")
        names = sorted(stages)
        t = torch.tensor([stages[k] for k in names], dtype=torch.float64,
                         device="cpu" if host_comm else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        stages_max = {k: float(v) for k, v in zip(names, t.tolist())}
    per_launch_s, pkts_per_launch, achieved = kernel_rate(kms, B, args.steps, alg_bytes)
    # the classify tile's memory-shape ceiling on this box (vp_probe_slots:
    # the same grid and 1 KiB access shape, every slot read and written back
    # whole, nothing else), beside the kernel it bounds
    kname = kernel_label(knames, NAT64 if slot == SLOT else "nat_classify_wide")
    ceiling = None
    if world == 1 and slot in (64, 128) and not args.route_all:
        mark("shape ceiling probe")
        ceiling = shape_ceiling(nat.L, B, slot, dev, waves=probe_waves(kname) if slot == SLOT
                                else 4)
    traffic = None  # PMC bytes of the same kernel (profiles/, per launch)
    tpath = os.path.join(ROOT, "profiles", TRAFFIC_PROFILE)
    if (os.path.exists(tpath) and B == 1 << 24 and args.flows == 1 << 20
            and world == 1 and slot == SLOT and args.order == "rr"):
        with open(tpath) as fh:
            tb = json.load(fh)["traffic_bytes_per_launch"]
        traffic = round(tb * pkts_per_launch / (1 << 24) / per_launch_s / 1e9, 1)
    flen = bank.frame_len
    if world == 1 and args.flows == 1 << 20 and slot == SLOT and args.order == "rr":
        workload = ("vignat 64B, 1M flows, 1xMI355X (parse+hash+map-probe "
                    "kernel, checksum rewrite)")
    elif world > 1:
        via = "gloo (host)" if host_comm else "RCCL/xGMI"
        how = ("flow-hash sharded dictionary: keys owned by another GPU looked up "
               "through an all-to-all over %s" % via if mode == "owner"
               else "replicated dictionary over %s" % via)
        workload = ("vignat %dB, %d flows, %dxMI355X: one NF over all GPUs, "
                    "each ingesting a contiguous 1/%d of every global batch "
                    "(%s; new flows all-gathered)" % (flen, args.flows, world, world, how))
    else:
        workload = "vignat %dB frames in %dB slots, %d flows, %s order, 1xMI355X" % (
            flen, slot, args.flows, args.order)
    if args.route_all:
        workload = ("vignat %dB, %d flows, 1xMI355X, owner-mode pipeline with every key "
                    "routed through a one-rank RCCL exchange (profiling)" % (flen, args.flows))
    if ((world > 1 and mode == "owner") or args.route_all) and "+" not in kname:
        kname += "+nat_remote64"
    extra = {}
    if not args.no_extra and world == 1 and args.order == "rr":
        # SURVEY.md §8(d) secondary order on the same warm table
        mark("secondary order")
        kn2 = {}
        el2, kms2, bufs2 = timed_steps(nat, bank, dev, lens, in_dev, out, B, slot, world,
                                       rank, args.warmup + 2 * args.steps, args.steps,
                                       "uniform", host_comm, knames=kn2)
        del bufs2
        pl2, pk2, ach2 = kernel_rate(kms2, B, args.steps, alg_bytes)
        extra["secondary_order"] = {
            "kernel": kernel_label(kn2, NAT64),
            "kernel_over_ceiling": round(pl2 * 1e3 / ceiling[0], 4) if ceiling else None,
            "order": "uniform (flow = splitmix64(0x5EED, p) mod N)",
            "value": round(B * args.steps / el2 / 1e6, 2), "unit": "Mpps",
            "ms_per_step": round(el2 / args.steps * 1e3, 4),
            "timing_events": True,
            "kernel_ms_per_launch": round(pl2 * 1e3, 4),
            "kernel_mpps": round(pk2 / pl2 / 1e6, 1),
            "frac": round(ach2 / HBM_PEAK_GBS, 4)}
    nat.kernel_timing(False)
    e2e = None
    if world == 1 and not args.no_e2e and slot == SLOT and args.order == "rr":
        mark("end to end")
        e2e = {"value": round(end_to_end(nat, bank, dev, (args.warmup + 3 * args.steps) * B), 1),
               "unit": "Mpps",
               "path": "page-locked host frames and per-packet arrays -> "
                       "hipMemcpyAsync H2D -> process -> D2H, %d-packet chunks "
                       "over three buffer sets (H2D two chunks ahead), H2D and "
                       "D2H on two copy streams "
                       "(vp_process_host_batch, affine time)" % E2E_CHUNK,
               "batch_packets": E2E_BATCH,
               "pcie_bytes_per_packet": SLOT + 4 + SLOT + 2}
        base = (args.warmup + 3 * args.steps) * B + 4 * E2E_BATCH
        mark("end to end (mbufs)")
        extra["end_to_end_mbuf"] = end_to_end_mbuf(nat, bank, dev, base)
        mark("end to end (mbufs, IMIX)")
        extra["end_to_end_mbuf_imix"] = end_to_end_mbuf(nat, bank, dev,
                                                        base + 4 * MBUF_BATCH, imix=True)
        mark("per-packet drop-in")
        pp = per_packet_drop_in(mark=mark)
        pp.update({"path": "host/nf_loop (nf.c's loop) over libvignat_nf.so: nf_process "
                           "per packet (vp_process_one: vignat's persistent kernel polling a "
                           "host-coherent mailbox), and the batched loop (vp_process_batch) "
                           "for comparison; frames in pageable host memory",
                   "packets": 20000, "flows": 1024})
        extra["per_packet_drop_in"] = pp
    if (world == 1 and not args.no_extra and slot == SLOT and args.order == "rr"
            and not args.route_all and args.flows == 1 << 20):
        L0 = nat.L
        nat.close()
        bank = None
        torch.cuda.empty_cache()
        gold = golden_configs()
        steps_x = min(args.steps, EXTRA_STEPS)
        mark("config 3 (vigbridge)")
        extra["config3_bridge"] = bench_bridge_c3(dev, B, steps_x, gold.get("bridge"))
        mark("config 4 (viglb)")
        extra["config4_lb"] = bench_lb_c4(dev, B, steps_x, gold.get("lb"))
        mark("random keys")
        extra["nat_random_keys"] = bench_nat_random(dev, B, steps_x, gold.get("random"))
        mark("churn")
        extra["nat_churn"] = bench_nat_churn(dev, B, steps_x, gold.get("churn"),
                                             gold.get("churn_state"))
        if ceiling:  # the 64-byte read(+write) shape at each kernel's own block shape
            probes = {ceiling[2]: ceiling}
            for k in ("config3_bridge", "config4_lb", "nat_random_keys", "nat_churn"):
                w = probe_waves(extra[k]["kernel"])
                if w not in probes:
                    mark("shape ceiling probe (%d waves)" % w)
                    probes[w] = shape_ceiling(L0, B, SLOT, dev, waves=w)
                rw, rd, _ = probes[w]
                # (per step: a batch may run as several segments, e.g. the
                # churn's first-sighting cut; the ceiling is a whole batch's)
                if k == "config3_bridge":  # (writes no frame: the read-only shape)
                    extra[k]["shape_read_ms"] = round(rd, 4)
                    extra[k]["kernel_over_read_ceiling"] = round(
                        extra[k]["kernel_ms_per_step"] / rd, 4)
                else:
                    extra[k]["shape_ceiling_ms"] = round(rw, 4)
                    extra[k]["kernel_over_ceiling"] = round(
                        extra[k]["kernel_ms_per_step"] / rw, 4)
    if owner_run and world > 1 and not args.no_extra:
        # the chunked owner pipeline (VIGPATH_OWN_CHUNK, read per call; the
        # same on every rank), same context and workload, the next batches:
        # one pass for the rate, one with events for its stages
        os.environ["VIGPATH_OWN_CHUNK"] = str(OWN_CHUNK)
        try:
            nat.kernel_timing(False)
            el4, _, b4 = timed_steps(nat, bank, dev, lens, in_dev, out, B, slot, world, rank,
                                     args.warmup + 2 * args.steps, args.steps, args.order,
                                     host_comm, wd=wd, label="owner chunked")
            del b4
            nat.kernel_timing(True)
            st4 = {}
            _, _, b4 = timed_steps(nat, bank, dev, lens, in_dev, out, B, slot, world, rank,
                                   args.warmup + 3 * args.steps, args.steps, args.order,
                                   host_comm, st4, wd=wd, label="owner chunked, stages")
            del b4
            nat.kernel_timing(False)
        finally:
            os.environ.pop("VIGPATH_OWN_CHUNK", None)
        extra["owner_chunked"] = {
            "mode": "owner", "chunk_packets": OWN_CHUNK,
            "value": round(B * args.steps * world / el4 / 1e6, 2), "unit": "Mpps",
            "ms_per_step": round(el4 / args.steps * 1e3, 4),
            "stages_ms_rank0": {k: round(v, 4) for k, v in st4.items()},
            "note": "the owner pipeline in chunks of %d packets per rank (exchange of "
                    "one chunk beside the next chunk's pass 1 and the last one's probe "
                    "and pass 2); the headline value stays the unchunked owner "
                    "pipeline" % OWN_CHUNK}
    if world > 1 and not args.no_extra:
        # the other dictionary placement, same workload
        other = "replicated" if mode == "owner" else "owner"
        mark("other shard mode: %s" % other)
        nat_ref.clear()
        nat.close()
        nat2 = make_nat(other)
        warm(nat2)
        el3, kms3, bufs3 = timed_steps(nat2, bank, dev, lens, in_dev, out, B, slot, world,
                                       rank, args.warmup, args.steps, "rr", host_comm,
                                       wd=wd, label="other mode")
        del bufs3
        extra["other_shard_mode"] = {
            "mode": other, "value": round(B * args.steps * world / el3 / 1e6, 2),
            "unit": "Mpps", "ms_per_step": round(el3 / args.steps * 1e3, 4)}
        extra["shard_modes"] = {  # every candidate of the same run, side by side
            mode: round(mpps, 2), other: extra["other_shard_mode"]["value"],
            **({"owner_chunked": extra["owner_chunked"]["value"]}
               if "owner_chunked" in extra else {})}
        nat_ref.clear()
        nat2.close()
    mark("report")
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1 and slot == SLOT:
            cmpps, rates, sample, core, warm = cpu_baseline(args.flows, args.cpu_sample)
            cpu = {"value": round(cmpps, 3), "unit": "Mpps", "cores": 1,
                   "kind": "port",
                   "samples": [round(r, 3) for r in rates],
                   "warmup_sample": round(warm, 3),
                   "spread": round((max(rates) - min(rates)) / cmpps, 4),
                   "sample": "median of %d samples after one discarded warm-up "
                             "sample, %d steady-state packets in "
                             "all, of the same trace (64B, %d flows warm, round "
                             "robin); oracle restatement built here -O3 "
                             "-march=native with hardware crc32 (oracle/"
                             "liborc_native.so), 1 thread pinned to cpu %d (%s)"
                             % (len(rates), sample, args.flows, core, cpu_model())}
        line = {
            "metric": METRIC, "value": round(mpps, 2), "unit": "Mpps",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "timed_loop": "python (one ctypes call a step)" if PY_LOOP else
                          "C (host/steps.c: one vp_process_device call a batch, as "
                          "nf.c's loop; descriptors prepared before the timed region)",
            "config": {"workload": workload, "flows": args.flows,
                       "batch_packets_per_gpu": B,
                       "global_batch_packets": B * world,
                       "frame_bytes": flen, "slot_bytes": slot,
                       "order": args.order,
                       "port": "per-packet array" if port_array
                               else "one per burst (vp_dev_batch.in_port)",
                       "parallelism": ("%s%d" % (mode, world))
                       if world > 1 else "single"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "frac_step": round(mpps / world * 1e6 * alg_bytes / 1e9
                                            / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": "profiles/%s: (2 x FETCH_SIZE + "
                                           "WRITE_SIZE) per launch / this "
                                           "run's kernel time" % TRAFFIC_PROFILE
                                           if traffic else None,
                         "kernel": kname,
                         "kernel_ms_per_launch": round(per_launch_s * 1e3, 4),
                         "kernel_timing": "a second timed pass of %d steps (the next "
                                          "batches), each launch between HIP events "
                                          "on its stream; that pass: %.4f ms per step"
                                          % (args.steps, el_k / args.steps * 1e3),
                         "alg_bytes_per_packet": alg_bytes,
                         **(ceiling_fields(ceiling, per_launch_s, elapsed / args.steps)
                            if ceiling else {}),
                         "kernel_mpps": round(pkts_per_launch / per_launch_s
                                              / 1e6, 1)},
            "cpu_baseline": cpu,
            "parity": parity,
            "new_flow_mpps": round(new_flow_mpps, 2) if new_flow_mpps else None,
            "end_to_end": e2e,
        }
        if stages:
            line["stages_ms"] = {
                "rank0": {k: round(v, 4) for k, v in stages.items()},
                "max_over_ranks": ({k: round(v, 4) for k, v in stages_max.items()}
                                   if stages_max else None),
                "source": "the kernel-timing pass: HIP events between the owner "
                          "pipeline's stages of every segment (vp_last_stage_ms), "
                          "mean per step on rank 0; that pass's step: %.4f ms"
                          % (el_k / args.steps * 1e3)}
        if cpu is not None:
            mark("cpu config 1")
            line["cpu_config1"] = cpu_config1()
        line.update(extra)
        if wd is not None:
            line["stages_done"] = len(wd.done) + 1
        print(json.dumps(line), flush=True)
    if world > 1:
        mark("destroy process group")
        dist.destroy_process_group()
    if wd is not None:
        wd.stage("done")
        wd.stop()


if __name__ == "__main__":
    main()
