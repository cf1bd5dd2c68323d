"""Synthetic packet traces shaped like the reference benchmark (host side).

Workload definition follows SURVEY.md §8(d), derived from the reference's
MoonGen script (bench/bench.lua:45-71 packetConfigs/packetInit, 108-138
throughput task) and run-benchmark.sh:47 (60 B frames + 4 B FCS):

* 60 B UDP frame in a 64 B slot; eth dst 00:..:00, src FF:..:FF, type 0x0800;
  IPv4 ihl 5, total_length 46, ttl 64, proto 17, valid header checksum;
  UDP dst_port 0, length 26, checksum 0 (bench.lua:128 offloads only the IP
  checksum); 18 zero payload bytes.
* L4 flows (vignat): flow i has src_ip 10.0.0.0 + (i >> 16), src_port
  i & 0xFFFF (bench.lua:54 generalised past 65,536 flows), dst 0.0.0.0:0.
* L3 flows (viglb): src_ip 11.0.0.0 + i (bench.lua:51).
* L2 (vigbridge): station k = 02:00:00:kk:kk:kk.
* Packet p belongs to flow p mod N (round robin, bench.lua:125) or to
  splitmix64(0x5EED, p) mod N (uniform).
* now_p = 1e9 + p nanoseconds.

Everything is vectorised numpy; arrays are frames[n*slot] u8, len[n] u16,
in_dev[n] u16, now[n] i64.
"""
from __future__ import annotations

import numpy as np

ETH_IPV4 = b"\x08\x00"
NOW0 = 1_000_000_000


def ip4(a: int, b: int, c: int, d: int) -> int:
    """Address as the host-order integer nf_parse_ipv4addr builds
    (nf-parse.h:21-32): a.b.c.d -> a<<24|b<<16|c<<8|d."""
    return (a << 24) | (b << 16) | (c << 8) | d


def mac(s: str) -> bytes:
    return bytes(int(x, 16) for x in s.split(":"))


def splitmix64(seed: int, p: np.ndarray) -> np.ndarray:
    z = (np.uint64(seed) + (p.astype(np.uint64) + np.uint64(1)) *
         np.uint64(0x9E3779B97F4A7C15))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def flow_order(n_packets: int, n_flows: int, order: str = "rr",
               seed: int = 0x5EED, start: int = 0) -> np.ndarray:
    p = np.arange(start, start + n_packets, dtype=np.int64)
    if order == "rr":
        return (p % n_flows).astype(np.int64)
    if order == "uniform":
        with np.errstate(over="ignore"):
            return (splitmix64(seed, p) % np.uint64(n_flows)).astype(np.int64)
    raise ValueError(order)


def _be16(v: np.ndarray) -> np.ndarray:
    v = v.astype(np.uint32)
    return np.stack([(v >> 8) & 0xFF, v & 0xFF], axis=-1).astype(np.uint8)


def _be32(v: np.ndarray) -> np.ndarray:
    v = v.astype(np.uint64)
    return np.stack([(v >> 24) & 0xFF, (v >> 16) & 0xFF, (v >> 8) & 0xFF,
                     v & 0xFF], axis=-1).astype(np.uint8)


def ipv4_header_checksum(hdr: np.ndarray) -> np.ndarray:
    """Valid RFC 791 checksum (as the tester's NIC offload writes it) for
    n x 20-byte headers whose checksum field is zero. Returns n x 2 bytes."""
    w = hdr.reshape(-1, 10, 2).astype(np.uint32)
    s = (w[:, :, 0] << 8 | w[:, :, 1]).sum(axis=1)
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    c = (~s) & 0xFFFF
    return _be16(c)


def udp_frames(src_ip: np.ndarray, dst_ip: np.ndarray, src_port: np.ndarray,
               dst_port: np.ndarray, slot: int = 64, frame_len: int = 60,
               proto: int = 17,
               eth_src: bytes = b"\xff" * 6, eth_dst: bytes = b"\x00" * 6):
    """Build n UDP (or TCP when proto=6, same layout) frames of frame_len bytes
    in slot-byte slots. Addresses/ports are numeric, written network order."""
    n = src_ip.shape[0]
    assert frame_len >= 42 and slot >= frame_len
    f = np.zeros((n, slot), dtype=np.uint8)
    f[:, 0:6] = np.frombuffer(eth_dst, np.uint8)
    f[:, 6:12] = np.frombuffer(eth_src, np.uint8)
    f[:, 12:14] = np.frombuffer(ETH_IPV4, np.uint8)
    tot = frame_len - 14
    f[:, 14] = 0x45
    f[:, 16:18] = _be16(np.full(n, tot))
    f[:, 22] = 64
    f[:, 23] = proto
    f[:, 26:30] = _be32(src_ip)
    f[:, 30:34] = _be32(dst_ip)
    f[:, 24:26] = ipv4_header_checksum(f[:, 14:34])
    f[:, 34:36] = _be16(src_port)
    f[:, 36:38] = _be16(dst_port)
    if proto == 17:
        f[:, 38:40] = _be16(np.full(n, tot - 20))
    lens = np.full(n, frame_len, dtype=np.uint16)
    return f.reshape(-1), lens


def nat_lan_trace(n_packets: int, n_flows: int, order: str = "rr",
                  slot: int = 64, lan_dev: int = 0, start: int = 0,
                  seed: int = 0x5EED):
    """vignat LAN->WAN trace (config 1/2/5 shape)."""
    fl = flow_order(n_packets, n_flows, order, seed, start)
    src_ip = ip4(10, 0, 0, 0) + (fl >> 16)
    src_port = fl & 0xFFFF
    z = np.zeros_like(fl)
    frames, lens = udp_frames(src_ip, z, src_port, z, slot=slot)
    in_dev = np.full(n_packets, lan_dev, dtype=np.uint16)
    now = (NOW0 + np.arange(start, start + n_packets, dtype=np.int64))
    return frames, lens, in_dev, now


def fw_trace(n_packets: int, n_flows: int, order: str = "rr",
             slot: int = 64, lan_dev: int = 0, wan_dev: int = 1,
             reply_every: int = 0, start: int = 0, seed: int = 0x5EED):
    """vigfw trace: LAN->WAN packets of the vignat flows (flow i: 10.0.0.0 +
    (i >> 16) : i & 0xFFFF -> 0.0.0.0:0); with reply_every = k, every k-th
    packet is instead the WAN->LAN reply of its flow (addresses and ports
    swapped, arriving on wan_dev)."""
    fl = flow_order(n_packets, n_flows, order, seed, start)
    a_ip = ip4(10, 0, 0, 0) + (fl >> 16)
    a_port = fl & 0xFFFF
    z = np.zeros_like(fl)
    in_dev = np.full(n_packets, lan_dev, dtype=np.uint16)
    rep = np.zeros(n_packets, bool)
    if reply_every:
        rep = (np.arange(start, start + n_packets) % reply_every) == reply_every - 1
        in_dev[rep] = wan_dev
    frames, lens = udp_frames(np.where(rep, z, a_ip), np.where(rep, a_ip, z),
                              np.where(rep, z, a_port), np.where(rep, a_port, z),
                              slot=slot)
    now = (NOW0 + np.arange(start, start + n_packets, dtype=np.int64))
    return frames, lens, in_dev, now


def pol_trace(n_packets: int, n_dsts: int, order: str = "rr",
              slot: int = 64, wan_dev: int = 0, start: int = 0,
              seed: int = 0x5EED):
    """vigpol trace: 64 B packets arriving on the WAN device (the policed
    direction), destination i = 10.0.0.0 + i (a /8 of subscribers), one
    source; time advances 1 ns per packet like the vignat trace."""
    d = flow_order(n_packets, n_dsts, order, seed, start)
    z = np.zeros_like(d)
    frames, lens = udp_frames(np.full_like(d, ip4(192, 168, 0, 1)),
                              ip4(10, 0, 0, 0) + d, z + 53, z + 80, slot=slot)
    in_dev = np.full(n_packets, wan_dev, dtype=np.uint16)
    now = (NOW0 + np.arange(start, start + n_packets, dtype=np.int64))
    return frames, lens, in_dev, now


def bridge_trace(n_packets: int, n_stations: int, slot: int = 64,
                 start: int = 0, flood_pattern: bool = False):
    """vigbridge config 3: frame p from station p mod N (on port (k & 1)) to
    station (p + N/2) mod N; flood_pattern: dst = 0xFF0000000000 + k
    (bench.lua:47-48), never learned."""
    p = np.arange(start, start + n_packets, dtype=np.int64)
    src_k = p % n_stations
    dst_k = (p + n_stations // 2) % n_stations
    frames, lens = udp_frames(np.full(n_packets, ip4(10, 0, 0, 1)),
                              np.zeros(n_packets, np.int64),
                              np.zeros(n_packets, np.int64),
                              np.zeros(n_packets, np.int64), slot=slot)
    f = frames.reshape(n_packets, slot)
    f[:, 6:9] = np.array([0x02, 0, 0], np.uint8)
    f[:, 9:12] = _be32(src_k)[:, 1:]
    if flood_pattern:
        f[:, 0:6] = np.concatenate(
            [np.full((n_packets, 1), 0xFF, np.uint8),
             np.zeros((n_packets, 1), np.uint8), _be32(src_k)], axis=1)
    else:
        f[:, 0:3] = np.array([0x02, 0, 0], np.uint8)
        f[:, 3:6] = _be32(dst_k)[:, 1:]
    in_dev = (src_k & 1).astype(np.uint16)
    now = NOW0 + p
    return frames, lens, in_dev, now


def lb_traffic(n_packets: int, n_flows: int, wan_dev: int = 2, slot: int = 64,
               order: str = "rr", start: int = 0, seed: int = 0x5EED):
    """viglb config 4 WAN traffic: flow i = src_ip 11.0.0.0 + i."""
    fl = flow_order(n_packets, n_flows, order, seed, start)
    src_ip = ip4(11, 0, 0, 0) + fl
    z = np.zeros_like(fl)
    frames, lens = udp_frames(src_ip, z, z, z, slot=slot)
    in_dev = np.full(n_packets, wan_dev, dtype=np.uint16)
    now = NOW0 + np.arange(start, start + n_packets, dtype=np.int64)
    return frames, lens, in_dev, now


def lb_heartbeats(n_backends: int, slot: int = 64, t0: int = NOW0 - 1000):
    """Backend b: src_ip 192.168.(b>>8).(b&255) on port b & 1."""
    b = np.arange(n_backends, dtype=np.int64)
    src_ip = ip4(192, 168, 0, 0) + b
    z = np.zeros_like(b)
    frames, lens = udp_frames(src_ip, z, z, z, slot=slot)
    f = frames.reshape(n_backends, slot)
    f[:, 6:8] = np.array([0x02, 0xBE], np.uint8)
    f[:, 8:12] = _be32(b)
    in_dev = (b & 1).astype(np.uint16)
    now = t0 + b
    return frames, lens, in_dev, now


FNV64_BASIS = 0xCBF29CE484222325
FNV64_PRIME = 0x100000001B3


def batch_digest(frames: np.ndarray, out_dev: np.ndarray, slot: int,
                 p0: int = 0) -> int:
    """Order-sensitive digest of one processed batch: the wrapping u64 sum over
    packets p of an FNV-1a-style chain over 64-bit words, h = (h ^ w) * prime,
    of the word (p | out_dev[p] << 32) and then the slot's 8-byte LE words,
    finalised by splitmix64's mixer. Packet positions start at p0, so the
    digests of consecutive pieces of a batch add up to the batch's digest.
    Vectorised over packets (one pass per word): a 2^24-packet batch of 64 B
    slots digests in about a second."""
    n = out_dev.shape[0]
    words = np.ascontiguousarray(frames.reshape(n, slot)).view("<u8")
    prime = np.uint64(FNV64_PRIME)
    h = np.full(n, FNV64_BASIS, np.uint64)
    with np.errstate(over="ignore"):
        w0 = (np.arange(p0, p0 + n, dtype=np.uint64) |
              (out_dev.astype(np.uint64) << np.uint64(32)))
        np.bitwise_xor(h, w0, out=h)
        np.multiply(h, prime, out=h)
        for j in range(slot // 8):
            np.bitwise_xor(h, words[:, j], out=h)
            np.multiply(h, prime, out=h)
        return int(_avalanche(h).sum(dtype=np.uint64))


def state_digest(alloc: np.ndarray, ts: np.ndarray) -> int:
    """Digest of a table dump, same construction: per index i the words
    (i | alloc[i] << 32) and ts[i] (0 where not allocated)."""
    n = alloc.shape[0]
    prime = np.uint64(FNV64_PRIME)
    h = np.full(n, FNV64_BASIS, np.uint64)
    t = np.where(alloc != 0, ts, 0).astype(np.int64).view(np.uint64)
    with np.errstate(over="ignore"):
        w0 = np.arange(n, dtype=np.uint64) | (alloc.astype(np.uint64) << np.uint64(32))
        for w in (w0, t):
            np.bitwise_xor(h, w, out=h)
            np.multiply(h, prime, out=h)
        return int(_avalanche(h).sum(dtype=np.uint64))


def _avalanche(h: np.ndarray) -> np.ndarray:
    """splitmix64's finaliser, so every bit of the per-packet hash feeds the
    low bits of the sum."""
    with np.errstate(over="ignore"):
        np.bitwise_xor(h, h >> np.uint64(30), out=h)
        np.multiply(h, np.uint64(0xBF58476D1CE4E5B9), out=h)
        np.bitwise_xor(h, h >> np.uint64(27), out=h)
        np.multiply(h, np.uint64(0x94D049BB133111EB), out=h)
        np.bitwise_xor(h, h >> np.uint64(31), out=h)
    return h


class MbufPool:
    """A DPDK-shaped mbuf pool in host memory (SURVEY.md §8(d) "End-to-end":
    2 KB buffers, 128 B headroom): `n` elements of `stride` bytes, each a
    128-byte struct rte_mbuf, RTE_PKTMBUF_HEADROOM (128 B) and a 2048-byte
    data room (DPDK's RTE_MBUF_DEFAULT_BUF_SIZE = 2048 + 128), so a frame
    starts at `data_off` = 256 into its element (rte_pktmbuf_mtod). `mem` is
    one flat uint8 array (page-locked when `pinned`, as DPDK's hugepages are
    to the NIC; on 2 MB transparent huge pages when `huge`, as DPDK's are
    hugepages, then page-locked by vp_register_host); vp_register_host maps
    it for the GPU."""

    def __init__(self, n: int, stride: int = 2304, data_off: int = 256,
                 pinned: bool = False, huge: bool = False):
        self.n, self.stride, self.data_off = n, stride, data_off
        if huge:
            import mmap
            H = 1 << 21
            self._map = mmap.mmap(-1, n * stride + H)
            raw = np.frombuffer(self._map, np.uint8)
            a = (-raw.ctypes.data) % H
            if hasattr(mmap, "MADV_HUGEPAGE"):
                self._map.madvise(mmap.MADV_HUGEPAGE)
            self.mem = raw[a:a + n * stride]
            self.mem[::4096] = 0  # (fault the pages in)
        elif pinned:
            import torch
            self.mem = torch.zeros(n * stride, dtype=torch.uint8).pin_memory().numpy()
        else:  # page-aligned, as hugepages are
            raw = np.zeros(n * stride + 4096, np.uint8)
            a = (-raw.ctypes.data) % 4096
            self.mem = raw[a:a + n * stride]
        self.rows = self.mem.reshape(n, stride)

    def ptrs(self, bufs: np.ndarray, shift: np.ndarray | None = None) -> np.ndarray:
        """The data pointers (u64) of mbufs `bufs` (+ per-frame byte shifts)."""
        off = np.asarray(bufs, np.uint64) * np.uint64(self.stride) + np.uint64(self.data_off)
        if shift is not None:
            off = off + np.asarray(shift, np.uint64)
        return (np.uint64(self.mem.ctypes.data) + off).astype(np.uint64)

    def put(self, bufs: np.ndarray, frames: np.ndarray, slot: int, lens: np.ndarray,
            shift: np.ndarray | None = None):
        """Frame i (len[i] bytes of its `slot`-byte slot in `frames`) into
        mbuf bufs[i]. Equal lengths and shifts are copied in one step."""
        f = frames.reshape(-1, slot)
        lens = np.asarray(lens)
        o = self.data_off
        if shift is None and (lens == lens[0]).all():
            L = int(lens[0])
            self.rows[np.asarray(bufs), o:o + L] = f[:, :L]
            return
        for i, b in enumerate(np.asarray(bufs)):
            s = o + (int(shift[i]) if shift is not None else 0)
            self.rows[b, s:s + int(lens[i])] = f[i, :int(lens[i])]

    def get(self, bufs: np.ndarray, slot: int, lens: np.ndarray,
            shift: np.ndarray | None = None) -> np.ndarray:
        """The frames back in `slot`-byte slots (zeros past each length)."""
        out = np.zeros((len(bufs), slot), np.uint8)
        o = self.data_off
        for i, b in enumerate(np.asarray(bufs)):
            s = o + (int(shift[i]) if shift is not None else 0)
            out[i, :int(lens[i])] = self.rows[b, s:s + int(lens[i])]
        return out.reshape(-1)


def random_flow_keys(n_flows: int, seed: int = 0xF10E5):
    """Flow i of the unstructured-key workload: a 5-tuple with no counter
    structure (src_ip a bijective mix of i, so the n keys are distinct;
    dst_ip, ports from splitmix64), for the random-key steady state the
    allocation-order layout cannot fit."""
    i = np.arange(n_flows, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (i * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)   # odd multiplier: bijective
        x = x ^ (x >> np.uint64(15))                               # (xorshift: bijective)
        x = (x * np.uint64(0x2C1B3C6D)) & np.uint64(0xFFFFFFFF)
        src_ip = (x ^ (x >> np.uint64(12))).astype(np.int64)
        r = splitmix64(seed, i)
    dst_ip = (r & np.uint64(0xFFFFFFFF)).astype(np.int64)
    sp = ((r >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
    dp = ((r >> np.uint64(48)) & np.uint64(0xFFFF)).astype(np.int64)
    return src_ip, dst_ip, sp, dp


# Steady turnover (SURVEY.md §8(f) rank 1 at the reference's latency-run
# expiry, run-middlebox.sh:16): CHURN_W flow slots in round robin; slot s of
# batch k carries flow epoch(s, k) * CHURN_W + s with epoch = (k + s % 4) // 4,
# so every batch a quarter of the slots (CHURN_W / 4 flows) starts new flows
# while the flows they retire go idle; batch k is stamped NOW0 + k *
# CHURN_DT (one current_time() per batch, as nf.c stamps a polling sweep,
# nf.c:56), and with 1 s expiry a retired flow expires at the first packet of
# the fifth batch after its last one. Live flows settle at 2 * CHURN_W.
CHURN_W = 1 << 18
CHURN_DT = 250_000_000
CHURN_EXPIRE_US = 1_000_000


def churn_flow_ids(p: np.ndarray, k: int, w: int = CHURN_W) -> np.ndarray:
    """Flow ids of packets p (positions in batch k) of the turnover trace."""
    s = np.asarray(p, np.int64) % w
    return (k + s % 4) // 4 * w + s


def churn_trace(k: int, n_packets: int, start: int = 0, w: int = CHURN_W, slot: int = 64):
    """Packets [start, start + n_packets) of batch k of the turnover trace
    (vignat flow keys of churn_flow_ids; time NOW0 + k * CHURN_DT)."""
    fl = churn_flow_ids(np.arange(start, start + n_packets), k, w)
    z = np.zeros_like(fl)
    frames, lens = udp_frames(ip4(10, 0, 0, 0) + (fl >> 16), z, fl & 0xFFFF, z, slot=slot)
    in_dev = np.zeros(n_packets, np.uint16)
    now = np.full(n_packets, NOW0 + k * CHURN_DT, np.int64)
    return frames, lens, in_dev, now


def random_key_trace(n_packets: int, n_flows: int, start: int = 0, slot: int = 64,
                     keys=None):
    """Round robin over the random_flow_keys flows, time NOW0 + p ns."""
    src, dst, sp, dp = keys if keys is not None else random_flow_keys(n_flows)
    fl = flow_order(n_packets, n_flows, "rr", start=start)
    frames, lens = udp_frames(src[fl], dst[fl], sp[fl], dp[fl], slot=slot)
    in_dev = np.zeros(n_packets, np.uint16)
    now = NOW0 + np.arange(start, start + n_packets, dtype=np.int64)
    return frames, lens, in_dev, now
