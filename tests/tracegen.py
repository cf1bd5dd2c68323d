"""Adversarial trace builders shared by the oracle and GPU parity tests."""
import numpy as np

from vigor_amd import traces as T


def mixed_nat_trace(rng, n, n_flows, slot=64, max_idx=64):
    """LAN packets over n_flows plus WAN replies to existing/unknown ports,
    some malformed frames, monotone time with ties."""
    fl = rng.integers(0, n_flows, n)
    sip = T.ip4(10, 0, 0, 0) + fl
    dip = T.ip4(8, 8, 0, 0) + (fl % 7)
    sp = 1000 + fl % 13
    dp = np.full(n, 53)
    proto = np.where(fl % 5 == 0, 6, 17)
    frames = np.zeros((n, slot), np.uint8)
    lens = np.zeros(n, np.uint16)
    for p_ in (6, 17):
        m = proto == p_
        f, ln = T.udp_frames(sip[m], dip[m], sp[m], dp[m], slot=slot, proto=p_)
        frames[m] = f.reshape(-1, slot)
        lens[m] = ln
    in_dev = np.zeros(n, np.uint16)
    wan = rng.random(n) < 0.3
    in_dev[wan] = 1
    # WAN replies: swap addresses, dst port = an index (raw LE u16 on wire)
    idx = rng.integers(0, max_idx, n).astype(np.uint16)
    w = frames[wan]
    w[:, 26:30], w[:, 30:34] = frames[wan][:, 30:34], frames[wan][:, 26:30]
    w[:, 34:36] = frames[wan][:, 36:38]
    w[:, 36] = (idx[wan] & 0xFF).astype(np.uint8)
    w[:, 37] = (idx[wan] >> 8).astype(np.uint8)
    frames[wan] = w
    # malformed: non-IPv4, short total_length, ihl<5, non tcp/udp
    bad = rng.random(n)
    frames[bad < 0.02, 12] = 0x86
    frames[(bad >= 0.02) & (bad < 0.04), 17] = 200
    frames[(bad >= 0.04) & (bad < 0.05), 14] = 0x44
    frames[(bad >= 0.05) & (bad < 0.06), 23] = 1
    now = T.NOW0 + np.cumsum(rng.integers(0, 3, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)


def edge_nat_trace(rng, n, n_flows, slot=128, long_frames=False):
    """Header edge cases of nf-util.h:116-162 / nf-util.c:45-64: IP options
    (borrowed or not), odd and short lengths, total_length < 20 or beyond the
    packet, pkt_len < 14 (u16 wrap), TCP and UDP, long frames."""
    fl = rng.integers(0, n_flows, n)
    frames = np.zeros((n, slot), np.uint8)
    lens = np.zeros(n, np.uint16)
    in_dev = np.where(rng.random(n) < 0.2, 1, 0).astype(np.uint16)
    maxlen = min(slot, 1514 if long_frames else slot)
    for i in range(n):
        ihl = 5 if rng.random() < 0.6 else int(rng.integers(0, 16))
        proto = int(rng.choice([6, 17, 17, 1]))
        flen = int(rng.integers(14, maxlen + 1)) if rng.random() < 0.7 else \
            int(rng.integers(0, 64))
        f = frames[i]
        f[:slot] = rng.integers(0, 256, slot, dtype=np.uint8)  # dirty bytes
        f[12:14] = (8, 0) if rng.random() < 0.95 else (0x86, 0xDD)
        f[14] = 0x40 | ihl
        tl = max(0, flen - 14) if rng.random() < 0.7 else \
            int(rng.integers(0, 2 * maxlen))
        f[16:18] = (tl >> 8, tl & 0xFF)
        f[23] = proto
        k = int(fl[i])
        f[26:30] = (10, 0, (k >> 8) & 0xFF, k & 0xFF)
        f[30:34] = (8, 8, 8, k % 3)
        l4 = 14 + 4 * max(ihl, 5)
        if l4 + 4 <= slot:
            f[l4:l4 + 2] = (0, 53)
            if in_dev[i] == 1:  # WAN: dst port = small index, raw LE
                idx = int(rng.integers(0, 70))
                f[l4 + 2:l4 + 4] = (idx & 0xFF, idx >> 8)
            else:
                f[l4 + 2:l4 + 4] = (k >> 8, k & 0xFF)
        lens[i] = flen
    return frames.reshape(-1), lens, in_dev


def mixed_bridge_trace(rng, n, n_stations, n_dev=3, slot=64):
    """vigbridge stress: stations 02:00:00:00:kk:kk on random ports (MAC
    moves), dst from the same pool (known, unknown, the frame's own src) or
    broadcast/never-learned, short frames, monotone time with ties."""
    src = rng.integers(0, n_stations, n)
    dst = rng.integers(0, n_stations + n_stations // 4, n)  # some never seen
    same = rng.random(n) < 0.05
    dst[same] = src[same]
    frames = np.zeros((n, slot), np.uint8)
    frames[:, 0:4] = [0x02, 0, 0, 0]
    frames[:, 4] = (dst >> 8) & 0xFF
    frames[:, 5] = dst & 0xFF
    frames[:, 6:10] = [0x02, 0, 0, 0]
    frames[:, 10] = (src >> 8) & 0xFF
    frames[:, 11] = src & 0xFF
    bc = rng.random(n) < 0.03
    frames[bc, 0:6] = 0xFF
    frames[:, 12:14] = [0x08, 0x00]
    frames[:, 14:] = rng.integers(0, 256, (n, slot - 14), dtype=np.uint8)
    lens = rng.integers(60, slot + 1, n).astype(np.uint16)
    lens[rng.random(n) < 0.02] = rng.integers(0, 14)  # runts: no length check
    in_dev = rng.integers(0, n_dev, n).astype(np.uint16)
    now = T.NOW0 + np.cumsum(rng.integers(0, 3, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)


def mixed_lb_trace(rng, n, n_flows, n_backends, hb_frac=0.05, quiet=None,
                   wan=2, slot=64, bad_frac=0.03):
    """viglb stress: WAN traffic over n_flows (uniform) with heartbeats from
    n_backends IPs on ports 0/1 mixed in; no heartbeats inside the packet
    window `quiet` (so backends can all expire), malformed frames, monotone
    time with ties."""
    fl = rng.integers(0, n_flows, n)
    sip = T.ip4(11, 0, 0, 0) + fl
    dip = T.ip4(10, 9, 8, 7) + (fl % 3)
    sp = 2000 + fl % 11
    dp = np.full(n, 80)
    proto = np.where(fl % 4 == 0, 6, 17)
    hb = rng.random(n) < hb_frac
    if quiet is not None:
        hb[quiet[0]:quiet[1]] = False
    be = rng.integers(0, n_backends, n)
    sip = np.where(hb, T.ip4(192, 168, 0, 0) + be, sip)
    frames = np.zeros((n, slot), np.uint8)
    lens = np.zeros(n, np.uint16)
    for p_ in (6, 17):
        m = proto == p_
        f, ln = T.udp_frames(sip[m], dip[m], sp[m], dp[m], slot=slot, proto=p_)
        frames[m] = f.reshape(-1, slot)
        lens[m] = ln
    frames[:, 6:8] = [0x02, 0xBE]
    frames[:, 8] = (be >> 8) & 0xFF
    frames[:, 9] = be & 0xFF
    frames[:, 10:12] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    in_dev = np.where(hb, be & 1, wan).astype(np.uint16)
    bad = rng.random(n)
    frames[bad < bad_frac / 3, 12] = 0x86
    frames[(bad >= bad_frac / 3) & (bad < 2 * bad_frac / 3), 23] = 1
    frames[(bad >= 2 * bad_frac / 3) & (bad < bad_frac), 17] = 250
    now = T.NOW0 + np.cumsum(rng.integers(0, 3, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)


def mixed_fw_trace(rng, n, n_flows, n_dev=3, wan=1, slot=64, reply_frac=0.35,
                   unknown_frac=0.1):
    """vigfw stress: LAN packets over n_flows from the non-WAN devices (the
    same 5-tuple may arrive on different LAN devices), WAN replies (reversed
    5-tuple) of pool flows (known, not yet seen, or expired) and of unknown
    flows, malformed frames, TCP and UDP, monotone time with ties."""
    fl = rng.integers(0, n_flows, n)
    sip = T.ip4(10, 0, 0, 0) + fl
    dip = T.ip4(8, 8, 0, 0) + (fl % 7)
    sp = 1000 + fl % 13
    dp = np.full(n, 53) + (fl % 3)
    proto = np.where(fl % 5 == 0, 6, 17)
    lan_devs = np.array([d for d in range(n_dev) if d != wan])
    in_dev = lan_devs[rng.integers(0, lan_devs.size, n)].astype(np.uint16)
    r = rng.random(n)
    rep = r < reply_frac
    unk = rep & (r < unknown_frac)
    in_dev[rep] = wan
    sip = np.where(unk, sip + 0x10000, sip)  # a flow no LAN packet opens
    a_ip, b_ip = np.where(rep, dip, sip), np.where(rep, sip, dip)
    a_p, b_p = np.where(rep, dp, sp), np.where(rep, sp, dp)
    frames = np.zeros((n, slot), np.uint8)
    lens = np.zeros(n, np.uint16)
    for p_ in (6, 17):
        m = proto == p_
        f, ln = T.udp_frames(a_ip[m], b_ip[m], a_p[m], b_p[m], slot=slot,
                             proto=p_)
        frames[m] = f.reshape(-1, slot)
        lens[m] = ln
    bad = rng.random(n)
    frames[bad < 0.02, 12] = 0x86
    frames[(bad >= 0.02) & (bad < 0.04), 17] = 200
    frames[(bad >= 0.04) & (bad < 0.05), 14] = 0x44
    frames[(bad >= 0.05) & (bad < 0.06), 23] = 1
    frames[(bad >= 0.06) & (bad < 0.08), 14] = 0x46  # IP options (generic path)
    now = T.NOW0 + np.cumsum(rng.integers(0, 3, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)


def mixed_pol_trace(rng, n, n_dsts, n_dev=3, lan=1, wan=0, slot=64,
                    lan_frac=0.2, other_frac=0.05, gap_ns=2000, big=1400):
    """vigpol stress: WAN packets to n_dsts destination addresses with random
    sizes (some above the burst), LAN packets (forwarded, not policed),
    packets from a third device (dropped), non-IPv4 / truncated frames (no
    expiry runs for them, policer_main.c:124-130), monotone time with ties
    and gaps long enough to refill buckets and expire entries."""
    d = rng.integers(0, n_dsts, n)
    sip = T.ip4(9, 9, 0, 0) + (d % 5)
    dip = T.ip4(10, 0, 0, 0) + d
    f, _ = T.udp_frames(sip, dip, 1000 + d % 13, np.full(n, 80), slot=slot)
    frames = f.reshape(n, slot)
    lens = rng.integers(60, big, n).astype(np.uint16)
    lens[rng.random(n) < 0.3] = 64
    frames[:, 16] = 0  # total_length = 46 <= every size (nf-util.h:140)
    frames[:, 17] = 46
    in_dev = np.full(n, wan, np.uint16)
    r = rng.random(n)
    in_dev[r < lan_frac] = lan
    if n_dev > 2:
        in_dev[(r >= lan_frac) & (r < lan_frac + other_frac)] = 2
    bad = rng.random(n)
    frames[bad < 0.02, 12] = 0x86                          # not IPv4
    frames[(bad >= 0.02) & (bad < 0.03), 14] = 0x44        # ihl < 5
    frames[(bad >= 0.03) & (bad < 0.04), 16] = 0x40        # total_length > len
    frames[(bad >= 0.04) & (bad < 0.06), 14] = 0x46        # IP options
    now = T.NOW0 + np.cumsum(rng.integers(0, gap_ns, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)


def lan_tile_trace(rng, n, n_flows, bad_tiles=0.1, slot=64):
    """LAN-only traffic (TCP and UDP, several devices below the WAN port) in
    which most 64-packet tiles are entirely fast-path packets (the classify
    kernel's lean tile) and a fraction `bad_tiles` of the tiles carry one
    malformed packet each (those tiles take the per-lane path)."""
    fl = rng.integers(0, n_flows, n)
    sip = T.ip4(10, 1, 0, 0) + fl
    dip = T.ip4(9, 9, 0, 0) + (fl % 11)
    sp = 2000 + fl % 17
    dp = 80 + fl % 3
    proto = np.where(fl % 3 == 0, 6, 17)
    frames = np.zeros((n, slot), np.uint8)
    lens = np.zeros(n, np.uint16)
    for p_ in (6, 17):
        m = proto == p_
        f, ln = T.udp_frames(sip[m], dip[m], sp[m], dp[m], slot=slot, proto=p_)
        frames[m] = f.reshape(-1, slot)
        lens[m] = ln
    tiles = (n + 63) // 64
    for t in np.nonzero(rng.random(tiles) < bad_tiles)[0]:
        p = min(n - 1, int(t) * 64 + int(rng.integers(0, 64)))
        kind = int(rng.integers(0, 3))
        if kind == 0:
            frames[p, 12] = 0x86  # not IPv4
        elif kind == 1:
            frames[p, 14] = 0x46  # IHL 6: the byte-addressed path
        else:
            frames[p, 23] = 1  # ICMP: dropped
    in_dev = np.zeros(n, np.uint16)
    now = T.NOW0 + np.cumsum(rng.integers(0, 4, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)


def wide_nat_trace(rng, n, n_flows, slot, max_len=1518, wan_frac=0.25,
                   bad_frac=0.03, pad_frac=0.1):
    """vignat traffic in wide slots (65-1518 B frames, SURVEY.md §8(d) "R =
    slot(len) + 28"): frame lengths uniform in [60, min(slot, max_len)],
    random payload bytes (so the L4 checksum covers real data), TCP and UDP,
    LAN packets over n_flows and WAN replies to indices 0..2 n_flows (known,
    unknown, wrong protocol), some frames padded past total_length (the L4 sum ends at
    14 + total_length, not at the frame's end), odd lengths, and a few
    malformed frames (not IPv4, IHL 6, total_length past the frame) that
    take the byte-addressed path. Monotone time with ties."""
    top = min(slot, max_len)
    fl = rng.integers(0, n_flows, n)
    sip = T.ip4(10, 2, 0, 0) + fl
    dip = np.full(n, T.ip4(9, 9, 0, 1))
    sp = 3000 + fl % 19
    dp = np.full(n, 443)
    proto = np.where(fl % 3 == 0, 6, 17)
    lens = rng.integers(60, top + 1, n).astype(np.uint16)
    frames = rng.integers(0, 256, (n, slot), dtype=np.uint8)
    for p_ in (6, 17):
        m = proto == p_
        f, _ = T.udp_frames(sip[m], dip[m], sp[m], dp[m], slot=slot, proto=p_)
        f = f.reshape(-1, slot)
        frames[m, :38] = f[:, :38]
        if p_ == 17:  # UDP length; checksum field left random (recomputed)
            frames[m, 38:40] = 0
    tl = lens.astype(np.int64) - 14
    pad = rng.random(n) < pad_frac  # total_length short of the frame
    tl[pad] = np.maximum(20, tl[pad] - rng.integers(1, 40, int(pad.sum())))
    frames[:, 16] = (tl >> 8).astype(np.uint8)
    frames[:, 17] = (tl & 0xFF).astype(np.uint8)
    udp = proto == 17
    ul = tl[udp] - 20
    frames[udp, 38] = (ul >> 8).astype(np.uint8)
    frames[udp, 39] = (ul & 0xFF).astype(np.uint8)
    in_dev = np.zeros(n, np.uint16)
    wan = rng.random(n) < wan_frac
    in_dev[wan] = 1
    w = frames[wan]
    w[:, 26:30], w[:, 30:34] = frames[wan][:, 30:34], frames[wan][:, 26:30]
    w[:, 34:36] = frames[wan][:, 36:38]
    idx = rng.integers(0, n_flows + n_flows // 4, int(wan.sum())).astype(np.uint16)
    w[:, 36] = (idx & 0xFF).astype(np.uint8)
    w[:, 37] = (idx >> 8).astype(np.uint8)
    frames[wan] = w
    bad = rng.random(n)
    frames[bad < bad_frac / 3, 12] = 0x86
    frames[(bad >= bad_frac / 3) & (bad < 2 * bad_frac / 3), 14] = 0x46
    big = (bad >= 2 * bad_frac / 3) & (bad < bad_frac)
    frames[big, 16] = 0xFF  # total_length past the packet: dropped
    now = T.NOW0 + np.cumsum(rng.integers(0, 3, n))
    return frames.reshape(-1), lens, in_dev, now.astype(np.int64)
