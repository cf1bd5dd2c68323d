"""vignat on the GPU vs the oracle (bit-exact out ports, frames and state).

Every test calls the product through the C-ABI (libvigpath.so via
vigor_amd); the oracle (oracle/liborc.so) is only the checker.
"""
import numpy as np
import pytest
import orc
import vigor_amd
from gpuh import check_batches, run_gpu
from tracegen import edge_nat_trace, lan_tile_trace, mixed_nat_trace, wide_nat_trace
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu

DEV_MACS = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17"),
            T.mac("22:23:24:25:26:27")]
END_MACS = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01"),
            T.mac("01:23:45:67:89:02")]


def make_pair(max_flows=65536, expire_us=60_000_000, start_port=0, wan=1,
              n_dev=2):
    args = ["--wan", str(wan), "--expire", str(expire_us), "--starting-port",
            str(start_port), "--max-flows", str(max_flows), "--extip",
            "192.168.4.2"]
    for d in range(n_dev):
        args += ["--eth-dest", "%d,%s" % (d, END_MACS[d].hex(":"))]
    cfg = vigor_amd.nat_config_from_args(args, n_dev, DEV_MACS[:n_dev])
    gpu = vigor_amd.Nat(cfg, gpu=0)
    ocfg = orc.nat_cfg(wan=wan, start_port=start_port,
                       ext_ip=T.ip4(192, 168, 4, 2), expire_us=expire_us,
                       max_flows=max_flows, device_macs=DEV_MACS[:n_dev],
                       endpoint_macs=END_MACS[:n_dev], n_devices=n_dev)
    return gpu, orc.Oracle("nat", ocfg)


def check_state(nat, oracle, max_flows):
    ga, gts, gk = nat.dump()
    oa, ots, ok = oracle.nat_dump(max_flows)
    np.testing.assert_array_equal(ga, oa)
    np.testing.assert_array_equal(gts[oa == 1], ots[oa == 1])
    np.testing.assert_array_equal(gk[oa == 1], ok[oa == 1])


def test_config1_roundrobin_1k_flows():
    nat, o = make_pair(max_flows=65536)
    fr, ln, dv, now = T.nat_lan_trace(50_000, 1000)
    check_batches(nat, o, fr, ln, dv, now, 64, [1000, 1500, 20_000],
                  affine=True)
    check_state(nat, o, 65536)
    assert nat.live_count() == 1000


@pytest.mark.parametrize("seed,max_flows,expire_us,n_flows,cuts", [
    (0, 64, 60_000_000, 40, [100, 2000]),       # steady + WAN replies
    (1, 64, 1, 100, [1, 2, 3, 500, 4000]),       # expiry every few packets
    (2, 16, 60_000_000, 40, [2500]),             # table full
    (3, 256, 5, 300, [1000, 1001, 3000]),        # expiry + reuse (LIFO)
    (4, 1024, 3, 2000, []),                      # one batch, heavy churn
])
def test_mixed_traces(seed, max_flows, expire_us, n_flows, cuts):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_nat_trace(rng, 5000, n_flows, max_idx=max_flows)
    nat, o = make_pair(max_flows=max_flows, expire_us=expire_us)
    check_batches(nat, o, fr, ln, dv, now, 64, cuts)
    check_state(nat, o, max_flows)


@pytest.mark.parametrize("slot,long_frames", [(64, False), (128, False), (256, True),
                                              (1536, True), (2048, True)])
def test_header_edge_cases(slot, long_frames):
    rng = np.random.default_rng(slot)
    n = 3000
    fr, ln, dv = edge_nat_trace(rng, n, 60, slot=slot, long_frames=long_frames)
    now = T.NOW0 + np.arange(n, dtype=np.int64) * 3
    nat, o = make_pair(max_flows=64)
    check_batches(nat, o, fr, ln, dv, now, slot, [700])
    check_state(nat, o, 64)


def test_time_ties_and_wrapping_expiry():
    # one `now` per nf.c sweep (many packets share a time); expire 4295 s
    # wraps the u32 x1000 (nat_flowmanager.c:62) to a ~0.7 s window
    rng = np.random.default_rng(7)
    fr, ln, dv, _ = mixed_nat_trace(rng, 6000, 300, max_idx=512)
    now = T.NOW0 + (np.arange(6000) // 7).astype(np.int64) * 1_000_000
    nat, o = make_pair(max_flows=512, expire_us=4_295_000)
    check_batches(nat, o, fr, ln, dv, now, 64, [1234, 3000])
    check_state(nat, o, 512)


def test_start_port_and_three_devices():
    rng = np.random.default_rng(11)
    fr, ln, dv, now = mixed_nat_trace(rng, 4000, 100, max_idx=200)
    dv = np.where(dv == 1, 2, dv % 2).astype(np.uint16)  # wan = 2, lan 0/1
    f = fr.reshape(-1, 64)
    wan = dv == 2
    port = (f[wan, 36].astype(np.int64) | (f[wan, 37].astype(np.int64) << 8))
    port = port + 1000
    f[wan, 36], f[wan, 37] = port & 0xFF, port >> 8
    nat, o = make_pair(max_flows=256, start_port=1000, wan=2, n_dev=3)
    check_batches(nat, o, fr, ln, dv, now, 64, [2000])


def test_host_batch_entry_points():
    rng = np.random.default_rng(5)
    fr, ln, dv, now = mixed_nat_trace(rng, 3000, 50, max_idx=64)
    nat, o = make_pair(max_flows=64)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    got = fr.copy()
    out = nat.process_host(got[:1500 * 64], ln[:1500], dv[:1500], now[:1500],
                           64)
    bufs = [bytearray(got[i * 64:i * 64 + int(ln[i])].tobytes())
            for i in range(1500, 3000)]
    out2 = nat.process_mbufs(bufs, dv[1500:], now[1500:])
    np.testing.assert_array_equal(np.concatenate([out, out2]), exp_out)
    np.testing.assert_array_equal(got[:1500 * 64], exp[:1500 * 64])
    for i, b in enumerate(bufs):
        k = 1500 + i
        assert bytes(b) == exp[k * 64:k * 64 + int(ln[k])].tobytes()


def test_per_packet_nf_process():
    nat, o = make_pair()
    fr, ln, dv, now = T.nat_lan_trace(20, 5)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    for i in range(20):
        b = bytearray(fr[i * 64:i * 64 + 60].tobytes())
        assert nat.process(int(dv[i]), b, int(now[i])) == exp_out[i]
        assert bytes(b) == exp[i * 64:i * 64 + 60].tobytes()


@pytest.mark.parametrize("seed,slot,max_flows,expire_us", [
    (0, 64, 64, 60_000_000),   # LAN/WAN mix, malformed frames, the table fills
    (1, 256, 128, 60_000_000),  # header edge cases (options, odd lengths) up to 256 B
    (2, 64, 256, 7),           # expiry due often: the kernel and the batch path alternate
    (3, 2048, 64, 60_000_000),  # long frames (up to 1514 B: the mailbox's whole frame)
])
def test_process_one_server(seed, slot, max_flows, expire_us):
    """vp_process_one (nf_process of the nf.h shims): vignat's persistent
    per-packet kernel, packet for packet against the oracle, with batch calls
    and an idle exit (the kernel leaves, the next packet launches it again)
    in between, and the flow state compared at the end. Each frame is its own
    buffer of len bytes (as an mbuf's data), so the oracle's frames are
    zeroed past len."""
    import time
    rng = np.random.default_rng(seed)
    n = 600
    if slot == 64:
        fr, ln, dv, now = mixed_nat_trace(rng, n, 150, max_idx=max_flows)
    else:
        fr, ln, dv = edge_nat_trace(rng, n, 100, slot=slot, long_frames=True)
        now = T.NOW0 + np.arange(n, dtype=np.int64) * 3
    F = fr.reshape(n, slot).copy()
    for i in range(n):
        F[i, ln[i]:] = 0
    exp = F.reshape(-1).copy()
    nat, o = make_pair(max_flows=max_flows, expire_us=expire_us)
    exp_out = o.run(exp, ln, dv, now, slot)
    E = exp.reshape(n, slot)
    i = 0
    while i < n:
        if i % 200 == 150:  # a batch call between single packets
            k = 20
            bufs = [bytearray(F[j, :ln[j]].tobytes()) for j in range(i, i + k)]
            out = nat.process_mbufs(bufs, dv[i:i + k], now[i:i + k])
            np.testing.assert_array_equal(out, exp_out[i:i + k])
            for j in range(k):
                assert bytes(bufs[j]) == E[i + j, :ln[i + j]].tobytes(), i + j
            i += k
            continue
        if i == 300:
            time.sleep(0.1)  # past the idle exit (VIGPATH_SERVE_IDLE_MS, 20)
        b = bytearray(F[i, :ln[i]].tobytes())
        assert nat.process(int(dv[i]), b, int(now[i])) == exp_out[i], i
        assert bytes(b) == E[i, :ln[i]].tobytes(), i
        i += 1
    check_state(nat, o, max_flows)


@pytest.mark.parametrize("slot", [64, 128])
def test_burst_port(slot):
    """vp_dev_batch.in_port: batches whose packets all arrived on one port
    (nf.c's rx bursts) pass that port instead of a per-packet array; 64-byte
    slots read it in the kernels, wider slots get an array made for them.
    Bursts alternate LAN and WAN as the trace's ports change."""
    rng = np.random.default_rng(21 + slot)
    n = 1500
    fr, ln, dv, now = mixed_nat_trace(rng, n, 60, slot=slot, max_idx=64)
    cuts = [i for i in range(1, n) if dv[i] != dv[i - 1]]
    nat, o = make_pair(max_flows=64, expire_us=50)
    check_batches(nat, o, fr, ln, dv, now, slot, cuts, one_port=True)
    check_state(nat, o, 64)


def test_first_sighting_cut():
    """The churn shape (traces.churn_trace: a quarter of the flow slots start
    new flows every batch, each flow seen many times per batch): once a
    batch's misses are mostly repeats of flows first seen in its opening
    packets, the next batches start with a segment of that many packets
    (FlowTable::fs_hint, run_batch), then the rest hits. Every batch's out
    ports and frames, and the final flow state, against the oracle; the cut
    batches run two classify launches; batches without new flows drop the
    cut again."""
    W, B = 4096, 1 << 17
    nat, o = make_pair(max_flows=1 << 14, expire_us=T.CHURN_EXPIRE_US)
    launches = []
    for k in range(10):
        fr, ln, dv, now = T.churn_trace(k, B, w=W)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        got, out = run_gpu(nat, fr, ln, dv, now, 64, affine=(int(now[0]), 0))
        assert np.array_equal(out, exp_out), k
        assert np.array_equal(got, exp), k
        launches.append(nat.last_kernel_ms()[1])
    check_state(nat, o, 1 << 14)
    assert launches[0] == 1 and all(x == 2 for x in launches[2:]), launches
    # steady batches (the flows of batch 9 again, no new flow): one cut
    # batch that finds no new flow, then single segments
    for j in range(3):
        fr, ln, dv, now = T.churn_trace(9, B, w=W)
        now = now + (j + 1)  # (later times, same flows)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        got, out = run_gpu(nat, fr, ln, dv, now, 64, affine=(int(now[0]), 0))
        assert np.array_equal(out, exp_out) and np.array_equal(got, exp), j
        launches.append(nat.last_kernel_ms()[1])
    assert launches[-2:] == [1, 1], launches
    check_state(nat, o, 1 << 14)


def test_burst_port_out_of_range():
    """A burst's port is nf_process's uint16_t device (nf.h:14): a larger
    vp_dev_batch.in_port is rejected before anything runs."""
    import torch
    nat, _ = make_pair(max_flows=64)
    n = 64
    d = torch.device("cuda:0")
    f = torch.zeros(n * 64, dtype=torch.uint8, device=d)
    ln = torch.full((n,), 60, dtype=torch.int16, device=d)
    out = torch.zeros(n, dtype=torch.int16, device=d)
    with pytest.raises(vigor_amd.VigpathError):
        nat.process_device(f, ln, 0x10000, out, 64, now0=T.NOW0, now_step=1)
    nat.process_device(f, ln, 0xFFFF, out, 64, now0=T.NOW0, now_step=1)  # (accepted)


def test_process_one_long_frame_and_empty():
    """Frames the mailbox does not take (longer than its 2048 bytes) go
    through the batch path, a zero-length frame drops, and the kernel
    serves the packets around them; all against the oracle."""
    nat, o = make_pair(max_flows=64)
    fr, ln, dv, now = T.nat_lan_trace(6, 3)
    slot = 4096
    F = np.zeros((6, slot), np.uint8)
    F[:, :64] = fr.reshape(6, 64)
    lens = ln.astype(np.int64).copy()
    lens[2] = 3000                          # past the mailbox: the batch path
    lens[4] = 0                             # nothing to parse: dropped
    # (total_length as the frame says: 46 bytes of IP; the rest is padding;
    # a frame is its buffer of len bytes, so the oracle sees zeros past len)
    for i in range(6):
        F[i, lens[i]:] = 0
    exp = F.reshape(-1).copy()
    exp_out = o.run(exp, lens.astype(np.uint16), dv, now, slot)
    E = exp.reshape(6, slot)
    for i in range(6):
        b = bytearray(F[i, :lens[i]].tobytes())
        assert nat.process(int(dv[i]), b, int(now[i])) == exp_out[i], i
        assert bytes(b) == E[i, :lens[i]].tobytes(), i
    check_state(nat, o, 64)


def test_process_one_two_contexts():
    """Two vignat contexts served one packet at a time, alternately: each
    has its own resident kernel and mailbox on its own stream; both agree
    with their oracles, then one is destroyed while the other keeps
    serving."""
    rng = np.random.default_rng(41)
    n = 300
    pairs, traces = [], []
    for k in range(2):
        fr, ln, dv, now = mixed_nat_trace(rng, n, 80, max_idx=128)
        nat, o = make_pair(max_flows=128)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        pairs.append((nat, o))
        traces.append((fr, ln, dv, now, exp, exp_out))
    import time
    t0 = time.perf_counter()
    for i in range(n):
        for k in range(2):
            if k == 1 and i == n // 2:
                pairs[0][0].close()  # the other context's kernel keeps serving
            if k == 0 and i >= n // 2:
                continue
            nat = pairs[k][0]
            fr, ln, dv, now, exp, exp_out = traces[k]
            b = bytearray(fr[i * 64:i * 64 + int(ln[i])].tobytes())
            assert nat.process(int(dv[i]), b, int(now[i])) == exp_out[i], (k, i)
            assert bytes(b) == exp[i * 64:i * 64 + int(ln[i])].tobytes(), (k, i)
    # no context waits out the other's idle exit (20 ms) at a switch: a
    # server launch stops the other context's server first (serve_yield)
    per = (time.perf_counter() - t0) / (n + n // 2)
    assert per < 5e-3, "%.2f ms per packet" % (per * 1e3)
    check_state(pairs[1][0], pairs[1][1], 128)


def test_config2_1m_flows_full_size():
    """BASELINE config 2 at its full table size (1M flows, cap 2^20): a
    warm-up batch creating every flow, then steady-state batches, checked
    packet-for-packet against the oracle."""
    nf = 1 << 20
    nat, o = make_pair(max_flows=nf)
    B = 1 << 21
    for j in range(3):
        fr, ln, dv, now = T.nat_lan_trace(B, nf, start=j * B)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        got, out = run_gpu(nat, fr, ln, dv, now, 64, affine=(int(now[0]), 1))
        assert np.array_equal(out, exp_out)
        assert orc.digest(got, 64, ln, out) == orc.digest(exp, 64, ln, exp_out)
    assert nat.live_count() == nf


def test_rejects_bad_config():
    args = ["--wan", "1", "--max-flows", "1000", "--expire", "10"]
    cfg = vigor_amd.nat_config_from_args(args, 2, DEV_MACS[:2])
    with pytest.raises(vigor_amd.VigpathError):
        vigor_amd.Nat(cfg)  # map_allocate rejects a non power of two


@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline_chunks(pinned, monkeypatch):
    """vp_process_host in several double-buffered chunks (copy stream beside
    the compute stream), pageable and page-locked frames."""
    import torch
    monkeypatch.setenv("VIGPATH_HOST_CHUNK", "700")
    rng = np.random.default_rng(17)
    fr, ln, dv, now = mixed_nat_trace(rng, 5000, 200, max_idx=256)
    nat, o = make_pair(max_flows=256, expire_us=3)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    if pinned:
        t = torch.from_numpy(fr.copy()).pin_memory()
        got = t.numpy()
    else:
        got = fr.copy()
    out = nat.process_host(got, ln, dv, now, 64)
    np.testing.assert_array_equal(out, exp_out)
    np.testing.assert_array_equal(got, exp)
    check_state(nat, o, 256)


@pytest.mark.parametrize("pinned,affine", [(False, False), (True, False),
                                           (True, True), (False, True)])
def test_host_batch_entry(pinned, affine, monkeypatch):
    """vp_process_host_batch: every per-packet array page-locked (DMA'd in
    place) or pageable (staged), time per packet or affine (nf.c's one
    current_time() per sweep is now_step 0), several chunks."""
    import torch
    monkeypatch.setenv("VIGPATH_HOST_CHUNK", "700")
    rng = np.random.default_rng(23)
    fr, ln, dv, now = mixed_nat_trace(rng, 5000, 200, max_idx=256)
    if affine:  # churn with one stamp per 64-packet sweep
        now = (now[0] + (np.arange(len(now)) // 64) * 3000).astype(np.int64)
    nat, o = make_pair(max_flows=256, expire_us=3)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)

    def host(a):
        if not pinned:
            return a.copy()
        return torch.from_numpy(a.copy()).pin_memory().numpy()
    got, lens, ind = host(fr), host(ln), host(dv)
    out = host(np.zeros(len(ln), np.uint16))
    if affine:  # one call per 64-packet sweep, its packets stamped alike
        for s in range(0, len(ln), 64):
            e = min(len(ln), s + 64)
            nat.process_host_batch(got[s * 64:e * 64], lens[s:e], ind[s:e], out[s:e],
                                   64, now0=int(now[s]), now_step=0)
    else:
        nat.process_host_batch(got, lens, ind, out, 64, now=host(now))
    np.testing.assert_array_equal(out, exp_out)
    np.testing.assert_array_equal(got, exp)
    check_state(nat, o, 256)


@pytest.mark.parametrize("n_flows,order", [(4096, "uniform"), (3, "rr"),
                                          (1 << 16, "rr")])
def test_touch_bins_steady_state(n_flows, order):
    """Steady-state batches (every packet a hit) fold their touches through
    the classify kernel's touch bins; a hot flow set overflows a bin slice
    and the fold falls back to the full log. Timestamps and LRU state must
    equal the oracle's either way."""
    nat, o = make_pair(max_flows=1 << 17)
    fr, ln, dv, now = T.nat_lan_trace(n_flows, n_flows)  # warm-up: allocate
    check_batches(nat, o, fr, ln, dv, now, 64, [])
    for j in range(2):
        start = n_flows + j * 40_000
        fr, ln, dv, now = T.nat_lan_trace(40_000, n_flows, order=order,
                                          start=start, seed=j)
        check_batches(nat, o, fr, ln, dv, now, 64, [], affine=order == "rr")
        check_state(nat, o, 1 << 17)


@pytest.mark.parametrize("order,slot", [("rr", 64), ("uniform", 64), ("rr", 128)])
def test_multiplicative_home_buckets_reprobe(order, slot, monkeypatch):
    """With the multiplicative home-bucket spread (VIGPATH_MIX=1, the layout
    the table rebuilds into for clustering key sets) a full home bucket is
    common at load 0.65. A lean 64-byte tile (every lane a fast LAN packet)
    walks the probe path on in the lane; the other tiles' packets leave the
    classify wave and finish in nat_reprobe (per-block slices for 64-byte
    tiles, one list for the per-lane path of wider slots). Outputs and state
    equal the oracle's either way."""
    monkeypatch.setenv("VIGPATH_MIX", "1")
    monkeypatch.setenv("VIGPATH_SPARSE", "-1")  # load 2/3: many reprobes
    monkeypatch.setenv("VIGPATH_LIN", "0")  # (no allocation-order layout)
    def wide(fr):  # 64-byte slots -> `slot`-byte slots, zero padded
        w = np.zeros((fr.size // 64, slot), np.uint8)
        w[:, :64] = fr.reshape(-1, 64)
        return w.reshape(-1)

    nat, o = make_pair(max_flows=4096)
    fr, ln, dv, now = T.nat_lan_trace(4000, 4000)
    check_batches(nat, o, wide(fr), ln, dv, now, slot, [1000])
    fr, ln, dv, now = T.nat_lan_trace(60_000, 4000, order=order, start=4000)
    check_batches(nat, o, wide(fr), ln, dv, now, slot, [30_000])
    check_state(nat, o, 4096)
    rng = np.random.default_rng(9)
    fr, ln, dv, now = mixed_nat_trace(rng, 5000, 3000, max_idx=4096)
    now = now + 10**8
    check_batches(nat, o, wide(fr), ln, dv, now, slot, [2000])
    check_state(nat, o, 4096)


def test_now_buffer_reusable_after_return():
    """vp_process_device with a per-packet time array: the array may be
    overwritten (or freed) as soon as the call returns, with no
    synchronisation, and the timestamps the batch leaves behind must still be
    the ones it carried (the steady-state fold must not read it late)."""
    import torch
    nat, o = make_pair(max_flows=1 << 16)
    n_flows = 4096
    fr, ln, dv, now = T.nat_lan_trace(n_flows, n_flows)
    check_batches(nat, o, fr, ln, dv, now, 64, [])
    d = torch.device("cuda:0")
    B = 1 << 18  # steady state: every packet a hit, touch bins
    fr, ln, dv, now = T.nat_lan_trace(B, n_flows, start=n_flows)
    o.run(fr.copy(), ln, dv, now, 64)
    f = torch.from_numpy(fr).to(d)
    l_ = torch.from_numpy(ln.view(np.int16)).to(d)
    i_ = torch.from_numpy(dv.view(np.int16)).to(d)
    out = torch.zeros(B, dtype=torch.int16, device=d)
    nt = torch.from_numpy(now).to(d)
    nat.process_device(f, l_, i_, out, 64, now=nt)
    nt.fill_(0)  # on torch's stream, unordered with the library's
    del nt
    torch.cuda.synchronize()
    check_state(nat, o, 1 << 16)


@pytest.mark.parametrize("max_flows,n_flows,expire_us,mix", [
    (4096, 3000, 60_000_000, "0"),   # misses in lean tiles, then hits
    (256, 400, 60_000_000, "0"),     # table full inside lean tiles
    (1024, 900, 2, "0"),             # expiry between lean tiles
    (4096, 3000, 60_000_000, "1"),   # multiplicative home buckets: reprobes
])
def test_lean_tiles(max_flows, n_flows, expire_us, mix, monkeypatch):
    """The classify kernel's lean tile (every lane a fast-path LAN packet:
    batched CRC reads, branch-free bucket match, whole-tile store) beside
    per-lane tiles (one malformed packet each), TCP and UDP, with new flows,
    a full table, expiry and reprobes; several batches."""
    monkeypatch.setenv("VIGPATH_MIX", mix)
    if mix == "1":  # (keep the spread: no allocation-order layout)
        monkeypatch.setenv("VIGPATH_LIN", "0")
    rng = np.random.default_rng(max_flows + n_flows)
    fr, ln, dv, now = lan_tile_trace(rng, 40_000, n_flows)
    nat, o = make_pair(max_flows=max_flows, expire_us=expire_us)
    check_batches(nat, o, fr, ln, dv, now, 64, [4096, 4100, 20_000])
    check_state(nat, o, max_flows)


def test_prepared_device_step():
    """Nat.device_step (the bench's prepared C-ABI call over fixed buffers,
    affine time) gives what the oracle gives, batch after batch, with the
    per-launch timing events (vp_kernel_timing) off, on and off again."""
    import torch
    nf = 1 << 12
    nat, o = make_pair(max_flows=nf)
    B = 1 << 14
    d = torch.device("cuda:0")
    f_t = torch.empty(B * 64, dtype=torch.uint8, device=d)
    l_t = torch.empty(B, dtype=torch.int16, device=d)
    i_t = torch.empty(B, dtype=torch.int16, device=d)
    o_t = torch.zeros(B, dtype=torch.int16, device=d)
    step = nat.device_step(f_t, l_t, i_t, o_t, 64)
    for j in range(3):
        nat.kernel_timing(j == 1)
        fr, ln, dv, now = T.nat_lan_trace(B, nf + 100, start=j * B)
        f_t.copy_(torch.from_numpy(fr))
        l_t.copy_(torch.from_numpy(ln.view(np.int16)))
        i_t.copy_(torch.from_numpy(dv.view(np.int16)))
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        step(int(now[0]), 1)
        torch.cuda.synchronize()
        ms, launches = nat.last_kernel_ms()
        assert launches >= 1 and (ms > 0) == (j == 1), (j, ms, launches)
        assert np.array_equal(o_t.cpu().numpy().view(np.uint16), exp_out)
        assert np.array_equal(f_t.cpu().numpy(), exp)
    check_state(nat, o, nf)


def test_rebuild_inside_phase_b_then_phase_c():
    """One vp_process_device call whose phase B allocates enough flows to
    switch the table to the allocation-order layout (tbl_try_linear rebuilds
    the buckets at half the count, freeing the old array), followed in the
    same segment by WAN replies to those flows (phase C reads the buckets).
    Round 2's nat_churn EIO was a stale bucket pointer in exactly this spot;
    the layout switch must happen here and the results equal the oracle's."""
    cap, n_new = 1024, 600  # > cap / 2 live: the linear layout is tried
    nat, o = make_pair(max_flows=cap)
    fr, ln, dv, now = T.nat_lan_trace(n_new, n_new)
    rep = fr.reshape(n_new, 64).copy()  # WAN replies to flows 0..n_new-1
    rep[:, 26:34] = 0                                  # src 0.0.0.0, dst (unchecked)
    rep[:, 34:36] = 0                                  # src_port = flow dst_port 0
    idx = np.arange(n_new)
    rep[:, 36], rep[:, 37] = idx & 0xFF, idx >> 8      # dst_port = external port (raw)
    fr2 = np.concatenate([fr, rep.reshape(-1)])
    ln2 = np.concatenate([ln, ln])
    dv2 = np.concatenate([dv, np.ones(n_new, np.uint16)])
    now2 = T.NOW0 + np.arange(2 * n_new, dtype=np.int64)
    before = nat.table_stats()
    check_batches(nat, o, fr2, ln2, dv2, now2, 64, [])
    after = nat.table_stats()
    assert after["rebuilds"] > before["rebuilds"], (before, after)
    assert after["buckets"] < before["buckets"], (before, after)  # the array moved
    fr3, ln3, dv3, now3 = T.nat_lan_trace(3 * n_new, n_new, start=2 * n_new)
    check_batches(nat, o, fr3, ln3, dv3, now3, 64, [1000])
    check_state(nat, o, cap)


@pytest.mark.parametrize("slot,max_len", [(80, 80), (96, 96), (128, 128), (192, 192),
                                          (256, 256), (512, 512), (1536, 1518),
                                          (2048, 1518)])
def test_wide_slots(slot, max_len):
    """Frames of 60..1518 bytes in wide slots through nat_classify_wide<G>
    (tile_tail_sums: the L4 sum's bytes past the first 64, G lanes per
    frame): new flows, hits, WAN replies, padded frames, odd lengths and
    malformed frames, several batches; out ports, every slot byte and the
    table state equal the oracle's."""
    rng = np.random.default_rng(slot)
    fr, ln, dv, now = wide_nat_trace(rng, 6000, 400, slot, max_len=max_len)
    nat, o = make_pair(max_flows=1024)
    check_batches(nat, o, fr, ln, dv, now, slot, [700, 700 + 64 * 5, 4100])
    check_state(nat, o, 1024)


@pytest.mark.parametrize("slot", [128, 1536])
def test_wide_steady_state(slot):
    """Bench-shaped wide traffic (every packet a hit after the warm-up, the
    lean tile with the touch bins) in 1518-byte or 124-byte frames with a
    payload pattern."""
    nf = 1 << 12
    nat, o = make_pair(max_flows=nf)
    flen = min(slot - 4, 1514)
    for j, B in enumerate((nf, 1 << 15, 1 << 15)):
        start = 0 if j == 0 else nf + (j - 1) * (1 << 15)
        fl = T.flow_order(B, nf, start=start)
        z = np.zeros_like(fl)
        fr, ln = T.udp_frames(T.ip4(10, 0, 0, 0) + (fl >> 16), z, fl & 0xFFFF, z,
                              slot=slot, frame_len=flen)
        f2 = fr.reshape(B, slot)
        f2[:, 42:flen] = (np.arange(42, flen) * 7 % 251).astype(np.uint8)
        dv = np.zeros(B, np.uint16)
        now = T.NOW0 + np.arange(start, start + B, dtype=np.int64)
        check_batches(nat, o, fr, ln, dv, now, slot, [], affine=True)
    check_state(nat, o, nf)
