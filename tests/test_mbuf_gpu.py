"""DPDK-shaped host batches on the GPU (vp_process_mbufs, vp_mbuf.hip): every
frame in its own mbuf of a pool (2304-byte elements, data at 256: DPDK's
rte_mbuf + headroom + 2 KB data room), the batch a pointer array in rx order
(reference nf.c:186-214), frames read and rewritten in place by the GPU
through vp_register_host (mode "gpu") or gathered and written back by host
threads (mode "host"). Out ports, the frames' bytes and the final state
are compared with the oracle run over the same packets (frames in slots,
bytes past each length zero: the mbuf path reads them as 0)."""
import numpy as np
import pytest
import orc
from tracegen import (edge_nat_trace, mixed_bridge_trace, mixed_fw_trace,
                      mixed_lb_trace, mixed_pol_trace, wide_nat_trace)
from vigor_amd import traces as T

import test_nat_gpu as NG

pytestmark = pytest.mark.gpu

SLOT = 2048  # the oracle's slots (frames up to 1518 B)

# VIGPATH_MBUF_MODE: "gpu" (the GPU reads and writes the registered mbufs),
# "host" (host threads gather headers into pinned slots and write them back)
MODES = ["gpu", "host"]


def zero_past_len(fr, ln, slot):
    f = fr.reshape(-1, slot)
    for i in np.nonzero(ln < slot)[0]:
        f[i, ln[i]:] = 0
    return fr


def to_pool(fr, ln, slot, rng, spare=1.3, shift=None, pinned=False):
    """The trace's frames in shuffled mbufs of a pool; returns (pool, bufs,
    ptrs)."""
    n = len(ln)
    pool = T.MbufPool(int(n * spare) + 1, pinned=pinned)
    bufs = rng.permutation(pool.n)[:n]
    pool.put(bufs, fr, slot, ln, shift)
    return pool, bufs, pool.ptrs(bufs, shift)


def run_mbufs(nf, pool, ptrs, ln, dv, now, register=True, affine=None):
    if register:
        nf.register_host(pool.mem)
    out = np.zeros(len(ln), np.uint16)
    ln16, dv16 = np.ascontiguousarray(ln, np.uint16), np.ascontiguousarray(dv, np.uint16)
    if affine is None:
        nf.process_mbuf_batch(ptrs, ln16, dv16, out, now=np.ascontiguousarray(now, np.int64))
    else:
        nf.process_mbuf_batch(ptrs, ln16, dv16, out, now0=affine[0], now_step=affine[1])
    return out


def compare(pool, bufs, ln, exp, exp_out, out, slot, shift=None):
    bad = np.nonzero(out != exp_out)[0]
    assert bad.size == 0, "out port mismatch at %s: %s vs %s" % (bad[:10], out[bad[:10]],
                                                                exp_out[bad[:10]])
    got = pool.get(bufs, slot, ln, shift).reshape(-1, slot)
    e = exp.reshape(-1, slot)
    badf = [i for i in range(len(ln)) if got[i, :ln[i]].tobytes() != e[i, :ln[i]].tobytes()]
    assert not badf, "frame mismatch at %s" % badf[:10]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("chunk", ["700", "4096"])
def test_nat_mixed_sizes(chunk, mode, monkeypatch):
    """60-1518-byte frames (tail sums over the bytes past 64, padding past
    total_length, TCP and UDP), WAN replies, malformed frames, new flows and
    hits, churn; several chunks of the pipeline."""
    monkeypatch.setenv("VIGPATH_HOST_CHUNK", chunk)
    monkeypatch.setenv("VIGPATH_MBUF_MODE", mode)
    rng = np.random.default_rng(41)
    n = 6000
    fr, ln, dv, now = wide_nat_trace(rng, n, 300, SLOT)
    zero_past_len(fr, ln, SLOT)
    nat, o = NG.make_pair(max_flows=512, expire_us=2)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, SLOT)
    pool, bufs, ptrs = to_pool(fr, ln, SLOT, rng)
    out = run_mbufs(nat, pool, ptrs, ln, dv, now)
    compare(pool, bufs, ln, exp, exp_out, out, SLOT)
    assert (out == 1).sum() > 1000  # (forwarded LAN packets)
    NG.check_state(nat, o, 512)


@pytest.mark.parametrize("mode", MODES)
def test_nat_options_take_whole_frames(mode, monkeypatch):
    """IPv4 options on frames longer than 64 bytes (the rewrite reaches past
    byte 64: the chunk takes whole-frame slots), short and odd frames, IHL <
    5, total_length past the packet (edge_nat_trace), mixed with plain
    chunks; affine time."""
    monkeypatch.setenv("VIGPATH_HOST_CHUNK", "500")
    monkeypatch.setenv("VIGPATH_MBUF_MODE", mode)
    rng = np.random.default_rng(42)
    n = 3000
    fr, ln, dv = edge_nat_trace(rng, n, 200, slot=SLOT, long_frames=True)
    # the first 1500 packets without options (header-slot chunks)
    f = fr.reshape(n, SLOT)
    f[:1500, 14] = (f[:1500, 14] & 0xF0) | 5
    zero_past_len(fr, ln, SLOT)
    now = T.NOW0 + np.arange(n, dtype=np.int64)
    nat, o = NG.make_pair(max_flows=512)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, SLOT)
    pool, bufs, ptrs = to_pool(fr, ln, SLOT, rng)
    out = run_mbufs(nat, pool, ptrs, ln, dv, now, affine=(T.NOW0, 1))
    compare(pool, bufs, ln, exp, exp_out, out, SLOT)
    NG.check_state(nat, o, 512)


@pytest.mark.parametrize("mode", MODES)
def test_nat_unregistered_and_unaligned(mode, monkeypatch):
    """Frames outside the registered memory (their chunks are staged through
    the host), frames at data offsets that are not multiples of 16 (read and
    written byte by byte), a pinned pool and pinned arrays."""
    import torch
    monkeypatch.setenv("VIGPATH_HOST_CHUNK", "600")
    monkeypatch.setenv("VIGPATH_MBUF_MODE", mode)
    rng = np.random.default_rng(43)
    n = 4000
    fr, ln, dv, now = wide_nat_trace(rng, n, 200, SLOT, max_len=600)
    zero_past_len(fr, ln, SLOT)
    shift = np.zeros(n, np.int64)
    shift[rng.random(n) < 0.05] = 3
    nat, o = NG.make_pair(max_flows=512)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, SLOT)
    pool = T.MbufPool(2 * n, pinned=True)
    bufs = rng.permutation(n)             # the registered half
    bufs[2400:3000] = n + np.arange(600)  # chunk 4: all in the unregistered half
    bufs[100] = n + 700                   # chunk 0: one frame there
    pool.put(bufs, fr, SLOT, ln, shift)
    ptrs = pool.ptrs(bufs, shift)
    ok = bufs < n
    nat.register_host(pool.mem[:n * pool.stride])
    pin = lambda a: torch.from_numpy(a).pin_memory().numpy()  # noqa: E731
    out = pin(np.zeros(n, np.uint16))
    nat.process_mbuf_batch(pin(ptrs), pin(ln.astype(np.uint16)), pin(dv.astype(np.uint16)),
                           out, now=pin(now.astype(np.int64)))
    compare(pool, bufs, ln, exp, exp_out, out, SLOT, shift)
    assert ok.sum() < n
    NG.check_state(nat, o, 512)


def test_nat_pool_not_registered():
    """No registered memory: the whole batch is staged through the host
    (the nf.h shims' path), bit-exact as well."""
    rng = np.random.default_rng(44)
    fr, ln, dv, now = wide_nat_trace(rng, 1500, 100, SLOT, max_len=400)
    zero_past_len(fr, ln, SLOT)
    nat, o = NG.make_pair(max_flows=256)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, SLOT)
    pool, bufs, ptrs = to_pool(fr, ln, SLOT, rng)
    out = run_mbufs(nat, pool, ptrs, ln, dv, now, register=False)
    compare(pool, bufs, ln, exp, exp_out, out, SLOT)


def _other(kind):
    if kind == "fw":
        import test_fw_gpu as M
        return M.make_pair(max_flows=256, expire_us=5)
    if kind == "pol":
        import test_pol_gpu as M
        return M.make_pair()
    if kind == "bridge":
        import test_bridge_gpu as M
        return M.make_pair()
    import test_lb_gpu as M
    return M.make_pair()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("kind", ["fw", "pol", "bridge", "lb"])
def test_other_nfs(kind, mode, monkeypatch):
    """vigfw (MACs rewritten: header slots), vigpol and vigbridge (never
    rewritten: no write-back), viglb (whole-frame slots) through the mbuf
    path, frames longer than 64 bytes where the NF reads them."""
    monkeypatch.setenv("VIGPATH_HOST_CHUNK", "800")
    monkeypatch.setenv("VIGPATH_MBUF_MODE", mode)
    rng = np.random.default_rng(45)
    n = 3000
    slot = 256
    if kind == "fw":
        fr, ln, dv, now = mixed_fw_trace(rng, n, 100, slot=slot)
    elif kind == "pol":
        fr, ln, dv, now = mixed_pol_trace(rng, n, 100, slot=slot, big=250)
    elif kind == "bridge":
        fr, ln, dv, now = mixed_bridge_trace(rng, n, 120, n_dev=3, slot=slot)
    else:
        fr, ln, dv, now = mixed_lb_trace(rng, n, 150, 12)
        slot = 64
    zero_past_len(fr, ln, slot)
    nf, o = _other(kind)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, slot)
    pool, bufs, ptrs = to_pool(fr, ln, slot, rng)
    out = run_mbufs(nf, pool, ptrs, ln, dv, now)
    compare(pool, bufs, ln, exp, exp_out, out, slot)
