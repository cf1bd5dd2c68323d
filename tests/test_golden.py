"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py
from the oracle glue over the REFERENCE's own libVig, oracle/_ref): the
restated oracle and the GPU path must both reproduce them bit-exact: out
ports, every frame byte, and which indices are allocated with their
timestamps. These run where the reference is absent (the GPU box). They pin
the libVig layer; NF-level glue semantics are parity-unpinned by them (the
restated glue is on both sides; see golden_cases.py and DESIGN.md §7)."""
import numpy as np
import pytest

import golden_cases as G
from vigor_amd import traces as T
from gpuh import run_gpu

NAMES = sorted(G.CASES)


def check(name, out, frames, alloc, ts):
    g = G.load(name)
    bad = np.nonzero(out != g["out_dev"])[0]
    assert bad.size == 0, "%s: out port mismatch at %s" % (name, bad[:10])
    badf = np.nonzero((frames.reshape(-1, 64) != g["out_frames"].reshape(-1, 64))
                      .any(axis=1))[0]
    assert badf.size == 0, "%s: frame mismatch at %s" % (name, badf[:10])
    np.testing.assert_array_equal(alloc, g["alloc"])
    np.testing.assert_array_equal(ts, g["ts"])


@pytest.mark.parametrize("name", NAMES)
def test_fixture_made_by_reference_libvig(name):
    g = G.load(name)
    assert str(g["impl"]) == "reference"
    assert g["lens"].shape[0] == G.N and g["frames"].size == G.N * 64


@pytest.mark.parametrize("name", NAMES)
def test_restated_oracle_reproduces_golden(name):
    g = G.load(name)
    o = G.oracle(name, ref=False)
    fr = g["frames"].copy()
    out = o.run(fr, g["lens"], g["in_dev"], g["now"], 64)
    check(name, out, fr, *G.oracle_state(name, o))


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(name):
    """Two batches (split at packet 1500) through vp_process_device."""
    g = G.load(name)
    nf = G.gpu(name)
    fr = g["frames"]
    outs, frames = [], []
    for a, b in ((0, 1500), (1500, G.N)):
        f, o = run_gpu(nf, fr[a * 64:b * 64], g["lens"][a:b], g["in_dev"][a:b],
                       g["now"][a:b], 64)
        frames.append(f)
        outs.append(o)
    check(name, np.concatenate(outs), np.concatenate(frames), *G.gpu_state(name, nf))


def _big_check(fr, out, live):
    import orc
    g = G.load("nat_1m_digest")
    assert str(g["impl"]) == "reference"
    k = 1024 * 64
    np.testing.assert_array_equal(out[:1024], g["head_out"])
    np.testing.assert_array_equal(out[-1024:], g["tail_out"])
    np.testing.assert_array_equal(fr[:k], g["head_frames"])
    np.testing.assert_array_equal(fr[-k:], g["tail_frames"])
    lens = np.full(out.shape[0], 60, np.uint16)
    assert orc.digest(fr, 64, lens, out) == int(g["digest"])
    assert live == int(g["live"])


def test_restated_oracle_reproduces_1m_digest():
    fr, ln, dv, now = G.big_trace()
    o = G.big_oracle()
    out = o.run(fr, ln, dv, now, 64)
    _big_check(fr, out, o.L.orc_nat_flow_count(o.h))


@pytest.mark.gpu
def test_gpu_reproduces_1m_digest():
    """BASELINE configs[1] table size through vp_process_device: 1M new
    flows then 1M hits (two 2^20-packet batches, affine time)."""
    fr, ln, dv, now = G.big_trace()
    nat = G.big_gpu()
    h = G.BIG_PACKETS // 2
    frames, outs = [], []
    for a in (0, h):
        f, o = run_gpu(nat, fr[a * 64:(a + h) * 64], ln[a:a + h], dv[a:a + h],
                       now[a:a + h], 64, affine=(int(now[a]), 1))
        frames.append(f)
        outs.append(o)
    _big_check(np.concatenate(frames), np.concatenate(outs), nat.live_count())


# ---- the bench's own shape (BASELINE configs[1]; bench.py) ----------------

def _bench_golden():
    g = G.load("nat_bench_shape")
    assert str(g["impl"]) == "reference"
    return g


def test_restated_oracle_reproduces_bench_shape():
    g = _bench_golden()
    o = G.nat_oracle(G.BENCH_FLOWS)
    for k in range(G.BENCH_BATCHES):
        acc = [0]

        def add(p0, fr, out, k=k):
            acc[0] += T.batch_digest(fr, out, 64, p0 - k * G.BENCH_BATCH)
        G.run_oracle_chunks(o, G.BENCH_BATCH, G.BENCH_FLOWS, k * G.BENCH_BATCH, add)
        assert acc[0] % (1 << 64) == int(g["batch_digest"][k]), k
    alloc, ts, _ = o.nat_dump(G.BENCH_FLOWS)
    assert T.state_digest(alloc, ts) == int(g["state_digest"])


@pytest.mark.gpu
def test_gpu_reproduces_bench_shape():
    """bench.py's workload through vp_process_device: 2^24-packet batches
    over 1M flows (affine time), batch 0 allocating every flow and batch 1
    in steady state, where each flow is touched 16 times and the stamps fold
    through the touch bins. Every output byte (batch digest) and the whole
    table state (alloc + ts digest) equal the reference's."""
    import torch
    g = _bench_golden()
    nat = G.nat_gpu(G.BENCH_FLOWS)
    d = torch.device("cuda:0")
    B = G.BENCH_BATCH
    lens = torch.full((B,), 60, dtype=torch.int16, device=d)
    ind = torch.zeros(B, dtype=torch.int16, device=d)
    out = torch.zeros(B, dtype=torch.int16, device=d)
    for k in range(G.BENCH_BATCHES):
        fr, _, _, _ = T.nat_lan_trace(B, G.BENCH_FLOWS, start=k * B)
        f = torch.from_numpy(fr).to(d)
        del fr
        nat.process_device(f, lens, ind, out, 64, now0=T.NOW0 + k * B, now_step=1)
        torch.cuda.synchronize()
        dig = T.batch_digest(f.cpu().numpy(), out.cpu().numpy().view(np.uint16), 64)
        assert dig == int(g["batch_digest"][k]), "batch %d digest" % k
        del f
    alloc, ts, _ = nat.dump()
    assert T.state_digest(alloc, ts) == int(g["state_digest"])
    assert nat.live_count() == int(g["live"])


@pytest.mark.gpu
def test_c_step_loop_reproduces_bench_shape():
    """The same batches through bench.py's timed loop in C (host/steps.c,
    Nat.device_steps: one vp_process_device per batch with no interpreter
    between them): the last batch's bytes and the table state equal the
    reference's, as through one call at a time."""
    import torch
    g = _bench_golden()
    nat = G.nat_gpu(G.BENCH_FLOWS)
    d = torch.device("cuda:0")
    B = G.BENCH_BATCH
    lens = torch.full((B,), 60, dtype=torch.int16, device=d)
    ind = torch.zeros(B, dtype=torch.int16, device=d)
    out = torch.zeros(B, dtype=torch.int16, device=d)
    bufs = []
    for k in range(G.BENCH_BATCHES):
        fr, _, _, _ = T.nat_lan_trace(B, G.BENCH_FLOWS, start=k * B)
        bufs.append(torch.from_numpy(fr).to(d))
        del fr
    run = nat.device_steps(bufs, lens, ind, out, 64)
    run([T.NOW0 + k * B for k in range(G.BENCH_BATCHES)], 1)
    torch.cuda.synchronize()
    k = G.BENCH_BATCHES - 1
    dig = T.batch_digest(bufs[k].cpu().numpy(), out.cpu().numpy().view(np.uint16), 64)
    assert dig == int(g["batch_digest"][k]), "batch %d digest" % k
    del bufs
    alloc, ts, _ = nat.dump()
    assert T.state_digest(alloc, ts) == int(g["state_digest"])
    assert nat.live_count() == int(g["live"])


# ---- BASELINE configs[4] table size (16M flows) ---------------------------

def _16m_golden():
    g = G.load("nat_16m_digest")
    assert str(g["impl"]) == "reference"
    return g


def test_restated_oracle_reproduces_16m_digest():
    g = _16m_golden()
    o = G.nat_oracle(G.F16M_FLOWS)
    acc = [0]

    def add(p0, fr, out):
        acc[0] += T.batch_digest(fr, out, 64, p0)
        if p0 == 0:
            np.testing.assert_array_equal(fr[:1024 * 64], g["head_frames"])
    G.run_oracle_chunks(o, G.F16M_PACKETS, G.F16M_FLOWS, 0, add)
    assert acc[0] % (1 << 64) == int(g["digest"])
    alloc, ts, _ = o.nat_dump(G.F16M_FLOWS)
    assert T.state_digest(alloc, ts) == int(g["state_digest"])


# ---- wide slots: 60..1518-byte frames in 2048-byte slots ------------------

def _wide_golden():
    g = G.load("nat_wide")
    assert str(g["impl"]) == "reference"
    fr, ln, dv, now = G.wide_trace()
    # the trace regenerates bit-identically from its seed (no generator drift)
    np.testing.assert_array_equal(G.slot_hashes(fr, G.WIDE_SLOT), g["in_hash"])
    assert int(ln.max()) == 1518
    return g, (fr, ln, dv, now)


def _wide_check(g, out, frames, alloc, ts):
    bad = np.nonzero(out != g["out_dev"])[0]
    assert bad.size == 0, "out port mismatch at %s" % bad[:10]
    badf = np.nonzero(G.slot_hashes(frames, G.WIDE_SLOT) != g["out_hash"])[0]
    assert badf.size == 0, "frame mismatch at %s" % badf[:10]
    np.testing.assert_array_equal(alloc, g["alloc"])
    np.testing.assert_array_equal(np.where(alloc == 1, ts, 0), g["ts"])


def test_restated_oracle_reproduces_wide():
    g, (fr, ln, dv, now) = _wide_golden()
    o = G.wide_oracle()
    f = fr.copy()
    out = o.run(f, ln, dv, now, G.WIDE_SLOT)
    alloc, ts, _ = o.nat_dump(G.WIDE_CAP)
    _wide_check(g, out, f, alloc, ts)


@pytest.mark.gpu
@pytest.mark.parametrize("slot", [2048, 1536])
def test_gpu_reproduces_wide(slot):
    """The reference's answers for 1518-byte frames through the wide-slot
    kernels, in the fixture's 2048-byte slots and re-packed into 1536-byte
    slots (every frame fits; the bytes past 1536 are not the NF's), two
    batches."""
    g, (fr, ln, dv, now) = _wide_golden()
    S = G.WIDE_SLOT
    src = fr.reshape(-1, S)[:, :slot].copy().reshape(-1)
    nat = G.wide_gpu()
    outs, frames = [], []
    for a, b in ((0, 1500), (1500, G.WIDE_N)):
        f, o = run_gpu(nat, src[a * slot:b * slot], ln[a:b], dv[a:b], now[a:b], slot)
        frames.append(f)
        outs.append(o)
    got = np.concatenate(frames).reshape(-1, slot)
    full = fr.reshape(-1, S).copy()
    full[:, :slot] = got  # the tail past `slot` is the unmodified input
    alloc, ts, _ = nat.dump()
    _wide_check(g, np.concatenate(outs), full.reshape(-1), alloc, ts)
