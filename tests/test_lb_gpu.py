"""viglb on the GPU vs the oracle (bit-exact out ports, rewritten frames,
flow and backend state).

Every test calls the product through the C-ABI (libvigpath.so via
vigor_amd); the oracle (oracle/liborc.so) is only the checker.
"""
import numpy as np
import pytest

import orc
import vigor_amd
from gpuh import check_batches, run_gpu
from tracegen import mixed_lb_trace
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu

DEV_MACS = [bytes([0x10 * d + i for i in range(6)]) for d in range(3)]


def make_pair(flow_cap=1024, bcap=32, height=97, fexp=60_000_000,
              bexp=3_600_000_000, wan=2, n_dev=3):
    args = ["--flow-capacity", str(flow_cap), "--backend-capacity", str(bcap),
            "--cht-height", str(height), "--flow-expiration", str(fexp),
            "--backend-expiration", str(bexp), "--wan", str(wan)]
    cfg = vigor_amd.lb_config_from_args(args, n_dev, DEV_MACS[:n_dev])
    gpu = vigor_amd.Lb(cfg, gpu=0)
    ocfg = orc.LbCfg(flow_capacity=flow_cap, flow_expiration_time=fexp,
                     backend_capacity=bcap, cht_height=height,
                     backend_expiration_time=bexp, wan_device=wan,
                     n_devices=n_dev)
    for d in range(n_dev):
        ocfg.device_macs[d][:] = list(DEV_MACS[d])
    return gpu, orc.Oracle("lb", ocfg)


def check_state(lb, oracle):
    g = lb.dump()
    o = oracle.lb_dump(lb.cfg.flow_capacity, lb.cfg.backend_capacity)
    for x, y in zip(g, o):  # flows, then backends
        np.testing.assert_array_equal(x[0], y[0])
        live = y[0] == 1
        for a, b in zip(x[1:], y[1:]):
            np.testing.assert_array_equal(a[live], b[live])


def concat(*traces):
    return tuple(np.concatenate(x) for x in zip(*traces))


def test_config4_heartbeats_then_traffic():
    lb, o = make_pair(flow_cap=4096, bcap=256, height=257)
    hb = T.lb_heartbeats(256)
    tr = T.lb_traffic(30_000, 3000)
    fr, ln, dv, now = concat(hb, tr)
    check_batches(lb, o, fr, ln, dv, now, 64, [100, 256, 5000])
    check_state(lb, o)


@pytest.mark.parametrize("seed,fcap,fexp,bexp,quiet,cuts", [
    (0, 1024, 60_000_000, 3_600_000, None, [100, 2000]),   # steady + hb mix
    (1, 64, 60_000_000, 3_600_000, None, [2500]),          # flow table full
    (2, 256, 2, 3_600_000, None, [1, 2, 500, 4000]),       # flow expiry
    (3, 1024, 60_000_000, 2, (1000, 3500), [1500, 3600]),  # backends die
    (4, 1024, 3, 2, (500, 4500), []),                      # both, one batch
])
def test_mixed_traces(seed, fcap, fexp, bexp, quiet, cuts):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_lb_trace(rng, 6000, 300, 20, quiet=quiet)
    lb, o = make_pair(flow_cap=fcap, fexp=fexp, bexp=bexp)
    check_batches(lb, o, fr, ln, dv, now, 64, cuts)
    check_state(lb, o)


def test_burst_port():
    """vp_dev_batch.in_port: bursts of heartbeats (LAN ports) and WAN
    traffic, each passed with its one port instead of a port array (the
    64-byte tile and the queue rounds read it), state compared at the end."""
    rng = np.random.default_rng(31)
    fr, ln, dv, now = mixed_lb_trace(rng, 3000, 200, 20)
    cuts = [i for i in range(1, len(dv)) if dv[i] != dv[i - 1]]
    lb, o = make_pair(flow_cap=256, fexp=40)
    check_batches(lb, o, fr, ln, dv, now, 64, cuts, one_port=True)
    check_state(lb, o)


def test_backend_table_full_and_generic_slots():
    rng = np.random.default_rng(8)
    fr, ln, dv, now = mixed_lb_trace(rng, 4000, 200, 40, hb_frac=0.1,
                                     slot=128)
    lb, o = make_pair(bcap=16, height=17)
    check_batches(lb, o, fr, ln, dv, now, 128, [333, 2000])
    check_state(lb, o)


def test_config4_256_backends_1m_flows_full_size():
    """BASELINE config 4 at full size: 256 backends, CHT height 257, flow
    capacity 2^20, 1M flows."""
    nf = 1 << 20
    lb, o = make_pair(flow_cap=nf, bcap=256, height=257)
    hb = T.lb_heartbeats(256)
    exp = hb[0].copy()
    exp_out = o.run(exp, hb[1], hb[2], hb[3], 64)
    got, out = run_gpu(lb, *hb, 64)
    assert np.array_equal(out, exp_out) and np.array_equal(got, exp)
    B = 1 << 21
    for j in range(2):
        fr, ln, dv, now = T.lb_traffic(B, nf, start=j * B)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        got, out = run_gpu(lb, fr, ln, dv, now, 64, affine=(int(now[0]), 1))
        assert np.array_equal(out, exp_out)
        assert orc.digest(got, 64, ln, out) == orc.digest(exp, 64, ln, exp_out)
    assert lb.live_count() == nf + 256


def test_rejects_bad_config():
    with pytest.raises(vigor_amd.VigpathError):
        make_pair(height=96)  # not prime
    with pytest.raises(vigor_amd.VigpathError):
        make_pair(bcap=128, height=97)  # backends >= height
    with pytest.raises(vigor_amd.VigpathError):
        make_pair(flow_cap=1000)


def test_stale_frees_keep_shard_count():
    """Flows whose backend died while no backend is alive are erased and
    their indices freed (lb_stale_free_seq) — cycle after cycle. The bucket
    bookkeeping must follow (shard_live == live: the layout and rebuild
    checks count it), so the table does not rebuild on every check; outputs
    and state equal the oracle's throughout."""
    nb, nfl = 20, 200
    lb, o = make_pair(flow_cap=256, bexp=5_000)  # backends expire after 5 ms
    for c in range(12):
        t = T.NOW0 + c * 10_000_000
        stale = T.lb_traffic(nfl, nfl)            # backends expired: stale frees
        hb = T.lb_heartbeats(nb, t0=t + 1_000)
        fresh = T.lb_traffic(2 * nfl, nfl)        # re-balanced, new indices
        stale = stale[:3] + (t + np.arange(nfl, dtype=np.int64),)
        fresh = fresh[:3] + (t + 2_000 + np.arange(2 * nfl, dtype=np.int64),)
        fr, ln, dv, now = concat(stale, hb, fresh)
        check_batches(lb, o, fr, ln, dv, now, 64, [nfl + 7])
        st = lb.table_stats(0)
        assert st["shard_live"] == st["live"], (c, st)
    check_state(lb, o)
    assert lb.table_stats(0)["rebuilds"] <= 4, lb.table_stats(0)
