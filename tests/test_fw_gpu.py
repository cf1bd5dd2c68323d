"""vigfw on the GPU vs the oracle (bit-exact out ports, frames and state).

Every test calls the product through the C-ABI (libvigpath.so via
vigor_amd); the oracle (oracle/liborc.so) is only the checker. Reference
behaviour: vigfw/fw_main.c:21-80, fw_flowmanager.c:38-86.
"""
import numpy as np
import pytest
import orc
import vigor_amd
from gpuh import check_batches, run_gpu
from tracegen import mixed_fw_trace
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu

DEV_MACS = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17"),
            T.mac("22:23:24:25:26:27")]
END_MACS = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01"),
            T.mac("01:23:45:67:89:02")]


def make_pair(max_flows=65536, expire_us=60_000_000, wan=1, n_dev=3):
    args = ["--wan", str(wan), "--expire", str(expire_us), "--max-flows",
            str(max_flows)]
    for d in range(n_dev):
        args += ["--eth-dest", "%d,%s" % (d, END_MACS[d].hex(":"))]
    cfg = vigor_amd.fw_config_from_args(args, n_dev, DEV_MACS[:n_dev])
    gpu = vigor_amd.Fw(cfg, gpu=0)
    ocfg = orc.fw_cfg(wan=wan, expire_us=expire_us, max_flows=max_flows,
                      device_macs=DEV_MACS[:n_dev],
                      endpoint_macs=END_MACS[:n_dev], n_devices=n_dev)
    return gpu, orc.Oracle("fw", ocfg)


def check_state(fw, oracle, max_flows):
    ga, gts, gk, gd = fw.dump()
    oa, ots, ok, od = oracle.fw_dump(max_flows)
    np.testing.assert_array_equal(ga, oa)
    live = oa == 1
    np.testing.assert_array_equal(gts[live], ots[live])
    np.testing.assert_array_equal(gk[live], ok[live])
    np.testing.assert_array_equal(gd[live], od[live])


@pytest.mark.parametrize("seed,max_flows,expire_us,n_flows,cuts", [
    (0, 64, 60_000_000, 40, [100, 2000]),       # steady + replies
    (1, 64, 1, 100, [1, 2, 3, 500, 4000]),       # expiry every few packets
    (2, 16, 60_000_000, 40, [2500]),             # table full: LAN still out
    (3, 256, 5, 300, [1000, 1001, 3000]),        # expiry + reuse (LIFO)
    (4, 1024, 3, 2000, []),                      # one batch, heavy churn
])
def test_mixed_traces(seed, max_flows, expire_us, n_flows, cuts):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_fw_trace(rng, 5000, n_flows)
    fw, o = make_pair(max_flows=max_flows, expire_us=expire_us)
    check_batches(fw, o, fr, ln, dv, now, 64, cuts)
    check_state(fw, o, max_flows)


@pytest.mark.parametrize("slot", [128, 2048])
def test_generic_slots(slot):
    """Slots other than 64 B take the per-lane byte path; same results."""
    rng = np.random.default_rng(slot)
    fr, ln, dv, now = mixed_fw_trace(rng, 3000, 80, slot=slot)
    fw, o = make_pair(max_flows=64, expire_us=2)
    check_batches(fw, o, fr, ln, dv, now, slot, [900])
    check_state(fw, o, 64)


def test_replies_in_same_batch_as_opening_packet():
    """A WAN reply queued in phase A (its flow does not exist at segment
    start) is a hit only if the opening LAN packet precedes it."""
    n = 4
    lan, ll = T.udp_frames(np.full(n, T.ip4(10, 0, 0, 1)), np.full(n, T.ip4(9, 9, 9, 9)),
                           np.arange(n) + 100, np.full(n, 80))
    rep, rl = T.udp_frames(np.full(n, T.ip4(9, 9, 9, 9)), np.full(n, T.ip4(10, 0, 0, 1)),
                           np.full(n, 80), np.arange(n) + 100)
    lan, rep = lan.reshape(n, 64), rep.reshape(n, 64)
    # reply 0 before its LAN packet, reply 1..3 after; flow 2 opened from dev 2
    order = [("r", 0), ("l", 0), ("r", 0), ("l", 1), ("l", 2), ("r", 2),
             ("r", 1), ("r", 3), ("l", 3), ("r", 3)]
    fr = np.concatenate([(rep if k == "r" else lan)[i] for k, i in order])
    dv = np.array([1 if k == "r" else (2 if i == 2 else 0) for k, i in order],
                  np.uint16)
    ln = np.full(len(order), 60, np.uint16)
    now = T.NOW0 + np.arange(len(order), dtype=np.int64)
    fw, o = make_pair(max_flows=16)
    check_batches(fw, o, fr, ln, dv, now, 64, [])
    check_state(fw, o, 16)


def test_time_ties_and_long_expiry():
    """vigfw multiplies expiration_time in 64 bits: 4295 s does not wrap."""
    rng = np.random.default_rng(7)
    fr, ln, dv, _ = mixed_fw_trace(rng, 6000, 300)
    now = T.NOW0 + (np.arange(6000) // 7).astype(np.int64) * 1_000_000
    fw, o = make_pair(max_flows=512, expire_us=4_295_000)
    check_batches(fw, o, fr, ln, dv, now, 64, [1234, 3000])
    check_state(fw, o, 512)


def test_host_batch_entry_points():
    rng = np.random.default_rng(5)
    fr, ln, dv, now = mixed_fw_trace(rng, 3000, 50)
    fw, o = make_pair(max_flows=64)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    got = fr.copy()
    out = fw.process_host(got[:1500 * 64], ln[:1500], dv[:1500], now[:1500], 64)
    bufs = [bytearray(got[i * 64:i * 64 + int(ln[i])].tobytes())
            for i in range(1500, 3000)]
    out2 = fw.process_mbufs(bufs, dv[1500:], now[1500:])
    np.testing.assert_array_equal(np.concatenate([out, out2]), exp_out)
    np.testing.assert_array_equal(got[:1500 * 64], exp[:1500 * 64])
    for i, b in enumerate(bufs):
        k = 1500 + i
        assert bytes(b) == exp[k * 64:k * 64 + int(ln[k])].tobytes()


def test_1m_flows_with_replies():
    """1M flows (cap 2^20): a warm-up batch opening every flow, then
    steady-state batches with every 4th packet a WAN reply."""
    nf = 1 << 20
    fw, o = make_pair(max_flows=nf)
    B = 1 << 21
    for j in range(3):
        fr, ln, dv, now = T.fw_trace(B, nf, start=j * B,
                                     reply_every=4 if j else 0)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        got, out = run_gpu(fw, fr, ln, dv, now, 64, affine=(int(now[0]), 1))
        assert np.array_equal(out, exp_out)
        assert orc.digest(got, 64, ln, out) == orc.digest(exp, 64, ln, exp_out)
    assert fw.live_count() == nf


def test_rejects_bad_config():
    args = ["--wan", "1", "--max-flows", "1000", "--expire", "10"]
    cfg = vigor_amd.fw_config_from_args(args, 2, DEV_MACS[:2])
    with pytest.raises(vigor_amd.VigpathError):
        vigor_amd.Fw(cfg)  # map_allocate rejects a non power of two


@pytest.mark.parametrize("n_flows", [3, 5000])
def test_touch_bins_steady_state(n_flows):
    """vigfw steady state (LAN hits + WAN replies) through the touch bins
    (and their overflow fallback for a hot flow set): state equals the
    oracle's."""
    fw, o = make_pair(max_flows=1 << 16)
    fr, ln, dv, now = T.fw_trace(n_flows, n_flows)
    check_batches(fw, o, fr, ln, dv, now, 64, [])
    fr, ln, dv, now = T.fw_trace(30_000, n_flows, start=n_flows, reply_every=3)
    check_batches(fw, o, fr, ln, dv, now, 64, [])
    check_state(fw, o, 1 << 16)


def test_multiplicative_home_buckets_reprobe(monkeypatch):
    """VIGPATH_MIX=1 at load 0.65: full home buckets finish in fw_reprobe
    (LAN hits, WAN replies and new flows alike)."""
    monkeypatch.setenv("VIGPATH_MIX", "1")
    monkeypatch.setenv("VIGPATH_SPARSE", "-1")  # load 2/3: many reprobes
    monkeypatch.setenv("VIGPATH_LIN", "0")  # (no allocation-order layout)
    fw, o = make_pair(max_flows=4096)
    fr, ln, dv, now = T.fw_trace(4000, 4000)
    check_batches(fw, o, fr, ln, dv, now, 64, [1500])
    fr, ln, dv, now = T.fw_trace(50_000, 4000, start=4000, reply_every=3)
    check_batches(fw, o, fr, ln, dv, now, 64, [20_000])
    check_state(fw, o, 4096)
    rng = np.random.default_rng(3)
    fr, ln, dv, now = mixed_fw_trace(rng, 5000, 3500)
    check_batches(fw, o, fr, ln, dv, now + 10**8, 64, [2500])
    check_state(fw, o, 4096)
