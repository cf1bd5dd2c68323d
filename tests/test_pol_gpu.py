"""vigpol on the GPU vs the oracle (bit-exact out ports, untouched frames,
dchain state and every token bucket).

Every test calls the product through the C-ABI (libvigpath.so via
vigor_amd); the oracle (oracle/liborc.so) is only the checker. Reference
behaviour: vigpol/policer_main.c:21-145, policer_config.c:17-93.
"""
import numpy as np
import pytest
import orc
import vigor_amd
from gpuh import check_batches, run_gpu
from tracegen import mixed_pol_trace
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu


def make_pair(cap=64, rate=1_000_000, burst=1000, lan=1, wan=0, n_dev=3):
    args = ["--lan", str(lan), "--wan", str(wan), "--rate", str(rate),
            "--burst", str(burst), "--capacity", str(cap)]
    gpu = vigor_amd.Pol(vigor_amd.pol_config_from_args(args, n_dev), gpu=0)
    o = orc.Oracle("pol", orc.pol_cfg(lan=lan, wan=wan, rate=rate, burst=burst,
                                      capacity=cap, n_devices=n_dev))
    return gpu, o


def check_state(pol, oracle, cap):
    ga, gts, gk, gs, gt = pol.dump()
    oa, ots, ok, os_, ot = oracle.pol_dump(cap)
    np.testing.assert_array_equal(ga, oa)
    live = oa == 1
    for g, o in ((gts, ots), (gk, ok), (gs, os_), (gt, ot)):
        np.testing.assert_array_equal(g[live], o[live])


@pytest.mark.parametrize("seed,cap,n_dsts,burst,gap,cuts", [
    (0, 64, 40, 3000, 500, [100, 2000]),        # steady, refills
    (1, 16, 60, 1000, 2000, [1, 2, 3, 2500]),    # table full + expiry
    (2, 256, 300, 2000, 50, [3000]),             # many addresses, long runs
    (3, 64, 20, 1000, 10, []),                   # hot addresses, tiny gaps
    (4, 1024, 900, 1500, 3000, [1000, 1001]),    # churn: expiry + reuse
])
def test_mixed_traces(seed, cap, n_dsts, burst, gap, cuts):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_pol_trace(rng, 6000, n_dsts, gap_ns=gap)
    pol, o = make_pair(cap=cap, burst=burst)
    check_batches(pol, o, fr, ln, dv, now, 64, cuts)
    check_state(pol, o, cap)


def test_generic_slot_and_affine_time():
    rng = np.random.default_rng(7)
    fr, ln, dv, now = mixed_pol_trace(rng, 3000, 50, slot=128, gap_ns=1)
    now = T.NOW0 + np.arange(3000, dtype=np.int64) * 700
    pol, o = make_pair(cap=64, burst=1200)
    check_batches(pol, o, fr, ln, dv, now, 128, [1500], affine=True)
    check_state(pol, o, 64)


def test_trailing_non_ipv4_runs_no_expiry():
    """policer_main.c:124-132: a frame whose IPv4 header does not parse
    returns before the expiry, so entries stay until the next IPv4 packet."""
    pol, o = make_pair(cap=64, burst=1000)  # entries live 1 ms
    f, _ = T.udp_frames(np.array([T.ip4(9, 9, 9, 9)] * 3),
                        np.array([T.ip4(10, 0, 0, 1), T.ip4(10, 0, 0, 2),
                                  T.ip4(10, 0, 0, 3)]),
                        np.array([53] * 3), np.array([80] * 3))
    fr = f.reshape(3, 64).copy()
    fr[2, 12] = 0x86  # not IPv4, two seconds later
    ln = np.array([100, 100, 100], np.uint16)
    dv = np.zeros(3, np.uint16)
    now = np.array([T.NOW0, T.NOW0 + 1, T.NOW0 + 2_000_000_000], np.int64)
    check_batches(pol, o, fr.reshape(-1), ln, dv, now, 64, [])
    check_state(pol, o, 64)
    assert pol.dump()[0].sum() == 2 and vigor_amd.lib().vp_live_count(pol.h) == 2


def test_single_address_serial_bucket():
    """One address, many packets per batch: the replay is a long serial run
    (rate 1 B/us, sizes around the refill)."""
    n = 4000
    f, _ = T.udp_frames(np.full(n, T.ip4(9, 9, 9, 9)), np.full(n, T.ip4(10, 0, 0, 1)),
                        np.full(n, 53), np.full(n, 80))
    rng = np.random.default_rng(11)
    ln = rng.integers(40, 400, n).astype(np.uint16)
    dv = np.zeros(n, np.uint16)
    now = (T.NOW0 + np.cumsum(rng.integers(0, 300_000, n))).astype(np.int64)
    pol, o = make_pair(cap=16, burst=1000)
    check_batches(pol, o, f.copy(), ln, dv, now, 64, [2000])
    check_state(pol, o, 16)


def test_config_rejects_like_reference():
    with pytest.raises(ValueError):
        vigor_amd.pol_config_from_args(["--rate", "0"], 2)
    with pytest.raises(ValueError):
        vigor_amd.pol_config_from_args(["--lan", "2"], 2)
    cfg = vigor_amd.pol_config_from_args(["--capacity", "100"], 2)
    with pytest.raises(vigor_amd.VigpathError):
        vigor_amd.Pol(cfg, gpu=0)  # not a power of two (map.c:73)


def test_steady_state_grouping_path():
    """Segments without misses and with short runs take the grouping path
    (per-index hit counts from phase A, scan + scatter, per-lane insertion
    sort); uniformly random order puts each run's packets out of order in
    the scatter. A hot address (run > 64) in the last batch sends that
    segment to the radix-sort path instead. Both must equal the oracle."""
    rng = np.random.default_rng(21)
    n_dst, n = 5000, 60000
    d = np.concatenate([np.arange(n_dst), rng.integers(0, n_dst, n - n_dst)])
    d[-3000::7] = 17  # hot address in the last batch
    f, _ = T.udp_frames(np.full(n, T.ip4(9, 9, 9, 9)), T.ip4(10, 0, 0, 0) + d,
                        np.full(n, 53), np.full(n, 80))
    ln = rng.integers(60, 900, n).astype(np.uint16)
    dv = np.zeros(n, np.uint16)
    now = (T.NOW0 + np.cumsum(rng.integers(0, 40, n))).astype(np.int64)
    pol, o = make_pair(cap=8192, rate=2_000_000, burst=2000)
    check_batches(pol, o, f.copy(), ln, dv, now, 64, [n_dst, 25000, 45000])
    check_state(pol, o, 8192)
