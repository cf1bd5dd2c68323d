"""vigbridge on the GPU vs the oracle (bit-exact out ports, untouched frames,
dynamic table state: allocation, timestamps, MACs, learned ports).

Every test calls the product through the C-ABI (libvigpath.so via
vigor_amd); the oracle (oracle/liborc.so) is only the checker.
"""
import numpy as np
import pytest

import orc
import vigor_amd
from gpuh import check_batches, run_gpu
from tracegen import mixed_bridge_trace
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu

STATICS = [
    (bytes([2, 0, 0, 0, 0, 7]), 0, 2),     # forward
    (bytes([2, 0, 0, 0, 0, 9]), 1, -2),    # filter (drop)
    (bytes([2, 0, 0, 0, 0, 9]), 1, 0),     # duplicate key: first rule wins
    (bytes([2, 0, 0, 0, 0, 11]), 2, -1),   # explicit flood
    (bytes([0xFF] * 6), 0, 1),             # broadcast from port 0
]


def make_pair(cap=1024, expire_us=300_000_000, statics=(), n_dev=3):
    args = ["--expire", str(expire_us), "--capacity", str(cap)]
    cfg = vigor_amd.bridge_config_from_args(args, n_dev, list(statics))
    gpu = vigor_amd.Bridge(cfg, gpu=0)
    ocfg = orc.BridgeCfg(expiration_time=expire_us, dyn_capacity=cap,
                         n_devices=n_dev)
    return gpu, orc.Oracle("bridge", ocfg, statics=list(statics))


def check_state(br, oracle, cap):
    ga, gts, gm, gp = br.dump()
    oa, ots, om, op = oracle.bridge_dump(cap)
    np.testing.assert_array_equal(ga, oa)
    live = oa == 1
    np.testing.assert_array_equal(gts[live], ots[live])
    np.testing.assert_array_equal(gm[live], om[live])
    np.testing.assert_array_equal(gp[live], op[live])


def test_config3_learn_then_forward():
    br, o = make_pair(cap=4096)
    fr, ln, dv, now = T.bridge_trace(40_000, 3000)
    check_batches(br, o, fr, ln, dv, now, 64, [100, 3000, 7000], affine=True)
    check_state(br, o, 4096)
    assert br.live_count() == 3000


def test_config3_flood_pattern():
    br, o = make_pair(cap=4096)
    fr, ln, dv, now = T.bridge_trace(20_000, 2000, flood_pattern=True)
    check_batches(br, o, fr, ln, dv, now, 64, [5000])
    check_state(br, o, 4096)


@pytest.mark.parametrize("seed,cap,expire_us,n_st,statics,cuts", [
    (0, 1024, 300_000_000, 200, False, [100, 2000]),   # learn + MAC moves
    (1, 64, 300_000_000, 300, False, [2500]),          # table full
    (2, 256, 3, 300, False, [1, 2, 3, 500, 4000]),     # expiry every few pkts
    (3, 128, 10, 150, True, [1000, 1001]),             # statics + expiry
    (4, 2048, 1, 3000, True, []),                      # one batch, churn
])
def test_mixed_traces(seed, cap, expire_us, n_st, statics, cuts):
    rng = np.random.default_rng(seed)
    fr, ln, dv, now = mixed_bridge_trace(rng, 5000, n_st)
    if statics:  # make the static MACs appear as destinations
        f = fr.reshape(-1, 64)
        k = rng.random(5000) < 0.2
        pick = rng.integers(0, len(STATICS), 5000)
        for i in np.nonzero(k)[0]:
            f[i, 0:6] = list(STATICS[pick[i]][0])
    br, o = make_pair(cap=cap, expire_us=expire_us,
                      statics=STATICS if statics else ())
    check_batches(br, o, fr, ln, dv, now, 64, cuts)
    check_state(br, o, cap)


def test_time_ties_and_wrapping_expiry():
    rng = np.random.default_rng(9)
    fr, ln, dv, _ = mixed_bridge_trace(rng, 6000, 400)
    now = T.NOW0 + (np.arange(6000) // 5).astype(np.int64) * 1_000_000
    br, o = make_pair(cap=512, expire_us=4_295_000)  # u32 wrap: ~0.7 s
    check_batches(br, o, fr, ln, dv, now, 64, [999, 3000])
    check_state(br, o, 512)


def test_host_batch_and_per_packet():
    rng = np.random.default_rng(4)
    fr, ln, dv, now = mixed_bridge_trace(rng, 2000, 50)
    ln = np.maximum(ln, 14).astype(np.uint16)
    br, o = make_pair(cap=64)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    out = br.process_host(fr[:1000 * 64].copy(), ln[:1000], dv[:1000],
                          now[:1000], 64)
    np.testing.assert_array_equal(out, exp_out[:1000])
    for i in range(1000, 1100):
        b = bytearray(fr[i * 64:i * 64 + int(ln[i])].tobytes())
        assert br.process(int(dv[i]), b, int(now[i])) == exp_out[i]


def test_config3_1m_macs_full_size():
    """BASELINE config 3 at full size (1M MACs, capacity 2^20)."""
    n = 1 << 20
    br, o = make_pair(cap=n, expire_us=60_000_000, n_dev=2)
    B = 1 << 21
    for j in range(2):
        fr, ln, dv, now = T.bridge_trace(B, n, start=j * B)
        exp = fr.copy()
        exp_out = o.run(exp, ln, dv, now, 64)
        got, out = run_gpu(br, fr, ln, dv, now, 64, affine=(int(now[0]), 1))
        assert np.array_equal(out, exp_out)
        assert np.array_equal(got, exp)
    assert br.live_count() == n


def test_rejects_bad_config():
    with pytest.raises(vigor_amd.VigpathError):
        make_pair(cap=1000)
    with pytest.raises(vigor_amd.VigpathError):
        make_pair(statics=[(bytes(6), 0, 1)] * 4096)
