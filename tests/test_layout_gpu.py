"""The allocation-order home-bucket layout of the vignat table
(vp_table.hip tbl_try_linear): fitted when the live keys are a
GF(2)-linear sequence in index order (the bench's sequential flows), dropped
when later keys cluster in it. The layout is free (outputs depend only on the
key -> index map), so every case checks out ports, frames and the dumped
state against the oracle; the debug log says which layout ran."""
import numpy as np
import pytest

from test_nat_gpu import check_state, make_pair
from gpuh import run_gpu
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu


def _run(nat, o, fr, ln, dv, now):
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    got, out = run_gpu(nat, fr, ln, dv, now, 64)
    assert np.array_equal(out, exp_out)
    assert np.array_equal(got, exp)


def _random_flows(n, seed, start):
    r = np.random.default_rng(seed)
    src_ip = r.integers(0, 1 << 32, n, dtype=np.int64)
    src_port = r.integers(0, 1 << 16, n, dtype=np.int64)
    dst_ip = r.integers(0, 1 << 32, n, dtype=np.int64)
    fr, ln = T.udp_frames(src_ip, dst_ip, src_port, np.zeros(n, np.int64))
    dv = np.zeros(n, dtype=np.uint16)
    now = T.NOW0 + np.arange(start, start + n, dtype=np.int64)
    return fr, ln, dv, now


@pytest.mark.parametrize("lin", ["1", "2"])
def test_sequential_flows_take_the_linear_layout(lin, monkeypatch, capfd):
    monkeypatch.setenv("VIGPATH_DEBUG", "1")
    monkeypatch.setenv("VIGPATH_LIN", lin)
    cap = 1 << 16
    nat, o = make_pair(max_flows=cap)
    B = 3 * cap // 2
    for j in range(3):  # warm-up (every flow new) then steady state
        _run(nat, o, *T.nat_lan_trace(B, cap, start=j * B))
    assert "linear layout:" in capfd.readouterr().err
    assert nat.live_count() == cap
    check_state(nat, o, cap)


def test_random_keys_drop_the_linear_layout(monkeypatch, capfd):
    """Sequential flows fill 5/8 of the table (layout fitted), then keys
    with no structure arrive: they cluster at load 2/3 and the table goes
    back to the CRC bits at full size, exact throughout."""
    monkeypatch.setenv("VIGPATH_DEBUG", "1")
    cap = 1 << 16
    nat, o = make_pair(max_flows=cap)
    n_seq = 5 * cap // 8
    _run(nat, o, *T.nat_lan_trace(n_seq, n_seq))
    assert "linear layout:" in capfd.readouterr().err
    _run(nat, o, *_random_flows(3 * cap // 8, 7, n_seq))
    _run(nat, o, *T.nat_lan_trace(n_seq, n_seq, start=n_seq + 3 * cap // 8))
    assert "linear layout dropped" in capfd.readouterr().err
    check_state(nat, o, cap)


def test_linear_layout_under_expiry_and_reuse():
    """Sequential flows with a short expiry: indices freed in LRU order and
    reused LIFO by new flows, so the index order stops matching the key
    order; lookups stay exact whatever layout the table keeps."""
    cap = 1 << 14
    nat, o = make_pair(max_flows=cap, expire_us=20_000)
    n = 3 * cap
    fr, ln, dv, now = T.nat_lan_trace(n, 2 * cap)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    outs, frames = [], []
    for a in range(0, n, cap):
        got, out = run_gpu(nat, fr[a * 64:(a + cap) * 64], ln[a:a + cap],
                           dv[a:a + cap], now[a:a + cap], 64)
        outs.append(out)
        frames.append(got)
    assert np.array_equal(np.concatenate(outs), exp_out)
    assert np.array_equal(np.concatenate(frames).reshape(-1), exp.reshape(-1))
    check_state(nat, o, cap)
