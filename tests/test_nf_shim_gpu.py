"""The nf.h drop-in end to end: host/nf_loop (nf.c's loop restated in C over
a trace file) linked against libvignat_nf.so, per packet (nf_process) and
batched (vp_process_batch), checked bit-exact against the oracle."""
import os
import subprocess

import numpy as np
import pytest

import orc
from tracegen import (mixed_bridge_trace, mixed_fw_trace, mixed_lb_trace,
                      mixed_nat_trace, mixed_pol_trace)
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOOP = os.path.join(ROOT, "host", "nf_loop")
DEV = [bytes.fromhex("020000000000"), bytes.fromhex("020000000001")]
END = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01")]
ARGS = ["--wan", "1", "--expire", "7", "--starting-port", "0",
        "--max-flows", "256", "--extip", "192.168.4.2",
        "--eth-dest", "0,01:23:45:67:89:00", "--eth-dest", "1,01:23:45:67:89:01"]


def write_trace(path, frames, lens, in_dev, now, slot):
    with open(path, "wb") as f:
        f.write(b"VPTR")
        f.write(np.array([lens.shape[0], slot], np.uint32).tobytes())
        f.write(in_dev.astype(np.uint16).tobytes())
        f.write(lens.astype(np.uint16).tobytes())
        f.write(now.astype(np.int64).tobytes())
        f.write(frames.tobytes())


def read_out(path, n, slot, tx=False):
    b = open(path, "rb").read()
    assert b[:4] == b"VPTO"
    out = np.frombuffer(b, np.uint16, n, 12)
    frames = np.frombuffer(b, np.uint8, n * slot, 12 + 2 * n)
    if not tx:
        return out, frames
    o = 12 + 2 * n + n * slot
    assert b[o:o + 4] == b"VPTX"
    return out, frames, np.frombuffer(b, np.uint32, n, o + 4)


def expected_tx(out, in_dev, nb_devices):
    """nf.c:158-175 + flood() nf.c:83-96: the ports a packet leaves on."""
    all_ports = (1 << nb_devices) - 1
    m = np.where(out == 0xFFFF, all_ports & ~(1 << in_dev.astype(np.int64)),
                 1 << np.minimum(out, 31).astype(np.int64))
    return np.where(out == in_dev, 0, m).astype(np.uint32)


def run_loop(tmp_path, loop, fr, ln, dv, now, slot, batch, args, nb_devices):
    tin, tout = tmp_path / "t.in", tmp_path / "t.out"
    write_trace(tin, fr, ln, dv, now, slot)
    cmd = [LOOP + loop, str(tin), str(tout)]
    if batch:
        cmd += ["--batch", str(batch)]
    env = dict(os.environ, VIGPATH_NB_DEVICES=str(nb_devices))
    r = subprocess.run(cmd + ["--"] + args, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    return read_out(tout, ln.shape[0], slot, tx=True)


@pytest.mark.parametrize("batch", [0, 700])
def test_nf_loop_matches_oracle(tmp_path, batch):
    rng = np.random.default_rng(3)
    n = 3000 if batch else 400
    fr, ln, dv, now = mixed_nat_trace(rng, n, 150, max_idx=256)
    cfg = orc.nat_cfg(wan=1, ext_ip=T.ip4(192, 168, 4, 2), expire_us=7,
                      max_flows=256, device_macs=DEV, endpoint_macs=END)
    exp = fr.copy()
    exp_out = orc.Oracle("nat", cfg).run(exp, ln, dv, now, 64)
    tin, tout = tmp_path / "t.in", tmp_path / "t.out"
    write_trace(tin, fr, ln, dv, now, 64)
    cmd = [LOOP, str(tin), str(tout)]
    if batch:
        cmd += ["--batch", str(batch)]
    env = dict(os.environ, VIGPATH_NB_DEVICES="2")
    r = subprocess.run(cmd + ["--"] + ARGS, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    out, frames = read_out(tout, n, 64)
    np.testing.assert_array_equal(out, exp_out)
    # frames compared over each packet's valid bytes (the batched entry point
    # stages len bytes per mbuf)
    f, e = frames.reshape(n, 64), exp.reshape(n, 64)
    for i in range(n):
        assert f[i, :ln[i]].tobytes() == e[i, :ln[i]].tobytes(), i


@pytest.mark.parametrize("batch", [0, 700])
def test_fw_loop_matches_oracle(tmp_path, batch):
    """host/nf_loop_fw: nf.c's loop linked against libvigfw_nf.so."""
    rng = np.random.default_rng(4)
    n = 3000 if batch else 400
    fr, ln, dv, now = mixed_fw_trace(rng, n, 150)
    dev3 = DEV + [bytes.fromhex("020000000002")]
    end3 = END + [T.mac("01:23:45:67:89:02")]
    cfg = orc.fw_cfg(wan=1, expire_us=7, max_flows=256, device_macs=dev3,
                     endpoint_macs=end3, n_devices=3)
    exp = fr.copy()
    exp_out = orc.Oracle("fw", cfg).run(exp, ln, dv, now, 64)
    tin, tout = tmp_path / "t.in", tmp_path / "t.out"
    write_trace(tin, fr, ln, dv, now, 64)
    cmd = [LOOP + "_fw", str(tin), str(tout)]
    if batch:
        cmd += ["--batch", str(batch)]
    args = ["--wan", "1", "--expire", "7", "--max-flows", "256",
            "--eth-dest", "0,01:23:45:67:89:00", "--eth-dest",
            "1,01:23:45:67:89:01", "--eth-dest", "2,01:23:45:67:89:02"]
    env = dict(os.environ, VIGPATH_NB_DEVICES="3")
    r = subprocess.run(cmd + ["--"] + args, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    out, frames = read_out(tout, n, 64)
    np.testing.assert_array_equal(out, exp_out)
    f, e = frames.reshape(n, 64), exp.reshape(n, 64)
    for i in range(n):
        assert f[i, :ln[i]].tobytes() == e[i, :ln[i]].tobytes(), i


@pytest.mark.parametrize("batch", [0, 700])
def test_pol_loop_matches_oracle(tmp_path, batch):
    """host/nf_loop_pol: nf.c's loop linked against libvigpol_nf.so (frames
    up to 1.4 kB in 1536-byte buffers, so every mbuf holds its length)."""
    rng = np.random.default_rng(5)
    n = 3000 if batch else 400
    slot = 1536
    fr, ln, dv, now = mixed_pol_trace(rng, n, 100, slot=slot, gap_ns=1500)
    cfg = orc.pol_cfg(lan=1, wan=0, rate=1_000_000, burst=1500, capacity=64,
                      n_devices=3)
    exp = fr.copy()
    exp_out = orc.Oracle("pol", cfg).run(exp, ln, dv, now, slot)
    tin, tout = tmp_path / "t.in", tmp_path / "t.out"
    write_trace(tin, fr, ln, dv, now, slot)
    cmd = [LOOP + "_pol", str(tin), str(tout)]
    if batch:
        cmd += ["--batch", str(batch)]
    args = ["--lan", "1", "--wan", "0", "--rate", "1000000", "--burst", "1500",
            "--capacity", "64"]
    env = dict(os.environ, VIGPATH_NB_DEVICES="3")
    r = subprocess.run(cmd + ["--"] + args, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    out, frames = read_out(tout, n, slot)
    np.testing.assert_array_equal(out, exp_out)
    assert (out == 1).sum() > 50 and (out == 0).sum() > 50
    np.testing.assert_array_equal(frames, fr)  # the policer never writes


SHIM_MACS3 = [bytes.fromhex("02000000000%d" % d) for d in range(3)]  # vp_nf_common.h


@pytest.mark.parametrize("batch", [0, 700])
def test_bridge_loop_floods_like_nf_c(tmp_path, batch):
    """host/nf_loop_bridge: nf.c's loop linked against libvigbridge_nf.so.
    vigbridge returns FLOOD_FRAME for unknown and broadcast destinations and
    the per-packet path's flood() sends the frame on every port but the input
    one (flood(mbuf, VIGOR_DEVICES_COUNT), nf.c:83-96, 159-166). With three
    ports the dispatch is the per-packet path's in both runs: nf.c's batched
    loop refuses any port count but two (nf.c:179-182), so batch=700 batches
    only the processing (vp_process_batch). Out ports, frames (never
    rewritten) and the transmit sets equal the oracle's."""
    rng = np.random.default_rng(6)
    n = 3000 if batch else 400
    fr, ln, dv, now = mixed_bridge_trace(rng, n, 120, n_dev=3)
    # runts (len < 14: vigbridge borrows the Ethernet header without a length
    # check) read past their length; the batch entry point stages len bytes
    # per mbuf, so bytes past a frame's length read as 0 (DESIGN.md §7,
    # out-of-domain conventions): the trace zeroes them for the oracle too
    f2 = fr.reshape(n, 64)
    for i in np.nonzero(ln < 64)[0]:
        f2[i, ln[i]:] = 0
    cfg = orc.BridgeCfg(expiration_time=9, dyn_capacity=128, n_devices=3)
    exp = fr.copy()
    exp_out = orc.Oracle("bridge", cfg).run(exp, ln, dv, now, 64)
    args = ["--expire", "9", "--capacity", "128"]
    out, frames, txm = run_loop(tmp_path, "_bridge", fr, ln, dv, now, 64, batch, args, 3)
    np.testing.assert_array_equal(out, exp_out)
    assert (out == 0xFFFF).sum() > 20 and ((out != 0xFFFF) & (out != dv)).sum() > 20
    np.testing.assert_array_equal(txm, expected_tx(exp_out, dv, 3))
    f, e = frames.reshape(n, 64), exp.reshape(n, 64)
    for i in range(n):
        assert f[i, :ln[i]].tobytes() == e[i, :ln[i]].tobytes(), i


@pytest.mark.parametrize("batch", [0, 700])
def test_lb_loop_matches_oracle(tmp_path, batch):
    """host/nf_loop_lb: nf.c's loop linked against libviglb_nf.so
    (heartbeats from backends on ports 0/1, WAN traffic on port 2)."""
    rng = np.random.default_rng(7)
    n = 3000 if batch else 400
    fr, ln, dv, now = mixed_lb_trace(rng, n, 150, 12)
    cfg = orc.LbCfg(flow_capacity=256, flow_expiration_time=60_000_000,
                    backend_capacity=16, cht_height=17,
                    backend_expiration_time=3_600_000, wan_device=2, n_devices=3)
    for d in range(3):
        cfg.device_macs[d][:] = list(SHIM_MACS3[d])
    exp = fr.copy()
    exp_out = orc.Oracle("lb", cfg).run(exp, ln, dv, now, 64)
    args = ["--flow-capacity", "256", "--backend-capacity", "16", "--cht-height", "17",
            "--flow-expiration", "60000000", "--backend-expiration", "3600000",
            "--wan", "2"]
    out, frames, txm = run_loop(tmp_path, "_lb", fr, ln, dv, now, 64, batch, args, 3)
    np.testing.assert_array_equal(out, exp_out)
    assert ((out != dv)).sum() > 100
    np.testing.assert_array_equal(txm, expected_tx(exp_out, dv, 3))
    f, e = frames.reshape(n, 64), exp.reshape(n, 64)
    for i in range(n):
        assert f[i, :ln[i]].tobytes() == e[i, :ln[i]].tobytes(), i
