"""The nf.h drop-in end to end: host/nf_loop (nf.c's loop restated in C over
a trace file) linked against libvignat_nf.so, per packet (nf_process) and
batched (vp_process_batch), checked bit-exact against the oracle."""
import os
import subprocess

import numpy as np
import pytest

import orc
from tracegen import mixed_fw_trace, mixed_nat_trace, mixed_pol_trace
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


def read_out(path, n, slot):
    b = open(path, "rb").read()
    assert b[:4] == b"VPTO"
    out = np.frombuffer(b, np.uint16, n, 12)
    frames = np.frombuffer(b, np.uint8, n * slot, 12 + 2 * n)
    return out, frames


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
