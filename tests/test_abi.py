"""CPU-side checks of the drop-in boundary: the C-ABI library and the nf.h
shims load and export every symbol include/vigpath.h (and the reference's
nf.h, nf.h:8-18) declares; config parsing follows the reference's option
semantics. No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import vigor_amd
from vigor_amd import config as cfgmod

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIMS = {nf: os.path.join(ROOT, "vigor_amd", "libvig%s_nf.so" % nf)
         for nf in ("nat", "bridge", "lb", "fw", "pol")}
NF_H = ["nf_init", "nf_process", "nf_config_init", "nf_config_usage",
        "nf_config_print", "config"]


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^[\w\s\*]*?\b(vp_\w+)\s*\(", txt, re.M)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], check=True,
                         capture_output=True, text=True).stdout
    return {l.split()[-1] for l in out.splitlines()
            if len(l.split()) == 3 and l.split()[1] in "TBD"}


def test_library_exports_every_declared_symbol():
    syms = exported(vigor_amd.LIB_PATH)
    want = [s for s in declared("vigpath.h") if s != "vp_nf_context"]
    assert want, "no declarations parsed"
    missing = [s for s in want if s not in syms]
    assert not missing, missing
    assert set(vigor_amd.EXPORTS) <= set(want)
    vigor_amd.lib()  # loads (resolves every ctypes binding)


def test_bench_step_loop_library():
    # bench.py's timed loop in C (host/steps.c): loads against libvigpath.so
    path = os.path.join(ROOT, "vigor_amd", "libvp_steps.so")
    assert "vp_steps_device" in exported(path)
    C.CDLL(path).vp_steps_device


@pytest.mark.parametrize("nf", sorted(SHIMS))
def test_shim_exports_nf_h_surface(nf):
    syms = exported(SHIMS[nf])
    missing = [s for s in NF_H + ["vp_nf_context"] if s not in syms]
    assert not missing, missing


class RteEther(C.Structure):
    _fields_ = [("b", C.c_uint8 * 6)]


class NatNfConfig(C.Structure):
    """vignat/nat_config.h:5-31 as the shim defines it."""
    _fields_ = [("lan_main_device", C.c_uint16), ("wan_device", C.c_uint16),
                ("external_addr", C.c_uint32),
                ("device_macs", C.POINTER(RteEther)),
                ("endpoint_macs", C.POINTER(RteEther)),
                ("start_port", C.c_uint16), ("expiration_time", C.c_uint32),
                ("max_flows", C.c_uint32)]


def test_shim_nf_config_init_parses_like_reference():
    os.environ["VIGPATH_NB_DEVICES"] = "2"
    L = C.CDLL(SHIMS["nat"])
    args = [b"nf", b"--wan", b"1", b"--expire", b"10", b"--starting-port",
            b"5", b"--max-flows", b"65536", b"--extip", b"192.168.4.2",
            b"--eth-dest", b"1,01:23:45:67:89:01"]
    argv = (C.c_char_p * (len(args) + 1))(*args, None)
    L.nf_config_init(len(args), argv)
    cfg = NatNfConfig.in_dll(L, "config")
    assert (cfg.wan_device, cfg.start_port, cfg.max_flows) == (1, 5, 65536)
    assert cfg.expiration_time == 10
    assert cfg.external_addr == 0xC0A80402  # host order (nf-parse.h:25-28)
    assert bytes(cfg.endpoint_macs[1].b) == bytes.fromhex("012345678901")
    assert bytes(cfg.device_macs[1].b) == bytes.fromhex("020000000001")


def test_nat_config_parse_semantics():
    c = cfgmod.nat_config_from_args(
        ["--wan", "1", "--expire", "10", "--extip", "192.168.4.2",
         "--max-flows", "65536", "--starting-port", "7",
         "--eth-dest", "1,01:23:45:67:89:01"], 2, [b"\x02" * 6, b"\x12" * 6])
    assert c.external_addr == 0xC0A80402
    assert (c.wan_device, c.start_port, c.max_flows) == (1, 7, 65536)
    assert bytes(c.endpoint_macs[1]) == bytes.fromhex("012345678901")
    with pytest.raises(ValueError):
        cfgmod.nat_config_from_args(["--expire", "0"], 2, [])
    with pytest.raises(ValueError):
        cfgmod.nat_config_from_args(["--wan", "5"], 2, [])
    with pytest.raises(ValueError):
        cfgmod.nat_config_from_args(["--max-flows", "12x"], 2, [])


class FwNfConfig(C.Structure):
    """vigfw/fw_config.h:9-24 as the shim defines it."""
    _fields_ = [("wan_device", C.c_uint16),
                ("device_macs", C.POINTER(RteEther)),
                ("endpoint_macs", C.POINTER(RteEther)),
                ("expiration_time", C.c_uint32), ("max_flows", C.c_uint32)]


class LbNfConfig(C.Structure):
    """viglb/lb_config.h:8-38 as the shim defines it."""
    _fields_ = [("backend_count", C.c_uint16),
                ("device_macs", C.POINTER(RteEther)),
                ("flow_capacity", C.c_uint32),
                ("flow_expiration_time", C.c_uint32),
                ("backend_capacity", C.c_uint32), ("cht_height", C.c_uint32),
                ("backend_expiration_time", C.c_uint32),
                ("wan_device", C.c_uint16)]


class BridgeNfConfig(C.Structure):
    """vigbridge/bridge_config.h:8-18 as the shim defines it."""
    _fields_ = [("expiration_time", C.c_uint32), ("dyn_capacity", C.c_uint32),
                ("static_config_fname", C.c_char * 512)]


def _init(lib, args):
    args = [b"nf"] + [a.encode() for a in args]
    argv = (C.c_char_p * (len(args) + 1))(*args, None)
    lib.nf_config_init(len(args), argv)


def test_fw_shim_parses_like_reference():
    os.environ["VIGPATH_NB_DEVICES"] = "3"
    L = C.CDLL(SHIMS["fw"])
    _init(L, ["--wan", "2", "--expire", "99", "--max-flows", "1024",
              "--eth-dest", "1,01:23:45:67:89:01"])
    cfg = FwNfConfig.in_dll(L, "config")
    assert (cfg.wan_device, cfg.expiration_time, cfg.max_flows) == (2, 99, 1024)
    assert bytes(cfg.endpoint_macs[1].b) == bytes.fromhex("012345678901")
    assert bytes(cfg.device_macs[2].b) == bytes.fromhex("020000000002")


def test_lb_shim_parses_like_reference():
    os.environ["VIGPATH_NB_DEVICES"] = "3"
    L = C.CDLL(SHIMS["lb"])
    _init(L, ["--flow-capacity", "1024", "--backend-capacity", "32",
              "--cht-height", "97", "--flow-expiration", "10",
              "--backend-expiration", "20", "--wan", "2"])
    cfg = LbNfConfig.in_dll(L, "config")
    assert (cfg.flow_capacity, cfg.backend_capacity, cfg.cht_height) == \
        (1024, 32, 97)
    assert (cfg.flow_expiration_time, cfg.backend_expiration_time,
            cfg.wan_device) == (10, 20, 2)
    assert bytes(cfg.device_macs[1].b) == bytes.fromhex("020000000001")


def test_bridge_shim_parses_like_reference(tmp_path):
    L = C.CDLL(SHIMS["bridge"])
    _init(L, [])
    cfg = BridgeNfConfig.in_dll(L, "config")
    # DEFAULT_EXP_TIME / DEFAULT_CAPACITY (bridge_config.c:14-15)
    assert (cfg.expiration_time, cfg.dyn_capacity) == (300000000, 128)
    f = tmp_path / "static.cfg"
    f.write_text("02:00:00:00:00:07 0 1\n")
    _init(L, ["--expire", "5", "--capacity", "256", "--config", str(f)])
    assert (cfg.expiration_time, cfg.dyn_capacity) == (5, 256)
    assert cfg.static_config_fname == str(f).encode()


def test_fw_config_parse_semantics():
    c = cfgmod.fw_config_from_args(
        ["--wan", "1", "--expire", "10", "--max-flows", "65536",
         "--eth-dest", "0,01:23:45:67:89:00"], 2, [b"\x02" * 6, b"\x12" * 6])
    assert (c.wan_device, c.expiration_time, c.max_flows) == (1, 10, 65536)
    assert bytes(c.endpoint_macs[0]) == bytes.fromhex("012345678900")
    for bad in (["--expire", "0"], ["--wan", "2"], ["--max-flows", "1k"],
                ["--extip", "1.2.3.4"]):
        with pytest.raises(ValueError):
            cfgmod.fw_config_from_args(bad, 2, [])


class PolNfConfig(C.Structure):
    """vigpol/policer_config.h:9-24 as the shim defines it."""
    _fields_ = [("lan_device", C.c_uint16), ("wan_device", C.c_uint16),
                ("rate", C.c_uint64), ("burst", C.c_uint64),
                ("dyn_capacity", C.c_uint32)]


def test_pol_shim_parses_like_reference():
    """policer_config.c:20-93: defaults, then the options."""
    os.environ["VIGPATH_NB_DEVICES"] = "3"
    L = C.CDLL(SHIMS["pol"])
    _init(L, [])
    cfg = PolNfConfig.in_dll(L, "config")
    assert (cfg.lan_device, cfg.wan_device, cfg.rate, cfg.burst,
            cfg.dyn_capacity) == (1, 0, 1000000, 100000, 128)
    _init(L, ["--lan", "2", "--wan", "1", "--rate", "375000000", "--burst",
              "3750000000", "--capacity", "65536"])
    assert (cfg.lan_device, cfg.wan_device, cfg.rate, cfg.burst,
            cfg.dyn_capacity) == (2, 1, 375000000, 3750000000, 65536)


def test_pol_config_parse_semantics():
    c = vigor_amd.pol_config_from_args(["--wan", "1", "--lan=0"], 2)
    assert (c.lan_device, c.wan_device, c.rate, c.burst, c.dyn_capacity) == \
        (0, 1, 1000000, 100000, 128)
    for bad in (["--burst", "0"], ["--wan", "5"], ["--capacity", "0"],
                ["--rate", "12x"], ["--bogus", "1"]):
        with pytest.raises(ValueError):
            vigor_amd.pol_config_from_args(bad, 2)
