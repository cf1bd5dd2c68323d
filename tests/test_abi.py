"""CPU-side checks of the drop-in boundary: the C-ABI library loads and
exports every symbol include/vigpath.h declares; host config parsing follows
the reference's option semantics. No compute calls (no GPU here)."""
import os
import re
import subprocess

import pytest

import vigor_amd
from vigor_amd import config as cfgmod

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^[\w\s\*]*?\b(vp_\w+|nf_\w+)\s*\(", txt,
                                 re.M)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], check=True,
                         capture_output=True, text=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_library_exports_every_declared_symbol():
    syms = exported(vigor_amd.LIB_PATH)
    want = [s for s in declared("vigpath.h") if s.startswith("vp_")]
    assert want, "no declarations parsed"
    missing = [s for s in want if s not in syms]
    assert not missing, missing
    assert set(vigor_amd.EXPORTS) <= set(want)
    vigor_amd.lib()  # loads (resolves every ctypes binding)


def test_nat_config_parse_semantics():
    c = cfgmod.nat_config_from_args(
        ["--wan", "1", "--expire", "10", "--extip", "192.168.4.2",
         "--max-flows", "65536", "--starting-port", "7",
         "--eth-dest", "1,01:23:45:67:89:01"], 2, [b"\x02" * 6, b"\x12" * 6])
    assert c.external_addr == 0xC0A80402  # host order (nf-parse.h:25-28)
    assert (c.wan_device, c.start_port, c.max_flows) == (1, 7, 65536)
    assert bytes(c.endpoint_macs[1]) == bytes.fromhex("012345678901")
    with pytest.raises(ValueError):
        cfgmod.nat_config_from_args(["--expire", "0"], 2, [])
    with pytest.raises(ValueError):
        cfgmod.nat_config_from_args(["--wan", "5"], 2, [])
    with pytest.raises(ValueError):
        cfgmod.nat_config_from_args(["--max-flows", "12x"], 2, [])
