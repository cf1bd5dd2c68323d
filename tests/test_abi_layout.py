"""The ctypes mirrors in vigor_amd/__init__.py have the C layout of the
structs include/vigpath.h declares: sizes and every field's offset, compiled
here with gcc against the header (CPU only). A field added on one side only
(round 5's vp_dev_batch.in_port) would shift what the library reads."""
import ctypes as C
import os
import subprocess

import pytest

import vigor_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# C struct name -> its ctypes mirror
PAIRS = {
    "vp_nat_config": vigor_amd.NatConfigC,
    "vp_bridge_rule": vigor_amd.BridgeRuleC,
    "vp_bridge_config": vigor_amd.BridgeConfigC,
    "vp_lb_config": vigor_amd.LbConfigC,
    "vp_fw_config": vigor_amd.FwConfigC,
    "vp_pol_config": vigor_amd.PolConfigC,
    "vp_comm_ops": vigor_amd.CommOpsC,
    "vp_dev_batch": vigor_amd.DevBatchC,
    "vp_mbuf_batch": vigor_amd.MbufBatchC,
    "vp_table_stats": vigor_amd.TableStatsC,
}


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("abi")
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "vigpath.h"',
             "int main(void) {"]
    for cname, py in PAIRS.items():
        lines.append('  printf("%s size %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in py._fields_:
            lines.append('  printf("%s %s %%zu\\n", offsetof(%s, %s));'
                         % (cname, fname, cname, fname))
    lines += ["  return 0;", "}"]
    src = d / "abi.c"
    src.write_text("\n".join(lines) + "\n")
    exe = d / "abi"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    got = {}
    for line in out.splitlines():
        a, b, v = line.split()
        got[(a, b)] = int(v)
    return got


@pytest.mark.parametrize("cname", sorted(PAIRS))
def test_ctypes_mirror_matches_header(c_layout, cname):
    py = PAIRS[cname]
    assert C.sizeof(py) == c_layout[(cname, "size")], cname
    for fname, _ in py._fields_:
        assert getattr(py, fname).offset == c_layout[(cname, fname)], (cname, fname)
