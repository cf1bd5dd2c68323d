"""The GPU path (C-ABI, two batches) against the fixtures derived from the
reference's own NF specifications (tests/test_spec.py)."""
import numpy as np
import pytest

import spec_cases as C
import vigor_amd
from gpuh import run_gpu
from test_spec import check, load

pytestmark = pytest.mark.gpu


def make(nf):
    if nf == "nat":
        return vigor_amd.Nat(vigor_amd.nat_config_from_args(C.nat_gpu_args(), 2,
                                                            C.DEV3[:2]), gpu=0)
    if nf == "fw":
        return vigor_amd.Fw(vigor_amd.fw_config_from_args(C.fw_gpu_args(), 3, C.DEV3),
                            gpu=0)
    if nf == "lb":
        return vigor_amd.Lb(vigor_amd.lb_config_from_args(C.lb_gpu_args(), 3, C.LB_MACS),
                            gpu=0)
    if nf == "pol":
        return vigor_amd.Pol(vigor_amd.pol_config_from_args(C.pol_gpu_args(), 3), gpu=0)
    return vigor_amd.Bridge(vigor_amd.bridge_config_from_args(C.bridge_gpu_args(), 2,
                                                              []), gpu=0)


@pytest.mark.parametrize("nf", ["nat", "fw", "bridge", "pol", "lb"])
def test_gpu_matches_reference_spec(nf):
    g = load(nf)
    dev = make(nf)
    n = g["lens"].shape[0]
    outs, frames = [], []
    for a, b in ((0, 1100), (1100, n)):
        f, o = run_gpu(dev, g["frames"][a * 64:b * 64], g["lens"][a:b],
                       g["in_dev"][a:b], g["now"][a:b], 64)
        frames.append(f)
        outs.append(o)
    check(nf, np.concatenate(outs), np.concatenate(frames), g)
