"""SURVEY.md §8(c) calibration of the CPU baseline: the clean-room oracle
restatement (oracle/liborc.so; and its -march=native hardware-crc32 build,
liborc_native.so, which bench.py times) against the oracle glue over the
reference's own libVig (oracle/_ref/liborc_ref.so, this container only) on
identical traces, one pinned core, median of several samples.

  python3 tools/calibrate_cpu.py [flows] [packets_per_sample] [samples]

Reports each implementation's median Mpps, the ratio of medians, and the
paired per-round ratio (median and a 90 % bootstrap interval).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import orc  # noqa: E402
import bench  # noqa: E402
from vigor_amd import traces as T  # noqa: E402


def make(ref, flows):
    cfg = orc.nat_cfg(wan=1, ext_ip=T.ip4(192, 168, 4, 2), expire_us=60_000_000,
                      max_flows=flows, device_macs=bench.DEV_MACS,
                      endpoint_macs=[T.mac("90:e2:ba:55:12:20"),
                                     T.mac("90:e2:ba:55:12:21")])
    o = orc.Oracle("nat", cfg, ref=ref)
    fr, ln, dv, now = T.nat_lan_trace(flows, flows)
    o.run(fr, ln, dv, now, 64)
    return o


def rates(impls, flows, per, samples):
    """Interleaved rounds (every implementation on the same chunk in turn),
    so host-speed drift hits all of them alike."""
    out = {k: [] for k in impls}
    pos = flows
    for _ in range(samples):
        fr, ln, dv, now = T.nat_lan_trace(per, flows, start=pos)
        for name, o in impls.items():
            f = fr.copy()
            t0 = time.perf_counter()
            o.run(f, ln, dv, now, 64)
            out[name].append(per / (time.perf_counter() - t0) / 1e6)
        pos += per
    return out


def main():
    flows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 22
    samples = int(sys.argv[3]) if len(sys.argv) > 3 else 9
    mask = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(mask)})
    impls = {name: make(ref, flows) for name, ref in
             (("reference_libvig", True), ("restated", False),
              ("restated_native", "native"))}
    res = {}
    for name, r in rates(impls, flows, per, samples).items():
        res[name] = {"median_mpps": round(float(np.median(r)), 3),
                     "samples": [round(x, 3) for x in r]}
    base = res["reference_libvig"]["median_mpps"]
    ref_s = np.array(res["reference_libvig"]["samples"])
    for k in ("restated", "restated_native"):
        res[k]["ratio_to_reference"] = round(res[k]["median_mpps"] / base, 3)
        # paired: each interleaved round's ratio (host-speed drift cancels),
        # median with a 90 % bootstrap interval of the median
        pr = np.array(res[k]["samples"]) / ref_s
        rng = np.random.default_rng(0)
        boot = np.median(rng.choice(pr, (4000, pr.size)), axis=1)
        res[k]["paired_ratio_median"] = round(float(np.median(pr)), 3)
        res[k]["paired_ratio_90ci"] = [round(float(np.percentile(boot, 5)), 3),
                                       round(float(np.percentile(boot, 95)), 3)]
    res["trace"] = ("vignat 64B, %d flows warm, round robin, %d interleaved "
                    "samples of %d steady-state packets, 1 pinned core (%s)"
                    % (flows, samples, per, bench.cpu_model()))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
