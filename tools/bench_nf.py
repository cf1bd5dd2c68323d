"""Side benchmarks for the other NFs on the path (BASELINE configs 3 and 4,
and vigfw / vigpol, SURVEY.md §8(f);
the headline line is bench.py's vignat). One JSON line per workload:
device-resident Mpps over pre-generated batches, kernel time of the
classification kernel, and the oracle's 1-core rate on a sample.

  python3 tools/bench_nf.py [--batch 4194304] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import vigor_amd  # noqa: E402
from vigor_amd import traces as T  # noqa: E402

SLOT = 64
LB_MACS = [bytes([0x10 * d + i for i in range(6)]) for d in range(3)]


def to_dev(tr, dev):
    fr, ln, dv, now = tr
    return (torch.from_numpy(fr).to(dev),
            torch.from_numpy(ln.astype(np.uint16).view(np.int16)).to(dev),
            torch.from_numpy(dv.astype(np.uint16).view(np.int16)).to(dev),
            int(now[0]))


def run(nf, batches, B, dev):
    """Step rate over the first half of `batches` (no timing events), kernel
    rate over the second half (each classify launch between HIP events)."""
    half = len(batches) // 2
    out = torch.zeros(B, dtype=torch.int16, device=dev)

    def timed(part):
        kms = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for fr, ln, dv, t in part:
            nf.process_device(fr, ln, dv, out, SLOT, now0=t, now_step=1)
            kms.append(nf.last_kernel_ms())
        torch.cuda.synchronize()
        return time.perf_counter() - t0, kms

    nf.kernel_timing(False)
    el, _ = timed(batches[:half])
    nf.kernel_timing(True)
    _, kms = timed(batches[half:])
    nf.kernel_timing(False)
    kernel_s = max(1e-12, sum(m for m, _ in kms) / 1e3)
    launches = sum(k for _, k in kms)
    n = B * half
    return n / el / 1e6, B * (len(batches) - half) / kernel_s / 1e6, out


def cpu_rate(kind, cfg, warm, sample, statics=None):
    import orc
    o = orc.Oracle(kind, cfg, statics=statics)
    for tr in warm:
        o.run(tr[0].copy(), tr[1], tr[2], tr[3], SLOT)
    t0 = time.perf_counter()
    n = 0
    for tr in sample:
        o.run(tr[0].copy(), tr[1], tr[2], tr[3], SLOT)
        n += tr[1].shape[0]
    return n / (time.perf_counter() - t0) / 1e6


def bench_bridge(args, dev, flood):
    import orc
    N = args.stations
    cfg = vigor_amd.bridge_config_from_args(
        ["--capacity", str(N), "--expire", "60000000"], 2)
    br = vigor_amd.Bridge(cfg, gpu=0)
    B = args.batch
    gen = lambda s: T.bridge_trace(B, N, start=s, flood_pattern=flood)  # noqa
    t0 = time.perf_counter()
    warm = [to_dev(gen(w * B), dev) for w in range(max(1, N // B))]
    run(br, warm, B, dev)
    warm_s = time.perf_counter() - t0
    base = len(warm) * B
    batches = [to_dev(gen(base + k * B), dev) for k in range(2 * args.steps)]
    if os.environ.get("BENCH_NF_SAME"):  # diagnostics: one batch's frames every step
        fr0 = batches[0]
        batches = [(fr0[0], fr0[1], fr0[2], fr0[3] + k * B) for k in range(2 * args.steps)]
    mpps, kmpps, out = run(br, batches, B, dev)
    ocfg = orc.BridgeCfg(expiration_time=60_000_000, dyn_capacity=N, n_devices=2)
    cpu = None
    if not args.no_cpu:
        cpu = cpu_rate("bridge", ocfg, [T.bridge_trace(N, N, flood_pattern=flood)],
                       [T.bridge_trace(1 << 21, N, start=N, flood_pattern=flood)])
    return {"workload": "vigbridge 64B, %d MACs%s" % (N, ", flood pattern"
                                                       if flood else ""),
            "value": round(mpps, 1), "unit": "Mpps", "kernel_mpps": round(kmpps, 1),
            "kernel": "bridge_classify", "batch_packets": B, "steps": args.steps,
            "warm_s": round(warm_s, 2),
            "flooded": int((out == -1).sum().item()),
            "cpu_baseline": {"value": round(cpu, 2), "unit": "Mpps", "cores": 1,
                             "kind": "port"} if cpu else None}


def bench_lb(args, dev):
    import orc
    N = args.flows
    argv = ["--flow-capacity", str(N), "--backend-capacity", "256",
            "--cht-height", "257", "--flow-expiration", "60000000",
            "--backend-expiration", "3600000000", "--wan", "2"]
    cfg = vigor_amd.lb_config_from_args(argv, 3, LB_MACS)
    lb = vigor_amd.Lb(cfg, gpu=0)
    B = args.batch
    hb = T.lb_heartbeats(256)
    fr, ln, dv, now = (torch.from_numpy(hb[0]).to(dev),
                       torch.from_numpy(hb[1].astype(np.int16)).to(dev),
                       torch.from_numpy(hb[2].astype(np.int16)).to(dev), None)
    lb.process_device(fr, ln, dv, torch.zeros(256, dtype=torch.int16, device=dev),
                      SLOT, now=torch.from_numpy(hb[3]).to(dev))
    gen = lambda s: T.lb_traffic(B, N, start=s)  # noqa
    t0 = time.perf_counter()
    warm = [to_dev(gen(w * B), dev) for w in range(max(1, N // B))]
    run(lb, warm, B, dev)
    warm_s = time.perf_counter() - t0
    base = len(warm) * B
    batches = [to_dev(gen(base + k * B), dev) for k in range(2 * args.steps)]
    mpps, kmpps, out = run(lb, batches, B, dev)
    cpu = None
    if not args.no_cpu:
        ocfg = orc.LbCfg(flow_capacity=N, flow_expiration_time=60_000_000,
                         backend_capacity=256, cht_height=257,
                         backend_expiration_time=3_600_000_000, wan_device=2,
                         n_devices=3)
        cpu = cpu_rate("lb", ocfg, [hb, T.lb_traffic(N, N)],
                       [T.lb_traffic(1 << 21, N, start=N)])
    return {"workload": "viglb 64B, 256 backends / %d flows" % N,
            "value": round(mpps, 1), "unit": "Mpps", "kernel_mpps": round(kmpps, 1),
            "kernel": "lb_classify64", "batch_packets": B, "steps": args.steps,
            "warm_s": round(warm_s, 2),
            "dropped": int((out == 2).sum().item()),
            "cpu_baseline": {"value": round(cpu, 2), "unit": "Mpps", "cores": 1,
                             "kind": "port"} if cpu else None}


def bench_fw(args, dev):
    """vigfw 64 B, 1M flows: warm-up opens every flow, then steady state with
    every 4th packet the WAN reply of its flow (reversed-key lookup)."""
    import orc
    N = args.flows
    macs = [bytes([2, 0, 0, 0, 0, d]) for d in range(2)]
    argv = ["--max-flows", str(N), "--expire", "60000000", "--wan", "1",
            "--eth-dest", "0,90:e2:ba:55:12:20", "--eth-dest", "1,90:e2:ba:55:12:21"]
    cfg = vigor_amd.fw_config_from_args(argv, 2, macs)
    fw = vigor_amd.Fw(cfg, gpu=0)
    B = args.batch
    gen = lambda s, r: T.fw_trace(B, N, start=s, reply_every=r)  # noqa
    t0 = time.perf_counter()
    warm = [to_dev(gen(w * B, 0), dev) for w in range(max(1, N // B))]
    run(fw, warm, B, dev)
    warm_s = time.perf_counter() - t0
    base = len(warm) * B
    batches = [to_dev(gen(base + k * B, 4), dev) for k in range(2 * args.steps)]
    mpps, kmpps, out = run(fw, batches, B, dev)
    cpu = None
    if not args.no_cpu:
        ocfg = orc.fw_cfg(wan=1, expire_us=60_000_000, max_flows=N,
                          device_macs=macs, n_devices=2)
        cpu = cpu_rate("fw", ocfg, [T.fw_trace(N, N)],
                       [T.fw_trace(1 << 21, N, start=N, reply_every=4)])
    return {"workload": "vigfw 64B, %d flows, 1/4 WAN replies" % N,
            "value": round(mpps, 1), "unit": "Mpps", "kernel_mpps": round(kmpps, 1),
            "kernel": "fw_classify64", "batch_packets": B, "steps": args.steps,
            "warm_s": round(warm_s, 2),
            "dropped": int((out == 1).sum().item()) - (B - B // 4),
            "cpu_baseline": {"value": round(cpu, 2), "unit": "Mpps", "cores": 1,
                             "kind": "port"} if cpu else None}


def bench_pol(args, dev):
    """vigpol 64 B, 1M destinations, the reference's own NF_ARGS rate and
    burst (vigpol/Makefile:5: 375 MB/s, 3.75 GB): warm-up allocates every
    destination, then steady state (every packet a hit, replayed through its
    token bucket)."""
    import orc
    N = args.flows
    argv = ["--lan", "1", "--wan", "0", "--rate", "375000000", "--burst",
            "3750000000", "--capacity", str(N)]
    pol = vigor_amd.Pol(vigor_amd.pol_config_from_args(argv, 2), gpu=0)
    B = args.batch
    gen = lambda s: T.pol_trace(B, N, start=s)  # noqa
    t0 = time.perf_counter()
    warm = [to_dev(gen(w * B), dev) for w in range(max(1, N // B))]
    run(pol, warm, B, dev)
    warm_s = time.perf_counter() - t0
    base = len(warm) * B
    batches = [to_dev(gen(base + k * B), dev) for k in range(2 * args.steps)]
    mpps, kmpps, out = run(pol, batches, B, dev)
    cpu = None
    if not args.no_cpu:
        ocfg = orc.pol_cfg(lan=1, wan=0, capacity=N, n_devices=2)
        cpu = cpu_rate("pol", ocfg, [T.pol_trace(N, N)],
                       [T.pol_trace(1 << 21, N, start=N)])
    return {"workload": "vigpol 64B, %d destinations" % N,
            "value": round(mpps, 1), "unit": "Mpps", "kernel_mpps": round(kmpps, 1),
            "kernel": "pol_classify", "batch_packets": B, "steps": args.steps,
            "warm_s": round(warm_s, 2),
            "forwarded": int((out == 1).sum().item()),
            "cpu_baseline": {"value": round(cpu, 2), "unit": "Mpps", "cores": 1,
                             "kind": "port"} if cpu else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--stations", type=int, default=1 << 20)
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", default="bridge,flood,lb,fw,pol")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    todo = args.only.split(",")
    if "bridge" in todo:
        print(json.dumps(bench_bridge(args, dev, False)), flush=True)
    if "flood" in todo:
        print(json.dumps(bench_bridge(args, dev, True)), flush=True)
    if "lb" in todo:
        print(json.dumps(bench_lb(args, dev)), flush=True)
    if "fw" in todo:
        print(json.dumps(bench_fw(args, dev)), flush=True)
    if "pol" in todo:
        print(json.dumps(bench_pol(args, dev)), flush=True)


if __name__ == "__main__":
    main()
