"""End-to-end (host-resident) vignat rate: frames start and end in host
memory, as DPDK mbufs would (SURVEY.md §8(d) "End-to-end"). vp_process_host
moves chunks over PCIe on a copy stream beside the compute stream (double
buffered); page-locked frames (a registered mbuf pool) are DMA'd in place,
pageable ones are staged through pinned memory.

  python3 tools/bench_e2e.py [--batch 4194304] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import vigor_amd  # noqa: E402
from vigor_amd import traces as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--flows", type=int, default=1 << 20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = vigor_amd.nat_config_from_args(
        bench.NAT_ARGS + ["--max-flows", str(args.flows)], 2, bench.DEV_MACS)
    nat = vigor_amd.Nat(cfg, gpu=0)
    B = args.batch
    bank = bench.FlowBank(args.flows, 0, dev)
    # warm every flow through the device path
    w = torch.empty(args.flows * 64, dtype=torch.uint8, device=dev)
    bank.fill(w, 0)
    z = torch.zeros(args.flows, dtype=torch.int16, device=dev)
    nat.process_device(w, torch.full_like(z, 60), z, z.clone(), 64,
                       now0=T.NOW0, now_step=1)
    del w
    start = args.flows
    lens = np.full(B, 60, np.uint16)
    ind = np.zeros(B, np.uint16)
    res = []
    for mode in ("pinned", "pageable"):
        bufs = []
        d = torch.empty(B * 64, dtype=torch.uint8, device=dev)
        for k in range(args.steps):
            bank.fill(d, start + k * B)
            h = d.cpu()
            bufs.append(h.pin_memory().numpy() if mode == "pinned" else
                        h.numpy().copy())
        nows = [T.NOW0 + start + k * B + np.arange(B, dtype=np.int64)
                for k in range(args.steps)]
        t0 = time.perf_counter()
        for k in range(args.steps):
            out = nat.process_host(bufs[k], lens, ind, nows[k], 64)
        el = time.perf_counter() - t0
        assert (out == 1).all()
        start += args.steps * B
        res.append({"workload": "vignat 64B, %d flows, host-resident frames "
                                "(%s), H2D + process + D2H" % (args.flows, mode),
                    "value": round(B * args.steps / el / 1e6, 1),
                    "unit": "Mpps", "batch_packets": B, "steps": args.steps,
                    "chunk": int(os.environ.get("VIGPATH_HOST_CHUNK", 1 << 20)),
                    "pcie_bytes_per_packet": 64 + 12 + 64 + 2})
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
