"""End-to-end (host-resident) vignat rate: frames start and end in host
memory, as DPDK mbufs would (SURVEY.md §8(d) "End-to-end").
vp_process_host_batch moves chunks over PCIe, host->device and
device->host on two copy streams beside the compute stream (three buffer
sets); page-locked arrays (a registered mbuf pool) are DMA'd in place,
pageable ones are staged through pinned memory. Three cases:
  pinned+affine     every array page-locked, one time per packet as
                    now0 + p (bench.py's end_to_end)
  pinned+time[]     page-locked frames, pageable per-packet arrays and an
                    int64 time per packet (vp_process_host)
  pageable+time[]   everything pageable (host memcpy into staging)

  python3 tools/bench_e2e.py [--batch 16777216] [--steps 3] [--chunk 2097152]
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
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--chunk", type=int, default=1 << 21)
    args = ap.parse_args()
    os.environ["VIGPATH_HOST_CHUNK"] = str(args.chunk)
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
    pin = lambda a: torch.from_numpy(a).pin_memory().numpy()  # noqa: E731
    res = []
    for mode in ("pinned+affine", "pinned+time[]", "pageable+time[]"):
        pinned_arrays = mode == "pinned+affine"
        lens = np.full(B, 60, np.uint16)
        ind = np.zeros(B, np.uint16)
        out = np.zeros(B, np.uint16)
        if pinned_arrays:
            lens, ind, out = pin(lens), pin(ind), pin(out)
        bufs = []
        d = torch.empty(B * 64, dtype=torch.uint8, device=dev)
        for k in range(args.steps + 1):  # batch 0: untimed warm-up
            bank.fill(d, start + k * B)
            h = d.cpu()
            bufs.append(h.pin_memory().numpy() if mode.startswith("pinned") else
                        h.numpy().copy())
        del d

        def step(k):
            t0 = T.NOW0 + start + k * B
            if mode == "pinned+affine":
                nat.process_host_batch(bufs[k], lens, ind, out, 64, now0=t0, now_step=1)
                return out
            now = t0 + np.arange(B, dtype=np.int64)
            return nat.process_host(bufs[k], lens, ind, now, 64)
        step(0)
        t = time.perf_counter()
        for k in range(1, args.steps + 1):
            o = step(k)
        el = time.perf_counter() - t
        assert (o == 1).all()
        start += (args.steps + 1) * B
        per_pkt = 64 + 4 + (0 if mode == "pinned+affine" else 8) + 64 + 2
        res.append({"workload": "vignat 64B, %d flows, host-resident batches (%s), "
                                "H2D + process + D2H" % (args.flows, mode),
                    "value": round(B * args.steps / el / 1e6, 1),
                    "unit": "Mpps", "batch_packets": B, "steps": args.steps,
                    "chunk": args.chunk, "pcie_bytes_per_packet": per_pkt})
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
