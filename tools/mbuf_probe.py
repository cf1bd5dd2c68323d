"""Diagnostics for the mbuf path (vp_process_mbufs, vp_mbuf.hip): vignat
over a warm 1M-flow table, 2^22 64-byte frames per call in a page-locked
pool, timed per call, for several pointer layouts and pipeline settings.

  python3 tools/mbuf_probe.py [--variants shuffled,sequential,dense] ...

layouts: shuffled   mbufs of 2304 bytes, data at 256, in random order (the
                    bench's end_to_end_mbuf)
         sequential the same mbufs in pool order
         dense      frames packed 64 bytes apart (no mbuf stride)
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

import bench  # noqa: E402
from vigor_amd import traces as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="shuffled,sequential,dense")
    ap.add_argument("--chunks", default="1048576")
    ap.add_argument("--blocks", default="256")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--modes", default="gpu",
                    help="VIGPATH_MBUF_MODE values: gpu (zero-copy), host (host threads gather)")
    ap.add_argument("--pools", default="pinned",
                    help="pinned (page-locked 4 KB pages), huge (2 MB THP, registered)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = bench.MBUF_BATCH
    flows = 1 << 20
    nat = bench.make_nat(flows)
    bank = bench.FlowBank(flows, 0, dev)
    lens_d = torch.full((B,), 60, dtype=torch.int16, device=dev)
    ind_d = torch.zeros(B, dtype=torch.int16, device=dev)
    out_d = torch.zeros(B, dtype=torch.int16, device=dev)
    d = torch.empty(B * 64, dtype=torch.uint8, device=dev)
    for w in range(2):  # allocate and warm every flow
        bank.fill(d, w * B)
        nat.process_device(d, lens_d, ind_d, out_d, 64, now0=T.NOW0 + w * B, now_step=1)
    torch.cuda.synchronize()
    try:
        print(json.dumps({"thp": open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()}))
    except OSError:
        pass
    start = 4 * B  # (times only move forward, across pools too)
    for kind in args.pools.split(","):
        pool = T.MbufPool(B, pinned=kind == "pinned", huge=kind == "huge")
        nat.register_host(pool.mem)
        pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()  # noqa
        lens = pin(np.full(B, 60, np.uint16))
        ind = pin(np.zeros(B, np.uint16))
        out = pin(np.zeros(B, np.uint16))
        rng = np.random.default_rng(3)
        hdr = np.empty((B, 64), np.uint8)
        for var in args.variants.split(","):
            if var == "shuffled":
                bufs = rng.permutation(B)
                ptrs = pin(pool.ptrs(bufs))
            elif var == "sequential":
                bufs = np.arange(B)
                ptrs = pin(pool.ptrs(bufs))
            else:  # dense: frame i at pool base + 64 i
                bufs = None
                ptrs = pin(np.uint64(pool.mem.ctypes.data) + np.arange(B, dtype=np.uint64) * 64)
            for ch in args.chunks.split(","):
                for blk, mode in [(b, m) for b in args.blocks.split(",")
                                  for m in args.modes.split(",")]:
                    os.environ["VIGPATH_MBUF_MODE"] = mode
                    os.environ["VIGPATH_HOST_CHUNK"] = ch
                    os.environ["VIGPATH_MBUF_BLOCKS"] = blk
                    call = nat.mbuf_step(ptrs, lens, ind, out)
                    times = []
                    for k in range(args.steps + 1):
                        bank.fill(d, start)
                        hdr[:] = d.view(B, 64).cpu().numpy()
                        if bufs is None:
                            pool.mem[:B * 64] = hdr.reshape(-1)
                        else:
                            pool.rows[bufs, 256:320] = hdr
                        t0 = time.perf_counter()
                        call(T.NOW0 + start, 1)
                        el = time.perf_counter() - t0
                        start += B
                        if k:
                            times.append(el)
                    assert (out == 1).all()
                    el = sum(times) / len(times)
                    print(json.dumps({"pool": kind, "layout": var, "chunk": int(ch), "blocks": int(blk),
                                      "mode": mode,
                                      "threads": os.environ.get("VIGPATH_MBUF_THREADS", "8"),
                                      "ms_per_call": round(el * 1e3, 3),
                                      "mpps": round(B / el / 1e6, 1)}), flush=True)
        nat.unregister_host(pool.mem)
        del pool


if __name__ == "__main__":
    main()
