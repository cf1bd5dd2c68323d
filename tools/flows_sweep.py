"""Diagnostic: classify-kernel rate vs flow-table size (cache residency)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import vigor_amd  # noqa: E402
from vigor_amd import traces as T  # noqa: E402

B = 1 << 24
dev = torch.device("cuda:0")
lens = torch.full((B,), 60, dtype=torch.int16, device=dev)
ind = torch.zeros(B, dtype=torch.int16, device=dev)
out = torch.zeros(B, dtype=torch.int16, device=dev)
buf = torch.empty(B * 64, dtype=torch.uint8, device=dev)
libs = [None] + [os.path.join(ROOT, "vigor_amd", "abl", x)
                 for x in sys.argv[1:]]
SIZES = [int(x) for x in os.environ.get("SWEEP_FLOWS", "").split(",") if x] or \
    [1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 22]
for nf in SIZES:
    for lp in libs:
        cfg = vigor_amd.nat_config_from_args(
            bench.NAT_ARGS + ["--max-flows", str(nf)], 2, bench.DEV_MACS)
        nat = vigor_amd.Nat(cfg, 0, libpath=lp)
        nat.kernel_timing(True)
        bank = bench.FlowBank(nf, 0, dev)
        start = 0
        ms = []
        for r in range(4):
            bank.fill(buf, start)
            torch.cuda.synchronize()
            nat.process_device(buf, lens, ind, out, 64, now0=T.NOW0 + start,
                               now_step=1)
            ms.append(nat.last_kernel_ms()[0])
            start += B
        best = min(ms[1:])
        print("flows %8d %-24s table %6.1f MB  %.3f ms  %.2f Gpps" %
              (nf, os.path.basename(lp or "full"),
               32 * 2 * nf / 1e6, best, B / best / 1e6), flush=True)
        nat.close()
        del bank
