"""Diagnostic: classify-kernel rate by packet order (round robin over the
flows, as bench.lua:125, vs a uniform hash of the packet index) for the
product build and ablation builds given on the command line
(vigor_amd/abl/libvigpath_<X>.so), 1M flows, B = 2^24."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import vigor_amd  # noqa: E402
from vigor_amd import traces as T  # noqa: E402

B, NF = 1 << 24, 1 << 20
dev = torch.device("cuda:0")


def fill(bank, buf, start, order):
    fv = buf.view(B, 64)
    fv.copy_(bank.template.expand(B, 64))
    p = torch.arange(start, start + B, device=dev, dtype=torch.int64)
    if order == "uniform":  # murmur-style finaliser of the packet index
        x = p * 0x5851F42D + 0x14057B7E
        x = x ^ (x >> 17)
        x = (x & 0x7FFFFFFF) * 0x2545F491
        x = x ^ (x >> 13)
        fl = x % NF
    else:
        fl = p % NF
    v = bank.var.index_select(0, fl)
    fv[:, 24:30] = v[:, 0:6]
    fv[:, 34:36] = v[:, 6:8]


def main():
    lens = torch.full((B,), 60, dtype=torch.int16, device=dev)
    ind = torch.zeros(B, dtype=torch.int16, device=dev)
    out = torch.zeros(B, dtype=torch.int16, device=dev)
    buf = torch.empty(B * 64, dtype=torch.uint8, device=dev)
    bank = bench.FlowBank(NF, 0, dev)
    libs = [None] + [os.path.join(ROOT, "vigor_amd", "abl", "libvigpath_%s.so" % x)
                     for x in sys.argv[1:]]
    for lp in libs:
        cfg = vigor_amd.nat_config_from_args(
            bench.NAT_ARGS + ["--max-flows", str(NF)], 2, bench.DEV_MACS)
        nat = vigor_amd.Nat(cfg, 0, libpath=lp)
        nat.kernel_timing(True)
        fill(bank, buf, 0, "rr")  # warm-up: every flow allocated
        nat.process_device(buf, lens, ind, out, 64, now0=T.NOW0, now_step=1)
        start = B
        for order in ("rr", "uniform"):
            ms = []
            for r in range(4):
                fill(bank, buf, start, order)
                torch.cuda.synchronize()
                nat.process_device(buf, lens, ind, out, 64, now0=T.NOW0 + start,
                                   now_step=1)
                ms.append(nat.last_kernel_ms()[0])
                start += B
            assert int((out != 1).sum().item()) == 0
            best = min(ms[1:])
            print("%-10s %-8s %.3f ms  %.2f Gpps" % (
                os.path.basename(lp or "product")[11:-3] or "product", order, best,
                B / best / 1e6), flush=True)
        nat.close()


if __name__ == "__main__":
    main()
