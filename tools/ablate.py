"""Diagnostic: where does nat_classify's time go? Runs the steady-state
config-2 step on the product build and on ablation builds
(vigor_amd/abl/libvigpath_<X>.so, `make -C vigor_amd/csrc ablate`) in one
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24), and
prints kernel time per variant. Ablated builds compute wrong results and are
never used for anything else."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import vigor_amd  # noqa: E402
from vigor_amd import traces as T  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    B, NF = 1 << 24, 1 << 20
    dev = torch.device("cuda:0")
    variants = {"full": (None, {}), "perlane": (None, {"VIGPATH_COALESCED": "0"})}
    variants["bpc3"] = (None, {"VIGPATH_BLOCKS_PER_CU": "3"})
    variants["bpc2"] = (None, {"VIGPATH_BLOCKS_PER_CU": "2"})
    variants["nolin"] = (None, {"VIGPATH_LIN": "0"})  # CRC-bit home buckets
    variants["lin1"] = (None, {"VIGPATH_LIN": "1"})  # one index per bucket
    only = os.environ.get("ABLATE_ONLY")  # comma-separated variant names
    abl = os.path.join(ROOT, "vigor_amd", "abl")
    names = sorted(f[len("libvigpath_"):-3] for f in os.listdir(abl)
                   if f.startswith("libvigpath_") and f.endswith(".so")) \
        if os.path.isdir(abl) else []
    for v in names:  # ablation builds, or any other build to compare (A/B)
        p = os.path.join(abl, "libvigpath_%s.so" % v)
        # NOFRAME lives in the per-lane kernel
        variants[v] = (p, {"VIGPATH_COALESCED": "0"} if v == "NOFRAME" else {})
    if only:
        keep = set(only.split(",")) | {"full"}
        variants = {k: v for k, v in variants.items() if k in keep}
    bank = bench.FlowBank(NF, 0, dev)
    lens = torch.full((B,), 60, dtype=torch.int16, device=dev)
    ind = torch.zeros(B, dtype=torch.int16, device=dev)
    out = torch.zeros(B, dtype=torch.int16, device=dev)
    buf = torch.empty(B * 64, dtype=torch.uint8, device=dev)
    nfs = {}
    def use_env(env):  # read at context creation and at every launch
        for k in ("VIGPATH_COALESCED", "VIGPATH_BLOCKS_PER_CU", "VIGPATH_LIN"):
            os.environ.pop(k, None)
        os.environ.update(env)

    for name, (path, env) in variants.items():
        use_env(env)
        cfg = vigor_amd.nat_config_from_args(
            bench.NAT_ARGS + ["--max-flows", str(NF)], 2, bench.DEV_MACS)
        nat = vigor_amd.Nat(cfg, 0, libpath=path)
        bank.fill(buf, 0)
        nat.process_device(buf, lens, ind, out, 64, now0=T.NOW0, now_step=1)
        nfs[name] = nat
    res = {k: [] for k in nfs}
    step_ms = {k: [] for k in nfs}
    start = B
    for r in range(rounds):
        for name, nat in nfs.items():
            use_env(variants[name][1])
            bank.fill(buf, start)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nat.process_device(buf, lens, ind, out, 64, now0=T.NOW0 + start,
                               now_step=1)
            torch.cuda.synchronize()
            nat.step_ms = (time.perf_counter() - t0) * 1e3
            res[name].append(nat.last_kernel_ms()[0])
            step_ms[name].append(nat.step_ms)
        start += B
    for name, v in res.items():
        med = statistics.median(v)
        sm = statistics.median(step_ms[name])
        print("%-11s kernel median %.3f ms min %.3f ms -> %.2f Gpps | step "
              "%.3f ms -> %.2f Gpps" % (name, med, min(v), B / med / 1e6, sm,
                                        B / sm / 1e6))


if __name__ == "__main__":
    main()
