"""One of bench.py's extra workloads alone (for a kernel trace or counters of
that workload only): config3_bridge, config4_lb, nat_random_keys, nat_churn.

  python3 tools/bench_extra.py NAME [--steps K]

Prints the workload's JSON object as bench.py puts it into its line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name", choices=["config3_bridge", "config4_lb", "nat_random_keys",
                                     "nat_churn"])
    ap.add_argument("--steps", type=int, default=bench.EXTRA_STEPS)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = 1 << 24
    gold = bench.golden_configs()
    if args.name == "config3_bridge":
        r = bench.bench_bridge_c3(dev, B, args.steps, gold.get("bridge"))
    elif args.name == "config4_lb":
        r = bench.bench_lb_c4(dev, B, args.steps, gold.get("lb"))
    elif args.name == "nat_random_keys":
        r = bench.bench_nat_random(dev, B, args.steps, gold.get("random"))
    else:
        r = bench.bench_nat_churn(dev, B, args.steps, gold.get("churn"),
                                  gold.get("churn_state"))
    print(json.dumps({args.name: r}), flush=True)


if __name__ == "__main__":
    main()
