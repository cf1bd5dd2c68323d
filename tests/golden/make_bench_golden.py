"""tests/golden/bench_configs.npz: the reference's outputs for the extra
workloads bench.py times (this container only: needs /root/reference for
oracle/_ref). Per workload, the digest (traces.batch_digest) of every batch
bench.py may check, computed by the oracle glue over the reference's own
libVig on exactly the batches bench.py feeds the GPU:

  bridge   BASELINE configs[2]: vigbridge, 1M MACs, 2^24-packet batches of
           traces.bridge_trace (batch 0 learns every station; from batch 1
           on every batch has the same frames and outputs)
  lb       BASELINE configs[3]: viglb, 256 backends (heartbeats first), 1M
           flows of traces.lb_traffic, 2^24-packet batches
  random   vignat, 1M flows with random 5-tuples (traces.random_flow_keys),
           round robin, 2^24-packet batches
  churn    vignat, 1 s expiry (run-middlebox.sh:16), the steady-turnover
           trace traces.churn_trace, CHURN_BATCHES batches of 2^24 packets

  python3 tests/golden/make_bench_golden.py [--only bridge,lb,random,churn]
"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import orc  # noqa: E402
from vigor_amd import traces as T  # noqa: E402

B = 1 << 24
CHUNK = 1 << 22
FLOWS = 1 << 20
CHURN_BATCHES = 16
# the configurations of bench.py (configs_bench)
NAT_DEV = [T.mac("02:00:00:00:00:00"), T.mac("02:00:00:00:00:01")]
NAT_END = [T.mac("90:e2:ba:55:12:20"), T.mac("90:e2:ba:55:12:21")]
LB_MACS = [bytes([0x10 * d + i for i in range(6)]) for d in range(3)]
OUT = os.path.join(HERE, "bench_configs.npz")


def nat_oracle(expire_us):
    cfg = orc.nat_cfg(wan=1, ext_ip=T.ip4(192, 168, 4, 2), expire_us=expire_us,
                      max_flows=FLOWS, device_macs=NAT_DEV, endpoint_macs=NAT_END)
    return orc.Oracle("nat", cfg, ref=True)


def batch_digests(o, gen, batches):
    """Digest of every batch k < batches; gen(k, start, m) -> trace piece."""
    out = []
    for k in range(batches):
        acc = 0
        for s in range(0, B, CHUNK):
            fr, ln, dv, now = gen(k, s, CHUNK)
            res = o.run(fr, ln, dv, now, 64)
            acc += T.batch_digest(fr, res, 64, s)
        out.append(acc % (1 << 64))
        print("  batch", k, hex(out[-1]), flush=True)
    return np.array(out, np.uint64)


def bridge():
    cfg = orc.BridgeCfg(expiration_time=60_000_000, dyn_capacity=FLOWS, n_devices=2)
    o = orc.Oracle("bridge", cfg, ref=True)
    return batch_digests(o, lambda k, s, m: T.bridge_trace(m, FLOWS, start=k * B + s), 2)


def lb():
    cfg = orc.LbCfg(flow_capacity=FLOWS, flow_expiration_time=60_000_000,
                    backend_capacity=256, cht_height=257,
                    backend_expiration_time=3_600_000_000, wan_device=2, n_devices=3)
    for d in range(3):
        cfg.device_macs[d][:] = list(LB_MACS[d])
    o = orc.Oracle("lb", cfg, ref=True)
    hb = T.lb_heartbeats(256)
    o.run(hb[0].copy(), hb[1], hb[2], hb[3], 64)
    return batch_digests(o, lambda k, s, m: T.lb_traffic(m, FLOWS, start=k * B + s), 2)


def random_keys():
    o = nat_oracle(60_000_000)
    keys = T.random_flow_keys(FLOWS)
    return batch_digests(
        o, lambda k, s, m: T.random_key_trace(m, FLOWS, start=k * B + s, keys=keys), 2)


def churn():
    """Per-batch digests and the state digest (traces.state_digest of the
    dchain: allocated indices and their stamps) after the last batch."""
    o = nat_oracle(T.CHURN_EXPIRE_US)
    d = batch_digests(o, lambda k, s, m: T.churn_trace(k, m, start=s), CHURN_BATCHES)
    alloc, ts, _ = o.nat_dump(FLOWS)
    return d, np.array(T.state_digest(alloc, ts), np.uint64), np.array(int(alloc.sum()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="bridge,lb,random,churn")
    args = ap.parse_args()
    have = dict(np.load(OUT, allow_pickle=False)) if os.path.exists(OUT) else {}
    for name, fn in (("bridge", bridge), ("lb", lb), ("random", random_keys),
                     ("churn", churn)):
        if name not in args.only.split(","):
            continue
        t0 = time.time()
        print(name, flush=True)
        r = fn()
        if isinstance(r, tuple):  # churn: + state digest, live flows after the last batch
            have[name], have[name + "_state"], have[name + "_live"] = r
        else:
            have[name] = r
        print(name, "%.0f s" % (time.time() - t0), flush=True)
    have["batch"] = np.array(B)
    have["impl"] = np.array("reference")
    np.savez_compressed(OUT, **have)


if __name__ == "__main__":
    main()
