"""Multi-GPU vignat parity: N ranks (processes) act as ONE vignat over the
concatenation of their slices of every global batch (rank 0 first), and the
result must equal the oracle over the whole trace — out ports, frames, and
the merged table state. The ranks share the box's one GPU and talk through
the host-callback transport (gloo); the 8-GPU bench uses RCCL, same library
code above the transport."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import orc
from tracegen import mixed_nat_trace
from vigor_amd import traces as T

pytestmark = pytest.mark.gpu

DEV_MACS = [T.mac("02:03:04:05:06:07"), T.mac("12:13:14:15:16:17")]
END_MACS = [T.mac("01:23:45:67:89:00"), T.mac("01:23:45:67:89:01")]


def _trace(spec):
    kind = spec["kind"]
    if kind == "rr":
        return T.nat_lan_trace(spec["n"], spec["flows"])
    rng = np.random.default_rng(spec["seed"])
    fr, ln, dv, now = mixed_nat_trace(rng, spec["n"], spec["flows"],
                                      max_idx=spec["max_flows"])
    if spec.get("ties"):
        now = T.NOW0 + (np.arange(spec["n"]) // 7).astype(np.int64) * 1_000_000
    return fr, ln, dv, now


def _slices(spec, a, b, world):
    """Per-rank sizes of global batch [a, b)."""
    n = b - a
    if spec.get("uneven"):
        cut = sorted(np.random.default_rng(a).integers(0, n + 1, world - 1))
        cut = [0] + list(cut) + [n]
        return [int(cut[r + 1] - cut[r]) for r in range(world)]
    base, extra = divmod(n, world)
    return [base + (1 if r < extra else 0) for r in range(world)]


def _worker(rank, world, port, spec, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if spec.get("own_cap"):  # owner mode: force the padded exchange's capacity
        os.environ["VIGPATH_OWN_CAP"] = str(spec["own_cap"])
    os.environ.update(spec.get("env", {}))  # (e.g. the chunked pipeline's geometry)
    import vigor_amd
    from gpuh import run_gpu
    from vigor_amd import shard
    args = ["--wan", "1", "--expire", str(spec["expire_us"]),
            "--starting-port", "0", "--max-flows", str(spec["max_flows"]),
            "--extip", "192.168.4.2", "--eth-dest",
            "0," + END_MACS[0].hex(":"), "--eth-dest", "1," + END_MACS[1].hex(":")]
    cfg = vigor_amd.nat_config_from_args(args, 2, DEV_MACS)
    nat = vigor_amd.Nat(cfg, gpu=0)
    shard.attach_torch(nat, rank, world, mode=spec.get("mode", "replicated"))
    fr, ln, dv, now = _trace(spec)
    n = ln.shape[0]
    bounds = [0] + spec["cuts"] + [n]
    outs, frames, pos = [], [], []
    for a, b in zip(bounds[:-1], bounds[1:]):
        sizes = _slices(spec, a, b, world)
        s = a + sum(sizes[:rank])
        e = s + sizes[rank]
        got, out = run_gpu(nat, fr[s * 64:e * 64], ln[s:e], dv[s:e], now[s:e],
                           64, affine=(int(now[s]), 1) if spec.get("affine")
                           and e > s else None)
        outs.append(out)
        frames.append(got)
        pos.append(np.arange(s, e))
    nat.sync_state()
    res = dict(out=np.concatenate(outs), frames=np.concatenate(frames),
               pos=np.concatenate(pos))
    if rank == 0:
        a_, t_, k_ = nat.dump()
        res.update(alloc=a_, ts=t_, keys=k_, live=np.array([nat.live_count()]))
    np.savez(os.path.join(outdir, "r%d.npz" % rank), **res)
    torch.cuda.synchronize()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_sharded(spec, world):
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        ps = [ctx.Process(target=_worker, args=(r, world, port, spec, d))
              for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=300)
        codes = [p.exitcode for p in ps]
        assert codes == [0] * world, codes
        return [dict(np.load(os.path.join(d, "r%d.npz" % r)))
                for r in range(world)]


def test_rccl_transport_single_rank():
    """The RCCL transport in-process (one rank: every collective is a copy on
    the context's stream) through the multi-GPU batch driver."""
    import vigor_amd
    from gpuh import check_batches
    from vigor_amd import shard
    args = ["--wan", "1", "--expire", "5", "--starting-port", "0",
            "--max-flows", "256", "--extip", "192.168.4.2", "--eth-dest",
            "0," + END_MACS[0].hex(":"), "--eth-dest", "1," + END_MACS[1].hex(":")]
    nat = vigor_amd.Nat(vigor_amd.nat_config_from_args(args, 2, DEV_MACS), gpu=0)
    import ctypes as C
    uid = (C.c_uint8 * 128).from_buffer_copy(shard.rccl_unique_id())
    assert nat.L.vp_attach_rccl(nat.h, uid, 1, 0) == 0
    rng = np.random.default_rng(3)
    fr, ln, dv, now = mixed_nat_trace(rng, 6000, 300, max_idx=256)
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=5, max_flows=256, device_macs=DEV_MACS,
                      endpoint_macs=END_MACS)
    o = orc.Oracle("nat", cfg)
    check_batches(nat, o, fr, ln, dv, now, 64, [1000, 1001, 3000])
    nat.sync_state()
    oa, ots, ok = o.nat_dump(256)
    ga, gts, gk = nat.dump()
    np.testing.assert_array_equal(ga, oa)
    np.testing.assert_array_equal(gts[oa == 1], ots[oa == 1])


SPECS = [
    (2, dict(kind="rr", n=40_000, flows=1000, max_flows=65536,
             expire_us=60_000_000, cuts=[1000, 20_000], affine=True)),
    (3, dict(kind="mixed", seed=1, n=5000, flows=100, max_flows=64,
             expire_us=1, cuts=[1, 2, 500, 4000], uneven=True)),
    (2, dict(kind="mixed", seed=2, n=5000, flows=40, max_flows=16,
             expire_us=60_000_000, cuts=[2500], uneven=True)),
    (4, dict(kind="mixed", seed=3, n=6000, flows=300, max_flows=256,
             expire_us=5, cuts=[1000, 1001, 3000])),
    (2, dict(kind="mixed", seed=7, n=6000, flows=300, max_flows=512,
             expire_us=4_295_000, cuts=[1234, 3000], ties=True)),
]


@pytest.mark.parametrize("mode", ["replicated", "owner"])
@pytest.mark.parametrize("world,spec", SPECS)
def test_sharded_nat_equals_single_nf(world, spec, mode):
    """Both dictionary placements: replicated, and owner-sharded by flow hash
    (LAN lookups of other ranks' keys through the all-to-all)."""
    check_sharded(dict(spec, mode=mode), world)


@pytest.mark.parametrize("world,spec", [
    (2, dict(SPECS[0][1], own_cap=64)),
    (3, dict(SPECS[1][1], own_cap=8)),
    (4, dict(SPECS[3][1], own_cap=40)),
])
def test_owner_padded_exchange_overflow(world, spec):
    """Owner mode with the padded exchange's capacity forced small: segments
    whose keys for some owner exceed it are detected on the device (every
    rank agrees through the allreduced flag), pass 2 leaves the routed
    packets alone and the exact exchange answers them; the results are
    still the single NF's."""
    check_sharded(dict(spec, mode="owner"), world)


# The chunked owner pipeline in chunks of 4 blocks x 4 tiles
# (1024 packets) instead of the resident grid x 2^20 packets: batches of
# thousands of packets take many chunks, alternating the two buffer sets.
CHUNKS = {"VIGPATH_OWN_BLOCKS": "4", "VIGPATH_OWN_CHUNK": "1024"}


@pytest.mark.parametrize("world,spec", [
    (2, dict(SPECS[0][1], env=CHUNKS)),
    (3, dict(SPECS[1][1], env=CHUNKS)),
    (4, dict(SPECS[3][1], env=CHUNKS)),
    (2, dict(SPECS[4][1], env=CHUNKS)),
    (2, dict(SPECS[0][1], env=CHUNKS, own_cap=64)),
    (4, dict(SPECS[3][1], env=CHUNKS, own_cap=40)),
])
def test_owner_chunked_pipeline(world, spec):
    """Owner mode through the chunked pipeline with many chunks per segment
    (pass 1 / exchange / probe / pass 2 per chunk on two streams, touch bins
    over virtual blocks), with and without slices that overflow (the
    leftover exchange and the second, stamp-raising fold): the single NF's
    results."""
    check_sharded(dict(spec, mode="owner"), world)


def _worker_route_all(outdir, env, n, cuts):
    """One rank with a one-rank RCCL communicator, every LAN key routed
    through the exchange to itself (bench.py --route-all), in chunks."""
    os.environ.update(env)
    os.environ["VIGPATH_ROUTE_ALL"] = "1"
    import ctypes as C
    import vigor_amd
    from gpuh import check_batches
    from vigor_amd import shard
    args = ["--wan", "1", "--expire", "60000000", "--starting-port", "0",
            "--max-flows", "4096", "--extip", "192.168.4.2", "--eth-dest",
            "0," + END_MACS[0].hex(":"), "--eth-dest", "1," + END_MACS[1].hex(":")]
    nat = vigor_amd.Nat(vigor_amd.nat_config_from_args(args, 2, DEV_MACS), gpu=0)
    uid = (C.c_uint8 * 128).from_buffer_copy(shard.rccl_unique_id())
    assert nat.L.vp_attach_rccl(nat.h, uid, 1, 0) == 0
    shard.set_mode(nat, "owner")
    rng = np.random.default_rng(11)
    fr, ln, dv, now = mixed_nat_trace(rng, n, 3000, max_idx=4096)
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=60_000_000, max_flows=4096, device_macs=DEV_MACS,
                      endpoint_macs=END_MACS)
    o = orc.Oracle("nat", cfg)
    check_batches(nat, o, fr, ln, dv, now, 64, cuts)
    oa, ots, ok = o.nat_dump(4096)
    ga, gts, gk = nat.dump()
    np.testing.assert_array_equal(ga, oa)
    np.testing.assert_array_equal(gts[oa == 1], ots[oa == 1])
    np.testing.assert_array_equal(gk[oa == 1], ok[oa == 1])
    # ABI 0.3 on a chunked step with kernel timing on: vp_stage_ms reports
    # the pipeline's eighth stage into a caller-sized array, the 0.2 entry
    # point vp_last_stage_ms writes exactly seven floats (a canary after them
    # survives), and vp_last_kernel names owner pass 1's kernels
    from gpuh import run_gpu
    nat.kernel_timing(True)
    f2, l2, d2, n2 = T.nat_lan_trace(2048, 1024, start=int(now[-1]) - T.NOW0 + 1)
    run_gpu(nat, f2, l2, d2, n2, 64)
    ms8, k8 = (C.c_float * 8)(), C.c_int()
    assert nat.L.vp_stage_ms(nat.h, ms8, 8, C.byref(k8)) == 0
    assert k8.value == 8 and ms8[7] > 0, (k8.value, list(ms8))
    ms7 = (C.c_float * 8)(*([0.0] * 7 + [-1.0]))
    k7 = C.c_int()
    assert nat.L.vp_last_stage_ms(nat.h, ms7, C.byref(k7)) == 0
    assert k7.value == 7 and ms7[7] == -1.0 and list(ms7[:7]) == list(ms8[:7])
    assert nat.L.vp_stage_ms(nat.h, None, 0, C.byref(k8)) == 0 and k8.value == 8
    assert "nat_remote64" in nat.last_kernel()
    open(os.path.join(outdir, "ok"), "w").write("ok")


@pytest.mark.parametrize("env", [dict(CHUNKS), dict(CHUNKS, VIGPATH_OWN_CAP="96")])
def test_owner_route_all_chunked_rccl(env):
    """bench.py --route-all's configuration (one rank, a real RCCL
    communicator, every key through the exchange) in many chunks, with and
    without overflowing slices: bit-exact with the oracle."""
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        p = ctx.Process(target=_worker_route_all, args=(d, env, 30_000, [6400, 19_200]))
        p.start()
        p.join(timeout=300)
        assert p.exitcode == 0
        assert os.path.exists(os.path.join(d, "ok"))


def check_sharded(spec, world):
    res = run_sharded(spec, world)
    fr, ln, dv, now = _trace(spec)
    cfg = orc.nat_cfg(wan=1, start_port=0, ext_ip=T.ip4(192, 168, 4, 2),
                      expire_us=spec["expire_us"], max_flows=spec["max_flows"],
                      device_macs=DEV_MACS, endpoint_macs=END_MACS)
    o = orc.Oracle("nat", cfg)
    exp = fr.copy()
    exp_out = o.run(exp, ln, dv, now, 64)
    n = ln.shape[0]
    got_out = np.zeros(n, np.uint16)
    got_fr = np.zeros((n, 64), np.uint8)
    seen = np.zeros(n, bool)
    for r in res:
        got_out[r["pos"]] = r["out"]
        got_fr[r["pos"]] = r["frames"].reshape(-1, 64)
        seen[r["pos"]] = True
    assert seen.all()
    bad = np.nonzero(got_out != exp_out)[0]
    assert bad.size == 0, "out mismatch at %s" % bad[:10]
    badf = np.nonzero((got_fr != exp.reshape(n, 64)).any(axis=1))[0]
    assert badf.size == 0, "frame mismatch at %s" % badf[:10]
    oa, ots, ok = o.nat_dump(spec["max_flows"])
    np.testing.assert_array_equal(res[0]["alloc"], oa)
    np.testing.assert_array_equal(res[0]["ts"][oa == 1], ots[oa == 1])
    np.testing.assert_array_equal(res[0]["keys"][oa == 1], ok[oa == 1])


def _worker16m(rank, world, port, mode, outdir):
    """BASELINE configs[4] table size over `world` ranks: 16M flows, the
    round-robin trace in global batches of 2^24 packets (rank r ingests the
    r-th contiguous slice), every flow allocated in batch 0 and hit in
    batch 1. Each rank digests its own outputs at their global positions."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import golden_cases as G
    from vigor_amd import shard
    nat = G.nat_gpu(G.F16M_FLOWS)
    shard.attach_torch(nat, rank, world, mode=mode)
    d = torch.device("cuda:0")
    GB = 1 << 24
    per = GB // world
    lens = torch.full((per,), 60, dtype=torch.int16, device=d)
    ind = torch.zeros(per, dtype=torch.int16, device=d)
    out = torch.zeros(per, dtype=torch.int16, device=d)
    dig = 0
    for k in range(G.F16M_PACKETS // GB):
        s0 = k * GB + rank * per
        fr, _, _, _ = T.nat_lan_trace(per, G.F16M_FLOWS, start=s0)
        f = torch.from_numpy(fr).to(d)
        del fr
        nat.process_device(f, lens, ind, out, 64, now0=T.NOW0 + s0, now_step=1)
        torch.cuda.synchronize()
        dig += T.batch_digest(f.cpu().numpy(), out.cpu().numpy().view(np.uint16), 64, s0)
        del f
    nat.sync_state()
    res = dict(digest=np.array(dig % (1 << 64), np.uint64))
    if rank == 0:
        a_, t_, _ = nat.dump()
        res.update(state=np.array(T.state_digest(a_, t_), np.uint64),
                   live=np.array(nat.live_count()))
    np.savez(os.path.join(outdir, "r%d.npz" % rank), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["replicated", "owner"])
def test_sharded_16m_flows_equals_reference(mode):
    """configs[4]'s table (16M flows) over 2 ranks sharing the GPU (gloo
    transport): output bytes of all 2^25 packets and the merged table state
    equal the reference's (tests/golden/nat_16m_digest.npz)."""
    import golden_cases as G
    g = G.load("nat_16m_digest")
    assert str(g["impl"]) == "reference"
    world = 2
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        ps = [ctx.Process(target=_worker16m, args=(r, world, port, mode, d))
              for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=400)
        assert [p.exitcode for p in ps] == [0] * world
        res = [dict(np.load(os.path.join(d, "r%d.npz" % r))) for r in range(world)]
    assert sum(int(r["digest"]) for r in res) % (1 << 64) == int(g["digest"])
    assert int(res[0]["state"]) == int(g["state_digest"])
    assert int(res[0]["live"]) == int(g["live"])
