"""CPU side of the multi-GPU path (world_size 2, gloo): the host-callback
collectives the library calls (vigor_amd.shard.TorchComm through the same
C function pointers libvigpath.so receives), the slice layout, and the
attach entry points' argument checks. The GPU parity of the sharded NF is
tests/test_shard_gpu.py."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import vigor_amd
from vigor_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = shard.TorchComm()
        ops = comm.ops
        # allgather through the C function pointer
        send = (C.c_uint8 * 5)(*[rank * 10 + i for i in range(5)])
        recv = (C.c_uint8 * (5 * world))()
        rc = ops.allgather(None, C.addressof(send), C.addressof(recv), 5)
        ag = list(recv)
        # zero-byte gather still participates
        rc0 = ops.allgather(None, None, None, 0)
        # element-wise max of u64 (< 2^63)
        vals = (C.c_uint64 * 4)(rank, 5 - rank, 1 << 62 if rank else 7, 3)
        rc2 = ops.allreduce_max_u64(None, C.addressof(vals), 4)
        # personalised exchange: q + rank + 1 bytes between rank and q (the
        # owner mode's key / answer all-to-alls), then an all-empty one
        sb = [q_ + rank + 1 for q_ in range(world)]
        data = [rank * 100 + q_ * 10 + i for q_ in range(world) for i in range(sb[q_])]
        send = (C.c_uint8 * len(data))(*data)
        recv = (C.c_uint8 * sum(sb))()
        sz = (C.c_size_t * world)(*sb)
        rc3 = ops.alltoallv(None, C.addressof(send), sz, C.addressof(recv), sz)
        zero = (C.c_size_t * world)()
        rc4 = ops.alltoallv(None, None, zero, None, zero)
        q.put((rank, rc, rc0, rc2, ag, list(vals), rc3, rc4, list(recv)))
    finally:
        dist.destroy_process_group()


def test_torch_comm_collectives_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rc, rc0, rc2, ag, vals, rc3, rc4, a2a in res:
        assert rc == rc0 == rc2 == rc3 == rc4 == 0
        assert ag == [0, 1, 2, 3, 4, 10, 11, 12, 13, 14]
        assert vals == [1, 5, 1 << 62, 3]
        # chunk from q: q's bytes for `rank`, in rank order
        want = [q_ * 100 + rank * 10 + i for q_ in range(world)
                for i in range(q_ + rank + 1)]
        assert a2a == want


def test_slice_layout():
    assert shard.split_even(10, 3) == [4, 3, 3]
    assert shard.split_even(2, 4) == [1, 1, 0, 0]
    assert shard.slice_bounds([4, 0, 3]) == [(0, 4), (4, 4), (4, 7)]


def test_attach_rejects_bad_arguments():
    L = vigor_amd.lib()
    ops = vigor_amd.CommOpsC()
    # no context / bad ranks are rejected before any device call
    assert L.vp_attach_comm(None, C.byref(ops), 2, 0) == -22
    assert L.vp_attach_rccl(None, None, 2, 0) == -22
    assert L.vp_sync_state(None) == -22
    assert L.vp_shard_mode(None, 1) == -22
