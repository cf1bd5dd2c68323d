"""Multi-GPU vignat: one process and one NF context per GPU, acting as ONE
vignat over the concatenation of the ranks' slices of every global batch
(include/vigpath.h "multi-GPU").

Two transports for the library's collectives:
  * RCCL over xGMI (`attach_rccl`): rank 0 makes the RCCL id, the host hands
    it to every rank through torch.distributed; the library then runs its
    all-gathers / all-reduces on device buffers on its own stream.
  * host callbacks (`attach_torch`): the library calls back into
    torch.distributed (gloo) with host buffers. Used when several ranks share
    one GPU (parity tests on a one-GPU box) and on CPU-only hosts.
"""
from __future__ import annotations

import ctypes as C
import sys
import traceback

import numpy as np

from . import (ALLGATHER_FN, ALLREDUCE_FN, ALLTOALLV_FN, SHARD_OWNER,
               SHARD_REPLICATED, CommOpsC, _check, lib)

MODES = {"replicated": SHARD_REPLICATED, "owner": SHARD_OWNER}


def slice_bounds(sizes):
    """Global positions [start, end) of each rank's slice (rank order)."""
    off = np.concatenate([[0], np.cumsum(np.asarray(sizes, np.int64))])
    return [(int(off[r]), int(off[r + 1])) for r in range(len(sizes))]


def split_even(n: int, world: int):
    """Contiguous near-equal slice sizes of an n-packet global batch."""
    base, extra = divmod(n, world)
    return [base + (1 if r < extra else 0) for r in range(world)]


class TorchComm:
    """vp_comm_ops over torch.distributed on host memory (any backend that
    takes CPU tensors, e.g. gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self._ag = ALLGATHER_FN(self._allgather)
        self._ar = ALLREDUCE_FN(self._allreduce)
        self._a2a = ALLTOALLV_FN(self._alltoallv)
        self.ops = CommOpsC(user=None, allgather=self._ag,
                            allreduce_max_u64=self._ar, alltoallv=self._a2a)

    def allgather_bytes(self, data: bytes) -> list:
        import torch
        n = len(data)
        t = torch.from_numpy(np.frombuffer(data, np.uint8).copy()) if n \
            else torch.zeros(1, dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [bytes(o.numpy()[:n]) for o in outs]

    def allreduce_max(self, vals: np.ndarray) -> np.ndarray:
        import torch
        t = torch.from_numpy(vals.astype(np.int64))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t.numpy().astype(np.uint64)

    def _allgather(self, user, send, recv, nbytes):
        try:
            data = C.string_at(send, nbytes) if nbytes else b""
            parts = self.allgather_bytes(data)
            if nbytes:
                C.memmove(recv, b"".join(parts), nbytes * self.world)
            return 0
        except Exception:  # never raise through the C frame
            traceback.print_exc(file=sys.stderr)
            return 1

    def _alltoallv(self, user, send, send_bytes, recv, recv_bytes):
        try:
            import torch
            sb = [int(send_bytes[q]) for q in range(self.world)]
            rb = [int(recv_bytes[q]) for q in range(self.world)]

            def view(addr, n):
                if n == 0:
                    return torch.empty(0, dtype=torch.uint8)
                return torch.from_numpy(np.ctypeslib.as_array(
                    (C.c_uint8 * n).from_address(addr)))
            self.dist.all_to_all_single(view(recv, sum(rb)), view(send, sum(sb)),
                                        rb, sb, group=self.group)
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1

    def _allreduce(self, user, buf, count):
        try:
            if count == 0:
                self.allreduce_max(np.zeros(1, np.uint64))
                return 0
            arr = np.ctypeslib.as_array((C.c_uint64 * count).from_address(buf))
            arr[:] = self.allreduce_max(arr.copy())
            return 0
        except Exception:
            traceback.print_exc(file=sys.stderr)
            return 1


def rccl_unique_id() -> bytes:
    L = lib()
    buf = (C.c_uint8 * 128)()
    _check(L.vp_comm_unique_id(buf), "vp_comm_unique_id", L)
    return bytes(buf)


def set_mode(nf, mode: str):
    """Dictionary placement (vp_shard_mode): "replicated" (every rank holds
    every key) or "owner" (keys sharded by flow hash, LAN lookups of other
    ranks' keys through an all-to-all)."""
    _check(nf.L.vp_shard_mode(nf.h, MODES[mode]), "vp_shard_mode", nf.L)


def attach_rccl(nf, rank: int, world: int, group=None, mode: str = "replicated"):
    """RCCL communicator for `nf` (collective over the torch.distributed
    group): rank 0's id is broadcast with torch.distributed."""
    import torch.distributed as dist
    obj = [rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    buf = (C.c_uint8 * 128).from_buffer_copy(obj[0])
    _check(nf.L.vp_attach_rccl(nf.h, buf, world, rank), "vp_attach_rccl", nf.L)
    set_mode(nf, mode)


def attach_torch(nf, rank: int, world: int, group=None,
                 mode: str = "replicated") -> TorchComm:
    """Host-callback communicator over torch.distributed; keep the returned
    object alive as long as `nf`."""
    comm = TorchComm(group)
    _check(nf.L.vp_attach_comm(nf.h, C.byref(comm.ops), world, rank),
           "vp_attach_comm", nf.L)
    nf._comm = comm
    set_mode(nf, mode)
    return comm
