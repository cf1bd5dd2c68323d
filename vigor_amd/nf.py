"""NF instances on the GPU: the batch form of the reference operator
`int nf_process(uint16_t device, uint8_t *buffer, uint16_t len, vigor_time_t
now)` (nf.h:13), driven the way nf.c's loop drives it (nf.c:150-176).

`process_device` takes torch tensors already in HBM; `process_host` takes
numpy arrays and stages them through pinned memory (hipMemcpyAsync);
`process` is the per-packet nf_process equivalent (one-packet batch).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import (BridgeConfigC, DevBatchC, FwConfigC, LbConfigC, MbufBatchC,
               NatConfigC, PolConfigC, TableStatsC, _check, lib)


def _dptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


class NfBase:
    kind = "?"

    def __init__(self, libpath=None):
        self.h = C.c_void_p()
        self.L = lib(libpath)

    def _ck(self, rc: int, what: str):
        _check(rc, what, self.L)  # vp_last_error() of this instance's library

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            self.L.vp_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------- device --
    def process_device(self, frames, lens, in_dev, out, slot: int, now=None,
                       now0: int = 0, now_step: int = 0, stream=None):
        """frames: uint8 CUDA tensor of n*slot bytes (mutated in place);
        lens/in_dev/out: int16/uint16-sized CUDA tensors of n (in_dev an int:
        every packet on that port, vp_dev_batch.in_port); now: int64 CUDA
        tensor of n, or None for now0 + i*now_step."""
        n = lens.numel()
        assert frames.numel() == n * slot and frames.is_cuda
        port = isinstance(in_dev, int)
        b = DevBatchC(frames=frames.data_ptr(), slot=slot, n=n,
                      len=lens.data_ptr(), in_dev=None if port else in_dev.data_ptr(),
                      now=now.data_ptr() if now is not None else None,
                      now0=now0, now_step=now_step, out_dev=out.data_ptr(),
                      in_port=in_dev if port else 0)
        s = C.c_void_p(stream.cuda_stream) if stream is not None else None
        self._ck(self.L.vp_process_device(self.h, C.byref(b), s),
               "vp_process_device")

    def device_step(self, frames, lens, in_dev, out, slot: int):
        """A prepared vp_process_device call over fixed device buffers with
        affine time: returns f(now0, now_step). The batch descriptor and its
        pointers are built once (a C caller's per-burst cost), so a loop of
        calls pays only the C-ABI call itself. The callable keeps the tensors
        alive: the descriptor holds their raw device pointers. in_dev: as for
        process_device (an int: the burst's one port)."""
        n = lens.numel()
        assert frames.numel() == n * slot and frames.is_cuda
        port = isinstance(in_dev, int)
        b = DevBatchC(frames=frames.data_ptr(), slot=slot, n=n,
                      len=lens.data_ptr(), in_dev=None if port else in_dev.data_ptr(),
                      now=None, now0=0, now_step=0, out_dev=out.data_ptr(),
                      in_port=in_dev if port else 0)
        ref, fn, h, L = C.byref(b), self.L.vp_process_device, self.h, self.L
        keep = (frames, lens, in_dev, out)

        def step(now0: int, now_step: int):
            b.now0, b.now_step = now0, now_step
            rc = fn(h, ref, None)
            if rc:
                _check(rc, "vp_process_device", L)
        step.tensors = keep
        return step

    def device_steps(self, frames_list, lens, in_dev, out, slot: int):
        """The loop of device_step calls in C (host/steps.c,
        libvp_steps.so): one vp_process_device per buffer of frames_list, in
        order, as nf.c's loop makes one call per burst. Returns
        f(now0s, now_step) that runs them all (now0s: each batch's first time
        stamp). Measurement infrastructure: no interpreter between the
        calls."""
        import os
        n = lens.numel()
        port = isinstance(in_dev, int)
        arr = (DevBatchC * len(frames_list))()
        for k, fr in enumerate(frames_list):
            assert fr.numel() == n * slot and fr.is_cuda
            arr[k] = DevBatchC(frames=fr.data_ptr(), slot=slot, n=n, len=lens.data_ptr(),
                               in_dev=None if port else in_dev.data_ptr(), now=None,
                               now0=0, now_step=0, out_dev=out.data_ptr(),
                               in_port=in_dev if port else 0)
        S = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(self.L._name)),
                                "libvp_steps.so"))
        S.vp_steps_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int,
                                      C.POINTER(C.c_int)]
        keep = (list(frames_list), lens, in_dev, out)

        def run(now0s, now_step: int):
            assert len(now0s) == len(arr)
            for k, t0 in enumerate(now0s):
                arr[k].now0, arr[k].now_step = t0, now_step
            done = C.c_int()
            rc = S.vp_steps_device(self.h, C.cast(arr, C.c_void_p), len(arr),
                                   C.byref(done))
            if rc:
                _check(rc, "vp_process_device (call %d)" % done.value, self.L)
        run.tensors = keep
        return run

    def sync_state(self):
        """Multi-GPU: merge the ranks' timestamps (collective)."""
        self._ck(self.L.vp_sync_state(self.h), "vp_sync_state")

    def kernel_timing(self, on: bool = True):
        """Bracket every classification kernel launch with HIP events
        (vp_kernel_timing; off by default: the events cost a step about 6 us),
        so that last_kernel_ms() reports its time."""
        self._ck(self.L.vp_kernel_timing(self.h, 1 if on else 0), "vp_kernel_timing")

    def last_kernel_ms(self):
        if not hasattr(self, "_kms"):  # (built once: called every batch)
            ms, k = C.c_float(), C.c_int()
            self._kms = (ms, k, C.byref(ms), C.byref(k))
        ms, k, rms, rk = self._kms
        self._ck(self.L.vp_last_kernel_ms(self.h, rms, rk), "vp_last_kernel_ms")
        return ms.value, k.value

    def last_kernel(self) -> str:
        """vp_last_kernel: the tile kernel the last call launched ("" if none)."""
        return (self.L.vp_last_kernel(self.h) or b"").decode()

    STAGES = ("pass1", "offsets", "a2a_keys", "probe", "a2a_answers", "pass2", "fold",
              "pipeline")

    def last_stage_ms(self) -> dict:
        """vp_stage_ms: owner mode with kernel timing on, the last call's
        phase-A stage times (ms) by stage name ({} if none); the chunked
        pipeline reports "pipeline" (its overlapped chunks) and "fold"
        only."""
        cap = len(self.STAGES)
        ms, k = (C.c_float * cap)(), C.c_int()
        self._ck(self.L.vp_stage_ms(self.h, ms, cap, C.byref(k)), "vp_stage_ms")
        d = {self.STAGES[i]: ms[i] for i in range(min(cap, k.value))}
        if d.get("pipeline"):
            d = {"pipeline": d["pipeline"], "fold": d["fold"]}
        return d

    def table_stats(self, table: int = 0) -> dict:
        """vp_table_stats_get: live / shard_live / tombstones / buckets /
        rebuilds / layout of table 0 (flows) or 1 (viglb backends)."""
        st = TableStatsC()
        self._ck(self.L.vp_table_stats_get(self.h, table, C.byref(st)), "vp_table_stats_get")
        return {k: int(getattr(st, k)) for k, _ in TableStatsC._fields_ if k != "pad"}

    def live_count(self) -> int:
        v = self.L.vp_live_count(self.h)
        if v < 0:
            self._ck(int(v), "vp_live_count")
        return int(v)

    # ----------------------------------------------------------- host --
    def process_host(self, frames: np.ndarray, lens, in_dev, now, slot: int):
        """Contiguous host batch; frames (u8, n*slot) rewritten in place.
        Returns out_dev (u16)."""
        n = int(lens.shape[0])
        assert frames.dtype == np.uint8 and frames.flags.c_contiguous
        assert frames.size == n * slot
        lens = np.ascontiguousarray(lens, np.uint16)
        in_dev = np.ascontiguousarray(in_dev, np.uint16)
        now = np.ascontiguousarray(now, np.int64)
        out = np.zeros(n, np.uint16)
        P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.L.vp_process_host(self.h, n, P(in_dev), P(frames), slot,
                                     P(lens), P(now), P(out)),
               "vp_process_host")
        return out

    def process_host_batch(self, frames: np.ndarray, lens, in_dev, out, slot: int,
                           now=None, now0: int = 0, now_step: int = 0):
        """vp_process_host_batch: host numpy arrays (page-locked ones, e.g.
        torch.pin_memory() views, are DMA'd in place), rewritten in place;
        out (u16/i16, n) receives the out ports. now: int64 array, or None
        for now0 + i * now_step."""
        n = int(lens.shape[0])
        assert frames.dtype == np.uint8 and frames.flags.c_contiguous
        assert frames.size == n * slot and out.shape[0] == n
        for a in (lens, in_dev, out):
            assert a.flags.c_contiguous and a.itemsize == 2
        if now is not None:
            assert now.dtype == np.int64 and now.flags.c_contiguous
        b = DevBatchC(frames=frames.ctypes.data, slot=slot, n=n, len=lens.ctypes.data,
                      in_dev=in_dev.ctypes.data,
                      now=now.ctypes.data if now is not None else None,
                      now0=now0, now_step=now_step, out_dev=out.ctypes.data)
        self._ck(self.L.vp_process_host_batch(self.h, C.byref(b)), "vp_process_host_batch")

    def process_mbufs(self, bufs, in_dev, now):
        """Per-frame host buffers (bytearray each, mbuf-like), rewritten in
        place. Returns out_dev."""
        n = len(bufs)
        ptrs = (C.c_void_p * n)()
        arrs = []
        lens = np.zeros(n, np.uint16)
        for i, b in enumerate(bufs):
            a = (C.c_uint8 * len(b)).from_buffer(b)
            arrs.append(a)
            ptrs[i] = C.cast(a, C.c_void_p)
            lens[i] = len(b)
        in_dev = np.ascontiguousarray(in_dev, np.uint16)
        now = np.ascontiguousarray(now, np.int64)
        out = np.zeros(n, np.uint16)
        P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.L.vp_process_batch(self.h, n, P(in_dev), ptrs, P(lens),
                                      P(now), P(out)), "vp_process_batch")
        return out

    def register_host(self, arr: np.ndarray):
        """vp_register_host: the GPU reads and writes frames inside `arr`
        (e.g. an mbuf pool) in place from now on (vp_process_mbufs)."""
        assert arr.flags.c_contiguous
        self._ck(self.L.vp_register_host(self.h, C.c_void_p(arr.ctypes.data), arr.nbytes),
                 "vp_register_host")
        self._hostmaps = getattr(self, "_hostmaps", []) + [arr]

    def unregister_host(self, arr: np.ndarray):
        self._ck(self.L.vp_unregister_host(self.h, C.c_void_p(arr.ctypes.data)),
                 "vp_unregister_host")
        self._hostmaps = [a for a in getattr(self, "_hostmaps", []) if a is not arr]

    def process_mbuf_batch(self, ptrs: np.ndarray, lens, in_dev, out, now=None,
                           now0: int = 0, now_step: int = 0):
        """vp_process_mbufs: ptrs (u64, n) = each frame's host address (the
        mbuf data pointers of an rx burst), lens / in_dev (u16, n), out (u16,
        n) receives the out ports; now (i64, n) or None for affine time.
        Arrays in page-locked memory are DMA'd in place."""
        n = int(ptrs.shape[0])
        assert ptrs.dtype == np.uint64 and ptrs.flags.c_contiguous
        for a in (lens, in_dev, out):
            assert a.flags.c_contiguous and a.itemsize == 2 and a.shape[0] == n
        if now is not None:
            assert now.dtype == np.int64 and now.flags.c_contiguous
        b = MbufBatchC(n=n, frames=ptrs.ctypes.data, len=lens.ctypes.data,
                       in_dev=in_dev.ctypes.data,
                       now=now.ctypes.data if now is not None else None,
                       now0=now0, now_step=now_step, out_dev=out.ctypes.data)
        self._ck(self.L.vp_process_mbufs(self.h, C.byref(b)), "vp_process_mbufs")

    def mbuf_step(self, ptrs, lens, in_dev, out):
        """A prepared vp_process_mbufs call over fixed host arrays with affine
        time: returns f(now0, now_step) (the batch descriptor built once, as
        device_step)."""
        n = int(ptrs.shape[0])
        b = MbufBatchC(n=n, frames=ptrs.ctypes.data, len=lens.ctypes.data,
                       in_dev=in_dev.ctypes.data, now=None, now0=0, now_step=0,
                       out_dev=out.ctypes.data)
        ref, fn, h, L = C.byref(b), self.L.vp_process_mbufs, self.h, self.L

        def step(now0: int, now_step: int):
            b.now0, b.now_step = now0, now_step
            rc = fn(h, ref)
            if rc:
                _check(rc, "vp_process_mbufs", L)
        step.arrays = (ptrs, lens, in_dev, out)
        return step

    def process(self, device: int, buffer: bytearray, now: int) -> int:
        """nf_process for one packet (nf.h:13): vp_process_one (vignat on one
        GPU: the persistent kernel's mailbox, no launch per packet)."""
        a = (C.c_uint8 * len(buffer)).from_buffer(buffer)
        out = C.c_uint16(device)
        self._ck(self.L.vp_process_one(self.h, device, C.cast(a, C.c_void_p), len(buffer),
                                       now, C.byref(out)), "vp_process_one")
        return int(out.value)


class Nat(NfBase):
    kind = "nat"

    def __init__(self, cfg: NatConfigC, gpu: int = 0, libpath=None):
        super().__init__(libpath)
        self.cfg = cfg
        self._ck(self.L.vp_nat_create(C.byref(cfg), gpu, C.byref(self.h)),
               "vp_nat_create")

    def dump(self):
        n = self.cfg.max_flows
        alloc = np.zeros(n, np.uint8)
        ts = np.zeros(n, np.int64)
        keys = np.zeros(n * 16, np.uint8)
        P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.L.vp_nat_dump(self.h, P(alloc), P(ts), P(keys)),
               "vp_nat_dump")
        return alloc, ts, keys.reshape(n, 16)


class Bridge(NfBase):
    kind = "bridge"

    def __init__(self, cfg: BridgeConfigC, gpu: int = 0, libpath=None):
        super().__init__(libpath)
        self.cfg = cfg
        self._ck(self.L.vp_bridge_create(C.byref(cfg), gpu, C.byref(self.h)),
               "vp_bridge_create")

    def dump(self):
        """Dynamic table by index: alloc, ts, MAC (6 B), learned port."""
        n = self.cfg.dyn_capacity
        alloc = np.zeros(n, np.uint8)
        ts = np.zeros(n, np.int64)
        macs = np.zeros(n * 6, np.uint8)
        port = np.zeros(n, np.uint16)
        P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.L.vp_bridge_dump(self.h, P(alloc), P(ts), P(macs), P(port)),
               "vp_bridge_dump")
        return alloc, ts, macs.reshape(n, 6), port


class Lb(NfBase):
    kind = "lb"

    def __init__(self, cfg: LbConfigC, gpu: int = 0, libpath=None):
        super().__init__(libpath)
        self.cfg = cfg
        self._ck(self.L.vp_lb_create(C.byref(cfg), gpu, C.byref(self.h)),
               "vp_lb_create")

    def dump(self):
        """(flow alloc, ts, keys[16], backend id), (backend alloc, ts, ip,
        mac[6], nic) by index."""
        nf_, nb = self.cfg.flow_capacity, self.cfg.backend_capacity
        fa, ft = np.zeros(nf_, np.uint8), np.zeros(nf_, np.int64)
        fk, fb = np.zeros(nf_ * 16, np.uint8), np.zeros(nf_, np.uint32)
        ba, bt = np.zeros(nb, np.uint8), np.zeros(nb, np.int64)
        bi, bm = np.zeros(nb, np.uint32), np.zeros(nb * 6, np.uint8)
        bn = np.zeros(nb, np.uint16)
        self._ck(self.L.vp_lb_dump(self.h, *[C.c_void_p(x.ctypes.data) for x in
                                           (fa, ft, fk, fb, ba, bt, bi, bm, bn)]),
               "vp_lb_dump")
        return ((fa, ft, fk.reshape(nf_, 16), fb),
                (ba, bt, bi, bm.reshape(nb, 6), bn))


class Fw(NfBase):
    kind = "fw"

    def __init__(self, cfg: FwConfigC, gpu: int = 0, libpath=None):
        super().__init__(libpath)
        self.cfg = cfg
        self._ck(self.L.vp_fw_create(C.byref(cfg), gpu, C.byref(self.h)),
               "vp_fw_create")

    def dump(self):
        """By flow index: alloc, ts, FlowId bytes (16), int_devices."""
        n = self.cfg.max_flows
        alloc = np.zeros(n, np.uint8)
        ts = np.zeros(n, np.int64)
        keys = np.zeros(n * 16, np.uint8)
        dev = np.zeros(n, np.uint32)
        P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.L.vp_fw_dump(self.h, P(alloc), P(ts), P(keys), P(dev)),
               "vp_fw_dump")
        return alloc, ts, keys.reshape(n, 16), dev


class Pol(NfBase):
    """vigpol (vigpol/policer_main.c): per-destination token buckets on the
    WAN device; frames are never rewritten."""
    kind = "pol"

    def __init__(self, cfg: PolConfigC, gpu: int = 0, libpath=None):
        super().__init__(libpath)
        self.cfg = cfg
        self._ck(self.L.vp_pol_create(C.byref(cfg), gpu, C.byref(self.h)),
               "vp_pol_create")

    def dump(self):
        """By index: alloc, ts, dyn_keys (raw u32 address), bucket_size,
        bucket_time."""
        n = self.cfg.dyn_capacity
        alloc = np.zeros(n, np.uint8)
        ts = np.zeros(n, np.int64)
        keys = np.zeros(n, np.uint32)
        size = np.zeros(n, np.uint64)
        btime = np.zeros(n, np.int64)
        P = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.L.vp_pol_dump(self.h, P(alloc), P(ts), P(keys), P(size),
                                  P(btime)), "vp_pol_dump")
        return alloc, ts, keys, size, btime
