"""ctypes binding to the ORACLE (oracle/liborc.so, oracle/_ref/liborc_ref.so).

Test infrastructure only: the checker the HIP path is compared against. The
product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_DIR = os.path.join(ROOT, "oracle")
MAX_DEV = 32


class NatCfg(C.Structure):
    _fields_ = [("wan_device", C.c_uint16), ("start_port", C.c_uint16),
                ("external_addr", C.c_uint32), ("expiration_time", C.c_uint32),
                ("max_flows", C.c_uint32), ("n_devices", C.c_uint16),
                ("device_macs", (C.c_uint8 * 6) * MAX_DEV),
                ("endpoint_macs", (C.c_uint8 * 6) * MAX_DEV)]


class BridgeCfg(C.Structure):
    _fields_ = [("expiration_time", C.c_uint32), ("dyn_capacity", C.c_uint32),
                ("n_devices", C.c_uint16), ("n_static", C.c_uint32),
                ("static_macs", C.c_void_p), ("static_from", C.c_void_p),
                ("static_to", C.c_void_p)]


class LbCfg(C.Structure):
    _fields_ = [("flow_capacity", C.c_uint32),
                ("flow_expiration_time", C.c_uint32),
                ("backend_capacity", C.c_uint32), ("cht_height", C.c_uint32),
                ("backend_expiration_time", C.c_uint32),
                ("wan_device", C.c_uint16), ("n_devices", C.c_uint16),
                ("device_macs", (C.c_uint8 * 6) * MAX_DEV)]


class FwCfg(C.Structure):
    _fields_ = [("wan_device", C.c_uint16), ("expiration_time", C.c_uint32),
                ("max_flows", C.c_uint32), ("n_devices", C.c_uint16),
                ("device_macs", (C.c_uint8 * 6) * MAX_DEV),
                ("endpoint_macs", (C.c_uint8 * 6) * MAX_DEV)]


class PolCfg(C.Structure):
    _fields_ = [("lan_device", C.c_uint16), ("wan_device", C.c_uint16),
                ("rate", C.c_uint64), ("burst", C.c_uint64),
                ("dyn_capacity", C.c_uint32), ("n_devices", C.c_uint16)]


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


# ref: False = the restatement (portable build, the checker); True = the
# reference's own libVig (oracle/_ref, this container only); "native" = the
# restatement built -O3 -march=native with the hardware crc32 instruction on
# the host that runs it (the CPU baseline, as the reference is built).
_PATHS = {False: "liborc.so", True: os.path.join("_ref", "liborc_ref.so"),
          "native": "liborc_native.so"}
_TARGETS = {False: "all", True: "ref", "native": "native"}


def build(ref=False) -> str:
    subprocess.run(["make", "-s", "-C", ORC_DIR, _TARGETS[ref]], check=True)
    return os.path.join(ORC_DIR, _PATHS[ref])


_LIBS = {}


def lib(ref=False):
    if ref in _LIBS:
        return _LIBS[ref]
    path = os.path.join(ORC_DIR, _PATHS[ref])
    if ref == "native" or not os.path.exists(path):
        build(ref)
    L = C.CDLL(path)
    L.orc_nat_create.restype = C.c_void_p
    L.orc_nat_create.argtypes = [C.POINTER(NatCfg)]
    L.orc_bridge_create.restype = C.c_void_p
    L.orc_bridge_create.argtypes = [C.POINTER(BridgeCfg)]
    L.orc_lb_create.restype = C.c_void_p
    L.orc_lb_create.argtypes = [C.POINTER(LbCfg)]
    L.orc_fw_create.restype = C.c_void_p
    L.orc_fw_create.argtypes = [C.POINTER(FwCfg)]
    L.orc_fw_dump.argtypes = [C.c_void_p] * 5
    L.orc_fw_flowid_hash.restype = C.c_uint32
    L.orc_fw_flowid_hash.argtypes = [C.c_uint16, C.c_uint16, C.c_uint32,
                                     C.c_uint32, C.c_uint8]
    L.orc_pol_create.restype = C.c_void_p
    L.orc_pol_create.argtypes = [C.POINTER(PolCfg)]
    L.orc_pol_dump.argtypes = [C.c_void_p] * 6
    L.orc_destroy.argtypes = [C.c_void_p]
    L.orc_process.restype = C.c_int
    L.orc_process.argtypes = [C.c_void_p, C.c_uint16, C.c_void_p, C.c_uint16,
                              C.c_uint32, C.c_int64]
    L.orc_run.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                          C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_digest.restype = C.c_uint64
    L.orc_digest.argtypes = [C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p,
                             C.c_void_p]
    L.orc_crc32c_u32.restype = C.c_uint32
    L.orc_crc32c_u32.argtypes = [C.c_uint32, C.c_uint32]
    L.orc_flowid_hash.restype = C.c_uint32
    L.orc_flowid_hash.argtypes = [C.c_uint16, C.c_uint16, C.c_uint32,
                                  C.c_uint32, C.c_uint16, C.c_uint8]
    L.orc_ether_hash.restype = C.c_uint32
    L.orc_ether_hash.argtypes = [C.c_char_p]
    L.orc_impl_name.restype = C.c_char_p
    L.orc_nat_flow_count.restype = C.c_uint32
    L.orc_nat_flow_count.argtypes = [C.c_void_p]
    L.orc_nat_dump.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_bridge_dump.argtypes = [C.c_void_p] * 5
    L.orc_lb_dump.argtypes = [C.c_void_p] * 10
    L.orc_test_dchain.restype = C.c_int
    L.orc_test_dchain.argtypes = [C.c_int, C.c_uint32] + [C.c_void_p] * 9
    L.orc_test_map.restype = C.c_int
    L.orc_test_map.argtypes = [C.c_uint, C.c_uint32, C.c_uint32] + \
        [C.c_void_p] * 4
    L.orc_test_cht.restype = C.c_int
    L.orc_test_cht.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                               C.c_uint32, C.c_void_p, C.c_void_p]
    _LIBS[ref] = L
    return L


def _macs(dst, macs):
    for d, m in enumerate(macs):
        for i in range(6):
            dst[d][i] = m[i]


def nat_cfg(wan=1, start_port=0, ext_ip=0, expire_us=60_000_000,
            max_flows=65536, device_macs=(), endpoint_macs=(), n_devices=2):
    c = NatCfg()
    c.wan_device, c.start_port, c.external_addr = wan, start_port, ext_ip
    c.expiration_time, c.max_flows, c.n_devices = expire_us, max_flows, n_devices
    _macs(c.device_macs, device_macs)
    _macs(c.endpoint_macs, endpoint_macs)
    return c


def fw_cfg(wan=1, expire_us=60_000_000, max_flows=65536, device_macs=(),
           endpoint_macs=(), n_devices=2):
    c = FwCfg()
    c.wan_device, c.expiration_time = wan, expire_us
    c.max_flows, c.n_devices = max_flows, n_devices
    _macs(c.device_macs, device_macs)
    _macs(c.endpoint_macs, endpoint_macs)
    return c


def pol_cfg(lan=1, wan=0, rate=375_000_000, burst=3_750_000_000,
            capacity=65536, n_devices=2):
    """vigpol defaults of vigpol/Makefile:5 (NF_ARGS)."""
    return PolCfg(lan, wan, rate, burst, capacity, n_devices)


class Oracle:
    """One NF instance in the oracle: 'nat' | 'bridge' | 'lb' | 'fw' | 'pol'."""

    def __init__(self, kind: str, cfg, ref: bool = False, statics=None):
        self.L = lib(ref)
        self.kind = kind
        self._keep = []
        if kind == "nat":
            self.h = self.L.orc_nat_create(C.byref(cfg))
        elif kind == "bridge":
            if statics:
                macs = np.frombuffer(b"".join(m for m, _, _ in statics),
                                     np.uint8).copy()
                fr = np.array([f for _, f, _ in statics], np.int32)
                to = np.array([t for _, _, t in statics], np.int32)
                self._keep += [macs, fr, to]
                cfg.n_static = len(statics)
                cfg.static_macs, cfg.static_from, cfg.static_to = \
                    macs.ctypes.data, fr.ctypes.data, to.ctypes.data
            self.h = self.L.orc_bridge_create(C.byref(cfg))
        elif kind == "lb":
            self.h = self.L.orc_lb_create(C.byref(cfg))
        elif kind == "fw":
            self.h = self.L.orc_fw_create(C.byref(cfg))
        elif kind == "pol":
            self.h = self.L.orc_pol_create(C.byref(cfg))
        else:
            raise ValueError(kind)
        if not self.h:
            raise ValueError("oracle rejected the configuration")

    def close(self):
        if self.h:
            self.L.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, frames, lens, in_dev, now, slot):
        """Mutates `frames` in place; returns out_dev (u16)."""
        n = lens.shape[0]
        out = np.zeros(n, np.uint16)
        lens = np.ascontiguousarray(lens, np.uint16)
        in_dev = np.ascontiguousarray(in_dev, np.uint16)
        now = np.ascontiguousarray(now, np.int64)
        assert frames.dtype == np.uint8 and frames.flags.c_contiguous
        assert frames.size == n * slot
        self.L.orc_run(self.h, n, _ptr(in_dev), _ptr(frames), slot, _ptr(lens),
                       _ptr(now), _ptr(out))
        return out

    def process(self, device, frame: bytearray, length=None, cap=None, now=0):
        buf = (C.c_uint8 * len(frame)).from_buffer(frame)
        return self.L.orc_process(self.h, device, buf,
                                  len(frame) if length is None else length,
                                  len(frame) if cap is None else cap, now)

    def nat_dump(self, max_flows):
        alloc = np.zeros(max_flows, np.uint8)
        ts = np.zeros(max_flows, np.int64)
        keys = np.zeros(max_flows * 16, np.uint8)
        self.L.orc_nat_dump(self.h, _ptr(alloc), _ptr(ts), _ptr(keys))
        return alloc, ts, keys.reshape(max_flows, 16)

    def fw_dump(self, max_flows):
        alloc = np.zeros(max_flows, np.uint8)
        ts = np.zeros(max_flows, np.int64)
        keys = np.zeros(max_flows * 16, np.uint8)
        dev = np.zeros(max_flows, np.uint32)
        self.L.orc_fw_dump(self.h, _ptr(alloc), _ptr(ts), _ptr(keys), _ptr(dev))
        return alloc, ts, keys.reshape(max_flows, 16), dev

    def pol_dump(self, cap):
        alloc = np.zeros(cap, np.uint8)
        ts = np.zeros(cap, np.int64)
        keys = np.zeros(cap, np.uint32)
        size = np.zeros(cap, np.uint64)
        btime = np.zeros(cap, np.int64)
        self.L.orc_pol_dump(self.h, _ptr(alloc), _ptr(ts), _ptr(keys),
                            _ptr(size), _ptr(btime))
        return alloc, ts, keys, size, btime

    def bridge_dump(self, cap):
        alloc = np.zeros(cap, np.uint8)
        ts = np.zeros(cap, np.int64)
        macs = np.zeros(cap * 6, np.uint8)
        port = np.zeros(cap, np.uint16)
        self.L.orc_bridge_dump(self.h, _ptr(alloc), _ptr(ts), _ptr(macs),
                               _ptr(port))
        return alloc, ts, macs.reshape(cap, 6), port

    def lb_dump(self, flow_cap, backend_cap):
        """(flow alloc, ts, keys[16], backend id), (backend alloc, ts, ip,
        mac[6], nic)."""
        fa = np.zeros(flow_cap, np.uint8)
        ft = np.zeros(flow_cap, np.int64)
        fk = np.zeros(flow_cap * 16, np.uint8)
        fb = np.zeros(flow_cap, np.uint32)
        ba = np.zeros(backend_cap, np.uint8)
        bt = np.zeros(backend_cap, np.int64)
        bi = np.zeros(backend_cap, np.uint32)
        bm = np.zeros(backend_cap * 6, np.uint8)
        bn = np.zeros(backend_cap, np.uint16)
        self.L.orc_lb_dump(self.h, *[_ptr(x) for x in
                                     (fa, ft, fk, fb, ba, bt, bi, bm, bn)])
        return ((fa, ft, fk.reshape(flow_cap, 16), fb),
                (ba, bt, bi, bm.reshape(backend_cap, 6), bn))


def digest(frames, slot, lens, out_dev, ref=False) -> int:
    L = lib(ref)
    return L.orc_digest(lens.shape[0], _ptr(frames), slot,
                        _ptr(np.ascontiguousarray(lens, np.uint16)),
                        _ptr(np.ascontiguousarray(out_dev, np.uint16)))
