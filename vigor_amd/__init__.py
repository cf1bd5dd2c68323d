"""vigor_amd — MI355X-native Vigor per-packet path (host-side mirror).

Thin ctypes layer over libvigpath.so (include/vigpath.h), the C-ABI the HIP
kernels sit behind. There is no CPU fallback: if the library or a GPU is
missing, every entry point raises. The CPU restatement used to check results
lives in oracle/ and is test infrastructure only.
"""
from __future__ import annotations

import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# VIGPATH_LIB: another build of the same ABI, for diagnostics (A/B builds)
LIB_PATH = os.environ.get("VIGPATH_LIB") or os.path.join(PKG, "libvigpath.so")
MAX_DEV = 32
FLOOD_FRAME = 0xFFFF

VP_OK, VP_EINVAL, VP_ENOMEM, VP_EIO, VP_ENOTSUP = 0, -22, -12, -5, -95
VP_ESTATE = -71
_ERR = {VP_EINVAL: "EINVAL", VP_ENOMEM: "ENOMEM", VP_EIO: "EIO (HIP)",
        VP_ESTATE: "ESTATE (device protocol)",
        VP_ENOTSUP: "ENOTSUP"}


class VigpathError(RuntimeError):
    def __init__(self, rc: int, what: str, detail: str = ""):
        super().__init__(f"{what}: {_ERR.get(rc, rc)}" + (f" [{detail}]" if detail else ""))
        self.rc = rc
        self.detail = detail


class TableStatsC(C.Structure):
    """vp_table_stats (include/vigpath.h)."""
    _fields_ = [("live", C.c_uint64), ("shard_live", C.c_uint64),
                ("tombstones", C.c_uint64), ("buckets", C.c_uint64),
                ("rebuilds", C.c_uint64), ("layout", C.c_uint32),
                ("pad", C.c_uint32)]


MacTable = (C.c_uint8 * 6) * MAX_DEV


class NatConfigC(C.Structure):
    """vp_nat_config (vignat/nat_config.h:5-31)."""
    _fields_ = [("wan_device", C.c_uint16), ("lan_main_device", C.c_uint16),
                ("start_port", C.c_uint16), ("external_addr", C.c_uint32),
                ("expiration_time", C.c_uint32), ("max_flows", C.c_uint32),
                ("n_devices", C.c_uint16), ("device_macs", MacTable),
                ("endpoint_macs", MacTable)]


class BridgeRuleC(C.Structure):
    _fields_ = [("mac", C.c_uint8 * 6), ("device_from", C.c_int32),
                ("device_to", C.c_int32)]


class BridgeConfigC(C.Structure):
    """vp_bridge_config (vigbridge/bridge_config.h:8-18)."""
    _fields_ = [("expiration_time", C.c_uint32), ("dyn_capacity", C.c_uint32),
                ("n_devices", C.c_uint16), ("n_static", C.c_uint32),
                ("static_rules", C.POINTER(BridgeRuleC))]


class LbConfigC(C.Structure):
    """vp_lb_config (viglb/lb_config.h:8-38)."""
    _fields_ = [("flow_capacity", C.c_uint32),
                ("flow_expiration_time", C.c_uint32),
                ("backend_capacity", C.c_uint32), ("cht_height", C.c_uint32),
                ("backend_expiration_time", C.c_uint32),
                ("wan_device", C.c_uint16), ("n_devices", C.c_uint16),
                ("device_macs", MacTable)]


class FwConfigC(C.Structure):
    """vp_fw_config (vigfw/fw_config.h:9-24)."""
    _fields_ = [("wan_device", C.c_uint16), ("expiration_time", C.c_uint32),
                ("max_flows", C.c_uint32), ("n_devices", C.c_uint16),
                ("device_macs", MacTable), ("endpoint_macs", MacTable)]


class PolConfigC(C.Structure):
    """vp_pol_config (vigpol/policer_config.h:8-24)."""
    _fields_ = [("lan_device", C.c_uint16), ("wan_device", C.c_uint16),
                ("rate", C.c_uint64), ("burst", C.c_uint64),
                ("dyn_capacity", C.c_uint32), ("n_devices", C.c_uint16)]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                           C.c_size_t)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p,
                           C.POINTER(C.c_size_t), C.c_void_p,
                           C.POINTER(C.c_size_t))

SHARD_REPLICATED, SHARD_OWNER = 0, 1  # vp_shard_mode


class CommOpsC(C.Structure):
    """vp_comm_ops: host-memory collectives supplied by the caller."""
    _fields_ = [("user", C.c_void_p), ("allgather", ALLGATHER_FN),
                ("allreduce_max_u64", ALLREDUCE_FN),
                ("alltoallv", ALLTOALLV_FN)]


class DevBatchC(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("slot", C.c_uint32), ("n", C.c_uint32),
                ("len", C.c_void_p), ("in_dev", C.c_void_p),
                ("now", C.c_void_p), ("now0", C.c_int64),
                ("now_step", C.c_int64), ("out_dev", C.c_void_p), ("in_port", C.c_uint32)]


class MbufBatchC(C.Structure):
    """vp_mbuf_batch (include/vigpath.h): a DPDK-shaped host batch."""
    _fields_ = [("n", C.c_uint32), ("frames", C.c_void_p), ("len", C.c_void_p),
                ("in_dev", C.c_void_p), ("now", C.c_void_p), ("now0", C.c_int64),
                ("now_step", C.c_int64), ("out_dev", C.c_void_p)]


# every symbol include/vigpath.h declares
EXPORTS = ["vp_nat_create", "vp_bridge_create", "vp_lb_create", "vp_fw_create",
           "vp_pol_create", "vp_pol_dump", "vp_destroy", "vp_process_device", "vp_process_batch",
           "vp_process_host", "vp_process_host_batch", "vp_nat_dump", "vp_bridge_dump", "vp_lb_dump",
           "vp_fw_dump", "vp_comm_unique_id", "vp_attach_rccl",
           "vp_attach_comm", "vp_shard_mode", "vp_sync_state", "vp_live_count",
           "vp_kernel_timing", "vp_last_kernel_ms", "vp_version", "vp_table_stats_get",
           "vp_last_error", "vp_register_host", "vp_unregister_host", "vp_process_mbufs",
           "vp_last_stage_ms", "vp_stage_ms", "vp_comm_abort", "vp_probe_slots",
           "vp_probe_slots_w", "vp_process_one", "vp_last_kernel"]

_libs = {}


def lib(path: str | None = None):
    """Load libvigpath.so (or, for diagnostics, another build of the same
    ABI); raises if it has not been built."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
    L = C.CDLL(path)
    L.vp_version.restype = C.c_char_p
    for name in ("vp_nat_create", "vp_bridge_create", "vp_lb_create",
                 "vp_fw_create"):
        getattr(L, name).restype = C.c_int
    L.vp_fw_create.argtypes = [C.POINTER(FwConfigC), C.c_int,
                               C.POINTER(C.c_void_p)]
    L.vp_fw_dump.argtypes = [C.c_void_p] * 5
    L.vp_fw_dump.restype = C.c_int
    L.vp_pol_create.restype = C.c_int
    L.vp_pol_create.argtypes = [C.POINTER(PolConfigC), C.c_int,
                                C.POINTER(C.c_void_p)]
    L.vp_pol_dump.argtypes = [C.c_void_p] * 6
    L.vp_pol_dump.restype = C.c_int
    L.vp_nat_create.argtypes = [C.POINTER(NatConfigC), C.c_int,
                                C.POINTER(C.c_void_p)]
    L.vp_bridge_create.argtypes = [C.POINTER(BridgeConfigC), C.c_int,
                                   C.POINTER(C.c_void_p)]
    L.vp_lb_create.argtypes = [C.POINTER(LbConfigC), C.c_int,
                               C.POINTER(C.c_void_p)]
    L.vp_destroy.argtypes = [C.c_void_p]
    L.vp_destroy.restype = None
    L.vp_process_device.argtypes = [C.c_void_p, C.POINTER(DevBatchC),
                                    C.c_void_p]
    L.vp_process_device.restype = C.c_int
    L.vp_process_host.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p,
                                  C.c_void_p, C.c_uint32, C.c_void_p,
                                  C.c_void_p, C.c_void_p]
    L.vp_process_host.restype = C.c_int
    L.vp_process_host_batch.argtypes = [C.c_void_p, C.POINTER(DevBatchC)]
    L.vp_process_host_batch.restype = C.c_int
    L.vp_process_batch.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p,
                                   C.POINTER(C.c_void_p), C.c_void_p,
                                   C.c_void_p, C.c_void_p]
    L.vp_process_batch.restype = C.c_int
    L.vp_process_one.argtypes = [C.c_void_p, C.c_uint16, C.c_void_p, C.c_uint16,
                                 C.c_int64, C.POINTER(C.c_uint16)]
    L.vp_process_one.restype = C.c_int
    L.vp_process_mbufs.argtypes = [C.c_void_p, C.POINTER(MbufBatchC)]
    L.vp_process_mbufs.restype = C.c_int
    L.vp_register_host.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.vp_register_host.restype = C.c_int
    L.vp_unregister_host.argtypes = [C.c_void_p, C.c_void_p]
    L.vp_unregister_host.restype = C.c_int
    L.vp_nat_dump.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.vp_nat_dump.restype = C.c_int
    L.vp_bridge_dump.argtypes = [C.c_void_p] * 5
    L.vp_bridge_dump.restype = C.c_int
    L.vp_lb_dump.argtypes = [C.c_void_p] * 10
    L.vp_lb_dump.restype = C.c_int
    L.vp_comm_unique_id.argtypes = [C.c_void_p]
    L.vp_comm_unique_id.restype = C.c_int
    L.vp_attach_rccl.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    L.vp_attach_rccl.restype = C.c_int
    L.vp_attach_comm.argtypes = [C.c_void_p, C.POINTER(CommOpsC), C.c_int,
                                 C.c_int]
    L.vp_attach_comm.restype = C.c_int
    L.vp_shard_mode.argtypes = [C.c_void_p, C.c_int]
    L.vp_shard_mode.restype = C.c_int
    L.vp_sync_state.argtypes = [C.c_void_p]
    L.vp_sync_state.restype = C.c_int
    L.vp_comm_abort.argtypes = [C.c_void_p]
    L.vp_comm_abort.restype = C.c_int
    L.vp_probe_slots.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                 C.POINTER(C.c_float)]
    L.vp_probe_slots.restype = C.c_int
    L.vp_probe_slots_w.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                   C.POINTER(C.c_float)]
    L.vp_probe_slots_w.restype = C.c_int
    L.vp_live_count.argtypes = [C.c_void_p]
    L.vp_live_count.restype = C.c_int64
    L.vp_last_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_float),
                                    C.POINTER(C.c_int)]
    L.vp_last_kernel_ms.restype = C.c_int
    L.vp_last_stage_ms.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    L.vp_last_stage_ms.restype = C.c_int
    L.vp_stage_ms.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]
    L.vp_stage_ms.restype = C.c_int
    L.vp_last_kernel.argtypes = [C.c_void_p]
    L.vp_last_kernel.restype = C.c_char_p
    L.vp_kernel_timing.argtypes = [C.c_void_p, C.c_int]
    L.vp_kernel_timing.restype = C.c_int
    L.vp_table_stats_get.argtypes = [C.c_void_p, C.c_int, C.POINTER(TableStatsC)]
    L.vp_table_stats_get.restype = C.c_int
    L.vp_last_error.argtypes = []
    L.vp_last_error.restype = C.c_char_p
    _libs[path] = L
    return L


_DETAILED = (-5, -12, -71)  # VP_EIO, VP_ENOMEM, VP_ESTATE record vp_last_error()


def _check(rc: int, what: str, L=None):
    """Raise VigpathError for a failing vp_* return code. `L` is the library
    that made the call (the first one loaded if omitted). Only the codes that
    record a reason (VP_EIO / VP_ENOMEM / VP_ESTATE) carry vp_last_error():
    the others record nothing, and the thread's text would belong to an
    earlier failure."""
    if rc != 0:
        detail = ""
        if L is None:
            L = next(iter(_libs.values()), None)
        if L is not None and rc in _DETAILED:
            detail = (L.vp_last_error() or b"").decode(errors="replace")
        raise VigpathError(rc, what, detail)


from .nf import Bridge, Fw, Lb, Nat, NfBase, Pol  # noqa: E402,F401
from .config import (bridge_config_from_args, fw_config_from_args,  # noqa
                     lb_config_from_args, nat_config_from_args,
                     pol_config_from_args)
