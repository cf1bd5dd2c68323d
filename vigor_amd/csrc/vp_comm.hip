// Comm transports (vp_comm.h) and the multi-GPU C-ABI entry points.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "vp_comm.h"
#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(comm)


static int nccl_fail(ncclResult_t e, const char *what) {
  state_fail("RCCL %s failed: %s", what, ncclGetErrorString(e));  // (the message)
  return VP_EIO;
}
#define VP_NCCL(call)                                  \
  do {                                                 \
    ncclResult_t e_ = (call);                          \
    if (e_ != ncclSuccess) return nccl_fail(e_, #call); \
  } while (0)

// RCCL on device buffers; host variants stage through a page-locked host
// buffer and a device buffer (a copy from pageable memory is staged by the
// runtime synchronously: the per-batch RankInfo gather spent ~30 us in
// its two copies).
struct RcclComm : Comm {
  ncclComm_t comm = nullptr;
  void *stage = nullptr;
  size_t stage_bytes = 0;
  uint8_t *hstage = nullptr;
  size_t hstage_bytes = 0;
  ~RcclComm() override {
    // (an aborted communicator is gone: ncclCommAbort freed it)
    if (comm && !aborted.load()) ncclCommDestroy(comm);
    if (stage) hipFree(stage);
    if (hstage) hipHostFree(hstage);
  }
  std::atomic<bool> aborted{false};
  int live() const {
    if (!aborted.load()) return 0;
    state_fail("RCCL communicator aborted (vp_comm_abort)");
    return VP_EIO;
  }
  int abort() override {
    bool was = false;
    if (!comm || !aborted.compare_exchange_strong(was, true)) return 0;
    VP_NCCL(ncclCommAbort(comm));
    return 0;
  }
  int reserve_host(size_t bytes) {
    if (bytes <= hstage_bytes) return 0;
    if (hstage) hipHostFree(hstage);
    hstage = nullptr;
    hstage_bytes = 0;
    VP_HIP(hipHostMalloc((void **)&hstage, bytes, hipHostMallocDefault));
    hstage_bytes = bytes;
    return 0;
  }
  int reserve(size_t bytes) {
    if (bytes <= stage_bytes) return 0;
    if (stage) hipFree(stage);
    stage = nullptr;
    stage_bytes = 0;
    VP_HIP(hipMalloc(&stage, bytes));
    stage_bytes = bytes;
    return 0;
  }
  int allgather_host(vp_ctx *c, const void *send, void *recv, size_t bytes) override {
    VP_TRY(live());
    VP_TRY(reserve(bytes * (n + 1)));
    VP_TRY(reserve_host(bytes * (n + 1)));
    uint8_t *s = static_cast<uint8_t *>(stage), *h = hstage;
    memcpy(h, send, bytes);
    VP_HIP(hipMemcpyAsync(s, h, bytes, hipMemcpyHostToDevice, c->stream));
    VP_NCCL(ncclAllGather(s, s + bytes, bytes, ncclUint8, comm, c->stream));
    VP_HIP(hipMemcpyAsync(h + bytes, s + bytes, bytes * n, hipMemcpyDeviceToHost,
                          c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    memcpy(recv, h + bytes, bytes * n);
    return 0;
  }
  int allgather_dev(vp_ctx *c, const void *send, void *recv, size_t bytes) override {
    VP_TRY(live());
    VP_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, comm, c->stream));
    return 0;
  }
  int allreduce_max_u64_dev(vp_ctx *c, uint64_t *buf, size_t count) override {
    VP_TRY(live());
    VP_NCCL(ncclAllReduce(buf, buf, count, ncclUint64, ncclMax, comm, c->stream));
    return 0;
  }
  // one grouped send/recv per peer: every pair of GPUs talks over its own
  // xGMI link at once
  int alltoallv_dev(vp_ctx *c, const void *send, const size_t *sbytes, void *recv,
                    const size_t *rbytes, bool skip_self, hipStream_t st) override {
    VP_TRY(live());
    if (!st) st = c->stream;
    const uint8_t *s = static_cast<const uint8_t *>(send);
    uint8_t *d = static_cast<uint8_t *>(recv);
    size_t so = 0, ro = 0;
    std::vector<size_t> soff(n), roff(n);
    for (int q = 0; q < n; q++) {
      soff[q] = so;
      roff[q] = ro;
      so += sbytes[q];
      ro += rbytes[q];
    }
    if (sbytes[r] != rbytes[r]) return VP_EINVAL;
    if (sbytes[r] && !skip_self)
      VP_HIP(hipMemcpyAsync(d + roff[r], s + soff[r], sbytes[r],
                            hipMemcpyDeviceToDevice, st));
    VP_NCCL(ncclGroupStart());
    for (int q = 0; q < n; q++) {
      if (q == r) continue;
      if (sbytes[q]) {
        ncclResult_t e = ncclSend(s + soff[q], sbytes[q], ncclUint8, q, comm, st);
        if (e != ncclSuccess) {
          ncclGroupEnd();
          return nccl_fail(e, "ncclSend");
        }
      }
      if (rbytes[q]) {
        ncclResult_t e = ncclRecv(d + roff[q], rbytes[q], ncclUint8, q, comm, st);
        if (e != ncclSuccess) {
          ncclGroupEnd();
          return nccl_fail(e, "ncclRecv");
        }
      }
    }
    VP_NCCL(ncclGroupEnd());
    return 0;
  }
};

static int comm_fail(const char *what) {
  state_fail("caller-supplied %s callback failed", what);  // (the message)
  return VP_EIO;
}

// Caller-supplied host-memory collectives; device variants stage through
// host memory.
struct HostComm : Comm {
  vp_comm_ops ops{};
  std::vector<uint8_t> hs, hr;
  int allgather_host(vp_ctx *c, const void *send, void *recv, size_t bytes) override {
    (void)c;
    return ops.allgather(ops.user, send, recv, bytes) ? comm_fail("allgather") : 0;
  }
  int allgather_dev(vp_ctx *c, const void *send, void *recv, size_t bytes) override {
    hs.resize(bytes ? bytes : 1);
    hr.resize(bytes * n ? bytes * n : 1);
    VP_HIP(hipMemcpyAsync(hs.data(), send, bytes, hipMemcpyDeviceToHost, c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    if (ops.allgather(ops.user, hs.data(), hr.data(), bytes)) return comm_fail("allgather");
    VP_HIP(hipMemcpyAsync(recv, hr.data(), bytes * n, hipMemcpyHostToDevice,
                          c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    return 0;
  }
  int allreduce_max_u64_dev(vp_ctx *c, uint64_t *buf, size_t count) override {
    hs.resize(count * 8 ? count * 8 : 1);
    VP_HIP(hipMemcpyAsync(hs.data(), buf, count * 8, hipMemcpyDeviceToHost,
                          c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    if (ops.allreduce_max_u64(ops.user, reinterpret_cast<uint64_t *>(hs.data()),
                              count))
      return comm_fail("allreduce_max_u64");
    VP_HIP(hipMemcpyAsync(buf, hs.data(), count * 8, hipMemcpyHostToDevice,
                          c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    return 0;
  }
  int alltoallv_dev(vp_ctx *c, const void *send, const size_t *sbytes, void *recv,
                    const size_t *rbytes, bool skip_self, hipStream_t st) override {
    if (!ops.alltoallv) return VP_ENOTSUP;
    if (!st) st = c->stream;
    size_t sn = 0, rt = 0, r0 = 0;  // r0: where this rank's own chunk lands in recv
    for (int q = 0; q < n; q++) {
      if (q == r) r0 = rt;
      sn += sbytes[q];
      rt += rbytes[q];
    }
    hs.resize(sn ? sn : 1);
    hr.resize(rt ? rt : 1);
    if (sn) VP_HIP(hipMemcpyAsync(hs.data(), send, sn, hipMemcpyDeviceToHost, st));
    VP_HIP(hipStreamSynchronize(st));
    if (ops.alltoallv(ops.user, hs.data(), sbytes, hr.data(), rbytes))
      return comm_fail("alltoallv");
    // (skip_self: the callback moved every chunk, the own one is not copied
    // back: the caller wrote it in place)
    const size_t own = skip_self ? rbytes[r] : 0;
    uint8_t *d = static_cast<uint8_t *>(recv);
    if (r0)
      VP_HIP(hipMemcpyAsync(d, hr.data(), r0, hipMemcpyHostToDevice, st));
    if (rt > r0 + own)
      VP_HIP(hipMemcpyAsync(d + r0 + own, hr.data() + r0 + own, rt - r0 - own,
                            hipMemcpyHostToDevice, st));
    VP_HIP(hipStreamSynchronize(st));
    return 0;
  }
};

int sync_tables(vp_ctx *c);

}  // namespace vp

using namespace vp;

extern "C" {

int vp_comm_unique_id(uint8_t id[VP_COMM_ID_BYTES]) {
  if (!id) return VP_EINVAL;
  ncclUniqueId u;
  VP_NCCL(ncclGetUniqueId(&u));
  memcpy(id, u.internal, VP_COMM_ID_BYTES);
  return 0;
}

static int attach_check(vp_ctx *c, int nranks, int rank) {
  if (!c || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks ||
      c->comm)
    return VP_EINVAL;
  if (c->kind != KIND_NAT) return VP_ENOTSUP;  // vignat only
  return 0;
}

int vp_attach_rccl(vp_ctx *c, const uint8_t id[VP_COMM_ID_BYTES], int nranks,
                   int rank) {
  VP_TRY(attach_check(c, nranks, rank));
  if (!id) return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  ncclUniqueId u;
  memcpy(u.internal, id, VP_COMM_ID_BYTES);
  RcclComm *m = new RcclComm();
  m->n = nranks;
  m->r = rank;
  ncclResult_t e = ncclCommInitRank(&m->comm, nranks, u, rank);
  if (e != ncclSuccess) {
    m->comm = nullptr;
    delete m;
    return nccl_fail(e, "ncclCommInitRank");
  }
  c->comm = m;
  return 0;
}

int vp_attach_comm(vp_ctx *c, const vp_comm_ops *ops, int nranks, int rank) {
  VP_TRY(attach_check(c, nranks, rank));
  if (!ops || !ops->allgather || !ops->allreduce_max_u64) return VP_EINVAL;
  VP_TRY(serve_stop(c));
  HostComm *m = new HostComm();
  m->n = nranks;
  m->r = rank;
  m->ops = *ops;
  c->comm = m;
  return 0;
}

int vp_shard_mode(vp_ctx *c, int mode) {
  if (!c || (mode != VP_SHARD_REPLICATED && mode != VP_SHARD_OWNER)) return VP_EINVAL;
  if (mode == c->shard_mode) return 0;
  // before the first batch, on an attached context (or a one-rank context
  // for VP_SHARD_REPLICATED, which is the default)
  if (!c->comm || c->seq != 0 || c->shard_mode != VP_SHARD_REPLICATED) return VP_EINVAL;
  if (c->kind != KIND_NAT) return VP_ENOTSUP;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  HostComm *h = dynamic_cast<HostComm *>(c->comm);
  if (h && !h->ops.alltoallv) return VP_EINVAL;
  VP_TRY(tbl_set_owner(c, c->ft, (uint32_t)c->comm->n, (uint32_t)c->comm->r));
  c->shard_mode = mode;
  return 0;
}

int vp_comm_abort(vp_ctx *c) {
  if (!c) return VP_EINVAL;
  if (!c->comm) return 0;
  return c->comm->abort();
}

int vp_sync_state(vp_ctx *c) {
  if (!c) return VP_EINVAL;
  if (!c->comm) return 0;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  return sync_tables(c);
}

}  // extern "C"
