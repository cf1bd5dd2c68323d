// Collectives between the ranks of one multi-GPU NF instance.
// Two transports: RCCL on device buffers (one GPU per rank, xGMI), and
// caller-supplied host-memory callbacks (vp_comm_ops; e.g. gloo, or several
// ranks sharing one GPU in tests). All calls are collective and ordered on
// the context's stream.
#pragma once

#include "vp_internal.h"

namespace vp {

struct Comm {
  int n = 1, r = 0;
  virtual ~Comm() {}
  // every rank contributes `bytes`; recv gets n * bytes in rank order
  virtual int allgather_host(vp_ctx *c, const void *send, void *recv,
                             size_t bytes) = 0;
  virtual int allgather_dev(vp_ctx *c, const void *send, void *recv,
                            size_t bytes) = 0;
  // in place, element-wise max over ranks (values < 2^63)
  virtual int allreduce_max_u64_dev(vp_ctx *c, uint64_t *buf, size_t count) = 0;
  // personalised exchange of device buffers: sbytes[q] bytes to rank q
  // (chunks consecutive in rank order), rbytes[q] bytes from rank q;
  // skip_self: this rank's own chunk is not copied into `recv` by either
  // transport (the caller reads it from `send` where it lies)
  // abandon every collective of this rank (vp_comm_abort; any thread)
  virtual int abort() { return 0; }
  // (on stream `s`, default the context's: the chunked owner pipeline runs its
  // exchanges on a stream of their own)
  virtual int alltoallv_dev(vp_ctx *c, const void *send, const size_t *sbytes,
                            void *recv, const size_t *rbytes, bool skip_self = false,
                            hipStream_t s = nullptr) = 0;
};

}  // namespace vp
