// Host-side context shared by the runtime translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/vigpath.h"
#include "vp_device.h"

#define VP_HIP(call)                                   \
  do {                                                 \
    hipError_t e_ = (call);                            \
    if (e_ != hipSuccess) return vp::hip_fail(e_, #call, __FILE__, __LINE__); \
  } while (0)

namespace vp {

int hip_fail(hipError_t e, const char *what, const char *file, int line);

enum Kind { KIND_NAT = 1, KIND_BRIDGE = 2, KIND_LB = 3 };

// Device control block of one NF table (libVig dchain + map bookkeeping).
struct Ctl {
  uint32_t stack_top;   // freed indices on the LIFO stack (dchain free list
                        // front, double-chain-impl.c:1968-1981)
  uint32_t fresh_next;  // first never-allocated index (free list tail part)
  uint32_t n_live;
  uint32_t n_tomb;
  uint32_t miss_count;
  uint32_t defer_count;
  uint32_t exp_count;
  uint32_t tomb_reused;
  uint64_t min_ts;
  uint32_t new_count;
  uint32_t pad;
};

// One open-addressed flow table + dchain-equivalent allocator in HBM.
struct FlowTable {
  FlowSlot *slots = nullptr;
  uint32_t tmask = 0;        // slots - 1
  uint32_t cap = 0;          // dchain index range (max_flows)
  uint32_t *slot_of = nullptr;  // index -> slot (kNone when free)
  uint64_t *birth = nullptr;    // index -> global packet seq of allocation
  uint64_t *tseq = nullptr;     // index -> global seq of last touch (ties)
  uint32_t *stack = nullptr;    // freed indices (LIFO)
  Ctl *ctl = nullptr;
  // host-side bookkeeping
  uint64_t ts_floor = UINT64_MAX;  // lower bound of min ts over live flows
};

struct Workspace {
  uint32_t cap_n = 0;        // batch capacity these buffers hold
  uint32_t *miss = nullptr;  // unordered miss positions
  uint32_t *miss_sorted = nullptr;
  uint32_t *defer = nullptr;  // deferred packet positions
  uint32_t *mkey = nullptr;   // 4 words per miss
  uint32_t *mhash = nullptr;
  uint32_t *first = nullptr;
  uint32_t *rank = nullptr;
  uint32_t *rep = nullptr;
  uint32_t *assign = nullptr;
  uint32_t *scratch = nullptr;
  uint32_t scratch_mask = 0;
  void *cub_tmp = nullptr;
  size_t cub_bytes = 0;
  // expiry workspace (sized by table capacity)
  uint32_t exp_cap = 0;
  uint64_t *ekey = nullptr, *ekey2 = nullptr;
  uint32_t *eidx = nullptr, *eidx2 = nullptr;
  // host staging (pinned) for the host-batch entry points
  uint8_t *h_frames = nullptr;
  size_t h_frames_bytes = 0;
  uint8_t *d_frames = nullptr;
  size_t d_frames_bytes = 0;
  uint16_t *d_len = nullptr, *d_in = nullptr, *d_out = nullptr;
  int64_t *d_now = nullptr;
  uint32_t d_meta_n = 0;
};

}  // namespace vp

struct vp_ctx {
  int kind = 0;
  int gpu = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = 0.f;
  int last_launches = 0;
  uint64_t seq = 0;       // packets processed so far (global packet order)
  int64_t last_now = -1;  // time of the last packet processed
  vp_nat_config nat{};
  vp::FlowTable ft;
  uint32_t *crc_tab = nullptr;  // position tables
  uint32_t *macw = nullptr;     // per device: d_addr|s_addr header words
  uint32_t wan_macw[3] = {0, 0, 0};
  vp::Workspace ws;
  vp::Ctl h_ctl{};
};
