// Host frames processed where they lie: the DPDK-shaped batch entry points
// (include/vigpath.h vp_process_mbufs / vp_process_batch) over mbuf data that
// the GPU reads and writes directly, through host memory registered with
// vp_register_host (a DPDK mbuf pool's hugepages).
//
// Reference: the path's ends are rte_eth_rx_burst / rte_eth_tx_burst over an
// array of mbuf pointers (nf.c:186-214, batch mode; nf.c:153,166 per
// packet); every frame sits at data_off inside its mbuf's buffer
// (rte_pktmbuf_mtod, nf.c:154) and nf_process rewrites it in place.
//
// A batch runs in chunks over kMbufSets buffer sets and three streams:
//   gather     (copy stream) the chunk's pointers, lengths and ports (and
//              times) H2D, then mbuf_gather_hdr reads every frame's first
//              64 bytes from host memory into a 64-byte header slot in HBM
//              and, for vignat, the raw sum of the frame's bytes
//              [64, 14 + total_length) that the L4 checksum covers
//              (nf-util.c:45-64): the rest of a frame crosses PCIe once and
//              is never stored;
//   process    (the context's stream) vp_process_device over the header
//              slots (vp_nat.hip nat_classify64x takes the tail sums);
//   write-back (second copy stream) mbuf_scatter writes the bytes a rewrite
//              can change, [0, min(len, 64)), of every frame that is not
//              dropped back into its mbuf, and the out ports go D2H.
// The gather of chunk k + 1 and k + 2 and the write-back of chunk k - 1 run
// while chunk k is processed (PCIe carries both directions at once).
// A frame whose rewrite may reach past byte 64 (IPv4 options on a frame
// longer than 64 bytes, nf-util.h:139-149) makes its chunk take whole-frame
// slots instead (mbuf_gather_full, slot = the chunk's longest frame), as
// does every chunk of viglb (it rewrites and checksums, no tail sums yet) and
// of a multi-GPU context. A chunk with a frame outside the registered memory
// is staged through the host (staged_range), as is every batch of a context
// with nothing registered.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "vp_comm.h"
#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(mbuf)


// Registered host ranges as the kernels see them: frame bytes [p, p + len)
// inside [hbase, hend) are at device address p + delta.
struct MapTab {
  uint64_t hbase[kMaxHostMaps], hend[kMaxHostMaps];
  int64_t delta[kMaxHostMaps];
  uint32_t n;
};

constexpr uint32_t kMbWhole = 1;     // a frame needs a whole-frame slot
constexpr uint32_t kMbUnmapped = 2;  // a frame lies outside the registered memory
enum : uint32_t { kRuleAll = 0, kRuleNoOpt = 1 };

__device__ __forceinline__ uint8_t *map_frame(const MapTab &m, uint64_t p, uint32_t len) {
  for (uint32_t i = 0; i < m.n; i++)
    if (p >= m.hbase[i] && p + len <= m.hend[i])
      return reinterpret_cast<uint8_t *>(p + (uint64_t)m.delta[i]);
  return nullptr;
}

// Bytes [o, o + 16) of a host frame of L bytes, those at or past L as 0. A
// 16-byte aligned chunk that holds a frame byte lies in that byte's page, so
// the aligned load never leaves mapped memory; frames at other alignments
// (rare: DPDK aligns data_off) are read byte by byte.
__device__ __forceinline__ uint4 host_ld16(const uint8_t *f, uint32_t o, uint32_t L) {
  if (o >= L) return make_uint4(0, 0, 0, 0);
  if ((reinterpret_cast<uintptr_t>(f) & 15) == 0) {
    uint4 v = *reinterpret_cast<const uint4 *>(f + o);
    if (L - o < 16) v = chunk_keep(v, 0, (int)(L - o));
    return v;
  }
  uint64_t lo = 0, hi = 0;
  for (uint32_t k = 0; k < 16 && o + k < L; k++) {
    const uint64_t b = f[o + k];
    if (k < 8) lo |= b << (8 * k); else hi |= b << (8 * (k - 8));
  }
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// The first nb (<= 16) bytes of v to host address d: one 16-byte store for a
// whole aligned chunk, else dword / byte stores of exactly those bytes.
__device__ __forceinline__ void host_st(uint8_t *d, uint32_t nb, uint4 v) {
  if (nb >= 16 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    *reinterpret_cast<uint4 *>(d) = v;
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  const bool al4 = (reinterpret_cast<uintptr_t>(d) & 3) == 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    if (4 * k >= nb) break;
    if (al4 && 4 * k + 4 <= nb) {
      *reinterpret_cast<uint32_t *>(d + 4 * k) = w[k];
    } else {
      for (uint32_t j = 0; j < 4 && 4 * k + j < nb; j++) d[4 * k + j] = (uint8_t)(w[k] >> (8 * j));
    }
  }
}

// Frames of the chunk, four lanes each (lane q: bytes [16q, 16q + 16) of the
// header), grid-stride; every wave ORs its flags into *flags once.
// Header slot: the frame's bytes [0, min(len, 64)), zeros after. TAIL:
// tail[i] = raw sum (vp_device.h sum16x4, the checksum's arithmetic) of bytes
// [64, min(len, 14 + total_length)) of an IPv4 IHL-5 frame, else 0 -- four
// lanes per frame, each a chunk of every 64 bytes, four loads in flight.
// rule kRuleNoOpt: an IPv4 frame with options longer than 64 bytes sets
// kMbWhole (its L4 header, and so its rewrite, may lie past byte 64).
template <bool TAIL>
__global__ __launch_bounds__(256) void mbuf_gather_hdr(const uint64_t *ptr, const uint16_t *len,
                                                      uint32_t n, MapTab m, uint32_t rule,
                                                      uint8_t *slots, uint32_t *tail,
                                                      uint32_t *flags) {
  const uint32_t lane = threadIdx.x & 63, q = lane & 3, lead = lane & ~3u;
  const uint32_t ng = (gridDim.x * blockDim.x) >> 2;
  uint32_t fl = 0;
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; i < n; i += ng) {
    const uint32_t L = len[i];
    const uint8_t *f = map_frame(m, ptr[i], L);
    const uint4 v = f ? host_ld16(f, 16 * q, L) : make_uint4(0, 0, 0, 0);
    if (!f) fl |= kMbUnmapped;
    reinterpret_cast<uint4 *>(slots + (size_t)i * 64)[q] = v;
    // ether_type, version/IHL (bytes 12-14: chunk 0), total_length (16-17)
    const uint32_t w3 = (uint32_t)__shfl((int)v.w, (int)lead);
    const uint32_t w4 = (uint32_t)__shfl((int)v.x, (int)lead + 1);
    const bool ip = (w3 & 0xFFFF) == 0x0008;
    const uint32_t ihl = (w3 >> 16) & 0x0F;
    if (f && rule == kRuleNoOpt && L > 64 && ip && ihl > 5) fl |= kMbWhole;
    if constexpr (TAIL) {
      uint32_t end = 0;
      if (f && ip && ihl == 5) end = min(L, 14u + bswap16((uint16_t)(w4 & 0xFFFF)));
      uint32_t s = 0;
      for (uint32_t c = 4 + q; 16 * c < end; c += 16) {
        const uint4 x0 = host_ld16(f, 16 * c, end), x1 = host_ld16(f, 16 * (c + 4), end),
                    x2 = host_ld16(f, 16 * (c + 8), end), x3 = host_ld16(f, 16 * (c + 12), end);
        s = sum16x4(x3, sum16x4(x2, sum16x4(x1, sum16x4(x0, s))));
      }
      s += (uint32_t)__shfl_xor((int)s, 1);
      s += (uint32_t)__shfl_xor((int)s, 2);
      if (q == 0) tail[i] = s;
    }
  }
  const uint64_t b1 = __ballot(fl & kMbWhole), b2 = __ballot(fl & kMbUnmapped);
  if (lane == 0 && (b1 | b2)) atomicOr(flags, (b1 ? kMbWhole : 0u) | (b2 ? kMbUnmapped : 0u));
}

// Whole frames into `slot`-byte slots (zeros past each frame), four lanes
// per frame.
__global__ __launch_bounds__(256) void mbuf_gather_full(const uint64_t *ptr, const uint16_t *len,
                                                       uint32_t n, MapTab m, uint8_t *slots,
                                                       uint32_t slot, uint32_t *flags) {
  const uint32_t lane = threadIdx.x & 63, q = lane & 3;
  const uint32_t ng = (gridDim.x * blockDim.x) >> 2;
  uint32_t fl = 0;
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; i < n; i += ng) {
    const uint32_t L = len[i];
    const uint8_t *f = map_frame(m, ptr[i], L);
    if (!f) fl |= kMbUnmapped;
    uint4 *d = reinterpret_cast<uint4 *>(slots + (size_t)i * slot);
    for (uint32_t c = q; c < slot / 16; c += 4)
      d[c] = f ? host_ld16(f, 16 * c, L) : make_uint4(0, 0, 0, 0);
  }
  const uint64_t b2 = __ballot(fl & kMbUnmapped);
  if (lane == 0 && b2) atomicOr(flags, kMbUnmapped);
}

// Write-back: bytes [0, min(len, wb)) of every frame that was not dropped
// (out != in: nf.c frees a dropped mbuf, nf.c:159-160, so its bytes are never
// seen again) from its slot into its mbuf, four lanes per frame.
__global__ __launch_bounds__(256) void mbuf_scatter(const uint64_t *ptr, const uint16_t *len,
                                                   const uint16_t *in_dev,
                                                   const uint16_t *out, uint32_t n, MapTab m,
                                                   const uint8_t *slots, uint32_t slot,
                                                   uint32_t wb) {
  const uint32_t q = threadIdx.x & 3;
  const uint32_t ng = (gridDim.x * blockDim.x) >> 2;
  for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 2; i < n; i += ng) {
    if (out[i] == in_dev[i]) continue;
    const uint32_t L = len[i];
    uint8_t *f = map_frame(m, ptr[i], L);
    if (!f) continue;
    const uint32_t bytes = min(L, wb);
    const uint4 *s = reinterpret_cast<const uint4 *>(slots + (size_t)i * slot);
    for (uint32_t c = q; 16 * c < bytes; c += 4) host_st(f + 16 * c, min(16u, bytes - 16 * c), s[c]);
  }
}

// ================================================================ host ==

// What each NF's rewrite can touch (the write-back) and whether its chunks
// can run on 64-byte header slots.
struct MbufPlan {
  bool header;       // 64-byte header slots (else whole frames)
  bool tail;         // with tail sums (vignat: the L4 checksum covers the frame)
  uint32_t rule;     // kRuleNoOpt: IPv4 options on a long frame need whole frames
  uint32_t wb_hdr;   // bytes written back per forwarded frame, header slots
  uint32_t wb_full;  // ... whole-frame slots
};
static MbufPlan mbuf_plan(const vp_ctx *c) {
  switch (c->kind) {
    case KIND_NAT:  // MACs, addresses, ports, checksums (nat_main.c:96-106)
      return {true, true, kRuleNoOpt, 64, 128};
    case KIND_FW:  // the MACs only (fw_main.c:76-77)
      return {true, false, kRuleNoOpt, 16, 16};
    case KIND_BRIDGE:  // never rewrites (bridge_main.c:311-329)
    case KIND_POL:     // never rewrites (policer_main.c:111-145)
      return {true, false, kRuleAll, 0, 0};
    default:  // viglb: dst address, MACs, checksums (lb_main.c:58-65)
      return {false, false, kRuleAll, 128, 128};
  }
}

static uint32_t mbuf_blocks() {  // (read per batch: tools/mbuf_probe.py sweeps it)
  const char *e = getenv("VIGPATH_MBUF_BLOCKS");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? (uint32_t)v : 256u;
}

// Wait for an event by polling (the host thread polls, as a DPDK lcore does;
// a blocking wait adds tens of microseconds of wake-up per chunk).
static hipError_t event_poll(hipEvent_t e) {
  hipError_t r;
  while ((r = hipEventQuery(e)) == hipErrorNotReady) {
  }
  return r;
}

static MapTab map_tab(const vp_ctx *c) {
  MapTab t{};
  t.n = (uint32_t)c->hmaps.size();
  for (uint32_t i = 0; i < t.n; i++) {
    t.hbase[i] = c->hmaps[i].hbase;
    t.hend[i] = c->hmaps[i].hend;
    t.delta[i] = c->hmaps[i].delta;
  }
  return t;
}

static bool host_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

template <class T>
static int dgrow(T **p, size_t *have, size_t count) {
  if (*p && count <= *have) return 0;
  hipFree(*p);
  *p = nullptr;
  *have = 0;
  VP_HIP(hipMalloc((void **)p, sizeof(T) * std::max<size_t>(count, 1)));
  *have = count;
  return 0;
}

// Frames [k0, k0 + m) of the batch through the host: gathered len bytes per
// mbuf into pinned slots (the batch's longest frame, so bytes past a frame's
// length read as 0), processed, scattered back. Synchronous.
static int staged_range(vp_ctx *c, const vp_mbuf_batch *b, uint32_t k0, uint32_t m) {
  Workspace &w = c->ws;
  uint32_t maxlen = 64;
  for (uint32_t i = 0; i < m; i++) maxlen = std::max<uint32_t>(maxlen, b->len[k0 + i]);
  const uint32_t slot = (maxlen + 15) & ~15u;
  const size_t bytes = (size_t)std::max<uint32_t>(m, 1) * slot;
  if (bytes > w.d_frames_bytes) {
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(w.d_frames);
    w.d_frames = nullptr;
    w.d_frames_bytes = 0;
    VP_HIP(hipMalloc((void **)&w.d_frames, bytes));
    w.d_frames_bytes = bytes;
  }
  if (bytes > w.h_frames_bytes) {
    if (w.h_frames) hipHostFree(w.h_frames);
    w.h_frames = nullptr;
    w.h_frames_bytes = 0;
    VP_HIP(hipHostMalloc((void **)&w.h_frames, bytes, hipHostMallocDefault));
    w.h_frames_bytes = bytes;
  }
  VP_TRY(dgrow(&w.st_meta, &w.st_meta_n, 14ull * m + 16));
  uint16_t *d_len = reinterpret_cast<uint16_t *>(w.st_meta);
  uint16_t *d_in = d_len + m, *d_out = d_in + m;
  int64_t *d_now = reinterpret_cast<int64_t *>(
      w.st_meta + ((6ull * m + 7) & ~7ull));  // (8-byte aligned after 3 u16 arrays)
  uint8_t *h = w.h_frames;
  for (uint32_t i = 0; i < m; i++) {  // gather the mbuf data into slots
    const uint32_t L = b->len[k0 + i];
    memcpy(h + (size_t)i * slot, b->frames[k0 + i], L);
    memset(h + (size_t)i * slot + L, 0, slot - L);
  }
  VP_HIP(hipMemcpyAsync(w.d_frames, h, (size_t)m * slot, hipMemcpyHostToDevice, c->stream));
  VP_HIP(hipMemcpyAsync(d_len, b->len + k0, 2ull * m, hipMemcpyHostToDevice, c->stream));
  VP_HIP(hipMemcpyAsync(d_in, b->in_dev + k0, 2ull * m, hipMemcpyHostToDevice, c->stream));
  vp_dev_batch db{};
  if (b->now)
    VP_HIP(hipMemcpyAsync(d_now, b->now + k0, 8ull * m, hipMemcpyHostToDevice, c->stream));
  db.frames = w.d_frames;
  db.slot = slot;
  db.n = m;
  db.len = d_len;
  db.in_dev = d_in;
  db.now = b->now ? d_now : nullptr;
  db.now0 = b->now0 + (int64_t)k0 * b->now_step;
  db.now_step = b->now_step;
  db.out_dev = d_out;
  c->host_now = b->now ? b->now + k0 : nullptr;
  const int rc = vp_process_device(c, &db, nullptr);
  c->host_now = nullptr;
  VP_TRY(rc);
  VP_HIP(hipMemcpyAsync(h, w.d_frames, (size_t)m * slot, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipMemcpyAsync(b->out_dev + k0, d_out, 2ull * m, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < m; i++)  // scatter back in place
    memcpy(b->frames[k0 + i], h + (size_t)i * slot, b->len[k0 + i]);
  return 0;
}

static int mbuf_reserve(vp_ctx *c, uint32_t ch) {
  Workspace &w = c->ws;
  constexpr uint32_t S = Workspace::kMbufSets;
  if (!w.cstream) {
    VP_HIP(hipStreamCreateWithFlags(&w.cstream, hipStreamNonBlocking));
    VP_HIP(hipStreamCreateWithFlags(&w.dstream, hipStreamNonBlocking));
  }
  if (!w.mb_ev_in[0])
    for (uint32_t i = 0; i < S; i++) {
      VP_HIP(hipEventCreateWithFlags(&w.mb_ev_in[i], hipEventDisableTiming));
      VP_HIP(hipEventCreateWithFlags(&w.mb_ev_done[i], hipEventDisableTiming));
      VP_HIP(hipEventCreateWithFlags(&w.mb_ev_out[i], hipEventDisableTiming));
    }
  if (ch <= w.mb_cap) return 0;
  VP_HIP(hipDeviceSynchronize());  // (the sets may still be in flight elsewhere)
  void *old[] = {w.mb_ptr, w.mb_slots, w.mb_tail, w.mb_len, w.mb_in, w.mb_out, w.mb_now};
  for (void *p : old) hipFree(p);
  w.mb_ptr = nullptr;
  w.mb_slots = nullptr;
  w.mb_tail = nullptr;
  w.mb_len = w.mb_in = w.mb_out = nullptr;
  w.mb_now = nullptr;
  w.mb_cap = 0;
  VP_HIP(hipMalloc((void **)&w.mb_ptr, 8ull * S * ch));
  VP_HIP(hipMalloc((void **)&w.mb_slots, 64ull * S * ch));
  VP_HIP(hipMalloc((void **)&w.mb_tail, 4ull * S * ch));
  VP_HIP(hipMalloc((void **)&w.mb_len, 2ull * S * ch));
  VP_HIP(hipMalloc((void **)&w.mb_in, 2ull * S * ch));
  VP_HIP(hipMalloc((void **)&w.mb_out, 2ull * S * ch));
  VP_HIP(hipMalloc((void **)&w.mb_now, 8ull * S * ch));
  if (!w.mb_flags) VP_HIP(hipMalloc((void **)&w.mb_flags, 4ull * S));
  if (!w.h_mbflags) VP_HIP(hipHostMalloc((void **)&w.h_mbflags, 4ull * S, hipHostMallocDefault));
  if (w.h_mbmeta) hipHostFree(w.h_mbmeta);
  w.h_mbmeta = nullptr;
  w.h_mbmeta_bytes = 0;
  VP_HIP(hipHostMalloc((void **)&w.h_mbmeta, 22ull * S * ch, hipHostMallocDefault));
  w.h_mbmeta_bytes = 22ull * S * ch;
  w.mb_cap = ch;
  return 0;
}

// Resets vp_ctx::hdr_tail / host_now when the pipeline leaves early.
struct CtxTailGuard {
  vp_ctx *c;
  ~CtxTailGuard() {
    c->hdr_tail = nullptr;
    c->host_now = nullptr;
  }
};

static int mbuf_pipeline(vp_ctx *c, const vp_mbuf_batch *b) {
  Workspace &w = c->ws;
  CtxTailGuard guard{c};
  const MbufPlan pl = mbuf_plan(c);
  const uint32_t n = b->n;
  // one device call per batch on a multi-GPU context (vp_process_device is a
  // collective there), on whole-frame slots (owner mode has no header slots)
  const bool one = c->comm != nullptr;
  const bool header = pl.header && !one;
  uint32_t ch = 1u << 20;
  if (const char *e = getenv("VIGPATH_HOST_CHUNK")) ch = std::max(1, atoi(e));
  if (one || ch > n) ch = std::max<uint32_t>(n, 1);
  const uint32_t K = one ? 1 : (n + ch - 1) / ch;
  constexpr uint32_t S = Workspace::kMbufSets;
  VP_TRY(mbuf_reserve(c, ch));
  const MapTab mt = map_tab(c);
  const bool pin_ptr = host_pinned(b->frames), pin_len = host_pinned(b->len),
             pin_in = host_pinned(b->in_dev), pin_out = host_pinned(b->out_dev),
             pin_now = b->now && host_pinned(b->now);
  const uint32_t G = mbuf_blocks();
  auto cnt = [&](uint32_t k) { return std::min(ch, n - k * ch); };
  auto hm = [&](uint32_t k, size_t at) { return w.h_mbmeta + (size_t)(k % S) * 22 * ch + at * ch; };
  // a per-packet array's chunk k: the caller's page-locked memory itself, or
  // a staged copy in the set's pinned block (`at`: offset in units of ch)
  auto src = [&](const void *arr, bool pinned, size_t esz, size_t at, uint32_t k) {
    const uint8_t *a = static_cast<const uint8_t *>(arr) + (size_t)k * ch * esz;
    if (pinned) return a;
    memcpy(hm(k, at), a, esz * cnt(k));
    return static_cast<const uint8_t *>(hm(k, at));
  };
  auto hout = [&](uint32_t k) {
    return pin_out ? b->out_dev + (size_t)k * ch : reinterpret_cast<uint16_t *>(hm(k, 20));
  };
  std::vector<uint32_t> wslot(K, 0);  // 0: header slots; else whole-frame slot bytes
  std::vector<uint8_t> staged(K, 0);  // processed through the host (staged_range)
  std::vector<uint8_t> retired(K, 0);
  auto retire = [&](uint32_t k) -> int {
    if (retired[k]) return 0;
    retired[k] = 1;
    if (staged[k]) return 0;
    VP_HIP(hipEventSynchronize(w.mb_ev_out[k % S]));
    if (!pin_out) memcpy(b->out_dev + (size_t)k * ch, hm(k, 20), 2ull * cnt(k));
    return 0;
  };
  auto issue_gather = [&](uint32_t k) -> int {
    const uint32_t i = k % S, m = cnt(k);
    if (k >= S) VP_TRY(retire(k - S));  // frees the set's pinned staging
    // the set's device buffers: free once chunk k - S's write-back read them
    if (k >= S && !staged[k - S]) VP_HIP(hipStreamWaitEvent(w.cstream, w.mb_ev_out[i], 0));
    VP_HIP(hipMemcpyAsync(w.mb_ptr + (size_t)i * ch, src(b->frames, pin_ptr, 8, 0, k), 8ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipMemcpyAsync(w.mb_len + (size_t)i * ch, src(b->len, pin_len, 2, 8, k), 2ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipMemcpyAsync(w.mb_in + (size_t)i * ch, src(b->in_dev, pin_in, 2, 10, k), 2ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    if (b->now)
      VP_HIP(hipMemcpyAsync(w.mb_now + (size_t)i * ch, src(b->now, pin_now, 8, 12, k), 8ull * m,
                            hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipMemsetAsync(w.mb_flags + i, 0, 4, w.cstream));
    if (header && m) {
      auto *kern = pl.tail ? mbuf_gather_hdr<true> : mbuf_gather_hdr<false>;
      kern<<<std::min<uint32_t>(G, (m + 63) / 64), 256, 0, w.cstream>>>(
          w.mb_ptr + (size_t)i * ch, w.mb_len + (size_t)i * ch, m, mt, pl.rule,
          w.mb_slots + (size_t)i * ch * 64, w.mb_tail + (size_t)i * ch, w.mb_flags + i);
      VP_HIP(hipGetLastError());
    }
    VP_HIP(hipMemcpyAsync(w.h_mbflags + i, w.mb_flags + i, 4, hipMemcpyDeviceToHost,
                          w.cstream));
    VP_HIP(hipEventRecord(w.mb_ev_in[i], w.cstream));
    return 0;
  };
  int32_t last_full = -1;  // the last chunk on whole-frame slots (mb_full's user)
  auto process = [&](uint32_t k) -> int {
    const uint32_t i = k % S, m = cnt(k);
    VP_HIP(event_poll(w.mb_ev_in[i]));
    uint32_t fl = header ? w.h_mbflags[i] : kMbWhole;
    vp_dev_batch db{};
    db.n = m;
    db.len = w.mb_len + (size_t)i * ch;
    db.in_dev = w.mb_in + (size_t)i * ch;
    db.now = b->now ? w.mb_now + (size_t)i * ch : nullptr;
    db.now0 = b->now0 + (int64_t)k * ch * b->now_step;
    db.now_step = b->now_step;
    db.out_dev = w.mb_out + (size_t)i * ch;
    VP_HIP(hipStreamWaitEvent(c->stream, w.mb_ev_in[i], 0));
    if (fl & kMbWhole) {  // whole-frame slots: the chunk's longest frame
      uint32_t maxlen = 64;
      for (uint32_t j = 0; j < m; j++) maxlen = std::max<uint32_t>(maxlen, b->len[(size_t)k * ch + j]);
      const uint32_t slot = (maxlen + 15) & ~15u;
      if ((size_t)m * slot > w.mb_full_bytes) {
        VP_HIP(hipDeviceSynchronize());
        hipFree(w.mb_full);
        w.mb_full = nullptr;
        w.mb_full_bytes = 0;
        VP_HIP(hipMalloc((void **)&w.mb_full, (size_t)std::max<uint32_t>(m, 1) * slot));
        w.mb_full_bytes = (size_t)std::max<uint32_t>(m, 1) * slot;
      } else if (last_full >= 0 && !staged[last_full]) {  // its write-back read mb_full
        VP_HIP(hipStreamWaitEvent(c->stream, w.mb_ev_out[last_full % S], 0));
      }
      if (m) {
        mbuf_gather_full<<<std::min<uint32_t>(G, (m + 63) / 64), 256, 0, c->stream>>>(
            w.mb_ptr + (size_t)i * ch, db.len, m, mt, w.mb_full, slot, w.mb_flags + i);
        VP_HIP(hipGetLastError());
      }
      if (!header) {  // (the header gather did not look: the unmapped flag now)
        VP_HIP(hipMemcpyAsync(w.h_mbflags + i, w.mb_flags + i, 4, hipMemcpyDeviceToHost,
                              c->stream));
        VP_HIP(stream_wait(c->stream));
        fl |= w.h_mbflags[i];
      }
      if (!(fl & kMbUnmapped)) {
        db.frames = w.mb_full;
        db.slot = slot;
        wslot[k] = slot;
        last_full = (int32_t)k;
      }
    } else {
      db.frames = w.mb_slots + (size_t)i * ch * 64;
      db.slot = 64;
      c->hdr_tail = pl.tail ? w.mb_tail + (size_t)i * ch : nullptr;
    }
    if (fl & kMbUnmapped) {  // a frame outside the registered memory
      c->hdr_tail = nullptr;
      staged[k] = 1;
      return staged_range(c, b, k * ch, m);
    }
    c->host_now = b->now ? b->now + (size_t)k * ch : nullptr;
    const int rc = vp_process_device(c, &db, nullptr);
    c->hdr_tail = nullptr;
    c->host_now = nullptr;
    VP_TRY(rc);
    VP_HIP(hipEventRecord(w.mb_ev_done[i], c->stream));
    return 0;
  };
  hipStream_t ws = w.dstream;  // (on the gather stream instead: 10-15 % slower, r04f)
  auto issue_scatter = [&](uint32_t k) -> int {
    if (staged[k]) return 0;
    const uint32_t i = k % S, m = cnt(k);
    VP_HIP(hipStreamWaitEvent(ws, w.mb_ev_done[i], 0));
    const uint32_t wb = wslot[k] ? pl.wb_full : pl.wb_hdr;
    if (wb && m) {
      mbuf_scatter<<<std::min<uint32_t>(G, (m + 63) / 64), 256, 0, ws>>>(
          w.mb_ptr + (size_t)i * ch, w.mb_len + (size_t)i * ch, w.mb_in + (size_t)i * ch,
          w.mb_out + (size_t)i * ch, m, mt,
          wslot[k] ? w.mb_full : w.mb_slots + (size_t)i * ch * 64, wslot[k] ? wslot[k] : 64,
          wb);
      VP_HIP(hipGetLastError());
    }
    VP_HIP(hipMemcpyAsync(hout(k), w.mb_out + (size_t)i * ch, 2ull * m, hipMemcpyDeviceToHost,
                          ws));
    VP_HIP(hipEventRecord(w.mb_ev_out[i], ws));
    return 0;
  };
  for (uint32_t k = 0; k < std::min<uint32_t>(K, 2); k++) VP_TRY(issue_gather(k));
  for (uint32_t k = 0; k < K; k++) {
    if (k + 2 < K) VP_TRY(issue_gather(k + 2));
    VP_TRY(process(k));
    VP_TRY(issue_scatter(k));
  }
  for (uint32_t k = 0; k < K; k++) VP_TRY(retire(k));
  return 0;
}

// ------------------------------------------------------ host-gather mode --
// The same batch with the host's cores doing the scattered part: worker
// threads copy every frame's first 64 bytes (and, for vignat, the raw sum of
// its bytes [64, 14 + total_length)) out of its mbuf into pinned header slots,
// the slots cross PCIe as one DMA per chunk, and after processing the threads
// copy the bytes a rewrite can change back into the mbufs of the frames that
// were not dropped. The GPU never touches host frames (nothing to register);
// PCIe carries large DMA transfers instead of one 64-byte read and one write
// request per frame (the zero-copy mode's bound). While chunk
// k is copied and processed, the threads write back chunk k - 1 and gather
// chunk k + 1. VIGPATH_MBUF_MODE=host|gpu picks the mode, VIGPATH_MBUF_THREADS
// the threads (default 8, the caller's thread included).
class HostPool {
 public:
  explicit HostPool(unsigned n) : n_(std::max(1u, n)) {
    for (unsigned i = 1; i < n_; i++) th_.emplace_back([this] { loop(); });
  }
  unsigned size() const { return n_; }
  // fn(part) for every part in [0, parts), over the pool and the caller;
  // returns when all parts are done
  void run(uint32_t parts, const std::function<void(uint32_t)> &fn) {
    std::lock_guard<std::mutex> one(run_m_);
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(m_);
      gen = ++gen_;
      fn_ = &fn;
      parts_ = parts;
      done_ = 0;
      next_.store(gen << 32);  // (job tag | next part: a late thread never takes a part of another job)
    }
    cv_.notify_all();
    work(gen, &fn, parts);
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [&] { return done_ == parts; });
  }

 private:
  void work(uint64_t gen, const std::function<void(uint32_t)> *fn, uint32_t parts) {
    uint32_t mine = 0;
    uint64_t cur = next_.load();
    while ((cur >> 32) == gen && (uint32_t)cur < parts) {
      if (next_.compare_exchange_weak(cur, cur + 1)) {
        (*fn)((uint32_t)cur);
        mine++;
        cur = next_.load();
      }
    }
    if (mine) {
      std::lock_guard<std::mutex> g(m_);
      done_ += mine;
      if (done_ == parts) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return gen_ != seen; });
      seen = gen_;
      const std::function<void(uint32_t)> *fn = fn_;
      const uint32_t parts = parts_;
      g.unlock();
      work(seen, fn, parts);
      g.lock();
    }
  }
  unsigned n_;
  std::vector<std::thread> th_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(uint32_t)> *fn_ = nullptr;
  uint32_t parts_ = 0, done_ = 0;
  uint64_t gen_ = 0;
  std::atomic<uint64_t> next_{0};
};

static HostPool &host_pool() {  // (process-wide; its threads live as long as the process)
  static HostPool *p = [] {
    const char *e = getenv("VIGPATH_MBUF_THREADS");
    const int v = e ? atoi(e) : 0;
    return new HostPool(v > 0 ? (unsigned)std::min(v, 256) : 8u);
  }();
  return *p;
}

static bool mbuf_mode_host() {
  const char *e = getenv("VIGPATH_MBUF_MODE");
  return e && !strcmp(e, "host");
}

// One frame of L bytes into its 64-byte header slot (zeros past L) and, with
// `tail`, its tail sum: the plain sum of the little-endian 16-bit words of
// bytes [64, min(L, 14 + total_length)) of an IPv4 IHL-5 frame (an odd last
// byte as a word of its own), the arithmetic of mbuf_gather_hdr's sum16x4.
// Returns kMbWhole where mbuf_gather_hdr would (rule kRuleNoOpt).
static inline uint32_t host_gather_one(const uint8_t *f, uint32_t L, uint8_t *d, uint32_t *tail,
                                       const MbufPlan &pl) {
  const uint32_t nb = std::min<uint32_t>(L, 64);
  memcpy(d, f, nb);
  if (nb < 64) memset(d + nb, 0, 64 - nb);
  const bool ip = d[12] == 0x08 && d[13] == 0x00;
  const uint32_t ihl = d[14] & 0x0F;
  if (pl.tail) {
    uint32_t s = 0;
    if (ip && ihl == 5) {
      const uint32_t end = std::min<uint32_t>(L, 14u + ((uint32_t)d[16] << 8 | d[17]));
      uint32_t o = 64;
      for (; o + 1 < end; o += 2) s += (uint32_t)f[o] | (uint32_t)f[o + 1] << 8;
      if (o < end) s += f[o];
    }
    *tail = s;
  }
  return pl.rule == kRuleNoOpt && L > 64 && ip && ihl > 5 ? kMbWhole : 0u;
}

static int mbuf_host_pipeline(vp_ctx *c, const vp_mbuf_batch *b, const MbufPlan &pl) {
  Workspace &w = c->ws;
  CtxTailGuard guard{c};
  constexpr uint32_t S = Workspace::kMbufSets;
  const uint32_t n = b->n;
  uint32_t ch = 1u << 20;
  if (const char *e = getenv("VIGPATH_HOST_CHUNK")) ch = std::max(1, atoi(e));
  ch = std::min<uint32_t>(ch, std::max<uint32_t>(n, 1));
  const uint32_t K = (n + ch - 1) / ch;
  VP_TRY(mbuf_reserve(c, ch));
  if (ch > w.mb_hcap) {
    VP_HIP(hipDeviceSynchronize());
    if (w.h_mbslots) hipHostFree(w.h_mbslots);
    if (w.h_mbtail) hipHostFree(w.h_mbtail);
    w.h_mbslots = nullptr;
    w.h_mbtail = nullptr;
    w.mb_hcap = 0;
    VP_HIP(hipHostMalloc((void **)&w.h_mbslots, 64ull * S * ch, hipHostMallocDefault));
    VP_HIP(hipHostMalloc((void **)&w.h_mbtail, 4ull * S * ch, hipHostMallocDefault));
    w.mb_hcap = ch;
  }
  const bool pin_len = host_pinned(b->len), pin_in = host_pinned(b->in_dev),
             pin_out = host_pinned(b->out_dev), pin_now = b->now && host_pinned(b->now);
  HostPool &hp = host_pool();
  auto cnt = [&](uint32_t k) { return std::min(ch, n - k * ch); };
  auto hm = [&](uint32_t k, size_t at) { return w.h_mbmeta + (size_t)(k % S) * 22 * ch + at * ch; };
  auto src = [&](const void *arr, bool pinned, size_t esz, size_t at, uint32_t k) {
    const uint8_t *a = static_cast<const uint8_t *>(arr) + (size_t)k * ch * esz;
    if (pinned) return a;
    memcpy(hm(k, at), a, esz * cnt(k));
    return static_cast<const uint8_t *>(hm(k, at));
  };
  auto hout = [&](uint32_t k) {
    return pin_out ? b->out_dev + (size_t)k * ch : reinterpret_cast<uint16_t *>(hm(k, 20));
  };
  auto slots = [&](uint32_t k) { return w.h_mbslots + (size_t)(k % S) * ch * 64; };
  auto tails = [&](uint32_t k) { return w.h_mbtail + (size_t)(k % S) * ch; };
  // pieces per pool job: several per thread, frame lengths vary
  const uint32_t parts = 4 * hp.size();
  auto gather = [&](uint32_t k) {
    const uint32_t m = cnt(k), k0 = k * ch;
    uint8_t *hs = slots(k);
    uint32_t *ht = tails(k);
    std::atomic<uint32_t> flags{0};
    hp.run(parts, [&](uint32_t part) {
      const uint32_t lo = (uint32_t)((uint64_t)m * part / parts),
                     hi = (uint32_t)((uint64_t)m * (part + 1) / parts);
      uint32_t fl = 0;
      for (uint32_t j = lo; j < hi; j++)
        fl |= host_gather_one(b->frames[k0 + j], b->len[k0 + j], hs + (size_t)j * 64, ht + j, pl);
      if (fl) flags.fetch_or(fl);
    });
    return flags.load();
  };
  auto launch = [&](uint32_t k) -> int {
    const uint32_t i = k % S, m = cnt(k);
    if (k >= S) VP_HIP(hipStreamWaitEvent(w.cstream, w.mb_ev_out[i], 0));
    VP_HIP(hipMemcpyAsync(w.mb_slots + (size_t)i * ch * 64, slots(k), 64ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    if (pl.tail)
      VP_HIP(hipMemcpyAsync(w.mb_tail + (size_t)i * ch, tails(k), 4ull * m,
                            hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipMemcpyAsync(w.mb_len + (size_t)i * ch, src(b->len, pin_len, 2, 8, k), 2ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipMemcpyAsync(w.mb_in + (size_t)i * ch, src(b->in_dev, pin_in, 2, 10, k), 2ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    if (b->now)
      VP_HIP(hipMemcpyAsync(w.mb_now + (size_t)i * ch, src(b->now, pin_now, 8, 12, k), 8ull * m,
                            hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipEventRecord(w.mb_ev_in[i], w.cstream));
    VP_HIP(hipStreamWaitEvent(c->stream, w.mb_ev_in[i], 0));
    vp_dev_batch db{};
    db.n = m;
    db.frames = w.mb_slots + (size_t)i * ch * 64;
    db.slot = 64;
    db.len = w.mb_len + (size_t)i * ch;
    db.in_dev = w.mb_in + (size_t)i * ch;
    db.now = b->now ? w.mb_now + (size_t)i * ch : nullptr;
    db.now0 = b->now0 + (int64_t)k * ch * b->now_step;
    db.now_step = b->now_step;
    db.out_dev = w.mb_out + (size_t)i * ch;
    c->hdr_tail = pl.tail ? w.mb_tail + (size_t)i * ch : nullptr;
    c->host_now = b->now ? b->now + (size_t)k * ch : nullptr;
    const int rc = vp_process_device(c, &db, nullptr);
    c->hdr_tail = nullptr;
    c->host_now = nullptr;
    VP_TRY(rc);
    VP_HIP(hipEventRecord(w.mb_ev_done[i], c->stream));
    VP_HIP(hipStreamWaitEvent(w.dstream, w.mb_ev_done[i], 0));
    if (pl.wb_hdr)
      VP_HIP(hipMemcpyAsync(slots(k), w.mb_slots + (size_t)i * ch * 64, 64ull * m,
                            hipMemcpyDeviceToHost, w.dstream));
    VP_HIP(hipMemcpyAsync(hout(k), w.mb_out + (size_t)i * ch, 2ull * m, hipMemcpyDeviceToHost,
                          w.dstream));
    VP_HIP(hipEventRecord(w.mb_ev_out[i], w.dstream));
    return 0;
  };
  auto scatter = [&](uint32_t k) -> int {
    const uint32_t i = k % S, m = cnt(k), k0 = k * ch;
    VP_HIP(event_poll(w.mb_ev_out[i]));
    if (!pin_out) memcpy(b->out_dev + k0, hm(k, 20), 2ull * m);
    if (!pl.wb_hdr) return 0;
    const uint8_t *hs = slots(k);
    const uint16_t *out = b->out_dev + k0, *in = b->in_dev + k0;
    hp.run(parts, [&](uint32_t part) {
      const uint32_t lo = (uint32_t)((uint64_t)m * part / parts),
                     hi = (uint32_t)((uint64_t)m * (part + 1) / parts);
      for (uint32_t j = lo; j < hi; j++)
        if (out[j] != in[j])  // (a dropped frame's mbuf is freed: nf.c:159-160)
          memcpy(b->frames[k0 + j], hs + (size_t)j * 64,
                 std::min<uint32_t>(b->len[k0 + j], pl.wb_hdr));
    });
    return 0;
  };
  bool pending = false;  // chunk k - 1 launched, not yet written back
  for (uint32_t k = 0; k < K; k++) {
    if (gather(k) & kMbWhole) {  // IPv4 options on a long frame: whole frames
      if (pending) VP_TRY(scatter(k - 1));
      pending = false;
      VP_TRY(staged_range(c, b, k * ch, cnt(k)));
      continue;
    }
    VP_TRY(launch(k));
    if (pending) VP_TRY(scatter(k - 1));
    pending = true;
  }
  if (pending) VP_TRY(scatter(K - 1));
  return 0;
}

}  // namespace vp

using namespace vp;

extern "C" {

int vp_register_host(vp_ctx *c, void *base, size_t bytes) {
  if (!c || !base || !bytes) return VP_EINVAL;
  if (c->hmaps.size() >= (size_t)kMaxHostMaps) {
    state_fail("vp_register_host: at most %d registered host ranges per context", kMaxHostMaps);
    return VP_ENOMEM;
  }
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  const uint64_t hb = reinterpret_cast<uint64_t>(base);
  for (const HostMap &h : c->hmaps)
    if (hb < h.hend && hb + bytes > h.hbase) return VP_EINVAL;  // overlaps
  HostMap h{hb, hb + bytes, 0, false};
  // page-locked already (hipHostMalloc'd, or registered by the application):
  // only mapped; else registered here (and unregistered with the context)
  hipPointerAttribute_t pa;
  const bool pinned = hipPointerGetAttributes(&pa, base) == hipSuccess &&
                      pa.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  if (!pinned) {
    const hipError_t r = hipHostRegister(base, bytes, hipHostRegisterMapped);
    if (r != hipSuccess && r != hipErrorHostMemoryAlreadyRegistered)
      return hip_fail(r, "hipHostRegister", __FILE__, __LINE__);
    (void)hipGetLastError();
    h.ours = r == hipSuccess;
  }
  hipError_t e;
  void *d = nullptr;
  e = hipHostGetDevicePointer(&d, base, 0);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    hipPointerAttribute_t a;
    e = hipPointerGetAttributes(&a, base);
    if (e != hipSuccess || !a.devicePointer) {
      if (h.ours) hipHostUnregister(base);
      return hip_fail(e != hipSuccess ? e : hipErrorInvalidValue, "hipHostGetDevicePointer",
                      __FILE__, __LINE__);
    }
    d = a.devicePointer;
  }
  h.delta = (int64_t)(reinterpret_cast<uint64_t>(d) - hb);
  {  // the range's last byte must map by the same offset (one mapping)
    hipPointerAttribute_t a;
    uint8_t *last = static_cast<uint8_t *>(base) + bytes - 1;
    if (hipPointerGetAttributes(&a, last) == hipSuccess && a.devicePointer &&
        reinterpret_cast<uint64_t>(a.devicePointer) !=
            reinterpret_cast<uint64_t>(last) + (uint64_t)h.delta) {
      if (h.ours) hipHostUnregister(base);
      return VP_EINVAL;
    }
    (void)hipGetLastError();
  }
  c->hmaps.push_back(h);
  return 0;
}

int vp_unregister_host(vp_ctx *c, void *base) {
  if (!c || !base) return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  const uint64_t hb = reinterpret_cast<uint64_t>(base);
  for (size_t i = 0; i < c->hmaps.size(); i++) {
    if (c->hmaps[i].hbase != hb) continue;
    VP_HIP(hipDeviceSynchronize());  // no kernel of the library still reads it
    if (c->hmaps[i].ours) VP_HIP(hipHostUnregister(base));
    c->hmaps.erase(c->hmaps.begin() + (long)i);
    return 0;
  }
  return VP_EINVAL;
}

int vp_process_mbufs(vp_ctx *c, const vp_mbuf_batch *b) {
  if (!c || !b) return VP_EINVAL;
  if (b->n && (!b->frames || !b->len || !b->in_dev || !b->out_dev)) return VP_EINVAL;
  if (!b->now && (b->now_step < 0 || b->now0 < 0)) return VP_ENOTSUP;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  if (b->n == 0 && !c->comm) return 0;
  const MbufPlan pl = mbuf_plan(c);
  if (pl.header && !c->comm && mbuf_mode_host()) return mbuf_host_pipeline(c, b, pl);
  if (c->hmaps.empty()) return staged_range(c, b, 0, b->n);
  return mbuf_pipeline(c, b);
}

int vp_process_batch(vp_ctx *c, uint32_t n, const uint16_t *in_dev, uint8_t *const *frames,
                     const uint16_t *len, const int64_t *now, uint16_t *out_dev) {
  if (!c || (n && (!in_dev || !frames || !len || !now || !out_dev))) return VP_EINVAL;
  vp_mbuf_batch b{};
  b.n = n;
  b.frames = frames;
  b.len = len;
  b.in_dev = in_dev;
  b.now = now;
  b.out_dev = out_dev;
  return vp_process_mbufs(c, &b);
}

}  // extern "C"
