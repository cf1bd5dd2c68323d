// Device-side building blocks shared by the NF kernels (gfx950, wave64).
//
// Semantics restate, per function, the reference's per-packet path (paths
// relative to the reference repository):
//   packet cursor + header parse   nf-util.h:116-162, packet-io.c:40-111
//   L3/L4 predicates               nf-util.c:21-31
//   checksum rewrite               nf-util.c:45-64 + DPDK 20.08 rte_ip.h
//   CRC32C key hash                codegen/main.ml:328-401 (generated
//                                  <Struct>_hash), libvig/verified/ether.c:61-90
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vp {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;  // slot index field: never used
constexpr uint32_t kTomb = 0xFFFFFFFEu;   // slot index field: erased
constexpr uint32_t kNone = 0xFFFFFFFFu;   // slot_of[]: index not allocated

__host__ __device__ inline uint16_t bswap16(uint16_t v) {
  return (uint16_t)((v >> 8) | (v << 8));
}

// ---------------------------------------------------------------- frames --
// A frame is `cap` bytes of a slot. Reads past the slot are 0 and writes past
// it are dropped: the reference touches mbuf bytes past pkt_len for some
// malformed headers; within the slot we read the same bytes it would.
struct GFrame {
  uint8_t *b;
  uint32_t cap;
  __device__ uint8_t r8(uint32_t o) const { return o < cap ? b[o] : 0; }
  __device__ uint16_t r16(uint32_t o) const {
    return (uint16_t)(r8(o) | (r8(o + 1) << 8));
  }
  __device__ uint32_t r32(uint32_t o) const {
    return (uint32_t)r16(o) | ((uint32_t)r16(o + 2) << 16);
  }
  __device__ void w8(uint32_t o, uint8_t v) const {
    if (o < cap) b[o] = v;
  }
  __device__ void w16(uint32_t o, uint16_t v) const {
    w8(o, (uint8_t)v);
    w8(o + 1, (uint8_t)(v >> 8));
  }
  __device__ void w32(uint32_t o, uint32_t v) const {
    w16(o, (uint16_t)v);
    w16(o + 2, (uint16_t)(v >> 16));
  }
};

struct L34 {
  uint32_t ip;  // offset of the IPv4 header
  uint32_t l4;  // offset of the TCP/UDP header (after borrowed options)
  bool ok;
};

// nf_then_get_rte_ether_header + nf_then_get_rte_ipv4_header +
// nf_then_get_tcpudp_header (nf-util.h:116-162). `total` is the packet-io
// cursor's total length (the mbuf pkt_len); lengths wrap like the
// reference's size_t -> u32 -> u16 narrowing.
__device__ inline L34 parse_l34(const GFrame &f, uint32_t total) {
  L34 r{14, 0, false};
  uint32_t read = 14;
  uint16_t unread = (uint16_t)(total - read);
  bool is_ip = f.r16(12) == bswap16(0x0800);
  if (!is_ip | (unread < 20)) return r;
  read += 20;
  uint8_t ihl = f.r8(14) & 0x0F;
  uint16_t tl = bswap16(f.r16(16));
  if ((ihl < 5) | (unread < tl)) return r;
  uint16_t opt = (uint16_t)((ihl - 5) * 4);
  if ((opt != 0) & ((uint32_t)unread - 20u >= opt)) read += opt;
  uint8_t proto = f.r8(23);
  if (!((proto == 6) | (proto == 17)) | ((uint32_t)(total - read) < 4u))
    return r;
  r.l4 = read;
  r.ok = true;
  return r;
}

// DPDK 20.08 __rte_raw_cksum + __rte_raw_cksum_reduce.
__device__ inline uint32_t fold16(uint32_t s) {
  s = (s >> 16) + (s & 0xFFFF);
  s = (s >> 16) + (s & 0xFFFF);
  return s;
}

// The raw sum's inner step over 16 bytes at an even offset: the four LE words'
// 16-bit halves added to s (v_sad_u16 against zero adds both halves at once).
__device__ __forceinline__ uint32_t sum16x4(const uint4 v, uint32_t s) {
  s = __builtin_amdgcn_sad_u16(v.x, 0u, s);
  s = __builtin_amdgcn_sad_u16(v.y, 0u, s);
  s = __builtin_amdgcn_sad_u16(v.z, 0u, s);
  return __builtin_amdgcn_sad_u16(v.w, 0u, s);
}
// Bytes [lo, hi) of a 16-byte chunk kept, the others zeroed (0 <= lo, hi <= 16).
__device__ __forceinline__ uint32_t bytes_mask(int lo, int hi) {
  lo = lo < 0 ? 0 : lo > 4 ? 4 : lo;
  hi = hi < 0 ? 0 : hi > 4 ? 4 : hi;
  const uint32_t below_hi = hi >= 4 ? 0xFFFFFFFFu : (1u << (8 * hi)) - 1;
  const uint32_t below_lo = lo >= 4 ? 0xFFFFFFFFu : (1u << (8 * lo)) - 1;
  return below_hi & ~below_lo;
}
__device__ __forceinline__ uint4 chunk_keep(uint4 v, int lo, int hi) {
  v.x &= bytes_mask(lo, hi);
  v.y &= bytes_mask(lo - 4, hi - 4);
  v.z &= bytes_mask(lo - 8, hi - 8);
  v.w &= bytes_mask(lo - 12, hi - 12);
  return v;
}

// __rte_raw_cksum over bytes [off, off + len) of a frame (off even): the sum
// of the LE 16-bit words, an odd last byte as a word's low byte; bytes past
// the slot count as 0. Aligned 16-byte loads (slots are multiples of 16 and
// start 16-byte aligned), the chunks at either end masked.
__device__ inline uint32_t raw_sum(const GFrame &f, uint32_t off, uint32_t len) {
  const uint32_t hi = min(off + len, f.cap);
  uint32_t s = 0;
  for (uint32_t c = off & ~15u; c < hi; c += 16) {
    uint4 v = *reinterpret_cast<const uint4 *>(f.b + c);
    if (c < off || c + 16 > hi) v = chunk_keep(v, (int)off - (int)c, (int)hi - (int)c);
    s = sum16x4(v, s);
  }
  return s;
}
__device__ inline uint32_t raw_cksum(const GFrame &f, uint32_t off,
                                     uint32_t len) {
  return fold16(raw_sum(f, off, len));
}
// rte_ipv4_phdr_cksum: {src, dst, 0, proto, be16(l4_len)} as 6 LE words.
__device__ inline uint32_t phdr_cksum(uint32_t src, uint32_t dst, uint8_t proto,
                                      uint32_t l4_len) {
  uint32_t s = (src & 0xFFFF) + (src >> 16) + (dst & 0xFFFF) + (dst >> 16) +
               ((uint32_t)proto << 8) + (((l4_len >> 8) & 0xFF) |
                                         ((l4_len & 0xFF) << 8));
  return fold16(s);
}
// rte_ipv4_udptcp_cksum given the folded L4 byte sum.
__device__ inline uint16_t finish_l4(uint32_t l4sum, uint32_t ph) {
  uint32_t c = l4sum + ph;
  c = ((c & 0xFFFF0000u) >> 16) + (c & 0xFFFF);
  c = (~c) & 0xFFFF;
  if (c == 0) c = 0xFFFF;  // DPDK 20.08: for TCP too (TCP-zero edge unpinned)
  return (uint16_t)c;
}

// nf_set_rte_ipv4_udptcp_checksum (nf-util.c:45-64), generic byte form.
// `tail`: the raw sum of the frame's bytes past the slot that the L4 sum
// covers (a 64-byte header slot of a longer host frame, vp_mbuf.hip; the
// slot's own bytes past 64 read as 0), else 0.
__device__ inline void set_checksums(const GFrame &f, uint32_t ip,
                                     uint32_t l4, uint32_t tail = 0) {
  f.w16(ip + 10, 0);
  uint8_t proto = f.r8(ip + 9);
  uint32_t at = proto == 6 ? l4 + 16 : l4 + 6;
  if (proto == 6 || proto == 17) {
    f.w16(at, 0);
    uint32_t l3 = bswap16(f.r16(ip + 2));
    uint16_t c = 0;
    if (l3 >= 20) {
      uint32_t l4len = l3 - 20;
      c = finish_l4(fold16(raw_sum(f, l4, l4len) + tail),
                    phdr_cksum(f.r32(ip + 12), f.r32(ip + 16), proto, l4len));
    }
    f.w16(at, c);
  }
  f.w16(ip + 10, (uint16_t)~raw_cksum(f, ip, 20));
}

__device__ inline void set_macs(const GFrame &f, const uint32_t mw[3]) {
  // mw = the 12 header bytes d_addr[6] s_addr[6] as 3 LE words
  for (int k = 0; k < 3; k++) f.w32(4 * k, mw[k]);
}

// Frame-stream loads/stores of the per-lane paths (64 B per packet, read
// once, written once; non-temporal variants measured no faster, round 2).
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) { return *p; }
__device__ __forceinline__ void st_stream(uint4 *p, uint4 v) { *p = v; }

// Tile frame loads / stores of frames64_tiles and the vignat classify loop.
// Stores are write-through (sc1: the written line leaves the XCD's L2 at
// once, so the frame stream leaves fewer dirty lines between the table rows
// and at the kernel boundary): 3.5 % faster nat_classify64 than write-back
// stores; non-temporal (evict-first) loads measured 30 % slower (round 2
// diagnostic builds).
__device__ __forceinline__ uint4 tile_ld(const uint4 *p) { return *p; }
__device__ __forceinline__ void tile_st(uint4 *g, uint32_t c, uint4 v) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, 4096, 0x00020000);
  const v4u x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)(c * 16), 0, 16);
}

// Stores of the wide-slot classify tiles: 16 bytes at byte `off` of the tile
// at g (64 slots, `bytes` in all), write-through like tile_st.
__device__ __forceinline__ void tile_st_at(uint8_t *g, uint32_t bytes, uint32_t off,
                                           uint4 v) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, (int)bytes, 0x00020000);
  const v4u x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)off, 0, 16);
}

// ------------------------------------------------------------ fast frames --
// The 64-byte slot held in 16 registers (LE words). Only compile-time word
// indices are used so nothing spills to scratch.
struct RFrame {
  uint32_t w[16];
  __device__ uint32_t u16at(int o) const {  // o even, compile-time
    return (o & 2) ? (w[o >> 2] >> 16) : (w[o >> 2] & 0xFFFF);
  }
  __device__ void set16(int o, uint32_t v) {
    if (o & 2)
      w[o >> 2] = (w[o >> 2] & 0x0000FFFFu) | (v << 16);
    else
      w[o >> 2] = (w[o >> 2] & 0xFFFF0000u) | (v & 0xFFFF);
  }
  // raw u32 at an offset == 2 (mod 4)
  __device__ uint32_t u32at2(int o) const {
    return (w[o >> 2] >> 16) | (w[(o >> 2) + 1] << 16);
  }
  __device__ void set32at2(int o, uint32_t v) {
    w[o >> 2] = (w[o >> 2] & 0x0000FFFFu) | (v << 16);
    w[(o >> 2) + 1] = (w[(o >> 2) + 1] & 0xFFFF0000u) | (v >> 16);
  }
};

// LDS image of one wave's 64 frames (64 x 64 B): 16-byte chunk c (packet
// c/4, part c%4) lives at c ^ ((c >> 4) & 3), so both the lane-contiguous
// global<->LDS copies and each lane's 4 reads of its own frame are
// bank-conflict-free ds_*_b128 accesses.
__device__ __forceinline__ uint32_t chunk_swz(uint32_t c) {
  return c ^ ((c >> 4) & 3u);
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lanes holding counter `ch` (valid `v`) that share the first valid lane's
// counter are served by one LDS atomic (traffic with locality would otherwise
// serialise a wave on one counter); the rest add individually. Returns this
// lane's reserved position.
__device__ __forceinline__ uint32_t group_reserve(uint32_t *ctr, uint32_t ch,
                                                  bool v) {
  const uint64_t vm = __ballot(v);
  if (!vm) return 0;
  const uint32_t lead = __shfl(ch, __ffsll((unsigned long long)vm) - 1);
  const bool grp = v && ch == lead;
  const uint64_t same = __ballot(grp);
  const uint32_t first = __ffsll((unsigned long long)same) - 1;
  uint32_t base = 0;
  if (grp && __lane_id() == first)
    base = atomicAdd(&ctr[ch], (uint32_t)__popcll(same));
  base = __shfl(base, first);
  if (grp) return base + (uint32_t)__popcll(same & ((1ull << __lane_id()) - 1ull));
  return v ? atomicAdd(&ctr[ch], 1u) : 0;
}

// Touch bins: besides the per-packet touch log, the 64-byte classify kernels
// sort each touch (flow index i of packet p) into one of 2^bbits bins (256 up
// to kMaxBins, chosen per table so that a bin's indices fit one LDS tile)
// while classifying, so the timestamp fold needs a single pass
// (touch_bins_reduce, vp_table.hip) instead of count + scan + scatter +
// reduce. Index i belongs to bin (i >> 6) & (2^bbits - 1), at in-bin position
// ((i >> (6 + bbits)) << 6) | (i & 63): runs of 64 consecutive indices per
// bin, so sequential flow sets spread over all bins, the fold writes whole
// 512-byte runs of ts, and a wave whose 64 packets touch consecutive indices
// appends them as one 256-byte run (whole lines; with runs of 16 a wave wrote
// four 64-byte pieces into four bins whose lines stayed partial in L2 for
// dozens of tiles: 11 % of the classify kernel, tools/ablate.py NOBINS).
// Each block appends to
// its own fixed-size slice of every bin (LDS cursors); a bin's slices are
// adjacent (bin-major), so the fold reads each bin as one region. With bins on, the
// classify kernels write no per-packet touch log: a touch that finds its
// slice full is logged alone (olog[p] = index) and queued on the block's
// overflow slice (oent/ocnt), and *ovf tells the host to apply the queued
// touches after the fold (tbl_late_touches, vp_table.hip).
constexpr uint32_t kMaxBins = 1024;
constexpr uint32_t kCurReprobe = kMaxBins;       // LDS cursor of the reprobe queue
constexpr uint32_t kCurOverflow = kMaxBins + 1;  // LDS cursor of the overflow queue
constexpr uint32_t kCurDest = kMaxBins + 2;      // LDS cursors per owner rank (owner mode)
constexpr uint32_t kMaxDest = 64;                // = kMaxRanks (vp_internal.h)
constexpr uint32_t kCurMiss = kCurDest + kMaxDest;  // LDS cursor of vignat's miss slice
constexpr uint32_t kCurs = kCurMiss + 1;
// finish() may set touch = kReprobe instead of an index: the packet leaves
// the wave and is queued on the block's reprobe slice (TileQueue).
constexpr uint32_t kReprobe = 0xFFFFFFFDu;
struct TileQueue {
  uint32_t *ent;    // [block][range] packet positions; null = off
  uint32_t *cnt;    // [block] entries queued
  uint32_t *total;  // += every block's count (one atomic per block)
};
struct TouchBins {
  // bin-major: the fold's block for bin b reads one contiguous region
  uint32_t *ent;  // [bin][block][cap] entries (in-bin << pbits | position); null = off
  uint32_t *cnt;  // [bin][block] entries written
  uint32_t *ovf;  // set when a slice overflowed
  uint32_t *oent;  // [block][range] positions of overflowed touches
  uint32_t *ocnt;  // [block] overflowed touches queued
  uint32_t *olog;  // olog[p] = index of an overflowed touch
  uint32_t cap, pbits, bbits;
  uint32_t nsrc;  // classify blocks (the launch's grid)
  // run entries (runs != 0): a wave whose 64 packets touch the 64
  // consecutive indices of one bin run records them as one word in its
  // block's row of rtab ([block][bin][rwords], kept whole in the L2 as the
  // block fills it), counted in the top byte of the bin's count; rwords per
  // block and bin (2; 8 for 1024-thread blocks, whose ranges are 4x longer)
  uint32_t *rtab;
  uint32_t runs;
  uint32_t rwords;
};
constexpr uint32_t kBinRunShift = 24;            // run words claimed: a count's top byte
constexpr uint32_t kBinRunFlags = 0xFF000000u;   // (that byte)
constexpr uint32_t kBinRunWordsMax = 8;

// Touch-log entry of packet p; `log` is null in the classify kernels that
// bin their touches.
__device__ __forceinline__ void log_put(uint32_t *log, uint32_t p, uint32_t v) {
  if (log) log[p] = v;
}
constexpr uint32_t kBinRunBits = 6;  // runs of 64 consecutive indices per bin
constexpr uint32_t kBinRun = 1u << kBinRunBits;
__device__ __forceinline__ uint32_t bin_of(uint32_t i, uint32_t bbits) {
  return (i >> kBinRunBits) & ((1u << bbits) - 1);
}
__device__ __forceinline__ uint32_t bin_local(uint32_t i, uint32_t bbits) {
  return ((i >> (kBinRunBits + bbits)) << kBinRunBits) | (i & (kBinRun - 1));
}
__device__ __forceinline__ uint32_t bin_index(uint32_t bin, uint32_t local,
                                              uint32_t bbits) {
  return ((local >> kBinRunBits) << (kBinRunBits + bbits)) | (bin << kBinRunBits) |
         (local & (kBinRun - 1));
}

// Append packet p's touch (kNone: none) to block rb's slice of its bin
// (wave-uniform call; `range` = packets per block, range0 = the block's first
// packet). A full slice logs the touch alone on the block's overflow queue.
// kOvf: the overflow queue's LDS cursor (a kernel whose tables stay at 256
// bins keeps only cursors 0..256, kOvf = 256, to make room in LDS).
// (runcnt: an LDS counter of the block's run tiles, or null)
template <uint32_t kOvf = kCurOverflow>
__device__ __forceinline__ void bins_put(const TouchBins &bins, uint32_t *cur,
                                         uint32_t rb, uint32_t range, uint32_t range0,
                                         uint32_t p, uint32_t touch,
                                         uint32_t *runcnt = nullptr) {
  if (!bins.ent) return;
  if (bins.runs) {  // the whole wave one run of 64 indices: one word
    const uint32_t lane = __lane_id();
    const uint32_t t0 = __builtin_amdgcn_readfirstlane(touch);
    const uint32_t q0 = __builtin_amdgcn_readfirstlane(p);
    const bool in_run = t0 != kNone && (t0 & (kBinRun - 1)) == 0 && touch == t0 + lane &&
                        p == q0 + lane;
    if (__ballot(in_run) == ~0ull) {
      const uint32_t b0 = bin_of(t0, bins.bbits);
      if (runcnt && lane == 0) atomicAdd(runcnt, 1u);
      uint32_t slot = kBinRunWordsMax;
      // (claims past rwords only by waves racing the check: at most the
      // block's waves more, well inside the byte)
      if (lane == 0 &&
          (__hip_atomic_load(&cur[b0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >>
           kBinRunShift) < bins.rwords)
        slot = atomicAdd(&cur[b0], 1u << kBinRunShift) >> kBinRunShift;
      slot = __builtin_amdgcn_readfirstlane(slot);
      if (slot < bins.rwords) {
        if (lane == 0)
          bins.rtab[(((size_t)rb << bins.bbits) + b0) * bins.rwords + slot] =
              ((bin_local(t0, bins.bbits) >> kBinRunBits) << 20) | (q0 - range0);
        return;
      }
      // (the block's run slots of this bin are taken: the touches one by one)
    }
  }
  const bool v = touch != kNone;
  const uint32_t b = v ? bin_of(touch, bins.bbits) : 0;
  const uint32_t k = group_reserve(cur, b, v) & ~kBinRunFlags;
  const bool fits = k < bins.cap;
  if (v && fits)
    bins.ent[((size_t)b * bins.nsrc + rb) * bins.cap + k] =
        (bin_local(touch, bins.bbits) << bins.pbits) | (p - range0);
  const bool spill = v && !fits;
  const uint32_t o = group_reserve(cur, kOvf, spill);
  if (spill) {
    bins.olog[p] = touch;
    bins.oent[(size_t)rb * range + o] = p;
  }
}

// Whole-line bin entries (1024-thread vignat blocks, up to 128 bins): a
// block stages each bin's entries in an LDS ring of kStageLines lines of 16
// entries (64 bytes) and stores a line only once all 16 are written, as one
// 64-byte piece, so no partly written slice line sits in the L2 (uniform
// order). Entry k of bin b goes to line k / 16, ring
// position (k / 16) % kStageLines; a position is free for line L once line
// L - kStageLines has been stored (gen[] holds the next line it may take),
// the lane whose write completes a line stores it. Every reserved entry
// belongs to a wave inside bins_put_staged's loop, and the oldest unstored
// line of a bin always has its position, so the loop always progresses (no
// block barrier inside it). The last partial line of each bin is stored by
// bins_flush_staged after the block's final barrier.
constexpr uint32_t kStageLines = 4, kStageBins = 128;
struct BinStage {
  uint32_t *ring;  // [bin][kStageLines][16] entries
  uint32_t *wc;    // [bin][kStageLines] entries written into the line
  uint32_t *gen;   // [bin][kStageLines] the line the position may take next
};
__device__ __forceinline__ void bins_stage_init(const BinStage &st) {
  for (uint32_t i = threadIdx.x; i < kStageBins * kStageLines; i += blockDim.x) {
    st.wc[i] = 0;
    st.gen[i] = i % kStageLines;
  }
}

template <uint32_t kOvf = kCurOverflow>
__device__ __forceinline__ void bins_put_staged(const TouchBins &bins, const BinStage &st,
                                                uint32_t *cur, uint32_t rb, uint32_t range,
                                                uint32_t range0, uint32_t p, uint32_t touch,
                                                uint32_t *runcnt = nullptr) {
  if (!bins.ent) return;
  if (bins.runs) {  // the whole wave one run of 64 indices: one word (as bins_put)
    const uint32_t lane = __lane_id();
    const uint32_t t0 = __builtin_amdgcn_readfirstlane(touch);
    const uint32_t q0 = __builtin_amdgcn_readfirstlane(p);
    const bool in_run = t0 != kNone && (t0 & (kBinRun - 1)) == 0 && touch == t0 + lane &&
                        p == q0 + lane;
    if (__ballot(in_run) == ~0ull) {
      const uint32_t b0 = bin_of(t0, bins.bbits);
      if (runcnt && lane == 0) atomicAdd(runcnt, 1u);
      uint32_t slot = kBinRunWordsMax;
      if (lane == 0 &&
          (__hip_atomic_load(&cur[b0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >>
           kBinRunShift) < bins.rwords)
        slot = atomicAdd(&cur[b0], 1u << kBinRunShift) >> kBinRunShift;
      slot = __builtin_amdgcn_readfirstlane(slot);
      if (slot < bins.rwords) {
        if (lane == 0)
          bins.rtab[(((size_t)rb << bins.bbits) + b0) * bins.rwords + slot] =
              ((bin_local(t0, bins.bbits) >> kBinRunBits) << 20) | (q0 - range0);
        return;
      }
    }
  }
  const bool v = touch != kNone;
  const uint32_t b = v ? bin_of(touch, bins.bbits) : 0;
  const uint32_t k = group_reserve(cur, b, v) & ~kBinRunFlags;
  const bool fits = k < bins.cap;
  const uint32_t e = (bin_local(touch, bins.bbits) << bins.pbits) | (p - range0);
  const uint32_t line = k >> 4, pos = b * kStageLines + (line % kStageLines);
  bool pend = v && fits;
  while (__ballot(pend)) {
    bool full = false;
    if (pend && __hip_atomic_load(&st.gen[pos], __ATOMIC_ACQUIRE,
                                  __HIP_MEMORY_SCOPE_WORKGROUP) == line) {
      st.ring[pos * 16 + (k & 15)] = e;
      full = __hip_atomic_fetch_add(&st.wc[pos], 1u, __ATOMIC_ACQ_REL,
                                    __HIP_MEMORY_SCOPE_WORKGROUP) == 15;
      pend = false;
    }
    if (full) {  // this lane's write completed the line: store it whole
      const uint4 *src = reinterpret_cast<const uint4 *>(st.ring + pos * 16);
      uint4 *dst = reinterpret_cast<uint4 *>(
          bins.ent + ((size_t)b * bins.nsrc + rb) * bins.cap + (size_t)line * 16);
      const uint4 x0 = src[0], x1 = src[1], x2 = src[2], x3 = src[3];
      dst[0] = x0;
      dst[1] = x1;
      dst[2] = x2;
      dst[3] = x3;
      __hip_atomic_store(&st.wc[pos], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&st.gen[pos], line + kStageLines, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (__ballot(pend)) __builtin_amdgcn_s_sleep(1);
  }
  const bool spill = v && !fits;
  const uint32_t o = group_reserve(cur, kOvf, spill);
  if (spill) {
    bins.olog[p] = touch;
    bins.oent[(size_t)rb * range + o] = p;
  }
}

// After the block's final barrier: each bin's last, partial line (the full
// ones were stored by the lanes that completed them).
__device__ __forceinline__ void bins_flush_staged(const TouchBins &bins, const BinStage &st,
                                                  const uint32_t *cur, uint32_t rb) {
  if (!bins.ent) return;
  for (uint32_t b = threadIdx.x; b < (1u << bins.bbits); b += blockDim.x) {
    const uint32_t c = min(cur[b] & ~kBinRunFlags, bins.cap);
    const uint32_t line = c >> 4, n = c & 15;
    if (!n) continue;
    const uint32_t pos = b * kStageLines + (line % kStageLines);
    uint32_t *dst = bins.ent + ((size_t)b * bins.nsrc + rb) * bins.cap + (size_t)line * 16;
    for (uint32_t i = 0; i < n; i++) dst[i] = st.ring[pos * 16 + i];
  }
}

// After the block's last bins_put and a barrier: publish its slice sizes.
template <uint32_t kOvf = kCurOverflow>
__device__ __forceinline__ void bins_publish(const TouchBins &bins, const uint32_t *cur,
                                             uint32_t rb) {
  if (!bins.ent) return;
  for (uint32_t b = threadIdx.x; b < (1u << bins.bbits); b += blockDim.x) {
    const uint32_t c = cur[b] & ~kBinRunFlags, nr = min(cur[b] >> kBinRunShift, bins.rwords);
    bins.cnt[(size_t)b * bins.nsrc + rb] = (c < bins.cap ? c : bins.cap) | (nr << kBinRunShift);
  }
  if (threadIdx.x == 0) {
    const uint32_t o = cur[kOvf];
    bins.ocnt[rb] = o;
    if (o) *bins.ovf = 1;
  }
}

// Packets [p0, p1) of a batch of n_all 64-byte slots, in tiles of 64
// consecutive packets per wave (256-thread blocks, 4 waves): every global
// load/store instruction moves 1 KiB contiguous (lane l <-> bytes
// 16l..16l+15 of a 1 KiB piece), staged through the wave's LDS tile S
// (256 x uint4).
//
// Each packet is handled in two halves around the prefetch of the wave's
// next tile (its four 1 KiB frame loads plus the lane's len / in_dev):
//   pend = issue(p, f, in, len, mine)  parse, hash, issue any per-lane read;
//                                      pend.row = the 64-byte table row
//                                      (bucket) this packet needs, or kNone;
//   mod  = finish(pend, row, p, f, in, len, touch)
//                                      consume the row, rewrite f, return
//                                      the mask of the 16-byte chunks of f
//                                      that must be written back (bit k =
//                                      bytes 16k..16k+15; a UDP rewrite leaves
//                                      chunk 3 alone);
//                                      touch = the flow index the packet
//                                      logged (kNone if none), for the bins,
//                                      or kReprobe to queue the packet on the
//                                      block's reprobe slice (rq).
// Rows are gathered cooperatively: four lanes fetch one row as 64 contiguous
// bytes (one memory request per row instead of four 16-byte pieces per
// lane) and the wave's LDS tile hands each lane its own row, the same
// layout as the frames. The gather is issued before the prefetch: vector-
// memory counters drain in issue order (MI355X_MICROARCH.md §Per-instruction
// cycle constants), so rows can be consumed while the prefetch is still in
// flight and the frame stream's HBM latency hides under the probes. The grid
// is persistent (resident_grid()); each block owns one contiguous range of
// tiles, its four waves interleaved over it: measured 12 % faster than
// dealing tiles round-robin over all waves, and 10 % faster than an
// XCD-aware range order, as every block streams its own DRAM
// pages and its packets' table rows stay near each other in its XCD's L2.
// `cur` is kCurs LDS counters, zeroed by the kernel before its barrier.
// Virtual blocks (vper != 0; the chunked owner pipeline, vp_nat.hip): the
// launch is blocks vb0 .. vb0 + gridDim.x - 1 of a grid whose every block
// owns vper tiles of [p0, p1); the per-block slices (bins, rq) are indexed by
// the virtual block.
// Packet p's input port: in_dev[p] + in0, where exactly one of the two is
// live: a batch without a port array (vp_dev_batch.in_port) has in_dev null,
// read as zeros through a buffer of no records (branch-free, no register
// more than the load), and in0 = its port; otherwise in0 = 0.
__device__ __forceinline__ uint32_t port_of(const uint16_t *in_dev, uint32_t in0, uint32_t p) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(in_dev), 0,
                                                    in_dev ? 0x7FFFFFFF : 0, 0x00020000);
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (int)(2 * p), 0, 0) + in0;
}

// PR: the issue half, the row requests and the next tile's prefetch at a
// raised wave priority (as vignat's lean tile: the SIMD issues them ahead of
// other waves' arithmetic, more requests in flight).
// W: waves per block (4, or 16 for one 1024-thread block per CU).
template <uint32_t kOvf = kCurOverflow, bool PR = false, uint32_t W = 4, class Issue,
          class Finish>
__device__ __forceinline__ void frames64_tiles(uint8_t *frames,
                                               const uint16_t *len,
                                               const uint16_t *in_dev,
                                               uint32_t p0, uint32_t p1,
                                               uint32_t n_all, uint4 *S,
                                               const uint4 *rows, Issue issue,
                                               Finish finish,
                                               const TouchBins &bins,
                                               const TileQueue &rq,
                                               uint32_t *cur, uint32_t vb0 = 0,
                                               uint32_t vper = 0, uint32_t in0 = 0) {
  // (the wave index as a scalar: the tile stores' buffer resources are
  // provably uniform, no waterfall loops)
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t first = p0 & ~63u;
  const uint32_t tiles = (p1 - first + 63) / 64;
  uint4 r[4];
  uint32_t m_in = 0, m_len = 0;
  auto fetch = [&](uint32_t tile) {
    const uint32_t tb = first + tile * 64;
    const uint4 *g = reinterpret_cast<const uint4 *>(frames + (size_t)tb * 64);
    const uint32_t avail = n_all - tb < 64 ? n_all - tb : 64u;  // in the batch
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t c = 64 * j + lane;
      r[j] = (c >> 2) < avail ? tile_ld(g + c) : make_uint4(0, 0, 0, 0);
    }
    const uint32_t p = tb + lane;
    m_in = p < n_all ? port_of(in_dev, in0, p) : 0u;
    m_len = p < n_all ? len[p] : 0u;
  };
  const uint32_t rb = vb0 + blockIdx.x;
  const uint32_t per_b = vper ? vper : (tiles + gridDim.x - 1) / gridDim.x;
  uint32_t tile = rb * per_b + wv;
  const uint32_t tend = min(tiles, rb * per_b + per_b), tstep = W;
  const uint32_t range0 = first + rb * per_b * 64;  // this block's first packet
  if (tile < tend) fetch(tile);
  for (; tile < tend; tile += tstep) {
    const uint32_t tb = first + tile * 64;
    uint4 *g = reinterpret_cast<uint4 *>(frames + (size_t)tb * 64);
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = r[j];
    wave_lds_sync();
    const uint32_t p = tb + lane;
    const bool mine = p >= p0 && p < p1;
    RFrame f;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint4 v = S[chunk_swz(4 * lane + k)];
      f.w[4 * k] = v.x;
      f.w[4 * k + 1] = v.y;
      f.w[4 * k + 2] = v.z;
      f.w[4 * k + 3] = v.w;
    }
    const uint32_t in = m_in, ln = m_len;
    if constexpr (PR) __builtin_amdgcn_s_setprio(1);
    auto pend = issue(p, f, in, ln, mine);
    // piece j of lane L: part L % 4 of the row of packet 16 j + L / 4; the
    // four row numbers come in by ds_bpermute, issued together and waited for
    // once, and the four loads go out unconditionally (a packet without a row
    // reads bucket 0, an L1 hit, and gets zeros): a load under a branch waited
    // for its own permute
    // (named registers: an array here stays in scratch memory)
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
    if (rows) {
      uint32_t b0, b1, b2, b3;
      const uint32_t src = lane & ~3u;  // byte address of lane L / 4
      const uint32_t want = pend.row;
      asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(b0) : "v"(src), "v"(want));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:64" : "=v"(b1) : "v"(src), "v"(want));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:128" : "=v"(b2) : "v"(src), "v"(want));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:192" : "=v"(b3) : "v"(src), "v"(want));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
      const uint32_t part = lane & 3;
      const uint4 z = q0;
      const uint4 r0 = rows[4 * (size_t)(b0 != kNone ? b0 : 0u) + part];
      const uint4 r1 = rows[4 * (size_t)(b1 != kNone ? b1 : 0u) + part];
      const uint4 r2 = rows[4 * (size_t)(b2 != kNone ? b2 : 0u) + part];
      const uint4 r3 = rows[4 * (size_t)(b3 != kNone ? b3 : 0u) + part];
      q0 = b0 != kNone ? r0 : z;
      q1 = b1 != kNone ? r1 : z;
      q2 = b2 != kNone ? r2 : z;
      q3 = b3 != kNone ? r3 : z;
    }
    if (tile + tstep < tend) fetch(tile + tstep);
    if constexpr (PR) __builtin_amdgcn_s_setprio(0);
    uint4 row[4] = {};
    if (rows) {  // S is free: f is in registers
      wave_lds_sync();
      S[chunk_swz(lane)] = q0;
      S[chunk_swz(64 + lane)] = q1;
      S[chunk_swz(128 + lane)] = q2;
      S[chunk_swz(192 + lane)] = q3;
      wave_lds_sync();
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) row[k] = S[chunk_swz(4 * lane + k)];
    }
    uint32_t mod = 0;
    uint32_t touch = kNone;
    if (mine) mod = finish(pend, row, p, f, in, ln, touch);
    if (rq.ent) {  // queue on this block's reprobe slice
      const bool v = touch == kReprobe;
      const uint32_t k = group_reserve(cur, kCurReprobe, v);
      if (v) rq.ent[(size_t)rb * per_b * 64 + k] = p;
    }
    if (touch == kReprobe) touch = kNone;
    bins_put<kOvf>(bins, cur, rb, per_b * 64, range0, p, touch);
    if (mod) {
#pragma unroll
      for (uint32_t k = 0; k < 4; k++)
        S[chunk_swz(4 * lane + k)] =
            make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
    }
    // chunk c (lane-contiguous) is part c % 4 = lane % 4 of packet c / 4
    const uint32_t part = lane & 3;
    const uint64_t m0 = __ballot(mod & 1u), m1 = __ballot(mod & 2u),
                   m2 = __ballot(mod & 4u), m3 = __ballot(mod & 8u);
    const uint64_t partmask = part == 0 ? m0 : part == 1 ? m1 : part == 2 ? m2 : m3;
    wave_lds_sync();
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t c = 64 * j + lane;
      if ((partmask >> (c >> 2)) & 1ull) tile_st(g, c, S[chunk_swz(c)]);
    }
    wave_lds_sync();  // the next tile overwrites S
  }
  if (bins.ent || rq.ent) __syncthreads();
  bins_publish<kOvf>(bins, cur, rb);
  if (rq.ent && threadIdx.x == 0) {
    const uint32_t c = cur[kCurReprobe];
    rq.cnt[rb] = c;
    if (c) atomicAdd(rq.total, c);
  }
}

// Wave-cooperative 64-byte row gather (wave-uniform call): lane L receives
// the 64 bytes at base + row_L * stride (row_L == kNone: zeros). Four lanes
// fetch each row as one contiguous request and the wave's LDS tile S
// (256 x 16 B) hands every lane its own row, as in frames64_tiles. A lane
// loading its own row as four 16-byte pieces costs four requests instead.
__device__ __forceinline__ void wave_gather64(const uint8_t *base, size_t stride,
                                              uint32_t row, uint4 *S, uint4 out[4]) {
  const uint32_t lane = threadIdx.x & 63;
  uint4 q[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t r = __shfl(row, 16 * j + (lane >> 2));
    q[j] = r != kNone
               ? reinterpret_cast<const uint4 *>(base + (size_t)r * stride)[lane & 3]
               : make_uint4(0, 0, 0, 0);
  }
  wave_lds_sync();  // earlier readers of S are done
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = q[j];
  wave_lds_sync();
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) out[k] = S[chunk_swz(4 * lane + k)];
}

// The inverse: the lanes with `st` store their 64 bytes at base + row * stride,
// four lanes per row.
__device__ __forceinline__ void wave_scatter64(uint8_t *base, size_t stride,
                                               uint32_t row, bool st, const uint4 v[4],
                                               uint4 *S) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t m = __ballot(st);
  if (!m) return;
  wave_lds_sync();
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) S[chunk_swz(4 * lane + k)] = v[k];
  wave_lds_sync();
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t c = 64 * j + lane;
    const uint32_t r = __shfl(row, c >> 2);
    if ((m >> (c >> 2)) & 1ull)
      reinterpret_cast<uint4 *>(base + (size_t)r * stride)[lane & 3] = S[chunk_swz(c)];
  }
}

// Reprobes: the packets a classify kernel queued because their home bucket
// held three other keys (touch == kReprobe), finished on the same register
// path with the probe walked on bucket by bucket (map_get's find_key,
// map-impl-pow2.c:629-732). Frames and buckets come in by wave_gather64, one
// request per row; finish() answering kReprobe again asks for the next bucket
// (it must leave no other trace in that case). Up to 64 packets per wave
// (act); wave-uniform call. Returns the lane's touch (kNone if none).
template <class Issue, class Finish>
__device__ __forceinline__ uint32_t reprobe_wave(uint8_t *frames, uint32_t slot,
                                                 const uint16_t *len,
                                                 const uint16_t *in_dev,
                                                 const uint8_t *buckets, uint32_t bmask,
                                                 uint32_t p, bool act, uint4 *S,
                                                 Issue issue, Finish finish,
                                                 uint32_t in0 = 0) {
  uint4 fr[4];
  wave_gather64(frames, slot, act ? p : kNone, S, fr);
  RFrame f;
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    f.w[4 * k] = fr[k].x;
    f.w[4 * k + 1] = fr[k].y;
    f.w[4 * k + 2] = fr[k].z;
    f.w[4 * k + 3] = fr[k].w;
  }
  const uint32_t in = act ? port_of(in_dev, in0, p) : 0u, ln = act ? len[p] : 0u;
  const auto pend = issue(p, f, in, ln, act);
  uint32_t want = act ? pend.row : kNone;
  bool live = act, mod = false;
  uint32_t touch = kNone;
  for (uint32_t step = 0;; step++) {
    uint4 row[4];
    wave_gather64(buckets, 64, live ? want : kNone, S, row);
    if (live) {
      touch = kNone;
      mod = finish(pend, row, p, f, in, ln, touch);
    }
    live = live && touch == kReprobe && step < bmask;
    if (!__ballot(live)) break;
    if (live) want = (want + 1) & bmask;
  }
#pragma unroll
  for (uint32_t k = 0; k < 4; k++)
    fr[k] = make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
  wave_scatter64(frames, slot, p, mod, fr, S);
  return touch == kReprobe ? kNone : touch;
}

// The reprobe queue: slice b holds cnt[b] packets at list + b * range (one
// slice per classify block), or with cnt == null slice b is the b-th run of
// `range` packets of one list of n.
__device__ __forceinline__ uint32_t reprobe_slice_len(const uint32_t *cnt, uint32_t n,
                                                      uint32_t range, uint32_t b) {
  return cnt ? cnt[b] : (n - b * range < range ? n - b * range : range);
}

// The reprobe kernels' loop: each block works whole slices, its waves 64
// packets at a time (`lane_fn(p, act)` runs reprobe_wave). The segment's
// touches were already folded into ts/tseq without these packets, so each
// touch raises tseq[i] to its sequence (atomicMax); tbl_reprobe_stamp then
// gives ts[i] the time of the packet that won (last toucher, exact).
template <class LaneFn>
__device__ __forceinline__ void reprobe_slices(const uint32_t *list, const uint32_t *cnt,
                                               uint32_t n, uint32_t range,
                                               uint32_t nblk, uint64_t *tseq,
                                               uint64_t seq_base, LaneFn lane_fn) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const uint32_t nb = reprobe_slice_len(cnt, n, range, b);
    for (uint32_t k0 = 64 * wv; k0 < nb; k0 += blockDim.x) {  // wave-uniform
      const uint32_t k = k0 + lane;
      const bool act = k < nb;
      const uint32_t p = act ? list[(size_t)b * range + k] : 0u;
      const uint32_t touch = lane_fn(p, act);
      if (touch != kNone)
        atomicMax(reinterpret_cast<unsigned long long *>(tseq + touch),
                  (unsigned long long)(seq_base + p));
    }
  }
}

// ------------------------------------------------------------ wide slots --
// Slots wider than 64 bytes (frames of 65-1518 B and mbuf-sized slots,
// DESIGN.md §5.4): the classify kernels keep each frame's first 64 bytes in
// registers, as for 64-byte slots, and take the rest of the L4 checksum's
// sum (nf-util.c:45-64: the L4 sum covers bytes [34, 14 + total_length) of an
// IHL-5 frame) from here: the raw sum of bytes [64, end) of every frame of
// the wave's tile (`end` = the lane's own frame's end, 64 = nothing).
//   G lanes per frame, 64 / G frames per load instruction, each lane 16
// contiguous bytes: a group reads 16 G contiguous bytes of one frame per
// instruction (256 B at G = 16). The steps are the wave's (frame batch,
// iteration) pairs flattened, U loads in flight; a frame batch's iterations
// cover the tile's longest tail, and loads past a frame's end go to an
// offset beyond the buffer resource (they return zeros and touch no memory).
// Loads use one buffer resource per tile (base in scalar registers) and
// 32-bit offsets, so no per-lane 64-bit addresses stay live. At a batch's
// last step the group's partial sums are added by xor shuffles and the
// frame's sum handed to its own lane. Returns that sum (< 2^27, unfolded).
__device__ __forceinline__ uint4 buf_ld16(const void *base, uint32_t bytes, uint32_t off) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes,
                                                    0x00020000);
  const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
  return make_uint4(x.x, x.y, x.z, x.w);
}
constexpr uint32_t kBufOff = 0x80000000u;  // an offset past every tile's resource

// One round's U loads of tile_tail_sums: the steps' frame ends (U
// bpermutes, one wait), then the loads (past a frame's end: kBufOff).
template <uint32_t G, uint32_t U>
struct TailRound {
  uint4 v[U];
  uint32_t rem[U];  // bytes of the frame from the lane's chunk on (0: none)
  __device__ __forceinline__ void issue(const uint8_t *tile, uint32_t slot, uint32_t bytes,
                                        uint32_t end, uint32_t k0, uint32_t K, uint32_t n_it,
                                        uint32_t &qq, uint32_t &ii, uint32_t gi, uint32_t gl) {
    constexpr uint32_t FPI = 64 / G;
    uint32_t off[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint32_t fr = qq * FPI + gi;
      const uint32_t o = 64 + 16 * (ii * G + gl);
      const uint32_t e = (uint32_t)__shfl((int)end, (int)fr);
      off[u] = fr * slot + o;
      rem[u] = ((k0 + u < K) & (o < e)) ? e - o : 0u;
      if (++ii == n_it) {
        ii = 0;
        qq++;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) v[u] = buf_ld16(tile, bytes, rem[u] ? off[u] : kBufOff);
  }
};

template <uint32_t G, uint32_t H = 1>  // H rounds of 8 loads in flight
__device__ __forceinline__ uint32_t tile_tail_sums(const uint8_t *tile, uint32_t slot,
                                                   uint32_t bytes, uint32_t end) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "lanes per frame");
  constexpr uint32_t FPI = 64 / G, U = 8;
  const uint32_t lane = threadIdx.x & 63, gl = lane % G, gi = lane / G;
  uint32_t mx = end;
#pragma unroll
  for (uint32_t m = 1; m < 64; m <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, m));
  // (wave-uniform: a scalar, so the step counters live in scalar registers)
  const uint32_t nch = __builtin_amdgcn_readfirstlane(mx > 64 ? (mx - 64 + 15) >> 4 : 0u);
  if (nch == 0) return 0;
  const uint32_t n_it = (nch + G - 1) / G, K = G * n_it;
  uint32_t tail = 0, acc = 0, q = 0, it = 0;  // (q, it): the next step's batch, iteration
  uint32_t qq = 0, ii = 0;                    // the next step to issue
  for (uint32_t k0 = 0; k0 < K; k0 += U * H) {
    TailRound<G, U> R[H];
#pragma unroll
    for (uint32_t h = 0; h < H; h++)
      R[h].issue(tile, slot, bytes, end, k0 + h * U, K, n_it, qq, ii, gi, gl);
#pragma unroll
    for (uint32_t h = 0; h < H; h++) {
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        if (k0 + h * U + u >= K) break;  // (wave-uniform)
        uint4 x = R[h].v[u];
        if (R[h].rem[u] < 16) x = chunk_keep(x, 0, (int)R[h].rem[u]);
        acc = sum16x4(x, acc);
        if (++it == n_it) {  // frame batch q complete: its sums to their lanes
          it = 0;
#pragma unroll
          for (uint32_t m = G / 2; m > 0; m >>= 1) acc += (uint32_t)__shfl_xor((int)acc, m);
          const uint32_t j = lane - q * FPI;  // this lane's frame in batch q (if < FPI)
          const uint32_t got = (uint32_t)__shfl((int)acc, (int)((j & (FPI - 1)) * G));
          if (j < FPI) tail = got;
          acc = 0;
          q++;
        }
      }
    }
  }
  return tail;
}

// Checksums of an IHL=5 frame whose first 64 bytes are in registers. With
// total_length <= 50 every byte the L4 sum covers lies in them; a longer
// frame (wide slots) brings the raw sum of its bytes [64, 14 + total_length)
// as `tail` (tile_tail_sums). Same arithmetic as set_checksums.
__device__ inline void fast_checksums(RFrame &f, uint32_t proto, uint32_t tl,
                                      uint32_t tail = 0) {
  f.set16(24, 0);
  if (proto == 6 || proto == 17) {
    const bool tcp = proto == 6;
    if (tcp) f.set16(50, 0); else f.set16(40, 0);
    uint32_t c = 0;
    if (tl >= 20) {
      const uint32_t L = tl - 20, end = 34 + L;
      uint32_t s = 0;
#pragma unroll
      for (int k = 0; k < 15; k++) {
        const int o = 34 + 2 * k;
        uint32_t word = f.u16at(o);
        uint32_t m = ((uint32_t)o + 2 <= end) ? 0xFFFFu
                     : (((uint32_t)o + 1 == end) ? 0xFFu : 0u);
        s += word & m;
      }
      s += tail;
      c = finish_l4(fold16(s), phdr_cksum(f.u32at2(26), f.u32at2(30),
                                          (uint8_t)proto, L));
    }
    if (tcp) f.set16(50, c); else f.set16(40, c);
  }
  uint32_t s = 0;
#pragma unroll
  for (int o = 14; o < 34; o += 2) s += f.u16at(o);
  f.set16(24, (~fold16(s)) & 0xFFFF);
}

// ------------------------------------------------------------------ CRC --
// The XOR of 13 position tables' entries (table j = 256 words at T + 256 j,
// T an LDS array), byte b_j for table j: the reads issued back to back and
// waited for once. (Compiled from an expression, each read waits for the one
// before it: 13 LDS round trips per packet.) viglb's and vigfw's flow hashes.
#define VP_CRC_RD(t, a, off) asm volatile("ds_read_b32 %0, %1 offset:" #off : "=v"(t) : "v"(a))
__device__ __forceinline__ uint32_t crc13_lds(const uint32_t *T, uint32_t b0, uint32_t b1,
                                              uint32_t b2, uint32_t b3, uint32_t b4,
                                              uint32_t b5, uint32_t b6, uint32_t b7,
                                              uint32_t b8, uint32_t b9, uint32_t b10,
                                              uint32_t b11, uint32_t b12) {
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)T;
  uint32_t t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12;
  VP_CRC_RD(t0, base + (b0 << 2), 0);
  VP_CRC_RD(t1, base + (b1 << 2), 1024);
  VP_CRC_RD(t2, base + (b2 << 2), 2048);
  VP_CRC_RD(t3, base + (b3 << 2), 3072);
  VP_CRC_RD(t4, base + (b4 << 2), 4096);
  VP_CRC_RD(t5, base + (b5 << 2), 5120);
  VP_CRC_RD(t6, base + (b6 << 2), 6144);
  VP_CRC_RD(t7, base + (b7 << 2), 7168);
  VP_CRC_RD(t8, base + (b8 << 2), 8192);
  VP_CRC_RD(t9, base + (b9 << 2), 9216);
  VP_CRC_RD(t10, base + (b10 << 2), 10240);
  VP_CRC_RD(t11, base + (b11 << 2), 11264);
  VP_CRC_RD(t12, base + (b12 << 2), 12288);
  // (the results as operands: nothing reads them before this wait)
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3), "+v"(t4), "+v"(t5), "+v"(t6),
                 "+v"(t7), "+v"(t8), "+v"(t9), "+v"(t10), "+v"(t11), "+v"(t12));
  return (t0 ^ t1 ^ t2) ^ (t3 ^ t4 ^ t5) ^ (t6 ^ t7 ^ t8) ^ (t9 ^ t10 ^ t11) ^ t12;
}
#undef VP_CRC_RD
// CRC-32C as SSE4.2 `crc32 r32` computes it (boilerplate-util.h:9): reflected
// polynomial 0x82F63B78, the operand's 4 LE bytes, no pre/post inversion.
__host__ __device__ inline uint32_t crc32c_byte(uint32_t crc, uint8_t b) {
  crc ^= b;
  for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
  return crc;
}
__host__ __device__ inline uint32_t crc32c_u32(uint32_t crc, uint32_t v) {
  for (int k = 0; k < 4; k++) crc = crc32c_byte(crc, (uint8_t)(v >> (8 * k)));
  return crc;
}

// Seed 0 and no final XOR make the chained hash GF(2)-linear in the message
// bytes, so a hash over a fixed field layout is the XOR of one 256-entry
// table per non-zero byte position: T_p[b] = CRC of the message whose only
// non-zero byte is b at position p. Built on the host, staged in LDS.
inline void build_position_table(uint32_t *tab, int pos, int msg_len) {
  for (int b = 0; b < 256; b++) {
    uint32_t c = 0;
    for (int k = pos; k < msg_len; k++)
      c = crc32c_byte(c, k == pos ? (uint8_t)b : 0);
    tab[b] = c;
  }
}

// ------------------------------------------------------------- flow slot --
// One 64-byte bucket of a device table (one aligned memory request): three
// entries, each a 16-byte key (reference struct layout, padding zero) and
// its dchain index (kEmpty / kTomb / index).
struct __align__(64) Bucket {
  uint32_t k[3][4];
  uint32_t idx[3];
  uint32_t pad;
};
constexpr uint32_t kBucketEntries = 3;

__device__ inline bool key_eq(const uint32_t a[4], const uint32_t b[4]) {
  return ((a[0] ^ b[0]) | (a[1] ^ b[1]) | (a[2] ^ b[2]) | (a[3] ^ b[3])) == 0;
}

// Wave-aggregated append: one atomic per wave for all active lanes that set
// `want`; returns this lane's position (valid only where want).
__device__ inline uint32_t wave_append(uint32_t *counter, bool want) {
  uint64_t mask = __ballot(want);
  if (mask == 0) return 0;
  uint32_t lane = __lane_id();
  uint32_t leader = __ffsll((unsigned long long)mask) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
  base = __shfl(base, leader);
  uint64_t below = mask & ((1ull << lane) - 1ull);
  return base + (uint32_t)__popcll(below);
}

}  // namespace vp
