// vigbridge on MI355X: MAC learning + forwarding lookup over a packet batch.
//
// Reference behaviour (paths relative to the reference repository):
//   nf_process                 vigbridge/bridge_main.c:311-329
//   expiry                     bridge_expire_entries, bridge_main.c:29-36
//                              (u32 wrap of expiration_time * 1000 as vignat)
//   learn src -> in port       bridge_put_update_entry, bridge_main.c:63-89
//                              (a known MAC is only rejuvenated; its port is
//                              not updated)
//   lookup {dst, in} static,   bridge_get_device, bridge_main.c:38-61
//   then dst dynamic; miss -> FLOOD_FRAME; -2 -> drop (return in port)
//   rte_ether_addr_hash        libvig/verified/ether.c:61-90 (6 CRC steps)
//   static table               read_static_ft_from_file, bridge_main.c:130-230
//
// Same segment scheme as vignat (vp_nat.hip header):
//   phase A  hash + probe src and dst; a known src is logged for
//            rejuvenation, an unknown one queued; a dst known at segment
//            start (or in the static table) is forwarded at once, an unknown
//            one flooded provisionally;
//   phase B  queued src MACs are de-duplicated (earliest packet wins) and
//            given dchain indices in packet order; the first sighting's in
//            port becomes the entry's port;
//   phase C  (only when B learned something) provisionally flooded frames are
//            looked up again: a MAC learned by a packet at or before this one
//            (the packet's own src counts: learn precedes lookup) forwards
//            there.
//
// Dynamic table entry: key words {mac[0..3], mac[4..5], port, 0}. Only words
// 0-1 identify the MAC; word 2 carries the DynamicValue (dyn_vals vector in
// the reference) so one bucket read resolves a lookup.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <vector>

#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(bridge)


// rte_ether_addr_hash: crc32c_u32 of each byte in turn, so the non-zero byte
// positions of the 24-byte CRC message are 0, 4, 8, 12, 16, 20.
constexpr int kEthTabs = 6;
// StaticKey hash (generated; nested struct field hashed by its own hash):
// crc(crc(0, ether_hash(addr)), device), an 8-byte message with non-zero
// bytes 0-3 (the MAC hash) and 4-5 (the u16 device).
constexpr int kStatTabs = 6;
constexpr int kBridgeTabs = kEthTabs + kStatTabs;

__device__ __forceinline__ uint32_t eth_hash(const uint32_t *T, uint32_t m0,
                                             uint32_t m1) {
  return T[0 * 256 + (m0 & 0xFF)] ^ T[1 * 256 + ((m0 >> 8) & 0xFF)] ^
         T[2 * 256 + ((m0 >> 16) & 0xFF)] ^ T[3 * 256 + (m0 >> 24)] ^
         T[4 * 256 + (m1 & 0xFF)] ^ T[5 * 256 + ((m1 >> 8) & 0xFF)];
}
__device__ __forceinline__ uint32_t static_hash(const uint32_t *T, uint32_t eh,
                                                uint32_t dev) {
  const uint32_t *S = T + kEthTabs * 256;
  return S[0 * 256 + (eh & 0xFF)] ^ S[1 * 256 + ((eh >> 8) & 0xFF)] ^
         S[2 * 256 + ((eh >> 16) & 0xFF)] ^ S[3 * 256 + (eh >> 24)] ^
         S[4 * 256 + (dev & 0xFF)] ^ S[5 * 256 + ((dev >> 8) & 0xFF)];
}

// eth_hash of two MACs, the 12 table reads issued back to back and waited
// for once (as vignat's flowid_hash_batched; T must be the kernel's LDS
// tables): *hs of src {s0, s1}, *hd of dst {d0, d1}.
__device__ __forceinline__ uint32_t bridge_lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
#define VP_ETH_RD(t, a, off) \
  asm volatile("ds_read_b32 %0, %1 offset:" #off : "=v"(t) : "v"(a))
__device__ __forceinline__ void eth_hash2(const uint32_t *T, uint32_t s0, uint32_t s1,
                                          uint32_t d0, uint32_t d1, uint32_t *hs,
                                          uint32_t *hd) {
  const uint32_t base = bridge_lds_addr(T);
  auto at = [&](uint32_t byte) { return base + (byte << 2); };
  uint32_t a0, a1, a2, a3, a4, a5, b0, b1, b2, b3, b4, b5;
  VP_ETH_RD(a0, at(s0 & 0xFF), 0);
  VP_ETH_RD(a1, at((s0 >> 8) & 0xFF), 1024);
  VP_ETH_RD(a2, at((s0 >> 16) & 0xFF), 2048);
  VP_ETH_RD(a3, at(s0 >> 24), 3072);
  VP_ETH_RD(a4, at(s1 & 0xFF), 4096);
  VP_ETH_RD(a5, at((s1 >> 8) & 0xFF), 5120);
  VP_ETH_RD(b0, at(d0 & 0xFF), 0);
  VP_ETH_RD(b1, at((d0 >> 8) & 0xFF), 1024);
  VP_ETH_RD(b2, at((d0 >> 16) & 0xFF), 2048);
  VP_ETH_RD(b3, at(d0 >> 24), 3072);
  VP_ETH_RD(b4, at(d1 & 0xFF), 4096);
  VP_ETH_RD(b5, at((d1 >> 8) & 0xFF), 5120);
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(b0),
                 "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5));
  *hs = (a0 ^ a1 ^ a2) ^ (a3 ^ a4 ^ a5);
  *hd = (b0 ^ b1 ^ b2) ^ (b3 ^ b4 ^ b5);
}
#undef VP_ETH_RD

// map_get on the dynamic table keyed by words 0-1, from bucket b on;
// *port = entry word 2.
__device__ __forceinline__ uint32_t mac_probe_from(const TableDev &t, uint32_t b,
                                                   uint32_t m0, uint32_t m1,
                                                   uint32_t *port) {
  for (uint32_t i = 0; i <= t.bmask; i++) {
    const uint4 *q = reinterpret_cast<const uint4 *>(t.bk + b);
    const uint4 k0 = q[0], k1 = q[1], k2 = q[2], ix = q[3];
    if (ix.x == kEmpty) return kNone;
    if (ix.x != kTomb && k0.x == m0 && k0.y == m1) {
      *port = k0.z;
      return ix.x;
    }
    if (ix.y == kEmpty) return kNone;
    if (ix.y != kTomb && k1.x == m0 && k1.y == m1) {
      *port = k1.z;
      return ix.y;
    }
    if (ix.z == kEmpty) return kNone;
    if (ix.z != kTomb && k2.x == m0 && k2.y == m1) {
      *port = k2.z;
      return ix.z;
    }
    b = (b + 1) & t.bmask;
  }
  return kNone;
}
__device__ __forceinline__ uint32_t mac_probe(const TableDev &t, uint32_t h,
                                              uint32_t m0, uint32_t m1,
                                              uint32_t *port) {
  return mac_probe_from(t, home_bucket(h, t.bmask, t.mix, t.lin), m0, m1, port);
}

struct BridgeArgs {
  const uint8_t *frames;
  const uint16_t *in_dev;
  uint16_t *out;
  uint32_t *log;
  uint64_t seq_base;
  uint32_t slot, p0, p1;
  TableDev t;
  TableDev st;  // static table: bk/bmask/mix only; idx = rule number
  const int32_t *st_val;
  uint32_t n_static;
  const uint32_t *crc_tab;
  uint32_t *miss;
  uint32_t *defer;
};

// nf_process's return value for a forwarding decision (bridge_main.c:322-328).
__device__ __forceinline__ uint16_t resolve(int32_t fwd, uint32_t in) {
  if (fwd == -1) return VP_FLOOD_FRAME;
  if (fwd == -2) return (uint16_t)in;
  return (uint16_t)fwd;
}

// Ethernet header words: dst = {w0, w1 & 0xFFFF}, src = {w1 >> 16 | w2 << 16,
// w2 >> 16} (bridge_main.c:312 borrows 14 bytes with no length check).
__device__ __forceinline__ uint4 eth_words(const BridgeArgs &a, uint32_t p) {
  return *reinterpret_cast<const uint4 *>(a.frames + (size_t)p * a.slot);
}

// One dynamic-table bucket against a MAC (words 0-1): the index and *port
// (entry word 2) on a match; kNone with *done on an empty entry; kNone with
// !*done when the probe continues in the next bucket. Entries in order, the
// first match or empty entry decides; branch-free with static indices (an
// early return per entry made the entry number dynamic and put the whole
// row in scratch memory: 64 B per packet of stores, the bridge's write
// traffic in round 2).
__device__ __forceinline__ uint32_t mac_match(const uint4 *row, uint32_t m0, uint32_t m1,
                                              uint32_t *port, bool *done) {
  const uint4 ix = row[3];
  const bool e0 = ix.x == kEmpty, e1 = ix.y == kEmpty, e2 = ix.z == kEmpty;
  const bool h0 = !e0 & (ix.x != kTomb) & (row[0].x == m0) & (row[0].y == m1);
  const bool h1 = !e1 & (ix.y != kTomb) & (row[1].x == m0) & (row[1].y == m1);
  const bool h2 = !e2 & (ix.z != kTomb) & (row[2].x == m0) & (row[2].y == m1);
  const bool t0 = h0 | e0, t1 = h1 | e1;
  const bool s1 = !t0 & h1, s2 = !t0 & !t1 & h2;
  // (masks, not a select: a select of row[e].z became a load through a
  // selected address, with the row in scratch memory again)
  const uint32_t z = (row[0].z & (0u - (uint32_t)h0)) | (row[1].z & (0u - (uint32_t)s1)) |
                     (row[2].z & (0u - (uint32_t)s2));
  if (h0 | s1 | s2) *port = z;
  *done = t0 | t1 | h2 | e2;
  return h0 ? ix.x : e0 ? kNone : h1 ? ix.y : e1 ? kNone : h2 ? ix.z : kNone;
}

// Phase A. Blocks own contiguous ranges of 64-packet tiles, their four waves
// interleaved (the frames64_tiles layout, so the launch can bin its touches:
// tbl_bins_plan); a lane takes one packet of its wave's tile. The src and
// dst home buckets are fetched together, four lanes per 64-byte row
// (wave-cooperative, one request per row), then handed to their lanes
// through LDS; a probe that continues past its home bucket walks on alone.
// W: waves per block (4; 16, one 1024-thread block per CU sharing one copy
// of the tables, bridge_classify_w: VIGPATH_BRIDGE_WAVES=16).
template <uint32_t W>
__device__ __forceinline__ void bridge_tiles(BridgeArgs a, TouchBins bins) {
  __shared__ uint32_t T[kBridgeTabs * 256 + 1024];  // + the layout's tables
  __shared__ uint4 stage[W][256];
  __shared__ uint32_t cur[kCurs];
  for (uint32_t i = threadIdx.x; i < kCurs; i += blockDim.x) cur[i] = 0;
  for (uint32_t i = threadIdx.x; i < kBridgeTabs * 256; i += blockDim.x)
    T[i] = a.crc_tab[i];
  const uint32_t *lin = T + kBridgeTabs * 256;
  if (a.t.mix == kMixLin)
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[kBridgeTabs * 256 + i] = a.t.lin[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint4 *S = stage[wv];
  const uint32_t first = a.p0 & ~63u;
  const uint32_t tiles = (a.p1 - first + 63) / 64;
  const uint32_t rb = blockIdx.x;
  const uint32_t per_b = (tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t tend = min(tiles, rb * per_b + per_b);
  const uint32_t range0 = first + rb * per_b * 64;
  const uint8_t *bk = reinterpret_cast<const uint8_t *>(a.t.bk);
  // the next tile's header chunk and port, requested behind this tile's rows
  // (prefetch: the header load's latency under this tile's work)
  uint4 hn = make_uint4(0, 0, 0, 0);
  uint32_t inn = 0;
  auto hfetch = [&](uint32_t tile) {
    const uint32_t p = first + tile * 64 + lane;
    if (p >= a.p0 && p < a.p1) {
      hn = eth_words(a, p);
      inn = a.in_dev[p];
    }
  };
  uint32_t tile = rb * per_b + wv;
  if (tile < tend) hfetch(tile);
  for (; tile < tend; tile += W) {  // wave-uniform
    const uint32_t p = first + tile * 64 + lane;
    const bool mine = p >= a.p0 && p < a.p1;
    const uint4 h = mine ? hn : make_uint4(0, 0, 0, 0);
    const uint32_t in = mine ? inn : 0u;
    const uint32_t d0 = h.x, d1 = h.y & 0xFFFF;
    const uint32_t s0 = (h.y >> 16) | (h.z << 16), s1 = h.z >> 16;
    uint32_t sh, dh;
    eth_hash2(T, s0, s1, d0, d1, &sh, &dh);
    // bridge_get_device: the static table first (bridge_main.c:38-61)
    int32_t st_fwd = 0;
    bool st_hit = false;
    if (a.n_static && mine) {
      const uint32_t key[4] = {d0, d1 | (in << 16), 0, 0};
      const uint32_t k = tbl_probe(a.st, static_hash(T, dh, in), key);
      if (k != kNone) {
        st_hit = true;
        st_fwd = a.st_val[k];
      }
    }
    // both home rows in flight at once: lane L fetches part L % 4 of the rows
    // of packet 16 j + L / 4, the row numbers by ds_bpermute issued together
    // and waited for once (as vignat's lean tile); kNone reads nothing
    const uint32_t sb = home_bucket(sh, a.t.bmask, a.t.mix, lin),
                   db = home_bucket(dh, a.t.bmask, a.t.mix, lin);
    const uint32_t vs = mine ? sb : kNone, vd = mine && !st_hit ? db : kNone;
    uint32_t r0, r1, r2, r3, r4, r5, r6, r7;
    const uint32_t src = lane & ~3u;  // byte address of lane L / 4
    asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(r0) : "v"(src), "v"(vs));
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:64" : "=v"(r1) : "v"(src), "v"(vs));
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:128" : "=v"(r2) : "v"(src), "v"(vs));
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:192" : "=v"(r3) : "v"(src), "v"(vs));
    asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(r4) : "v"(src), "v"(vd));
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:64" : "=v"(r5) : "v"(src), "v"(vd));
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:128" : "=v"(r6) : "v"(src), "v"(vd));
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:192" : "=v"(r7) : "v"(src), "v"(vd));
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6),
                   "+v"(r7));
    const uint32_t part = lane & 3;
    auto rowq = [&](uint32_t r) {
      return r != kNone ? reinterpret_cast<const uint4 *>(bk + (size_t)r * 64)[part]
                        : make_uint4(0, 0, 0, 0);
    };
    uint4 q[8] = {rowq(r0), rowq(r1), rowq(r2), rowq(r3),
                  rowq(r4), rowq(r5), rowq(r6), rowq(r7)};
    if (tile + W < tend) hfetch(tile + W);
    uint4 srow[4], drow[4];
    wave_lds_sync();
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = q[j];
    wave_lds_sync();
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) srow[k] = S[chunk_swz(4 * lane + k)];
    wave_lds_sync();
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = q[4 + j];
    wave_lds_sync();
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) drow[k] = S[chunk_swz(4 * lane + k)];
    uint32_t touch = kNone;
    if (mine) {
      // bridge_put_update_entry: a known src is rejuvenated, an unknown one
      // queued for phase B
      uint32_t unused = 0;
      bool done;
      uint32_t si = mac_match(srow, s0, s1, &unused, &done);
      if (!done) {
        TableDev t = a.t;
        si = mac_probe_from(t, (sb + 1) & t.bmask, s0, s1, &unused);
      }
      touch = si;
      log_put(a.log, p, si);  // kNone: phase B writes the real entry
      if (si == kNone) a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
      if (st_hit) {
        a.out[p] = resolve(st_fwd, in);
      } else {
        uint32_t port = 0;
        uint32_t di = mac_match(drow, d0, d1, &port, &done);
        if (!done) di = mac_probe_from(a.t, (db + 1) & a.t.bmask, d0, d1, &port);
        // unknown: flooded unless learned earlier in this segment (phase C
        // re-examines flooded frames only when phase B learned something)
        a.out[p] = di != kNone ? (uint16_t)port : VP_FLOOD_FRAME;
      }
    }
    bins_put(bins, cur, rb, per_b * 64, range0, p, touch);
  }
  __syncthreads();
  bins_publish(bins, cur, rb);
}

__global__ __launch_bounds__(256) void bridge_classify(BridgeArgs a, TouchBins bins) {
  bridge_tiles<4>(a, bins);
}
__global__ __launch_bounds__(1024, 1) void bridge_classify_w(BridgeArgs a, TouchBins bins) {
  bridge_tiles<16>(a, bins);
}

// Keys + hashes of the queued src MACs (packet order).
__global__ void bridge_miss_keys(BridgeArgs a, const uint32_t *list, uint32_t n,
                                 uint32_t *mkey, uint32_t *mhash) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint4 h = eth_words(a, list[j]);
    const uint32_t s0 = (h.y >> 16) | (h.z << 16), s1 = h.z >> 16;
    uint32_t *k = mkey + 4 * (size_t)j;
    k[0] = s0;
    k[1] = s1;
    k[2] = 0;
    k[3] = 0;
    mhash[j] = eth_hash(a.crc_tab, s0, s1);
  }
}

// Touch log for every queued src; the first sighting stores its in port as
// the entry's DynamicValue (bridge_main.c:80-84).
__global__ void bridge_learn_finish(BridgeArgs a, const uint32_t *list,
                                    uint32_t n, const uint32_t *scratch,
                                    const uint32_t *rep, const uint32_t *assign) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint32_t j0 = scratch[rep[j]];
    const uint32_t idx = assign[j0];
    a.log[p] = idx;  // kNone: table full, nothing learned (bridge_main.c:73-76)
    if (j0 == j && idx != kNone) {
      const uint32_t e = a.t.slot_of[idx];
      a.t.bk[e >> 2].k[e & 3][2] = a.in_dev[p];
    }
  }
}

// Phase C over the segment's flooded frames: a static rule (e.g. one that
// floods explicitly) still wins; otherwise a MAC learned by a packet q' <= p
// (the packet's own src is learned before its dst is looked up) forwards.
__global__ void bridge_defer_finish(BridgeArgs a) {
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += gridDim.x * blockDim.x) {
    if (a.out[p] != VP_FLOOD_FRAME) continue;
    const uint4 h = eth_words(a, p);
    const uint32_t d0 = h.x, d1 = h.y & 0xFFFF;
    const uint32_t dh = eth_hash(a.crc_tab, d0, d1);
    if (a.n_static) {
      const uint32_t in = a.in_dev[p];
      const uint32_t key[4] = {d0, d1 | (in << 16), 0, 0};
      if (tbl_probe(a.st, static_hash(a.crc_tab, dh, in), key) != kNone) continue;
    }
    uint32_t port = 0;
    const uint32_t di = mac_probe(a.t, dh, d0, d1, &port);
    if (di != kNone && tbl_allocated_before(a.t, di, a.seq_base + p + 1))
      a.out[p] = (uint16_t)port;
  }
}

// =============================================================== host ==

static inline int64_t bridge_cutoff(const vp_ctx *c, int64_t t) {
  const uint32_t e = c->brg.expiration_time * 1000u;  // u32, as vignat
  return (int64_t)((uint64_t)t - e);
}

static int bridge_segment(vp_ctx *c, const vp_dev_batch *b, const NowSpec &now,
                          uint32_t p0, uint32_t p1, float *ms, int *launches,
                          uint32_t *allocated) {
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  BridgeArgs a{};
  a.frames = b->frames;
  a.in_dev = b->in_dev;
  a.out = b->out_dev;
  a.log = w.log;
  a.seq_base = c->seq;
  a.slot = b->slot;
  a.p0 = p0;
  a.p1 = p1;
  a.t = tbl_dev(t);
  a.st = TableDev{};
  a.st.bk = c->st_bk;
  a.st.bmask = c->st_bmask;
  a.st.mix = kMixMul;
  a.st_val = c->st_val;
  a.n_static = c->n_static;
  a.crc_tab = c->crc_tab;
  a.miss = w.miss;
  a.defer = w.defer;

  // the classify launch bins its touches when it can (TouchBins; no touch
  // log then), else logs them and the log is folded
  BinsPlan bp{};
  static const uint32_t bw = [] {  // waves per block (VIGPATH_BRIDGE_WAVES: 4 or 16)
    const char *e = getenv("VIGPATH_BRIDGE_WAVES");
    return e && atoi(e) == 16 ? 16u : 4u;
  }();
  const void *bk = bw == 16 ? (const void *)bridge_classify_w : (const void *)bridge_classify;
  VP_TRY(tbl_bins_plan(c, t, bk, p0, p1, &bp, bw, 8));
  const uint32_t tiles = (p1 - (p0 & ~63u) + 63) / 64;
  const uint32_t grid = bp.on ? bp.grid : resident_grid(bk, (tiles + bw - 1) / bw, 64 * (int)bw);
  // (still zero after a segment that learned nothing: no reset launch)
  if (!t.ctl_clean) VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 16, c->stream));  // .. touch_ovf
  t.ctl_clean = false;
  VP_HIP(ev_record(c->ktime, c->ev0, c->stream));
  BridgeArgs a1 = a;
  if (bp.on) a1.log = nullptr;
  c->last_kernel = bw == 16 ? "bridge_classify_w" : "bridge_classify";
  if (bw == 16)
    bridge_classify_w<<<grid, 1024, 0, c->stream>>>(a1, bp.bins);
  else
    bridge_classify<<<grid, 256, 0, c->stream>>>(a1, bp.bins);
  VP_HIP(hipGetLastError());
  VP_HIP(ev_record(c->ktime, c->ev1, c->stream));
  VP_TRY(tbl_fold_read_ctl(c, t, bp, w.log, p0, p1, now, c->seq));
  float kms = 0.f;
  VP_HIP(ev_ms(c->ktime, c->ev0, c->ev1, &kms));
  *ms += kms;
  *launches += 1;
  const bool ovf = bp.on && t.h_ctl.touch_ovf != 0;
  if (ovf)  // touches that found their bin slice full, logged alone
    VP_TRY(tbl_late_touches(c, t, bp.bins.oent, bp.bins.ocnt, 0, bp.range, bp.grid,
                            w.log, now, c->seq));
  const uint32_t nmiss = t.h_ctl.miss_count;
  // nothing learned: provisional floods stand; only the fold may still run
  // (not when it reads the caller's time array)
  c->fold_pending = !nmiss && !ovf && !b->now;
  t.ctl_clean = !nmiss && !ovf;
  if (!nmiss) return 0;

  size_t need = 0;
  hipcub::DeviceRadixSort::SortKeys(nullptr, need, w.miss, w.miss_sorted,
                                    (int)nmiss, 0, 32, c->stream);
  VP_TRY(cub_reserve(c, need));
  VP_HIP(hipcub::DeviceRadixSort::SortKeys(w.cub_tmp, w.cub_bytes, w.miss,
                                           w.miss_sorted, (int)nmiss, 0, 32,
                                           c->stream));
  bridge_miss_keys<<<grid_for(nmiss), 256, 0, c->stream>>>(a, w.miss_sorted, nmiss,
                                                           w.mkey, w.mhash);
  VP_HIP(hipGetLastError());
  VP_TRY(tbl_new_keys(c, t, NewKeys{nmiss, w.miss_sorted}, c->seq, nullptr));
  a.t = tbl_dev(t);  // a rebuild may have changed the layout
  bridge_learn_finish<<<grid_for(nmiss), 256, 0, c->stream>>>(
      a, w.miss_sorted, nmiss, w.scratch, w.rep, w.assign);
  VP_HIP(hipGetLastError());
  bridge_defer_finish<<<grid_for(p1 - p0), 256, 0, c->stream>>>(a);
  VP_HIP(hipGetLastError());
  *allocated |= 1u;
  // the learning packets' touches on top of the fold (last toucher wins)
  VP_TRY(tbl_late_touches(c, t, w.miss_sorted, nullptr, nmiss, 256, (nmiss + 255) / 256,
                          w.log, now, c->seq));
  VP_TRY(read_ctl(c, t));
  return 0;
}

int bridge_process_device(vp_ctx *c, const vp_dev_batch *b) {
  ExpiringTable tabs[1] = {{&c->ft, bridge_cutoff}};
  return run_batch(c, b, tabs, 1, bridge_segment);
}

void build_bridge_tables(std::vector<uint32_t> &tab) {
  tab.assign(kBridgeTabs * 256, 0);
  for (int j = 0; j < kEthTabs; j++)
    build_position_table(&tab[j * 256], 4 * j, 24);
  for (int j = 0; j < kStatTabs; j++)
    build_position_table(&tab[(kEthTabs + j) * 256], j, 8);
}

// Static table (read_static_ft_from_file): rule k keyed {mac, (u16)from},
// value `to`. Built on the host into the device bucket layout. A repeated key
// keeps the first rule: the reference's map_put appends the duplicate
// further along the same probe path, so map_get finds the first.
int bridge_static_build(const vp_bridge_config *cfg, std::vector<Bucket> &bk,
                        uint32_t *bmask) {
  uint32_t nb = 64;
  while ((uint64_t)nb * kBucketEntries < 2ull * cfg->n_static) nb <<= 1;
  bk.assign(nb, Bucket{});
  for (auto &x : bk)
    for (uint32_t e = 0; e < kBucketEntries; e++) x.idx[e] = kEmpty;
  *bmask = nb - 1;
  std::vector<uint32_t> tab;
  build_bridge_tables(tab);
  const uint32_t *E = tab.data(), *S = tab.data() + kEthTabs * 256;
  for (uint32_t r = 0; r < cfg->n_static; r++) {
    const vp_bridge_rule &R = cfg->static_rules[r];
    const uint32_t m0 = R.mac[0] | (R.mac[1] << 8) | (R.mac[2] << 16) |
                        ((uint32_t)R.mac[3] << 24);
    const uint32_t m1 = R.mac[4] | (R.mac[5] << 8);
    const uint32_t dev = (uint16_t)R.device_from;
    const uint32_t key[4] = {m0, m1 | (dev << 16), 0, 0};
    uint32_t eh = 0;
    for (int j = 0; j < 6; j++) eh ^= E[j * 256 + R.mac[j]];
    const uint32_t h = S[0 * 256 + (eh & 0xFF)] ^ S[1 * 256 + ((eh >> 8) & 0xFF)] ^
                       S[2 * 256 + ((eh >> 16) & 0xFF)] ^ S[3 * 256 + (eh >> 24)] ^
                       S[4 * 256 + (dev & 0xFF)] ^ S[5 * 256 + (dev >> 8)];
    uint32_t b = home_bucket(h, *bmask, kMixMul);
    bool placed = false;
    while (!placed) {
      for (uint32_t e = 0; e < kBucketEntries && !placed; e++) {
        Bucket &x = bk[b];
        if (x.idx[e] == kEmpty) {
          memcpy(x.k[e], key, 16);
          x.idx[e] = r;
          placed = true;
        } else if (!memcmp(x.k[e], key, 16)) {
          placed = true;  // duplicate: the first rule stays visible
        }
      }
      b = (b + 1) & *bmask;
    }
  }
  return 0;
}

}  // namespace vp
