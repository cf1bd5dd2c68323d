// vigpol on MI355X: batch classification + per-destination token buckets.
//
// Reference behaviour (paths relative to the reference repository):
//   nf_process            vigpol/policer_main.c:120-145
//   policer_check_tb      vigpol/policer_main.c:34-111
//   expiry                vigpol/policer_main.c:21-32 (only for packets whose
//                         IPv4 header parsed: nf_process returns before it
//                         otherwise)
//   state                 vigpol/dataspec.ml:5-11 (dyn_map, dyn_keys,
//                         dyn_heap, dyn_vals)
// Same segment structure as the other NFs, one more phase:
//   phase A  parse; LAN packets go out on the WAN device, packets from other
//            devices and non-IPv4 frames are dropped; WAN packets look their
//            destination address up: a hit is recorded, a miss is queued
//            (sizes <= burst may allocate, larger ones may not);
//   phase B  allocating misses: de-duplicated, ranked and given dchain
//            indices in packet order (tbl_new_keys); a later packet of an
//            allocated address is a hit of that index;
//   phase C  misses larger than the burst: a hit iff an earlier packet of the
//            segment allocated their address, dropped otherwise;
//   phase T  token buckets: every policed packet (index known) is grouped
//            by index in packet order and one lane per index replays its
//            packets through policer_check_tb's arithmetic in order. The
//            bucket is a serial recurrence per address (refill, clamp,
//            conditional take), so it is replayed, not scanned. Grouping:
//            phase A counts hits per index (atomicAdd: the packet's rank in
//            its run, in arbitrary order); when the segment had no misses
//            and no run is longer than kRunMax, a scan + scatter groups the
//            runs and each lane puts its run back in packet order (insertion
//            sort of <= kRunMax positions); otherwise a stable radix sort of
//            (index, packet) pairs does it.
// Frames are never written (the policer only decides the output device).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <vector>

#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(pol)


int ws_reserve(vp_ctx *c, uint32_t n);  // vp_runtime.hip

// ip_addr_hash (generated for vigpol/ip_addr.h:6-8): crc32c_u32(0, addr);
// four byte-position tables of a 4-byte message.
constexpr uint32_t kPolTabs = 4;
constexpr uint64_t kNsPerS = 1000000000ull;  // VIGOR_TIME_SECONDS_MULTIPLIER

__device__ __forceinline__ uint32_t pol_hash(const uint32_t *T, uint32_t a) {
  return T[a & 0xFF] ^ T[256 + ((a >> 8) & 0xFF)] ^ T[512 + ((a >> 16) & 0xFF)] ^
         T[768 + (a >> 24)];
}

struct PolArgs {
  const uint8_t *frames;
  const uint16_t *len;
  const uint16_t *in_dev;
  uint16_t *out;
  uint32_t *pidx;  // policed packets: their index (kNone otherwise); every
                   // policed packet rejuvenates it (policer_main.c:38)
  uint64_t seq_base;
  uint32_t slot, p0, p1;
  TableDev t;
  const uint32_t *crc_tab;
  uint32_t *miss;   // allocating misses (size <= burst)
  uint32_t *defer;  // misses larger than the burst
  uint64_t burst, rate, thr;  // thr = burst * 1e9 / rate (u64, as the reference)
  uint32_t *cnt;     // hits per index in this segment (phase A)
  uint32_t *rnk;     // a hit's rank in its index's run (arbitrary order)
  uint32_t *runs;    // or (non-null) the hit's position straight into its
                     // index's run slots: runs[rank * cap + index] (rank-major:
                     // a tile of packets with consecutive indices writes
                     // consecutive slots, and the replay lanes read them so)
  uint32_t *runover; // set when a run is longer than kRunMax (ctl->aux_count)
  uint16_t lan, wan;
};

constexpr uint32_t kRunMax = 64;  // longest run the grouping path sorts per lane

// nf_then_get_rte_ipv4_header (nf-util.h:122-151): the dst address offset,
// or 0 when the header does not parse.
__device__ __forceinline__ uint32_t pol_ipv4(const GFrame &f, uint32_t total) {
  const uint16_t unread = (uint16_t)(total - 14);
  if (!(f.r16(12) == bswap16(0x0800)) | (unread < 20)) return 0;
  const uint8_t ihl = f.r8(14) & 0x0F;
  if ((ihl < 5) | (unread < bswap16(f.r16(16)))) return 0;
  return 14 + 16;
}

// The same predicate on a slot's first 48 bytes in three 16-byte loads
// (slots are >= 64 B and 16-B aligned): the dst address, or 0.
__device__ __forceinline__ uint32_t pol_ipv4_w(const uint4 *s, uint32_t total,
                                               uint32_t *dst) {
  const uint4 h0 = s[0], h1 = s[1], h2 = s[2];
  const uint16_t unread = (uint16_t)(total - 14);
  const uint32_t ihl = (h0.w >> 16) & 0x0F;
  const uint16_t tl = bswap16((uint16_t)(h1.x & 0xFFFF));
  *dst = (h1.w >> 16) | (h2.x << 16);  // bytes 30-33
  return ((h0.w & 0xFFFF) == 0x0008) & (unread >= 20) & (ihl >= 5) & (unread >= tl);
}

// Phase A: one packet per lane.
__global__ __launch_bounds__(256) void pol_classify(PolArgs a) {
  __shared__ uint32_t T[kPolTabs * 256];
  for (uint32_t i = threadIdx.x; i < kPolTabs * 256; i += blockDim.x)
    T[i] = a.crc_tab[i];
  __syncthreads();
  bool over = false;
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += gridDim.x * blockDim.x) {
    const uint32_t in = a.in_dev[p], len = a.len[p];
    uint32_t dst;
    const bool v4 = pol_ipv4_w(
        reinterpret_cast<const uint4 *>(a.frames + (size_t)p * a.slot), len, &dst);
    a.pidx[p] = kNone;
    if (!v4) {  // not IPv4: dropped before the expiry (policer_main.c:126-130)
      a.out[p] = (uint16_t)in;
      continue;
    }
    if (in == a.lan) {  // outgoing: not policed (policer_main.c:134-136)
      a.out[p] = a.wan;
      continue;
    }
    if (in != a.wan) {  // unknown port (policer_main.c:141-144)
      a.out[p] = (uint16_t)in;
      continue;
    }
    const uint32_t key[4] = {dst, 0, 0, 0};
    const uint32_t idx = tbl_probe(a.t, pol_hash(T, dst), key);
    if (idx != kNone) {
      a.pidx[p] = idx;
      if (a.cnt) {  // grouping path: this hit's rank in its index's run
        const uint32_t r = atomicAdd(&a.cnt[idx], 1u);
        if (a.runs) {
          if (r < kRunMax) a.runs[(size_t)r * a.t.cap + idx] = p;
        } else {
          a.rnk[p] = r;
        }
        over |= r >= kRunMax;
      }
    } else if (len <= a.burst) {
      a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
    } else {
      a.defer[wave_append(&a.t.ctl->defer_count, true)] = p;
    }
  }
  if (__ballot(over) && __lane_id() == 0) *a.runover = 1;
}

// Phase A for 64-byte slots (frames64_tiles, vp_device.h): every frame load
// moves 1 KiB contiguous through the wave's LDS tile, the home buckets come
// in by cooperative 64-byte row gathers, and the CRC and layout tables sit in
// LDS; frames are never written back. A bucket full of other keys finishes
// its probe walk in the lane (tbl_probe_from: rare, load <= 1/3).
struct PolPend {
  uint32_t row;  // home bucket (gathered by frames64_tiles) or kNone
  uint32_t dst;  // the policed destination address (row != kNone)
};
__global__ __launch_bounds__(256, 4) void pol_classify64(PolArgs a, uint32_t n_all) {
  __shared__ uint32_t T[kPolTabs * 256 + 1024];
  __shared__ uint4 stage[4][256];
  __shared__ uint32_t cur[kCurs];
  for (uint32_t i = threadIdx.x; i < kPolTabs * 256; i += blockDim.x) T[i] = a.crc_tab[i];
  if (a.t.mix == kMixLin)
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[kPolTabs * 256 + i] = a.t.lin[i];
  for (uint32_t i = threadIdx.x; i < kCurs; i += blockDim.x) cur[i] = 0;
  __syncthreads();
  const uint32_t *lin = T + kPolTabs * 256;
  bool over = false;
  frames64_tiles(
      const_cast<uint8_t *>(a.frames), a.len, a.in_dev, a.p0, a.p1, n_all,
      stage[threadIdx.x >> 6], reinterpret_cast<const uint4 *>(a.t.bk),
      [&](uint32_t p, const RFrame &f, uint32_t in, uint32_t len, bool mine) {
        PolPend P{kNone, 0};
        if (!mine) return P;
        // nf_then_get_rte_ipv4_header (nf-util.h:122-151), as pol_ipv4_w
        const uint16_t unread = (uint16_t)(len - 14);
        const uint32_t ihl = (f.w[3] >> 16) & 0x0F;
        const uint16_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
        const bool v4 = ((f.w[3] & 0xFFFF) == 0x0008) & (unread >= 20) & (ihl >= 5) &
                        (unread >= tl);
        if (!v4 || in != a.wan) {  // dropped / outgoing / unknown port
          a.pidx[p] = kNone;
          a.out[p] = (uint16_t)(v4 && in == a.lan ? a.wan : in);
          return P;
        }
        P.dst = f.u32at2(30);
        P.row = home_bucket(pol_hash(T, P.dst), a.t.bmask, a.t.mix, lin);
        return P;
      },
      [&](const PolPend &P, const uint4 *row, uint32_t p, RFrame &, uint32_t,
          uint32_t len, uint32_t &) -> uint32_t {
        if (P.row == kNone) return 0u;
        const uint32_t key[4] = {P.dst, 0, 0, 0};
        bool done;
        uint32_t idx = bucket_match(row[0], row[1], row[2], row[3], key, &done);
        if (!done) idx = tbl_probe_from(a.t, (P.row + 1) & a.t.bmask, key, a.t.bmask);
        a.pidx[p] = idx;
        if (idx != kNone) {
          if (a.cnt) {  // grouping path: this hit's rank in its index's run
            const uint32_t r = atomicAdd(&a.cnt[idx], 1u);
            if (a.runs) {
              if (r < kRunMax) a.runs[(size_t)r * a.t.cap + idx] = p;
            } else {
              a.rnk[p] = r;
            }
            over |= r >= kRunMax;
          }
        } else if (len <= a.burst) {
          a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
        } else {
          a.defer[wave_append(&a.t.ctl->defer_count, true)] = p;
        }
        return 0u;  // (the policer never writes frames)
      },
      TouchBins{}, TileQueue{}, cur);
  if (__ballot(over) && __lane_id() == 0) *a.runover = 1;
}

// ------------------------------------------------------------- phase B --

__global__ void pol_miss_keys(PolArgs a, const uint32_t *list, uint32_t n,
                              uint32_t *mkey, uint32_t *mhash) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const GFrame f{const_cast<uint8_t *>(a.frames) + (size_t)p * a.slot, a.slot};
    const uint32_t dst = f.r32(30);
    uint32_t *k = mkey + 4 * (size_t)j;
    k[0] = dst;
    k[1] = k[2] = k[3] = 0;
    mhash[j] = pol_hash(a.crc_tab, dst);
  }
}

// Allocating misses: the first sighting of an address took a free index (or
// the table was full: dropped, policer_main.c:84-89); later sightings are
// hits of that index.
__global__ void pol_miss_finish(PolArgs a, const uint32_t *list, uint32_t n,
                                const uint32_t *scratch, const uint32_t *rep,
                                const uint32_t *assign) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint32_t idx = assign[scratch[rep[j]]];
    if (idx == kNone) {
      a.out[p] = a.wan;
      continue;
    }
    a.pidx[p] = idx;
  }
}

// ------------------------------------------------------------- phase C --
// Misses larger than the burst (policer_main.c:79-82): a hit iff an earlier
// packet of the segment allocated the address.
__global__ void pol_defer_finish(PolArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const GFrame f{const_cast<uint8_t *>(a.frames) + (size_t)p * a.slot, a.slot};
    const uint32_t dst = f.r32(30);
    const uint32_t key[4] = {dst, 0, 0, 0};
    const uint32_t idx = tbl_probe(a.t, pol_hash(a.crc_tab, dst), key);
    if (idx == kNone || !tbl_allocated_before(a.t, idx, a.seq_base + p)) {
      a.out[p] = a.wan;
      continue;
    }
    a.pidx[p] = idx;
  }
}

// ------------------------------------------------------------- phase T --

// Sort keys: the packet's index, or `cap` (sorts last) when not policed.
__global__ void pol_sort_keys(const uint32_t *pidx, uint32_t p0, uint32_t n,
                              uint32_t cap, uint32_t *key) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x) {
    const uint32_t k = pidx[p0 + i];
    key[i] = k == kNone ? cap : k;
  }
}

// One lane per run of equal indices in the sorted list: policer_check_tb's
// bucket arithmetic over the run's packets in packet order. The run's first
// packet is the allocation when the index was born at it
// (policer_main.c:91-100: bucket = burst - size, time = now). The run's last
// packet is the index's last rejuvenation: the lane stamps ts/tseq itself
// (no touch-log fold for vigpol).
// N > 0: the loop unrolled N times (c <= N), so a run held in an N-element
// register array is indexed statically (a dynamically indexed array lives in
// scratch memory: per-lane stores and loads through the caches).
template <uint32_t N = 0, class Next>
__device__ __forceinline__ void pol_replay(const PolArgs &a, uint32_t k,
                                           uint32_t c, Next next, const NowSpec &now,
                                           uint64_t *bsize, int64_t *btime) {
  uint64_t size = bsize[k];
  uint64_t btu = (uint64_t)btime[k];
  uint32_t p = 0;
  auto step = [&](uint32_t j) {
    p = next(j);
    const uint64_t len = a.len[p];
    const uint64_t tu = (uint64_t)now.at(p);
    bool fwd;
    if (j == 0 && a.t.birth[k] == a.seq_base + p) {
      size = a.burst - len;  // new flow: forwarded (policer_main.c:91-103)
      fwd = true;
    } else {  // policer_main.c:39-72
      const uint64_t diff = tu - btu;
      if (diff < a.thr) {
        size += diff * a.rate / kNsPerS;
        if (size > a.burst) size = a.burst;
      } else {
        size = a.burst;
      }
      fwd = size > len;
      if (fwd) size -= len;
    }
    btu = tu;
    a.out[p] = fwd ? a.lan : a.wan;
  };
  if constexpr (N > 0) {
#pragma unroll
    for (uint32_t j = 0; j < N; j++)
      if (j < c) step(j);
  } else {
    for (uint32_t j = 0; j < c; j++) step(j);
  }
  bsize[k] = size;
  btime[k] = (int64_t)btu;
  a.t.ts[k] = btu;
  a.t.tseq[k] = a.seq_base + p;
}

// Sorted (index, packet) pairs: one lane per run.
__global__ void pol_buckets(PolArgs a, const uint32_t *skey, const uint32_t *sval,
                            uint32_t n, uint32_t cap, NowSpec now,
                            uint64_t *bsize, int64_t *btime) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x) {
    const uint32_t k = skey[i];
    if (k >= cap || (i > 0 && skey[i - 1] == k)) continue;
    uint32_t c = 1;
    while (i + c < n && skey[i + c] == k) c++;
    pol_replay(a, k, c, [&](uint32_t j) { return sval[i + j]; }, now, bsize, btime);
  }
}

// The grouping path applies when phase A found no misses and no run longer
// than kRunMax. Its kernels are enqueued right behind phase A, before the
// host has read the counts back, and check them on the device: in steady
// state the replay overlaps the control read-back instead of following it.
__device__ __forceinline__ bool pol_grouping_ok(const Ctl *ctl) {
  return (ctl->miss_count | ctl->defer_count | ctl->aux_count) == 0;
}

// Grouping path: hits scattered to their index's run (off = exclusive scan
// of cnt), in arbitrary order inside the run.
__global__ void pol_scatter(const uint32_t *pidx, const uint32_t *rnk, uint32_t p0,
                            uint32_t p1, const uint32_t *off, uint32_t *grouped,
                            const Ctl *ctl) {
  if (!pol_grouping_ok(ctl)) return;
  for (uint32_t p = p0 + blockIdx.x * blockDim.x + threadIdx.x; p < p1;
       p += gridDim.x * blockDim.x) {
    const uint32_t k = pidx[p];
    if (k != kNone) grouped[off[k] + rnk[p]] = p;
  }
}

// One lane per index with hits: its run (<= kRunMax positions) put back in
// packet order by an insertion sort, then replayed. The run is at
// grouped + off[k] (scan + scatter) or, off == null, in the index's slots
// that phase A filled (rank-major: slot j at grouped[j * cap + k]); the
// lane clears the index's count for the next segment. The first thread
// publishes phase A's control block to the host (ctl_publish), which learns
// the counts while the replay runs.
__global__ void pol_runs(PolArgs a, uint32_t *cnt, const uint32_t *off,
                         const uint32_t *grouped, uint32_t cap, NowSpec now,
                         uint64_t *bsize, int64_t *btime, PubArgs pub) {
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl_publish(pub);
  if (!pol_grouping_ok(a.t.ctl)) return;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < cap;
       k += gridDim.x * blockDim.x) {
    const uint32_t c = cnt[k];
    if (c == 0) continue;
    cnt[k] = 0;
    if (!off && c <= 8) {
      // short runs (the common case: a batch revisits each address a few
      // times) in registers: padded with ~0, sorted by an odd-even
      // transposition network, replayed with static indices
      uint32_t r[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) r[j] = j < c ? grouped[(size_t)j * cap + k] : ~0u;
#pragma unroll
      for (uint32_t round = 0; round < 8; round++)
#pragma unroll
        for (uint32_t j = round & 1; j + 1 < 8; j += 2) {
          const uint32_t lo = min(r[j], r[j + 1]), hi = max(r[j], r[j + 1]);
          r[j] = lo;
          r[j + 1] = hi;
        }
      pol_replay<8>(a, k, c, [&](uint32_t j) { return r[j]; }, now, bsize, btime);
      continue;
    }
    uint32_t q[kRunMax];
    for (uint32_t j = 0; j < c; j++) {
      const uint32_t v = off ? grouped[off[k] + j] : grouped[(size_t)j * cap + k];
      uint32_t i = j;
      while (i > 0 && q[i - 1] > v) {
        q[i] = q[i - 1];
        i--;
      }
      q[i] = v;
    }
    pol_replay(a, k, c, [&](uint32_t j) { return q[j]; }, now, bsize, btime);
  }
}

// The last packet of [0, n) whose IPv4 header parses (-1 if none): packets
// after it run no expiry (policer_main.c:124-132). One block walks back from
// the end 256 packets at a time.
__global__ __launch_bounds__(256) void pol_last_ipv4(const uint8_t *frames,
                                                     uint32_t slot,
                                                     const uint16_t *len,
                                                     uint32_t n, int32_t *out) {
  __shared__ int32_t found;
  if (threadIdx.x == 0) found = -1;
  __syncthreads();
  for (int64_t base = (int64_t)n - 1; base >= 0; base -= blockDim.x) {
    const int64_t p = base - threadIdx.x;
    if (p >= 0) {
      const GFrame f{const_cast<uint8_t *>(frames) + (size_t)p * slot, slot};
      if (pol_ipv4(f, len[p])) atomicMax(&found, (int32_t)p);
    }
    __syncthreads();
    if (found >= 0) break;
  }
  if (threadIdx.x == 0) *out = found;
}

// =============================================================== host ==

// policer_expire_entries (policer_main.c:21-32): exp_time and the cutoff in
// unsigned 64-bit arithmetic.
static inline int64_t pol_cutoff(const vp_ctx *c, int64_t t) {
  const uint64_t exp_time = kNsPerS * c->pol.burst / c->pol.rate;
  return (int64_t)((uint64_t)t - exp_time);
}

// The grouping path's run slots (kRunMax per index: 1 GiB at 4M indices),
// allocated once, by the first segment that groups, for tables up to 4M
// indices; a failed allocation leaves the scan + scatter grouping path
// (pol_runs null), which needs no slots.
static int pol_runs_reserve(vp_ctx *c) {
  if (c->pol_runs_tried) return 0;
  c->pol_runs_tried = true;
  const uint32_t cap = c->ft.cap;
  if (cap > (1u << 22)) return 0;
  const hipError_t e = hipMalloc((void **)&c->pol_runs, sizeof(uint32_t) * kRunMax * cap);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    c->pol_runs = nullptr;
  }
  return 0;
}

static int pol_segment(vp_ctx *c, const vp_dev_batch *b, const NowSpec &now,
                       uint32_t p0, uint32_t p1, float *ms, int *launches,
                       uint32_t *allocated) {
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  PolArgs a{};
  a.frames = b->frames;
  a.len = b->len;
  a.in_dev = b->in_dev;
  a.out = b->out_dev;
  a.pidx = w.log;
  const uint64_t seq0 = c->seq;
  a.seq_base = seq0;
  a.slot = b->slot;
  a.p0 = p0;
  a.p1 = p1;
  a.t = tbl_dev(t);
  a.crc_tab = c->crc_tab;
  a.miss = w.miss;
  a.defer = w.defer;
  a.burst = c->pol.burst;
  a.rate = c->pol.rate;
  a.thr = c->pol.burst * kNsPerS / c->pol.rate;
  a.lan = c->pol.lan_device;
  a.wan = c->pol.wan_device;
  a.rnk = w.aux;
  a.runover = &t.ctl->aux_count;
  const uint32_t n = p1 - p0;
  // The grouping path costs O(capacity) per segment (clear, scan and one
  // lane per index); segments much shorter than the table (per-packet
  // nf_process calls, churn cut into many segments) take the sorting path.
  const bool grouping = (uint64_t)n * 8 >= t.cap;
  if (grouping) VP_TRY(pol_runs_reserve(c));
  a.cnt = grouping ? c->pol_cnt : nullptr;
  a.runs = grouping ? c->pol_runs : nullptr;

  // the counters (and the hit counts) are still zero after a segment whose
  // phase A queued nothing and whose replay cleared its counts
  if (!t.ctl_clean) {
    VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 16, c->stream));  // .. reprobe
    VP_HIP(hipMemsetAsync(a.runover, 0, 4, c->stream));
  }
  if (grouping && !c->pol_cnt_clean)
    VP_HIP(hipMemsetAsync(c->pol_cnt, 0, 4ull * t.cap, c->stream));
  t.ctl_clean = false;
  c->pol_cnt_clean = false;
  const uint32_t epoch = ++t.pub_epoch;  // phase A's counts, published by pol_runs
  const PubArgs pub{t.d_pub, t.ctl, epoch, nullptr, nullptr, 0, 0};
  VP_HIP(ev_record(c->ktime, c->ev0, c->stream));
  if (b->slot == 64 && c->coalesced_io) {
    const uint32_t tiles = (p1 - (p0 & ~63u) + 63) / 64;
    pol_classify64<<<resident_grid((const void *)pol_classify64, (tiles + 3) / 4), 256, 0,
                     c->stream>>>(a, b->n);
  } else {
    pol_classify<<<grid_for(n), 256, 0, c->stream>>>(a);
  }
  VP_HIP(hipGetLastError());
  VP_HIP(ev_record(c->ktime, c->ev1, c->stream));
  if (grouping && c->pol_runs) {  // phase T, grouping path with per-index
    // run slots (phase A wrote them): no scan, no scatter
    pol_runs<<<grid_for(t.cap), 256, 0, c->stream>>>(a, c->pol_cnt, nullptr, c->pol_runs,
                                                     t.cap, now, c->pol_size, c->pol_time,
                                                     pub);
    VP_HIP(hipGetLastError());
  } else if (grouping) {  // phase T, grouping path (speculative: no-ops unless pol_grouping_ok)
    size_t need = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, need, c->pol_cnt, c->pol_off,
                                     (int)t.cap, c->stream);
    VP_TRY(cub_reserve(c, need));
    VP_HIP(hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, w.cub_bytes, c->pol_cnt,
                                            c->pol_off, (int)t.cap, c->stream));
    pol_scatter<<<grid_for(n), 256, 0, c->stream>>>(w.log, w.aux, p0, p1,
                                                    c->pol_off, w.sval, t.ctl);
    pol_runs<<<grid_for(t.cap), 256, 0, c->stream>>>(a, c->pol_cnt, c->pol_off,
                                                     w.sval, t.cap, now,
                                                     c->pol_size, c->pol_time, pub);
    VP_HIP(hipGetLastError());
  }
  if (grouping)
    VP_TRY(tbl_wait_pub(c, t, epoch));
  else
    VP_TRY(read_ctl(c, t));
  float kms = 0.f;
  VP_HIP(ev_ms(c->ktime, c->ev0, c->ev1, &kms));
  *ms += kms;
  *launches += 1;
  const uint32_t nmiss = t.h_ctl.miss_count, ndefer = t.h_ctl.defer_count;
  if (nmiss) {
    size_t need = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, need, w.miss, w.miss_sorted,
                                      (int)nmiss, 0, 32, c->stream);
    VP_TRY(cub_reserve(c, need));
    VP_HIP(hipcub::DeviceRadixSort::SortKeys(w.cub_tmp, w.cub_bytes, w.miss,
                                             w.miss_sorted, (int)nmiss, 0, 32,
                                             c->stream));
    pol_miss_keys<<<grid_for(nmiss), 256, 0, c->stream>>>(a, w.miss_sorted, nmiss,
                                                          w.mkey, w.mhash);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_new_keys(c, t, NewKeys{nmiss, w.miss_sorted}, c->seq, nullptr));
    a.t = tbl_dev(t);  // a rebuild may have moved the buckets
    pol_miss_finish<<<grid_for(nmiss), 256, 0, c->stream>>>(
        a, w.miss_sorted, nmiss, w.scratch, w.rep, w.assign);
    VP_HIP(hipGetLastError());
    *allocated |= 1u;
  }
  if (ndefer) {
    a.t = tbl_dev(t);  // a rebuild during phase B may have changed the layout
    pol_defer_finish<<<grid_for(ndefer), 256, 0, c->stream>>>(a, w.defer, ndefer);
    VP_HIP(hipGetLastError());
  }
  a.t = tbl_dev(t);
  // the grouping path already ran (every policed packet was a counted
  // phase-A hit and runs are short): nothing left
  if (grouping && !nmiss && !ndefer && t.h_ctl.aux_count == 0) {
    t.ctl_clean = true;       // nothing counted
    c->pol_cnt_clean = true;  // pol_runs cleared every count it read
    return 0;
  }
  // phase T, sorting path: (index, packet) pairs sorted by index; radix sort
  // is stable, so each index's packets stay in packet order
  uint32_t bits = 1;
  while ((1ull << bits) <= t.cap) bits++;
  pol_sort_keys<<<grid_for(n), 256, 0, c->stream>>>(w.log, p0, n, t.cap, w.rank);
  VP_HIP(hipGetLastError());
  size_t need = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, need, w.rank, w.skey, w.iota + p0,
                                     w.sval, (int)n, 0, (int)bits, c->stream);
  VP_TRY(cub_reserve(c, need));
  VP_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, w.cub_bytes, w.rank, w.skey,
                                            w.iota + p0, w.sval, (int)n, 0,
                                            (int)bits, c->stream));
  pol_buckets<<<grid_for(n), 256, 0, c->stream>>>(a, w.skey, w.sval, n, t.cap, now,
                                                  c->pol_size, c->pol_time);
  VP_HIP(hipGetLastError());
  if (nmiss || ndefer) VP_TRY(read_ctl(c, t));
  return 0;
}

int pol_process_device(vp_ctx *c, const vp_dev_batch *b) {
  // expiries only up to the batch's last IPv4 packet
  uint32_t exp_end = b->n;
  // With affine time the whole batch may be free of expiries (the cutoff
  // of its last packet is below every live stamp): then run_batch makes one
  // segment whatever exp_end is, and the search is skipped.
  bool may_expire = true;
  if (b->n && !b->now && b->now_step >= 0 && b->now0 >= 0) {
    const int64_t t_last = b->now0 + (int64_t)(b->n - 1) * b->now_step;
    may_expire = pol_cutoff(c, t_last) >
                 (int64_t)std::min<uint64_t>(c->ft.ts_floor, (uint64_t)b->now0);
  }
  if (may_expire && b->n && b->frames && b->len && b->slot >= 64) {
    VP_TRY(ws_reserve(c, b->n));
    int32_t *d_last = reinterpret_cast<int32_t *>(&c->ft.ctl->aux_count);
    pol_last_ipv4<<<1, 256, 0, c->stream>>>(b->frames, b->slot, b->len, b->n,
                                            d_last);
    VP_HIP(hipGetLastError());
    int32_t last = -1;
    VP_HIP(hipMemcpyAsync(&last, d_last, 4, hipMemcpyDeviceToHost, c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    exp_end = (uint32_t)(last + 1);
    c->ft.ctl_clean = false;  // (aux_count held the answer)
  }
  ExpiringTable tabs[1] = {{&c->ft, pol_cutoff}};
  return run_batch(c, b, tabs, 1, pol_segment, exp_end);
}

// State by index: alloc, ts, dyn_keys (u32 address), dyn_vals.
int pol_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint32_t *keys,
             uint64_t *bucket_size, int64_t *bucket_time) {
  const uint32_t cap = c->ft.cap;
  std::vector<uint32_t> k(4ull * cap);
  VP_TRY(tbl_dump(c, c->ft, alloc, ts, k.data()));
  for (uint32_t i = 0; i < cap; i++) keys[i] = k[4ull * i];
  VP_HIP(hipMemcpy(bucket_size, c->pol_size, 8ull * cap, hipMemcpyDeviceToHost));
  VP_HIP(hipMemcpy(bucket_time, c->pol_time, 8ull * cap, hipMemcpyDeviceToHost));
  return 0;
}

void build_pol_tables(std::vector<uint32_t> &tab) {
  tab.assign(kPolTabs * 256, 0);
  for (uint32_t j = 0; j < kPolTabs; j++)
    build_position_table(&tab[j * 256], (int)j, 4);
}

}  // namespace vp
