// Device-resident libVig map + dchain equivalent, shared by the NFs.
//
// The reference keeps, per NF table, a libVig Map (key -> index, linear
// probing with chain counters, map-impl-pow2.c), a Vector of keys by index and
// a DoubleChain (index allocator + LRU list + per-index timestamps,
// double-chain-impl.c). Outputs depend only on the key -> index mapping, the
// order indices are handed out, and which indices expire when (SURVEY.md §0
// fact 3), so the device keeps an equivalent, batch-friendly form:
//
//   buckets[]  open addressing over 64-byte buckets of 3 entries
//              (key 16 B + index 4 B each; one aligned 64 B line per probe
//              step); entries are scanned bucket by bucket, entry by entry;
//              erase leaves a tombstone, rebuilt when they pile up
//   slot_of[]  index -> entry (bucket * 4 + e)   (kNone = not allocated)
//   hash_of[]  index -> key hash (only for rebuilds)
//   ts[]       index -> dchain timestamp         (exact, see touch log)
//   tseq[]     index -> global packet seq of the last touch (LRU tie-break)
//   birth[]    index -> global packet seq of its allocation
//   stack[]    freed indices, LIFO (dchain free-list front); the rest of the
//              free list is the never-used range [fresh_next, cap)
//
// Rejuvenation is recorded as a touch log (one u32 index per packet) and
// folded into ts/tseq after each segment (last toucher in packet order
// wins); no per-packet atomics on shared timestamps.
#pragma once

#include "vp_device.h"
#include "vp_internal.h"

namespace vp {

struct TableDev {
  Bucket *bk;
  uint32_t bmask, cap, mix;
  uint32_t *slot_of;
  uint32_t *hash_of;
  uint64_t *ts;
  uint64_t *tseq;
  uint64_t *birth;
  uint32_t *stack;
  Ctl *ctl;
  uint4 *kv;               // owner mode: key by index (replicated); else null
  uint32_t own_n, own_r;   // owner mode: ranks and this rank; own_n == 0 off
  const uint32_t *lin;     // mix == kMixLin: the map's byte tables (4 x 256)
};

// slot_of[] in owner mode: allocated, but its key lives in another rank's
// buckets (entry ids are (bucket << 2) | e, always below this value).
constexpr uint32_t kElsewhere = 0xFFFFFFFCu;

// Owner rank of a key hash: the top bits (multiply-shift, so any rank
// count), independent of the home bucket's low bits.
__host__ __device__ __forceinline__ uint32_t owner_of(uint32_t h, uint32_t n) {
  return (uint32_t)(((uint64_t)h * n) >> 32);
}

// A fold kernel's publication of the control block into host-coherent
// memory (tbl_fold_read_ctl): pub == null means off. One thread calls
// ctl_publish after the launch that filled `ctl` has completed (or, the
// classify's last block, after every block's release: tile_publish):
// device-scope loads of the block, system-scope stores, the epoch last
// (release).
struct PubArgs {
  CtlPub *pub;
  const Ctl *ctl;
  uint32_t epoch;
  const uint32_t *x0, *x1;  // extra words (CtlPub::xtra): x0[0..n0), then x1[0..n1)
  uint32_t n0, n1;
  uint32_t rel = 0;  // the epoch stored with a system-scope release (A/B)
};
static_assert(sizeof(Ctl) % 8 == 0, "Ctl is published as 8-byte words");
__device__ __forceinline__ void ctl_publish(const PubArgs &a) {
  if (!a.pub) return;
  constexpr uint32_t kW = sizeof(Ctl) / 8;
  const uint64_t *s = reinterpret_cast<const uint64_t *>(a.ctl);
  uint64_t *d = reinterpret_cast<uint64_t *>(&a.pub->ctl);
  uint64_t v[kW];  // all loads issued before the first store waits
#pragma unroll
  for (uint32_t i = 0; i < kW; i++)
    v[i] = __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (uint32_t i = 0; i < kW; i++)
    __hip_atomic_store(d + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (uint32_t i = 0; i < a.n0 + a.n1; i++) {
    const uint32_t *s1 = i < a.n0 ? a.x0 + i : a.x1 + (i - a.n0);
    __hip_atomic_store(&a.pub->xtra[i],
                       __hip_atomic_load(s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // The epoch after every word above has completed. Those are system-scope
  // stores (past the GPU's caches), so waiting for them orders them; a
  // release would also write the XCD's L2 back (buffer_wbl2), which the fold
  // kernel could not end before (VIGPATH_PUB_RELEASE=1: that form, for A/B)
  if (a.rel) {
    __hip_atomic_store(&a.pub->epoch, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&a.pub->epoch, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

struct NowSpec {
  const int64_t *arr;
  int64_t now0, step;
  __host__ __device__ int64_t at(uint32_t p) const {
    return arr ? arr[p] : now0 + (int64_t)p * step;
  }
};

// Home bucket of a key hash. Modes 0-31 take the CRC's bits from bit `mix`
// on (a rotation, then the reference's mask: mode 0 is hash & (cap-1),
// map-impl-pow2.c:15-27). CRC32C is GF(2)-linear, so keys that differ in a
// few low bits (sequential ports/addresses, the benchmark's flows) land on a
// structured, well-spread set of buckets, which the memory system serves
// faster than random lines -- when the selected bits have full rank over the
// key set. For some key sets they lose rank and buckets cluster; the table
// detects long insert probes, scores every rotation over its live keys and
// rebuilds with the best one, or with the multiplicative spread (kMixMul)
// when none is clean (tbl_choose_layout). Only the key -> index mapping is
// observable, so every layout gives identical results.
constexpr uint32_t kMixMul = 32;
// kMixLin: bucket = L(h) & bmask for a GF(2)-linear map L of the hash bits
// fitted to the live keys so that indices allocated one after another sit in
// consecutive buckets (tbl_try_linear, vp_table.hip); L is given by four
// 256-entry tables, one per hash byte (`lin`, in LDS or global memory).
constexpr uint32_t kMixLin = 33;
__host__ __device__ __forceinline__ uint32_t lin_map(const uint32_t *L, uint32_t h) {
  return L[h & 255] ^ L[256 + ((h >> 8) & 255)] ^ L[512 + ((h >> 16) & 255)] ^
         L[768 + (h >> 24)];
}
__host__ __device__ __forceinline__ uint32_t home_bucket(uint32_t h,
                                                         uint32_t bmask,
                                                         uint32_t mix,
                                                         const uint32_t *lin = nullptr) {
  if (mix == kMixLin) return lin_map(lin, h) & bmask;
  if (mix >= kMixMul)
    return (uint32_t)(((uint64_t)(h * 0x9E3779B1u) * (bmask + 1ull)) >> 32);
  return ((h >> mix) | (h << ((32 - mix) & 31))) & bmask;
}

// One bucket (key words k0-k2, entry indices ix) against `key`, entries in
// order: the index on a match; kNone with *done on an empty entry (the probe
// path ends there); kNone with !*done when the probe continues in the next
// bucket. Word 3 is compared under M3: tables that keep a per-index value in
// the key's padding bytes (viglb's backend, vigfw's internal device) match
// on the protocol byte only.
template <uint32_t M3 = 0xFFFFFFFFu>
__device__ __forceinline__ uint32_t bucket_match(uint4 k0, uint4 k1, uint4 k2,
                                                 uint4 ix, const uint32_t key[4],
                                                 bool *done, uint32_t *w3 = nullptr) {
  *done = true;
  if (ix.x == kEmpty) return kNone;
  if (ix.x != kTomb && k0.x == key[0] && k0.y == key[1] && k0.z == key[2] &&
      ((k0.w ^ key[3]) & M3) == 0) {
    if (w3) *w3 = k0.w;
    return ix.x;
  }
  if (ix.y == kEmpty) return kNone;
  if (ix.y != kTomb && k1.x == key[0] && k1.y == key[1] && k1.z == key[2] &&
      ((k1.w ^ key[3]) & M3) == 0) {
    if (w3) *w3 = k1.w;
    return ix.y;
  }
  if (ix.z == kEmpty) return kNone;
  if (ix.z != kTomb && k2.x == key[0] && k2.y == key[1] && k2.z == key[2] &&
      ((k2.w ^ key[3]) & M3) == 0) {
    if (w3) *w3 = k2.w;
    return ix.z;
  }
  *done = false;
  return kNone;
}

// The rest of a probe path, from bucket b for at most `steps` buckets.
template <uint32_t M3 = 0xFFFFFFFFu>
__device__ __forceinline__ uint32_t tbl_probe_from(const TableDev &t, uint32_t b,
                                                   const uint32_t key[4],
                                                   uint32_t steps,
                                                   uint32_t *w3 = nullptr) {
  for (uint32_t i = 0; i < steps; i++) {
    const uint4 *q = reinterpret_cast<const uint4 *>(t.bk + b);
    bool done;
    const uint32_t r = bucket_match<M3>(q[0], q[1], q[2], q[3], key, &done, w3);
    if (done) return r;
    b = (b + 1) & t.bmask;
  }
  return kNone;
}

// map_get (find_key, map-impl-pow2.c:629-732) on the device table. Returns
// the index or kNone.
template <uint32_t M3 = 0xFFFFFFFFu>
__device__ __forceinline__ uint32_t tbl_probe(const TableDev &t, uint32_t h,
                                              const uint32_t key[4],
                                              uint32_t *w3 = nullptr) {
  return tbl_probe_from<M3>(t, home_bucket(h, t.bmask, t.mix, t.lin), key, t.bmask + 1,
                            w3);
}

// Key words of an allocated index's entry.
// Claim the first empty-or-erased entry on key hash h's probe path (the
// map_put position; the key is known to be absent) and store key + index.
// Returns the entry id. Concurrent claimers race on the index word only.
__device__ inline uint32_t tbl_insert(const TableDev &t, uint32_t h, const uint32_t *k,
                               uint32_t idx, bool *reused_tomb, uint32_t *disp) {
  uint32_t b = home_bucket(h, t.bmask, t.mix, t.lin);
  for (uint32_t d = 0;; d++) {
    if (d == 1) *disp += 1;  // past the home bucket
    if (d == 8) atomicMax(&t.ctl->max_disp, d);  // clustering signal
    for (uint32_t e = 0; e < kBucketEntries; e++) {
      uint32_t *w = &t.bk[b].idx[e];
      uint32_t cur = __hip_atomic_load(w, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
      while (cur == kEmpty || cur == kTomb) {
        const uint32_t old = atomicCAS(w, cur, idx);
        if (old == cur) {
          uint32_t *kk = t.bk[b].k[e];
          kk[0] = k[0];
          kk[1] = k[1];
          kk[2] = k[2];
          kk[3] = k[3];
          *reused_tomb = cur == kTomb;
          return (b << 2) | e;
        }
        cur = old;  // lost the race; look at this entry again
      }
    }
    b = (b + 1) & t.bmask;
  }
}

__device__ __forceinline__ uint4 tbl_key_of(const TableDev &t, uint32_t idx) {
  if (t.kv) return t.kv[idx];
  const uint32_t e = t.slot_of[idx];
  return reinterpret_cast<const uint4 *>(t.bk + (e >> 2))[e & 3];
}

// dchain_is_index_allocated as seen by the packet with global sequence q
// inside a segment: allocated before the segment, or earlier in it.
__device__ __forceinline__ bool tbl_allocated_before(const TableDev &t,
                                                     uint32_t idx, uint64_t q) {
  return t.slot_of[idx] != kNone && t.birth[idx] < q;
}

// ------------------------------------------------------------ host API --

// New-key pipeline input: `n` misses with keys/hashes already in
// ws.mkey/ws.mhash and positions (ascending) in `pos`.
// tbl_new_keys_unsorted's miss list: an entry with this bit is the index of
// a lean tile's slot in the classify blocks' slices (missq / mkq / mhq: its
// position, FlowId and hash there, not copied at the block's end); any other
// entry j is a position, its FlowId and hash at mkey[j] / mhash[j].
constexpr uint32_t kMissSlice = 0x80000000u;

struct NewKeys {
  uint32_t n;
  const uint32_t *pos;
};

int tbl_alloc(vp_ctx *c, FlowTable &t, uint32_t cap);
void tbl_free(FlowTable &t);
TableDev tbl_dev(const FlowTable &t);

// Dedup the misses by key (earliest packet wins), rank first sightings in
// packet order, hand out dchain indices (free-list order) and insert the
// keys. Afterwards ws.assign[j0] holds the index for first sighting j0 (or
// kNone when the table was full) and scratch[rep[j]] = j0 for every j.
// New flows of one segment on one GPU without sorting the misses (DESIGN.md
// §5.1, churn): n misses in any order, w.miss[j] = packet position p0 <= p <
// p1 with its FlowId in w.mkey[j] / hash w.mhash[j] (written by phase A).
// Per distinct key: the first and last packet (a tagged hash set, no reset);
// first sightings ranked in packet order by a bit per position; the r-th
// takes the r-th free-list entry (dchain_allocate_new_index order), is
// inserted, born at its first packet and stamped with its last. On return
// the low word of w.nkset[w.rep[j]] is miss j's index (kNone: table full)
// and h_ctl holds the counters.
// Asynchronous: the kernels are queued; tbl_new_keys_done reads the counters
// back and runs the layout checks (the caller queues its own work between).
int tbl_new_keys_unsorted(vp_ctx *c, FlowTable &t, uint32_t n, uint32_t p0, uint32_t p1,
                          const NowSpec &now, uint64_t seq_base);
int tbl_new_keys_done(vp_ctx *c, FlowTable &t);
int tbl_new_keys(vp_ctx *c, FlowTable &t, const NewKeys &nk, uint64_t seq_base,
                 uint32_t *n_new);

// Fold the touch log of packets [p0, p1) (log[p] = index or kNone) into
// ts/tseq: ts = time of the last toucher, tseq = its global sequence.
int tbl_touch_reduce(vp_ctx *c, FlowTable &t, const uint32_t *log, uint32_t p0,
                     uint32_t p1, const NowSpec &now, uint64_t seq_base);

// Touch bins for one 64-byte classify launch over [p0, p1) of `kernel`
// (vp_device.h TouchBins). plan->on is false when the launch cannot bin
// (unaligned segment, table or range too large, VIGPATH_TOUCH_BINS=0); then
// pass plan->bins (ent = null) to the kernel and fold with tbl_touch_reduce.
struct BinsPlan {
  bool on;
  uint32_t grid, range, L;
  uint32_t sbits;  // 2^sbits fold blocks per bin, each L >> sbits indices
  TouchBins bins;
  // a second fold of a segment whose first fold ran already (the owner
  // pipeline's leftover exchange): an index's stamp is only raised (its
  // touches here may precede the ones folded first)
  bool maxmode;
};
// min_bits: at least 2^min_bits bins (vigbridge keeps 256: measured 1.7 %
// slower at 128, tools/sessions/gpu_r04bc.sh).
// vper: virtual blocks of vper tiles each (the chunked owner pipeline's
// launches, frames64_tiles) instead of the kernel's resident grid.
int tbl_bins_plan(vp_ctx *c, FlowTable &t, const void *kernel, uint32_t p0,
                  uint32_t p1, BinsPlan *plan, uint32_t waves = 4, uint32_t min_bits = 0,
                  uint32_t vper = 0);
// ts of the indices the reprobe kernels touched (after their tseq atomicMax;
// the queue as in reprobe_slices, vp_device.h).
int tbl_reprobe_stamp(vp_ctx *c, FlowTable &t, const uint32_t *list,
                      const uint32_t *cnt, uint32_t n, uint32_t range, uint32_t nblk,
                      const uint32_t *log, const NowSpec &now, uint64_t seq_base);

// Touches applied after a fold, in any order: packets listed as in
// reprobe_slices (slices per classify block with `cnt`, or runs of `range`
// of one list of n), each with its index in log[p] (kNone: none); the last
// toucher in packet order still wins (tseq atomicMax, then ts).
int tbl_late_touches(vp_ctx *c, FlowTable &t, const uint32_t *list,
                     const uint32_t *cnt, uint32_t n, uint32_t range, uint32_t nblk,
                     const uint32_t *log, const NowSpec &now, uint64_t seq_base);

// Fold the bins into ts/tseq. A touch that found its slice full was queued
// instead (t.ctl->touch_ovf set; apply plan.bins.oent with tbl_late_touches).
int tbl_bins_reduce(vp_ctx *c, FlowTable &t, const BinsPlan &plan, uint32_t p0,
                    const NowSpec &now, uint64_t seq_base,
                    const PubArgs &pub = PubArgs{});
// Multi-GPU: also gathers the ranks' segment counters (Workspace::h_gath;
// owner mode: + this rank's `sends`, its key count per owner).
int tbl_wait_pub(vp_ctx *c, FlowTable &t, uint32_t epoch);
int tbl_fold_read_ctl(vp_ctx *c, FlowTable &t, const BinsPlan &bp, const uint32_t *log,
                      uint32_t p0, uint32_t p1, const NowSpec &now, uint64_t seq_base,
                      const uint32_t *sends = nullptr, uint32_t pub_epoch = 0);


// expire_items_single_map for cutoff: free every allocated index with
// ts < cutoff in LRU order (ts, then tseq) onto the stack, erase its key.
int tbl_expire(vp_ctx *c, FlowTable &t, int64_t cutoff, uint32_t *n_out);

// Purge tombstones (rebuild) once live + erased entries pass 85 %.
int tbl_check_tombs(vp_ctx *c, FlowTable &t);

// Owner mode (rank r of n): a fresh table keeps only the keys it owns in its
// buckets (sized for 1/n of the keys) and every key by index in kv.
int tbl_set_owner(vp_ctx *c, FlowTable &t, uint32_t n, uint32_t r);
// Owner mode: grow the buckets, if needed, before inserting the union of n
// new keys whose hashes are in ws.mhash.
int tbl_owner_reserve(vp_ctx *c, FlowTable &t, uint32_t n);

// Per index: alloc flag, ts, key words.
int tbl_dump(vp_ctx *c, FlowTable &t, uint8_t *alloc, int64_t *ts,
             uint32_t *keys);

int read_ctl(vp_ctx *c, FlowTable &t);
int read_ctl2(vp_ctx *c, FlowTable &a, FlowTable &b);
int read_ctl_post(vp_ctx *c, FlowTable &t);
int read_ctl_wait(vp_ctx *c, FlowTable &t);
int read_ctl2_post(vp_ctx *c, FlowTable &a, FlowTable &b);
int read_ctl2_wait(vp_ctx *c, FlowTable &a, FlowTable &b);

// ---------------------------------------------------------- batch driver --
// A table whose entries expire, and the cutoff for a packet at time t (the
// NF's own arithmetic, e.g. vignat's u32 wrap).
struct ExpiringTable {
  FlowTable *t;
  int64_t (*cutoff)(const vp_ctx *c, int64_t t);
};
// Process packets [p0, p1) of `b` with no expiry inside; set bit i of
// *allocated when table i got new indices.
using SegmentFn = int (*)(vp_ctx *c, const vp_dev_batch *b, const NowSpec &now,
                          uint32_t p0, uint32_t p1, float *kernel_ms,
                          int *launches, uint32_t *allocated);
// Validates the batch, then cuts it where any table may expire an entry and
// runs the exact expiries between segments (see vp_nat.hip header). Only
// packets [0, exp_end) run an expiry (vigpol expires after the IPv4 parse
// only); the others leave the tables as they are.
int run_batch(vp_ctx *c, const vp_dev_batch *b, ExpiringTable *tabs, int ntabs,
              SegmentFn seg, uint32_t exp_end = UINT32_MAX);

// ------------------------------------------------- multi-GPU new keys --
// (run_batch_sharded, vp_table.hip) Gather every rank's count of local new
// keys: the union size and this rank's offset in it.
int union_sizes(vp_ctx *c, uint32_t nl, uint32_t *total, uint32_t *mine_off);
// Local new keys (ws.mkey/ws.mhash [0, nl), sorted local positions in
// ws.miss_sorted) -> the union on every rank, in global packet order:
// ws.mkey/ws.mhash, global positions ws.skey, times ws.unow.
int union_exchange(vp_ctx *c, uint32_t nl, const NowSpec &now);
__global__ void union_stamp(const uint32_t *first, const uint32_t *assign,
                            const uint32_t *upos, const int64_t *unow, uint32_t n,
                            uint64_t seq, uint64_t *ts, uint64_t *tseq);

uint32_t grid_for(uint64_t n, uint32_t block = 256, uint32_t max_blocks = 2048);
// Persistent grid for a grid-stride kernel of 256-thread blocks: as many
// blocks as the device holds at once (occupancy of `kernel` x CUs; env
// VIGPATH_BLOCKS_PER_CU overrides the per-CU count), at most work_blocks. A
// larger grid leaves the blocks that do not fit to run after the first wave
// of blocks, as a tail at lower occupancy.
uint32_t resident_grid(const void *kernel, uint64_t work_blocks, int threads = 256);
// vignat owner mode: packets per chunk of the chunked pipeline (0: off;
// vp_nat.hip)
uint32_t nat_own_chunk_packets();
uint32_t next_pow2(uint64_t v);
int cub_reserve(vp_ctx *c, size_t bytes);

}  // namespace vp
