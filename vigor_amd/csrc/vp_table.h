// Device-resident libVig map + dchain equivalent, shared by the NFs.
//
// The reference keeps, per NF table, a libVig Map (key -> index, linear
// probing with chain counters, map-impl-pow2.c), a Vector of keys by index and
// a DoubleChain (index allocator + LRU list + per-index timestamps,
// double-chain-impl.c). Outputs depend only on the key -> index mapping, the
// order indices are handed out, and which indices expire when (SURVEY.md §0
// fact 3), so the device keeps an equivalent, batch-friendly form:
//
//   slots[]    open-addressed table, 32 B slot = key(16) | hash | index
//              (tombstones on erase, rebuilt when they pile up)
//   slot_of[]  index -> slot                    (kNone = index not allocated)
//   ts[]       index -> dchain timestamp         (exact, see touch log below)
//   tseq[]     index -> global packet seq of the last touch (LRU tie-break)
//   birth[]    index -> global packet seq of its allocation
//   stack[]    freed indices, LIFO (dchain free list front); the rest of the
//              free list is the never-used range [fresh_next, cap)
//
// Rejuvenation is recorded as a touch log (one u32 index per packet) and
// folded into ts/tseq after each segment by a stable radix sort: the last
// entry of each index's run is its last toucher in packet order. No
// per-packet atomics on shared timestamps.
#pragma once

#include "vp_device.h"
#include "vp_internal.h"

namespace vp {

struct TableDev {
  FlowSlot *slots;
  uint32_t tmask, cap;
  uint32_t *slot_of;
  uint64_t *ts;
  uint64_t *tseq;
  uint64_t *birth;
  uint32_t *stack;
  Ctl *ctl;
};

struct NowSpec {
  const int64_t *arr;
  int64_t now0, step;
  __host__ __device__ int64_t at(uint32_t p) const {
    return arr ? arr[p] : now0 + (int64_t)p * step;
  }
};

// map_get (find_key, map-impl-pow2.c:629-732) on the device table. Returns
// the index or kNone.
__device__ __forceinline__ uint32_t tbl_probe(const TableDev &t, uint32_t h,
                                              const uint32_t key[4]) {
  uint32_t s = h & t.tmask;
  for (uint32_t i = 0; i <= t.tmask; i++) {
    const uint4 *sp4 = reinterpret_cast<const uint4 *>(t.slots + s);
    const uint4 k = sp4[0];
    const uint4 m = sp4[1];
    if (m.y == kEmpty) return kNone;
    if (m.y != kTomb && m.x == h && k.x == key[0] && k.y == key[1] &&
        k.z == key[2] && k.w == key[3])
      return m.y;
    s = (s + 1) & t.tmask;
  }
  return kNone;
}

// dchain_is_index_allocated as seen by the packet with global sequence q
// inside a segment: allocated before the segment, or earlier in it.
__device__ __forceinline__ bool tbl_allocated_before(const TableDev &t,
                                                     uint32_t idx, uint64_t q) {
  return t.slot_of[idx] != kNone && t.birth[idx] < q;
}

// ------------------------------------------------------------ host API --

// New-key pipeline input: `n` misses with keys/hashes already in
// ws.mkey/ws.mhash and positions (ascending) in ws.miss_sorted.
struct NewKeys {
  uint32_t n;
  const uint32_t *pos;  // packet positions, ascending
};

int tbl_alloc(vp_ctx *c, FlowTable &t, uint32_t cap);
void tbl_free(FlowTable &t);
TableDev tbl_dev(const FlowTable &t);

// Dedup the misses by key (earliest packet wins), rank first sightings in
// packet order, hand out dchain indices (free-list order) and insert the
// keys. Afterwards ws.assign[j0] holds the index for first-sighting j0 (or
// kNone when the table was full) and scratch[rep[j]] = j0 for every j.
int tbl_new_keys(vp_ctx *c, FlowTable &t, const NewKeys &nk, uint64_t seq_base,
                 uint32_t *n_new);

// Fold the touch log of packets [p0, p1) (log[p] = index or kNone) into
// ts/tseq: ts = time of the last toucher, tseq = its global sequence.
int tbl_touch_reduce(vp_ctx *c, FlowTable &t, const uint32_t *log, uint32_t p0,
                     uint32_t p1, const NowSpec &now, uint64_t seq_base);

// Exact min ts over allocated indices -> t.ts_floor (~0 if none).
int tbl_exact_floor(vp_ctx *c, FlowTable &t);

// expire_items_single_map for cutoff: free every allocated index with
// ts < cutoff in LRU order (ts, then tseq) onto the stack, erase its key.
// *n_out = how many expired.
int tbl_expire(vp_ctx *c, FlowTable &t, int64_t cutoff, uint32_t *n_out);

// Per index: alloc flag, ts, key words.
int tbl_dump(vp_ctx *c, FlowTable &t, uint8_t *alloc, int64_t *ts,
             uint32_t *keys);

int read_ctl(vp_ctx *c, FlowTable &t);

uint32_t grid_for(uint64_t n, uint32_t block = 256, uint32_t max_blocks = 2048);
uint32_t next_pow2(uint64_t v);
int cub_reserve(vp_ctx *c, size_t bytes);

}  // namespace vp
