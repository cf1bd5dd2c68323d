// Device table kernels + host orchestration (see vp_table.h).
//
// Reference semantics (paths relative to the reference repository):
//   map_put / find_empty     libvig/verified/map-impl-pow2.c:1110-1217,2156-2222
//   dchain alloc / free      double-chain-impl.c:1197-1415, 1839-2078
//   dchain expire            double-chain.c:772-826 (strict ts < cutoff)
//   expire_items_single_map  expirator.c:110-218
#include <hip/hip_runtime.h>

#include <cstddef>
#include <hipcub/hipcub.hpp>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "vp_comm.h"
#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(table)


uint32_t grid_for(uint64_t n, uint32_t block, uint32_t max_blocks) {
  uint64_t g = (n + block - 1) / block;
  if (g == 0) g = 1;
  return (uint32_t)(g < max_blocks ? g : max_blocks);
}

uint32_t resident_grid(const void *kernel, uint64_t work_blocks, int threads) {
  struct Entry {
    const void *kernel;
    int dev;
    uint32_t cus, per;
  };
  static std::mutex mu;
  static std::vector<Entry> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  uint32_t cus = 0, per = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    for (const Entry &e : cache)
      if (e.kernel == kernel && e.dev == dev) cus = e.cus, per = e.per;
    if (!cus) {
      int c = 0, p = 0;
      if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) !=
              hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, kernel, threads, 0) !=
              hipSuccess)
        (void)hipGetLastError();
      cus = (uint32_t)std::max(c, 1);
      per = (uint32_t)std::max(p, 1);
      cache.push_back(Entry{kernel, dev, cus, per});
    }
  }
  const char *env = getenv("VIGPATH_BLOCKS_PER_CU");  // diagnostics
  if (env && atoi(env) > 0) per = (uint32_t)atoi(env);
  const uint64_t g = std::min<uint64_t>(work_blocks, (uint64_t)cus * per);
  return (uint32_t)std::max<uint64_t>(g, 1);
}

uint32_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return (uint32_t)p;
}

int cub_reserve(vp_ctx *c, size_t bytes) {
  Workspace &w = c->ws;
  if (bytes <= w.cub_bytes) return 0;
  if (w.cub_tmp) VP_HIP(hipFree(w.cub_tmp));
  w.cub_tmp = nullptr;
  w.cub_bytes = 0;
  VP_HIP(hipMalloc(&w.cub_tmp, bytes));
  w.cub_bytes = bytes;
  return 0;
}

int read_ctl(vp_ctx *c, FlowTable &t) {
  VP_HIP(hipMemcpyAsync(t.h_pin, t.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(stream_wait(c->stream));
  t.h_ctl = *t.h_pin;
  return 0;
}

// The control block as of the work enqueued so far, copied behind it; the
// caller may enqueue more (the timestamp fold) before waiting for the copy
// alone, so the host learns phase A's counts while the fold runs.
int read_ctl_post(vp_ctx *c, FlowTable &t) {
  VP_HIP(hipMemcpyAsync(t.h_pin, t.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(hipEventRecord(c->evc, c->stream));
  return 0;
}

int read_ctl_wait(vp_ctx *c, FlowTable &t) {
  hipError_t e;
  while ((e = hipEventQuery(c->evc)) == hipErrorNotReady) {
  }
  VP_HIP(e);
  t.h_ctl = *t.h_pin;
  return 0;
}

// Both tables' control blocks copied behind the work enqueued so far; wait
// with read_ctl2_wait (viglb: the fold runs in between).
int read_ctl2_post(vp_ctx *c, FlowTable &a, FlowTable &b) {
  VP_HIP(hipMemcpyAsync(a.h_pin, a.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(hipMemcpyAsync(b.h_pin, b.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(hipEventRecord(c->evc, c->stream));
  return 0;
}

int read_ctl2_wait(vp_ctx *c, FlowTable &a, FlowTable &b) {
  hipError_t e;
  while ((e = hipEventQuery(c->evc)) == hipErrorNotReady) {
  }
  VP_HIP(e);
  a.h_ctl = *a.h_pin;
  b.h_ctl = *b.h_pin;
  return 0;
}

// Both tables' control blocks with one wait (viglb reads its two together).
int read_ctl2(vp_ctx *c, FlowTable &a, FlowTable &b) {
  VP_HIP(hipMemcpyAsync(a.h_pin, a.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(hipMemcpyAsync(b.h_pin, b.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(stream_wait(c->stream));
  a.h_ctl = *a.h_pin;
  b.h_ctl = *b.h_pin;
  return 0;
}

TableDev tbl_dev(const FlowTable &t) {
  return TableDev{t.bk,  t.bmask, t.cap,   t.mix, t.slot_of, t.hash_of, t.ts,
                  t.tseq, t.birth, t.stack, t.ctl, t.kv,      t.own_n,   t.own_r,
                  t.lin};
}

template <class T>
static int dalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void **)p, sizeof(T) * count);
  return e == hipSuccess ? 0 : hip_fail(e, "hipMalloc", __FILE__, __LINE__);
}

static int tbl_rebuild(vp_ctx *c, FlowTable &t, uint64_t nb_new = 0);
static int tbl_choose_layout(vp_ctx *c, FlowTable &t);
static int tbl_try_linear(vp_ctx *c, FlowTable &t);
__global__ void lay_count(TableDev t, uint32_t mix, uint32_t *cnt);
__global__ void lay_score(const uint32_t *cnt, uint32_t nb, uint32_t *over);

static uint64_t tbl_entries(const FlowTable &t) {
  return (uint64_t)(t.bmask + 1) * kBucketEntries;
}

int tbl_alloc(vp_ctx *c, FlowTable &t, uint32_t cap) {
  (void)c;
  // Every NF's flow table (vignat, vigfw, vigpol flows, vigbridge MACs, viglb
  // flows and backends) gets two buckets (3 entries each) per index: load
  // <= 1/6, so a random key set puts ~0.2 % of its keys past their home
  // bucket (~2.3 % at load 1/3, ~13 % at 2/3, each one a reprobe: DESIGN.md
  // §4-5.1, random keys 0.80 -> 0.66 ms per step). 128 B of HBM per index,
  // 128 MB at 1M flows of 288 GB; the allocation-order layout (§4) rebuilds
  // at 32 B. Tombstones purged at 0.85 of one bucket per index
  // (tbl_check_tombs).
  uint64_t nb = 64;
  while (nb < cap) nb <<= 1;
  t.nb_base = nb;
  int k = 1;
  // (VIGPATH_SPARSE=k: 2^k buckets per index, k in -3..3; the tests use it to
  // force high loads and full home buckets)
  if (const char *sp = getenv("VIGPATH_SPARSE")) k = atoi(sp);
  if (k > 0) nb <<= std::min(k, 3);
  if (k < 0) nb = std::max<uint64_t>(64, nb >> std::min(-k, 3));
  t.bmask = (uint32_t)(nb - 1);
  t.nb_nominal = nb;
  t.cap = cap;
  const char *mix = getenv("VIGPATH_MIX");  // diagnostics: start multiplicative
  t.mix = mix && atoi(mix) ? kMixMul : 0;
  VP_TRY(dalloc(&t.bk, nb));
  VP_TRY(dalloc(&t.slot_of, cap));
  VP_TRY(dalloc(&t.hash_of, cap));
  VP_TRY(dalloc(&t.ts, cap));
  VP_TRY(dalloc(&t.tseq, cap));
  VP_TRY(dalloc(&t.birth, cap));
  VP_TRY(dalloc(&t.stack, cap));
  VP_TRY(dalloc(&t.lastg, cap));
  VP_TRY(dalloc(&t.ctl, 1));
  VP_HIP(hipHostMalloc((void **)&t.h_pin, sizeof(Ctl), hipHostMallocDefault));
  VP_HIP(hipHostMalloc((void **)&t.h_pub, sizeof(CtlPub),
                       hipHostMallocMapped | hipHostMallocCoherent));
  memset(t.h_pub, 0, sizeof(CtlPub));
  VP_HIP(hipHostGetDevicePointer((void **)&t.d_pub, t.h_pub, 0));
  VP_TRY(dalloc(&t.ttotal, 1));
  VP_TRY(dalloc(&t.ekey, cap));
  VP_TRY(dalloc(&t.ekey2, cap));
  VP_TRY(dalloc(&t.eidx, cap));
  VP_TRY(dalloc(&t.eidx2, cap));
  VP_HIP(hipMemset(t.bk, 0xFF, sizeof(Bucket) * nb));
  VP_HIP(hipMemset(t.slot_of, 0xFF, sizeof(uint32_t) * (size_t)cap));
  VP_HIP(hipMemset(t.ts, 0, sizeof(uint64_t) * (size_t)cap));
  VP_HIP(hipMemset(t.tseq, 0, sizeof(uint64_t) * (size_t)cap));
  VP_HIP(hipMemset(t.birth, 0, sizeof(uint64_t) * (size_t)cap));
  VP_HIP(hipMemset(t.ctl, 0, sizeof(Ctl)));
  t.ts_floor = ~0ull;
  return 0;
}

void tbl_free(FlowTable &t) {
  void *ptrs[] = {t.bk,    t.slot_of, t.hash_of, t.ts,    t.tseq,
                  t.birth, t.stack,   t.lastg,   t.ctl,   t.ekey,
                  t.ekey2, t.eidx,    t.eidx2};
  for (void *p : ptrs) hipFree(p);
  hipFree(t.ttotal);
  hipFree(t.lin);
  hipFree(t.kv);
  if (t.h_pin) hipHostFree(t.h_pin);
  if (t.h_pub) hipHostFree(t.h_pub);
  t = FlowTable{};
}

// ------------------------------------------------------------ new keys --

struct NkArgs {
  TableDev t;
  const uint32_t *pos;
  uint32_t n;
  uint32_t *mkey, *mhash, *first, *rank, *rep, *assign, *scratch;
  uint32_t smask;
  uint64_t seq_base;
};

// In-batch de-duplication: one scratch slot per distinct key holding the
// smallest miss ordinal (= earliest packet) with that key.
__global__ void nk_dedup(NkArgs m) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    const uint32_t *kj = m.mkey + 4 * (size_t)j;
    uint32_t s = home_bucket(m.mhash[j], m.smask, kMixMul);
    for (;;) {
      uint32_t old = atomicCAS(&m.scratch[s], kEmpty, j);
      if (old == kEmpty) break;
      const uint32_t *ko = m.mkey + 4 * (size_t)old;
      if (m.mhash[old] == m.mhash[j] && key_eq(ko, kj)) {
        if (j < old) atomicMin(&m.scratch[s], j);  // (a later packet holds the slot)
        break;
      }
      s = (s + 1) & m.smask;
    }
    m.rep[j] = s;
  }
}

__global__ void nk_first(NkArgs m) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x)
    m.first[j] = m.scratch[m.rep[j]] == j ? 1u : 0u;
}

// dchain_allocate_new_index for each first sighting in packet order: rank r
// takes the r-th free-list entry (stack top first, then never-used indices),
// then map_put of the key.
__global__ void nk_alloc(NkArgs m) {
  const TableDev &t = m.t;
  const uint32_t stack_top = t.ctl->stack_top;
  const uint32_t fresh = t.ctl->fresh_next;
  const uint32_t free_total = stack_top + (t.cap - fresh);
  uint32_t disp = 0, ins = 0;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    if (!m.first[j]) continue;
    const uint32_t r = m.rank[j];
    if (r >= free_total) {  // table full
      m.assign[j] = kNone;
      continue;
    }
    const uint32_t idx =
        r < stack_top ? t.stack[stack_top - 1 - r] : fresh + (r - stack_top);
    const uint32_t *key = m.mkey + 4 * (size_t)j;
    // owner mode: every rank allocates, only the key's owner inserts it
    const bool mine = !t.own_n || owner_of(m.mhash[j], t.own_n) == t.own_r;
    uint32_t e = kElsewhere;
    if (mine) {
      bool tomb = false;
      e = tbl_insert(t, m.mhash[j], key, idx, &tomb, &disp);
      if (tomb) atomicAdd(&t.ctl->tomb_reused, 1u);
      ins++;
    }
    if (t.kv) t.kv[idx] = make_uint4(key[0], key[1], key[2], key[3]);
    t.slot_of[idx] = e;
    t.hash_of[idx] = m.mhash[j];
    t.birth[idx] = m.seq_base + m.pos[j];
    m.assign[j] = idx;
  }
  for (uint32_t o = 32; o > 0; o >>= 1) {
    disp += __shfl_xor(disp, o);
    ins += __shfl_xor(ins, o);
  }
  if ((threadIdx.x & 63) == 0 && disp) atomicAdd(&t.ctl->disp_count, disp);
  if ((threadIdx.x & 63) == 0 && ins) atomicAdd(&t.ctl->sh_live, ins);
}

__global__ void nk_commit(NkArgs m) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Ctl *c = m.t.ctl;
  const uint32_t K = m.rank[m.n - 1] + m.first[m.n - 1];
  const uint32_t free_total = c->stack_top + (m.t.cap - c->fresh_next);
  const uint32_t used = K < free_total ? K : free_total;
  if (used <= c->stack_top) {
    c->stack_top -= used;
  } else {
    c->fresh_next += used - c->stack_top;
    c->stack_top = 0;
  }
  c->n_live += used;
  c->n_tomb -= c->tomb_reused;
  c->tomb_reused = 0;
  c->new_count = used;
}

// ---------------------------------------------------- unsorted new keys --
// (tbl_new_keys_unsorted, vp_table.h) Slot s of the key set: ord[s] = tag <<
// 32 | a miss ordinal holding the key, fpos = tag << 32 | ~first position
// (atomicMax keeps the earliest), lpos = tag << 32 | last position.
struct NkuArgs {
  TableDev t;
  const uint32_t *pos;  // miss j's entry: its packet position, or a slice slot
  const uint4 *key;
  const uint32_t *hash;
  const uint32_t *sq;  // the classify blocks' miss slices (kMissSlice entries)
  const uint4 *skey;
  const uint32_t *shash;
  uint32_t n, smask;
  unsigned long long *set;  // [3][smask + 1]
  uint32_t tag;
  uint32_t *rep, *bits, *pre, *first, *cnt;
  uint32_t p0, nwords;
  NowSpec now;
  uint64_t seq_base;
};

__device__ __forceinline__ uint32_t nku_pos(const NkuArgs &m, uint32_t j) {
  const uint32_t e = m.pos[j];
  return e & kMissSlice ? m.sq[e & ~kMissSlice] : e;
}
__device__ __forceinline__ uint4 nku_key(const NkuArgs &m, uint32_t j) {
  const uint32_t e = m.pos[j];
  return e & kMissSlice ? m.skey[e & ~kMissSlice] : m.key[j];
}
__device__ __forceinline__ uint32_t nku_hash(const NkuArgs &m, uint32_t j) {
  const uint32_t e = m.pos[j];
  return e & kMissSlice ? m.shash[e & ~kMissSlice] : m.hash[j];
}

__global__ void nku_dedup(NkuArgs m) {
  const size_t S = (size_t)m.smask + 1;
  unsigned long long *ord = m.set, *fp = m.set + S, *lp = m.set + 2 * S;
  const unsigned long long tg = (unsigned long long)m.tag << 32;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    const uint4 kj = nku_key(m, j);
    const uint32_t h = nku_hash(m, j);
    uint32_t s = home_bucket(h, m.smask, kMixMul);
    // (plain loads, which the XCD's L2 may serve stale: a slot word is
    // written once per call, from an older tag to this call's by the CAS, so
    // a stale word is an older tag, the CAS fails and returns the real one;
    // a stale fp / lp only costs an atomicMax that was not needed. Device-
    // scope loads bypassed the L2 on every probe.)
    for (;;) {
      unsigned long long cur = ord[s];
      if ((cur >> 32) != m.tag) {  // an empty slot (an older tag): claim it
        const unsigned long long old = atomicCAS(&ord[s], cur, tg | j);
        if (old == cur) break;
        cur = old;  // (someone of this call took it: compare)
      }
      const uint32_t o = (uint32_t)cur;
      const uint4 ko = nku_key(m, o);
      if (nku_hash(m, o) == h && ko.x == kj.x && ko.y == kj.y && ko.z == kj.z && ko.w == kj.w)
        break;
      s = (s + 1) & m.smask;
    }
    m.rep[j] = s;
    const uint32_t p = nku_pos(m, j);
    // (read first: a key's packets mostly arrive after its earliest and
    // before its latest was seen, and a load is cheaper than an atomic)
    const unsigned long long f = tg | (unsigned long long)(~p), l = tg | (unsigned long long)p;
    if (f > fp[s]) atomicMax(&fp[s], f);
    if (l > lp[s]) atomicMax(&lp[s], l);
  }
}

// First sightings: one bit per segment position, and their miss ordinals.
__global__ void nku_firsts(NkuArgs m) {
  const size_t S = (size_t)m.smask + 1;
  const unsigned long long *fp = m.set + S;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = nku_pos(m, j);
    bool f = (uint32_t)~(uint32_t)fp[m.rep[j]] == p;
    // (one first sighting per position: a packet queued twice counts once)
    if (f) {
      const uint32_t bit = 1u << ((p - m.p0) & 31);
      f = !(atomicOr(&m.bits[(p - m.p0) >> 5], bit) & bit);
    }
    if (f) atomicMax(&m.t.ctl->last_first, p - m.p0 + 1);  // (run_batch's cut)
    const uint32_t k = wave_append(m.cnt, f);
    if (f) m.first[k] = j;
  }
}

__global__ void nku_popc(const uint32_t *bits, uint32_t n, uint32_t *out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = (uint32_t)__popc(bits[i]);
}

// dchain_allocate_new_index for each first sighting by its rank in packet
// order, map_put of the key, birth at the first packet, stamps of the last.
__global__ void nku_alloc(NkuArgs m) {
  const TableDev &t = m.t;
  const size_t S = (size_t)m.smask + 1;
  const unsigned long long *lp = m.set + 2 * S;
  const uint32_t stack_top = t.ctl->stack_top;
  const uint32_t fresh = t.ctl->fresh_next;
  const uint32_t free_total = stack_top + (t.cap - fresh);
  const uint32_t K = *m.cnt;
  uint32_t disp = 0, ins = 0;
  for (uint32_t f = blockIdx.x * blockDim.x + threadIdx.x; f < K;
       f += gridDim.x * blockDim.x) {
    const uint32_t j = m.first[f];
    const uint32_t p = nku_pos(m, j), q = p - m.p0, s = m.rep[j];
    const uint32_t r = m.pre[q >> 5] + (uint32_t)__popc(m.bits[q >> 5] & ((1u << (q & 31)) - 1u));
    unsigned long long *ord = m.set;  // (the slot's word now carries the index)
    const unsigned long long tg = (unsigned long long)m.tag << 32;
    if (r >= free_total) {  // table full: nat_main.c:87-91
      ord[s] = tg | kNone;
      continue;
    }
    const uint32_t idx = r < stack_top ? t.stack[stack_top - 1 - r] : fresh + (r - stack_top);
    const uint4 k4 = nku_key(m, j);
    const uint32_t hj = nku_hash(m, j);
    const uint32_t key[4] = {k4.x, k4.y, k4.z, k4.w};
    bool tomb = false;
    const uint32_t e = tbl_insert(t, hj, key, idx, &tomb, &disp);
    if (tomb) atomicAdd(&t.ctl->tomb_reused, 1u);
    ins++;
    t.slot_of[idx] = e;
    t.hash_of[idx] = hj;
    t.birth[idx] = m.seq_base + p;
    const uint32_t last = (uint32_t)lp[s];  // the key's last packet: its stamps
    t.ts[idx] = (uint64_t)m.now.at(last);
    t.tseq[idx] = m.seq_base + last;
    ord[s] = tg | idx;
  }
  for (uint32_t o = 32; o > 0; o >>= 1) {
    disp += __shfl_xor(disp, o);
    ins += __shfl_xor(ins, o);
  }
  if ((threadIdx.x & 63) == 0 && disp) atomicAdd(&t.ctl->disp_count, disp);
  if ((threadIdx.x & 63) == 0 && ins) atomicAdd(&t.ctl->sh_live, ins);
}

__global__ void nku_commit(Ctl *c, uint32_t cap, const uint32_t *cnt) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t K = *cnt;
  const uint32_t free_total = c->stack_top + (cap - c->fresh_next);
  const uint32_t used = K < free_total ? K : free_total;
  if (used <= c->stack_top) {
    c->stack_top -= used;
  } else {
    c->fresh_next += used - c->stack_top;
    c->stack_top = 0;
  }
  c->n_live += used;
  c->n_tomb -= c->tomb_reused;
  c->tomb_reused = 0;
  c->new_count = used;
}

static int tbl_after_new_keys(vp_ctx *c, FlowTable &t);

int tbl_new_keys_unsorted(vp_ctx *c, FlowTable &t, uint32_t n, uint32_t p0, uint32_t p1,
                          const NowSpec &now, uint64_t seq_base) {
  Workspace &w = c->ws;
  if (!n) return 0;
  const uint64_t S = next_pow2(2ull * n);
  const uint32_t nwords = (p1 - p0 + 31) / 32;
  if (3 * S > w.nkset_n) {  // (zeroed once: tag 0 is never used)
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(w.nkset);
    w.nkset = nullptr;
    w.nkset_n = 0;
    VP_TRY(dalloc(&w.nkset, 3 * S));
    VP_HIP(hipMemsetAsync(w.nkset, 0, 8 * 3 * S, c->stream));
    w.nkset_n = 3 * S;
    w.nk_tag = 0;
  }
  if (nwords + 1 > w.nkbits_n) {
    VP_HIP(hipStreamSynchronize(c->stream));
    for (uint32_t **p : {&w.nkbits, &w.nkpre}) {
      hipFree(*p);
      *p = nullptr;
    }
    w.nkbits_n = 0;
    VP_TRY(dalloc(&w.nkbits, nwords + 1));
    VP_TRY(dalloc(&w.nkpre, nwords + 1));
    w.nkbits_n = nwords + 1;
  }
  if (n > w.nkfirst_n) {
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(w.nkfirst);
    w.nkfirst = nullptr;
    w.nkfirst_n = 0;
    VP_TRY(dalloc(&w.nkfirst, n));
    w.nkfirst_n = n;
  }
  if (!w.nkcnt) VP_TRY(dalloc(&w.nkcnt, 1));
  // the set's layout depends on its size: a new size starts a new tag space
  // (the memory of an older, larger set holds only older tags)
  if (++w.nk_tag == 0) {
    VP_HIP(hipMemsetAsync(w.nkset, 0, 8 * w.nkset_n, c->stream));
    w.nk_tag = 1;
  }
  NkuArgs m{};
  m.t = tbl_dev(t);
  m.pos = w.miss;
  m.key = reinterpret_cast<const uint4 *>(w.mkey);
  m.hash = w.mhash;
  m.sq = w.missq;
  m.skey = w.mkq;
  m.shash = w.mhq;
  m.n = n;
  m.smask = (uint32_t)(S - 1);
  m.set = w.nkset;
  m.tag = w.nk_tag;
  m.rep = w.rep;
  m.bits = w.nkbits;
  m.pre = w.nkpre;
  m.first = w.nkfirst;
  m.cnt = w.nkcnt;
  m.p0 = p0;
  m.nwords = nwords;
  m.now = now;
  m.seq_base = seq_base;
  size_t need = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, need, w.nkpre, w.nkpre, (int)nwords, c->stream);
  VP_TRY(cub_reserve(c, need));
  VP_HIP(hipMemsetAsync(w.nkbits, 0, 4ull * nwords, c->stream));
  VP_HIP(hipMemsetAsync(w.nkcnt, 0, 4, c->stream));
  VP_HIP(hipMemsetAsync(&t.ctl->last_first, 0, 4, c->stream));
  const uint32_t g = grid_for(n);
  nku_dedup<<<g, 256, 0, c->stream>>>(m);
  nku_firsts<<<g, 256, 0, c->stream>>>(m);
  nku_popc<<<grid_for(nwords), 256, 0, c->stream>>>(w.nkbits, nwords, w.nkpre);
  VP_HIP(hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, w.cub_bytes, w.nkpre, w.nkpre,
                                          (int)nwords, c->stream));
  nku_alloc<<<g, 256, 0, c->stream>>>(m);
  nku_commit<<<1, 64, 0, c->stream>>>(t.ctl, t.cap, w.nkcnt);
  VP_HIP(hipGetLastError());
  return 0;
}

int tbl_new_keys_done(vp_ctx *c, FlowTable &t) {
  VP_TRY(read_ctl(c, t));
  return tbl_after_new_keys(c, t);
}

int tbl_new_keys(vp_ctx *c, FlowTable &t, const NewKeys &nk, uint64_t seq_base,
                 uint32_t *n_new) {
  Workspace &w = c->ws;
  NkArgs m{};
  m.t = tbl_dev(t);
  m.pos = nk.pos;
  m.n = nk.n;
  m.mkey = w.mkey;
  m.mhash = w.mhash;
  m.first = w.first;
  m.rank = w.rank;
  m.rep = w.rep;
  m.assign = w.assign;
  m.scratch = w.scratch;
  m.seq_base = seq_base;
  const uint32_t ssize = next_pow2((uint64_t)nk.n * 2);
  m.smask = ssize - 1;
  size_t need = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, need, w.first, w.rank, (int)nk.n,
                                   c->stream);
  VP_TRY(cub_reserve(c, need));
  VP_HIP(hipMemsetAsync(w.scratch, 0xFF, sizeof(uint32_t) * (size_t)ssize,
                        c->stream));
  const uint32_t g = grid_for(nk.n);
  nk_dedup<<<g, 256, 0, c->stream>>>(m);
  nk_first<<<g, 256, 0, c->stream>>>(m);
  VP_HIP(hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, w.cub_bytes, w.first,
                                          w.rank, (int)nk.n, c->stream));
  nk_alloc<<<g, 256, 0, c->stream>>>(m);
  nk_commit<<<1, 64, 0, c->stream>>>(m);
  VP_HIP(hipGetLastError());
  VP_TRY(read_ctl(c, t));
  if (n_new) *n_new = t.h_ctl.new_count;
  return tbl_after_new_keys(c, t);
}

// After new keys went in (h_ctl read back): the home-bucket layout checks.
static int tbl_after_new_keys(vp_ctx *c, FlowTable &t) {
  // A linear layout is exact-structured for GF(2)-linear key sets: either
  // well spread or clustered (a long probe, or a tenth of the keys past
  // their home bucket). Clustered: choose another layout and rebuild.
  t.ins_since += t.h_ctl.new_count;
  // first chance for the allocation-order layout (below), whatever the
  // current layout's clustering: it replaces it
  if (t.lin_ok && !t.lin_tried && !t.own_n && t.mix != kMixLin &&
      2ull * t.h_ctl.n_live > t.nb_base) {
    VP_TRY(tbl_try_linear(c, t));
    if (t.mix == kMixLin) {
      VP_HIP(hipMemsetAsync(&t.ctl->max_disp, 0, 4, c->stream));
      return 0;
    }
  }
  if ((t.mix < kMixMul || t.mix == kMixLin) &&
      (t.h_ctl.max_disp ||
       (t.ins_since >= 4096 && 10ull * t.h_ctl.disp_count > t.ins_since))) {
    VP_HIP(hipMemsetAsync(&t.ctl->max_disp, 0, 4, c->stream));
    VP_TRY(tbl_choose_layout(c, t));
  }
  return 0;
}

// ------------------------------------------------------ linear layout --
// The NFs allocate indices in arrival order (dchain_allocate_new_index), so
// flows that arrive together get consecutive indices; when their keys differ
// in a GF(2)-linear way (a counter in a key field: the reference's MoonGen
// traffic, bench.lua:54,125, sets udp.src = counter) the CRC hashes of index
// pairs 2^k apart differ by fixed vectors a_k = h(2^k) ^ h(0). A linear map L
// with L(a_k) = e_k sends index i's hash to bucket i ^ L(h(0)) (in the low
// bits), so packets that touch neighbouring flows read neighbouring buckets;
// rotated right by one bit (the default, VIGPATH_LIN=2) it puts indices 2m
// and 2m + 1 in one bucket of half as many: a tile's 64 rows are one 2 KB
// run instead of 64 scattered lines. Every NF's flow table
// allocates this way. L is fitted once, from the hashes of indices 0 and 2^k,
// kept only if at least 90 % of a sample of live indices land exactly in
// index order and under 1 % of the keys overflow their home bucket, and
// dropped by the clustering check like any other layout. For keys without
// that structure any full-rank L spreads like the CRC bits themselves.
static bool gf2_inverse(const uint32_t cols[32], uint32_t inv_rows[32]) {
  uint32_t row[32], aug[32];
  for (int r = 0; r < 32; r++) {
    row[r] = 0;
    for (int cc = 0; cc < 32; cc++) row[r] |= ((cols[cc] >> r) & 1u) << cc;
    aug[r] = 1u << r;
  }
  for (int cc = 0; cc < 32; cc++) {
    int piv = -1;
    for (int r = cc; r < 32; r++)
      if ((row[r] >> cc) & 1u) {
        piv = r;
        break;
      }
    if (piv < 0) return false;
    std::swap(row[cc], row[piv]);
    std::swap(aug[cc], aug[piv]);
    for (int r = 0; r < 32; r++)
      if (r != cc && ((row[r] >> cc) & 1u)) {
        row[r] ^= row[cc];
        aug[r] ^= aug[cc];
      }
  }
  for (int r = 0; r < 32; r++) inv_rows[r] = aug[r];
  return true;
}
static uint32_t gf2_apply(const uint32_t rows[32], uint32_t h) {
  uint32_t o = 0;
  for (int r = 0; r < 32; r++) o |= (uint32_t)(__builtin_popcount(rows[r] & h) & 1) << r;
  return o;
}

static int tbl_try_linear(vp_ctx *c, FlowTable &t) {
  t.lin_tried = true;
  // index bits: indices live below cap <= 2^nbits (the nominal bucket count)
  uint32_t nbits = 0;
  while ((1ull << nbits) < t.cap) nbits++;
  if (nbits < 7 || nbits > 31) return 0;
  const uint32_t imask = (1u << nbits) - 1;
  const uint32_t S = std::min<uint32_t>(t.cap, 1u << 16);
  // hashes and entries of indices 0 .. S-1 and 2^k (k < nbits)
  std::vector<uint32_t> h(S), e(S), hk(nbits), ek(nbits);
  VP_HIP(hipMemcpyAsync(h.data(), t.hash_of, 4ull * S, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipMemcpyAsync(e.data(), t.slot_of, 4ull * S, hipMemcpyDeviceToHost, c->stream));
  for (uint32_t k = 0; k < nbits; k++) {
    VP_HIP(hipMemcpyAsync(&hk[k], t.hash_of + (1u << k), 4, hipMemcpyDeviceToHost, c->stream));
    VP_HIP(hipMemcpyAsync(&ek[k], t.slot_of + (1u << k), 4, hipMemcpyDeviceToHost, c->stream));
  }
  VP_HIP(hipStreamSynchronize(c->stream));
  const uint32_t kFree = 0xFFFFFFFFu;  // slot_of of an index never allocated
  if (e[0] == kFree || e[0] >= kElsewhere) return 0;
  for (uint32_t k = 0; k < nbits; k++)
    if (ek[k] == kFree || ek[k] >= kElsewhere) return 0;
  // basis: a_0 .. a_{nbits-1}, completed with unit vectors
  uint32_t cols[32], echelon[32] = {};
  uint32_t n = 0;
  auto add = [&](uint32_t v) {  // independent of the columns so far?
    uint32_t x = v;
    for (int b = 31; b >= 0; b--)
      if ((x >> b) & 1u) {
        if (!echelon[b]) {
          echelon[b] = x;
          cols[n++] = v;
          return true;
        }
        x ^= echelon[b];
      }
    return false;
  };
  for (uint32_t k = 0; k < nbits; k++)
    if (!add(hk[k] ^ h[0])) return 0;  // rank-deficient: no such layout
  for (uint32_t b = 0; b < 32 && n < 32; b++) add(1u << b);
  uint32_t inv[32];
  if (n != 32 || !gf2_inverse(cols, inv)) return 0;
  const uint32_t base = gf2_apply(inv, h[0]) & imask;
  uint64_t live = 0, exact = 0;
  for (uint32_t i = 0; i < S; i++) {
    if (e[i] == kFree || e[i] >= kElsewhere) continue;
    live++;
    exact += ((gf2_apply(inv, h[i]) & imask) ^ base) == i;
  }
  if (!live || 10 * exact < 9 * live) return 0;
  // 2^nbits buckets, one index each; pairs: rotate the map right by one bit,
  // so indices 2m and 2m + 1 share a bucket of half as many (2^nbits / 2
  // buckets x 3 entries >= cap; every key in its home bucket): a tile's 64
  // rows are 2 KB, half the row bytes per packet
  const bool pairs = t.lin_ok >= 2;
  const uint64_t nb = pairs ? 1ull << (nbits - 1) : 1ull << nbits;
  std::vector<uint32_t> tab(1024);
  for (uint32_t j = 0; j < 4; j++)
    for (uint32_t v = 0; v < 256; v++) {
      const uint32_t x = gf2_apply(inv, v << (8 * j));
      tab[256 * j + v] = pairs ? (x >> 1) | (x << 31) : x;
    }
  if (!t.lin) VP_TRY(dalloc(&t.lin, 1024));
  VP_HIP(hipMemcpyAsync(t.lin, tab.data(), 4096, hipMemcpyHostToDevice, c->stream));
  // spread check over every live key, then rebuild in the new layout
  uint32_t *cnt = nullptr, *over = nullptr;
  VP_TRY(dalloc(&cnt, nb));
  VP_TRY(dalloc(&over, 1));
  VP_HIP(hipMemsetAsync(over, 0, 4, c->stream));
  VP_HIP(hipMemsetAsync(cnt, 0, 4 * nb, c->stream));
  TableDev d = tbl_dev(t);
  d.bmask = (uint32_t)(nb - 1);
  lay_count<<<grid_for(t.cap), 256, 0, c->stream>>>(d, kMixLin, cnt);
  lay_score<<<grid_for(nb), 256, 0, c->stream>>>(cnt, (uint32_t)nb, over);
  VP_HIP(hipGetLastError());
  uint32_t h_over = 0;
  VP_HIP(hipMemcpyAsync(&h_over, over, 4, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipStreamSynchronize(c->stream));
  hipFree(cnt);
  hipFree(over);
  VP_TRY(read_ctl(c, t));
  if (100ull * h_over > t.h_ctl.sh_live) return 0;
  if (getenv("VIGPATH_DEBUG"))
    fprintf(stderr, "vigpath: linear layout: %llu of %llu sampled indices in order, "
            "%u keys past home\n", (unsigned long long)exact, (unsigned long long)live,
            h_over);
  t.mix = kMixLin;
  return tbl_rebuild(c, t, nb);
}

// ---------------------------------------------------------------- layout --
// Score a home-bucket mode over this rank's live keys: the number of keys
// beyond the 3 entries of their home bucket.
__global__ void lay_count(TableDev t, uint32_t mix, uint32_t *cnt) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < t.cap;
       i += gridDim.x * blockDim.x)
    if (t.slot_of[i] < kElsewhere)
      atomicAdd(&cnt[home_bucket(t.hash_of[i], t.bmask, mix, t.lin)], 1u);
}
__global__ void lay_score(const uint32_t *cnt, uint32_t nb, uint32_t *over) {
  uint32_t o = 0;
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nb;
       b += gridDim.x * blockDim.x)
    o += cnt[b] > kBucketEntries ? cnt[b] - kBucketEntries : 0;
  for (uint32_t s = 32; s > 0; s >>= 1) o += __shfl_xor(o, s);
  if ((threadIdx.x & 63) == 0 && o) atomicAdd(over, o);
}

// Every rotation of the CRC bits (modes 0-31) scored over the live keys; the
// cleanest one if few keys overflow their home bucket, else the
// multiplicative spread. Then rebuild. A table that keeps clustering after
// a few choices stays multiplicative.
static int tbl_choose_layout(vp_ctx *c, FlowTable &t) {
  if (t.mix == kMixLin) {  // the keys lost their structure: back to the CRC bits
    if (getenv("VIGPATH_DEBUG")) fprintf(stderr, "vigpath: linear layout dropped\n");
    t.mix = 0;
    return tbl_rebuild(c, t, t.nb_nominal);
  }
  const uint64_t nb = (uint64_t)t.bmask + 1;
  uint32_t best = kMixMul;
  if (++t.layout_tries <= 4) {
    uint32_t *cnt = nullptr, *over = nullptr;
    VP_TRY(dalloc(&cnt, nb));
    VP_TRY(dalloc(&over, 32));
    VP_HIP(hipMemsetAsync(over, 0, 4 * 32, c->stream));
    for (uint32_t m = 0; m < 32; m++) {
      VP_HIP(hipMemsetAsync(cnt, 0, 4 * nb, c->stream));
      lay_count<<<grid_for(t.cap), 256, 0, c->stream>>>(tbl_dev(t), m, cnt);
      lay_score<<<grid_for(nb), 256, 0, c->stream>>>(cnt, (uint32_t)nb, over + m);
    }
    VP_HIP(hipGetLastError());
    uint32_t h_over[32];
    VP_HIP(hipMemcpyAsync(h_over, over, sizeof h_over, hipMemcpyDeviceToHost, c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(cnt);
    hipFree(over);
    VP_TRY(read_ctl(c, t));
    uint32_t m_best = 0;
    for (uint32_t m = 1; m < 32; m++)
      if (h_over[m] < h_over[m_best]) m_best = m;
    // clean enough (under 1 % of the keys overflow) and not the layout
    // that just clustered
    if (m_best != t.mix && 100ull * h_over[m_best] <= t.h_ctl.sh_live) best = m_best;
  }
  t.mix = best;
  return tbl_rebuild(c, t);
}

// ---------------------------------------------------------- touch log --
// The index space is cut into chunks of 2^cb indices (one LDS tile of
// last-toucher positions per chunk; cb is chosen per table so that there are
// about 512 chunks, enough blocks to fill the chip in pass 3). The log is cut
// into spans of `span` entries. Pass 1 counts each span's touches per chunk,
// an exclusive scan turns the counts into (chunk, span) offsets, pass 2
// scatters one packed word per touch into chunk order:
//   (index within chunk) << 20 | (position within span)
// and pass 3 recovers each word's span from the chunk's span offsets (LDS),
// keeps the largest position per index with LDS atomics and writes ts/tseq.
// About 16 B of streaming traffic per packet, no global atomics.
constexpr uint32_t kPosBits = 20;  // position within a span (span <= 2^20)
constexpr uint32_t kMaxChunkBits = 12;
constexpr uint32_t kMaxSpans = 8192;  // pass-3 LDS offset table (+1)

__global__ __launch_bounds__(256) void touch_count(const uint32_t *log,
                                                   uint32_t n, uint32_t span,
                                                   uint32_t cb, uint32_t nchunks,
                                                   uint32_t nspans,
                                                   uint32_t *hist) {
  extern __shared__ uint32_t cnt[];
  for (uint32_t b = threadIdx.x; b < nchunks; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  const uint32_t s0 = blockIdx.x * span, s1 = min(n, s0 + span);
  for (uint32_t j = s0 + threadIdx.x; j < s1; j += 4 * blockDim.x) {
    uint32_t k[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {  // 4 independent loads in flight
      const uint32_t jj = j + u * blockDim.x;
      k[u] = jj < s1 ? log[jj] : kNone;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) group_reserve(cnt, k[u] >> cb, k[u] != kNone);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nchunks; b += blockDim.x)
    hist[(size_t)b * nspans + blockIdx.x] = cnt[b];
}

__global__ __launch_bounds__(256) void touch_scatter(const uint32_t *log,
                                                     uint32_t n, uint32_t span,
                                                     uint32_t cb, uint32_t nchunks,
                                                     uint32_t nspans,
                                                     const uint32_t *off,
                                                     uint32_t *out) {
  extern __shared__ uint32_t pos[];
  for (uint32_t b = threadIdx.x; b < nchunks; b += blockDim.x)
    pos[b] = off[(size_t)b * nspans + blockIdx.x];
  __syncthreads();
  const uint32_t cmask = (1u << cb) - 1;
  const uint32_t s0 = blockIdx.x * span, s1 = min(n, s0 + span);
  for (uint32_t j = s0 + threadIdx.x; j < s1; j += 4 * blockDim.x) {
    uint32_t k[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t jj = j + u * blockDim.x;
      k[u] = jj < s1 ? log[jj] : kNone;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const bool v = k[u] != kNone;
      const uint32_t at = group_reserve(pos, k[u] >> cb, v);
      if (v) out[at] = ((k[u] & cmask) << kPosBits) | (j + u * blockDim.x - s0);
    }
  }
}

__global__ void touch_total(const uint32_t *hist, const uint32_t *off,
                            uint32_t nh, uint32_t *total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *total = off[nh - 1] + hist[nh - 1];
}

// One block per (chunk, part); the part's words are taken in groups of 64
// consecutive ones per wave instruction. A group's first span is found by a
// wave-uniform binary search over the chunk's span offsets (LDS); each lane
// then steps forward over the span boundaries inside the group. With one part
// per chunk the block owns its indices and writes ts/tseq; with several
// (small tables: too few chunks to fill the chip) the parts combine their
// maxima in `lastg` and touch_finalize writes ts/tseq.
__global__ __launch_bounds__(1024) void touch_reduce_k2(
    const uint32_t *in, const uint32_t *off, uint32_t span, uint32_t nspans,
    uint32_t cb, uint32_t nchunks, uint32_t split, const uint32_t *total,
    uint32_t cap, uint32_t p0, NowSpec now, uint64_t seq_base, uint64_t *ts,
    uint64_t *tseq, uint32_t *lastg) {
  __shared__ uint32_t last[1u << kMaxChunkBits];  // 1 + last position, 0 = none
  __shared__ uint32_t so[kMaxSpans + 1];          // this chunk's span offsets
  const uint32_t ch = blockIdx.x / split, part = blockIdx.x % split;
  const uint32_t csize = 1u << cb;
  for (uint32_t i = threadIdx.x; i < csize; i += blockDim.x) last[i] = 0;
  for (uint32_t s = threadIdx.x; s < nspans; s += blockDim.x)
    so[s] = off[(size_t)ch * nspans + s];
  if (threadIdx.x == 0)
    so[nspans] = ch + 1 < nchunks ? off[(size_t)(ch + 1) * nspans] : *total;
  __syncthreads();
  const uint32_t ca = so[0], ce = so[nspans];
  const uint32_t per = (ce - ca + split - 1) / split;
  const uint32_t a = min(ce, ca + part * per), b = min(ce, a + per);
  const uint32_t lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t pmask = (1u << kPosBits) - 1;
  constexpr uint32_t kU = 4;  // groups in flight per wave
  for (uint32_t g0 = a + (threadIdx.x >> 6) * 64; g0 < b; g0 += kU * nw * 64) {
    uint32_t e[kU], sp[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t j0 = g0 + u * nw * 64, jj = j0 + lane;
      e[u] = jj < b ? in[jj] : kNone;
      uint32_t lo = 0, hi = nspans;  // largest s with so[s] <= j0 (uniform)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (so[mid] <= j0) lo = mid; else hi = mid;
      }
      while (lo + 1 < nspans && so[lo + 1] <= jj) lo++;
      sp[u] = lo;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; u++)
      if (e[u] != kNone)
        atomicMax(&last[e[u] >> kPosBits], sp[u] * span + (e[u] & pmask) + 1);
  }
  __syncthreads();
  const uint32_t base = ch << cb;
  for (uint32_t i = threadIdx.x; i < csize && base + i < cap; i += blockDim.x) {
    const uint32_t l = last[i];
    if (!l) continue;
    if (split > 1) {
      atomicMax(&lastg[base + i], l);
      continue;
    }
    const uint32_t p = p0 + l - 1;
    ts[base + i] = (uint64_t)now.at(p);
    tseq[base + i] = seq_base + p;
  }
}

__global__ void touch_finalize(const uint32_t *lastg, uint32_t cap, uint32_t p0,
                               NowSpec now, uint64_t seq_base, uint64_t *ts,
                               uint64_t *tseq) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += gridDim.x * blockDim.x) {
    const uint32_t l = lastg[i];
    if (!l) continue;
    const uint32_t p = p0 + l - 1;
    ts[i] = (uint64_t)now.at(p);
    tseq[i] = seq_base + p;
  }
}

int tbl_touch_reduce(vp_ctx *c, FlowTable &t, const uint32_t *log, uint32_t p0,
                     uint32_t p1, const NowSpec &now, uint64_t seq_base) {
  Workspace &w = c->ws;
  const uint32_t n = p1 - p0;
  if (n == 0) return 0;
  // ~512 chunks of 2^cb indices (64 <= 2^cb <= 4096)
  uint32_t cb = 6;
  while (cb < kMaxChunkBits && ((uint64_t)t.cap >> (cb + 1)) >= 512) cb++;
  const uint32_t nchunks = (t.cap + (1u << cb) - 1) >> cb;
  // spans of >= 16384 entries, at most kMaxSpans of them
  uint32_t span = 16384;
  while ((uint64_t)span * kMaxSpans < n) span <<= 1;
  if (span > (1u << kPosBits)) return VP_ENOTSUP;
  const uint32_t nspans = (n + span - 1) / span;
  const uint64_t nh = (uint64_t)nchunks * nspans;
  const size_t lds = sizeof(uint32_t) * nchunks;
  if (lds > 64 * 1024) return VP_ENOTSUP;
  hipStream_t ts = c->stream;
  if (nh > w.hist_cap) {
    VP_HIP(hipStreamSynchronize(ts));
    hipFree(w.hist);
    hipFree(w.hoff);
    w.hist = w.hoff = nullptr;
    w.hist_cap = 0;
    VP_TRY(dalloc(&w.hist, nh));
    VP_TRY(dalloc(&w.hoff, nh));
    w.hist_cap = nh;
  }
  size_t need = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, need, w.hist, w.hoff, (int)nh, ts);
  VP_TRY(cub_reserve(c, need));
  uint32_t *hist = w.hist, *off = w.hoff;
  // (a buffer of its own: phase A leaves one-GPU misses' keys in mkey)
  uint32_t *pairs = w.pairs;
  touch_count<<<nspans, 256, lds, ts>>>(log + p0, n, span, cb, nchunks, nspans,
                                        hist);
  VP_HIP(hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, w.cub_bytes, hist, off,
                                          (int)nh, ts));
  touch_scatter<<<nspans, 256, lds, ts>>>(log + p0, n, span, cb, nchunks, nspans,
                                          off, pairs);
  touch_total<<<1, 64, 0, ts>>>(hist, off, (uint32_t)nh, t.ttotal);
  // enough blocks to cover the chip, splitting chunks when there are few
  const uint32_t split = std::max<uint32_t>(1, 512 / nchunks);
  if (split > 1)
    VP_HIP(hipMemsetAsync(t.lastg, 0, sizeof(uint32_t) * (size_t)t.cap, ts));
  touch_reduce_k2<<<nchunks * split, 1024, 0, ts>>>(
      pairs, off, span, nspans, cb, nchunks, split, t.ttotal, t.cap, p0, now,
      seq_base, t.ts, t.tseq, t.lastg);
  if (split > 1)
    touch_finalize<<<grid_for(t.cap), 256, 0, ts>>>(t.lastg, t.cap, p0, now,
                                                   seq_base, t.ts, t.tseq);
  VP_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------- touch bins --
// Single-pass fold of the touch bins a 64-byte classify launch filled
// (TouchBins, vp_device.h): one block per bin keeps the largest position per
// in-bin index in LDS, reading every source block's slice of its bin (one
// contiguous region: the slices are bin-major), then
// writes ts/tseq in runs of 64 consecutive indices. About 8 B of traffic per
// packet (one write while classifying, one read here).
constexpr uint32_t kBinLocalMax = 16384;  // in-bin indices held in LDS

template <uint32_t kU>  // 64-entry chunks in flight per wave
__global__ __launch_bounds__(1024) void touch_bins_reduce(
    const uint32_t *ent, const uint32_t *cnt, uint32_t nsrc, uint32_t cap,
    uint32_t pbits, uint32_t bbits, uint32_t range, uint32_t L, uint32_t tcap,
    uint32_t p0, NowSpec now, uint64_t seq_base, uint64_t *ts, uint64_t *tseq,
    PubArgs pub, const uint32_t *rtab, uint32_t sbits, uint32_t maxmode, uint32_t rwords) {
  // 1 + position in the launch, 0 = none; L words of dynamic LDS (16 KB at
  // 1M flows: the 256 bin blocks spread over all CUs, where a 64 KB static
  // array let only two blocks share a CU and left half of them idle)
  // Behind it, one word per 64-index group of the bin: the largest base
  // (1 + position of lane 0) of the run words that cover the group, so a run
  // costs one lane's atomic instead of 64 (its lane j touched index 64 g + j
  // at base + j, the same winner for all 64).
  // With 2^sbits blocks per bin (fewer bins than fold blocks), block
  // (bin, part) keeps in-bin indices [lo, lo + Lp) and skips the rest of the
  // bin's entries and runs (each part reads them all).
  extern __shared__ uint32_t last[];
  const uint32_t Lp = L >> sbits;
  uint32_t *grp = last + Lp;
  const uint32_t bin = blockIdx.x >> sbits, lo = (blockIdx.x & ((1u << sbits) - 1)) * Lp;
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl_publish(pub);
  for (uint32_t i = threadIdx.x; i < Lp + (Lp >> kBinRunBits); i += blockDim.x) last[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t pmask = (1u << pbits) - 1;
  // wave w takes slices w, w + nw, ...; 64 of them per round, their sizes
  // loaded by one instruction (lane l <-> slice w + l * nw). The round's
  // slices are one list of 64-entry chunks (chunk t of the list belongs to
  // the lane whose exclusive prefix of chunk counts covers t), read kU chunks
  // at a time whatever the slices' lengths.
  for (uint32_t r0 = threadIdx.x >> 6; r0 < nsrc; r0 += 64 * nw) {
    const uint32_t my = r0 + lane * nw;
    // the slice's run words, all loaded beside its count (one round trip; a
    // word past the slice's count is stale and ignored). Loaded one by one
    // behind the first two, eight words of 1024-thread blocks cost the fold
    // six more round trips (profiles/r06af_fold_runs.txt); both addresses
    // first, so no load's address registers are reused while it is in
    // flight (a wait for it, in the compiled order)
    const size_t ri = (((size_t)my << bbits) + bin) * rwords;
    const uint32_t *cp = cnt + (size_t)bin * nsrc + my;
    uint32_t rw[kBinRunWordsMax];
    if (rwords == kBinRunWordsMax) {  // (32-byte aligned: ri is a multiple of 8)
      const uint4 *q = reinterpret_cast<const uint4 *>(rtab + ri);
      const uint4 x = my < nsrc ? q[0] : make_uint4(0, 0, 0, 0);
      const uint4 y = my < nsrc ? q[1] : make_uint4(0, 0, 0, 0);
      rw[0] = x.x, rw[1] = x.y, rw[2] = x.z, rw[3] = x.w;
      rw[4] = y.x, rw[5] = y.y, rw[6] = y.z, rw[7] = y.w;
    } else {
      rw[0] = my < nsrc ? rtab[ri] : 0u;
      rw[1] = my < nsrc ? rtab[ri + 1] : 0u;
#pragma unroll
      for (uint32_t j = 2; j < kBinRunWordsMax; j++) rw[j] = 0;
    }
    const uint32_t raw = my < nsrc ? *cp : 0;
    const uint32_t nv = raw & ~kBinRunFlags, nr = raw >> kBinRunShift;
    const uint32_t re = rw[0], re2 = rw[1];
    const bool run = nr > 0, run2 = nr > 1;
    const uint32_t ch = (nv + 63) >> 6;
    uint32_t inc = ch;  // inclusive prefix over the wave
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
      if (lane >= o) inc += t;
    }
    const uint32_t exc = inc - ch;
    const uint32_t total = __builtin_amdgcn_readlane(inc, 63);
    for (uint32_t t0 = 0; t0 < total; t0 += kU) {
      uint32_t e[kU], lim[kU], base[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; u++) {
        const uint32_t t = t0 + u;
        const uint64_t own = __ballot(exc <= t && t < inc);  // (none past the list)
        const uint32_t l = own ? (uint32_t)__ffsll((unsigned long long)own) - 1 : 0u;
        const uint32_t k = (t - __builtin_amdgcn_readlane(exc, l)) << 6;
        const uint32_t sb = r0 + l * nw;
        lim[u] = own ? __builtin_amdgcn_readlane(nv, l) - k : 0u;
        base[u] = sb * range + 1;
        e[u] = lane < lim[u] ? ent[((size_t)bin * nsrc + sb) * cap + k + lane] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < kU; u++)
        if (lane < lim[u] && (e[u] >> pbits) - lo < Lp)
          atomicMax(&last[(e[u] >> pbits) - lo], base[u] + (e[u] & pmask));
    }
    if (run && ((re >> 20) << kBinRunBits) - lo < Lp)
      atomicMax(&grp[(re >> 20) - (lo >> kBinRunBits)], my * range + 1 + (re & 0xFFFFFu));
    if (run2 && ((re2 >> 20) << kBinRunBits) - lo < Lp)
      atomicMax(&grp[(re2 >> 20) - (lo >> kBinRunBits)], my * range + 1 + (re2 & 0xFFFFFu));
#pragma unroll
    for (uint32_t j = 2; j < kBinRunWordsMax; j++) {  // (1024-thread classify blocks)
      const uint32_t rj = rw[j];
      if (j < rwords && j < nr && ((rj >> 20) << kBinRunBits) - lo < Lp)
        atomicMax(&grp[(rj >> 20) - (lo >> kBinRunBits)], my * range + 1 + (rj & 0xFFFFFu));
    }
  }
  __syncthreads();
  for (uint32_t l = threadIdx.x; l < Lp; l += blockDim.x) {
    const uint32_t g = grp[l >> kBinRunBits];
    const uint32_t v = max(last[l], g ? g + (l & (kBinRun - 1)) : 0u);
    const uint32_t i = bin_index(bin, lo + l, bbits);
    if (!v || i >= tcap) continue;
    const uint32_t p = p0 + v - 1;
    // (maxmode: a second fold of the same segment, BinsPlan::maxmode; one
    // thread per index, so the compare needs no atomic)
    if (maxmode && tseq[i] >= seq_base + p) continue;
    ts[i] = (uint64_t)now.at(p);
    tseq[i] = seq_base + p;
  }
}

static uint32_t ceil_log2(uint64_t v) {
  uint32_t b = 0;
  while ((1ull << b) < v) b++;
  return b;
}

int tbl_bins_plan(vp_ctx *c, FlowTable &t, const void *kernel, uint32_t p0,
                  uint32_t p1, BinsPlan *plan, uint32_t waves, uint32_t min_bits,
                  uint32_t vper) {
  Workspace &w = c->ws;
  *plan = BinsPlan{};
  const char *env = getenv("VIGPATH_TOUCH_BINS");  // diagnostics: 0 = off
  if ((env && !atoi(env)) || (p0 & 63) || p1 <= p0) return 0;
  const uint32_t tiles = (p1 - p0 + 63) / 64;
  const uint32_t grid = vper ? (tiles + vper - 1) / vper
                            : resident_grid(kernel, (tiles + waves - 1) / waves,
                                            64 * (int)waves);
  const uint32_t per_b = vper ? vper : (tiles + grid - 1) / grid;
  const uint32_t range = per_b * 64;
  // The fewest bins (>= 2^bbits_min) whose in-bin index range fits the
  // fold's LDS, and at least 256 fold blocks whatever the bin count (2^sbits
  // per bin). A block keeps one partly written line per bin slice: at 256
  // bins, 32 MB over the chip, as much as all the L2s, which shuffled
  // touches (no runs) pay for (tools/sessions/gpu_r04ba.sh);
  // two run words per block and bin keep round robin whole at 128.
  static const uint32_t bbits_min = [] {  // (VIGPATH_BIN_BITS, for A/B)
    const char *e = getenv("VIGPATH_BIN_BITS");
    const int v = e ? atoi(e) : 7;
    return v >= 6 && v <= 10 ? (uint32_t)v : 7u;
  }();
  auto split = [](uint32_t bb) { return bb < 8 ? 8 - bb : 0u; };
  auto in_bin = [&](uint32_t bb) {  // in-bin index range for 2^bb bins: a
    // whole number of runs per fold block
    const uint32_t q = kBinRunBits + split(bb);
    return (((uint64_t)t.cap + ((uint64_t)1 << (q + bb)) - 1) >> (q + bb)) << q;
  };
  uint32_t bbits = std::max(bbits_min, std::min<uint32_t>(min_bits, 10));
  while (bbits < 10 && (in_bin(bbits) >> split(bbits)) > kBinLocalMax) bbits++;
  const uint32_t sbits = split(bbits);
  const uint32_t nbins = 1u << bbits;
  const uint32_t L = (uint32_t)in_bin(bbits);
  const uint32_t pbits = std::max<uint32_t>(1, ceil_log2(range));
  if ((L >> sbits) > kBinLocalMax || ceil_log2(L) + pbits > 32) return 0;
  // twice a uniform share of a block's packets per bin, and at least two
  // waves' worth (a wave touching 64 consecutive indices fills one bin)
  const uint32_t cap =
      std::max<uint32_t>(((2 * range / nbins + 32) + 15) & ~15u, 2 * kBinRun);
  const size_t ne = (size_t)grid * nbins * cap, nc = (size_t)grid * nbins;
  if (ne > w.bins_ent_n) {
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(w.bins_ent);
    w.bins_ent = nullptr;
    w.bins_ent_n = 0;
    VP_TRY(dalloc(&w.bins_ent, ne));
    w.bins_ent_n = ne;
  }
  if (nc > w.bins_cnt_n) {
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(w.bins_cnt);
    w.bins_cnt = nullptr;
    w.bins_cnt_n = 0;
    VP_TRY(dalloc(&w.bins_cnt, nc));
    w.bins_cnt_n = nc;
  }
  plan->on = true;  // (the segment's counter reset clears touch_ovf)
  plan->grid = grid;
  plan->range = range;
  plan->L = L;
  plan->sbits = sbits;
  // run words per block and bin: two, eight for one block per CU (512- to
  // 1024-thread blocks: four times the range); positions below 2^20 within
  // a block
  const uint32_t rwords = waves >= 8 ? kBinRunWordsMax : 2u;
  const size_t nr = ((size_t)grid << bbits) * rwords;
  if (nr > w.bins_rtab_n) {
    VP_HIP(hipStreamSynchronize(c->stream));
    hipFree(w.bins_rtab);
    w.bins_rtab = nullptr;
    w.bins_rtab_n = 0;
    VP_TRY(dalloc(&w.bins_rtab, nr));
    w.bins_rtab_n = nr;
  }
  static const uint32_t runs_env = [] {  // (VIGPATH_BIN_RUNS=0: off, for A/B)
    const char *e = getenv("VIGPATH_BIN_RUNS");
    return e ? (uint32_t)atoi(e) : 1u;
  }();
  const uint32_t runs = runs_env && range <= (1u << 20) && (L >> kBinRunBits) < (1u << 12);
  plan->bins = TouchBins{w.bins_ent, w.bins_cnt, &t.ctl->touch_ovf, w.ovf_q,
                         w.ovf_cnt, w.log, cap, pbits, bbits, grid, w.bins_rtab, runs,
                         rwords};
  return 0;
}

static int bins_reduce(vp_ctx *c, FlowTable &t, const BinsPlan &plan, uint32_t p0,
                       const NowSpec &now, uint64_t seq_base, PubArgs pub) {
  static const uint32_t rel = [] {  // (VIGPATH_PUB_RELEASE=1: ctl_publish's release form)
    const char *e = getenv("VIGPATH_PUB_RELEASE");
    return e && atoi(e) ? 1u : 0u;
  }();
  pub.rel = rel;
  // chunks in flight per fold wave (VIGPATH_FOLD_U: 8, 16 or 32; 16 and 32
  // measured no faster than 8, r03k)
  static const uint32_t fold_u = [] {
    const char *e = getenv("VIGPATH_FOLD_U");
    const int v = e ? atoi(e) : 0;
    return v == 16 || v == 32 ? (uint32_t)v : 8u;
  }();
  auto *fold = fold_u == 8 ? touch_bins_reduce<8> : fold_u == 32 ? touch_bins_reduce<32>
                                                                 : touch_bins_reduce<16>;
  const uint32_t Lp = plan.L >> plan.sbits;
  fold<<<1u << (plan.bins.bbits + plan.sbits), 1024, 4u * (Lp + (Lp >> kBinRunBits)),
         c->stream>>>(plan.bins.ent, plan.bins.cnt, plan.grid, plan.bins.cap, plan.bins.pbits,
                      plan.bins.bbits, plan.range, plan.L, t.cap, p0, now, seq_base, t.ts,
                      t.tseq, pub, plan.bins.rtab, plan.sbits, plan.maxmode ? 1u : 0u,
                      plan.bins.rwords);
  VP_HIP(hipGetLastError());
  return 0;
}

int tbl_bins_reduce(vp_ctx *c, FlowTable &t, const BinsPlan &plan, uint32_t p0,
                    const NowSpec &now, uint64_t seq_base, const PubArgs &pub) {
  return bins_reduce(c, t, plan, p0, now, seq_base, pub);
}

// Phase A's control block for the host, and the fold of phase A's touches
// behind it. With touch bins the fold kernel's first thread reads the block
// (the classify launch has completed: kernel boundary) and publishes it into
// host-coherent memory, so no copy launch and its kernel boundary sit between
// the classify and the fold; the host polls for it while the fold runs.
// One GPU, 64-byte tiles (pub_epoch != 0): the classify's last block has
// published it already (tile_publish, vp_nat.hip) and the fold only folds.
// Without bins: a copy behind phase A, then the log fold. On return h_ctl
// holds phase A's counts; the fold may still be running.
// Multi-GPU (every rank, every segment, so the collective always matches):
// the ranks' segment counters (miss .. reprobe, kPubGath words) are gathered
// on the device before the fold, which publishes them with the control
// block, and owner mode adds this rank's key count per owner (`sends`): the
// host learns all of it with the one wait it makes anyway (union_sizes,
// DESIGN.md §6).
// Wait for the control block a kernel published with `epoch` (ctl_publish)
// and copy it to t.h_ctl; a stream that ends (or fails) without it is an
// error.
int tbl_wait_pub(vp_ctx *c, FlowTable &t, uint32_t epoch) {
  for (uint32_t spin = 1;; spin++) {
    if (__atomic_load_n(&t.h_pub->epoch, __ATOMIC_ACQUIRE) == epoch) break;
    if ((spin & 1023) == 0) {
      const hipError_t e = hipStreamQuery(c->stream);
      if (e == hipSuccess && __atomic_load_n(&t.h_pub->epoch, __ATOMIC_ACQUIRE) != epoch)
        return state_fail("a kernel ended without publishing epoch %u (seen %u)", epoch,
                          __atomic_load_n(&t.h_pub->epoch, __ATOMIC_ACQUIRE));
      if (e != hipSuccess && e != hipErrorNotReady) VP_HIP(e);
    }
  }
  memcpy(&t.h_ctl, (const void *)&t.h_pub->ctl, sizeof(Ctl));
  return 0;
}

int tbl_fold_read_ctl(vp_ctx *c, FlowTable &t, const BinsPlan &bp, const uint32_t *log,
                      uint32_t p0, uint32_t p1, const NowSpec &now, uint64_t seq_base,
                      const uint32_t *sends, uint32_t pub_epoch) {
  Workspace &w = c->ws;
  const uint32_t nr = c->comm ? (uint32_t)c->comm->n : 0u;
  const uint32_t ns = sends ? nr : 0u;
  w.gath_ok = false;
  if (nr) {
    if (!w.gath) VP_TRY(dalloc(&w.gath, (size_t)kPubGath * kMaxRanks));
    static_assert(offsetof(Ctl, route_ovf) - offsetof(Ctl, miss_count) ==
                      4 * (kPubGath - 1), "miss_count .. route_ovf contiguous");
    VP_TRY(c->comm->allgather_dev(c, &t.ctl->miss_count, w.gath, 4 * kPubGath));
  }
  if (!bp.on) {
    VP_TRY(read_ctl_post(c, t));
    VP_TRY(tbl_touch_reduce(c, t, log, p0, p1, now, seq_base));
    VP_TRY(read_ctl_wait(c, t));
    if (nr) {
      std::vector<uint32_t> x((size_t)kPubGath * nr + ns);
      VP_HIP(hipMemcpy(x.data(), w.gath, 4ull * kPubGath * nr, hipMemcpyDeviceToHost));
      if (ns) VP_HIP(hipMemcpy(x.data() + kPubGath * nr, sends, 4ull * ns,
                               hipMemcpyDeviceToHost));
      w.h_gath.swap(x);
      w.gath_ok = true;
    }
    return 0;
  }
  // (pub_epoch != 0: the classify launch publishes the block itself, one GPU)
  const uint32_t epoch = pub_epoch ? pub_epoch : ++t.pub_epoch;
  VP_TRY(bins_reduce(c, t, bp, p0, now, seq_base,
                     pub_epoch ? PubArgs{}
                               : PubArgs{t.d_pub, t.ctl, epoch, w.gath, sends, kPubGath * nr,
                                         ns}));
  hostprof(3);
  VP_TRY(tbl_wait_pub(c, t, epoch));
  if (nr) {
    w.h_gath.assign(t.h_pub->xtra, t.h_pub->xtra + kPubGath * nr + ns);
    w.gath_ok = true;
  }
  return 0;
}

// After a reprobe kernel raised tseq[i] to the sequence of its packets'
// touches: the packet whose sequence won writes ts[i] (exactly one per index).
__global__ void reprobe_stamp(const uint32_t *list, const uint32_t *cnt, uint32_t n,
                              uint32_t range, uint32_t nblk, const uint32_t *log,
                              NowSpec now, uint64_t seq_base, uint64_t *ts,
                              const uint64_t *tseq) {
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const uint32_t nb = reprobe_slice_len(cnt, n, range, b);
    for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
      const uint32_t p = list[(size_t)b * range + k];
      const uint32_t i = log[p];
      if (i != kNone && tseq[i] == seq_base + p) ts[i] = (uint64_t)now.at(p);
    }
  }
}

// Late touches: every listed packet p with log[p] = i != kNone raises tseq[i]
// to its sequence; reprobe_stamp then stamps ts[i] for the winner.
__global__ void late_max(const uint32_t *list, const uint32_t *cnt, uint32_t n,
                         uint32_t range, uint32_t nblk, const uint32_t *log,
                         uint64_t seq_base, uint64_t *tseq) {
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const uint32_t nb = reprobe_slice_len(cnt, n, range, b);
    for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
      const uint32_t p = list[(size_t)b * range + k];
      const uint32_t i = log[p];
      if (i != kNone)
        atomicMax(reinterpret_cast<unsigned long long *>(tseq + i),
                  (unsigned long long)(seq_base + p));
    }
  }
}

int tbl_late_touches(vp_ctx *c, FlowTable &t, const uint32_t *list,
                     const uint32_t *cnt, uint32_t n, uint32_t range, uint32_t nblk,
                     const uint32_t *log, const NowSpec &now, uint64_t seq_base) {
  if (nblk == 0) return 0;
  const uint32_t g = std::min<uint32_t>(nblk, 2048);
  late_max<<<g, 256, 0, c->stream>>>(list, cnt, n, range, nblk, log, seq_base, t.tseq);
  reprobe_stamp<<<g, 256, 0, c->stream>>>(list, cnt, n, range, nblk, log, now,
                                          seq_base, t.ts, t.tseq);
  VP_HIP(hipGetLastError());
  return 0;
}

int tbl_reprobe_stamp(vp_ctx *c, FlowTable &t, const uint32_t *list,
                      const uint32_t *cnt, uint32_t n, uint32_t range, uint32_t nblk,
                      const uint32_t *log, const NowSpec &now, uint64_t seq_base) {
  reprobe_stamp<<<std::min<uint32_t>(nblk, 2048), 256, 0, c->stream>>>(
      list, cnt, n, range, nblk, log, now, seq_base, t.ts, t.tseq);
  VP_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- expiry --

// Every allocated index with ts < cutoff: the set expire_items_single_map
// frees (LRU order is (ts, last-touch) order, so the loop stops exactly at
// the first stamp >= cutoff).
// Two passes over the block's contiguous range of indices: count, one global
// atomic for the block's base, then append behind it (the set is sorted
// afterwards: its order here does not matter).
// The same pass also gives the exact floor after the expiry: the least ts of
// the allocated indices that stay (atomicMin into ctl->min_ts, reset by the
// caller), so no separate scan over the stamps and read-back follows.
__global__ __launch_bounds__(256) void exp_collect(TableDev t, int64_t cutoff, uint64_t *ekey,
                                                   uint32_t *eidx) {
  __shared__ uint32_t cnt, base;
  __shared__ unsigned long long wmin[4];
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const uint32_t per = (t.cap + gridDim.x - 1) / gridDim.x;
  const uint32_t i0 = blockIdx.x * per, i1 = min(t.cap, i0 + per);
  auto take_at = [&](uint32_t i) { return t.slot_of[i] != kNone && (int64_t)t.ts[i] < cutoff; };
  unsigned long long low = ~0ull;
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const bool live = t.slot_of[i] != kNone;
    const uint64_t ts = live ? t.ts[i] : ~0ull;
    const bool take = live && (int64_t)ts < cutoff;
    wave_append(&cnt, take);
    if (live && !take && ts < low) low = ts;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long v = __shfl_xor(low, o);
    low = v < low ? v : low;
  }
  if (__lane_id() == 0) wmin[threadIdx.x >> 6] = low;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t w = 1; w < blockDim.x / 64; w++) low = wmin[w] < low ? wmin[w] : low;
    if (low != ~0ull) atomicMin((unsigned long long *)&t.ctl->min_ts, low);
  }
  if (threadIdx.x == 0) {
    base = cnt ? atomicAdd(&t.ctl->exp_count, cnt) : 0u;
    cnt = 0;
  }
  __syncthreads();
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const bool take = take_at(i);
    const uint32_t k = base + wave_append(&cnt, take);
    if (take) {
      eidx[k] = i;
      ekey[k] = t.tseq[i];
    }
  }
}

// Free in LRU order: the oldest is pushed first, so the youngest expired
// index ends on top (double-chain-impl.c:1968-1981); erase the keys.
// (Owner mode: every rank frees the index; only the key's owner erases it.)
__global__ __launch_bounds__(256) void exp_apply(TableDev t, const uint32_t *eidx, uint32_t n) {
  __shared__ uint32_t tombs;
  if (threadIdx.x == 0) tombs = 0;
  __syncthreads();
  const uint32_t top = t.ctl->stack_top;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t idx = eidx[j];
    const uint32_t e = t.slot_of[idx];
    t.stack[top + j] = idx;
    const bool own = e < kElsewhere;
    if (own) t.bk[e >> 2].idx[e & 3] = kTomb;
    t.slot_of[idx] = kNone;
    wave_append(&tombs, own);  // (counted per block, one global atomic)
  }
  __syncthreads();
  if (threadIdx.x == 0 && tombs) atomicAdd(&t.ctl->n_tomb, tombs);
}

__global__ void exp_commit(Ctl *ctl, uint32_t n, uint32_t n_tomb_before) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    ctl->stack_top += n;
    ctl->n_live -= n;
    ctl->sh_live -= ctl->n_tomb - n_tomb_before;  // this rank's erasures
  }
}

// Rebuild (tombstone purge, layout change or growth): keys of this rank's
// live indices out, clear, re-insert.
__global__ void rb_collect(TableDev t, uint32_t *keys) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < t.cap;
       i += gridDim.x * blockDim.x) {
    if (t.slot_of[i] >= kElsewhere) continue;
    const uint4 k = tbl_key_of(t, i);
    reinterpret_cast<uint4 *>(keys)[i] = k;
  }
}
__global__ void rb_insert(TableDev t, const uint32_t *keys) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < t.cap;
       i += gridDim.x * blockDim.x) {
    if (t.slot_of[i] >= kElsewhere) continue;
    bool tomb = false;
    uint32_t disp = 0;
    t.slot_of[i] = tbl_insert(t, t.hash_of[i], keys + 4 * (size_t)i, i, &tomb, &disp);
  }
}

// nb_new: bucket count afterwards (0 = unchanged).
static int tbl_rebuild(vp_ctx *c, FlowTable &t, uint64_t nb_new) {
  t.rebuilds++;
  uint32_t *keys = reinterpret_cast<uint32_t *>(t.kv);  // owner mode: kv has them
  if (!keys) {
    VP_TRY(dalloc(&keys, 4ull * t.cap));
    rb_collect<<<grid_for(t.cap), 256, 0, c->stream>>>(tbl_dev(t), keys);
  }
  if (nb_new && nb_new != (uint64_t)t.bmask + 1) {
    VP_HIP(hipStreamSynchronize(c->stream));
    VP_HIP(hipFree(t.bk));
    t.bk = nullptr;
    VP_TRY(dalloc(&t.bk, nb_new));
    t.bmask = (uint32_t)(nb_new - 1);
  }
  VP_HIP(hipMemsetAsync(t.bk, 0xFF, sizeof(Bucket) * ((size_t)t.bmask + 1),
                        c->stream));
  rb_insert<<<grid_for(t.cap), 256, 0, c->stream>>>(tbl_dev(t), keys);
  VP_HIP(hipMemsetAsync(&t.ctl->n_tomb, 0, 4, c->stream));
  VP_HIP(hipMemsetAsync(&t.ctl->disp_count, 0, 4, c->stream));
  t.ins_since = 0;
  VP_HIP(hipStreamSynchronize(c->stream));
  if (!t.kv) VP_HIP(hipFree(keys));
  return 0;
}

int tbl_set_owner(vp_ctx *c, FlowTable &t, uint32_t n, uint32_t r) {
  // a fresh table: keys by index replicated, buckets sized for this rank's
  // share (grown on demand, tbl_owner_reserve)
  VP_TRY(dalloc(&t.kv, t.cap));
  t.own_n = n;
  t.own_r = r;
  uint64_t nb = 64;
  while (nb * n < t.cap) nb <<= 1;
  return tbl_rebuild(c, t, nb);
}

// Owner mode, before inserting a union of n keys (hashes in mhash): grow
// this rank's buckets so its keys stay at load <= 1/3 (one bucket per key).
__global__ void own_count(const uint32_t *mhash, uint32_t n, uint32_t own_n,
                          uint32_t own_r, Ctl *ctl) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t k = wave_append(&ctl->own_new, owner_of(mhash[j], own_n) == own_r);
    (void)k;
  }
}

int tbl_owner_reserve(vp_ctx *c, FlowTable &t, uint32_t n) {
  if (!t.own_n || !n) return 0;
  VP_HIP(hipMemsetAsync(&t.ctl->own_new, 0, 4, c->stream));
  own_count<<<grid_for(n), 256, 0, c->stream>>>(c->ws.mhash, n, t.own_n, t.own_r,
                                                t.ctl);
  VP_HIP(hipGetLastError());
  VP_TRY(read_ctl(c, t));
  const uint64_t need = (uint64_t)t.h_ctl.sh_live + t.h_ctl.n_tomb + t.h_ctl.own_new;
  if (need <= (uint64_t)t.bmask + 1) return 0;
  uint64_t nb = (uint64_t)t.bmask + 1;
  while (nb < need) nb <<= 1;
  return tbl_rebuild(c, t, nb);
}

// Expiry at `cutoff` (expire_items_single_map, expirator.c:110-218): every
// allocated index with ts < cutoff is freed in LRU order, and t.ts_floor
// becomes the exact least stamp of what stays. One scan (exp_collect, which
// also finds that floor), one read-back, one sort. LRU order is (ts, tseq)
// order, and a sort by tseq alone gives it: ts and tseq are the time and the
// global sequence of the same (last) touch, and times never decrease along
// the sequence (every batch's times are monotone and start at or after the
// last), so tseq_a < tseq_b implies ts_a <= ts_b.
int tbl_expire(vp_ctx *c, FlowTable &t, int64_t cutoff, uint32_t *n_out) {
  VP_HIP(hipMemsetAsync(&t.ctl->exp_count, 0, 4, c->stream));
  VP_HIP(hipMemsetAsync(&t.ctl->min_ts, 0xFF, 8, c->stream));
  exp_collect<<<grid_for(t.cap, 256, 512), 256, 0, c->stream>>>(tbl_dev(t), cutoff, t.ekey,
                                                                t.eidx);
  VP_HIP(hipGetLastError());
  VP_TRY(read_ctl(c, t));
  const uint32_t k = t.h_ctl.exp_count;
  t.ts_floor = t.h_ctl.min_ts;  // (~0: nothing stays)
  if (n_out) *n_out = k;
  if (k == 0) return 0;
  size_t need = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, need, t.ekey, t.ekey2, t.eidx,
                                     t.eidx2, (int)k, 0, 64, c->stream);
  VP_TRY(cub_reserve(c, need));
  VP_HIP(hipcub::DeviceRadixSort::SortPairs(c->ws.cub_tmp, c->ws.cub_bytes,
                                            t.ekey, t.ekey2, t.eidx, t.eidx2,
                                            (int)k, 0, 64, c->stream));
  exp_apply<<<grid_for(k), 256, 0, c->stream>>>(tbl_dev(t), t.eidx2, k);
  exp_commit<<<1, 64, 0, c->stream>>>(t.ctl, k, t.h_ctl.n_tomb);
  VP_HIP(hipGetLastError());
  if (t.own_n) return tbl_check_tombs(c, t);  // (only the owners' erasures are tombs)
  // one GPU: every expired index leaves a tombstone; the counters follow
  // without a read-back
  Ctl &h = t.h_ctl;
  h.stack_top += k;
  h.n_live -= k;
  h.n_tomb += k;
  h.sh_live -= k;
  const uint64_t base = std::min<uint64_t>(tbl_entries(t), t.nb_base * kBucketEntries);
  if ((uint64_t)h.n_tomb + h.sh_live > base * 85 / 100) return tbl_rebuild(c, t);
  return 0;
}

// Tombstones are purged (a rebuild) when they and the live entries fill 85 %
// of the entries of one bucket per index (nb_base), or of the table when it
// is smaller (the allocation-order layout): the spread tables' second bucket
// per index is headroom for short probe paths, not room for tombstones.
int tbl_check_tombs(vp_ctx *c, FlowTable &t) {
  VP_TRY(read_ctl(c, t));
  const uint64_t base = std::min<uint64_t>(tbl_entries(t), t.nb_base * kBucketEntries);
  if ((uint64_t)t.h_ctl.n_tomb + t.h_ctl.sh_live > base * 85 / 100)
    return tbl_rebuild(c, t);
  return 0;
}

// ---------------------------------------------------------- batch driver --

int ws_reserve(vp_ctx *c, uint32_t n);

// No entry of a table can expire at packet p while cutoff(t_p) <= min(live
// stamps); inside a segment starting at packet a the live stamps are
// >= min(ts_floor, t_a) (rejuvenation only raises stamps, new entries are
// stamped >= t_a). The batch is cut at the first packet where that fails for
// some table; there the exact expiry of that packet's nf_process runs.
static int run_batch_sharded(vp_ctx *c, const vp_dev_batch *b,
                             ExpiringTable *tabs, int ntabs, SegmentFn seg);

int run_batch(vp_ctx *c, const vp_dev_batch *b, ExpiringTable *tabs, int ntabs,
              SegmentFn seg, uint32_t exp_end) {
  if (c->comm) return run_batch_sharded(c, b, tabs, ntabs, seg);
  c->off = 0;
  const uint32_t n = b->n;
  c->last_ms = 0.f;
  c->last_launches = 0;
  if (n == 0) return 0;
  if (b->slot < 64 || (b->slot & 15) || !b->frames || ((uintptr_t)b->frames & 15) ||
      !b->len || (!b->in_dev && ((c->kind != KIND_NAT && c->kind != KIND_LB) || b->slot != 64)) || !b->out_dev)
    return VP_EINVAL;  // (frames are read as aligned 16-byte chunks; in_dev: see vp_process_device)
  VP_TRY(ws_reserve(c, n));

  std::vector<int64_t> h_copy;
  const int64_t *h_now = c->host_now;  // the caller's host copy, if any
  int64_t t_first, t_last;
  if (b->now) {
    if (!h_now) {
      h_copy.resize(n);
      VP_HIP(hipMemcpyAsync(h_copy.data(), b->now, sizeof(int64_t) * (size_t)n,
                            hipMemcpyDeviceToHost, c->stream));
      VP_HIP(hipStreamSynchronize(c->stream));
      h_now = h_copy.data();
    }
    for (uint32_t i = 1; i < n; i++)
      if (h_now[i] < h_now[i - 1]) return VP_ENOTSUP;
    t_first = h_now[0];
    t_last = h_now[n - 1];
  } else {
    if (b->now_step < 0) return VP_ENOTSUP;
    t_first = b->now0;
    t_last = b->now0 + (int64_t)(n - 1) * b->now_step;
  }
  if (t_first < 0 || t_first < c->last_now) return VP_ENOTSUP;
  const NowSpec now{b->now, b->now0, b->now_step};
  auto at = [&](uint32_t p) { return b->now ? h_now[p] : now.at(p); };

  float ms = 0.f;
  int launches = 0;
  uint32_t a0 = 0;
  const uint32_t ne = std::min(n, exp_end);  // packets that may expire
  // The first-sighting cut (FlowTable::fs_hint, vignat's unsorted new keys):
  // when most of the last batch's misses were repeats of flows it first saw
  // in its opening packets, this batch starts with a segment of that many
  // packets; its new flows are in the table when the rest is classified, so
  // their later packets are phase-A hits rather than misses to deduplicate
  // and rewrite. Segments are exact wherever they are cut (§3).
  const uint32_t fs = ntabs ? tabs[0].t->fs_hint : 0u;
  auto fs_cut = [&](uint32_t a, uint32_t e) {
    c->seg_fs = a == 0 && fs && fs < e && e - fs >= 64;
    return c->seg_fs ? fs : e;
  };
  while (a0 < n) {
    if (a0 >= ne) {  // the rest runs no expiry: one segment
      const uint32_t e = fs_cut(a0, n);
      uint32_t allocated = 0;
      c->fold_pending = false;
      VP_TRY(seg(c, b, now, a0, e, &ms, &launches, &allocated));
      if (e < n) {  // (the rest after the cut: its flows' stamps as below)
        if (allocated & 1u)
          tabs[0].t->ts_floor = std::min<uint64_t>(tabs[0].t->ts_floor, (uint64_t)at(a0));
        a0 = e;
        continue;
      }
      break;
    }
    const int64_t ta = at(a0);
    auto lim = [&](int i) { return std::min<uint64_t>(tabs[i].t->ts_floor, (uint64_t)ta); };
    auto safe = [&](uint32_t p) {
      for (int i = 0; i < ntabs; i++)
        if (tabs[i].cutoff(c, at(p)) > (int64_t)lim(i)) return false;
      return true;
    };
    for (int i = 0; i < ntabs; i++) {  // expiries due at packet a0, in order
      FlowTable &t = *tabs[i].t;
      const int64_t cut = tabs[i].cutoff(c, ta);
      if (cut <= (int64_t)lim(i)) continue;
      VP_TRY(tbl_expire(c, t, cut, nullptr));  // (and the exact floor after it)
    }
    uint32_t b1 = n;
    if (!safe(ne - 1)) {  // first unsafe packet (cutoffs are monotone in time)
      uint32_t lo = a0 + 1, hi = ne - 1;
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (safe(mid)) lo = mid + 1; else hi = mid;
      }
      b1 = lo;
    }
    b1 = fs_cut(a0, b1);
    uint32_t allocated = 0;
    c->fold_pending = false;
    VP_TRY(seg(c, b, now, a0, b1, &ms, &launches, &allocated));
    for (int i = 0; i < ntabs; i++)
      if (allocated & (1u << i))
        tabs[i].t->ts_floor = std::min<uint64_t>(tabs[i].t->ts_floor, (uint64_t)ta);
    a0 = b1;
  }
  c->seg_fs = false;
  // Results are complete once every segment's work is; a trailing timestamp
  // fold alone may keep running (ordered before any later call on the
  // stream, and before the caller's stream through vp_process_device).
  if (!c->fold_pending) VP_HIP(stream_wait(c->stream));
  c->fold_pending = false;
  c->seq += n;
  c->last_now = t_last;
  c->last_ms = ms;
  c->last_launches = launches;
  return 0;
}

// ------------------------------------------------------ multi-GPU batch --
// Every rank holds the same dictionary and allocator (new keys are
// all-gathered, vp_nat.hip) and partial stamps: ts_r[i] / tseq_r[i] describe
// rank r's own last touch of i (or its allocation), so the true stamp is the
// maximum over ranks. Because ts_r <= ts, max_r(floor_r) is still a lower
// bound of the live minimum and the no-expiry test of run_batch stays exact.
// Where an expiry may happen the stamps are merged (all-reduce MAX of ts and
// tseq) and the single-GPU expiry then runs identically on every rank.

static int sync_ts(vp_ctx *c, FlowTable &t) {
  VP_TRY(c->comm->allreduce_max_u64_dev(c, t.ts, t.cap));
  VP_TRY(c->comm->allreduce_max_u64_dev(c, t.tseq, t.cap));
  return 0;
}

int sync_tables(vp_ctx *c) {
  VP_TRY(sync_ts(c, c->ft));
  if (c->kind == KIND_LB) VP_TRY(sync_ts(c, c->ft2));
  VP_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

struct RankInfo {
  int64_t bad, n, t_first, t_last;
  uint64_t floor[2];
  uint64_t maxsend;  // owner mode: this rank's largest per-owner key count last seen
};

// New keys of a segment, exchanged so that every rank allocates the same
// union in global packet order (ranks' slices are consecutive, each sorted).
struct NewRec {
  uint32_t k[4];
  uint32_t hash, gp;
  int64_t now;
};
struct RankSlices {
  uint32_t n, maxn;
  uint32_t cnt[kMaxRanks], pre[kMaxRanks];
};

// The segment's new-key count of every rank. Taken from the counters the
// fold published (tbl_fold_read_ctl) unless some rank ran reprobes after it
// (they may find new keys): all ranks see the same gathered words, so they
// agree on which way to go.
int union_sizes(vp_ctx *c, uint32_t nl, uint32_t *total, uint32_t *mine_off) {
  Comm &m = *c->comm;
  Workspace &w = c->ws;
  c->rank_cnt.assign(m.n, 0);
  bool pub = w.gath_ok;
  for (int r = 0; pub && r < m.n; r++) pub = w.h_gath[kPubGath * r + 3] == 0;  // reprobes
  if (pub) {
    for (int r = 0; r < m.n; r++) c->rank_cnt[r] = w.h_gath[kPubGath * r];
    // A broken invariant on this rank alone must not leave the other ranks
    // waiting in this segment's collectives: the segment goes on with the
    // gathered counts (all ranks agree on them), this call returns VP_ESTATE
    // at its end, and every rank returns it from the next call on (the
    // RankInfo gather carries the flag, run_batch_sharded).
    if (c->rank_cnt[m.r] != nl && !c->estate_pending) {
      (void)state_fail("published miss count %u != %u", c->rank_cnt[m.r], nl);
      c->estate_pending = true;
    }
  } else {
    VP_TRY(m.allgather_host(c, &nl, c->rank_cnt.data(), sizeof nl));
  }
  uint32_t t = 0;
  *mine_off = 0;
  for (int r = 0; r < m.n; r++) {
    if (r == m.r) *mine_off = t;
    t += c->rank_cnt[r];
  }
  *total = t;
  return 0;
}

__global__ void rec_pack(const uint32_t *mkey, const uint32_t *mhash,
                         const uint32_t *pos, uint32_t n, uint32_t off, NowSpec now,
                         NewRec *out) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    NewRec r;
    for (int k = 0; k < 4; k++) r.k[k] = mkey[4 * (size_t)j + k];
    r.hash = mhash[j];
    r.gp = off + pos[j];
    r.now = now.at(pos[j]);
    out[j] = r;
  }
}

__global__ void rec_unpack(const NewRec *in, RankSlices rs, uint32_t *mkey,
                           uint32_t *mhash, uint32_t *upos, int64_t *unow) {
  const uint64_t total = (uint64_t)rs.n * rs.maxn;
  for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < total;
       x += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = (uint32_t)(x / rs.maxn), j = (uint32_t)(x % rs.maxn);
    if (j >= rs.cnt[r]) continue;
    const NewRec v = in[x];
    const uint32_t u = rs.pre[r] + j;
    for (int k = 0; k < 4; k++) mkey[4 * (size_t)u + k] = v.k[k];
    mhash[u] = v.hash;
    upos[u] = v.gp;
    unow[u] = v.now;
  }
}

static int grow(void **p, size_t *have, size_t bytes) {
  if (bytes <= *have) return 0;
  if (*p) hipFree(*p);
  *p = nullptr;
  *have = 0;
  VP_HIP(hipMalloc(p, bytes));
  *have = bytes;
  return 0;
}

int union_exchange(vp_ctx *c, uint32_t nl, const NowSpec &now) {
  Comm &m = *c->comm;
  Workspace &w = c->ws;
  RankSlices rs{};
  rs.n = (uint32_t)m.n;
  uint32_t pre = 0;
  for (int r = 0; r < m.n; r++) {
    rs.cnt[r] = c->rank_cnt[r];
    rs.pre[r] = pre;
    pre += c->rank_cnt[r];
    rs.maxn = std::max(rs.maxn, c->rank_cnt[r]);
  }
  const size_t bytes = sizeof(NewRec) * (size_t)rs.maxn;
  nl = std::min(nl, c->rank_cnt[m.r]);  // (differs only after a broken invariant)
  VP_HIP(hipStreamSynchronize(c->stream));  // buffers may be reallocated
  VP_TRY(grow(&w.sbuf, &w.sbuf_bytes, bytes));
  VP_TRY(grow(&w.rbuf, &w.rbuf_bytes, bytes * m.n));
  if (nl)
    rec_pack<<<grid_for(nl), 256, 0, c->stream>>>(w.mkey, w.mhash, w.miss_sorted,
                                                  nl, c->off, now,
                                                  static_cast<NewRec *>(w.sbuf));
  VP_HIP(hipGetLastError());
  VP_TRY(m.allgather_dev(c, w.sbuf, w.rbuf, bytes));
  rec_unpack<<<grid_for((uint64_t)rs.n * rs.maxn), 256, 0, c->stream>>>(
      static_cast<const NewRec *>(w.rbuf), rs, w.mkey, w.mhash, w.skey, w.unow);
  VP_HIP(hipGetLastError());
  return 0;
}

// Allocation stamps on every rank (the allocating packet's rank would also
// log it): ts = its time, tseq = its global sequence.
__global__ void union_stamp(const uint32_t *first, const uint32_t *assign,
                            const uint32_t *upos, const int64_t *unow, uint32_t n,
                            uint64_t seq, uint64_t *ts, uint64_t *tseq) {
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < n;
       u += gridDim.x * blockDim.x) {
    if (!first[u] || assign[u] == kNone) continue;
    ts[assign[u]] = (uint64_t)unow[u];
    tseq[assign[u]] = seq + upos[u];
  }
}

// VIGPATH_STALL="rank:ms:call" (watchdog rehearsals, bench.py): rank `rank`
// sleeps `ms` at the start of its `call`-th multi-GPU batch (0-based), while
// its peers wait for it inside the batch's first collective.
static void maybe_stall(int rank) {
  static int calls = 0;
  static const struct S { int r, ms, call; } st = [] {
    S v{-1, 0, 0};
    if (const char *e = getenv("VIGPATH_STALL")) sscanf(e, "%d:%d:%d", &v.r, &v.ms, &v.call);
    return v;
  }();
  if (st.r == rank && calls++ == st.call) {
    fprintf(stderr, "vigpath: rank %d stalls %d ms in batch %d (VIGPATH_STALL)\n", rank, st.ms,
            st.call);
    usleep((useconds_t)st.ms * 1000u);
  }
}

static int run_batch_sharded(vp_ctx *c, const vp_dev_batch *b,
                             ExpiringTable *tabs, int ntabs, SegmentFn seg) {
  Comm &m = *c->comm;
  maybe_stall(m.r);
  const uint32_t n = b->n;
  c->last_ms = 0.f;
  c->last_launches = 0;
  for (float &x : c->stage_ms) x = 0.f;
  c->stage_n = 0;
  // 1. every rank's slice size, time range and floors (one small gather);
  //    errors are decided from the gathered data so all ranks agree
  RankInfo me{};
  me.n = n;
  if (n && (b->slot < 64 || (b->slot & 15) || !b->frames ||
            ((uintptr_t)b->frames & 15) || !b->len || !b->in_dev || !b->out_dev))
    me.bad = 1;
  std::vector<int64_t> h_now;
  if (!me.bad && n) {
    if (b->now) {
      h_now.resize(n);
      VP_HIP(hipMemcpyAsync(h_now.data(), b->now, sizeof(int64_t) * (size_t)n,
                            hipMemcpyDeviceToHost, c->stream));
      VP_HIP(hipStreamSynchronize(c->stream));
      for (uint32_t i = 1; i < n; i++)
        if (h_now[i] < h_now[i - 1]) me.bad = 2;
      me.t_first = h_now[0];
      me.t_last = h_now[n - 1];
    } else {
      if (b->now_step < 0) me.bad = 2;
      me.t_first = b->now0;
      me.t_last = b->now0 + (int64_t)(n - 1) * b->now_step;
    }
  }
  if (c->estate_pending) me.bad |= 4;  // an earlier call broke an invariant
  for (int i = 0; i < ntabs; i++) me.floor[i] = tabs[i].t->ts_floor;
  me.maxsend = c->own_maxsend;
  std::vector<RankInfo> all(m.n);
  VP_TRY(m.allgather_host(c, &me, all.data(), sizeof me));
  {  // owner mode: the padded exchange's keys per peer for this batch, the
     // same on every rank: the largest per-owner count any
     // rank last sent (its whole slice before it knows) + 1/8 + 256, at most
     // the largest slice; a segment that exceeds it takes the exact exchange
    // (a rank that has sent nothing yet: its slice's uniform share per owner;
    // a skewed first batch takes the exact exchange once, and no rank pins
    // ranks x slice entries of exchange buffers)
    // (the chunked pipeline, vp_nat.hip: keys per peer and chunk, so a rank's
    // part counts at most one chunk)
    const uint64_t pk = c->shard_mode == VP_SHARD_OWNER && b->slot == 64
                            ? nat_own_chunk_packets() : 0;
    auto part = [&](uint64_t x) { return pk ? std::min<uint64_t>(x, pk) : x; };
    uint64_t maxs = 0, maxn = 0;
    for (int r = 0; r < m.n; r++) {
      maxn = std::max<uint64_t>(maxn, part((uint64_t)all[r].n));
      maxs = std::max<uint64_t>(maxs, all[r].maxsend
                                          ? all[r].maxsend
                                          : (part((uint64_t)all[r].n) + m.n - 1) / m.n);
    }
    uint64_t C = (maxs + maxs / 8 + 256 + 255) & ~255ull;
    if (const char *e = getenv("VIGPATH_OWN_CAP")) C = strtoull(e, nullptr, 10);  // tests
    c->own_cap = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(C, 1), std::max<uint64_t>(maxn, 1));
  }
  int bad = 0;
  uint64_t G = 0;
  uint32_t off = 0;
  int64_t prev = c->last_now, t_first_g = 0, t_last_g = 0;
  bool seen = false;
  c->rank_n.assign(m.n, 0);
  for (int r = 0; r < m.n; r++) {
    bad |= (int)all[r].bad;
    c->rank_n[r] = (uint32_t)all[r].n;
    if (r < m.r) off += (uint32_t)all[r].n;
    if (all[r].n) {  // global order: rank 0's packets first
      if (all[r].t_first < 0 || all[r].t_first < prev) bad |= 2;
      if (!seen) t_first_g = all[r].t_first;
      seen = true;
      prev = t_last_g = all[r].t_last;
    }
    G += (uint64_t)all[r].n;
  }
  if (bad & 4) return c->estate_pending ? VP_ESTATE
                                         : state_fail("another rank broke an invariant");
  if (bad & 1) return VP_EINVAL;
  if (bad & 2) return VP_ENOTSUP;
  if (G == 0) return 0;
  if (G > 0xFFFFFFF0ull) return VP_EINVAL;
  c->off = off;
  VP_TRY(ws_reserve(c, (uint32_t)G));  // the union of new keys can reach G
  uint64_t F[2] = {0, 0};
  for (int i = 0; i < ntabs; i++)
    for (int r = 0; r < m.n; r++) F[i] = std::max(F[i], all[r].floor[i]);

  const NowSpec now{b->now, b->now0, b->now_step};
  auto at = [&](uint32_t p) { return b->now ? h_now[p] : now.at(p); };
  float ms = 0.f;
  int launches = 0;
  uint64_t A = 0;
  int64_t tA = t_first_g;
  while (A < G) {
    // 2. expiries due at global packet A (identical decisions everywhere)
    for (int i = 0; i < ntabs; i++) {
      FlowTable &t = *tabs[i].t;
      const int64_t cut = tabs[i].cutoff(c, tA);
      if (cut <= (int64_t)std::min<uint64_t>(F[i], (uint64_t)tA)) continue;
      VP_TRY(sync_ts(c, t));
      VP_TRY(tbl_expire(c, t, cut, nullptr));  // (and the exact floor after it)
      F[i] = t.ts_floor;
    }
    auto safe_t = [&](int64_t tp) {
      for (int i = 0; i < ntabs; i++)
        if (tabs[i].cutoff(c, tp) > (int64_t)std::min<uint64_t>(F[i], (uint64_t)tA))
          return false;
      return true;
    };
    // 3. the next cut: the first unsafe packet over all ranks
    uint64_t B1 = G;
    int64_t tB1 = 0;
    if (!safe_t(t_last_g)) {
      int64_t mine[2] = {(int64_t)G, 0};
      const uint64_t lo_g = std::max<uint64_t>(A + 1, off), hi_g = (uint64_t)off + n;
      if (lo_g < hi_g && !safe_t(at(n - 1))) {
        uint32_t lo = (uint32_t)(lo_g - off), hi = n - 1;
        while (lo < hi) {
          const uint32_t mid = lo + (hi - lo) / 2;
          if (safe_t(at(mid))) lo = mid + 1; else hi = mid;
        }
        mine[0] = (int64_t)off + lo;
        mine[1] = at(lo);
      }
      std::vector<int64_t> cuts(2 * (size_t)m.n);
      VP_TRY(m.allgather_host(c, mine, cuts.data(), sizeof mine));
      for (int r = 0; r < m.n; r++)
        if ((uint64_t)cuts[2 * r] < B1) {
          B1 = (uint64_t)cuts[2 * r];
          tB1 = cuts[2 * r + 1];
        }
    }
    // 4. this rank's part of [A, B1); collectives inside run on every rank
    c->seg_g0 = A;
    c->seg_g1 = B1;
    const uint32_t lp0 = (uint32_t)(std::min<uint64_t>(std::max<uint64_t>(A, off), off + (uint64_t)n) - off);
    const uint32_t lp1 = (uint32_t)(std::min<uint64_t>(std::max<uint64_t>(B1, off), off + (uint64_t)n) - off);
    uint32_t allocated = 0;
    c->fold_pending = false;
    VP_TRY(seg(c, b, now, lp0, lp1, &ms, &launches, &allocated));
    for (int i = 0; i < ntabs; i++)
      if (allocated & (1u << i)) {
        F[i] = std::min<uint64_t>(F[i], (uint64_t)tA);
        tabs[i].t->ts_floor = std::min<uint64_t>(tabs[i].t->ts_floor, (uint64_t)tA);
      }
    A = B1;
    tA = tB1;
  }
  // as in run_batch: a trailing timestamp fold alone may keep running; the
  // next call's collectives queue behind it on the same stream
  if (!c->fold_pending) VP_HIP(hipStreamSynchronize(c->stream));
  c->fold_pending = false;
  if (c->estate_pending) return VP_ESTATE;  // (union_sizes; the text is recorded)
  c->seq += G;
  c->last_now = t_last_g;
  c->last_ms = ms;
  c->last_launches = launches;
  return 0;
}

// ------------------------------------------------------------------ dump --

__global__ void dump_k(TableDev t, uint8_t *alloc, int64_t *ts, uint32_t *keys) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < t.cap;
       i += gridDim.x * blockDim.x) {
    const bool live = t.slot_of[i] != kNone;
    alloc[i] = live;
    ts[i] = live ? (int64_t)t.ts[i] : 0;
    const uint4 k = live ? tbl_key_of(t, i) : make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4 *>(keys)[i] = k;
  }
}

int tbl_dump(vp_ctx *c, FlowTable &t, uint8_t *alloc, int64_t *ts,
             uint32_t *keys) {
  const uint32_t cap = t.cap;
  uint8_t *d_alloc = nullptr;
  int64_t *d_ts = nullptr;
  uint32_t *d_keys = nullptr;
  VP_TRY(dalloc(&d_alloc, cap));
  VP_TRY(dalloc(&d_ts, cap));
  VP_TRY(dalloc(&d_keys, 4ull * cap));
  dump_k<<<grid_for(cap), 256, 0, c->stream>>>(tbl_dev(t), d_alloc, d_ts, d_keys);
  VP_HIP(hipMemcpyAsync(alloc, d_alloc, cap, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipMemcpyAsync(ts, d_ts, 8ull * cap, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipMemcpyAsync(keys, d_keys, 16ull * cap, hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(hipStreamSynchronize(c->stream));
  hipFree(d_alloc);
  hipFree(d_ts);
  hipFree(d_keys);
  return 0;
}

}  // namespace vp
