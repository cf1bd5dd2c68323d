// vignat on MI355X: batch classification + flow-state update + rewrite.
//
// Reference behaviour (paths relative to the reference repository):
//   nf_process            vignat/nat_main.c:22-109
//   flow manager          vignat/nat_flowmanager.c:20-94
//   expiry                libvig/verified/expirator.c:110-218 +
//                         double-chain.c:772-826 (strict ts < cutoff)
//   index allocation      double-chain-impl.c:1197-1415 (free-list head),
//                         1839-2078 (freed indices pushed to the front)
// Sequential semantics are reproduced exactly for a whole batch; DESIGN.md
// §3 gives the argument. In short, a batch is cut into segments inside which
// no flow can expire; within a segment
//   phase A  every packet is parsed and hashed; LAN packets whose flow exists
//            at segment start are rewritten at once; WAN packets whose index
//            is allocated at segment start likewise; the rest are queued;
//   phase B  queued LAN misses are ordered, de-duplicated by key (earliest
//            packet wins), ranked, and given dchain indices in packet order;
//            then rewritten;
//   phase C  queued WAN packets see an index as allocated iff it was
//            allocated before them in packet order;
// rejuvenation is an atomic max of the packet time (times are monotone), and
// expiry between segments frees flows in LRU order onto a LIFO stack.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "vp_internal.h"

namespace vp {

// FlowId (vignat/flow.h:3-10) hashed as 6 CRC steps; the non-zero byte
// positions of that 24-byte CRC message:
//   src_port 0,1  dst_port 4,5  src_ip 8-11  dst_ip 12-15  device 16,17
//   protocol 20
static const int kFlowIdPos[15] = {0, 1, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15,
                                   16, 17, 20};
constexpr int kFlowIdMsg = 24;

__device__ __forceinline__ uint32_t flowid_hash(const uint32_t *T, uint32_t sp,
                                                uint32_t dp, uint32_t sip,
                                                uint32_t dip, uint32_t dev,
                                                uint32_t proto) {
  return T[0 * 256 + (sp & 0xFF)] ^ T[1 * 256 + ((sp >> 8) & 0xFF)] ^
         T[2 * 256 + (dp & 0xFF)] ^ T[3 * 256 + ((dp >> 8) & 0xFF)] ^
         T[4 * 256 + (sip & 0xFF)] ^ T[5 * 256 + ((sip >> 8) & 0xFF)] ^
         T[6 * 256 + ((sip >> 16) & 0xFF)] ^ T[7 * 256 + (sip >> 24)] ^
         T[8 * 256 + (dip & 0xFF)] ^ T[9 * 256 + ((dip >> 8) & 0xFF)] ^
         T[10 * 256 + ((dip >> 16) & 0xFF)] ^ T[11 * 256 + (dip >> 24)] ^
         T[12 * 256 + (dev & 0xFF)] ^ T[13 * 256 + ((dev >> 8) & 0xFF)] ^
         T[14 * 256 + (proto & 0xFF)];
}

struct NatArgs {
  uint8_t *frames;
  const uint16_t *len;
  const uint16_t *in_dev;
  const int64_t *now;
  uint16_t *out;
  int64_t now0, now_step;
  uint64_t seq_base;
  uint32_t slot, p0, p1;
  FlowSlot *slots;
  uint32_t tmask, cap;
  uint32_t *slot_of;
  uint64_t *birth;
  uint64_t *tseq;
  uint32_t *stack;
  Ctl *ctl;
  const uint32_t *crc_tab;
  const uint32_t *macw;
  uint32_t wan_macw0, wan_macw1, wan_macw2;
  uint32_t *miss;
  uint32_t *defer;
  uint32_t ext_ip;
  uint16_t wan, start_port, n_dev;
  int ties;
};

__device__ __forceinline__ int64_t now_at(const NatArgs &a, uint32_t p) {
  return a.now ? a.now[p] : a.now0 + (int64_t)p * a.now_step;
}

__device__ __forceinline__ void rejuvenate(const NatArgs &a, uint32_t s,
                                           uint32_t idx, int64_t now,
                                           uint64_t q) {
  // dchain_rejuvenate_index: new stamp = this packet's time; with monotone
  // time the last toucher in packet order has the largest stamp.
  atomicMax((unsigned long long *)&a.slots[s].ts, (unsigned long long)now);
  if (a.ties) atomicMax((unsigned long long *)&a.tseq[idx], (unsigned long long)q);
}

// map_get (find_key, map-impl-pow2.c:629-732) on the device table. Returns
// the dchain index or kNone; *slot_out = the slot.
__device__ __forceinline__ uint32_t probe(const NatArgs &a, uint32_t h,
                                          const uint32_t key[4],
                                          uint32_t *slot_out) {
  uint32_t s = h & a.tmask;
  for (uint32_t i = 0; i <= a.tmask; i++) {
    const uint4 *sp4 = reinterpret_cast<const uint4 *>(a.slots + s);
    uint4 k = sp4[0];
    uint4 m = sp4[1];
    if (m.y == kEmpty) return kNone;
    if (m.y != kTomb && m.x == h && k.x == key[0] && k.y == key[1] &&
        k.z == key[2] && k.w == key[3]) {
      *slot_out = s;
      return m.y;
    }
    s = (s + 1) & a.tmask;
  }
  return kNone;
}

__device__ __forceinline__ void macs_for(const NatArgs &a, uint32_t dst,
                                         uint32_t mw[3]) {
  if (dst == a.wan) {
    mw[0] = a.wan_macw0;
    mw[1] = a.wan_macw1;
    mw[2] = a.wan_macw2;
  } else if (dst < a.n_dev) {
    mw[0] = a.macw[3 * dst];
    mw[1] = a.macw[3 * dst + 1];
    mw[2] = a.macw[3 * dst + 2];
  } else {
    mw[0] = mw[1] = mw[2] = 0;
  }
}

// Generic (byte-addressed) form of nat_main.c:22-109 for frames the register
// fast path does not cover (IP options, long frames). `stage` 0 = phase A
// (may queue), 1 = phase B/C completion with a known decision.
__device__ void nat_generic_a(const NatArgs &a, const uint32_t *T, uint32_t p,
                              uint64_t q, int64_t now, uint32_t in,
                              uint32_t len) {
  GFrame f{a.frames + (size_t)p * a.slot, a.slot};
  L34 h = parse_l34(f, len);
  if (!h.ok) {
    a.out[p] = (uint16_t)in;
    return;
  }
  uint32_t proto = f.r8(h.ip + 9);
  uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
  uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
  uint32_t dst;
  if (in == a.wan) {
    int idx = (int)dp - (int)a.start_port;
    if (idx < 0 || idx >= (int)a.cap) {  // reference UB range: not allocated
      a.out[p] = (uint16_t)in;
      return;
    }
    uint32_t s = a.slot_of[idx];
    if (s == kNone) {
      a.defer[wave_append(&a.ctl->defer_count, true)] = p;
      return;
    }
    const FlowSlot &fs = a.slots[s];
    uint32_t k0 = fs.k[0], k1 = fs.k[1], k2 = fs.k[2], k3 = fs.k[3];
    rejuvenate(a, s, (uint32_t)idx, now, q);
    if ((k2 != sip) | ((k0 >> 16) != sp) | (((k3 >> 16) & 0xFF) != proto)) {
      a.out[p] = (uint16_t)in;
      return;
    }
    f.w32(h.ip + 16, k1);
    f.w16(h.l4 + 2, (uint16_t)(k0 & 0xFFFF));
    dst = k3 & 0xFFFF;
  } else {
    uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
    uint32_t hh = flowid_hash(T, sp, dp, sip, dip, in, proto);
    uint32_t s = 0;
    uint32_t idx = probe(a, hh, key, &s);
    if (idx == kNone) {
      a.miss[wave_append(&a.ctl->miss_count, true)] = p;
      return;
    }
    rejuvenate(a, s, idx, now, q);
    f.w32(h.ip + 12, a.ext_ip);
    f.w16(h.l4, (uint16_t)(a.start_port + idx));
    dst = a.wan;
  }
  set_checksums(f, h.ip, h.l4);
  uint32_t mw[3];
  macs_for(a, dst, mw);
  set_macs(f, mw);
  a.out[p] = (uint16_t)dst;
}

// Phase A. One packet per lane, grid-stride; 64-byte slots are loaded with
// four 16-byte loads per lane and processed in registers.
__global__ __launch_bounds__(256) void nat_classify(NatArgs a) {
  __shared__ uint32_t T[15 * 256];
  for (uint32_t i = threadIdx.x; i < 15 * 256; i += blockDim.x)
    T[i] = a.crc_tab[i];
  __syncthreads();

  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += stride) {
    const uint64_t q = a.seq_base + p;
    const int64_t now = now_at(a, p);
    const uint32_t in = a.in_dev[p];
    const uint32_t len = a.len[p];
    uint4 *fp = reinterpret_cast<uint4 *>(a.frames + (size_t)p * a.slot);
    RFrame f;
    {
      uint4 c0 = fp[0], c1 = fp[1], c2 = fp[2], c3 = fp[3];
      f.w[0] = c0.x; f.w[1] = c0.y; f.w[2] = c0.z; f.w[3] = c0.w;
      f.w[4] = c1.x; f.w[5] = c1.y; f.w[6] = c1.z; f.w[7] = c1.w;
      f.w[8] = c2.x; f.w[9] = c2.y; f.w[10] = c2.z; f.w[11] = c2.w;
      f.w[12] = c3.x; f.w[13] = c3.y; f.w[14] = c3.z; f.w[15] = c3.w;
    }
    const uint32_t et = f.w[3] & 0xFFFF;
    const uint32_t ihl = (f.w[3] >> 16) & 0x0F;
    const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
    if (!(et == 0x0008 && ihl == 5 && tl <= 50)) {
      nat_generic_a(a, T, p, q, now, in, len);
      continue;
    }
    // nf_then_get_rte_ipv4_header / nf_then_get_tcpudp_header, IHL = 5
    const uint16_t unread = (uint16_t)(len - 14);
    const uint32_t proto = f.w[5] >> 24;
    const bool ok = (unread >= 20) & (unread >= tl) &
                    ((proto == 6) | (proto == 17)) &
                    ((uint32_t)(len - 34) >= 4u);
    if (!ok) {
      a.out[p] = (uint16_t)in;
      continue;
    }
    const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
    const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
    uint32_t dst;
    uint32_t mw[3];
    if (in == a.wan) {
      // flow_manager_get_external (nat_flowmanager.c:78-94)
      const int idx = (int)dp - (int)a.start_port;
      if (idx < 0 || idx >= (int)a.cap) {
        a.out[p] = (uint16_t)in;
        continue;
      }
      const uint32_t s = a.slot_of[idx];
      if (s == kNone) {  // maybe allocated earlier in this segment: phase C
        a.defer[wave_append(&a.ctl->defer_count, true)] = p;
        continue;
      }
      const uint4 k = *reinterpret_cast<const uint4 *>(a.slots + s);
      rejuvenate(a, s, (uint32_t)idx, now, q);
      // anti-spoofing, nat_main.c:55-60
      if ((k.z != sip) | ((k.x >> 16) != sp) | (((k.w >> 16) & 0xFF) != proto)) {
        a.out[p] = (uint16_t)in;
        continue;
      }
      f.set32at2(30, k.y);       // dst_addr = flow.src_ip
      f.set16(36, k.x & 0xFFFF);  // dst_port = flow.src_port
      dst = k.w & 0xFFFF;         // flow.internal_device
      macs_for(a, dst, mw);
    } else {
      // flow_manager_get_internal (nat_flowmanager.c:67-76)
      const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
      const uint32_t hh = flowid_hash(T, sp, dp, sip, dip, in, proto);
      uint32_t s = 0;
      const uint32_t idx = probe(a, hh, key, &s);
      if (idx == kNone) {  // new flow or not yet visible: phase B
        a.miss[wave_append(&a.ctl->miss_count, true)] = p;
        continue;
      }
      rejuvenate(a, s, idx, now, q);
      f.set32at2(26, a.ext_ip);                       // src_addr = external_addr
      f.set16(34, (uint16_t)(a.start_port + idx));    // src_port = ext port
      dst = a.wan;
      mw[0] = a.wan_macw0;
      mw[1] = a.wan_macw1;
      mw[2] = a.wan_macw2;
    }
    fast_checksums(f, proto, tl);
    f.w[0] = mw[0];
    f.w[1] = mw[1];
    f.w[2] = mw[2];
    fp[0] = make_uint4(f.w[0], f.w[1], f.w[2], f.w[3]);
    fp[1] = make_uint4(f.w[4], f.w[5], f.w[6], f.w[7]);
    fp[2] = make_uint4(f.w[8], f.w[9], f.w[10], f.w[11]);
    if (proto == 6) fp[3] = make_uint4(f.w[12], f.w[13], f.w[14], f.w[15]);
    a.out[p] = (uint16_t)dst;
  }
}

// ------------------------------------------------------------- phase B --

struct MissArgs {
  NatArgs a;
  const uint32_t *list;  // miss positions, ascending packet order
  uint32_t n;
  uint32_t *mkey, *mhash, *first, *rank, *rep, *assign, *scratch;
  uint32_t smask;
};

// Keys and hashes of the queued misses (frames still unmodified).
__global__ void nat_miss_keys(MissArgs m) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = m.list[j];
    GFrame f{m.a.frames + (size_t)p * m.a.slot, m.a.slot};
    L34 h = parse_l34(f, m.a.len[p]);
    uint32_t proto = f.r8(h.ip + 9), in = m.a.in_dev[p];
    uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
    uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
    uint32_t *k = m.mkey + 4 * (size_t)j;
    k[0] = sp | (dp << 16);
    k[1] = sip;
    k[2] = dip;
    k[3] = in | (proto << 16);
    m.mhash[j] = flowid_hash(m.a.crc_tab, sp, dp, sip, dip, in, proto);
  }
}

// In-batch de-duplication: one scratch slot per distinct key holding the
// smallest miss ordinal j (= earliest packet) with that key.
__global__ void nat_miss_dedup(MissArgs m) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    const uint32_t *kj = m.mkey + 4 * (size_t)j;
    uint32_t s = m.mhash[j] & m.smask;
    for (;;) {
      uint32_t old = atomicCAS(&m.scratch[s], kEmpty, j);
      if (old == kEmpty) break;
      const uint32_t *ko = m.mkey + 4 * (size_t)old;
      if (m.mhash[old] == m.mhash[j] && key_eq(ko, kj)) {
        atomicMin(&m.scratch[s], j);
        break;
      }
      s = (s + 1) & m.smask;
    }
    m.rep[j] = s;
  }
}

__global__ void nat_miss_first(MissArgs m) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x)
    m.first[j] = m.scratch[m.rep[j]] == j ? 1u : 0u;
}


// dchain_allocate_new_index for every first sighting, in packet order: rank
// r takes the r-th entry of the free list (LIFO stack of freed indices, then
// never-used indices in order); map_put of its key into the device table.
__global__ void nat_miss_alloc(MissArgs m) {
  const NatArgs &a = m.a;
  const uint32_t stack_top = a.ctl->stack_top;
  const uint32_t fresh = a.ctl->fresh_next;
  const uint32_t free_total = stack_top + (a.cap - fresh);
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    if (!m.first[j]) continue;
    const uint32_t r = m.rank[j];
    if (r >= free_total) {  // table full: drop (nat_main.c:87-91)
      m.assign[j] = kNone;
      continue;
    }
    const uint32_t idx =
        r < stack_top ? a.stack[stack_top - 1 - r] : fresh + (r - stack_top);
    const uint32_t p = m.list[j];
    const uint64_t q = a.seq_base + p;
    const int64_t now = now_at(a, p);
    const uint32_t h = m.mhash[j];
    uint32_t s = h & a.tmask;
    for (;;) {
      uint32_t cur = __hip_atomic_load(&a.slots[s].index, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
      if (cur == kEmpty || cur == kTomb) {
        if (atomicCAS(&a.slots[s].index, cur, idx) == cur) {
          if (cur == kTomb) atomicAdd(&a.ctl->tomb_reused, 1u);
          break;
        }
        continue;  // lost the race for this slot; look at it again
      }
      s = (s + 1) & a.tmask;
    }
    FlowSlot &fs = a.slots[s];
    const uint32_t *k = m.mkey + 4 * (size_t)j;
    fs.k[0] = k[0];
    fs.k[1] = k[1];
    fs.k[2] = k[2];
    fs.k[3] = k[3];
    fs.hash = h;
    fs.ts = (uint64_t)now;
    a.slot_of[idx] = s;
    a.birth[idx] = q;
    a.tseq[idx] = q;
    m.assign[j] = idx;
  }
}

// Free-list bookkeeping after the allocations (one thread).
__global__ void nat_miss_commit(MissArgs m) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Ctl *c = m.a.ctl;
  const uint32_t K = m.rank[m.n - 1] + m.first[m.n - 1];
  const uint32_t free_total = c->stack_top + (m.a.cap - c->fresh_next);
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

// LAN rewrite for a packet whose flow index is known (generic byte path).
__device__ void nat_write_lan(const NatArgs &a, uint32_t p, uint32_t idx) {
  GFrame f{a.frames + (size_t)p * a.slot, a.slot};
  L34 h = parse_l34(f, a.len[p]);
  f.w32(h.ip + 12, a.ext_ip);
  f.w16(h.l4, (uint16_t)(a.start_port + idx));
  set_checksums(f, h.ip, h.l4);
  const uint32_t mw[3] = {a.wan_macw0, a.wan_macw1, a.wan_macw2};
  set_macs(f, mw);
  a.out[p] = a.wan;
}

__global__ void nat_miss_finish(MissArgs m) {
  const NatArgs &a = m.a;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m.n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = m.list[j];
    const uint32_t j0 = m.scratch[m.rep[j]];
    const uint32_t idx = m.assign[j0];
    if (idx == kNone) {
      a.out[p] = a.in_dev[p];
      continue;
    }
    if (j != j0) rejuvenate(a, a.slot_of[idx], idx, now_at(a, p), a.seq_base + p);
    nat_write_lan(a, p, idx);
  }
}

// ------------------------------------------------------------- phase C --
// WAN packets whose index was not allocated at segment start: allocated for
// this packet iff allocated earlier in packet order (birth < q).
__global__ void nat_defer_finish(NatArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint64_t q = a.seq_base + p;
    const uint32_t in = a.in_dev[p];
    GFrame f{a.frames + (size_t)p * a.slot, a.slot};
    L34 h = parse_l34(f, a.len[p]);
    const uint32_t proto = f.r8(h.ip + 9);
    const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
    const uint32_t sip = f.r32(h.ip + 12);
    const uint32_t idx = dp - a.start_port;  // range checked in phase A
    const uint32_t s = a.slot_of[idx];
    if (s == kNone || a.birth[idx] >= q) {
      a.out[p] = (uint16_t)in;
      continue;
    }
    const FlowSlot &fs = a.slots[s];
    const uint32_t k0 = fs.k[0], k1 = fs.k[1], k2 = fs.k[2], k3 = fs.k[3];
    rejuvenate(a, s, idx, now_at(a, p), q);
    if ((k2 != sip) | ((k0 >> 16) != sp) | (((k3 >> 16) & 0xFF) != proto)) {
      a.out[p] = (uint16_t)in;
      continue;
    }
    f.w32(h.ip + 16, k1);
    f.w16(h.l4 + 2, (uint16_t)(k0 & 0xFFFF));
    const uint32_t dst = k3 & 0xFFFF;
    set_checksums(f, h.ip, h.l4);
    uint32_t mw[3];
    macs_for(a, dst, mw);
    set_macs(f, mw);
    a.out[p] = (uint16_t)dst;
  }
}

// ---------------------------------------------------------------- expiry --

__global__ void table_min_ts(const FlowSlot *slots, uint32_t nslots, Ctl *ctl) {
  unsigned long long best = ~0ull;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += gridDim.x * blockDim.x) {
    const FlowSlot &fs = slots[s];
    if (fs.index < kTomb && fs.ts < best) best = fs.ts;
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long v = __shfl_xor(best, o);
    best = v < best ? v : best;
  }
  if (__lane_id() == 0 && best != ~0ull)
    atomicMin((unsigned long long *)&ctl->min_ts, best);
}

// Every live flow with ts < cutoff (the set expire_items_single_map frees:
// LRU order is ts order, so the loop stops exactly at the first ts >= cutoff).
__global__ void table_exp_collect(const FlowSlot *slots, uint32_t nslots,
                                  int64_t cutoff, const uint64_t *tseq,
                                  uint64_t *ekey, uint32_t *eidx, Ctl *ctl) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += gridDim.x * blockDim.x) {
    const FlowSlot &fs = slots[s];
    const bool take = fs.index < kTomb && (int64_t)fs.ts < cutoff;
    const uint32_t k = wave_append(&ctl->exp_count, take);
    if (take) {
      eidx[k] = fs.index;
      ekey[k] = tseq[fs.index];
    }
  }
}

__global__ void table_exp_gather_ts(const uint32_t *eidx, uint32_t n,
                                    const FlowSlot *slots,
                                    const uint32_t *slot_of, uint64_t *ekey) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x)
    ekey[j] = slots[slot_of[eidx[j]]].ts;
}

// Free in LRU order: the oldest is pushed first, so the youngest expired
// index ends on top of the stack (double-chain-impl.c:1968-1981), then the
// map entries are erased (tombstones).
__global__ void table_exp_apply(const uint32_t *eidx, uint32_t n,
                                uint32_t *stack, FlowSlot *slots,
                                uint32_t *slot_of, Ctl *ctl) {
  const uint32_t top = ctl->stack_top;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t idx = eidx[j];
    stack[top + j] = idx;
    slots[slot_of[idx]].index = kTomb;
    slot_of[idx] = kNone;
  }
}

__global__ void table_exp_commit(Ctl *ctl, uint32_t n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    ctl->stack_top += n;
    ctl->n_live -= n;
    ctl->n_tomb += n;
  }
}

// Rebuild (tombstone purge): copy live slots out, clear, re-insert.
__global__ void table_collect_live(const FlowSlot *slots, uint32_t nslots,
                                   FlowSlot *out, Ctl *ctl) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots;
       s += gridDim.x * blockDim.x) {
    const bool live = slots[s].index < kTomb;
    const uint32_t k = wave_append(&ctl->exp_count, live);
    if (live) out[k] = slots[s];
  }
}
__global__ void table_reinsert(const FlowSlot *in, uint32_t n, FlowSlot *slots,
                               uint32_t tmask, uint32_t *slot_of) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const FlowSlot v = in[j];
    uint32_t s = v.hash & tmask;
    while (atomicCAS(&slots[s].index, kEmpty, v.index) != kEmpty)
      s = (s + 1) & tmask;
    FlowSlot &d = slots[s];
    d.k[0] = v.k[0];
    d.k[1] = v.k[1];
    d.k[2] = v.k[2];
    d.k[3] = v.k[3];
    d.hash = v.hash;
    d.ts = v.ts;
    slot_of[v.index] = s;
  }
}

__global__ void table_dump(const FlowSlot *slots, const uint32_t *slot_of,
                           uint32_t cap, uint8_t *alloc, int64_t *ts,
                           uint32_t *keys) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += gridDim.x * blockDim.x) {
    const uint32_t s = slot_of[i];
    alloc[i] = s != kNone;
    ts[i] = s != kNone ? (int64_t)slots[s].ts : 0;
    for (int w = 0; w < 4; w++) keys[4 * i + w] = s != kNone ? slots[s].k[w] : 0;
  }
}

// =============================================================== host ==

static inline uint32_t grid_for(uint64_t n, uint32_t block = 256,
                                uint32_t max_blocks = 2048) {
  uint64_t g = (n + block - 1) / block;
  if (g == 0) g = 1;
  return (uint32_t)(g < max_blocks ? g : max_blocks);
}

static uint32_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return (uint32_t)p;
}

int ws_reserve(vp_ctx *c, uint32_t n);

// cutoff for expiry at time t: nat_flowmanager.c:57-65, where the u32
// expiration_time * 1000 wraps in 32-bit arithmetic.
static inline int64_t nat_cutoff(const vp_ctx *c, int64_t t) {
  const uint32_t e = c->nat.expiration_time * 1000u;
  return (int64_t)((uint64_t)t - e);
}

static int read_ctl(vp_ctx *c) {
  VP_HIP(hipMemcpyAsync(&c->h_ctl, c->ft.ctl, sizeof(Ctl), hipMemcpyDeviceToHost,
                        c->stream));
  VP_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

// Exact min ts over live flows -> c->ft.ts_floor.
static int nat_exact_floor(vp_ctx *c) {
  const uint64_t all = ~0ull;
  VP_HIP(hipMemcpyAsync(&c->ft.ctl->min_ts, &all, 8, hipMemcpyHostToDevice,
                        c->stream));
  const uint32_t ns = c->ft.tmask + 1;
  table_min_ts<<<grid_for(ns), 256, 0, c->stream>>>(c->ft.slots, ns, c->ft.ctl);
  VP_HIP(hipGetLastError());
  int rc = read_ctl(c);
  if (rc) return rc;
  c->ft.ts_floor = c->h_ctl.min_ts;
  return 0;
}

static int table_rebuild(vp_ctx *c) {
  FlowTable &t = c->ft;
  const uint32_t ns = t.tmask + 1;
  FlowSlot *tmp = nullptr;
  VP_HIP(hipMallocAsync((void **)&tmp, sizeof(FlowSlot) * (size_t)t.cap, c->stream));
  VP_HIP(hipMemsetAsync(&t.ctl->exp_count, 0, 4, c->stream));
  table_collect_live<<<grid_for(ns), 256, 0, c->stream>>>(t.slots, ns, tmp, t.ctl);
  int rc = read_ctl(c);
  if (rc) return rc;
  const uint32_t live = c->h_ctl.exp_count;
  VP_HIP(hipMemsetAsync(t.slots, 0xFF, sizeof(FlowSlot) * (size_t)ns, c->stream));
  if (live)
    table_reinsert<<<grid_for(live), 256, 0, c->stream>>>(tmp, live, t.slots,
                                                         t.tmask, t.slot_of);
  VP_HIP(hipMemsetAsync(&t.ctl->n_tomb, 0, 4, c->stream));
  VP_HIP(hipMemsetAsync(&t.ctl->exp_count, 0, 4, c->stream));
  VP_HIP(hipFreeAsync(tmp, c->stream));
  VP_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

// Expire every live flow with ts < cutoff, in LRU order (ts, then last-touch
// sequence for equal stamps).
static int nat_expire(vp_ctx *c, int64_t cutoff) {
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  const uint32_t ns = t.tmask + 1;
  VP_HIP(hipMemsetAsync(&t.ctl->exp_count, 0, 4, c->stream));
  table_exp_collect<<<grid_for(ns), 256, 0, c->stream>>>(
      t.slots, ns, cutoff, t.tseq, w.ekey, w.eidx, t.ctl);
  VP_HIP(hipGetLastError());
  int rc = read_ctl(c);
  if (rc) return rc;
  const uint32_t k = c->h_ctl.exp_count;
  if (k == 0) return 0;
  size_t need = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, need, w.ekey, w.ekey2, w.eidx,
                                     w.eidx2, (int)k, 0, 64, c->stream);
  if (need > w.cub_bytes) {
    if (w.cub_tmp) VP_HIP(hipFree(w.cub_tmp));
    VP_HIP(hipMalloc(&w.cub_tmp, need));
    w.cub_bytes = need;
  }
  // 1) by last-touch sequence, 2) stable by timestamp
  VP_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, w.cub_bytes, w.ekey, w.ekey2,
                                            w.eidx, w.eidx2, (int)k, 0, 64,
                                            c->stream));
  table_exp_gather_ts<<<grid_for(k), 256, 0, c->stream>>>(w.eidx2, k, t.slots,
                                                          t.slot_of, w.ekey);
  VP_HIP(hipcub::DeviceRadixSort::SortPairs(w.cub_tmp, w.cub_bytes, w.ekey, w.ekey2,
                                            w.eidx2, w.eidx, (int)k, 0, 64,
                                            c->stream));
  table_exp_apply<<<grid_for(k), 256, 0, c->stream>>>(w.eidx, k, t.stack,
                                                      t.slots, t.slot_of, t.ctl);
  table_exp_commit<<<1, 64, 0, c->stream>>>(t.ctl, k);
  VP_HIP(hipGetLastError());
  rc = read_ctl(c);
  if (rc) return rc;
  if ((uint64_t)c->h_ctl.n_tomb + c->h_ctl.n_live > (uint64_t)ns * 3 / 4)
    return table_rebuild(c);
  return 0;
}

struct BatchView {
  const vp_dev_batch *b;
  const int64_t *h_now;  // host copy of the times (array mode, slow path)
  int64_t at(uint32_t p) const {
    return b->now ? h_now[p] : b->now0 + (int64_t)p * b->now_step;
  }
};

static int nat_segment(vp_ctx *c, const vp_dev_batch *b, uint32_t p0,
                       uint32_t p1, bool ties, float *ms, int *launches) {
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  NatArgs a{};
  a.frames = b->frames;
  a.len = b->len;
  a.in_dev = b->in_dev;
  a.now = b->now;
  a.out = b->out_dev;
  a.now0 = b->now0;
  a.now_step = b->now_step;
  a.seq_base = c->seq;
  a.slot = b->slot;
  a.p0 = p0;
  a.p1 = p1;
  a.slots = t.slots;
  a.tmask = t.tmask;
  a.cap = t.cap;
  a.slot_of = t.slot_of;
  a.birth = t.birth;
  a.tseq = t.tseq;
  a.stack = t.stack;
  a.ctl = t.ctl;
  a.crc_tab = c->crc_tab;
  a.macw = c->macw;
  a.wan_macw0 = c->wan_macw[0];
  a.wan_macw1 = c->wan_macw[1];
  a.wan_macw2 = c->wan_macw[2];
  a.miss = w.miss;
  a.defer = w.defer;
  a.ext_ip = c->nat.external_addr;
  a.wan = c->nat.wan_device;
  a.start_port = c->nat.start_port;
  a.n_dev = c->nat.n_devices;
  a.ties = ties ? 1 : 0;

  VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 8, c->stream));  // + defer
  VP_HIP(hipEventRecord(c->ev0, c->stream));
  nat_classify<<<grid_for(p1 - p0), 256, 0, c->stream>>>(a);
  VP_HIP(hipGetLastError());
  VP_HIP(hipEventRecord(c->ev1, c->stream));
  int rc = read_ctl(c);
  if (rc) return rc;
  float kms = 0.f;
  VP_HIP(hipEventElapsedTime(&kms, c->ev0, c->ev1));
  *ms += kms;
  *launches += 1;
  const uint32_t nmiss = c->h_ctl.miss_count, ndefer = c->h_ctl.defer_count;

  if (nmiss) {
    MissArgs m{};
    m.a = a;
    m.n = nmiss;
    m.mkey = w.mkey;
    m.mhash = w.mhash;
    m.first = w.first;
    m.rank = w.rank;
    m.rep = w.rep;
    m.assign = w.assign;
    m.scratch = w.scratch;
    const uint32_t ssize = next_pow2((uint64_t)nmiss * 2);
    m.smask = ssize - 1;
    size_t need = 0, need2 = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, need, w.miss, w.miss_sorted,
                                      (int)nmiss, 0, 32, c->stream);
    hipcub::DeviceScan::ExclusiveSum(nullptr, need2, w.first, w.rank, (int)nmiss,
                                     c->stream);
    need = std::max(need, need2);
    if (need > w.cub_bytes) {
      if (w.cub_tmp) VP_HIP(hipFree(w.cub_tmp));
      VP_HIP(hipMalloc(&w.cub_tmp, need));
      w.cub_bytes = need;
    }
    // miss ordinals in packet order
    VP_HIP(hipcub::DeviceRadixSort::SortKeys(w.cub_tmp, w.cub_bytes, w.miss,
                                             w.miss_sorted, (int)nmiss, 0, 32,
                                             c->stream));
    m.list = w.miss_sorted;
    VP_HIP(hipMemsetAsync(w.scratch, 0xFF, sizeof(uint32_t) * (size_t)ssize,
                          c->stream));
    const uint32_t g = grid_for(nmiss);
    nat_miss_keys<<<g, 256, 0, c->stream>>>(m);
    nat_miss_dedup<<<g, 256, 0, c->stream>>>(m);
    nat_miss_first<<<g, 256, 0, c->stream>>>(m);
    VP_HIP(hipcub::DeviceScan::ExclusiveSum(w.cub_tmp, w.cub_bytes, w.first,
                                            w.rank, (int)nmiss, c->stream));
    nat_miss_alloc<<<g, 256, 0, c->stream>>>(m);
    nat_miss_commit<<<1, 64, 0, c->stream>>>(m);
    nat_miss_finish<<<g, 256, 0, c->stream>>>(m);
    VP_HIP(hipGetLastError());
  }
  if (ndefer) {
    nat_defer_finish<<<grid_for(ndefer), 256, 0, c->stream>>>(a, w.defer, ndefer);
    VP_HIP(hipGetLastError());
  }
  if (nmiss) {
    rc = read_ctl(c);
    if (rc) return rc;
    // flows created in this segment carry stamps >= the segment's first time
    const int64_t t0 = b->now ? -1 : b->now0 + (int64_t)p0 * b->now_step;
    (void)t0;
    if ((uint64_t)c->h_ctl.n_tomb + c->h_ctl.n_live > (uint64_t)(t.tmask + 1) * 3 / 4) {
      rc = table_rebuild(c);
      if (rc) return rc;
    }
  } else if (ndefer) {
    VP_HIP(hipStreamSynchronize(c->stream));
  }
  return 0;
}

// Whole batch: cut it where an expiry may happen (see file header).
int nat_process_device(vp_ctx *c, const vp_dev_batch *b) {
  const uint32_t n = b->n;
  c->last_ms = 0.f;
  c->last_launches = 0;
  if (n == 0) return 0;
  if (b->slot < 64 || (b->slot & 15) || !b->frames || !b->len || !b->in_dev ||
      !b->out_dev)
    return VP_EINVAL;
  int rc = ws_reserve(c, n);
  if (rc) return rc;

  // times: monotone, >= 0; ties need last-touch sequence numbers
  std::vector<int64_t> h_now;
  int64_t t_first, t_last;
  bool ties;
  if (b->now) {
    h_now.resize(n);
    VP_HIP(hipMemcpyAsync(h_now.data(), b->now, sizeof(int64_t) * (size_t)n,
                          hipMemcpyDeviceToHost, c->stream));
    VP_HIP(hipStreamSynchronize(c->stream));
    ties = false;
    for (uint32_t i = 1; i < n; i++) {
      if (h_now[i] < h_now[i - 1]) return VP_ENOTSUP;
      ties |= h_now[i] == h_now[i - 1];
    }
    t_first = h_now[0];
    t_last = h_now[n - 1];
  } else {
    if (b->now_step < 0) return VP_ENOTSUP;
    t_first = b->now0;
    t_last = b->now0 + (int64_t)(n - 1) * b->now_step;
    ties = n > 1 && b->now_step == 0;
  }
  if (t_first < 0 || t_first < c->last_now) return VP_ENOTSUP;
  ties |= t_first == c->last_now;
  BatchView v{b, h_now.data()};

  float ms = 0.f;
  int launches = 0;
  uint32_t a0 = 0;
  while (a0 < n) {
    const int64_t ta = v.at(a0);
    // no flow can expire at p while cutoff(t_p) <= min(live stamps); live
    // stamps are >= min(ts_floor, ta) for the whole segment
    uint64_t lim = std::min<uint64_t>(c->ft.ts_floor, (uint64_t)ta);
    auto safe = [&](uint32_t p) { return nat_cutoff(c, v.at(p)) <= (int64_t)lim; };
    if (!safe(a0)) {
      rc = nat_exact_floor(c);
      if (rc) return rc;
      if (c->ft.ts_floor != ~0ull && (int64_t)c->ft.ts_floor < nat_cutoff(c, ta)) {
        rc = nat_expire(c, nat_cutoff(c, ta));
        if (rc) return rc;
        rc = nat_exact_floor(c);
        if (rc) return rc;
      }
      lim = std::min<uint64_t>(c->ft.ts_floor, (uint64_t)ta);
    }
    uint32_t b1;
    if (safe(n - 1)) {
      b1 = n;
    } else {  // first unsafe packet (cutoff is monotone in time)
      uint32_t lo = a0 + 1, hi = n - 1;
      while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (safe(mid)) lo = mid + 1; else hi = mid;
      }
      b1 = lo;
    }
    rc = nat_segment(c, b, a0, b1, ties, &ms, &launches);
    if (rc) return rc;
    if (c->h_ctl.miss_count)  // new flows are stamped >= ta
      c->ft.ts_floor = std::min<uint64_t>(c->ft.ts_floor, (uint64_t)ta);
    a0 = b1;
  }
  c->seq += n;
  c->last_now = t_last;
  c->last_ms = ms;
  c->last_launches = launches;
  return 0;
}

int nat_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys) {
  const uint32_t cap = c->ft.cap;
  uint8_t *d_alloc = nullptr;
  int64_t *d_ts = nullptr;
  uint32_t *d_keys = nullptr;
  VP_HIP(hipMalloc((void **)&d_alloc, cap));
  VP_HIP(hipMalloc((void **)&d_ts, 8ull * cap));
  VP_HIP(hipMalloc((void **)&d_keys, 16ull * cap));
  table_dump<<<grid_for(cap), 256, 0, c->stream>>>(c->ft.slots, c->ft.slot_of,
                                                   cap, d_alloc, d_ts, d_keys);
  VP_HIP(hipMemcpyAsync(alloc, d_alloc, cap, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipMemcpyAsync(ts, d_ts, 8ull * cap, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipMemcpyAsync(keys, d_keys, 16ull * cap, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(hipStreamSynchronize(c->stream));
  hipFree(d_alloc);
  hipFree(d_ts);
  hipFree(d_keys);
  return 0;
}

void build_flowid_tables(std::vector<uint32_t> &tab) {
  tab.assign(15 * 256, 0);
  for (int j = 0; j < 15; j++)
    build_position_table(&tab[j * 256], kFlowIdPos[j], kFlowIdMsg);
}

}  // namespace vp
