// vignat on MI355X: batch classification + flow-state update + rewrite.
//
// Reference behaviour (paths relative to the reference repository):
//   nf_process            vignat/nat_main.c:22-109
//   flow manager          vignat/nat_flowmanager.c:20-94
//   expiry                nat_flowmanager.c:57-65 -> expirator.c:110-218
// A batch is cut into segments inside which no flow can expire (DESIGN.md
// §3); within a segment
//   phase A  every packet is parsed and hashed; LAN packets whose flow exists
//            at segment start are rewritten at once; WAN packets whose index
//            is allocated at segment start likewise; the rest are queued;
//   phase B  queued LAN misses are ordered, de-duplicated by key (earliest
//            packet wins), ranked and given dchain indices in packet order
//            (vp_table.hip), then rewritten;
//   phase C  queued WAN packets see an index as allocated iff it was
//            allocated before them in packet order;
// every packet that touches a flow writes its index to the touch log, which
// tbl_touch_reduce folds into the dchain timestamps (last toucher wins).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "vp_comm.h"
#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(nat)


// FlowId (vignat/flow.h:3-10) is hashed as 6 CRC steps (generated FlowId_hash,
// codegen/main.ml:328-401); the non-zero byte positions of that 24-byte CRC
// message: src_port 0,1  dst_port 4,5  src_ip 8-11  dst_ip 12-15
// device 16,17  protocol 20.
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

// The CRC position tables and, for the linear home-bucket layout, its four
// byte tables behind them (T[kCrcWords ..], see nat_lin).
constexpr uint32_t kCrcWords = 15 * 256;
constexpr uint32_t kNatTabWords = kCrcWords + 1024;
__device__ __forceinline__ const uint32_t *nat_lin(const uint32_t *T) { return T + kCrcWords; }

// flowid_hash for the lean classify tile: the 15 table reads are issued back
// to back and waited for once (compiled from the expression above, every read
// waits for the one before it: 15 LDS round trips per packet). The tables
// must be the kernel's LDS array T (15 x 256 words).
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
#define VP_TAB_RD(t, a, off) \
  asm volatile("ds_read_b32 %0, %1 offset:" #off : "=v"(t) : "v"(a))
__device__ __forceinline__ uint32_t flowid_hash_batched(const uint32_t *T, uint32_t sp,
                                                        uint32_t dp, uint32_t sip,
                                                        uint32_t dip, uint32_t dev,
                                                        uint32_t proto) {
  const uint32_t base = lds_addr(T);
  auto at = [&](uint32_t byte) { return base + (byte << 2); };
  uint32_t t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14;
  VP_TAB_RD(t0, at(sp & 0xFF), 0);
  VP_TAB_RD(t1, at((sp >> 8) & 0xFF), 1024);
  VP_TAB_RD(t2, at(dp & 0xFF), 2048);
  VP_TAB_RD(t3, at((dp >> 8) & 0xFF), 3072);
  VP_TAB_RD(t4, at(sip & 0xFF), 4096);
  VP_TAB_RD(t5, at((sip >> 8) & 0xFF), 5120);
  VP_TAB_RD(t6, at((sip >> 16) & 0xFF), 6144);
  VP_TAB_RD(t7, at(sip >> 24), 7168);
  VP_TAB_RD(t8, at(dip & 0xFF), 8192);
  VP_TAB_RD(t9, at((dip >> 8) & 0xFF), 9216);
  VP_TAB_RD(t10, at((dip >> 16) & 0xFF), 10240);
  VP_TAB_RD(t11, at(dip >> 24), 11264);
  VP_TAB_RD(t12, at(dev & 0xFF), 12288);
  VP_TAB_RD(t13, at((dev >> 8) & 0xFF), 13312);
  VP_TAB_RD(t14, at(proto & 0xFF), 14336);
  // (the results as operands: nothing reads them before this wait)
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3), "+v"(t4), "+v"(t5), "+v"(t6),
                 "+v"(t7), "+v"(t8), "+v"(t9), "+v"(t10), "+v"(t11), "+v"(t12),
                 "+v"(t13), "+v"(t14));
  return (t0 ^ t1 ^ t2) ^ (t3 ^ t4 ^ t5) ^ (t6 ^ t7 ^ t8) ^ (t9 ^ t10 ^ t11) ^
         (t12 ^ t13 ^ t14);
}
#undef VP_TAB_RD

// Owner mode (vp_shard_mode): a LAN packet whose FlowId is
// owned by another rank leaves phase A as a 16-byte key in this block's
// slice for that owner (desc), and route[p] says where its answer will be:
//   route[p] = kRouteBit | owner << 24 | k   k-th key of the block's slice
//            = index < 2^30                  a phase-A touch, frame done
//            = kNone                         nothing left (drop, queued, ...)
// After the exchange, pass 2 (nat_remote64 / nat_remote_lane) finishes the
// routed packets from the owners' replies.
constexpr uint32_t kRouteBit = 0x80000000u;
constexpr uint32_t kRouted = 0xFFFFFFFBu;  // touch: the packet was routed
// Exchange modes (Route::mode):
//   kOwnPadded    one pass 1 / exchange / pass 2 per segment over the padded
//                 exchange, the slice counts exchanged beside the keys and a
//                 slice overflow allreduced (every rank then takes the exact
//                 exchange; cap == 0: the exact exchange itself);
//   kOwnChunked   the chunked pipeline (nat_phase_a_owner_chunked): one
//                 padded exchange per chunk of the segment, on a stream of its
//                 own beside the passes; a block closes its key slices with
//                 sentinel keys (the owner needs no counts), a key past its
//                 slice sets this rank's *lovf and waits;
//   kOwnLeftover  after any rank's *lovf: the exact exchange of the keys
//                 past their slices only (pass 2 finishes just those packets).
enum : uint32_t { kOwnPadded = 0, kOwnChunked = 1, kOwnLeftover = 2 };
constexpr uint32_t kKeySentinelW = 0xFFFFFFFFu;  // key.w of an empty slot (a routed
                                                 // key's is in_dev | proto << 16)
struct Route {
  uint32_t n, r;          // ranks, this rank (n == 0: single table)
  uint4 *desc;            // [block][n][range] keys by owner
  uint32_t *dcnt;         // [block][n] keys per slice
  uint32_t *route;        // per packet
  uint32_t *cur;          // the kernel's LDS cursors per owner
  uint32_t first, range;  // packets of block b: [first + b * range, +range)
  const uint32_t *dbase;  // pass 2: [block][n] offset of the slice's replies
  const uint32_t *rreply; // pass 2: replies (index or kNone), in send order
  // the padded exchange: owner o's replies at [o cap, (o + 1) cap); a key
  // past its owner's cap, or any rank's overflow (*ovf), has no reply in
  // this pass (cap == 0: the exact exchange, every key answered)
  uint32_t cap;
  const uint64_t *ovf;
  // VIGPATH_ROUTE_ALL=1 (profiling): every LAN key goes through the
  // exchange, this rank's own included (one rank: the whole pipeline at 100 %
  // routed)
  uint32_t all;
  // padded exchange: owner o's chunk of the send buffer is one slice of
  // `sub` keys per block, block b's keys for o at o cap + b sub + k (k <
  // sub; pass 1 writes them there itself, past sub into desc)
  uint4 *sendk;
  uint32_t sub;
  uint32_t mode;   // kOwnPadded / kOwnChunked / kOwnLeftover
  uint32_t *lovf;  // kOwnChunked: this rank's slice-overflow flag (Ctl::route_ovf)
  uint32_t *need;  // kOwnChunked: per owner, the largest slice of any block (atomicMax)
};
constexpr uint32_t kNoReply = 0xFFFFFFFAu;  // route_answer: not answered in this pass
constexpr uint32_t kAnswered = 0xFFFFFFF9u;  // route_answer: answered by an earlier pass

struct NatArgs {
  uint8_t *frames;
  const uint16_t *len;
  const uint16_t *in_dev;  // null: every packet on port in0 (vp_dev_batch.in_port)
  uint32_t in0;
  uint16_t *out;
  uint32_t *log;
  NowSpec now;
  uint64_t seq_base;
  uint32_t slot, p0, p1;
  TableDev t;
  const uint32_t *crc_tab;
  const uint32_t *macw;
  uint32_t wan_macw0, wan_macw1, wan_macw2;
  uint32_t *miss;
  uint32_t *defer;
  uint32_t *reprobe;
  uint32_t tileq;  // 64-byte tiles: reprobes go to the block's TileQueue slice
  uint32_t ext_ip;
  uint16_t wan, start_port, n_dev;
  Route own;
  // Host frames (vp_process_mbufs, vp_mbuf.hip): 64-byte header slots of
  // longer frames, tail[p] = the raw sum of frame p's bytes [64, end) the L4
  // checksum covers (0 where nothing lies past 64); null otherwise.
  const uint32_t *tail;
  // 64-byte tiles (nat_tiles): the lean tiles' phase-A misses go to the
  // block's slice of mq (LDS cursor kCurMiss) and are appended to `miss` once
  // per block at its end, not by one global atomic per wave (a churn batch
  // has misses in every wave); null elsewhere
  uint32_t *mq;
  // virtual blocks (vper != 0, the chunked owner pipeline): this launch is
  // blocks vb0 .. vb0 + gridDim.x - 1 of a segment-wide grid whose blocks own
  // vper tiles each (frames64_tiles, vp_device.h)
  uint32_t vb0, vper;
  // one GPU (tbl_new_keys_unsorted): every queued miss also leaves its FlowId
  // and hash, miss[k] <-> mkey[k] / mhash[k] (the lean tiles through their
  // block's slices mkq / mhq beside mq); null: positions only
  uint4 *mkey;
  uint32_t *mhash;
  uint4 *mkq;
  uint32_t *mhq;
  // 1024-thread tiles: bin entries staged in LDS and stored a whole line at
  // a time (bins_put_staged; VIGPATH_BIN_STAGE=0 off, for A/B)
  uint32_t bstage;
  // 1024-thread tiles: the block's range cut into `split` contiguous
  // sub-ranges, W / split waves interleaved over each (tile_split(); 0 or 1:
  // all W waves over the whole range)
  uint32_t split;
  // one GPU, touch bins: the launch's last block publishes phase A's control
  // block (tile_publish; pub.pub null: the fold does)
  PubArgs pub;
};

// The end of a 64-byte tile block: every block releases its counters (its
// XCD's L2 written back, so plain stores such as TouchBins' overflow flag
// reach memory too) and counts itself in Ctl::arrive; the last one acquires
// and publishes the control block to the host (ctl_publish), which then
// learns phase A's counts a fold-kernel dispatch earlier and launches the
// next batch while the fold still runs.
// Off by default (VIGPATH_TILE_PUB=1: on): every block's release lengthened
// the headline kernel by 6 us and the step by 5 (profiles/r06s_tile_pub.txt)
// -- the host is not on the step's critical path; the fold and the two
// dispatches around it are.
static bool tile_pub_on() {
  static const bool on = [] {
    const char *e = getenv("VIGPATH_TILE_PUB");
    return e && atoi(e) != 0;
  }();
  return on;
}
__device__ __forceinline__ void tile_publish(const NatArgs &a) {
  if (!a.pub.pub) return;
  // every wave's stores and atomics acknowledged (in its XCD's L2) before the
  // barrier, so thread 0's release writes them back with its own
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return;
  Ctl *ctl = const_cast<Ctl *>(a.pub.ctl);
  const uint32_t n =
      __hip_atomic_fetch_add(&ctl->arrive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (n != gridDim.x - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the other blocks' releases)
  __hip_atomic_store(&ctl->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ctl_publish(a.pub);
}

// Queue packet p (FlowId key, hash h) as a phase-B miss.
__device__ __forceinline__ void miss_add(const NatArgs &a, uint32_t p, const uint32_t key[4],
                                         uint32_t h) {
  const uint32_t k = wave_append(&a.t.ctl->miss_count, true);
  a.miss[k] = p;
  if (a.mkey) {
    a.mkey[k] = make_uint4(key[0], key[1], key[2], key[3]);
    a.mhash[k] = h;
  }
}

// The register path's total_length bound for 64-byte slots (every L4 byte in
// the slot), or any total_length for header slots with tail sums.
__device__ __forceinline__ uint32_t nat_lim64(const NatArgs &a) {
  return a.tail ? 0xFFFFu : 50u;
}
__device__ __forceinline__ uint32_t nat_tail(const NatArgs &a, uint32_t p) {
  return a.tail ? a.tail[p] : 0u;
}

// Lanes with `v` reserve consecutive slots of counter ctr[ch] (LDS): one
// atomic per distinct counter in the wave (a wave's routed keys go to few
// owners; one atomic per lane serialised a wave 64 deep on one counter).
// Returns the lane's slot.
__device__ __forceinline__ uint32_t multi_reserve(uint32_t *ctr, uint32_t ch, bool v) {
  uint64_t pend = __ballot(v);
  uint32_t res = 0;
  const uint32_t lane = __lane_id();
  while (pend) {
    const uint32_t lead = (uint32_t)__ffsll((unsigned long long)pend) - 1;
    const uint32_t lc = (uint32_t)__shfl((int)ch, (int)lead);
    const uint64_t same = __ballot(v && ch == lc) & pend;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(&ctr[lc], (uint32_t)__popcll(same));
    base = (uint32_t)__shfl((int)base, (int)lead);
    if ((same >> lane) & 1ull) res = base + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
    pend &= ~same;
  }
  return res;
}

// Owner mode: hand the LAN packet with key `key` (hash h) to its owner if
// that is another rank. Returns true when routed. (Lanes that do not call
// it take no part in the reservation: it runs on the calling lanes.)
__device__ __forceinline__ bool nat_route(const NatArgs &a, uint32_t p, uint32_t h,
                                          const uint32_t key[4]) {
  if (!a.own.n) return false;
  const uint32_t o = owner_of(h, a.own.n);
  const bool go = o != a.own.r || a.own.all;
  const uint32_t k = multi_reserve(a.own.cur, o, go);
  if (!go) return false;
  const uint4 v = make_uint4(key[0], key[1], key[2], key[3]);
  if (k < a.own.sub) {  // (the padded exchange's own slice: no packing pass)
    a.own.sendk[(size_t)o * a.own.cap + (size_t)blockIdx.x * a.own.sub + k] = v;
  } else {
    a.own.desc[((size_t)(a.vb0 + blockIdx.x) * a.own.n + o) * a.own.range + k] = v;
    if (a.own.mode == kOwnChunked) atomicOr(a.own.lovf, 1u);  // (rare: skew)
  }
  a.own.route[p] = kRouteBit | (o << 24) | k;
  return true;
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

// Generic (byte-addressed) phase A for frames outside the register fast path
// (IP options, long frames, odd headers). Same decisions as nat_classify.
// (inlined: measured faster than a call, round 2)
__device__ uint32_t nat_generic_a(const NatArgs &a, const uint32_t *T,
                                       uint32_t p, uint32_t in, uint32_t len) {
  GFrame f{a.frames + (size_t)p * a.slot, a.slot};
  L34 h = parse_l34(f, len);
  if (!h.ok) {
    a.out[p] = (uint16_t)in;
    log_put(a.log, p, kNone);
    return kNone;
  }
  const uint32_t proto = f.r8(h.ip + 9);
  const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
  const uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
  uint32_t dst, logged;
  if (in == a.wan) {
    const int idx = (int)dp - (int)a.start_port;
    if (idx < 0 || idx >= (int)a.t.cap) {  // reference UB range: unallocated
      a.out[p] = (uint16_t)in;
      log_put(a.log, p, kNone);
      return kNone;
    }
    const uint32_t s = a.t.slot_of[idx];
    if (s == kNone) {
      a.defer[wave_append(&a.t.ctl->defer_count, true)] = p;
      log_put(a.log, p, kNone);  // phase C writes the real entry
      return kNone;
    }
    const uint4 fk = tbl_key_of(a.t, (uint32_t)idx);
    const uint32_t k0 = fk.x, k1 = fk.y, k2 = fk.z, k3 = fk.w;
    log_put(a.log, p, (uint32_t)idx);  // rejuvenated before the anti-spoof check
    if ((k2 != sip) | ((k0 >> 16) != sp) | (((k3 >> 16) & 0xFF) != proto)) {
      a.out[p] = (uint16_t)in;
      return (uint32_t)idx;
    }
    logged = (uint32_t)idx;
    f.w32(h.ip + 16, k1);
    f.w16(h.l4 + 2, (uint16_t)(k0 & 0xFFFF));
    dst = k3 & 0xFFFF;
  } else {
    const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
    const uint32_t hh = flowid_hash(T, sp, dp, sip, dip, in, proto);
    if (nat_route(a, p, hh, key)) {
      log_put(a.log, p, kNone);  // pass 2 writes the real entry
      return kRouted;
    }
    const uint32_t idx = tbl_probe(a.t, hh, key);
    if (idx == kNone) {
      miss_add(a, p, key, hh);
      log_put(a.log, p, kNone);  // phase B writes the real entry
      return kNone;
    }
    log_put(a.log, p, idx);
    logged = idx;
    f.w32(h.ip + 12, a.ext_ip);
    f.w16(h.l4, (uint16_t)(a.start_port + idx));
    dst = a.wan;
  }
  set_checksums(f, h.ip, h.l4, nat_tail(a, p));
  uint32_t mw[3];
  macs_for(a, dst, mw);
  set_macs(f, mw);
  a.out[p] = (uint16_t)dst;
  return logged;
}

// Phase A for one packet whose 64-byte slot is in registers, in two halves
// (frames64_tiles): nat_issue parses the headers and issues the packet's
// first dependent read — the home bucket of a LAN packet's FlowId, the
// entry slot of a WAN packet's index — and nat_finish consumes it, rewrites
// the frame and returns true when it must be stored back.
enum : uint32_t { kPendDone = 0, kPendGeneric = 1, kPendLan = 2, kPendWan = 3,
                  kPendRemote = 4 };
struct NatPend {
  uint32_t kind;
  uint32_t row;  // LAN: home bucket, gathered by frames64_tiles; else kNone
  uint32_t b;    // LAN: home bucket; WAN: flow index
  uint32_t s;    // WAN: slot_of[index]; LAN: the FlowId hash
};

// `lim`: the longest total_length the register path takes (50: the L4 bytes
// all lie in the 64 registers; slot - 14 in the wide-slot kernels, whose
// nat_finish gets the rest of the sum as `tail`).
__device__ __forceinline__ NatPend nat_issue(const NatArgs &a, const uint32_t *T,
                                             uint32_t p, const RFrame &f,
                                             uint32_t in, uint32_t len,
                                             bool mine, uint32_t lim = 50) {
  NatPend P;
  P.kind = kPendDone;
  P.row = kNone;
  if (!mine) return P;
  const uint32_t et = f.w[3] & 0xFFFF;
  const uint32_t ihl = (f.w[3] >> 16) & 0x0F;
  const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
  if (!(et == 0x0008 && ihl == 5 && tl <= lim)) {
    P.kind = kPendGeneric;  // byte-addressed path (nat_generic_a)
    return P;
  }
  // nf_then_get_rte_ipv4_header / nf_then_get_tcpudp_header with IHL = 5
  const uint16_t unread = (uint16_t)(len - 14);
  const uint32_t proto = f.w[5] >> 24;
  const bool ok = (unread >= 20) & (unread >= tl) &
                  ((proto == 6) | (proto == 17)) & ((uint32_t)(len - 34) >= 4u);
  if (!ok) {
    a.out[p] = (uint16_t)in;
    log_put(a.log, p, kNone);
    return P;
  }
  const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
  if (in == a.wan) {
    // flow_manager_get_external (nat_flowmanager.c:78-94)
    const int idx = (int)dp - (int)a.start_port;
    if (idx < 0 || idx >= (int)a.t.cap) {
      a.out[p] = (uint16_t)in;
      log_put(a.log, p, kNone);
      return P;
    }
    P.kind = kPendWan;
    P.b = (uint32_t)idx;
    P.s = a.t.slot_of[idx];
  } else {
    // flow_manager_get_internal (nat_flowmanager.c:67-76): map_get's hash
    const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
    const uint32_t hh = flowid_hash(T, sp, dp, sip, dip, in, proto);
    if (a.own.n && (owner_of(hh, a.own.n) != a.own.r || a.own.all)) {  // another rank's key
      P.kind = kPendRemote;
      P.b = hh;
      return P;
    }
    P.kind = kPendLan;
    P.b = home_bucket(hh, a.t.bmask, a.t.mix, nat_lin(T));
    P.row = P.b;
    P.s = hh;
  }
  return P;
}

__device__ __forceinline__ bool nat_finish(const NatArgs &a, const uint32_t *T,
                                           const NatPend &P, const uint4 *row,
                                           uint32_t p, RFrame &f, uint32_t in,
                                           uint32_t len, uint32_t &touch,
                                           uint32_t tail = 0) {
  if (P.kind == kPendDone) return false;
  if (P.kind == kPendGeneric) {
    touch = nat_generic_a(a, T, p, in, len);  // writes global memory itself
    return false;
  }
  const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
  const uint32_t proto = f.w[5] >> 24;
  const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
  const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
  uint32_t dst;
  uint32_t mw[3];
  if (P.kind == kPendRemote) {
    const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
    nat_route(a, p, P.b, key);
    log_put(a.log, p, kNone);  // pass 2 writes the real entry
    touch = kRouted;
    return false;
  }
  if (P.kind == kPendWan) {
    const uint32_t idx = P.b;
    const uint32_t s = P.s;
    if (s == kNone) {  // maybe allocated earlier in this segment: phase C
      a.defer[wave_append(&a.t.ctl->defer_count, true)] = p;
      log_put(a.log, p, kNone);  // phase C writes the real entry
      return false;
    }
    const uint4 k = a.t.kv ? a.t.kv[idx]  // owner mode: keys by index
                           : reinterpret_cast<const uint4 *>(a.t.bk + (s >> 2))[s & 3];
    log_put(a.log, p, idx);  // rejuvenated before the anti-spoof check
    touch = idx;
    if ((k.z != sip) | ((k.x >> 16) != sp) | (((k.w >> 16) & 0xFF) != proto)) {
      a.out[p] = (uint16_t)in;  // nat_main.c:55-60
      return false;
    }
    f.set32at2(30, k.y);        // dst_addr = flow.src_ip
    f.set16(36, k.x & 0xFFFF);  // dst_port = flow.src_port
    dst = k.w & 0xFFFF;         // flow.internal_device
    macs_for(a, dst, mw);
  } else {
    const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
    bool done;
    const uint32_t idx = bucket_match(row[0], row[1], row[2], row[3], key, &done);
    if (!done) {  // the bucket is full of other keys: nat_reprobe walks the
      // rest of the path, so this wave does not wait for a dependent read
      log_put(a.log, p, kNone);
      if (a.tileq)
        touch = kReprobe;
      else
        a.reprobe[wave_append(&a.t.ctl->reprobe_count, true)] = p;
      return false;
    }
    if (idx == kNone) {  // new flow, or not yet visible: phase B
      miss_add(a, p, key, P.s);
      log_put(a.log, p, kNone);  // phase B writes the real entry
      return false;
    }
    log_put(a.log, p, idx);
    touch = idx;
    f.set32at2(26, a.ext_ip);                     // src_addr = external_addr
    f.set16(34, (uint16_t)(a.start_port + idx));  // src_port = external port
    dst = a.wan;
    mw[0] = a.wan_macw0;
    mw[1] = a.wan_macw1;
    mw[2] = a.wan_macw2;
  }
  fast_checksums(f, proto, tl, tail);
  f.w[0] = mw[0];
  f.w[1] = mw[1];
  f.w[2] = mw[2];
  a.out[p] = (uint16_t)dst;
  return true;
}

__device__ __forceinline__ void load_crc_tables(uint32_t *T, const uint32_t *g) {
  for (uint32_t i = threadIdx.x; i < 15 * 256; i += blockDim.x) T[i] = g[i];
  __syncthreads();
}
__device__ __forceinline__ void load_nat_tables(uint32_t *T, const NatArgs &a) {
  if (a.t.mix == kMixLin)
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[kCrcWords + i] = a.t.lin[i];
  load_crc_tables(T, a.crc_tab);
}


// Owner mode: the route of a packet phase A did not hand to another rank
// (its touch, or nothing); returns the touch for this launch's bins.
__device__ __forceinline__ uint32_t route_note(const NatArgs &a, uint32_t p,
                                               uint32_t touch) {
  if (!a.own.n) return touch;
  if (touch == kRouted) return kNone;
  a.own.route[p] = touch == kReprobe ? kNone : touch;
  return touch == kReprobe ? kReprobe : kNone;  // pass 2 bins the touches
}

// Owner mode: publish (virtual) block rb's key count per owner (after a
// barrier); the chunked pipeline also closes each of the block's slices with
// sentinel keys and raises need[o] to its slice's count.
__device__ __forceinline__ void route_publish(const NatArgs &a, const uint32_t *cur,
                                              uint32_t rb) {
  if (!a.own.n) return;
  __syncthreads();
  for (uint32_t o = threadIdx.x; o < a.own.n; o += blockDim.x) {
    a.own.dcnt[(size_t)rb * a.own.n + o] = cur[o];
    if (a.own.mode == kOwnChunked && cur[o]) atomicMax(&a.own.need[o], cur[o]);
  }
  if (a.own.mode != kOwnChunked) return;
  const uint4 none = make_uint4(0u, 0u, 0u, kKeySentinelW);
  for (uint32_t o = 0; o < a.own.n; o++) {
    uint4 *sl = a.own.sendk + (size_t)o * a.own.cap + (size_t)blockIdx.x * a.own.sub;
    for (uint32_t j = min(cur[o], a.own.sub) + threadIdx.x; j < a.own.sub; j += blockDim.x)
      sl[j] = none;
  }
}

// One packet, its slot's first 64 bytes in registers (any slot size; frames
// outside the fast path take nat_generic_a). Returns the logged index.
__device__ __forceinline__ uint32_t nat_lane(const NatArgs &a, const uint32_t *T,
                                             uint32_t p) {
  uint4 *fp = reinterpret_cast<uint4 *>(a.frames + (size_t)p * a.slot);
  RFrame f;
  const uint4 c0 = ld_stream(fp), c1 = ld_stream(fp + 1), c2 = ld_stream(fp + 2),
              c3 = ld_stream(fp + 3);
  f.w[0] = c0.x; f.w[1] = c0.y; f.w[2] = c0.z; f.w[3] = c0.w;
  f.w[4] = c1.x; f.w[5] = c1.y; f.w[6] = c1.z; f.w[7] = c1.w;
  f.w[8] = c2.x; f.w[9] = c2.y; f.w[10] = c2.z; f.w[11] = c2.w;
  f.w[12] = c3.x; f.w[13] = c3.y; f.w[14] = c3.z; f.w[15] = c3.w;
  const uint32_t in = port_of(a.in_dev, a.in0, p), len = a.len[p];
  uint32_t touch = kNone;
  const NatPend P = nat_issue(a, T, p, f, in, len, true, nat_lim64(a));
  uint4 row[4] = {};
  if (P.row != kNone) {
    const uint4 *q = reinterpret_cast<const uint4 *>(a.t.bk + P.row);
    row[0] = q[0];
    row[1] = q[1];
    row[2] = q[2];
    row[3] = q[3];
  }
  if (nat_finish(a, T, P, row, p, f, in, len, touch, nat_tail(a, p))) {
    st_stream(fp, make_uint4(f.w[0], f.w[1], f.w[2], f.w[3]));
    st_stream(fp + 1, make_uint4(f.w[4], f.w[5], f.w[6], f.w[7]));
    st_stream(fp + 2, make_uint4(f.w[8], f.w[9], f.w[10], f.w[11]));
    if ((f.w[5] >> 24) == 6)
      st_stream(fp + 3, make_uint4(f.w[12], f.w[13], f.w[14], f.w[15]));
  }
  return route_note(a, p, touch);
}

// Phase A, any slot size: one packet per lane, grid-stride, the first 64
// bytes of the slot as four 16-byte loads per lane.
__global__ __launch_bounds__(256) void nat_classify(NatArgs a) {
  __shared__ uint32_t T[kNatTabWords];
  __shared__ uint32_t dcur[kMaxDest];
  if (a.own.n) {  // owner mode: block b takes packets [first + b * range, +range)
    for (uint32_t o = threadIdx.x; o < kMaxDest; o += blockDim.x) dcur[o] = 0;
    a.own.cur = dcur;
  }
  load_nat_tables(T, a);  // (its barrier also covers dcur)
  if (a.own.n) {
    const uint32_t b0 = a.own.first + blockIdx.x * a.own.range;
    const uint32_t b1 = min(a.p1, b0 + a.own.range);
    for (uint32_t p = b0 + threadIdx.x; p < b1; p += blockDim.x) nat_lane(a, T, p);
    route_publish(a, dcur, blockIdx.x);
    return;
  }
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += stride)
    nat_lane(a, T, p);
}

// The fast-path predicate of nat_issue for a LAN packet: IPv4, IHL 5,
// total_length <= 50 (every L4 byte in the slot), and the parse accepts it
// (nf_then_get_rte_ipv4_header / nf_then_get_tcpudp_header, nf-util.h:116-162).
// The register path's parse (any direction): IPv4, IHL 5, total_length <=
// lim (nat_issue), and nf_then_get_* accept it (nf-util.h:116-162).
__device__ __forceinline__ bool nat_reg_ok(const RFrame &f, uint32_t len, uint32_t lim) {
  const uint32_t et = f.w[3] & 0xFFFF;
  const uint32_t ihl = (f.w[3] >> 16) & 0x0F;
  const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
  const uint32_t proto = f.w[5] >> 24;
  const uint16_t unread = (uint16_t)(len - 14);
  return (et == 0x0008) & (ihl == 5) & (tl <= lim) & (unread >= 20) & (unread >= tl) &
         ((proto == 6) | (proto == 17)) & ((uint32_t)(len - 34) >= 4u);
}
__device__ __forceinline__ bool nat_lan_fast_ok(const NatArgs &a, const RFrame &f,
                                                uint32_t in, uint32_t len,
                                                uint32_t lim = 50) {
  return (in != a.wan) & nat_reg_ok(f, len, lim);
}

// bucket_match without branches (the same answer): entries in order, the
// first empty entry ends the probe, a tombstone never matches.
__device__ __forceinline__ uint32_t bucket_match_sel(const uint4 *row,
                                                    const uint32_t key[4], bool *done) {
  const uint4 ix = row[3];
  const bool e0 = ix.x == kEmpty, e1 = ix.y == kEmpty, e2 = ix.z == kEmpty;
  const bool m0 = (ix.x != kTomb) & !e0 &
                  (((row[0].x ^ key[0]) | (row[0].y ^ key[1]) | (row[0].z ^ key[2]) |
                    (row[0].w ^ key[3])) == 0);
  const bool m1 = (ix.y != kTomb) & !e1 &
                  (((row[1].x ^ key[0]) | (row[1].y ^ key[1]) | (row[1].z ^ key[2]) |
                    (row[1].w ^ key[3])) == 0);
  const bool m2 = (ix.z != kTomb) & !e2 &
                  (((row[2].x ^ key[0]) | (row[2].y ^ key[1]) | (row[2].z ^ key[2]) |
                    (row[2].w ^ key[3])) == 0);
  *done = m0 | e0 | m1 | e1 | m2 | e2;
  return m0 ? ix.x : e0 ? kNone : m1 ? ix.y : e1 ? kNone : m2 ? ix.z : kNone;
}

// A lean tile's probe walk on from a full home bucket b, in the lane
// (tbl_probe_from's order; lanes with !*done walk, `idx` is the home
// bucket's answer). Random keys leave ~0.2 % of their packets here every
// batch, whose reprobe launch and control-block read-back this spares. The
// loop is wave-uniform, so one long path would stall all 64 lanes: it stops
// after kLeanWalk buckets past home (tombstone-heavy tables, the
// multiplicative spread at high load), and a lane still !*done then queues
// for nat_reprobe, which walks the whole path.
constexpr uint32_t kLeanWalk = 4;
__device__ __forceinline__ uint32_t lean_walk(const NatArgs &a, const uint4 *rows, uint32_t b,
                                              const uint32_t key[4], uint32_t idx, bool *done) {
  if (__ballot(!*done)) {
    uint32_t nb = b;
    const uint32_t steps = min(a.t.bmask, kLeanWalk);
    for (uint32_t st = 0; st < steps && __ballot(!*done); st++) {
      if (!*done) {
        nb = (nb + 1) & a.t.bmask;
        const uint4 *q = rows + 4 * (size_t)nb;
        const uint4 r2[4] = {q[0], q[1], q[2], q[3]};
        idx = bucket_match_sel(r2, key, done);
      }
    }
  }
  return idx;
}

// 128-byte slots: the tail sums of the wave's tile from the registers the
// dense fetch left (d[j] = chunk 64 j + lane: frame 8 j + lane / 8, part
// lane % 8; parts 4-7 are the bytes 64-127 the L4 sum may cover), right
// after the loads so the 8 chunks die early: each 8-lane group takes its
// frame's end, 14 + total_length (bytes 16-17: part 1, the group's second
// lane; only register-path frames, whose total_length is at most 114, use
// the sum), adds the masked chunks, and frame f's sum goes to lane f (round
// j = f / 8, from lane 8 (f % 8)).
__device__ __forceinline__ uint32_t dense128_tail(const uint4 d[8]) {
  const uint32_t lane = threadIdx.x & 63, part = lane & 7;
  uint32_t tail = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; j++) {
    const uint32_t w4 = (uint32_t)__shfl((int)d[j].x, (int)((lane & ~7u) | 1u));
    const uint32_t e = min(128u, 14u + bswap16((uint16_t)(w4 & 0xFFFF)));
    const uint32_t o = 16 * part;
    uint32_t s = 0;
    if (part >= 4 && o < e) {
      uint4 x = d[j];
      if (e - o < 16) x = chunk_keep(x, 0, (int)(e - o));
      s = sum16x4(x, 0u);
    }
    s += (uint32_t)__shfl_xor((int)s, 1);
    s += (uint32_t)__shfl_xor((int)s, 2);
    s += (uint32_t)__shfl_xor((int)s, 4);
    const uint32_t got = (uint32_t)__shfl((int)s, (int)((lane & 7) * 8));
    if ((lane >> 3) == j) tail = got;
  }
  return tail;
}

// Phase A over tiles of 64 consecutive packets per wave, the frames staged
// through the wave's LDS tile. G = 0: 64-byte slots (nat_classify64), every
// global load/store instruction 1 KiB contiguous (the loop of frames64_tiles,
// vp_device.h, whose comments describe the layout and the order of the
// memory operations). G > 0: wider slots (nat_classify_wide<G>, DESIGN.md
// §5.4): the same tile with each frame's first 64 bytes gathered four lanes
// per frame (16 frames per instruction, 64 contiguous bytes each), the L4
// sum's remainder from tile_tail_sums (G lanes per frame, contiguous 16 G-byte
// runs), and only the header chunks a rewrite changed stored back. A wave
// whose 64 packets are all register-path LAN packets (the steady state of a
// LAN->WAN stream, BASELINE config 2) takes a straight-line tile: hash, one
// cooperative bucket-row gather, branch-free match, rewrite and checksums in
// registers, (64-byte slots) the whole tile stored back (packets left for
// phase B or the reprobe walk are stored unchanged). Any other tile runs
// nat_issue / nat_finish per lane. Owner mode's pass 1 has a lean tile of its
// own (keys of other ranks routed, this rank's looked up).
// W: waves per block (4: 256-thread blocks, four per CU; 16: one 1024-thread
// block per CU, nat_classify64w).
// O: owner mode compiled in (false: the single-table kernels, whose owner
// paths -- pass 1's routing tile, nat_issue's remote keys, route notes --
// fold away with own.n a constant 0, fewer registers for the lean tile).
template <uint32_t G, uint32_t H = 1, bool D = false, bool X = false, bool PR = G == 0,
          uint32_t W = 4, bool ST = false, bool O = true>
__device__ __forceinline__ void nat_tiles(NatArgs a, uint32_t n_all, TouchBins bins,
                                          TileQueue rq) {
  static_assert(!X || G == 0, "header slots (X) are 64-byte slots");
  if constexpr (!O) {
    a.own.n = 0;
    a.own.all = 0;
  }
  __shared__ uint32_t T[kNatTabWords];
  __shared__ uint4 stage[W][256];
  __shared__ uint32_t cur[kCurs];
  __shared__ uint32_t mbase;
  // (ST, 1024-thread blocks: whole-line bin entries, bins_put_staged)
  constexpr bool kStaged = ST && W == 16;
  __shared__ uint32_t nruns;  // this block's run tiles (Ctl::run_tiles)
  __shared__ uint32_t sring[kStaged ? kStageBins * kStageLines * 16 : 1];
  __shared__ uint32_t swc[kStaged ? kStageBins * kStageLines : 1];
  __shared__ uint32_t sgen[kStaged ? kStageBins * kStageLines : 1];
  const BinStage bst{sring, swc, sgen};
  const bool staged = kStaged && bins.ent && bins.bbits <= 7 && a.bstage;
  if (kStaged) bins_stage_init(bst);
  if (threadIdx.x == 0) nruns = 0;
  for (uint32_t i = threadIdx.x; i < kCurs; i += blockDim.x) cur[i] = 0;
  a.own.cur = cur + kCurDest;
  load_nat_tables(T, a);  // (its barrier also covers cur)
  uint4 *S = stage[threadIdx.x >> 6];
  const uint4 *rows = reinterpret_cast<const uint4 *>(a.t.bk);
  const uint32_t lane = threadIdx.x & 63;
  // the wave index as a scalar, so tile addresses (the buffer resources of the
  // tile stores, tile_tail_sums and the header gathers) are provably uniform
  // and need no waterfall loop (cdna_hip_programming.md T20; as a vector
  // value every 64-byte tile store ran a readfirstlane loop)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t first = a.p0 & ~63u;
  const uint32_t tiles = (a.p1 - first + 63) / 64;
  const bool lean_ok = a.own.n == 0 && rq.ent != nullptr;
  const bool lean_own = G == 0 && a.own.n != 0 && rq.ent != nullptr;  // owner pass 1
  const uint32_t slot = G ? a.slot : 64u;
  const uint32_t lim = slot - 14;  // total_length bound of the register path
  // 64-byte slots: every L4 byte in the slot, or (X: header slots of longer
  // host frames) any total_length, the L4 sum's rest from a.tail
  const uint32_t lim64 = X ? 0xFFFFu : 50u;
  // byte offset in the tile of chunk c (packet c / 4, part c % 4)
  auto chunk_at = [&](uint32_t c) -> uint32_t {
    return G ? (c >> 2) * slot + (c & 3) * 16 : c * 16;
  };
  uint4 r[4];
  uint32_t m_in = 0, m_len = 0, m_tail = 0;
  auto fetch = [&](uint32_t tile) {
    const uint32_t tb = first + tile * 64;
    const uint8_t *g8 = a.frames + (size_t)tb * slot;
    const uint32_t p = tb + lane;
    if constexpr (X) m_tail = p < n_all ? a.tail[p] : 0u;
    if constexpr (G > 0) {  // one buffer resource per tile: slots past the
      // batch read as zeros
      const uint32_t bytes = min(64u, n_all - tb) * slot;
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) r[j] = buf_ld16(g8, bytes, chunk_at(64 * j + lane));
      m_in = p < n_all ? port_of(a.in_dev, a.in0, p) : 0u;
      m_len = p < n_all ? a.len[p] : 0u;
      return;
    }
    if (tb + 64 <= n_all) {  // (wave-uniform) a whole tile: no per-lane guards
#pragma unroll
      for (uint32_t j = 0; j < 4; j++)
        r[j] = tile_ld(reinterpret_cast<const uint4 *>(g8 + chunk_at(64 * j + lane)));
      m_in = port_of(a.in_dev, a.in0, p);
      m_len = a.len[p];
      return;
    }
    const uint32_t avail = n_all - tb;  // in the batch
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t c = 64 * j + lane;
      r[j] = (c >> 2) < avail ? tile_ld(reinterpret_cast<const uint4 *>(g8 + chunk_at(c)))
                              : make_uint4(0, 0, 0, 0);
    }
    m_in = p < n_all ? port_of(a.in_dev, a.in0, p) : 0u;
    m_len = p < n_all ? a.len[p] : 0u;
  };
  const uint32_t rb = a.vb0 + blockIdx.x;  // (virtual blocks: the chunked pipeline)
  const uint32_t per_b = a.vper ? a.vper : (tiles + gridDim.x - 1) / gridDim.x;
  // (split: sub-range wv / (W / split) of the block's range, W / split waves
  // interleaved over it -- the streams of `split` smaller blocks)
  const uint32_t ks = W == 16 && (a.split == 2 || a.split == 4) ? a.split : 1u;
  const uint32_t tstep = W / ks, per_s = (per_b + ks - 1) / ks, sub = wv / tstep;
  uint32_t tile = rb * per_b + sub * per_s + (wv - sub * tstep);
  const uint32_t tend = min(tiles, rb * per_b + min(per_b, (sub + 1) * per_s));
  const uint32_t range0 = first + rb * per_b * 64;  // this block's first packet
  // a lean tile's misses (wave-uniform call), with their FlowIds and hashes
  // when phase B takes them unsorted (a.mkq)
  auto miss_put = [&](bool miss, const uint32_t key[4], uint32_t h) {
    if (a.mq) {
      const uint32_t k = group_reserve(cur, kCurMiss, miss);
      const size_t at = (size_t)rb * per_b * 64 + k;
      if (miss) a.mq[at] = tile * 64 + first + lane;
      if (miss && a.mkq) {
        a.mkq[at] = make_uint4(key[0], key[1], key[2], key[3]);
        a.mhq[at] = h;
      }
    } else if (miss) {
      miss_add(a, first + tile * 64 + lane, key, h);
    }
  };
  // (wide slots: the headers of the wave's own tile at its start; a prefetch
  // of the next tile's would keep 16 registers the tail sums need)
  if (G == 0 && tile < tend) fetch(tile);
  for (; tile < tend; tile += tstep) {
    const uint32_t tb = first + tile * 64;
    uint8_t *g8 = a.frames + (size_t)tb * slot;
    uint4 *g = reinterpret_cast<uint4 *>(g8);
    uint4 d8[D ? 8 : 1];  // D: the whole tile (128-byte slots)
    uint32_t tail128 = 0;
    if constexpr (D) {
      // 128-byte slots: the tile's 8 KiB as eight 1 KiB-contiguous loads,
      // header chunks (part < 4 of a slot) into the frame image, the tail
      // chunks summed from registers below (dense128_tail): one round trip
      const uint32_t bytes = min(64u, n_all - tb) * 128u;
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) d8[j] = buf_ld16(g8, bytes, (64 * j + lane) * 16);
      const uint32_t pp = tb + lane;
      m_in = pp < n_all ? a.in_dev[pp] : 0u;  // (wide slots: always an array)
      m_len = pp < n_all ? a.len[pp] : 0u;
#pragma unroll
      for (uint32_t j = 0; j < 8; j++)
        if ((lane & 7) < 4) S[chunk_swz(4 * (8 * j + (lane >> 3)) + (lane & 3))] = d8[j];
      tail128 = dense128_tail(d8);
    } else {
      if constexpr (G > 0) fetch(tile);
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = r[j];
    }
    wave_lds_sync();
    const uint32_t p = tb + lane;
    const bool mine = p >= a.p0 && p < a.p1;
    RFrame f;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint4 v = S[chunk_swz(4 * lane + k)];
      f.w[4 * k] = v.x;
      f.w[4 * k + 1] = v.y;
      f.w[4 * k + 2] = v.z;
      f.w[4 * k + 3] = v.w;
    }
    const uint32_t in = m_in, ln = m_len, xtail = X ? m_tail : 0u;
    // wide slots: the tail sums run while the frame image stays in S; the
    // frame is read back from it afterwards instead of held in registers
    const uint32_t tbytes = G ? min(64u, n_all - tb) * slot : 0u;
    auto reread = [&]() {
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint4 v = S[chunk_swz(4 * lane + k)];
        f.w[4 * k] = v.x;
        f.w[4 * k + 1] = v.y;
        f.w[4 * k + 2] = v.z;
        f.w[4 * k + 3] = v.w;
      }
    };
    if constexpr (G > 0) {
      // ---- wide slots: one structure for lean and per-lane tiles, so the
      // tail sums (the bulk of the loads) are inlined once, with the fewest
      // values live: the issue half (hash or nat_issue) and its row gather,
      // the prefetch, the tail sums while all of those are in flight, the
      // frame read back from S, then the finish half
      uint32_t end = 64;  // where this frame's L4 sum ends (64: no tail)
      if (!D && mine && nat_reg_ok(f, ln, lim)) end = 14 + bswap16((uint16_t)(f.w[4] & 0xFFFF));
      uint32_t tail = tail128;
      const bool lean = lean_ok && __ballot(mine && nat_lan_fast_ok(a, f, in, ln, lim)) == ~0ull;
      NatPend pend{kPendDone, kNone, 0, 0};
      uint32_t rowid;
      if (lean) {
        rowid = home_bucket(flowid_hash_batched(T, f.w[8] >> 16, f.w[9] & 0xFFFF, f.u32at2(26),
                                                f.u32at2(30), in, f.w[5] >> 24),
                            a.t.bmask, a.t.mix, nat_lin(T));
      } else {
        pend = nat_issue(a, T, p, f, in, ln, mine, lim);
        rowid = pend.row;
      }
      uint4 q[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        const uint32_t rw = __shfl(rowid, 16 * j + (lane >> 2));
        q[j] = rw != kNone ? rows[4 * (size_t)rw + (lane & 3)] : make_uint4(0, 0, 0, 0);
      }
      if constexpr (!D) tail = tile_tail_sums<G, H>(g8, slot, tbytes, end);
      reread();
      wave_lds_sync();
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = q[j];
      wave_lds_sync();
      uint4 row[4];
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) row[k] = S[chunk_swz(4 * lane + k)];
      uint32_t touch = kNone, smask = 0;
      if (lean) {
        const uint32_t proto = f.w[5] >> 24;
        const uint32_t key[4] = {(f.w[8] >> 16) | ((f.w[9] & 0xFFFF) << 16), f.u32at2(26),
                                 f.u32at2(30), in | (proto << 16)};
        bool done;
        // (no walk in the lane here: it costs the wide kernels scratch)
        const uint32_t idx = bucket_match_sel(row, key, &done);
        const bool hit = done & (idx != kNone);
        if (__ballot(!hit)) {  // misses (phase B) and full home buckets (reprobes)
          const bool miss = done & !hit;
          // (the hash again, not kept across the tail sums: registers)
          const uint32_t lh = a.mkq ? flowid_hash_batched(T, key[0] & 0xFFFF, key[0] >> 16,
                                                          key[1], key[2], in, proto)
                                    : 0u;
          miss_put(miss, key, lh);
          const uint32_t k = group_reserve(cur, kCurReprobe, !done);
          if (!done) rq.ent[(size_t)rb * per_b * 64 + k] = p;
          if (!hit) log_put(a.log, p, kNone);
        }
        if (hit) {
          log_put(a.log, p, idx);
          touch = idx;
          f.set32at2(26, a.ext_ip);                     // src_addr = external_addr
          f.set16(34, (uint16_t)(a.start_port + idx));  // src_port = external port
          fast_checksums(f, proto, bswap16((uint16_t)(f.w[4] & 0xFFFF)), tail);
          f.w[0] = a.wan_macw0;
          f.w[1] = a.wan_macw1;
          f.w[2] = a.wan_macw2;
          a.out[p] = (uint16_t)a.wan;
          smask = 0xFu;  // bytes 0-47 (and the TCP checksum 50-51): the whole first 64 B
        }
      } else {
        bool m = false;
        if (mine) {
          m = nat_finish(a, T, pend, row, p, f, in, ln, touch, tail);
          touch = route_note(a, p, touch);
        }
        const bool v = touch == kReprobe;  // queue on this block's reprobe slice
        const uint32_t k = group_reserve(cur, kCurReprobe, v);
        if (v) rq.ent[(size_t)rb * per_b * 64 + k] = p;
        if (v) touch = kNone;
        smask = m ? 0xFu : 0u;  // (whole 64-byte pieces: no partial-sector writes)
      }
      bins_put(bins, cur, rb, per_b * 64, range0, p, touch);
      // the changed header chunks of the rewritten frames, four lanes per
      // frame (64 contiguous bytes), through the LDS tile
      const uint64_t m0 = __ballot(smask & 1u), m1 = __ballot(smask & 2u),
                     m2 = __ballot(smask & 4u), m3 = __ballot(smask & 8u);
      if (m0) {  // (every stored frame stores chunk 0)
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          S[chunk_swz(4 * lane + k)] =
              make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
        wave_lds_sync();
        const uint32_t part = lane & 3;
        const uint64_t pm = part == 0 ? m0 : part == 1 ? m1 : part == 2 ? m2 : m3;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
          const uint32_t c = 64 * j + lane;
          if ((pm >> (c >> 2)) & 1ull) tile_st_at(g8, 64 * slot, chunk_at(c), S[chunk_swz(c)]);
        }
      }
      wave_lds_sync();  // the next tile overwrites S
      continue;
    }
    uint4 row[4];
    uint32_t touch = kNone;
    bool store_all;
    if (lean_ok && __ballot(mine && nat_lan_fast_ok(a, f, in, ln, lim64)) == ~0ull) {
      // ---- lean tile: every lane a fast-path LAN packet
      const uint32_t proto = f.w[5] >> 24;
      const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
      const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
      // the hash and the row and next-tile requests at a raised wave
      // priority: the SIMD issues them ahead of other waves' rewrite and
      // checksum arithmetic, which keeps more requests in flight (PR;
      // 64-byte slots 0.4-0.6 % faster, 128-byte slots no change: r04ah/ai)
      if constexpr (PR) __builtin_amdgcn_s_setprio(1);
      const uint32_t lh = flowid_hash_batched(T, sp, dp, sip, dip, in, proto);
      const uint32_t b = home_bucket(lh, a.t.bmask, a.t.mix, nat_lin(T));
      // lane L fetches part L % 4 of the row of packet 16 j + L / 4: the four
      // row numbers come in by ds_bpermute, issued together and waited for
      // once; named registers (an array here stays in scratch memory)
      uint32_t b0, b1, b2, b3;
      const uint32_t src = lane & ~3u;  // byte address of lane L / 4
      asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(b0) : "v"(src), "v"(b));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:64" : "=v"(b1) : "v"(src), "v"(b));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:128" : "=v"(b2) : "v"(src), "v"(b));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:192" : "=v"(b3) : "v"(src), "v"(b));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
      const uint32_t part = lane & 3;
      const uint4 q0 = rows[4 * (size_t)b0 + part];
      const uint4 q1 = rows[4 * (size_t)b1 + part];
      const uint4 q2 = rows[4 * (size_t)b2 + part];
      const uint4 q3 = rows[4 * (size_t)b3 + part];
      if (tile + tstep < tend) fetch(tile + tstep);
      if constexpr (PR) __builtin_amdgcn_s_setprio(0);
      wave_lds_sync();
      S[chunk_swz(lane)] = q0;
      S[chunk_swz(64 + lane)] = q1;
      S[chunk_swz(128 + lane)] = q2;
      S[chunk_swz(192 + lane)] = q3;
      wave_lds_sync();
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) row[k] = S[chunk_swz(4 * lane + k)];
      const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
      bool done;
      const uint32_t idx = lean_walk(a, rows, b, key, bucket_match_sel(row, key, &done), &done);
      const bool hit = done & (idx != kNone);
      if (__ballot(!hit)) {  // misses (phase B) and longer walks (reprobes)
        const bool miss = done & !hit;
        miss_put(miss, key, lh);
        const uint32_t k = group_reserve(cur, kCurReprobe, !done);
        if (!done) rq.ent[(size_t)rb * per_b * 64 + k] = p;
        if (!hit) log_put(a.log, p, kNone);
      }
      if (hit) {
        log_put(a.log, p, idx);
        touch = idx;
        f.set32at2(26, a.ext_ip);                     // src_addr = external_addr
        f.set16(34, (uint16_t)(a.start_port + idx));  // src_port = external port
        fast_checksums(f, proto, bswap16((uint16_t)(f.w[4] & 0xFFFF)), xtail);
        f.w[0] = a.wan_macw0;
        f.w[1] = a.wan_macw1;
        f.w[2] = a.wan_macw2;
        a.out[p] = (uint16_t)a.wan;
      }
      store_all = true;
    } else if (lean_own && __ballot(mine && nat_lan_fast_ok(a, f, in, ln)) == ~0ull) {
      // ---- owner mode, pass 1, every lane a fast-path LAN packet: keys
      // another rank owns leave for their owner (nat_route); this rank's are
      // looked up as in the lean tile above and their frames rewritten
      const uint32_t proto = f.w[5] >> 24;
      const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
      const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
      const uint32_t h = flowid_hash_batched(T, sp, dp, sip, dip, in, proto);
      const uint32_t o = owner_of(h, a.own.n);
      const bool routed = o != a.own.r || a.own.all;
      const uint32_t b = routed ? kNone : home_bucket(h, a.t.bmask, a.t.mix, nat_lin(T));
      uint32_t b0, b1, b2, b3;
      const uint32_t src = lane & ~3u;  // byte address of lane L / 4
      asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(b0) : "v"(src), "v"(b));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:64" : "=v"(b1) : "v"(src), "v"(b));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:128" : "=v"(b2) : "v"(src), "v"(b));
      asm volatile("ds_bpermute_b32 %0, %1, %2 offset:192" : "=v"(b3) : "v"(src), "v"(b));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
      // a routed packet's lanes read bucket 0 (an L1 hit) and ignore it: a
      // conditional load here became a load through a selected address
      // (flat, with a zero row in scratch memory)
      const uint32_t part = lane & 3;
      const uint4 q0 = rows[4 * (size_t)(b0 != kNone ? b0 : 0u) + part];
      const uint4 q1 = rows[4 * (size_t)(b1 != kNone ? b1 : 0u) + part];
      const uint4 q2 = rows[4 * (size_t)(b2 != kNone ? b2 : 0u) + part];
      const uint4 q3 = rows[4 * (size_t)(b3 != kNone ? b3 : 0u) + part];
      if (tile + tstep < tend) fetch(tile + tstep);
      wave_lds_sync();
      S[chunk_swz(lane)] = q0;
      S[chunk_swz(64 + lane)] = q1;
      S[chunk_swz(128 + lane)] = q2;
      S[chunk_swz(192 + lane)] = q3;
      wave_lds_sync();
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) row[k] = S[chunk_swz(4 * lane + k)];
      const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
      bool m = false;
      uint32_t t1 = kRouted;
      if (routed) {
        nat_route(a, p, h, key);
      } else {
        bool done;
        const uint32_t idx = bucket_match_sel(row, key, &done);
        t1 = !done ? kReprobe : idx;  // kNone: a new flow, phase B
        miss_put(done & (idx == kNone), key, h);
        if (done & (idx != kNone)) {
          f.set32at2(26, a.ext_ip);                     // src_addr = external_addr
          f.set16(34, (uint16_t)(a.start_port + idx));  // src_port = external port
          fast_checksums(f, proto, bswap16((uint16_t)(f.w[4] & 0xFFFF)));
          f.w[0] = a.wan_macw0;
          f.w[1] = a.wan_macw1;
          f.w[2] = a.wan_macw2;
          a.out[p] = (uint16_t)a.wan;
          m = true;
        }
      }
      // (the touch log is off in owner pass 1 when pass 2 bins; an unaligned
      // segment folds the log: every packet's entry, pass 2 writes the routed)
      log_put(a.log, p, t1 == kRouted || t1 == kReprobe ? kNone : t1);
      touch = route_note(a, p, t1);
      {  // queue on this block's reprobe slice
        const bool v = touch == kReprobe;
        const uint32_t k = group_reserve(cur, kCurReprobe, v);
        if (v) rq.ent[(size_t)rb * per_b * 64 + k] = p;
      }
      touch = kNone;
      // the rewritten frames only (pass 2 rewrites the routed ones), whole slots
      store_all = false;
      const uint64_t mm = __ballot(m);
      if (mm) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          S[chunk_swz(4 * lane + k)] =
              make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
        wave_lds_sync();
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
          const uint32_t c = 64 * j + lane;
          if ((mm >> (c >> 2)) & 1ull) tile_st(g, c, S[chunk_swz(c)]);
        }
      }
      wave_lds_sync();  // the next tile overwrites S
    } else {
      // ---- per-lane tile (nat_issue / nat_finish)
      const NatPend pend = nat_issue(a, T, p, f, in, ln, mine, lim64);
      uint4 q[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        const uint32_t rw = __shfl(pend.row, 16 * j + (lane >> 2));
        q[j] = rw != kNone ? rows[4 * (size_t)rw + (lane & 3)] : make_uint4(0, 0, 0, 0);
      }
      if (tile + tstep < tend) fetch(tile + tstep);
      wave_lds_sync();
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = q[j];
      wave_lds_sync();
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) row[k] = S[chunk_swz(4 * lane + k)];
      bool m = false;
      if (mine) {
        m = nat_finish(a, T, pend, row, p, f, in, ln, touch, xtail);
        touch = route_note(a, p, touch);
      }
      {  // queue on this block's reprobe slice
        const bool v = touch == kReprobe;
        const uint32_t k = group_reserve(cur, kCurReprobe, v);
        if (v) rq.ent[(size_t)rb * per_b * 64 + k] = p;
      }
      if (touch == kReprobe) touch = kNone;
      // a rewrite touches bytes 0-47; the TCP checksum (bytes 50-51) also
      // dirties chunk 3: whole tiles are stored only when every lane rewrote
      store_all = __ballot(m) == ~0ull;
      if (!store_all) {
        const uint64_t mm = __ballot(m);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          S[chunk_swz(4 * lane + k)] =
              make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
        wave_lds_sync();
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
          const uint32_t c = 64 * j + lane;
          if ((mm >> (c >> 2)) & 1ull) tile_st(g, c, S[chunk_swz(c)]);
        }
        wave_lds_sync();  // the next tile overwrites S
      }
    }
    if (staged)
      bins_put_staged(bins, bst, cur, rb, per_b * 64, range0, p, touch, &nruns);
    else
      bins_put(bins, cur, rb, per_b * 64, range0, p, touch, &nruns);
    if (store_all) {
#pragma unroll
      for (uint32_t k = 0; k < 4; k++)
        S[chunk_swz(4 * lane + k)] =
            make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
      wave_lds_sync();
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) tile_st(g, 64 * j + lane, S[chunk_swz(64 * j + lane)]);
      wave_lds_sync();  // the next tile overwrites S
    }
  }
  __syncthreads();
  if (staged) bins_flush_staged(bins, bst, cur, rb);
  if (threadIdx.x == 0 && nruns) atomicAdd(&a.t.ctl->run_tiles, nruns);
  bins_publish(bins, cur, rb);
  if (rq.ent && threadIdx.x == 0) {
    const uint32_t c = cur[kCurReprobe];
    rq.cnt[rb] = c;
    if (c) atomicAdd(rq.total, c);
  }
  if (a.mq) {  // the block's lean-tile misses onto the phase-B list (one atomic)
    const uint32_t c = cur[kCurMiss];
    if (threadIdx.x == 0 && c) mbase = atomicAdd(&a.t.ctl->miss_count, c);
    __syncthreads();
    const size_t s0 = (size_t)rb * per_b * 64;
    // (unsorted phase B: the slots themselves, kMissSlice, their keys stay)
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x)
      a.miss[mbase + i] = a.mkq ? (uint32_t)(s0 + i) | kMissSlice : a.mq[s0 + i];
  }
  route_publish(a, cur + kCurDest, rb);
  tile_publish(a);
}

__global__ __launch_bounds__(256, 4) void nat_classify64(NatArgs a, uint32_t n_all,
                                                        TouchBins bins, TileQueue rq) {
  nat_tiles<0>(a, n_all, bins, rq);
}
// One 1024-thread block per CU (the default, nat_block_waves); the ws
// variant stages its bin entries in LDS (traffic without runs: the host
// picks it when the last segment's tiles were mostly not runs, since its
// extra registers cost round robin 2.5 %)
__global__ __launch_bounds__(1024, 1) void nat_classify64w(NatArgs a, uint32_t n_all,
                                                          TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, false, true, 16, false, false>(a, n_all, bins, rq);
}
__global__ __launch_bounds__(1024, 1) void nat_classify64ws(NatArgs a, uint32_t n_all,
                                                           TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, false, true, 16, true, false>(a, n_all, bins, rq);
}
// Two 512-thread blocks per CU (VIGPATH_TILE_WAVES=8, for A/B): between the
// 256-thread shape's faster bare pass and the 1024-thread kernel
__global__ __launch_bounds__(512, 4) void nat_classify64h(NatArgs a, uint32_t n_all,
                                                         TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, false, true, 8, false, false>(a, n_all, bins, rq);
}
// Four 256-thread blocks per CU with the owner paths compiled out
// (VIGPATH_TILE_WAVES=4, for A/B; nat_classify64 keeps them)
__global__ __launch_bounds__(256, 4) void nat_classify64q(NatArgs a, uint32_t n_all,
                                                         TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, false, true, 4, false, false>(a, n_all, bins, rq);
}
// owner mode's pass 1 on the 1024-thread tile (nat_phase_a_owner)
__global__ __launch_bounds__(1024, 1) void nat_classify64wo(NatArgs a, uint32_t n_all,
                                                           TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, false, true, 16>(a, n_all, bins, rq);
}
// (diagnostics, VIGPATH_PRIO=0: the lean tile without the raised priority)
__global__ __launch_bounds__(256, 4) void nat_classify64_p0(NatArgs a, uint32_t n_all,
                                                           TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, false, false>(a, n_all, bins, rq);
}

// 64-byte header slots of longer host frames (vp_process_mbufs, vp_mbuf.hip):
// the 64-byte tile loop with the L4 sum's rest of every frame from a.tail.
__global__ __launch_bounds__(256, 4) void nat_classify64x(NatArgs a, uint32_t n_all,
                                                         TouchBins bins, TileQueue rq) {
  nat_tiles<0, 1, false, true>(a, n_all, bins, rq);
}

// Wide slots (slot > 64): G lanes per frame in the tail sums.
// Up to 8 tail chunks per lane and tile (slots <= 192 B): 4 waves per SIMD,
// 8 loads in flight per wave. Longer tails (G = 16): 2 waves per SIMD with
// 16 loads in flight each (measured 3 % faster at 1518-byte frames and 1.4 %
// at 508: r03d; more waves with 8 loads each spill registers).
template <uint32_t G>
__global__ __launch_bounds__(256, G == 16 ? 2 : 4) void nat_classify_wide(
    NatArgs a, uint32_t n_all, TouchBins bins, TileQueue rq) {
  nat_tiles<G, G == 16 ? 2 : 1>(a, n_all, bins, rq);
}

// 128-byte slots (124-byte frames and the like): the dense tile (nat_tiles
// D), one round trip for all of a tile's bytes.
__global__ __launch_bounds__(256, 4) void nat_classify128(NatArgs a, uint32_t n_all,
                                                         TouchBins bins, TileQueue rq) {
  nat_tiles<4, 1, true>(a, n_all, bins, rq);
}

// The classify kernel for a slot: 64 bytes, or the wide kernel whose G is the
// tail's 16-byte chunks (slot - 64) / 16 rounded up to a power of two, at most 16.
typedef void (*NatTileKernel)(NatArgs, uint32_t, TouchBins, TileQueue);
// Waves per block of the 64-byte classify: 16 (one 1024-thread block per
// CU, nat_classify64w) unless VIGPATH_BLOCK_WAVES=4 (four 256-thread blocks,
// nat_classify64, for A/B). A block's range is then four times longer, so
// the chip keeps a quarter of the partly written bin-slice lines, and its
// LDS has room to stage whole bin lines (nat_classify64ws): uniform order
// 0.800 -> 0.678 ms per step, round robin 0.464-0.469 -> 0.461 with eight
// run words per block and bin.
static uint32_t nat_block_waves() {
  static const uint32_t w = [] {
    const char *e = getenv("VIGPATH_BLOCK_WAVES");
    return e && atoi(e) == 4 ? 4u : 16u;
  }();
  return w;
}

static uint32_t nat_tile_waves_env() {
  static const uint32_t w = [] {
    const char *e = getenv("VIGPATH_TILE_WAVES");
    const int v = e ? atoi(e) : 16;
    return v == 8 || v == 4 ? (uint32_t)v : 16u;
  }();
  return w;
}

static const char *nat_tile_kernel_name(NatTileKernel k) {
  return k == nat_classify64w    ? "nat_classify64w"
         : k == nat_classify64h  ? "nat_classify64h"
         : k == nat_classify64q  ? "nat_classify64q"
         : k == nat_classify64ws ? "nat_classify64ws"
         : k == nat_classify64   ? "nat_classify64"
         : k == nat_classify64x  ? "nat_classify64x"
         : k == nat_classify64_p0 ? "nat_classify64_p0"
         : k == nat_classify128  ? "nat_classify128"
                                 : "nat_classify_wide";
}

static uint32_t nat_tile_waves(NatTileKernel k) {
  return k == nat_classify64w || k == nat_classify64ws ? 16u : k == nat_classify64h ? 8u : 4u;  // (64q: 4)
}

static NatTileKernel nat_tile_kernel(uint32_t slot, bool hdr_tail = false,
                                     bool staged = false) {
  static const bool p0 = [] {
    const char *e = getenv("VIGPATH_PRIO");
    return e && atoi(e) == 0;
  }();
  if (slot == 64 && !hdr_tail && nat_block_waves() == 16)
    return staged ? nat_classify64ws
           : nat_tile_waves_env() == 8 ? nat_classify64h
           : nat_tile_waves_env() == 4 ? nat_classify64q
                                       : nat_classify64w;
  if (slot == 64) return hdr_tail ? nat_classify64x : p0 ? nat_classify64_p0 : nat_classify64;
  if (slot == 128) return nat_classify128;
  const uint32_t nch = (slot - 64) / 16;
  if (nch <= 1) return nat_classify_wide<1>;
  if (nch <= 2) return nat_classify_wide<2>;
  if (nch <= 4) return nat_classify_wide<4>;
  if (nch <= 8) return nat_classify_wide<8>;
  return nat_classify_wide<16>;
}

// ------------------------------------------------------------- phase B --

// The first 64 bytes of slot p as a register frame (slots that are a
// multiple of 16 bytes, at least 64: every coalesced slot size).
__device__ __forceinline__ bool nat_slot_regs(const NatArgs &a, uint32_t p, RFrame &f) {
  if (a.slot < 64 || (a.slot & 15)) return false;
  const uint4 *fp = reinterpret_cast<const uint4 *>(a.frames + (size_t)p * a.slot);
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint4 v = fp[k];
    f.w[4 * k] = v.x;
    f.w[4 * k + 1] = v.y;
    f.w[4 * k + 2] = v.z;
    f.w[4 * k + 3] = v.w;
  }
  return true;
}

// The first 64 bytes of the 64-byte slots of the wave's lanes' packets
// (p == kNone: zeros), four lanes per frame, so each load instruction reads
// 16 frames of 64 contiguous bytes instead of 64 scattered 16-byte pieces;
// the wave's LDS tile S hands each lane its frame (the tiles' layout, chunk
// c = part c % 4 of the frame of lane c / 4). Wave-uniform call.
__device__ __forceinline__ void gather_slots64(const uint8_t *frames, uint32_t p, uint4 *S,
                                               RFrame &f) {
  const uint32_t lane = threadIdx.x & 63;
  uint4 q[4];
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t ps = (uint32_t)__shfl((int)p, (int)(16 * j + (lane >> 2)));
    q[j] = ps != kNone ? reinterpret_cast<const uint4 *>(frames + (size_t)ps * 64)[lane & 3]
                       : make_uint4(0, 0, 0, 0);
  }
  wave_lds_sync();
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) S[chunk_swz(64 * j + lane)] = q[j];
  wave_lds_sync();
#pragma unroll
  for (uint32_t k = 0; k < 4; k++) {
    const uint4 v = S[chunk_swz(4 * lane + k)];
    f.w[4 * k] = v.x;
    f.w[4 * k + 1] = v.y;
    f.w[4 * k + 2] = v.z;
    f.w[4 * k + 3] = v.w;
  }
}
// ... and back: the frames of the lanes with `st` stored whole, four lanes
// per frame (wave-uniform call).
__device__ __forceinline__ void scatter_slots64(uint8_t *frames, uint32_t p, bool st, uint4 *S,
                                                const RFrame &f) {
  const uint32_t lane = threadIdx.x & 63;
  wave_lds_sync();
#pragma unroll
  for (uint32_t k = 0; k < 4; k++)
    S[chunk_swz(4 * lane + k)] =
        make_uint4(f.w[4 * k], f.w[4 * k + 1], f.w[4 * k + 2], f.w[4 * k + 3]);
  wave_lds_sync();
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const uint32_t src = 16 * j + (lane >> 2);
    const uint32_t ps = (uint32_t)__shfl((int)p, (int)src);
    const bool ok = __shfl((int)st, (int)src) != 0;
    if (ok) reinterpret_cast<uint4 *>(frames + (size_t)ps * 64)[lane & 3] = S[chunk_swz(64 * j + lane)];
  }
  wave_lds_sync();
}

// FlowId keys and hashes of the queued misses (frames still unmodified):
// register frames with the tile kernels' field reads and the batched hash
// from the LDS tables, the generic byte path for any other frame.
__global__ __launch_bounds__(256) void nat_miss_keys(NatArgs a, const uint32_t *list,
                                                     uint32_t n, uint32_t *mkey,
                                                     uint32_t *mhash) {
  __shared__ uint32_t T[kNatTabWords];
  __shared__ uint4 stage[4][256];
  load_nat_tables(T, a);
  uint4 *S = stage[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63;
  // (the loop is wave-uniform: the 64-byte-slot gather is cooperative)
  for (uint32_t j0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); j0 < n;
       j0 += gridDim.x * blockDim.x) {
    const uint32_t j = j0 + lane;
    const bool v = j < n;
    const uint32_t p = v ? list[j] : kNone;
    const uint32_t in = v ? port_of(a.in_dev, a.in0, p) : 0u, len = v ? a.len[p] : 0u;
    RFrame r;
    bool reg;
    if (a.slot == 64) {
      gather_slots64(a.frames, p, S, r);
      reg = true;
    } else {
      reg = v && nat_slot_regs(a, p, r);
    }
    if (!v) continue;
    uint32_t proto, sp, dp, sip, dip;
    if (reg && nat_reg_ok(r, len, 0xFFFFu)) {
      proto = r.w[5] >> 24;
      sp = r.w[8] >> 16;
      dp = r.w[9] & 0xFFFF;
      sip = r.u32at2(26);
      dip = r.u32at2(30);
    } else {
      GFrame f{a.frames + (size_t)p * a.slot, a.slot};
      const L34 h = parse_l34(f, len);
      proto = f.r8(h.ip + 9);
      sp = f.r16(h.l4);
      dp = f.r16(h.l4 + 2);
      sip = f.r32(h.ip + 12);
      dip = f.r32(h.ip + 16);
    }
    reinterpret_cast<uint4 *>(mkey)[j] = make_uint4(sp | (dp << 16), sip, dip, in | (proto << 16));
    mhash[j] = flowid_hash_batched(T, sp, dp, sip, dip, in, proto);
  }
}

// LAN rewrite of a packet whose flow index is known (generic byte path).
__device__ void nat_write_lan(const NatArgs &a, uint32_t p, uint32_t idx) {
  GFrame f{a.frames + (size_t)p * a.slot, a.slot};
  const L34 h = parse_l34(f, a.len[p]);
  f.w32(h.ip + 12, a.ext_ip);
  f.w16(h.l4, (uint16_t)(a.start_port + idx));
  set_checksums(f, h.ip, h.l4, nat_tail(a, p));
  const uint32_t mw[3] = {a.wan_macw0, a.wan_macw1, a.wan_macw2};
  set_macs(f, mw);
  a.out[p] = a.wan;
}

// Every miss: the index its first sighting got (or drop: table full). A
// register-path frame of a 64-byte slot is rewritten as the tile kernels
// rewrite a hit (gathered and stored four lanes per frame); any other takes
// the byte path.
// (nkord: tbl_new_keys_unsorted's key set, whose slot word carries the
// index; then no touch-log entries: the set stamped the new flows itself)
__global__ __launch_bounds__(256) void nat_miss_finish(NatArgs a, const uint32_t *list,
                                                       uint32_t n, const uint32_t *scratch,
                                                       const uint32_t *rep,
                                                       const uint32_t *assign,
                                                       const unsigned long long *nkord) {
  __shared__ uint4 stage[4][256];
  uint4 *S = stage[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63;
  // (the loop is wave-uniform: the 64-byte-slot gather and store are
  // cooperative)
  for (uint32_t j0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); j0 < n;
       j0 += gridDim.x * blockDim.x) {
    const uint32_t j = j0 + lane;
    const bool v = j < n;
    uint32_t p = v ? list[j] : kNone;
    if (v && nkord && (p & kMissSlice)) p = a.mq[p & ~kMissSlice];  // (a lean tile's slot)
    const uint32_t idx = !v ? kNone : nkord ? (uint32_t)nkord[rep[j]] : assign[scratch[rep[j]]];
    if (v) {
      if (!nkord) a.log[p] = idx;
      if (idx == kNone) a.out[p] = port_of(a.in_dev, a.in0, p);  // nat_main.c:87-91
    }
    const bool live = v && idx != kNone;
    bool fast = false;
    if (a.slot == 64) {
      RFrame f;
      gather_slots64(a.frames, live ? p : kNone, S, f);
      fast = live && nat_lan_fast_ok(a, f, port_of(a.in_dev, a.in0, p), a.len[p], nat_lim64(a));
      if (fast) {
        const uint32_t proto = f.w[5] >> 24;
        f.set32at2(26, a.ext_ip);                     // src_addr = external_addr
        f.set16(34, (uint16_t)(a.start_port + idx));  // src_port = external port
        fast_checksums(f, proto, bswap16((uint16_t)(f.w[4] & 0xFFFF)), nat_tail(a, p));
        f.w[0] = a.wan_macw0;
        f.w[1] = a.wan_macw1;
        f.w[2] = a.wan_macw2;
        a.out[p] = a.wan;
      }
      scatter_slots64(a.frames, p, fast, S, f);
    }
    if (live && !fast) nat_write_lan(a, p, idx);
  }
}

// LAN packets whose home bucket held three other keys finish here: phase A's
// register path with the probe walked on bucket by bucket (reprobe_wave, one
// cooperative 64-byte request per frame and per bucket). Slices per classify
// block (cnt, 64-byte tiles) or runs of 256 of one list (cnt == null, the
// per-lane classify path).
__global__ __launch_bounds__(256) void nat_reprobe(NatArgs a, const uint32_t *list,
                                                   const uint32_t *cnt, uint32_t n,
                                                   uint32_t range, uint32_t nblk,
                                                   uint64_t seq_base) {
  __shared__ uint32_t T[kNatTabWords];
  __shared__ uint4 stage[4][256];
  load_nat_tables(T, a);
  a.tileq = 1;  // a full bucket answers kReprobe: reprobe_wave walks on
  uint4 *S = stage[threadIdx.x >> 6];
  reprobe_slices(list, cnt, n, range, nblk, a.t.tseq, seq_base, [&](uint32_t p, bool act) {
    return reprobe_wave(
        a.frames, a.slot, a.len, a.in_dev, reinterpret_cast<const uint8_t *>(a.t.bk),
        a.t.bmask, p, act, S,
        [&](uint32_t q, const RFrame &f, uint32_t in, uint32_t len, bool mine) {
          return nat_issue(a, T, q, f, in, len, mine, nat_lim64(a));
        },
        [&](const NatPend &P, const uint4 *row, uint32_t q, RFrame &f, uint32_t in,
            uint32_t len, uint32_t &touch) {
          return nat_finish(a, T, P, row, q, f, in, len, touch, nat_tail(a, q));
        },
        a.in0);
  });
}

// ------------------------------------------------------- owner mode --
//  Pass 1 leaves each block's keys per owner rank in the
// padded send buffer, owner o's chunk [o cap, (o + 1) cap) cut into one
// slice of `sub` keys per block (keys past a slice in desc). route_counts
// gives the owners their per-block counts (exchanged beside the keys) and
// flags a slice that overflowed; the keys go to their owners (all-to-all),
// nat_own_probe answers them against the owner's buckets, the answers come
// back in the same slots, and pass 2 finishes the packets. After an overflow
// (any rank) the exact exchange packs every slice tight: route_scan +
// route_base give the slices their offsets, route_pack gathers them.

// The slice counts travel as one row per owner: [blocks, sub, count of
// block 0, 1, ...] (ranks may run different pass-1 grids for one segment).
constexpr uint32_t kSliceRowMax = 4096;  // pass-1 blocks
constexpr uint32_t kSliceRow = 2 + kSliceRowMax;

// Per owner o (one block each): row o = [nblk, sub, block b's keys for o (at
// most sub) ...], need[o] = the largest slice times the blocks (the chunk
// size that would have held it: the next batch's capacity), *ovf when a
// slice overflowed.
__global__ __launch_bounds__(256) void route_counts(const uint32_t *dcnt, uint32_t nblk,
                                                    uint32_t n, uint32_t sub, uint32_t *rows,
                                                    uint32_t *need, uint64_t *ovf) {
  __shared__ uint32_t mx[256];
  const uint32_t o = blockIdx.x;
  uint32_t *row = rows + (size_t)o * kSliceRow;
  uint32_t m = 0;
  for (uint32_t b = threadIdx.x; b < nblk; b += blockDim.x) {
    const uint32_t v = dcnt[(size_t)b * n + o];
    m = max(m, v);
    row[2 + b] = min(v, sub);
  }
  if (threadIdx.x == 0) {
    row[0] = nblk;
    row[1] = sub;
  }
  mx[threadIdx.x] = m;
  __syncthreads();
  for (uint32_t h = 128; h; h >>= 1) {
    if (threadIdx.x < h) mx[threadIdx.x] = max(mx[threadIdx.x], mx[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    need[o] = mx[0] * nblk;
    if (mx[0] > sub) *ovf = 1;
  }
}

// Exact exchange, per owner o (one block each): exclusive scan over blocks of
// dcnt[.][o], offsets inside the owner's chunk (route_base adds the chunk's
// start), dtot[o] the owner's total.
__global__ __launch_bounds__(256) void route_scan(const uint32_t *dcnt, uint32_t nblk,
                                                  uint32_t n, uint32_t *dbase,
                                                  uint32_t *dtot) {
  __shared__ uint32_t part[256];
  const uint32_t o = blockIdx.x;
  const uint32_t per = (nblk + 255) / 256;
  const uint32_t b0 = threadIdx.x * per, b1 = min(nblk, b0 + per);
  uint32_t sum = 0;
  for (uint32_t b = b0; b < b1; b++) sum += dcnt[(size_t)b * n + o];
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < 256; i++) {
      const uint32_t v = part[i];
      part[i] = acc;
      acc += v;
    }
    dtot[o] = acc;
  }
  __syncthreads();
  uint32_t acc = part[threadIdx.x];
  for (uint32_t b = b0; b < b1; b++) {
    dbase[(size_t)b * n + o] = acc;
    acc += dcnt[(size_t)b * n + o];
  }
}

// Owner o's chunk starts after the chunks of owners < o.
__global__ void route_base(uint32_t *dbase, const uint32_t *dtot, uint32_t nblk,
                           uint32_t n) {
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < nblk * n;
       x += gridDim.x * blockDim.x) {
    const uint32_t o = x % n;
    uint32_t start = 0;
    for (uint32_t q = 0; q < o; q++) start += dtot[q];
    dbase[x] += start;
  }
}

// Exact exchange: one block per source block, its slices packed tight into
// `out` (a slice's first `sub` keys from its padded slot, the rest from desc).
__global__ __launch_bounds__(256) void route_pack(const uint4 *desc, const uint4 *padded,
                                                  const uint32_t *dcnt, const uint32_t *dbase,
                                                  uint32_t n, uint32_t range, uint32_t cap,
                                                  uint32_t sub, uint4 *out) {
  const uint32_t b = blockIdx.x;
  for (uint32_t o = 0; o < n; o++) {
    const uint32_t cnt = dcnt[(size_t)b * n + o];
    const uint32_t base = dbase[(size_t)b * n + o];
    const uint4 *src = desc + ((size_t)b * n + o) * range;
    const uint4 *pad = padded + (size_t)o * cap + (size_t)b * sub;
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x)
      out[base + k] = k < sub ? pad[k] : src[k];
  }
}

// Leftover exchange (the chunked pipeline, after a slice overflowed): per
// (virtual block, owner) the keys past the slice's `sub`, and those keys
// packed tight from desc (route_scan / route_base give the offsets).
__global__ void route_left(const uint32_t *dcnt, uint32_t m, uint32_t sub, uint32_t *lcnt) {
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < m; x += gridDim.x * blockDim.x)
    lcnt[x] = dcnt[x] > sub ? dcnt[x] - sub : 0u;
}
__global__ __launch_bounds__(256) void route_pack_left(const uint4 *desc, const uint32_t *dcnt,
                                                       const uint32_t *dbase, uint32_t n,
                                                       uint32_t range, uint32_t sub,
                                                       uint4 *out) {
  const uint32_t b = blockIdx.x;
  for (uint32_t o = 0; o < n; o++) {
    const uint32_t cnt = dcnt[(size_t)b * n + o];
    const uint32_t base = dbase[(size_t)b * n + o];
    const uint4 *src = desc + ((size_t)b * n + o) * range;
    for (uint32_t k = sub + threadIdx.x; k < cnt; k += blockDim.x) out[base + k - sub] = src[k];
  }
}

// The owner side of C1: map_get (find_key, map-impl-pow2.c:629-732) of every
// received FlowId in this rank's buckets. Tiles of 64 keys per wave (one
// 1 KiB load; the next tile's keys in flight while this one is matched), a
// persistent grid with a contiguous tile range per block (keys arrive in
// their senders' packet order, so a block's keys reuse nearby rows, as in
// nat_tiles), the hash from the LDS position tables with the 15 reads issued
// together (flowid_hash_batched), the home bucket through the layout's
// tables in LDS, one cooperative 64-byte row request per key
// (wave_gather64) and the branch-free match; a key whose home bucket holds
// three other keys walks on bucket by bucket (rare). Answers the index or
// kNone (a new flow: the ingest rank queues the packet for phase B).
// Padded exchange (cap > 0): n keys arrived as ranks x cap, peer q's chunk
// one slice per block of its pass 1, the first rcnt row q's count of each
// slice valid (route_counts); no work when any rank overflowed (*ovf, published as
// ctl->route_ovf for the host). This rank's own keys (q == self) are read
// where pass 1 wrote them (`own_keys`, the send buffer, same layout) and
// answered in place (`own_reply`, the answers' receive buffer): the
// exchanges skip the rank's own chunk. cap == 0: n keys, all valid.
__global__ __launch_bounds__(256, 4) void nat_own_probe(TableDev t, const uint32_t *crc_tab,
                                                        const uint4 *keys, uint32_t n,
                                                        uint32_t cap, const uint32_t *rcnt,
                                                        const uint64_t *ovf, Ctl *ctl,
                                                        uint32_t *reply, uint32_t self,
                                                        const uint4 *own_keys,
                                                        uint32_t *own_reply) {
  __shared__ uint32_t T[kNatTabWords];
  __shared__ uint4 stage[4][256];
  // (sentinel slices, the chunked pipeline: rcnt and ovf null; the rank's
  // own flag is pass 1's)
  const bool skip = cap && ovf && *ovf;
  if (ovf && blockIdx.x == 0 && threadIdx.x == 0) ctl->route_ovf = skip ? 1u : 0u;
  if (skip) return;
  if (t.mix == kMixLin)
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[kCrcWords + i] = t.lin[i];
  load_crc_tables(T, crc_tab);  // (its barrier covers the layout tables)
  uint4 *S = stage[threadIdx.x >> 6];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tiles = (n + 63) / 64;
  const uint32_t per_b = (tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t tend = min(tiles, blockIdx.x * per_b + per_b);
  // key j of the padded exchange: peer q = j / cap, its pass-1 block b's
  // slice (peer q's row of slice counts: [blocks, sub, counts]), slot k;
  // valid when k < that slice's count
  auto valid_at = [&](uint32_t j) {
    if (j >= n) return false;
    if (!cap) return true;
    const uint32_t q = j / cap, l = j - q * cap;
    const uint32_t *row = rcnt + (size_t)q * kSliceRow;
    const uint32_t sub = row[1], b = l / sub;
    return b < row[0] && l - b * sub < row[2 + b];
  };
  auto own = [&](uint32_t j) { return cap && j / cap == self; };
  // Software-pipelined over the wave's tiles: in the iteration for tile t
  // the keys of tile t + 2 are loaded, tile t + 1 is hashed and its rows
  // requested, and tile t's rows (requested one iteration earlier) are
  // matched: two tiles' row requests in flight per wave.
  const uint4 *rows = reinterpret_cast<const uint4 *>(t.bk);
  struct Tile {
    bool act;
    uint4 k;
  };
  auto load = [&](uint32_t tl) {
    Tile x{false, make_uint4(0, 0, 0, 0)};
    if (tl < tend) {
      const uint32_t j0 = tl * 64, j = j0 + lane;
      if (cap && !rcnt) {  // sentinel slices: every slot loaded, empty ones marked
        if (j < n) {
          x.k = (own(j) ? own_keys + j : keys + j)[0];
          x.act = x.k.w != kKeySentinelW;
        }
      } else if (cap && (cap & 63) == 0) {
        // the tile's peer and slice, once per tile (scalar): with chunks and
        // slices of whole tiles a tile lies in one slice
        const uint32_t q = j0 / cap, l0 = j0 - q * cap;
        const uint32_t *row = rcnt + (size_t)q * kSliceRow;
        const uint32_t sub = row[1];
        if ((sub & 63) == 0) {
          const uint32_t b = l0 / sub, k0 = l0 - b * sub;
          const uint32_t c = b < row[0] ? row[2 + b] : 0u;
          x.act = j < n && k0 + lane < c;
        } else {
          x.act = valid_at(j);
        }
        if (x.act) x.k = (q == self ? own_keys + j : keys + j)[0];
      } else {
        x.act = valid_at(j);
        if (x.act) x.k = (own(j) ? own_keys + j : keys + j)[0];
      }
    }
    return x;
  };
  struct Rows {
    uint32_t b;
    uint4 q0, q1, q2, q3;
  };
  auto request = [&](const Tile &x) {  // hash, request the home rows
    const uint4 k = x.k;
    Rows r;
    r.b = home_bucket(flowid_hash_batched(T, k.x & 0xFFFF, k.x >> 16, k.y, k.z, k.w & 0xFFFF,
                                          (k.w >> 16) & 0xFF),
                      t.bmask, t.mix, nat_lin(T));
    const uint32_t want = x.act ? r.b : kNone;
    // lane L: part L % 4 of the row of key 16 j + L / 4
    auto part = [&](uint32_t j) {
      const uint32_t rw = (uint32_t)__shfl((int)want, (int)(16 * j + (lane >> 2)));
      return rw != kNone ? rows[4 * (size_t)rw + (lane & 3)] : make_uint4(0, 0, 0, 0);
    };
    r.q0 = part(0);
    r.q1 = part(1);
    r.q2 = part(2);
    r.q3 = part(3);
    return r;
  };
  uint32_t tile = blockIdx.x * per_b + wv;
  Tile cur = load(tile), nxt = load(tile + 4);
  const Rows zero{0, make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0),
                  make_uint4(0, 0, 0, 0)};
  Rows rc = __ballot(cur.act) ? request(cur) : zero;
  for (; tile < tend; tile += 4) {
    const Tile after = load(tile + 8);
    const Rows rn = __ballot(nxt.act) ? request(nxt) : zero;
    if (__ballot(cur.act)) {
      const uint32_t j = tile * 64 + lane;
      const uint32_t key[4] = {cur.k.x, cur.k.y, cur.k.z, cur.k.w};
      uint4 row[4];
      wave_lds_sync();  // (earlier readers of S are done)
      S[chunk_swz(lane)] = rc.q0;
      S[chunk_swz(64 + lane)] = rc.q1;
      S[chunk_swz(128 + lane)] = rc.q2;
      S[chunk_swz(192 + lane)] = rc.q3;
      wave_lds_sync();
#pragma unroll
      for (uint32_t kk = 0; kk < 4; kk++) row[kk] = S[chunk_swz(4 * lane + kk)];
      bool done;
      uint32_t res = bucket_match_sel(row, key, &done);
      bool live = cur.act && !done;
      uint32_t b = rc.b;
      for (uint32_t step = 1; __ballot(live) && step <= t.bmask; step++) {  // (rare)
        b = (b + 1) & t.bmask;
        wave_gather64(reinterpret_cast<const uint8_t *>(t.bk), 64, live ? b : kNone, S, row);
        if (live) {
          const uint32_t r2 = bucket_match(row[0], row[1], row[2], row[3], key, &done);
          if (done) {
            res = r2;
            live = false;
          }
        }
      }
      if (cur.act) (own(j) ? own_reply + j : reply + j)[0] = res;
    }
    cur = nxt;
    nxt = after;
    rc = rn;
  }
}

// LAN rewrite of a routed packet whose index came back (register frame).
__device__ __forceinline__ void nat_lan_fast(const NatArgs &a, RFrame &f, uint32_t p,
                                             uint32_t idx) {
  const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
  const uint32_t proto = f.w[5] >> 24;
  f.set32at2(26, a.ext_ip);
  f.set16(34, (uint16_t)(a.start_port + idx));
  fast_checksums(f, proto, tl);
  f.w[0] = a.wan_macw0;
  f.w[1] = a.wan_macw1;
  f.w[2] = a.wan_macw2;
  a.out[p] = a.wan;
}

// The answer for packet p's route (kRouteBit set), kNoReply (the exact
// exchange's) or kAnswered (an earlier pass 2 finished it).
__device__ __forceinline__ uint32_t route_answer(const NatArgs &a, uint32_t p,
                                                 uint32_t rt) {
  const uint32_t o = (rt >> 24) & 63, k = rt & 0xFFFFFFu;
  const uint32_t blk = (p - a.own.first) / a.own.range;
  if (a.own.mode == kOwnChunked)  // this chunk's replies; the launch's blocks
    return k < a.own.sub                                   // are its slices
               ? a.own.rreply[(size_t)o * a.own.cap + (size_t)(blk - a.vb0) * a.own.sub + k]
               : kNoReply;
  if (a.own.mode == kOwnLeftover)  // the exact exchange of the keys past their slices
    return k < a.own.sub ? kAnswered
                         : a.own.rreply[a.own.dbase[(size_t)blk * a.own.n + o] + k - a.own.sub];
  if (a.own.cap) {  // padded (no rank overflowed a slice: every k < sub)
    if (*a.own.ovf) return kNoReply;
    return a.own.rreply[(size_t)o * a.own.cap + (size_t)blk * a.own.sub + k];
  }
  return a.own.rreply[a.own.dbase[(size_t)blk * a.own.n + o] + k];
}

// Pass 2 for 64-byte slots: the same coalesced tiles as pass 1; routed
// packets are rewritten with their answer (or queued as phase-B misses) and
// every touch of the segment, pass 1's included, goes to the touch bins.
struct RemPend {
  uint32_t row;  // (no table rows: always kNone)
  uint32_t kind, idx;
};
__global__ __launch_bounds__(256, 4) void nat_remote64(NatArgs a, uint32_t n_all,
                                                      TouchBins bins) {
  __shared__ uint4 stage[4][256];
  __shared__ uint32_t cur[kCurs];
  for (uint32_t i = threadIdx.x; i < kCurs; i += blockDim.x) cur[i] = 0;
  __syncthreads();
  frames64_tiles(
      a.frames, a.len, a.in_dev, a.p0, a.p1, n_all, stage[threadIdx.x >> 6], nullptr,
      [&](uint32_t p, const RFrame &, uint32_t, uint32_t, bool mine) {
        RemPend P{kNone, 0, kNone};
        if (!mine) return P;
        const uint32_t rt = a.own.route[p];
        if (rt == kNone) return P;
        if (!(rt & kRouteBit)) {
          if (a.own.mode == kOwnLeftover) return P;  // (binned by the first pass 2)
          P.kind = 1;  // pass 1's own touch
          P.idx = rt;
        } else {
          P.idx = route_answer(a, p, rt);
          // (no reply: the exact exchange's; answered: an earlier pass 2's)
          P.kind = P.idx == kNoReply || P.idx == kAnswered ? 0 : 2;
        }
        return P;
      },
      [&](const RemPend &P, const uint4 *, uint32_t p, RFrame &f, uint32_t in,
          uint32_t len, uint32_t &touch) -> uint32_t {
        if (P.kind == 0) return 0u;
        if (P.kind == 1) {
          log_put(a.log, p, P.idx);  // (the lean pass-1 tile logs nothing)
          touch = P.idx;
          return 0u;
        }
        if (P.idx == kNone) {  // a new flow (or not yet visible): phase B
          a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
          log_put(a.log, p, kNone);
          return 0u;
        }
        log_put(a.log, p, P.idx);
        touch = P.idx;
        const uint32_t et = f.w[3] & 0xFFFF, ihl = (f.w[3] >> 16) & 0x0F;
        const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
        if (!(et == 0x0008 && ihl == 5 && tl <= 50)) {  // byte path, in place
          nat_write_lan(a, p, P.idx);
          return 0u;
        }
        nat_lan_fast(a, f, p, P.idx);
        return 0xFu;  // the whole slot: whole-line writes
      },
      bins, TileQueue{}, cur, a.vb0, a.vper);
}

// Pass 2, any slot size: routed packets only, one lane each (byte path).
__global__ void nat_remote_lane(NatArgs a) {
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += gridDim.x * blockDim.x) {
    const uint32_t rt = a.own.route[p];
    if (rt == kNone || !(rt & kRouteBit)) continue;
    const uint32_t idx = route_answer(a, p, rt);
    if (idx == kNoReply || idx == kAnswered) continue;  // the exact exchange's
    a.log[p] = idx;
    if (idx == kNone) {
      a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
      continue;
    }
    nat_write_lan(a, p, idx);
  }
}

// ------------------------------------------------------------- phase C --
__global__ void nat_defer_finish(NatArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint64_t q = a.seq_base + p;
    const uint32_t in = port_of(a.in_dev, a.in0, p);
    GFrame f{a.frames + (size_t)p * a.slot, a.slot};
    const L34 h = parse_l34(f, a.len[p]);
    const uint32_t proto = f.r8(h.ip + 9);
    const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
    const uint32_t sip = f.r32(h.ip + 12);
    const uint32_t idx = dp - a.start_port;  // range checked in phase A
    if (!tbl_allocated_before(a.t, idx, q)) {
      a.out[p] = (uint16_t)in;
      a.log[p] = kNone;
      continue;
    }
    const uint4 fk = tbl_key_of(a.t, idx);
    const uint32_t k0 = fk.x, k1 = fk.y, k2 = fk.z, k3 = fk.w;
    a.log[p] = idx;
    if ((k2 != sip) | ((k0 >> 16) != sp) | (((k3 >> 16) & 0xFF) != proto)) {
      a.out[p] = (uint16_t)in;
      continue;
    }
    f.w32(h.ip + 16, k1);
    f.w16(h.l4 + 2, (uint16_t)(k0 & 0xFFFF));
    const uint32_t dst = k3 & 0xFFFF;
    set_checksums(f, h.ip, h.l4, nat_tail(a, p));
    uint32_t mw[3];
    macs_for(a, dst, mw);
    set_macs(f, mw);
    a.out[p] = (uint16_t)dst;
  }
}

// ========================================================= one packet ==
// nf.c's per-packet loop (nf.c:150-176) calls nf_process once per packet.
// Through the batch path one packet costs a launch sequence and a host round
// trip per call (≈68 µs); vp_process_one instead hands it to
// nat_serve, one wave that stays resident and polls a host-coherent mailbox
// (ServeBox, vp_internal.h): no launch per packet. The host serves through it
// only while no expiry is due (nat_process_one), so the kernel restates
// nat_main.c:22-109 without the expiry step.

// flow_manager_get_internal / allocate_flow (nat_main.c:68-97) for one LAN
// key at global sequence seq: its index, allocated when new (*fresh = 1), and
// stamped; kNone when the table is full (drop).
__device__ __forceinline__ uint32_t one_lan(const TableDev &t, uint32_t hh, const uint32_t key[4],
                                            int64_t now, uint64_t seq, uint32_t *fresh) {
  uint32_t idx = tbl_probe(t, hh, key);
  if (idx == kNone) {  // dchain_allocate_new_index: the freed stack, then fresh
    Ctl *c = t.ctl;
    const uint32_t st = c->stack_top, fn = c->fresh_next;
    if (st) {
      idx = t.stack[st - 1];
      c->stack_top = st - 1;
    } else if (fn < t.cap) {
      idx = fn;
      c->fresh_next = fn + 1;
    } else {
      return kNone;  // nat_main.c:87-91
    }
    bool tomb = false;
    uint32_t disp = 0;
    const uint32_t e = tbl_insert(t, hh, key, idx, &tomb, &disp);
    if (tomb) c->n_tomb -= 1;
    c->n_live += 1;
    c->sh_live += 1;
    c->disp_count += disp;
    t.slot_of[idx] = e;
    t.hash_of[idx] = hh;
    t.birth[idx] = seq;
    *fresh = 1;
  }
  return idx;  // (the caller stamps it: one_stamp)
}

// The touch of index idx at (now, seq), right behind the lookup: stamped
// after the answer instead, the stores' acknowledgement held the wave from
// its next poll (4.6-4.8 against 4.3-4.4 us per packet,
// profiles/r06z_serve_stamp.txt).
__device__ __forceinline__ void one_stamp(const TableDev &t, uint32_t idx, int64_t now,
                                          uint64_t seq) {
  t.ts[idx] = (uint64_t)now;
  t.tseq[idx] = seq;
}

// flow_manager_get_external (nat_main.c:42-67) for external port dp: false
// when no flow holds it; else the flow's key in *k, stamped (rejuvenated
// before the anti-spoof check).
__device__ __forceinline__ bool one_wan(const NatArgs &a, uint32_t dp, int64_t now,
                                        uint64_t seq, uint4 *k, uint32_t *ix) {
  const TableDev &t = a.t;
  const int idx = (int)dp - (int)a.start_port;
  if (idx < 0 || idx >= (int)t.cap || t.slot_of[idx] == kNone) return false;
  *k = tbl_key_of(t, (uint32_t)idx);
  *ix = (uint32_t)idx;  // (the caller stamps it, before the anti-spoof check)
  return true;
}

// nat_main.c:30-106 for one frame, byte-addressed (f: its bytes, cap = its
// length; IP options, odd headers): returns the output port.
__device__ __forceinline__ uint32_t nat_one(const NatArgs &a, const uint32_t *T,
                                            const GFrame &f, uint32_t in, uint32_t len,
                                            int64_t now, uint64_t seq, uint32_t *fresh) {
  const L34 h = parse_l34(f, len);
  if (!h.ok) return in;  // nat_main.c:30-38
  const uint32_t proto = f.r8(h.ip + 9);
  const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
  const uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
  uint32_t dst;
  if (in == a.wan) {
    uint4 k;
    uint32_t ix;
    if (!one_wan(a, dp, now, seq, &k, &ix)) return in;
    one_stamp(a.t, ix, now, seq);
    if ((k.z != sip) | ((k.x >> 16) != sp) | (((k.w >> 16) & 0xFF) != proto)) return in;
    f.w32(h.ip + 16, k.y);
    f.w16(h.l4 + 2, (uint16_t)(k.x & 0xFFFF));
    dst = k.w & 0xFFFF;
  } else {
    const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
    const uint32_t idx = one_lan(a.t, flowid_hash(T, sp, dp, sip, dip, in, proto), key, now,
                                 seq, fresh);
    if (idx == kNone) return in;
    one_stamp(a.t, idx, now, seq);
    f.w32(h.ip + 12, a.ext_ip);
    f.w16(h.l4, (uint16_t)(a.start_port + idx));
    dst = a.wan;
  }
  set_checksums(f, h.ip, h.l4);  // (the whole frame is in f)
  uint32_t mw[3];
  macs_for(a, dst, mw);
  set_macs(f, mw);
  return dst;
}

// The same for a frame with a 20-byte IPv4 header, its first 64 bytes in
// registers (nat_issue / nat_finish's register path; `tail` = the raw sum of
// the L4 bytes past byte 64). kNone: not such a frame (nat_one takes it).
__device__ __forceinline__ uint32_t nat_one_reg(const NatArgs &a, const uint32_t *T, RFrame &f,
                                                uint32_t in, uint32_t len, uint32_t tail,
                                                int64_t now, uint64_t seq, uint32_t *fresh,
                                                bool prof, uint64_t &mk0, uint64_t &mk1) {
  const uint32_t et = f.w[3] & 0xFFFF, ihl = (f.w[3] >> 16) & 0x0F;
  if (!(et == 0x0008 && ihl == 5)) return kNone;
  const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
  const uint16_t unread = (uint16_t)(len - 14);
  const uint32_t proto = f.w[5] >> 24;
  if (!((unread >= 20) & (unread >= tl) & ((proto == 6) | (proto == 17)) &
        ((uint32_t)(len - 34) >= 4u)))
    return in;
  const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
  const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
  uint32_t dst, mw[3], ix;
  if (in == a.wan) {
    uint4 k;
    if (!one_wan(a, dp, now, seq, &k, &ix)) return in;
    one_stamp(a.t, ix, now, seq);  // (rejuvenated before the anti-spoof check)
    if ((k.z != sip) | ((k.x >> 16) != sp) | (((k.w >> 16) & 0xFF) != proto)) return in;
    f.set32at2(30, k.y);        // dst_addr = flow.src_ip
    f.set16(36, k.x & 0xFFFF);  // dst_port = flow.src_port
    dst = k.w & 0xFFFF;
  } else {
    const uint32_t key[4] = {sp | (dp << 16), sip, dip, in | (proto << 16)};
    const uint32_t hh = flowid_hash_batched(T, sp, dp, sip, dip, in, proto);
    if (prof) mk0 = wall_clock64();
    const uint32_t idx = one_lan(a.t, hh, key, now, seq, fresh);
    if (prof) mk1 = wall_clock64();
    if (idx == kNone) return in;
    one_stamp(a.t, idx, now, seq);
    f.set32at2(26, a.ext_ip);
    f.set16(34, (uint16_t)(a.start_port + idx));
    dst = a.wan;
  }
  macs_for(a, dst, mw);
  fast_checksums(f, proto, tl, tail);
  f.w[0] = mw[0];
  f.w[1] = mw[1];
  f.w[2] = mw[2];
  return dst;
}

// The server: one wave. Every poll reads the request chunks whole (ServeBox,
// vp_internal.h: one PCIe read brings the doorbell, the time and a frame of up
// to kServeInline bytes), one poll in flight per wave (VIGPATH_SERVE_WAVES
// waves poll, staggered; the first to claim a request serves it); longer frames are read from `frame` afterwards. The frame goes into LDS, the
// wave sums the L4 bytes past byte 64, lane 0 runs the packet, the frame goes
// back (16-byte system-coherent stores) and the answer word follows once
// every store has completed. Packets take global sequence numbers seq, seq +
// 1, ... It leaves on the leave request or after `idle` wall-clock ticks
// without a request; a request posted as it leaves finds the stream idle and
// the host launches it again (nat_process_one). flags: bit 0, the stage
// clock (VIGPATH_SERVE_PROF); bits 3-9: the waves' stagger in wall-clock
// ticks; bits 10-17: the first poll's delay after an answer; bit 18: adapt it;
// bits 19-23: the ticks a late poll adds to it.
__global__ __launch_bounds__(256) void nat_serve(NatArgs a, ServeBox *box, uint64_t seq0,
                                                 uint64_t idle, uint32_t flags) {
  __shared__ uint32_t T[kNatTabWords];
  __shared__ uint4 fr[kServeFrame / 16];
  __shared__ uint32_t done_s, claim_s;  // the last answered / claimed request
  __shared__ uint64_t t0_s;             // the last answer's wall clock
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    const uint32_t d = (uint32_t)__hip_atomic_load(&box->ans, __ATOMIC_ACQUIRE,
                                                   __HIP_MEMORY_SCOPE_SYSTEM);
    done_s = d;
    claim_s = d;
    t0_s = wall_clock64();
  }
  load_nat_tables(T, a);  // (its barrier covers the words above)
  const uint32_t done0 = done_s;
  const bool prof = flags & 1u;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  constexpr int kSys = 17;  // sc0 | sc1: system-coherent (bypasses the GPU caches)
  const auto ms = __builtin_amdgcn_make_buffer_rsrc(box->msg, 0, 16 * kServeChunks, 0x00020000);
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(box->frame, 0, kServeFrame, 0x00020000);
  const auto as = __builtin_amdgcn_make_buffer_rsrc(box->amsg, 0, 16 * kServeChunks, 0x00020000);
  // (lanes past the chunks read nothing: an offset past the resource)
  const int moff = lane < kServeChunks ? (int)(16 * lane) : (int)(16 * kServeChunks);
  auto poll = [&]() -> v4u { return __builtin_amdgcn_raw_buffer_load_b128(ms, moff, 0, kSys); };
  auto lds_ld = [](uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  uint32_t *fw = reinterpret_cast<uint32_t *>(fr);
  // one poll's chunks: -1 nothing new (not yet whole, or another wave's),
  // 0 a request served, 1 leave
  auto serve = [&](const v4u &c) -> int {
    const uint32_t want = __builtin_amdgcn_readfirstlane(lds_ld(&done_s)) + 1;
    const uint32_t tag0 = __builtin_amdgcn_readfirstlane(c[3]);
    if (tag0 != want) return -1;
    const uint32_t hi = __builtin_amdgcn_readfirstlane(c[0]);
    if (hi == kServeLeave) return 1;
    const uint32_t len = min(hi & 0xFFFFu, kServeFrame), in = hi >> 16;
    const bool inl = len <= kServeInline;
    const uint32_t need = inl ? (12 + len + 11) / 12 : 1u;  // chunks carrying it
    if (__ballot(lane < need && c[3] != want)) return -1;  // not whole yet: poll again
    // one wave serves it: the first to claim it
    uint32_t won = 0;
    if (lane == 0) won = atomicCAS(&claim_s, want - 1, want) == want - 1;
    if (!__builtin_amdgcn_readfirstlane(won)) return -1;
    const uint64_t s0 = wall_clock64();
    const uint64_t t0_prev = prof ? t0_s : 0;  // (the last answer's clock)
    const uint64_t seq = seq0 + (want - done0 - 1);
    const int64_t now =
        (int64_t)((uint64_t)__builtin_amdgcn_readfirstlane(c[1]) |
                  ((uint64_t)__builtin_amdgcn_readfirstlane(c[2]) << 32));
    const uint32_t nch = (len + 15) / 16;
    if (inl) {  // chunk k >= 1: frame bytes 12k - 12 .. 12k - 1
      if (lane >= 1 && lane < need) {
        fw[3 * lane - 3] = c[0];
        fw[3 * lane - 2] = c[1];
        fw[3 * lane - 1] = c[2];
      }
    } else {  // the whole frame from `frame` (the host wrote it before the chunks)
      for (uint32_t i = lane; i < nch; i += 64) {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16 * i), 0, kSys);
        fr[i] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
    wave_lds_sync();
    // the L4 checksum's bytes past 64: [64, min(14 + total_length, len))
    uint32_t tail = 0;
    if (len > 64) {
      const uint8_t *fb = reinterpret_cast<const uint8_t *>(fr);
      const uint32_t tl = ((uint32_t)fb[16] << 8) | fb[17];
      const uint32_t end = min(14 + tl, len);
      for (uint32_t cc = 64 + 16 * lane; cc < end; cc += 1024)
        tail = sum16x4(chunk_keep(fr[cc / 16], 0, (int)end - (int)cc), tail);
      for (int o = 32; o > 0; o >>= 1) tail += __shfl_xor(tail, o);
    }
    const uint64_t s1 = wall_clock64();
    const uint64_t c1 = prof ? __builtin_amdgcn_s_memtime() : 0;  // (shader clock)
    uint32_t res = 0;
    uint64_t mk0 = 0, mk1 = 0, mk2 = 0;
    if (lane == 0) {
      uint32_t fresh = 0;
      RFrame f;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint4 v = chunk_keep(fr[j], 0, (int)len - 16 * j);
        f.w[4 * j] = v.x;
        f.w[4 * j + 1] = v.y;
        f.w[4 * j + 2] = v.z;
        f.w[4 * j + 3] = v.w;
      }
      uint32_t out = nat_one_reg(a, T, f, in, len, tail, now, seq, &fresh, prof, mk0, mk1);
      if (prof) mk2 = wall_clock64();
      if (out == kNone) {
        const GFrame g{reinterpret_cast<uint8_t *>(fr), len};
        out = nat_one(a, T, g, in, len, now, seq, &fresh);
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++)
          fr[j] = make_uint4(f.w[4 * j], f.w[4 * j + 1], f.w[4 * j + 2], f.w[4 * j + 3]);
      }
      res = out | (fresh << 16);
    }
    wave_lds_sync();
    const uint64_t s2 = wall_clock64();
    const uint64_t c2 = prof ? __builtin_amdgcn_s_memtime() : 0;
    res = __builtin_amdgcn_readfirstlane(res);
    if (inl) {  // the answer chunks: the result and the frame in one store
      if (lane < need) {
        const v4u v = lane == 0 ? (v4u){res, 0u, 0u, want}
                                : (v4u){fw[3 * lane - 3], fw[3 * lane - 2], fw[3 * lane - 1], want};
        __builtin_amdgcn_raw_buffer_store_b128(v, as, (int)(16 * lane), 0, kSys);
      }
    } else {
      for (uint32_t i = lane; i < nch; i += 64) {
        const uint4 v = fr[i];
        __builtin_amdgcn_raw_buffer_store_b128((v4u){v.x, v.y, v.z, v.w}, rs, (int)(16 * i), 0,
                                               kSys);
      }
      // (the frame complete before the answer chunk that announces it)
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      __builtin_amdgcn_s_waitcnt(0);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (lane == 0)
        __builtin_amdgcn_raw_buffer_store_b128((v4u){res, 0u, 0u, want}, as, 0, 0, kSys);
    }
    if (lane == 0) {
      // (the answer word: where a relaunched server starts counting; the
      // host reads the answer chunks. No release fence, which would write
      // back the whole L2)
      const uint64_t ans = (uint64_t)want | ((uint64_t)res << 32);
      __hip_atomic_store(&box->ans, ans, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      t0_s = wall_clock64();
      if (prof) {
        auto put = [&](int k, uint64_t v) {
          __hip_atomic_store(&box->prof[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        };
        put(0, t0_prev);
        put(1, s0);
        put(2, s1);
        put(3, mk0);
        put(4, mk1);
        put(5, mk2);
        put(6, s2);
        put(7, wall_clock64());
        put(8, c1);
        put(9, c2);
      }
      // (the table writes of this request before the next request's wave
      // reads them: the waves share the CU, workgroup scope; an agent-scope
      // release would write the XCD's L2 back)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __hip_atomic_store(&done_s, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    wave_lds_sync();
    return 0;
  };
  // every wave polls on its own (flags bits 3-9: the waves' stagger, in
  // wall-clock ticks), one poll in flight per wave: a wave's polls return in
  // order, so polls queued behind a stale one would see a request late
  const uint32_t gap = (flags >> 3) & 0x7Fu;
  {
    const uint64_t w = wall_clock64();
    while (wall_clock64() - w < (uint64_t)gap * wv) __builtin_amdgcn_s_sleep(1);
  }
  // After an answer the next request cannot come before the answer has
  // crossed to the host and the host's loop has turned round (about half a
  // round trip plus its own time): a poll issued at once reads the mailbox
  // too early and the request waits for the poll after it, a whole round
  // trip later. The first poll after an answer waits `after` wall-clock ticks
  // (flags bits 10-17; VIGPATH_SERVE_AFTER) so that it reads about when the
  // request lands.
  // The delay adapts (flags bit 18): a request the first poll caught takes
  // a tick off it, one that needed a later poll adds eight -- a late poll
  // costs a round trip, an early one only its excess -- so it settles just
  // past where the caller's requests land, whatever the caller's loop.
  uint32_t after = (flags >> 10) & 0xFFu;
  const uint32_t up = (flags >> 19) & 0x1Fu;  // ticks added after a late poll
  const bool adapt = (flags >> 18) & 1u;
  uint32_t polls = 0;  // polls since the last answer
  for (;;) {
    const v4u q = poll();
    const int st = serve(q);
    if (st == 1) break;
    polls++;
    if (st < 0) {
      if (wall_clock64() - __hip_atomic_load(&t0_s, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP) > idle)
        break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (adapt && polls == 1 && after > 0) after--;
    if (adapt && polls > 1 && polls < 64) after = min(after + up, 200u);
    polls = 0;
    if (after) {
      const uint64_t w = wall_clock64();
      while (wall_clock64() - w < after) __builtin_amdgcn_s_sleep(1);
    }
  }
}

// =============================================================== host ==

// nat_flowmanager.c:57-65: expiration_time (u32 us) * 1000 is computed in
// unsigned 32-bit arithmetic, so it wraps for > 4294967 us.
static inline int64_t nat_cutoff(const vp_ctx *c, int64_t t) {
  const uint32_t e = c->nat.expiration_time * 1000u;
  return (int64_t)((uint64_t)t - e);
}

// Device scratch of at least `count` elements. It is also reallocated down
// when it holds more than twice what is asked and over 64 MiB (the padded
// exchange's buffers after the first batches settle C).
template <class T>
static int grow_dev(T **p, size_t *have, size_t count, hipStream_t s) {
  const bool oversized = *have > 2 * std::max<size_t>(count, 1) && sizeof(T) * *have > (64u << 20);
  if (count <= *have && *p && !oversized) return 0;
  VP_HIP(hipStreamSynchronize(s));
  hipFree(*p);
  *p = nullptr;
  *have = 0;
  VP_HIP(hipMalloc((void **)p, sizeof(T) * std::max<size_t>(count, 1)));
  *have = count;
  return 0;
}

// Phase A in owner mode: pass 1 classifies what this rank can
// answer and routes the other LAN keys to their owners, the keys and answers
// cross in two all-to-alls, pass 2 finishes the routed packets and bins every
// touch, then the fold. On return h_ctl holds phase A's counts.
struct PhaseA {
  BinsPlan bp;
  bool tiles64;
  uint32_t grid1, range1;  // pass 1 layout (reprobe slices)
  float ms;
};

// Owner-mode stage times: HIP events between the stages of every segment's
// phase A when kernel timing is on (vp_kernel_timing: the timing pass of
// bench.py --gpus N), summed into vp_ctx::stage_ms for vp_last_stage_ms;
// VIGPATH_PHASES=1 also prints them per segment on stderr (diagnostics).
struct PhaseMarks {
  hipEvent_t ev[kStages + 1] = {};
  int id[kStages + 1] = {};  // the stage that ends at mark i
  int n = 0;
  bool on = false, print_on = false;
  PhaseMarks(hipStream_t s, bool timing) : stream(s) {
    const char *e = getenv("VIGPATH_PHASES");
    print_on = e && atoi(e);
    on = timing || print_on;
    if (on)
      for (auto &x : ev) (void)hipEventCreate(&x);
  }
  ~PhaseMarks() {
    if (on)
      for (auto &x : ev) (void)hipEventDestroy(x);
  }
  // (stage: the one this mark ends; default the next in kStageNames order)
  void mark(int stage = -1) {
    if (!on || n > kStages) return;
    id[n] = stage >= 0 ? stage : n - 1;
    (void)hipEventRecord(ev[n++], stream);
  }
  void finish(vp_ctx *c, int rank, uint32_t np) {
    if (!on || n < 2) return;
    (void)hipEventSynchronize(ev[n - 1]);
    if (print_on) fprintf(stderr, "vigpath owner r%d n=%u:", rank, np);
    for (int i = 1; i < n; i++) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, ev[i - 1], ev[i]);
      c->stage_ms[id[i]] += ms;
      c->stage_n = std::max(c->stage_n, id[i] + 1);
      if (print_on) fprintf(stderr, " %s %.3f", kStageNames[id[i]], ms);
    }
    if (print_on) fprintf(stderr, " ms\n");
  }
  hipStream_t stream;
};

static int nat_phase_a_owner(vp_ctx *c, const vp_dev_batch *b, NatArgs &a,
                             const NowSpec &now, uint32_t p0, uint32_t p1,
                             uint64_t seq0, PhaseA *ph) {
  PhaseMarks pm(c->stream, c->ktime);
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  Comm &m = *c->comm;
  const uint32_t n = (uint32_t)m.n, r = (uint32_t)m.r;
  const uint32_t np = p1 - p0;
  ph->tiles64 = np && b->slot == 64 && c->coalesced_io;
  uint32_t first;
  if (ph->tiles64) {
    first = p0 & ~63u;
    const uint32_t tiles = (p1 - first + 63) / 64;
    // pass 1: the 1024-thread tile unless VIGPATH_BLOCK_WAVES=4 (one block
    // per CU: four times fewer, longer key slices)
    const uint32_t tw = nat_block_waves();
    ph->grid1 = tw == 16 ? resident_grid((const void *)nat_classify64wo, (tiles + 15) / 16, 1024)
                         : resident_grid((const void *)nat_classify64, (tiles + 3) / 4);
    ph->range1 = (tiles + ph->grid1 - 1) / ph->grid1 * 64;
    VP_TRY(tbl_bins_plan(c, t, (const void *)nat_remote64, p0, p1, &ph->bp));
  } else {
    first = p0;
    ph->grid1 = std::max<uint32_t>(1, std::min<uint32_t>(2048, (np + 255) / 256));
    ph->range1 = std::max<uint32_t>(1, (np + ph->grid1 - 1) / ph->grid1);
  }
  if (ph->range1 >= (1u << 24) - 1) return VP_ENOTSUP;
  const uint32_t C = std::max<uint32_t>(1, c->own_cap);  // keys per peer (padded)
  uint32_t sub = std::max<uint32_t>(1, C / ph->grid1);  // keys per block slice
  if (sub >= 64) sub &= ~63u;  // (whole 64-key probe tiles per slice)
  if (ph->grid1 > kSliceRowMax) return VP_ENOTSUP;
  const size_t slices = (size_t)ph->grid1 * n;
  VP_TRY(grow_dev(&w.desc, &w.desc_n, slices * ph->range1, c->stream));
  VP_TRY(grow_dev(&w.dcnt, &w.dcnt_n, slices, c->stream));
  VP_TRY(grow_dev(&w.dbase, &w.dbase_n, slices, c->stream));
  VP_TRY(grow_dev(&w.dtot, &w.dtot_n, kMaxDest, c->stream));
  VP_TRY(grow_dev(&w.dneed, &w.dneed_n, kMaxDest, c->stream));
  VP_TRY(grow_dev(&w.cnt_t, &w.cnt_t_n, (size_t)n * kSliceRow, c->stream));
  VP_TRY(grow_dev(&w.rcnt_t, &w.rcnt_t_n, (size_t)n * kSliceRow, c->stream));
  VP_TRY(grow_dev(&w.route, &w.route_n, b->n, c->stream));
  VP_TRY(grow_dev(&w.sendk, &w.sendk_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.recvk, &w.recvk_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.reply, &w.reply_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.rreply, &w.rreply_n, (size_t)n * C, c->stream));
  if (!w.ovf64) VP_HIP(hipMalloc((void **)&w.ovf64, 8));
  if (!w.h_tot) VP_HIP(hipHostMalloc((void **)&w.h_tot, 4 * kMaxDest, hipHostMallocDefault));
  static const uint32_t route_all = [] {
    const char *e = getenv("VIGPATH_ROUTE_ALL");
    return e && atoi(e) ? 1u : 0u;
  }();
  a.own = Route{n,       r,        w.desc, w.dcnt,    w.route, nullptr,
                first,   ph->range1, w.dbase, w.rreply, C,      w.ovf64,
                route_all, w.sendk, sub};

  // (counters still zero after a segment that appended nothing, and the
  // overflow flag after an exchange that fit: no reset launches)
  if (!t.ctl_clean) VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 16, c->stream));  // .. reprobe
  t.ctl_clean = false;
  if (!w.ovf64_clean) VP_HIP(hipMemsetAsync(w.ovf64, 0, 8, c->stream));
  w.ovf64_clean = false;
  VP_HIP(ev_record(c->ktime, c->ev0, c->stream));
  pm.mark();
  if (np) {
    if (ph->tiles64) {
      NatArgs a1 = a;
      a1.tileq = 1;
      a1.mq = w.missq;
      if (ph->bp.on) a1.log = nullptr;  // pass 2 bins every touch
      const TileQueue rq1{w.reprobe, w.reprobe_cnt, &t.ctl->reprobe_count};
      if (nat_block_waves() == 16) {
        c->last_kernel = "nat_classify64wo+nat_remote64";
        nat_classify64wo<<<ph->grid1, 1024, 0, c->stream>>>(a1, b->n, TouchBins{}, rq1);
      } else {
        c->last_kernel = "nat_classify64+nat_remote64";
        nat_classify64<<<ph->grid1, 256, 0, c->stream>>>(a1, b->n, TouchBins{}, rq1);
      }
    } else {
      nat_classify<<<ph->grid1, 256, 0, c->stream>>>(a);
    }
    VP_HIP(hipGetLastError());
  } else {
    VP_HIP(hipMemsetAsync(w.dcnt, 0, sizeof(uint32_t) * slices, c->stream));
  }
  VP_HIP(ev_record(c->ktime, c->ev1, c->stream));
  pm.mark();
  // C1 over the padded exchange, no host round trip: pass 1 wrote owner o's
  // keys into [o C, (o + 1) C) of the send buffer, one slice of `sub` per
  // block; the per-block counts cross in their own small all-to-all, and a
  // slice past `sub` (any rank: allreduced) leaves the routed packets to the
  // exact exchange below
  route_counts<<<n, 256, 0, c->stream>>>(w.dcnt, ph->grid1, n, sub, w.cnt_t, w.dneed,
                                         w.ovf64);
  VP_HIP(hipGetLastError());
  // (this rank's own chunk stays where pass 1 put it: the probe reads it
  // from sendk and answers it into rreply, no self copies)
  std::vector<size_t> sc(n, 4ull * kSliceRow), sk(n, 16ull * C), sr(n, 4ull * C);
  VP_TRY(m.alltoallv_dev(c, w.cnt_t, sc.data(), w.rcnt_t, sc.data()));
  VP_TRY(m.allreduce_max_u64_dev(c, w.ovf64, 1));
  pm.mark();
  VP_TRY(m.alltoallv_dev(c, w.sendk, sk.data(), w.recvk, sk.data(), true));
  pm.mark();
  nat_own_probe<<<resident_grid((const void *)nat_own_probe, ((uint64_t)n * C + 255) / 256), 256,
                  0, c->stream>>>(tbl_dev(t), c->crc_tab, w.recvk, n * C, C, w.rcnt_t, w.ovf64,
                                  t.ctl, w.reply, r, w.sendk, w.rreply);
  VP_HIP(hipGetLastError());
  pm.mark();
  VP_TRY(m.alltoallv_dev(c, w.reply, sr.data(), w.rreply, sr.data(), true));
  pm.mark();
  auto pass2 = [&]() -> int {
    if (!np) return 0;
    if (ph->tiles64) {
      NatArgs a2 = a;
      uint32_t grid2 = ph->bp.grid;
      if (ph->bp.on) {
        a2.log = nullptr;
      } else {
        const uint32_t tiles = (p1 - first + 63) / 64;
        grid2 = resident_grid((const void *)nat_remote64, (tiles + 3) / 4);
      }
      nat_remote64<<<grid2, 256, 0, c->stream>>>(a2, b->n, ph->bp.bins);
    } else {
      nat_remote_lane<<<grid_for(np), 256, 0, c->stream>>>(a);
    }
    VP_HIP(hipGetLastError());
    return 0;
  };
  VP_HIP(ev_record(c->ktime, c->ev2, c->stream));
  VP_TRY(pass2());
  VP_HIP(ev_record(c->ktime, c->ev3, c->stream));
  pm.mark();
  VP_TRY(tbl_fold_read_ctl(c, t, ph->bp, w.log, p0, p1, now, seq0, w.dneed));
  pm.mark();
  pm.finish(c, m.r, np);
  uint32_t maxsend = 0;  // for the next batch's capacity (run_batch_sharded)
  for (uint32_t o = 0; o < n; o++)
    if (o != r) maxsend = std::max(maxsend, w.h_gath[kPubGath * n + o]);
  c->own_maxsend = maxsend;
  float k1 = 0.f, k2 = 0.f;
  VP_HIP(ev_ms(c->ktime, c->ev0, c->ev1, &k1));
  VP_HIP(ev_ms(c->ktime, c->ev2, c->ev3, &k2));
  ph->ms = k1 + k2;
  w.ovf64_clean = !t.h_ctl.route_ovf;  // (every rank's flag was 0: allreduced)
  if (!t.h_ctl.route_ovf) return 0;
  // Some rank had more keys for an owner than C (every rank sees the flag):
  // pass 2 answered none of the routed packets; the exact exchange does,
  // with the sizes learned on the host, then the fold again (pass 1's own
  // touches fold twice, to the same stamps).
  route_scan<<<n, 256, 0, c->stream>>>(w.dcnt, ph->grid1, n, w.dbase, w.dtot);
  route_base<<<grid_for(slices), 256, 0, c->stream>>>(w.dbase, w.dtot, ph->grid1, n);
  VP_HIP(hipGetLastError());
  VP_HIP(hipMemcpyAsync(w.h_tot, w.dtot, 4ull * n, hipMemcpyDeviceToHost, c->stream));
  VP_HIP(stream_wait(c->stream));
  std::vector<uint32_t> M((size_t)n * n);  // M[q * n + o] = keys rank q sends to owner o
  VP_TRY(m.allgather_host(c, w.h_tot, M.data(), 4ull * n));
  uint64_t S = 0, R = 0;
  std::vector<size_t> ek(n), er(n), fr(n), fa(n);
  for (uint32_t q = 0; q < n; q++) {
    S += M[(size_t)r * n + q];
    R += M[(size_t)q * n + r];
    ek[q] = 16ull * M[(size_t)r * n + q];
    er[q] = 16ull * M[(size_t)q * n + r];
    fr[q] = 4ull * M[(size_t)q * n + r];  // answers go back the way keys came
    fa[q] = 4ull * M[(size_t)r * n + q];
  }
  VP_TRY(grow_dev(&w.xsend, &w.xsend_n, S, c->stream));
  VP_TRY(grow_dev(&w.rreply, &w.rreply_n, S, c->stream));
  VP_TRY(grow_dev(&w.recvk, &w.recvk_n, R, c->stream));
  VP_TRY(grow_dev(&w.reply, &w.reply_n, R, c->stream));
  a.own.rreply = w.rreply;
  a.own.cap = 0;
  route_pack<<<ph->grid1, 256, 0, c->stream>>>(w.desc, w.sendk, w.dcnt, w.dbase, n, ph->range1,
                                               C, sub, w.xsend);
  VP_HIP(hipGetLastError());
  VP_TRY(m.alltoallv_dev(c, w.xsend, ek.data(), w.recvk, er.data()));
  nat_own_probe<<<resident_grid((const void *)nat_own_probe, (std::max<uint64_t>(R, 1) + 255) / 256),
                  256, 0, c->stream>>>(tbl_dev(t), c->crc_tab, w.recvk, (uint32_t)R, 0, nullptr,
                                       nullptr, t.ctl, w.reply, kNone, nullptr, nullptr);
  VP_HIP(hipGetLastError());
  VP_TRY(m.alltoallv_dev(c, w.reply, fr.data(), w.rreply, fa.data()));
  VP_HIP(ev_record(c->ktime, c->ev2, c->stream));
  VP_TRY(pass2());
  VP_HIP(ev_record(c->ktime, c->ev3, c->stream));
  VP_TRY(tbl_fold_read_ctl(c, t, ph->bp, w.log, p0, p1, now, seq0, w.dneed));
  VP_HIP(ev_ms(c->ktime, c->ev2, c->ev3, &k2));
  ph->ms += k2;
  return 0;
}

// ------------------------------------------------ chunked owner pipeline --
// (off by default, nat_own_chunk_packets) The segment's tiles
// are cut into K chunks of G blocks x vper
// tiles. Chunk k runs pass 1 on the context's stream S; its keys cross, are
// answered by nat_own_probe and come back on the exchange stream X while S
// runs pass 1 of chunk k + 1; then S runs chunk k's pass 2, whose frame
// reads find chunk k's frames still in the Infinity Cache (read by its pass 1
// one chunk earlier; a chunk of 2^20 packets is 64 MB of the 256 MB), as do
// the keys, routes and answers. Per chunk the exchange is the keys'
// all-to-all, the probe and the answers' all-to-all: a block closes its
// slices with sentinel keys, so no counts cross, and a key past its slice
// raises this rank's overflow flag, gathered before the fold (no allreduce
// per chunk). Two buffer sets alternate between chunks. Every rank runs the
// same K (computed from every rank's part of the segment), so the exchanges
// match. After the fold, if any rank overflowed, the keys past their slices
// take the exact exchange (route_left / route_pack_left), a pass 2 over the
// leftovers and a second fold that only raises stamps (BinsPlan::maxmode).
struct OwnChunks {
  uint32_t K = 0;     // chunks (0: the unchunked pipeline)
  uint32_t G = 0;     // blocks per chunk launch
  uint32_t vper = 0;  // tiles per (virtual) block
};

// Blocks per chunk launch: the resident grid of both passes (VIGPATH_OWN_BLOCKS
// lowers it: tests cut small batches into many chunks).
static uint32_t own_grid() {
  static const uint32_t g = std::min(resident_grid((const void *)nat_classify64, 1u << 30),
                                     resident_grid((const void *)nat_remote64, 1u << 30));
  const char *e = getenv("VIGPATH_OWN_BLOCKS");
  const uint32_t v = e ? (uint32_t)atoi(e) : 0u;
  return v ? std::min(v, g) : g;
}

// Packets per chunk (VIGPATH_OWN_CHUNK; 0, the default: the unchunked
// pipeline), rounded up to whole blocks of whole tiles. Off by default: on
// one MI355X (bench.py --route-all) chunks of 2^19-2^21 packets made the
// owner step 1.39-2.43 ms against 1.04 unchunked -- each chunk's launches
// pay their ramp, tail and per-block table loads, pass 2 did not get faster
// from the Infinity Cache, and a probe beside a pass 2 slows both (DESIGN.md
// §6.1, profiles/r05de_owner_chunked_traces.txt). (Read per call: the tests
// change it.)
uint32_t nat_own_chunk_packets() {
  const char *e = getenv("VIGPATH_OWN_CHUNK");
  const uint64_t want = e ? strtoull(e, nullptr, 10) : 0;
  if (!want) return 0u;
  const uint64_t G = own_grid();
  const uint64_t vper = std::max<uint64_t>(1, (want / 64 + G - 1) / G);
  return (uint32_t)std::min<uint64_t>(vper * G * 64, 1ull << 30);
}

// The same decision on every rank: 64-byte slots with coalesced tiles, and
// every rank's part of the segment starting on a tile (touch bins); K = the
// most chunks any rank's part needs.
static OwnChunks own_chunks_plan(vp_ctx *c, const vp_dev_batch *b) {
  OwnChunks oc;
  const uint32_t pk = nat_own_chunk_packets();
  if (!pk || b->slot != 64 || !c->coalesced_io || c->rank_n.empty()) return oc;
  const uint32_t G = own_grid();
  const uint32_t vper = pk / 64 / G;
  uint64_t off = 0, K = 0;
  for (uint32_t q = 0; q < c->rank_n.size(); q++) {
    const uint64_t n = c->rank_n[q];
    const uint64_t l0 = std::min(std::max(c->seg_g0, off), off + n) - off;
    const uint64_t l1 = std::min(std::max(c->seg_g1, off), off + n) - off;
    off += n;
    if (l1 <= l0) continue;
    if (l0 & 63) return oc;  // (a cut inside a tile: no touch bins there)
    const uint64_t tiles = (l1 - l0 + 63) / 64;
    const uint64_t vg = (tiles + vper - 1) / vper;
    K = std::max<uint64_t>(K, (vg + G - 1) / G);
  }
  oc.K = (uint32_t)K;
  oc.G = G;
  oc.vper = vper;
  return oc;
}

static int nat_phase_a_owner_chunked(vp_ctx *c, const vp_dev_batch *b, NatArgs &a,
                                     const NowSpec &now, uint32_t p0, uint32_t p1,
                                     uint64_t seq0, const OwnChunks &oc, PhaseA *ph) {
  c->last_kernel = "nat_classify64+nat_remote64 (chunked)";
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  Comm &m = *c->comm;
  const uint32_t n = (uint32_t)m.n, r = (uint32_t)m.r;
  const uint32_t np = p1 - p0;
  const uint32_t G = oc.G, vper = oc.vper, K = oc.K;
  const uint32_t tiles = np ? (p1 - p0 + 63) / 64 : 0;
  const uint32_t vg = (tiles + vper - 1) / vper;  // this rank's virtual blocks
  ph->tiles64 = np != 0;
  ph->grid1 = std::max<uint32_t>(vg, 1);
  ph->range1 = vper * 64;
  if (np) {
    VP_TRY(tbl_bins_plan(c, t, (const void *)nat_remote64, p0, p1, &ph->bp, 4, 0, vper));
    if (!ph->bp.on || ph->bp.grid != vg || ph->bp.range != vper * 64)
      return state_fail("chunked owner pipeline: no touch bins for [%u, %u)", p0, p1);
  }
  const uint32_t C = std::max<uint32_t>(1, c->own_cap);  // keys per peer and chunk
  // keys per block slice: C over the blocks a chunk launch of this rank has
  // (the sender's layout alone: owners find the keys by their sentinels)
  uint32_t sub = std::max<uint32_t>(1, C / std::max<uint32_t>(1, std::min(G, vg)));
  if (sub >= 64) sub &= ~63u;  // (whole 64-key probe tiles per slice)
  const size_t slices = (size_t)std::max<uint32_t>(vg, 1) * n;
  VP_TRY(grow_dev(&w.desc, &w.desc_n, slices * ph->range1, c->stream));
  VP_TRY(grow_dev(&w.dcnt, &w.dcnt_n, slices, c->stream));
  if (!vg) VP_HIP(hipMemsetAsync(w.dcnt, 0, 4ull * n, c->stream));  // (leftovers: none)
  VP_TRY(grow_dev(&w.dbase, &w.dbase_n, slices, c->stream));
  VP_TRY(grow_dev(&w.dtot, &w.dtot_n, kMaxDest, c->stream));
  VP_TRY(grow_dev(&w.dneed, &w.dneed_n, kMaxDest, c->stream));
  VP_TRY(grow_dev(&w.route, &w.route_n, b->n, c->stream));
  uint4 *sk[2], *rk[2];
  uint32_t *rp[2], *rr[2];
  VP_TRY(grow_dev(&w.sendk, &w.sendk_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.recvk, &w.recvk_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.reply, &w.reply_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.rreply, &w.rreply_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.sendk2, &w.sendk2_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.recvk2, &w.recvk2_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.reply2, &w.reply2_n, (size_t)n * C, c->stream));
  VP_TRY(grow_dev(&w.rreply2, &w.rreply2_n, (size_t)n * C, c->stream));
  sk[0] = w.sendk, sk[1] = w.sendk2, rk[0] = w.recvk, rk[1] = w.recvk2;
  rp[0] = w.reply, rp[1] = w.reply2, rr[0] = w.rreply, rr[1] = w.rreply2;
  if (!w.h_tot) VP_HIP(hipHostMalloc((void **)&w.h_tot, 4 * kMaxDest, hipHostMallocDefault));
  if (!w.xstream) {
    VP_HIP(hipStreamCreateWithFlags(&w.xstream, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
      VP_HIP(hipEventCreateWithFlags(&w.ev_p1[i], hipEventDisableTiming));
      VP_HIP(hipEventCreateWithFlags(&w.ev_ans[i], hipEventDisableTiming));
    }
  }
  static const bool one_stream = [] {  // (diagnostics: no overlap between the streams)
    const char *e = getenv("VIGPATH_OWN_ONESTREAM");
    return e && atoi(e);
  }();
  hipStream_t S = c->stream, X = one_stream ? c->stream : w.xstream;
  static const uint32_t route_all = [] {
    const char *e = getenv("VIGPATH_ROUTE_ALL");
    return e && atoi(e) ? 1u : 0u;
  }();
  const uint32_t first = p0 & ~63u;
  a.own = Route{n,       r,          w.desc, w.dcnt,    w.route, nullptr,
                first,   ph->range1, w.dbase, nullptr,  C,       nullptr,
                route_all, nullptr,  sub,    kOwnChunked, &t.ctl->route_ovf, w.dneed};
  // (miss .. route_ovf; the per-owner slice maxima)
  if (!t.ctl_clean) VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 20, S));
  t.ctl_clean = false;
  VP_HIP(hipMemsetAsync(w.dneed, 0, 4ull * n, S));
  VP_HIP(ev_record(c->ktime, c->ev0, S));
  PhaseMarks pm(S, c->ktime);
  pm.mark();
  const uint32_t gp = resident_grid((const void *)nat_own_probe, ((uint64_t)n * C + 255) / 256);
  std::vector<size_t> sz(n, 16ull * C), sa(n, 4ull * C);
  auto blocks = [&](uint32_t k) {  // this rank's blocks of chunk k
    const uint32_t b0 = k * G;
    return b0 < vg ? std::min(G, vg - b0) : 0u;
  };
  auto pass2 = [&](uint32_t k) -> int {
    const uint32_t nb = blocks(k);
    if (!nb) return 0;
    NatArgs a2 = a;
    a2.log = nullptr;  // (pass 2 bins every touch)
    a2.vb0 = k * G;
    a2.vper = vper;
    a2.own.rreply = rr[k & 1];
    nat_remote64<<<nb, 256, 0, S>>>(a2, b->n, ph->bp.bins);
    VP_HIP(hipGetLastError());
    return 0;
  };
  for (uint32_t k = 0; k < K; k++) {
    const uint32_t i = k & 1;
    // pass 1 of chunk k (its buffer set was last used by chunk k - 2)
    if (k >= 2) VP_HIP(hipStreamWaitEvent(S, w.ev_ans[i], 0));
    const uint32_t nb = blocks(k);
    if (nb) {
      NatArgs a1 = a;
      a1.tileq = 1;
      a1.mq = w.missq;
      a1.log = nullptr;  // pass 2 bins every touch
      a1.vb0 = k * G;
      a1.vper = vper;
      a1.own.sendk = sk[i];
      nat_classify64<<<nb, 256, 0, S>>>(
          a1, b->n, TouchBins{}, TileQueue{w.reprobe, w.reprobe_cnt, &t.ctl->reprobe_count});
      VP_HIP(hipGetLastError());
    } else {  // (no packets of this rank in chunk k: empty slices)
      VP_HIP(hipMemsetAsync(sk[i], 0xFF, 16ull * n * C, S));
    }
    VP_HIP(hipEventRecord(w.ev_p1[i], S));
    // chunk k's exchange on X: keys out, answered by their owners, back
    VP_HIP(hipStreamWaitEvent(X, w.ev_p1[i], 0));
    VP_TRY(m.alltoallv_dev(c, sk[i], sz.data(), rk[i], sz.data(), true, X));
    nat_own_probe<<<gp, 256, 0, X>>>(tbl_dev(t), c->crc_tab, rk[i], n * C, C, nullptr, nullptr,
                                     t.ctl, rp[i], r, sk[i], rr[i]);
    VP_HIP(hipGetLastError());
    VP_TRY(m.alltoallv_dev(c, rp[i], sa.data(), rr[i], sa.data(), true, X));
    VP_HIP(hipEventRecord(w.ev_ans[i], X));
    // pass 2 of chunk k - 1 behind pass 1 of chunk k
    if (k >= 1) {
      VP_HIP(hipStreamWaitEvent(S, w.ev_ans[i ^ 1], 0));
      VP_TRY(pass2(k - 1));
    }
  }
  if (K) {
    VP_HIP(hipStreamWaitEvent(S, w.ev_ans[(K - 1) & 1], 0));
    VP_TRY(pass2(K - 1));
  }
  VP_HIP(ev_record(c->ktime, c->ev3, S));
  pm.mark(kStagePipeline);
  VP_TRY(tbl_fold_read_ctl(c, t, ph->bp, nullptr, p0, p1, now, seq0, w.dneed));
  pm.mark(kStageFold);
  pm.finish(c, m.r, np);
  uint32_t maxsend = 0;  // the next batch's capacity per chunk (run_batch_sharded)
  for (uint32_t o = 0; o < n; o++)
    if (o != r || route_all) maxsend = std::max(maxsend, w.h_gath[kPubGath * n + o]);
  c->own_maxsend = maxsend * G;
  float k1 = 0.f;
  VP_HIP(ev_ms(c->ktime, c->ev0, c->ev3, &k1));
  ph->ms = k1;
  bool any = false;
  for (uint32_t q = 0; q < n; q++) any |= w.h_gath[kPubGath * q + 4] != 0;
  if (!any) return 0;
  // Leftovers (some rank's slice overflowed): the exact exchange of every
  // rank's keys past their slices, pass 2 over those packets, a second fold
  VP_TRY(grow_dev(&w.lcnt, &w.lcnt_n, slices, S));
  route_left<<<grid_for(slices), 256, 0, S>>>(w.dcnt, (uint32_t)slices, sub, w.lcnt);
  route_scan<<<n, 256, 0, S>>>(w.lcnt, ph->grid1, n, w.dbase, w.dtot);
  route_base<<<grid_for(slices), 256, 0, S>>>(w.dbase, w.dtot, ph->grid1, n);
  VP_HIP(hipGetLastError());
  VP_HIP(hipMemcpyAsync(w.h_tot, w.dtot, 4ull * n, hipMemcpyDeviceToHost, S));
  VP_HIP(stream_wait(S));
  std::vector<uint32_t> M((size_t)n * n);  // M[q * n + o] = keys rank q sends to owner o
  VP_TRY(m.allgather_host(c, w.h_tot, M.data(), 4ull * n));
  uint64_t Ssum = 0, R = 0;
  std::vector<size_t> ek(n), er(n), fr(n), fa(n);
  for (uint32_t q = 0; q < n; q++) {
    Ssum += M[(size_t)r * n + q];
    R += M[(size_t)q * n + r];
    ek[q] = 16ull * M[(size_t)r * n + q];
    er[q] = 16ull * M[(size_t)q * n + r];
    fr[q] = 4ull * M[(size_t)q * n + r];  // answers go back the way keys came
    fa[q] = 4ull * M[(size_t)r * n + q];
  }
  VP_TRY(grow_dev(&w.xsend, &w.xsend_n, Ssum, S));
  VP_TRY(grow_dev(&w.rreply, &w.rreply_n, Ssum, S));
  VP_TRY(grow_dev(&w.recvk, &w.recvk_n, R, S));
  VP_TRY(grow_dev(&w.reply, &w.reply_n, R, S));
  if (vg)
    route_pack_left<<<vg, 256, 0, S>>>(w.desc, w.dcnt, w.dbase, n, ph->range1, sub, w.xsend);
  VP_HIP(hipGetLastError());
  VP_TRY(m.alltoallv_dev(c, w.xsend, ek.data(), w.recvk, er.data()));
  nat_own_probe<<<resident_grid((const void *)nat_own_probe, (std::max<uint64_t>(R, 1) + 255) / 256),
                  256, 0, S>>>(tbl_dev(t), c->crc_tab, w.recvk, (uint32_t)R, 0, nullptr,
                               nullptr, t.ctl, w.reply, kNone, nullptr, nullptr);
  VP_HIP(hipGetLastError());
  VP_TRY(m.alltoallv_dev(c, w.reply, fr.data(), w.rreply, fa.data()));
  // The first pass 2's touches that found their bin slice full sit on the
  // blocks' overflow queues, which the leftover pass 2 rewrites: apply them
  // now (late touches commute: tseq atomicMax, then the winner's ts).
  if (t.h_ctl.touch_ovf)
    VP_TRY(tbl_late_touches(c, t, ph->bp.bins.oent, ph->bp.bins.ocnt, 0, ph->bp.range,
                            ph->bp.grid, w.log, now, seq0));
  if (vg) {  // (the touch bins are rewritten by these blocks: leftover touches only)
    NatArgs a2 = a;
    a2.log = nullptr;
    a2.vb0 = 0;
    a2.vper = vper;
    a2.own.mode = kOwnLeftover;
    a2.own.rreply = w.rreply;
    nat_remote64<<<vg, 256, 0, S>>>(a2, b->n, ph->bp.bins);
    VP_HIP(hipGetLastError());
  }
  BinsPlan again = ph->bp;
  again.maxmode = true;
  VP_TRY(tbl_fold_read_ctl(c, t, again, nullptr, p0, p1, now, seq0, w.dneed));
  // (the flag is this segment's: a next segment whose counters need no reset
  // must not find it set)
  VP_HIP(hipMemsetAsync(&t.ctl->route_ovf, 0, 4, S));
  return 0;
}

static int nat_segment(vp_ctx *c, const vp_dev_batch *b, const NowSpec &now,
                       uint32_t p0, uint32_t p1, float *ms, int *launches,
                       uint32_t *allocated) {
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  NatArgs a{};
  a.frames = b->frames;
  a.len = b->len;
  a.in_dev = b->in_dev;
  a.in0 = b->in_dev ? 0u : b->in_port;  // (port_of: exactly one is live)
  a.out = b->out_dev;
  a.log = w.log;
  a.now = now;
  const uint64_t seq0 = c->seq + c->off;  // global sequence of local packet 0
  a.seq_base = seq0;
  a.slot = b->slot;
  a.p0 = p0;
  a.p1 = p1;
  a.t = tbl_dev(t);
  a.crc_tab = c->crc_tab;
  a.macw = c->macw;
  a.wan_macw0 = c->wan_macw[0];
  a.wan_macw1 = c->wan_macw[1];
  a.wan_macw2 = c->wan_macw[2];
  a.miss = w.miss;
  a.defer = w.defer;
  a.reprobe = w.reprobe;
  a.ext_ip = c->nat.external_addr;
  a.wan = c->nat.wan_device;
  a.start_port = c->nat.start_port;
  a.n_dev = c->nat.n_devices;
  a.tail = c->hdr_tail;  // (vp_process_mbufs' header slots; null otherwise)
  // one GPU: phase B takes the misses unsorted, with the keys phase A leaves
  // (tbl_new_keys_unsorted; VIGPATH_NK_SORTED=1: the sorted path, for A/B);
  // multi-GPU ranks allocate the union in global order (sorted)
  static const bool nk_sorted = [] {
    const char *e = getenv("VIGPATH_NK_SORTED");
    return e && atoi(e);
  }();
  const bool nku = !c->comm && !nk_sorted;
  static const bool bin_stage = [] {
    const char *e = getenv("VIGPATH_BIN_STAGE");
    return !e || atoi(e) != 0;
  }();
  a.bstage = bin_stage ? 1u : 0u;
  a.split = tile_split();
  if (nku) {
    a.mkey = reinterpret_cast<uint4 *>(w.mkey);
    a.mhash = w.mhash;
    a.mkq = w.mkq;
    a.mhq = w.mhq;
  }

  const bool owner = c->shard_mode == VP_SHARD_OWNER && c->comm;
  if (owner && a.tail) return VP_ENOTSUP;  // (vp_mbuf.hip never asks for it)
  PhaseA ph{};
  if (owner) {
    const OwnChunks oc = own_chunks_plan(c, b);
    if (oc.K)
      VP_TRY(nat_phase_a_owner_chunked(c, b, a, now, p0, p1, seq0, oc, &ph));
    else
      VP_TRY(nat_phase_a_owner(c, b, a, now, p0, p1, seq0, &ph));
  }
  // tiles of 64 packets (64-byte slots, or wider ones: nat_tiles): the
  // classify launch also bins its touches (TouchBins) and queues reprobes
  // per block (TileQueue)
  const bool tiles64 = owner ? ph.tiles64 : p1 > p0 && c->coalesced_io;
  // (staged bin lines unless the last segment's tiles were mostly runs)
  const NatTileKernel tk = nat_tile_kernel(b->slot, a.tail != nullptr, !t.runs_seen);
  const uint32_t tw = nat_tile_waves(tk);
  BinsPlan bp = ph.bp;
  uint32_t grid64 = ph.grid1, range64 = ph.range1;
  TileQueue rq{};
  if (tiles64 && !owner) {
    VP_TRY(tbl_bins_plan(c, t, (const void *)tk, p0, p1, &bp, tw));
    const uint32_t tiles = (p1 - (p0 & ~63u) + 63) / 64;
    grid64 = resident_grid((const void *)tk, (tiles + tw - 1) / tw, 64 * (int)tw);
    range64 = (tiles + grid64 - 1) / grid64 * 64;
    rq = TileQueue{w.reprobe, w.reprobe_cnt, &t.ctl->reprobe_count};
    a.tileq = 1;
    a.mq = w.missq;
  }
  if (!owner) {
  if (!t.ctl_clean)
    VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 16, c->stream));  // .. reprobe
  t.ctl_clean = false;
  hostprof(1);
  uint32_t pub_epoch = 0;  // (nonzero: the classify publishes, tile_publish)
  if (p1 > p0) {  // (the launch's own timestamps in ev0 / ev1)
    if (tiles64) {
      NatArgs a64 = a;
      if (bp.on) a64.log = nullptr;  // touches go to the bins only
      if (bp.on && !c->comm && tile_pub_on()) {
        pub_epoch = ++t.pub_epoch;
        a64.pub = PubArgs{t.d_pub, t.ctl, pub_epoch, nullptr, nullptr, 0, 0};
      }
      c->last_kernel = nat_tile_kernel_name(tk);
      if (c->ktime) {
        VP_HIP(launch_timed(tk, grid64, 64 * tw, c->stream, c->ev0, c->ev1, a64,
                            (uint32_t)b->n, bp.bins, rq));
      } else {
        tk<<<grid64, 64 * tw, 0, c->stream>>>(a64, (uint32_t)b->n, bp.bins, rq);
        VP_HIP(hipGetLastError());
      }
    } else {
      VP_HIP(launch_timed(nat_classify, grid_for(p1 - p0), 256, c->stream, c->ev0,
                          c->ev1, a));
    }
  } else {
    VP_HIP(ev_record(c->ktime, c->ev0, c->stream));
    VP_HIP(ev_record(c->ktime, c->ev1, c->stream));
  }
  // Phase A's counts for the host, and the fold of its touches right away;
  // the packets it queued (reprobes, overflowed bin entries, phase B/C) are
  // applied on top of it afterwards as late touches (tbl_late_touches: last
  // toucher still wins).
  hostprof(2);
  VP_TRY(tbl_fold_read_ctl(c, t, bp, w.log, p0, p1, now, seq0, nullptr, pub_epoch));
  if (tiles64 && bp.on) {  // (the run tiles of this launch: the next one's kernel)
    const uint32_t nrun = t.h_ctl.run_tiles - t.last_run_tiles;
    t.last_run_tiles = t.h_ctl.run_tiles;
    t.runs_seen = 2ull * nrun >= (uint64_t)(p1 - p0) / 64;
  }
  hostprof(4);
  VP_HIP(ev_ms(c->ktime, c->ev0, c->ev1, &ph.ms));
  hostprof(5);
  }  // !owner
  a.own.n = 0;  // below: this rank's own table only
  const uint32_t nre = t.h_ctl.reprobe_count;
  if (nre) {  // probes past a full home bucket: finish them, patch the fold
    const uint32_t *rcnt = tiles64 ? w.reprobe_cnt : nullptr;
    const uint32_t range = tiles64 ? range64 : 256;
    const uint32_t nblk = tiles64 ? grid64 : (nre + 255) / 256;
    nat_reprobe<<<std::min<uint32_t>(nblk, 2048), 256, 0, c->stream>>>(
        a, w.reprobe, rcnt, nre, range, nblk, seq0);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_reprobe_stamp(c, t, w.reprobe, rcnt, nre, range, nblk, w.log, now,
                             seq0));
    VP_TRY(read_ctl(c, t));  // the walk may have found new flows
  }
  const bool ovf = bp.on && t.h_ctl.touch_ovf != 0;
  if (ovf)  // touches that found their bin slice full, logged alone
    VP_TRY(tbl_late_touches(c, t, bp.bins.oent, bp.bins.ocnt, 0, bp.range, bp.grid,
                            w.log, now, seq0));
  *ms += ph.ms;
  *launches += 1;
  const uint32_t nmiss = t.h_ctl.miss_count, ndefer = t.h_ctl.defer_count;
  if (c->seg_fs && !nmiss) t.fs_hint = 0;  // the cut met no new flow: stop cutting

  uint32_t union_n = nmiss, union_off = 0;  // this rank's misses in the union
  if (c->comm) VP_TRY(union_sizes(c, nmiss, &union_n, &union_off));
  if (nmiss && nku) {  // (one GPU: no sort, no key gather, no late touches)
    VP_TRY(tbl_new_keys_unsorted(c, t, nmiss, p0, p1, now, c->seq));
    // (the frames before the counters come back: the host's round trip hides
    // behind the rewrite)
    nat_miss_finish<<<grid_for(nmiss), 256, 0, c->stream>>>(a, w.miss, nmiss, nullptr, w.rep,
                                                            nullptr, w.nkset);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_new_keys_done(c, t));
    a.t = tbl_dev(t);  // a rebuild may have moved the buckets
    *allocated |= 1u;
    // the first-sighting cut for the next batch (run_batch): set when most
    // misses repeated flows first seen in the segment's opening half
    const uint64_t nnew = t.h_ctl.new_count, span = t.h_ctl.last_first;
    const uint64_t rep = nmiss > nnew ? nmiss - nnew : 0;
    if (!c->seg_fs && p0 == 0 && rep >= (1u << 16) && rep >= 4 * nnew && span &&
        2 * span <= (uint64_t)(p1 - p0))
      t.fs_hint = (uint32_t)((span + 63) & ~63ull);
  } else if (nmiss) {
    size_t need = 0;
    hipcub::DeviceRadixSort::SortKeys(nullptr, need, w.miss, w.miss_sorted,
                                      (int)nmiss, 0, 32, c->stream);
    VP_TRY(cub_reserve(c, need));
    VP_HIP(hipcub::DeviceRadixSort::SortKeys(w.cub_tmp, w.cub_bytes, w.miss,
                                             w.miss_sorted, (int)nmiss, 0, 32,
                                             c->stream));
    nat_miss_keys<<<grid_for(nmiss), 256, 0, c->stream>>>(a, w.miss_sorted, nmiss,
                                                          w.mkey, w.mhash);
    VP_HIP(hipGetLastError());
  }
  if (union_n && !nku) {
    if (c->comm) {  // every rank allocates the union in global packet order
      VP_TRY(union_exchange(c, nmiss, now));
      if (owner) VP_TRY(tbl_owner_reserve(c, t, union_n));
      VP_TRY(tbl_new_keys(c, t, NewKeys{union_n, w.skey}, c->seq, nullptr));
      a.t = tbl_dev(t);  // the buckets may have been rebuilt
      union_stamp<<<grid_for(union_n), 256, 0, c->stream>>>(
          w.first, w.assign, w.skey, w.unow, union_n, c->seq, t.ts, t.tseq);
      VP_HIP(hipGetLastError());
    } else {
      VP_TRY(tbl_new_keys(c, t, NewKeys{nmiss, w.miss_sorted}, c->seq, nullptr));
      a.t = tbl_dev(t);  // a rebuild may have moved the buckets
    }
    if (nmiss) {
      nat_miss_finish<<<grid_for(nmiss), 256, 0, c->stream>>>(
          a, w.miss_sorted, nmiss, w.scratch, w.rep + union_off, w.assign, nullptr);
      VP_HIP(hipGetLastError());
      VP_TRY(tbl_late_touches(c, t, w.miss_sorted, nullptr, nmiss, 256,
                              (nmiss + 255) / 256, w.log, now, seq0));
    }
    *allocated |= 1u;
  }
  if (ndefer) {
    nat_defer_finish<<<grid_for(ndefer), 256, 0, c->stream>>>(a, w.defer, ndefer);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_late_touches(c, t, w.defer, nullptr, ndefer, 256, (ndefer + 255) / 256,
                            w.log, now, seq0));
  }
  if ((union_n && !nku) || ndefer) VP_TRY(read_ctl(c, t));  // (unsorted: read already)
  // steady state (every packet a phase-A hit): the frames and ports are
  // complete (the control copy waited for phase A); only the fold of the
  // stamps may still run — unless it reads the caller's time array, which
  // the caller may reuse as soon as the call returns
  c->fold_pending = !b->now && !nre && !nmiss && !ndefer && !union_n && !ovf;
  // phase A appended nothing and nothing ran after its counts were read:
  // the counters are still zero for the next segment
  t.ctl_clean = !nre && !nmiss && !ndefer && !union_n && !ovf;
  return 0;
}

// Whole batch: segments without expiry (run_batch, vp_table.hip).
int nat_process_device(vp_ctx *c, const vp_dev_batch *b) {
  ExpiringTable tabs[1] = {{&c->ft, nat_cutoff}};
  return run_batch(c, b, tabs, 1, nat_segment);
}

int nat_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys) {
  return tbl_dump(c, c->ft, alloc, ts, reinterpret_cast<uint32_t *>(keys));
}

// ---------------------------------------------------- vp_process_one --
// Contexts whose server may run: stopped at exit, before the runtime's own
// teardown (the kernel would otherwise keep the stream busy until its idle
// exit).
static std::mutex g_srv_mu;
static std::vector<vp_ctx *> g_srv;
static void serve_stop_all() {
  std::vector<vp_ctx *> v;
  {
    std::lock_guard<std::mutex> g(g_srv_mu);
    v = g_srv;
  }
  for (vp_ctx *c : v) serve_stop(c);
}

static const bool g_srv_prof = [] {
  const char *e = getenv("VIGPATH_SERVE_PROF");
  return e && atoi(e);
}();
// The server of c leaves (a leave request, then the stream drains); the
// caller holds c->srv_mu. Does not touch g_srv.
static hipError_t serve_halt(vp_ctx *c) {
  ServeBox *bx = c->sbox;
  const uint32_t req = ++c->srv_req;
  bx->msg[0][0] = kServeLeave;
  __atomic_store_n(&bx->msg[0][3], req, __ATOMIC_RELEASE);
  const hipError_t e = hipStreamSynchronize(c->stream);
  // (the kernel is gone: the leave request counts as answered for the next one)
  __atomic_store_n(&bx->ans, (uint64_t)req, __ATOMIC_RELEASE);
  c->srv_on = false;
  if (g_srv_prof && c->srv_prof[5] > 0) {
    const double n = c->srv_prof[5];
    fprintf(stderr,
            "vigpath serve: %.0f packets, us/packet: host call %.2f, bell->seen %.2f "
            "(idle poll), load %.2f, packet %.2f (LAN: hash %.2f, table %.2f, rewrite %.2f), "
            "store+answer %.2f; shader clock %.0f MHz\n",
            n, c->srv_prof[0] / n, c->srv_prof[1] / n, c->srv_prof[2] / n, c->srv_prof[3] / n,
            c->srv_prof[6] / std::max(1.0, c->srv_prof[9]),
            c->srv_prof[7] / std::max(1.0, c->srv_prof[9]),
            c->srv_prof[8] / std::max(1.0, c->srv_prof[9]), c->srv_prof[4] / n,
            c->srv_prof[10] / std::max(1e-9, c->srv_prof[3]));
    for (double &x : c->srv_prof) x = 0;
  }
  return e;
}

int serve_stop(vp_ctx *c) {
  if (!c) return 0;
  std::lock_guard<std::recursive_mutex> sg(c->srv_mu);
  if (!c->srv_on) return 0;
  const hipError_t e = serve_halt(c);
  {
    std::lock_guard<std::mutex> g(g_srv_mu);
    g_srv.erase(std::remove(g_srv.begin(), g_srv.end(), c), g_srv.end());
  }
  VP_HIP(e);
  return 0;
}

void serve_free(vp_ctx *c) {
  serve_stop(c);
  if (c->sbox) hipHostFree(c->sbox);
  c->sbox = nullptr;
}

// Another context's resident server on this GPU may share a hardware queue
// with c->stream (GPU_MAX_HW_QUEUES streams' worth): c's server would then
// wait behind it until its idle exit. Stop those first (contexts served by
// another thread right now keep theirs: try_lock).
static void serve_yield(vp_ctx *c) {
  // (under g_srv_mu throughout: a listed context is not destroyed meanwhile,
  // as vp_destroy's serve_stop unlists it under the same lock first)
  std::lock_guard<std::mutex> g(g_srv_mu);
  for (size_t i = 0; i < g_srv.size();) {
    vp_ctx *x = g_srv[i];
    if (x == c || x->gpu != c->gpu || !x->srv_mu.try_lock()) {
      i++;
      continue;
    }
    if (x->srv_on) serve_halt(x);  // (an error shows at x's next call)
    x->srv_mu.unlock();
    g_srv.erase(g_srv.begin() + (ptrdiff_t)i);
  }
}

static int serve_launch(vp_ctx *c) {
  serve_yield(c);
  const FlowTable &t = c->ft;
  NatArgs a{};
  a.t = tbl_dev(t);
  a.crc_tab = c->crc_tab;
  a.macw = c->macw;
  a.wan_macw0 = c->wan_macw[0];
  a.wan_macw1 = c->wan_macw[1];
  a.wan_macw2 = c->wan_macw[2];
  a.ext_ip = c->nat.external_addr;
  a.wan = c->nat.wan_device;
  a.start_port = c->nat.start_port;
  a.n_dev = c->nat.n_devices;
  ServeBox *dbox = nullptr;
  VP_HIP(hipHostGetDevicePointer((void **)&dbox, c->sbox, 0));
  // polling waves (VIGPATH_SERVE_WAVES: 1, 2 or 4) and their stagger
  // (VIGPATH_SERVE_GAP, wall-clock ticks of 10 ns)
  static const uint32_t waves = [] {
    const char *e = getenv("VIGPATH_SERVE_WAVES");
    const int v = e ? atoi(e) : 1;
    return v == 4 ? 4u : v == 2 ? 2u : 1u;
  }();
  static const uint32_t gap = [] {
    const char *e = getenv("VIGPATH_SERVE_GAP");
    return e ? (uint32_t)std::min(127, std::max(0, atoi(e))) : 35u;
  }();
  static const uint32_t after = [] {  // (wall-clock ticks of 10 ns, < 256)
    const char *e = getenv("VIGPATH_SERVE_AFTER");
    // (45: 4.59-4.65 us per packet, 60: 4.73-4.83, 0: 5.41-5.80 through
    // nf.c's loop, profiles/r06o_serve_after.txt, r06p_serve_after_sweep.txt)
    return e ? (uint32_t)std::min(255, std::max(0, atoi(e))) : 45u;
  }();
  static const uint32_t up = [] {  // (VIGPATH_SERVE_UP: ticks added after a late poll)
    const char *e = getenv("VIGPATH_SERVE_UP");
    return e ? (uint32_t)std::min(31, std::max(1, atoi(e))) : 8u;
  }();
  static const uint32_t adapt = [] {  // VIGPATH_SERVE_ADAPT=0: a fixed delay
    const char *e = getenv("VIGPATH_SERVE_ADAPT");
    return e && !atoi(e) ? 0u : 1u;
  }();
  nat_serve<<<1, 64 * waves, 0, c->stream>>>(a, dbox, c->seq, c->srv_idle,
                                             (g_srv_prof ? 1u : 0u) | (gap << 3) |
                                                 (after << 10) | (adapt << 18) | (up << 19));
  VP_HIP(hipGetLastError());
  if (!c->srv_on) {
    static std::once_flag once;
    std::call_once(once, [] { atexit(serve_stop_all); });
    std::lock_guard<std::mutex> g(g_srv_mu);
    g_srv.push_back(c);
  }
  c->srv_on = true;
  return 0;
}

int nat_process_one(vp_ctx *c, uint16_t in_dev, uint8_t *frame, uint16_t len, int64_t now,
                    uint16_t *out) {
  std::lock_guard<std::recursive_mutex> sg(c->srv_mu);
  static const bool off = [] {
    const char *e = getenv("VIGPATH_SERVE");
    return e && !atoi(e);
  }();
  FlowTable &t = c->ft;
  // no expiry due at this packet (run_batch's test for a segment of one)
  const bool ok = !off && !c->comm && len <= kServeFrame && now >= 0 && now >= c->last_now &&
                  nat_cutoff(c, now) <= (int64_t)std::min<uint64_t>(t.ts_floor, (uint64_t)now);
  if (!ok) {
    VP_TRY(serve_stop(c));
    return 1;
  }
  if (!c->sbox || !c->srv_on) VP_HIP(hipSetDevice(c->gpu));  // (HIP calls below)
  if (!c->sbox) {
    VP_HIP(hipHostMalloc((void **)&c->sbox, sizeof(ServeBox),
                         hipHostMallocCoherent | hipHostMallocMapped));
    memset(c->sbox, 0, sizeof(ServeBox));
    c->srv_req = 0;
    int khz = 0;
    VP_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->gpu));
    const char *e = getenv("VIGPATH_SERVE_IDLE_MS");
    c->srv_idle_ms = e ? std::max(1, atoi(e)) : 20;
    c->srv_idle = (uint64_t)std::max(khz, 1) * c->srv_idle_ms;
  }
  if (!c->srv_on) {
    // the batch path may leave a timestamp fold running: the server is
    // queued behind it on the same stream
    VP_TRY(serve_launch(c));
  }
  ServeBox *bx = c->sbox;
  const auto h0 = std::chrono::steady_clock::now();
  // the request chunks (ServeBox): payload words first, then each chunk's
  // tag; chunk 0 last; a longer frame whole through `frame` before them
  const uint32_t req = ++c->srv_req;
  uint32_t m[3 * kServeChunks] = {};
  m[0] = len | ((uint32_t)in_dev << 16);
  m[1] = (uint32_t)(uint64_t)now;
  m[2] = (uint32_t)((uint64_t)now >> 32);
  uint32_t need = 1;
  if (len <= kServeInline) {
    memcpy(&m[3], frame, len);
    need = (12 + len + 11) / 12;
  } else {
    memcpy(bx->frame, frame, len);
  }
  for (uint32_t k = need; k-- > 0;) {
    bx->msg[k][0] = m[3 * k];
    bx->msg[k][1] = m[3 * k + 1];
    bx->msg[k][2] = m[3 * k + 2];
    __atomic_store_n(&bx->msg[k][3], req, __ATOMIC_RELEASE);
  }
  // the answer: chunk 0's tag, then (frames of up to kServeInline bytes) the
  // other chunks' tags, each chunk's bytes final once its tag is the request's
  auto last = h0;  // (need: the chunks the request took, as many as the answer takes)
  auto answered = [&]() {
    for (uint32_t k = 0; k < need; k++)
      if (__atomic_load_n(&bx->amsg[k][3], __ATOMIC_ACQUIRE) != req) return false;
    return true;
  };
  uint32_t spins = 0;
  while (!answered()) {
    __builtin_ia32_pause();
    if (++spins & 255) continue;  // (the clock read every 256 spins, not each)
    const auto nw = std::chrono::steady_clock::now();
    if (nw - last < std::chrono::microseconds(200)) continue;
    last = nw;
    // the kernel left (idle) before it saw the request: launch it again
    VP_HIP(hipSetDevice(c->gpu));
    const hipError_t q = hipStreamQuery(c->stream);
    if (q == hipErrorNotReady) continue;
    VP_HIP(q);
    if (answered()) continue;
    VP_TRY(serve_launch(c));
  }
  const uint32_t res = bx->amsg[0][0];
  if (len <= kServeInline) {
    uint32_t m2[3 * kServeChunks];
    for (uint32_t k = 1; k < need; k++) {
      m2[3 * k] = bx->amsg[k][0];
      m2[3 * k + 1] = bx->amsg[k][1];
      m2[3 * k + 2] = bx->amsg[k][2];
    }
    memcpy(frame, &m2[3], len);
  } else {
    memcpy(frame, bx->frame, len);
  }
  const uint64_t ans = (uint64_t)req | ((uint64_t)res << 32);
  *out = (uint16_t)(ans >> 32);
  if ((ans >> 48) & 1u) t.ts_floor = std::min<uint64_t>(t.ts_floor, (uint64_t)now);
  c->seq += 1;
  c->last_now = now;
  if (g_srv_prof) {  // (device stamps: wall clock ticks, 100 MHz)
    const double us_tick = 1e3 / (double)(c->srv_idle / c->srv_idle_ms);
    c->srv_prof[0] +=
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
    const uint64_t *p = bx->prof;
    c->srv_prof[1] += us_tick * (double)(p[1] - p[0]);
    c->srv_prof[2] += us_tick * (double)(p[2] - p[1]);
    if (p[3] && p[4]) {  // (register-path LAN packets: hash | table | rewrite)
      c->srv_prof[6] += us_tick * (double)(p[3] - p[2]);
      c->srv_prof[7] += us_tick * (double)(p[4] - p[3]);
      c->srv_prof[8] += us_tick * (double)(p[5] - p[4]);
      c->srv_prof[9] += 1;
    }
    c->srv_prof[3] += us_tick * (double)(p[6] - p[2]);
    c->srv_prof[4] += us_tick * (double)(p[7] - p[6]);
    c->srv_prof[10] += (double)(p[9] - p[8]);  // (shader cycles over `packet`: MHz)
    c->srv_prof[5] += 1;
  }
  return 0;
}

void build_flowid_tables(std::vector<uint32_t> &tab) {
  tab.assign(15 * 256, 0);
  for (int j = 0; j < 15; j++)
    build_position_table(&tab[j * 256], kFlowIdPos[j], kFlowIdMsg);
}

}  // namespace vp
