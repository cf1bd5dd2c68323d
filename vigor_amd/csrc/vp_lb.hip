// viglb on MI355X: Maglev-style load balancing over a packet batch.
//
// Reference behaviour (paths relative to the reference repository):
//   nf_process              viglb/lb_main.c:20-68
//   lb_get_backend          viglb/lb_balancer.c:38-112
//   lb_process_heartbit     lb_balancer.c:114-143
//   lb_expire_flows/_backends  lb_balancer.c:145-167 (int64 x1000, no wrap)
//   cht_fill_cht            libvig/verified/cht.c:546-877
//   cht_find_preferred_available_backend  cht.c:969-1062
//
// Two expiring tables: flows (LoadBalancedFlow -> flow index, flow index ->
// backend index) and backends (ip -> backend index, backends[] records).
// Batches are cut where either may expire (run_batch). Inside a segment only
// two things change the state other packets observe: a heartbeat from an
// unknown IP allocates a backend (changes what the CHT scan finds), and a
// WAN packet whose flow points at a dead backend (the flow is erased, freed
// and looked up again). A segment is processed in rounds:
//   phase A (whole segment)  parse + hash + probe; WAN hits whose backend is
//            alive are rewritten at once; heartbeats of known IPs are logged
//            for rejuvenation; new flows (M), stale flows (S) and unknown
//            heartbeat IPs (H) are queued;
//   rounds   a round ends before the first queued WAN packet (M or S) that
//            follows a queued heartbeat, so every queued WAN packet of a
//            round precedes every backend allocation of that round and sees
//            the backend set of the round start. Per round:
//              S: if some backend is alive, free + re-allocate returns the
//                 same flow index (it is the free-list head), so a stale flow
//                 is re-pointed at its CHT choice and rejuvenated; with no
//                 backend alive it is freed (in packet order) and dropped;
//              M: de-duplicated, ranked and allocated in packet order (as
//                 vignat), each first sighting records its CHT choice; with
//                 no backend alive every M packet is dropped, nothing is
//                 allocated;
//              H: de-duplicated, ranked and allocated on the backend table;
//                 the first sighting writes the backend record;
//            later rounds first re-classify their queued packets against
//            the state earlier rounds left (lb_resolve).
// Flow table entry: key words {src_ip, dst_ip, src_port | dst_port << 16,
// protocol | backend_index << 8}; words 0-2 and the low byte of word 3 are
// the LoadBalancedFlow (lb_flow.h:6-12), the upper 24 bits carry
// flow_id_to_backend_id, so a hit resolves in one bucket read.
#include <hip/hip_runtime.h>
#include <cstddef>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(lb)


// LoadBalancedFlow_hash (generated, 5 CRC steps: src_ip, dst_ip, src_port,
// dst_port, protocol): non-zero byte positions of the 20-byte CRC message.
static const int kLbFlowPos[13] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 13, 16};
constexpr int kLbFlowMsg = 20;
// ip_addr hash: one CRC step over the u32 address.
constexpr uint32_t kLbFlowTabs = 13;  // LoadBalancedFlow's CRC byte positions
constexpr int kLbTabs = 13 + 4;        // + ip_addr's four

__device__ __forceinline__ uint32_t lbflow_hash(const uint32_t *T, uint32_t sip,
                                                uint32_t dip, uint32_t sp,
                                                uint32_t dp, uint32_t proto) {
  return T[0 * 256 + (sip & 0xFF)] ^ T[1 * 256 + ((sip >> 8) & 0xFF)] ^
         T[2 * 256 + ((sip >> 16) & 0xFF)] ^ T[3 * 256 + (sip >> 24)] ^
         T[4 * 256 + (dip & 0xFF)] ^ T[5 * 256 + ((dip >> 8) & 0xFF)] ^
         T[6 * 256 + ((dip >> 16) & 0xFF)] ^ T[7 * 256 + (dip >> 24)] ^
         T[8 * 256 + (sp & 0xFF)] ^ T[9 * 256 + ((sp >> 8) & 0xFF)] ^
         T[10 * 256 + (dp & 0xFF)] ^ T[11 * 256 + ((dp >> 8) & 0xFF)] ^
         T[12 * 256 + (proto & 0xFF)];
}
// lbflow_hash for the 64-byte tile, its 13 table reads batched (crc13_lds).
__device__ __forceinline__ uint32_t lbflow_hash_batched(const uint32_t *T, uint32_t sip,
                                                        uint32_t dip, uint32_t sp,
                                                        uint32_t dp, uint32_t proto) {
  return crc13_lds(T, sip & 0xFF, (sip >> 8) & 0xFF, (sip >> 16) & 0xFF, sip >> 24, dip & 0xFF,
                   (dip >> 8) & 0xFF, (dip >> 16) & 0xFF, dip >> 24, sp & 0xFF,
                   (sp >> 8) & 0xFF, dp & 0xFF, (dp >> 8) & 0xFF, proto & 0xFF);
}

__device__ __forceinline__ uint32_t ip_hash(const uint32_t *I, uint32_t ip) {
  return I[0 * 256 + (ip & 0xFF)] ^ I[1 * 256 + ((ip >> 8) & 0xFF)] ^
         I[2 * 256 + ((ip >> 16) & 0xFF)] ^ I[3 * 256 + (ip >> 24)];
}

// map_get on the flow table; *w3 = the entry's word 3 (protocol | backend).
__device__ __forceinline__ uint32_t flow_probe(const TableDev &t, uint32_t h,
                                               uint32_t k0, uint32_t k1,
                                               uint32_t k2, uint32_t proto,
                                               uint32_t *w3) {
  uint32_t b = home_bucket(h, t.bmask, t.mix, t.lin);
  for (uint32_t i = 0; i <= t.bmask; i++) {
    const uint4 *q = reinterpret_cast<const uint4 *>(t.bk + b);
    const uint4 e0 = q[0], e1 = q[1], e2 = q[2], ix = q[3];
    if (ix.x == kEmpty) return kNone;
    if (ix.x != kTomb && e0.x == k0 && e0.y == k1 && e0.z == k2 &&
        (e0.w & 0xFF) == proto) {
      *w3 = e0.w;
      return ix.x;
    }
    if (ix.y == kEmpty) return kNone;
    if (ix.y != kTomb && e1.x == k0 && e1.y == k1 && e1.z == k2 &&
        (e1.w & 0xFF) == proto) {
      *w3 = e1.w;
      return ix.y;
    }
    if (ix.z == kEmpty) return kNone;
    if (ix.z != kTomb && e2.x == k0 && e2.y == k1 && e2.z == k2 &&
        (e2.w & 0xFF) == proto) {
      *w3 = e2.w;
      return ix.z;
    }
    b = (b + 1) & t.bmask;
  }
  return kNone;
}

struct LbArgs {
  uint8_t *frames;
  const uint16_t *len;
  const uint16_t *in_dev;  // null: every packet on port in0 (vp_dev_batch.in_port)
  uint32_t in0;
  uint16_t *out;
  uint32_t *log, *log2;  // flow / backend touch logs
  uint32_t slot, p0, p1;
  TableDev ft, bt;
  uint4 *be_rec;
  const uint32_t *cht;
  uint32_t height, bcap;
  const uint32_t *crc_tab;
  const uint32_t *dmacw;
  uint32_t *miss, *stale, *hb;  // queues M, S, H
  uint32_t *hbl;  // phase A: every heartbeat's position (its backend touch)
  uint16_t wan, n_dev;
  // phase A with touch bins (lb_classify64): a hit's touch goes to the bins
  // only and a dropped packet logs nothing; the packets the rounds finish
  // log their touches themselves and are applied after the fold as late
  // touches (lb_segment)
  bool binned;
};

// cht_find_preferred_available_backend: bucket = (u64)hash % height, the
// first allocated backend in its priority list; kNone if none is.
__device__ __forceinline__ uint32_t cht_choose(const LbArgs &a, uint32_t h) {
  const uint32_t *row = a.cht + (size_t)((uint64_t)h % a.height) * a.bcap;
  for (uint32_t p = 0; p < a.bcap; p++) {
    const uint32_t cand = row[p];
    if (a.bt.slot_of[cand] != kNone) return cand;
  }
  return kNone;
}

__device__ __forceinline__ void backend_macs(const LbArgs &a, uint4 rec,
                                             uint32_t nic, uint32_t mw[3]) {
  uint32_t s1 = 0, s2 = 0;  // config.device_macs[nic] (zero if no such NIC)
  if (nic < a.n_dev) {
    s1 = a.dmacw[2 * nic];
    s2 = a.dmacw[2 * nic + 1];
  }
  mw[0] = rec.y;                   // d_addr = backend.mac
  mw[1] = (rec.z & 0xFFFF) | s1;   // d_addr[4..5] | s_addr[0..1]
  mw[2] = s2;                      // s_addr[2..5]
}

// lb_main.c:56-65 on a register frame (IHL 5, total_length <= 50).
__device__ __forceinline__ bool lb_rewrite_fast(const LbArgs &a, RFrame &f,
                                                uint4 rec, uint32_t proto,
                                                uint32_t tl, uint32_t p) {
  const uint32_t nic = rec.z >> 16;
  a.out[p] = (uint16_t)nic;
  if (nic == a.wan) return false;
  f.set32at2(30, rec.x);  // dst_addr = backend.ip
  uint32_t mw[3];
  backend_macs(a, rec, nic, mw);
  f.w[0] = mw[0];
  f.w[1] = mw[1];
  f.w[2] = mw[2];
  fast_checksums(f, proto, tl);
  return true;
}

__device__ __forceinline__ void lb_rewrite_generic(const LbArgs &a, const GFrame &f,
                                                   const L34 &h, uint4 rec,
                                                   uint32_t p) {
  const uint32_t nic = rec.z >> 16;
  a.out[p] = (uint16_t)nic;
  if (nic == a.wan) return;
  f.w32(h.ip + 16, rec.x);
  uint32_t mw[3];
  backend_macs(a, rec, nic, mw);
  set_macs(f, mw);
  set_checksums(f, h.ip, h.l4);
}

// Decision for a parsed packet (phase A / re-classification). Heartbeats are
// logged or queued (H); WAN packets hitting a flow with a live backend are
// handed to `rw` with the backend record; the rest are queued (M / S).
// The backend touch log (log2) is written only for heartbeats: phase A lists
// them (hbl) and the segment applies them as late touches.
// lb_process_heartbit for a packet from a backend; the packet itself is
// dropped. I = the ip_addr hash tables.
__device__ __forceinline__ void lb_heartbeat(const LbArgs &a, const uint32_t *I, uint32_t p,
                                             uint32_t in, uint32_t sip) {
  const uint32_t key[4] = {sip, 0, 0, 0};
  const uint32_t bi = tbl_probe(a.bt, ip_hash(I, sip), key);
  a.out[p] = (uint16_t)in;
  if (!a.binned) a.log[p] = kNone;
  a.log2[p] = bi;  // kNone: queued, the round writes the real entry
  const uint32_t k = wave_append(&a.bt.ctl->defer_count, true);  // heartbeats seen
  if (a.hbl) a.hbl[k] = p;
  if (bi == kNone) a.hb[wave_append(&a.bt.ctl->miss_count, true)] = p;
}

// A WAN packet after its flow lookup (fi, and the entry's word 3): a flow
// with a live backend is handed to `rw` with the backend record; the rest
// are queued (M: no flow, S: its backend is gone).
template <class Rw>
__device__ __forceinline__ bool lb_flow_found(const LbArgs &a, uint32_t p, uint32_t fi,
                                              uint32_t w3, Rw rw, uint32_t *touch) {
  if (fi == kNone) {
    if (!a.binned) a.log[p] = kNone;
    a.miss[wave_append(&a.ft.ctl->miss_count, true)] = p;
    return false;
  }
  const uint32_t bi = w3 >> 8;
  // (both depend on bi only; the record of a dead backend is read and ignored)
  const bool live = a.bt.slot_of[bi] != kNone;
  const uint4 rec = a.be_rec[bi];
  if (!live) {  // backend gone: erase + re-lookup
    if (!a.binned) a.log[p] = kNone;
    a.stale[wave_append(&a.ft.ctl->defer_count, true)] = p;
    return false;
  }
  if (!a.binned) a.log[p] = fi;
  if (touch) *touch = fi;
  return rw(rec);
}

// Decision for a parsed packet (phase A / re-classification). Heartbeats are
// logged or queued (H); WAN packets hitting a flow with a live backend are
// handed to `rw` with the backend record; the rest are queued (M / S).
// The backend touch log (log2) is written only for heartbeats: phase A lists
// them (hbl) and the segment applies them as late touches. T = the flow hash
// tables, I = the ip_addr hash tables.
template <class Rw>
__device__ __forceinline__ bool lb_decide(const LbArgs &a, const uint32_t *T,
                                          const uint32_t *I, uint32_t p, uint32_t in,
                                          uint32_t sip, uint32_t dip, uint32_t sp,
                                          uint32_t dp, uint32_t proto, Rw rw,
                                          uint32_t *touch = nullptr) {
  if (in != a.wan) {
    lb_heartbeat(a, I, p, in, sip);
    return false;
  }
  uint32_t w3 = 0;
  const uint32_t fi =
      flow_probe(a.ft, lbflow_hash(T, sip, dip, sp, dp, proto), sip, dip,
                 sp | (dp << 16), proto, &w3);
  return lb_flow_found(a, p, fi, w3, rw, touch);
}

__device__ __forceinline__ void lb_generic_a(const LbArgs &a, const uint32_t *T,
                                             const uint32_t *I,
                                             uint32_t p) {
  const GFrame f{a.frames + (size_t)p * a.slot, a.slot};
  const uint32_t in = port_of(a.in_dev, a.in0, p);
  const L34 h = parse_l34(f, a.len[p]);
  if (!h.ok) {
    a.out[p] = (uint16_t)in;
    if (!a.binned) a.log[p] = kNone;
    return;
  }
  const uint32_t proto = f.r8(h.ip + 9);
  const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
  const uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
  lb_decide(a, T, I, p, in, sip, dip, sp, dp, proto, [&](uint4 rec) {
    lb_rewrite_generic(a, f, h, rec, p);
    return false;
  });
}

__device__ __forceinline__ void lb_load_tables(uint32_t *T, const uint32_t *g) {
  for (uint32_t i = threadIdx.x; i < kLbTabs * 256; i += blockDim.x) T[i] = g[i];
  __syncthreads();
}

// Phase A for 64-byte slots (frames64_tiles, vp_device.h): frames 1 KiB
// contiguous per load through the wave's LDS tile, and a WAN packet's flow
// bucket gathered cooperatively (four lanes per 64-byte row) between the
// issue and finish halves, as vignat's tiles do. LDS holds the 13 flow-hash
// position tables and the allocation-order layout's four byte tables; the
// backend-address tables (heartbeats only) are read from global memory.
struct LbPend {
  uint32_t row;   // the flow's home bucket (kind 2), or kNone
  uint32_t kind;  // 0: done; 1: byte path; 2: WAN flow; 3: heartbeat
};
// The backends (up to 256: the BASELINE config's 256) are staged in LDS
// beside the tables, record and liveness in one 16-byte entry (the backend
// table does not change during phase A: heartbeats wait for the rounds), so a
// hit's backend costs one LDS read instead of a dependent global round trip.
// To make room, the tile loop keeps only the cursors of 256 touch bins and
// the overflow queue's (lb_segment keeps the flow table's bins at 256).
// Each staged backend is what a hit's rewrite needs, ready: bhdr[b] = {ip,
// the three MAC header words (backend_macs, the NIC's source MAC folded
// in)}, bnic[b] = its NIC | live << 16. The NIC's MAC was a global load that
// depended on the backend the row named (row -> backend -> NIC -> MAC): one
// more dependent round trip per packet.
constexpr uint32_t kLbLdsBackends = 256;
constexpr uint32_t kLbCurs = 257;  // bins 0..255, the overflow queue at 256
template <uint32_t W>  // waves per block
__device__ __forceinline__ void lb_tiles(LbArgs a, uint32_t n_all, TouchBins bins) {
  __shared__ uint32_t T[kLbFlowTabs * 256 + 1024];  // + the layout's byte tables
  __shared__ uint4 stage[W][256];
  __shared__ uint32_t cur[kLbCurs];
  __shared__ uint4 bhdr[kLbLdsBackends];
  __shared__ uint32_t bnic[kLbLdsBackends];
  for (uint32_t i = threadIdx.x; i < kLbCurs; i += blockDim.x) cur[i] = 0;
  for (uint32_t i = threadIdx.x; i < kLbFlowTabs * 256; i += blockDim.x) T[i] = a.crc_tab[i];
  const uint32_t *lin = T + kLbFlowTabs * 256;
  if (a.ft.mix == kMixLin)
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[kLbFlowTabs * 256 + i] = a.ft.lin[i];
  const bool lds_be = a.bcap <= kLbLdsBackends;
  if (lds_be)
    for (uint32_t b = threadIdx.x; b < a.bcap; b += blockDim.x) {
      const uint4 r = a.be_rec[b];
      const uint32_t nic = r.z >> 16;
      uint32_t mw[3];
      backend_macs(a, r, nic, mw);
      bhdr[b] = make_uint4(r.x, mw[0], mw[1], mw[2]);
      bnic[b] = nic | (a.bt.slot_of[b] != kNone ? 1u << 16 : 0u);
    }
  __syncthreads();
  const uint32_t *I = a.crc_tab + kLbFlowTabs * 256;  // ip_addr tables (global)
  frames64_tiles<kLbCurs - 1, true, W>(
      a.frames, a.len, a.in_dev, a.p0, a.p1, n_all, stage[threadIdx.x >> 6],
      reinterpret_cast<const uint4 *>(a.ft.bk),
      [&](uint32_t p, const RFrame &f, uint32_t in, uint32_t len, bool mine) {
        LbPend P{kNone, 0};
        if (!mine) return P;
        const uint32_t et = f.w[3] & 0xFFFF;
        const uint32_t ihl = (f.w[3] >> 16) & 0x0F;
        const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
        if (!(et == 0x0008 && ihl == 5 && tl <= 50)) {
          P.kind = 1;  // byte-addressed path (lb_generic_a)
          return P;
        }
        const uint16_t unread = (uint16_t)(len - 14);
        const uint32_t proto = f.w[5] >> 24;
        const bool ok = (unread >= 20) & (unread >= tl) &
                        ((proto == 6) | (proto == 17)) & ((uint32_t)(len - 34) >= 4u);
        if (!ok) {
          a.out[p] = (uint16_t)in;
          if (!a.binned) a.log[p] = kNone;
          return P;
        }
        if (in != a.wan) {
          P.kind = 3;
          return P;
        }
        const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
        P.kind = 2;
        P.row = home_bucket(lbflow_hash_batched(T, f.u32at2(26), f.u32at2(30), sp, dp, proto),
                            a.ft.bmask, a.ft.mix, lin);
        return P;
      },
      [&](const LbPend &P, const uint4 *row, uint32_t p, RFrame &f, uint32_t in,
          uint32_t len, uint32_t &touch) -> uint32_t {
        if (P.kind == 0) return 0u;
        if (P.kind == 1) {
          lb_generic_a(a, T, I, p);
          return 0u;
        }
        const uint32_t proto = f.w[5] >> 24;
        const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
        const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
        const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
        if (P.kind == 3) {
          lb_heartbeat(a, I, p, in, sip);
          return 0u;
        }
        // map_get on the flow table from the gathered home bucket (word 3:
        // protocol byte | backend << 8)
        const uint32_t key[4] = {sip, dip, sp | (dp << 16), proto};
        uint32_t w3 = 0;
        bool done;
        uint32_t fi = bucket_match<0xFFu>(row[0], row[1], row[2], row[3], key, &done, &w3);
        if (!done)
          fi = tbl_probe_from<0xFFu>(a.ft, (P.row + 1) & a.ft.bmask, key, a.ft.bmask, &w3);
        if (lds_be && fi != kNone) {  // a flow: its backend from LDS
          const uint32_t bi = w3 >> 8;
          const uint32_t meta = bnic[bi];
          const uint4 h = bhdr[bi];
          if (meta >> 16) {  // live: lb_main.c:56-65
            if (!a.binned) a.log[p] = fi;
            touch = fi;
            const uint32_t nic = meta & 0xFFFF;
            a.out[p] = (uint16_t)nic;
            if (nic == a.wan) return 0u;
            f.set32at2(30, h.x);  // dst_addr = backend.ip
            f.w[0] = h.y;
            f.w[1] = h.z;
            f.w[2] = h.w;
            fast_checksums(f, proto, tl);
            return 0xFu;
          }
        }
        // (no flow, a backend gone, or backends not staged: the queues)
        const bool rw = lb_flow_found(a, p, fi, w3, [&](uint4 rec) {
          return lb_rewrite_fast(a, f, rec, proto, tl, p);
        }, &touch);
        // dst address, MACs and checksums change bytes 0-47 (and the TCP
        // checksum 50-51): the whole 64-byte slot is stored back, since a
        // partial-line write costs more than a whole one
        return rw ? 0xFu : 0u;
      },
      bins, TileQueue{}, cur, 0, 0, a.in0);
}
__global__ __launch_bounds__(256, 4) void lb_classify64(LbArgs a, uint32_t n_all,
                                                       TouchBins bins) {
  lb_tiles<4>(a, n_all, bins);
}
// one 1024-thread block per CU (as vignat's nat_classify64w; VIGPATH_LB_WAVES)
__global__ __launch_bounds__(1024, 1) void lb_classify64w(LbArgs a, uint32_t n_all,
                                                         TouchBins bins) {
  lb_tiles<16>(a, n_all, bins);
}

__global__ __launch_bounds__(256) void lb_classify(LbArgs a) {
  __shared__ uint32_t T[kLbTabs * 256];
  lb_load_tables(T, a.crc_tab);
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += gridDim.x * blockDim.x)
    lb_generic_a(a, T, T + kLbFlowTabs * 256, p);
}

// Re-classify queued packets (unmodified frames) against the current state.
__global__ void lb_resolve(LbArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x)
    lb_generic_a(a, a.crc_tab, a.crc_tab + kLbFlowTabs * 256, list[j]);
}

struct Parsed {
  GFrame f;
  L34 h;
  uint32_t sip, dip, sp, dp, proto;
};
__device__ __forceinline__ Parsed lb_parse(const LbArgs &a, uint32_t p) {
  Parsed r;
  r.f = GFrame{a.frames + (size_t)p * a.slot, a.slot};
  r.h = parse_l34(r.f, a.len[p]);
  r.proto = r.f.r8(r.h.ip + 9);
  r.sp = r.f.r16(r.h.l4);
  r.dp = r.f.r16(r.h.l4 + 2);
  r.sip = r.f.r32(r.h.ip + 12);
  r.dip = r.f.r32(r.h.ip + 16);
  return r;
}

// Stale flows with some backend alive: free + allocate hands back the same
// index, so the flow keeps it, points at its CHT choice (every packet of the
// flow computes the same choice) and is rejuvenated.
__global__ void lb_stale_reassign(LbArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const Parsed q = lb_parse(a, p);
    const uint32_t h = lbflow_hash(a.crc_tab, q.sip, q.dip, q.sp, q.dp, q.proto);
    uint32_t w3 = 0;
    const uint32_t fi =
        flow_probe(a.ft, h, q.sip, q.dip, q.sp | (q.dp << 16), q.proto, &w3);
    const uint32_t c = cht_choose(a, h);
    const uint32_t e = a.ft.slot_of[fi];
    a.ft.bk[e >> 2].k[e & 3][3] = q.proto | (c << 8);
    a.log[p] = fi;
    lb_rewrite_generic(a, q.f, q.h, a.be_rec[c], p);
  }
}

// Stale flows with no backend alive (single thread, packet order): the first
// packet of each erases the key and frees the index onto the free-list front
// (double-chain-impl.c:1968-1981); every such packet is dropped.
__global__ void lb_stale_free_seq(LbArgs a, const uint32_t *list, uint32_t n) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Ctl *ctl = a.ft.ctl;
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t p = list[j];
    const Parsed q = lb_parse(a, p);
    const uint32_t h = lbflow_hash(a.crc_tab, q.sip, q.dip, q.sp, q.dp, q.proto);
    uint32_t w3 = 0;
    const uint32_t fi =
        flow_probe(a.ft, h, q.sip, q.dip, q.sp | (q.dp << 16), q.proto, &w3);
    a.out[p] = port_of(a.in_dev, a.in0, p);  // backend.nic = wan device = in
    a.log[p] = kNone;
    if (fi == kNone) continue;  // freed by an earlier packet of the flow
    const uint32_t e = a.ft.slot_of[fi];
    a.ft.bk[e >> 2].idx[e & 3] = kTomb;
    a.ft.slot_of[fi] = kNone;
    a.ft.stack[ctl->stack_top++] = fi;
    ctl->n_live--;
    ctl->sh_live--;  // (the layout and rebuild checks count this rank's entries)
    ctl->n_tomb++;
  }
}

__global__ void lb_miss_keys(LbArgs a, const uint32_t *list, uint32_t n,
                             uint32_t *mkey, uint32_t *mhash) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const Parsed q = lb_parse(a, list[j]);
    uint32_t *k = mkey + 4 * (size_t)j;
    k[0] = q.sip;
    k[1] = q.dip;
    k[2] = q.sp | (q.dp << 16);
    k[3] = q.proto;
    mhash[j] = lbflow_hash(a.crc_tab, q.sip, q.dip, q.sp, q.dp, q.proto);
  }
}

// New flows (some backend alive): every packet goes to its CHT choice (also
// when the flow table is full, lb_balancer.c:66 "doesn't matter if we can't
// insert"); the first sighting records the choice as the flow's backend.
__global__ void lb_miss_finish(LbArgs a, const uint32_t *list, uint32_t n,
                               const uint32_t *mkey, const uint32_t *mhash,
                               const uint32_t *scratch, const uint32_t *rep,
                               const uint32_t *assign) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint32_t j0 = scratch[rep[j]];
    const uint32_t idx = assign[j0];
    const uint32_t c = cht_choose(a, mhash[j]);
    if (idx != kNone && j0 == j) {
      const uint32_t e = a.ft.slot_of[idx];
      a.ft.bk[e >> 2].k[e & 3][3] = mkey[4 * (size_t)j + 3] | (c << 8);
    }
    a.log[p] = idx;
    const Parsed q = lb_parse(a, p);
    lb_rewrite_generic(a, q.f, q.h, a.be_rec[c], p);
  }
}

__global__ void lb_drop_list(LbArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    a.out[p] = port_of(a.in_dev, a.in0, p);
    a.log[p] = kNone;
  }
}

__global__ void lb_hb_keys(LbArgs a, const uint32_t *list, uint32_t n,
                           uint32_t *mkey, uint32_t *mhash) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const Parsed q = lb_parse(a, list[j]);
    uint32_t *k = mkey + 4 * (size_t)j;
    k[0] = q.sip;
    k[1] = k[2] = k[3] = 0;
    mhash[j] = ip_hash(a.crc_tab + kLbFlowTabs * 256, q.sip);
  }
}

// New backends: the first sighting of an IP writes backends[idx] = {ip,
// s_addr, in device} (lb_balancer.c:119-133).
__global__ void lb_hb_finish(LbArgs a, const uint32_t *list, uint32_t n,
                             const uint32_t *scratch, const uint32_t *rep,
                             const uint32_t *assign) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint32_t j0 = scratch[rep[j]];
    const uint32_t idx = assign[j0];
    a.log2[p] = idx;
    if (idx == kNone || j0 != j) continue;
    const GFrame f{a.frames + (size_t)p * a.slot, a.slot};
    const L34 h = parse_l34(f, a.len[p]);
    const uint32_t m0 = f.r32(6), m1 = f.r16(10);
    a.be_rec[idx] = make_uint4(f.r32(h.ip + 12), m0, m1 | (port_of(a.in_dev, a.in0, p) << 16), 0);
  }
}

// =============================================================== host ==

static inline int64_t lb_flow_cutoff(const vp_ctx *c, int64_t t) {
  return (int64_t)((uint64_t)t - (uint64_t)((int64_t)c->lb.flow_expiration_time * 1000));
}
static inline int64_t lb_backend_cutoff(const vp_ctx *c, int64_t t) {
  return (int64_t)((uint64_t)t -
                   (uint64_t)((int64_t)c->lb.backend_expiration_time * 1000));
}

static int sort_list(vp_ctx *c, const uint32_t *in, uint32_t *out, uint32_t n) {
  if (!n) return 0;
  size_t need = 0;
  hipcub::DeviceRadixSort::SortKeys(nullptr, need, in, out, (int)n, 0, 32, c->stream);
  VP_TRY(cub_reserve(c, need));
  VP_HIP(hipcub::DeviceRadixSort::SortKeys(c->ws.cub_tmp, c->ws.cub_bytes, in, out,
                                           (int)n, 0, 32, c->stream));
  return 0;
}

struct Queues {
  const uint32_t *m, *s, *h;
  uint32_t nm, ns, nh;
};

// One round (see the header): stale flows, new flows, then new backends.
static int lb_round(vp_ctx *c, LbArgs &a, const Queues &q, uint32_t *allocated) {
  Workspace &w = c->ws;
  VP_TRY(read_ctl(c, c->ft2));
  const bool alive = c->ft2.h_ctl.n_live > 0;
  if (q.ns) {
    if (alive) {
      lb_stale_reassign<<<grid_for(q.ns), 256, 0, c->stream>>>(a, q.s, q.ns);
    } else {
      lb_stale_free_seq<<<1, 64, 0, c->stream>>>(a, q.s, q.ns);
      VP_HIP(hipGetLastError());
      VP_TRY(tbl_check_tombs(c, c->ft));
      a.ft = tbl_dev(c->ft);
    }
    VP_HIP(hipGetLastError());
  }
  if (q.nm) {
    if (alive) {
      lb_miss_keys<<<grid_for(q.nm), 256, 0, c->stream>>>(a, q.m, q.nm, w.mkey,
                                                          w.mhash);
      VP_HIP(hipGetLastError());
      VP_TRY(tbl_new_keys(c, c->ft, NewKeys{q.nm, q.m}, c->seq, nullptr));
      a.ft = tbl_dev(c->ft);
      lb_miss_finish<<<grid_for(q.nm), 256, 0, c->stream>>>(
          a, q.m, q.nm, w.mkey, w.mhash, w.scratch, w.rep, w.assign);
      *allocated |= 1u;
    } else {
      lb_drop_list<<<grid_for(q.nm), 256, 0, c->stream>>>(a, q.m, q.nm);
    }
    VP_HIP(hipGetLastError());
  }
  if (q.nh) {
    lb_hb_keys<<<grid_for(q.nh), 256, 0, c->stream>>>(a, q.h, q.nh, w.mkey, w.mhash);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_new_keys(c, c->ft2, NewKeys{q.nh, q.h}, c->seq, nullptr));
    a.bt = tbl_dev(c->ft2);
    lb_hb_finish<<<grid_for(q.nh), 256, 0, c->stream>>>(a, q.h, q.nh, w.scratch,
                                                        w.rep, w.assign);
    VP_HIP(hipGetLastError());
    *allocated |= 2u;
  }
  return 0;
}

static int zero_queues(vp_ctx *c) {
  VP_HIP(hipMemsetAsync(&c->ft.ctl->miss_count, 0, 8, c->stream));  // M, S
  VP_HIP(hipMemsetAsync(&c->ft2.ctl->miss_count, 0, 4, c->stream));  // H
  return 0;
}

static int lb_segment(vp_ctx *c, const vp_dev_batch *b, const NowSpec &now,
                      uint32_t p0, uint32_t p1, float *ms, int *launches,
                      uint32_t *allocated) {
  Workspace &w = c->ws;
  LbArgs a{};
  a.frames = b->frames;
  a.len = b->len;
  a.in_dev = b->in_dev;
  a.in0 = b->in_dev ? 0u : b->in_port;  // (port_of: exactly one is live)
  a.out = b->out_dev;
  a.log = w.log;
  a.log2 = w.log2;
  a.slot = b->slot;
  a.p0 = p0;
  a.p1 = p1;
  a.ft = tbl_dev(c->ft);
  a.bt = tbl_dev(c->ft2);
  a.be_rec = c->be_rec;
  a.cht = c->cht;
  a.height = c->lb.cht_height;
  a.bcap = c->lb.backend_capacity;
  a.crc_tab = c->crc_tab;
  a.dmacw = c->dmacw;
  a.miss = w.miss;
  a.stale = w.defer;
  a.hb = w.aux;
  a.hbl = w.hbl;
  a.wan = c->lb.wan_device;
  a.n_dev = c->lb.n_devices;

  // the counters are still zero after a segment that queued nothing (no
  // misses, stale flows, heartbeats or bin overflows): no reset launches
  if (!c->ft.ctl_clean) {
    VP_TRY(zero_queues(c));
    VP_HIP(hipMemsetAsync(&c->ft2.ctl->defer_count, 0, 4, c->stream));  // heartbeats
    VP_HIP(hipMemsetAsync(&c->ft.ctl->touch_ovf, 0, 4, c->stream));
  }
  c->ft.ctl_clean = false;
  BinsPlan bp{};
  const bool tiles64 = b->slot == 64 && c->coalesced_io;
  VP_HIP(ev_record(c->ktime, c->ev0, c->stream));
  if (tiles64) {
    // the flow touches go to the touch bins (256 of them: lb_classify64 keeps
    // 256 bin cursors; a larger table logs every touch and refolds the log)
    static const uint32_t lw = [] {  // waves per block (VIGPATH_LB_WAVES: 4 or 16)
      const char *e = getenv("VIGPATH_LB_WAVES");
      return e && atoi(e) == 16 ? 16u : 4u;
    }();
    const void *k = lw == 16 ? (const void *)lb_classify64w : (const void *)lb_classify64;
    VP_TRY(tbl_bins_plan(c, c->ft, k, p0, p1, &bp, lw));
    if (bp.on && bp.bins.bbits > 8) bp = BinsPlan{};
    const uint32_t tiles = (p1 - (p0 & ~63u) + 63) / 64;
    const uint32_t grid = bp.on ? bp.grid : resident_grid(k, (tiles + lw - 1) / lw, 64 * (int)lw);
    LbArgs a64 = a;
    a64.binned = bp.on;
    c->last_kernel = lw == 16 ? "lb_classify64w" : "lb_classify64";
    if (lw == 16)
      lb_classify64w<<<grid, 1024, 0, c->stream>>>(a64, b->n, bp.bins);
    else
      lb_classify64<<<grid, 256, 0, c->stream>>>(a64, b->n, bp.bins);
  } else {
    lb_classify<<<grid_for(p1 - p0), 256, 0, c->stream>>>(a);
  }
  VP_HIP(hipGetLastError());
  VP_HIP(ev_record(c->ktime, c->ev1, c->stream));
  a.hbl = nullptr;  // re-classification rounds list no heartbeat twice
  if (bp.on) {
    // optimistic fold; its first thread publishes phase A's counts (the flow
    // table's control block, and the backend table's H and heartbeat counts
    // as extra words), which the host waits for while the fold runs
    static_assert(offsetof(Ctl, defer_count) == offsetof(Ctl, miss_count) + 4, "H, heartbeats");
    const uint32_t epoch = ++c->ft.pub_epoch;
    VP_TRY(tbl_bins_reduce(c, c->ft, bp, p0, now, c->seq,
                           PubArgs{c->ft.d_pub, c->ft.ctl, epoch, &c->ft2.ctl->miss_count,
                                   nullptr, 2, 0}));
    VP_TRY(tbl_wait_pub(c, c->ft, epoch));
    c->ft2.h_ctl.miss_count = c->ft.h_pub->xtra[0];
    c->ft2.h_ctl.defer_count = c->ft.h_pub->xtra[1];
  } else {
    // phase A's counts are copied out before the fold and waited for alone
    VP_TRY(read_ctl2_post(c, c->ft2, c->ft));
    VP_TRY(tbl_touch_reduce(c, c->ft, w.log, p0, p1, now, c->seq));
    VP_TRY(read_ctl2_wait(c, c->ft2, c->ft));
  }
  float kms = 0.f;
  VP_HIP(ev_ms(c->ktime, c->ev0, c->ev1, &kms));
  *ms += kms;
  *launches += 1;
  const uint32_t nm = c->ft.h_ctl.miss_count, ns = c->ft.h_ctl.defer_count;
  const uint32_t nh = c->ft2.h_ctl.miss_count, nhb = c->ft2.h_ctl.defer_count;
  const bool ovf = bp.on && c->ft.h_ctl.touch_ovf != 0;

  std::vector<uint32_t> M_all, S_all;  // phase A's queues (multi-round segments)
  if (nm || ns || nh) {
    VP_TRY(sort_list(c, w.miss, w.miss_sorted, nm));
    VP_TRY(sort_list(c, w.defer, w.defer_sorted, ns));
    VP_TRY(sort_list(c, w.aux, w.aux_sorted, nh));
    if (!nh) {
      VP_TRY(lb_round(c, a, Queues{w.miss_sorted, w.defer_sorted, nullptr, nm, ns, 0},
                      allocated));
    } else {
      std::vector<uint32_t> M(nm), S(ns), H(nh);
      VP_HIP(hipMemcpyAsync(M.data(), w.miss_sorted, 4ull * nm,
                            hipMemcpyDeviceToHost, c->stream));
      VP_HIP(hipMemcpyAsync(S.data(), w.defer_sorted, 4ull * ns,
                            hipMemcpyDeviceToHost, c->stream));
      VP_HIP(hipMemcpyAsync(H.data(), w.aux_sorted, 4ull * nh,
                            hipMemcpyDeviceToHost, c->stream));
      VP_HIP(hipStreamSynchronize(c->stream));
      M_all = M;
      S_all = S;
      uint32_t im = 0, is = 0, ih = 0;
      bool first = true;
      std::vector<uint32_t> rl;
      while (im < nm || is < ns || ih < nh) {
        uint32_t end = p1;
        if (ih < nh) {  // stop before the first WAN packet after H[ih]
          const uint32_t h = H[ih];
          const uint32_t wm = (uint32_t)(std::lower_bound(M.begin() + im, M.end(), h) - M.begin());
          const uint32_t ws_ = (uint32_t)(std::lower_bound(S.begin() + is, S.end(), h) - S.begin());
          end = std::min(wm < nm ? M[wm] : p1, ws_ < ns ? S[ws_] : p1);
        }
        const uint32_t jm = (uint32_t)(std::lower_bound(M.begin() + im, M.end(), end) - M.begin());
        const uint32_t js = (uint32_t)(std::lower_bound(S.begin() + is, S.end(), end) - S.begin());
        const uint32_t jh = (uint32_t)(std::lower_bound(H.begin() + ih, H.end(), end) - H.begin());
        if (first) {
          VP_TRY(lb_round(c, a,
                          Queues{w.miss_sorted + im, w.defer_sorted + is,
                                 w.aux_sorted + ih, jm - im, js - is, jh - ih},
                          allocated));
          first = false;
        } else {
          // re-classify against the state earlier rounds left
          rl.assign(M.begin() + im, M.begin() + jm);
          rl.insert(rl.end(), S.begin() + is, S.begin() + js);
          rl.insert(rl.end(), H.begin() + ih, H.begin() + jh);
          if (!rl.empty()) {
            VP_HIP(hipMemcpyAsync(w.rlist, rl.data(), 4 * rl.size(),
                                  hipMemcpyHostToDevice, c->stream));
            VP_TRY(zero_queues(c));
            a.ft = tbl_dev(c->ft);
            a.bt = tbl_dev(c->ft2);
            lb_resolve<<<grid_for(rl.size()), 256, 0, c->stream>>>(a, w.rlist,
                                                                  (uint32_t)rl.size());
            VP_HIP(hipGetLastError());
            VP_TRY(read_ctl2(c, c->ft2, c->ft));
            const uint32_t rm = c->ft.h_ctl.miss_count, rs = c->ft.h_ctl.defer_count;
            const uint32_t rh = c->ft2.h_ctl.miss_count;
            VP_TRY(sort_list(c, w.miss, w.miss_sorted, rm));
            VP_TRY(sort_list(c, w.defer, w.defer_sorted, rs));
            VP_TRY(sort_list(c, w.aux, w.aux_sorted, rh));
            VP_TRY(lb_round(c, a, Queues{w.miss_sorted, w.defer_sorted, w.aux_sorted,
                                         rm, rs, rh},
                            allocated));
          }
        }
        a.ft = tbl_dev(c->ft);
        a.bt = tbl_dev(c->ft2);
        im = jm;
        is = js;
        ih = jh;
      }
    }
  }
  if (bp.on) {
    // the fold applied phase A's binned touches; the packets the rounds
    // finished (the M and S queues) and the touches a full bin slice queued
    // follow as late touches (last toucher in packet order still wins)
    if (ovf)
      VP_TRY(tbl_late_touches(c, c->ft, bp.bins.oent, bp.bins.ocnt, 0, bp.range, bp.grid,
                              w.log, now, c->seq));
    if (nm || ns) {
      const uint32_t *lm = w.miss_sorted, *ls = w.defer_sorted;
      if (nh) {  // (the rounds re-sorted the queues: the phase-A lists again)
        VP_HIP(hipMemcpyAsync(w.rlist, M_all.data(), 4ull * nm, hipMemcpyHostToDevice,
                              c->stream));
        VP_HIP(hipMemcpyAsync(w.rlist + nm, S_all.data(), 4ull * ns, hipMemcpyHostToDevice,
                              c->stream));
        lm = w.rlist;
        ls = w.rlist + nm;
      }
      if (nm)
        VP_TRY(tbl_late_touches(c, c->ft, lm, nullptr, nm, 256, (nm + 255) / 256, w.log, now,
                                c->seq));
      if (ns)
        VP_TRY(tbl_late_touches(c, c->ft, ls, nullptr, ns, 256, (ns + 255) / 256, w.log, now,
                                c->seq));
    }
  } else if (nm || ns || nh) {
    // the rounds completed the log: refold it
    VP_TRY(tbl_touch_reduce(c, c->ft, w.log, p0, p1, now, c->seq));
  }
  if (nhb)  // the heartbeats' backend touches (log2 holds only theirs)
    VP_TRY(tbl_late_touches(c, c->ft2, w.hbl, nullptr, nhb, 256, (nhb + 255) / 256,
                            w.log2, now, c->seq));
  // steady state: frames and ports complete, only the flow fold may still
  // run (not when it reads the caller's time array)
  c->fold_pending = !(nm || ns || nh || ovf || nhb) && !b->now;
  c->ft.ctl_clean = !(nm || ns || nh || ovf || nhb);
  return 0;
}

int lb_process_device(vp_ctx *c, const vp_dev_batch *b) {
  ExpiringTable tabs[2] = {{&c->ft, lb_flow_cutoff}, {&c->ft2, lb_backend_cutoff}};
  return run_batch(c, b, tabs, 2, lb_segment);
}

void build_lb_tables(std::vector<uint32_t> &tab) {
  tab.assign(kLbTabs * 256, 0);
  for (int j = 0; j < 13; j++)
    build_position_table(&tab[j * 256], kLbFlowPos[j], kLbFlowMsg);
  for (int j = 0; j < 4; j++) build_position_table(&tab[(13 + j) * 256], j, 4);
}

// cht_fill_cht (cht.c:546-877): backend i visits bucket
// (31 i mod h + ((i mod (h-1)) + 1) j) mod h in round j; each bucket's
// priority list is filled round by round, backends in index order.
void lb_fill_cht(uint32_t height, uint32_t bcap, std::vector<uint32_t> &cht) {
  cht.assign((size_t)height * bcap, 0);
  std::vector<uint32_t> fill(height, 0);
  for (uint32_t j = 0; j < height; j++)
    for (uint32_t i = 0; i < bcap; i++) {
      const uint64_t off = (uint64_t)(uint32_t)(i * 31u) % height;
      const uint64_t shift = (uint64_t)i % (height - 1) + 1;
      const uint32_t bucket = (uint32_t)((off + shift * j) % height);
      cht[(size_t)bucket * bcap + fill[bucket]++] = i;
    }
}

int lb_dump(vp_ctx *c, uint8_t *f_alloc, int64_t *f_ts, uint8_t *f_keys,
            uint32_t *f_backend, uint8_t *b_alloc, int64_t *b_ts, uint32_t *b_ip,
            uint8_t *b_mac, uint16_t *b_nic) {
  const uint32_t fc = c->ft.cap, bc = c->ft2.cap;
  std::vector<uint32_t> keys(4ull * std::max(fc, bc));
  VP_TRY(tbl_dump(c, c->ft, f_alloc, f_ts, keys.data()));
  for (uint32_t i = 0; i < fc; i++) {
    const uint32_t *k = &keys[4ull * i];
    uint8_t *o = f_keys + 16ull * i;
    memcpy(o, k, 12);
    o[12] = (uint8_t)k[3];
    o[13] = o[14] = o[15] = 0;
    f_backend[i] = k[3] >> 8;
  }
  VP_TRY(tbl_dump(c, c->ft2, b_alloc, b_ts, keys.data()));
  std::vector<uint4> rec(bc);
  VP_HIP(hipMemcpy(rec.data(), c->be_rec, sizeof(uint4) * bc, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < bc; i++) {
    b_ip[i] = rec[i].x;
    memcpy(b_mac + 6ull * i, &rec[i].y, 4);
    memcpy(b_mac + 6ull * i + 4, &rec[i].z, 2);
    b_nic[i] = (uint16_t)(rec[i].z >> 16);
  }
  return 0;
}

}  // namespace vp
