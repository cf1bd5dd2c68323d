// vigfw on MI355X: batch classification + flow-state update + MAC rewrite.
//
// Reference behaviour (paths relative to the reference repository):
//   nf_process            vigfw/fw_main.c:21-80
//   flow manager          vigfw/fw_flowmanager.c:20-86
//   state                 vigfw/dataspec.ml:5-11 (fm, fv, int_devices, heap)
// Same segment / phase structure as vignat (vp_nat.hip header):
//   phase A  parse + hash; LAN packets whose FlowId exists at segment start
//            and WAN packets whose reversed FlowId exists are forwarded and
//            touch their flow; LAN misses and WAN misses are queued;
//   phase B  LAN misses: de-duplicated, ranked, given dchain indices in packet
//            order; the first sighting's input device is the flow's
//            int_devices entry; every LAN packet goes out on the WAN device,
//            table full or not (fw_flowmanager.c:49-53);
//   phase C  WAN misses look the reversed key up again: a flow allocated
//            earlier in packet order is a hit, anything else is dropped.
// The frame rewrite is the two MAC addresses only (fw_main.c:76-77).
//
// Table entry: key words {src_port | dst_port << 16, src_ip, dst_ip,
// protocol | int_device << 8}; the key is FlowId (vigfw/flow.h:3-9, 13 bytes
// + padding), the int_devices vector lives in the padding byte positions,
// and probes compare the protocol byte only (bucket_match<0xFF>).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <vector>

#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(fw)


// FlowId_hash for vigfw's FlowId (generated, codegen/main.ml:328-401): five
// CRC steps src_port, dst_port, src_ip, dst_ip, protocol; non-zero byte
// positions of the 20-byte CRC message.
static const int kFwPos[13] = {0, 1, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr int kFwMsg = 20;
constexpr uint32_t kFwTabs = 13;

__device__ __forceinline__ uint32_t fw_hash(const uint32_t *T, uint32_t sp,
                                            uint32_t dp, uint32_t sip,
                                            uint32_t dip, uint32_t proto) {
  return T[0 * 256 + (sp & 0xFF)] ^ T[1 * 256 + ((sp >> 8) & 0xFF)] ^
         T[2 * 256 + (dp & 0xFF)] ^ T[3 * 256 + ((dp >> 8) & 0xFF)] ^
         T[4 * 256 + (sip & 0xFF)] ^ T[5 * 256 + ((sip >> 8) & 0xFF)] ^
         T[6 * 256 + ((sip >> 16) & 0xFF)] ^ T[7 * 256 + (sip >> 24)] ^
         T[8 * 256 + (dip & 0xFF)] ^ T[9 * 256 + ((dip >> 8) & 0xFF)] ^
         T[10 * 256 + ((dip >> 16) & 0xFF)] ^ T[11 * 256 + (dip >> 24)] ^
         T[12 * 256 + (proto & 0xFF)];
}

struct FwArgs {
  uint8_t *frames;
  const uint16_t *len;
  const uint16_t *in_dev;
  uint16_t *out;
  uint32_t *log;
  uint64_t seq_base;
  uint32_t slot, p0, p1;
  TableDev t;
  const uint32_t *crc_tab;
  const uint32_t *macw;  // per device: d_addr|s_addr header words
  uint32_t *miss;
  uint32_t *defer;
  uint32_t *reprobe;
  uint32_t tileq;  // 64-byte tiles: reprobes go to the block's TileQueue slice
  uint16_t wan, n_dev;
};

__device__ __forceinline__ void fw_macs(const FwArgs &a, uint32_t dst,
                                        uint32_t mw[3]) {
  if (dst < a.n_dev) {
    mw[0] = a.macw[3 * dst];
    mw[1] = a.macw[3 * dst + 1];
    mw[2] = a.macw[3 * dst + 2];
  } else {  // outside the configured devices (reference: out-of-range read)
    mw[0] = mw[1] = mw[2] = 0;
  }
}

// The FlowId a packet looks up: its own 5-tuple on a LAN device, the
// reversed one on the WAN device (fw_main.c:46-53 / 62-68).
__device__ __forceinline__ void fw_key(bool wan, uint32_t sp, uint32_t dp,
                                       uint32_t sip, uint32_t dip, uint32_t proto,
                                       uint32_t key[4]) {
  if (wan) {
    key[0] = dp | (sp << 16);
    key[1] = dip;
    key[2] = sip;
  } else {
    key[0] = sp | (dp << 16);
    key[1] = sip;
    key[2] = dip;
  }
  key[3] = proto;
}

// Generic (byte-addressed) phase A: IP options, any slot size.
__device__ uint32_t fw_generic_a(const FwArgs &a, const uint32_t *T, uint32_t p,
                                 uint32_t in, uint32_t len) {
  GFrame f{a.frames + (size_t)p * a.slot, a.slot};
  const L34 h = parse_l34(f, len);
  if (!h.ok) {  // not IPv4 / not TCP-UDP: drop (fw_main.c:29-40)
    a.out[p] = (uint16_t)in;
    log_put(a.log, p, kNone);
    return kNone;
  }
  const uint32_t proto = f.r8(h.ip + 9);
  const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
  const uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
  const bool wan = in == a.wan;
  uint32_t key[4];
  fw_key(wan, sp, dp, sip, dip, proto, key);
  const uint32_t hh = wan ? fw_hash(T, dp, sp, dip, sip, proto)
                          : fw_hash(T, sp, dp, sip, dip, proto);
  uint32_t w3 = 0;
  const uint32_t idx = tbl_probe<0xFFu>(a.t, hh, key, &w3);
  if (idx == kNone) {
    if (wan)
      a.defer[wave_append(&a.t.ctl->defer_count, true)] = p;
    else
      a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
    log_put(a.log, p, kNone);  // phase B / C write the real entry
    return kNone;
  }
  log_put(a.log, p, idx);
  const uint32_t dst = wan ? (w3 >> 8) : a.wan;
  uint32_t mw[3];
  fw_macs(a, dst, mw);
  set_macs(f, mw);
  a.out[p] = (uint16_t)dst;
  return idx;
}

// Phase A, 64-byte slots in registers (frames64_tiles): fw_issue parses and
// hashes, fw_finish consumes the gathered home bucket.
enum : uint32_t { kFwDone = 0, kFwGeneric = 1, kFwProbe = 2 };
struct FwPend {
  uint32_t kind;
  uint32_t row;  // home bucket (gathered by frames64_tiles) or kNone
};

// T holds the CRC tables, then the layout's byte tables (fw_load_tables).
constexpr uint32_t kFwTabWords = kFwTabs * 256 + 1024;
__device__ __forceinline__ const uint32_t *fw_lin(const uint32_t *T) {
  return T + kFwTabs * 256;
}

__device__ __forceinline__ FwPend fw_issue(const FwArgs &a, const uint32_t *T,
                                           uint32_t p, const RFrame &f,
                                           uint32_t in, uint32_t len, bool mine) {
  FwPend P{kFwDone, kNone};
  if (!mine) return P;
  const uint32_t et = f.w[3] & 0xFFFF;
  const uint32_t ihl = (f.w[3] >> 16) & 0x0F;
  if (!(et == 0x0008 && ihl == 5)) {
    P.kind = kFwGeneric;
    return P;
  }
  // nf_then_get_rte_ipv4_header / nf_then_get_tcpudp_header with IHL = 5
  const uint32_t tl = bswap16((uint16_t)(f.w[4] & 0xFFFF));
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
  const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
  // (WAN packets hash the reversed FlowId; the 13 reads batched, crc13_lds)
  const bool w = in == a.wan;
  const uint32_t s0 = w ? dp : sp, d0 = w ? sp : dp, si = w ? dip : sip, di = w ? sip : dip;
  const uint32_t hh = crc13_lds(T, s0 & 0xFF, (s0 >> 8) & 0xFF, d0 & 0xFF, (d0 >> 8) & 0xFF,
                                si & 0xFF, (si >> 8) & 0xFF, (si >> 16) & 0xFF, si >> 24,
                                di & 0xFF, (di >> 8) & 0xFF, (di >> 16) & 0xFF, di >> 24,
                                proto & 0xFF);
  P.kind = kFwProbe;
  P.row = home_bucket(hh, a.t.bmask, a.t.mix, fw_lin(T));
  return P;
}

__device__ __forceinline__ bool fw_finish(const FwArgs &a, const uint32_t *T,
                                          const FwPend &P, const uint4 *row,
                                          uint32_t p, RFrame &f, uint32_t in,
                                          uint32_t len, uint32_t &touch) {
  if (P.kind == kFwDone) return false;
  if (P.kind == kFwGeneric) {
    touch = fw_generic_a(a, T, p, in, len);  // writes global memory itself
    return false;
  }
  const uint32_t proto = f.w[5] >> 24;
  const uint32_t sp = f.w[8] >> 16, dp = f.w[9] & 0xFFFF;
  const uint32_t sip = f.u32at2(26), dip = f.u32at2(30);
  const bool wan = in == a.wan;
  uint32_t key[4];
  fw_key(wan, sp, dp, sip, dip, proto, key);
  bool done;
  uint32_t w3 = 0;
  const uint32_t idx =
      bucket_match<0xFFu>(row[0], row[1], row[2], row[3], key, &done, &w3);
  if (!done) {  // the bucket is full of other keys: fw_reprobe walks on,
    log_put(a.log, p, kNone);  // so this wave does not wait for a dependent read
    if (a.tileq)
      touch = kReprobe;
    else
      a.reprobe[wave_append(&a.t.ctl->reprobe_count, true)] = p;
    return false;
  }
  if (idx == kNone) {
    if (wan)
      a.defer[wave_append(&a.t.ctl->defer_count, true)] = p;
    else
      a.miss[wave_append(&a.t.ctl->miss_count, true)] = p;
    log_put(a.log, p, kNone);
    return false;
  }
  log_put(a.log, p, idx);
  touch = idx;
  const uint32_t dst = wan ? (w3 >> 8) : a.wan;
  uint32_t mw[3];
  fw_macs(a, dst, mw);
  f.w[0] = mw[0];
  f.w[1] = mw[1];
  f.w[2] = mw[2];
  a.out[p] = (uint16_t)dst;
  return true;
}

// The CRC tables, and behind them the allocation-order layout's byte tables
// when the table uses it (fw_lin(T), vp_table.h kMixLin).
__device__ __forceinline__ void fw_load_tables(uint32_t *T, const FwArgs &a) {
  for (uint32_t i = threadIdx.x; i < kFwTabs * 256; i += blockDim.x) T[i] = a.crc_tab[i];
  if (a.t.mix == kMixLin)
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[kFwTabs * 256 + i] = a.t.lin[i];
  __syncthreads();
}

// Phase A, any slot size: one packet per lane (byte path; no checksum work).
__global__ __launch_bounds__(256) void fw_classify(FwArgs a) {
  __shared__ uint32_t T[kFwTabWords];
  fw_load_tables(T, a);
  for (uint32_t p = a.p0 + blockIdx.x * blockDim.x + threadIdx.x; p < a.p1;
       p += gridDim.x * blockDim.x)
    fw_generic_a(a, T, p, a.in_dev[p], a.len[p]);
}

// Phase A for 64-byte slots: LDS-staged coalesced frame I/O.
__global__ __launch_bounds__(256, 4) void fw_classify64(FwArgs a, uint32_t n_all,
                                                       TouchBins bins, TileQueue rq) {
  __shared__ uint32_t T[kFwTabWords];
  __shared__ uint4 stage[4][256];
  __shared__ uint32_t cur[kCurs];
  for (uint32_t i = threadIdx.x; i < kCurs; i += blockDim.x) cur[i] = 0;
  fw_load_tables(T, a);  // (its barrier also covers cur)
  frames64_tiles<kCurOverflow, true>(
      a.frames, a.len, a.in_dev, a.p0, a.p1, n_all, stage[threadIdx.x >> 6],
      reinterpret_cast<const uint4 *>(a.t.bk),
      [&](uint32_t p, const RFrame &f, uint32_t in, uint32_t len, bool mine) {
        return fw_issue(a, T, p, f, in, len, mine);
      },
      [&](const FwPend &P, const uint4 *row, uint32_t p, RFrame &f, uint32_t in,
          uint32_t len, uint32_t &touch) -> uint32_t {
        // the MACs change (bytes 0-11); the whole slot is stored back, a
        // whole-line write
        return fw_finish(a, T, P, row, p, f, in, len, touch) ? 0xFu : 0u;
      },
      bins, rq, cur);
}

// Packets whose home bucket held three other keys finish here, queued per
// classify block (TileQueue): phase A's register path with the probe walked
// on bucket by bucket (reprobe_wave); their touches join the block's bins.
__global__ __launch_bounds__(256) void fw_reprobe(FwArgs a, const uint32_t *list,
                                                  const uint32_t *cnt, uint32_t n,
                                                  uint32_t range, uint32_t nblk,
                                                  uint64_t seq_base) {
  __shared__ uint32_t T[kFwTabWords];
  __shared__ uint4 stage[4][256];
  fw_load_tables(T, a);
  a.tileq = 1;  // a full bucket answers kReprobe: reprobe_wave walks on
  uint4 *S = stage[threadIdx.x >> 6];
  reprobe_slices(list, cnt, n, range, nblk, a.t.tseq, seq_base, [&](uint32_t p, bool act) {
    return reprobe_wave(
        a.frames, a.slot, a.len, a.in_dev, reinterpret_cast<const uint8_t *>(a.t.bk),
        a.t.bmask, p, act, S,
        [&](uint32_t q, const RFrame &f, uint32_t in, uint32_t len, bool mine) {
          return fw_issue(a, T, q, f, in, len, mine);
        },
        [&](const FwPend &P, const uint4 *row, uint32_t q, RFrame &f, uint32_t in,
            uint32_t len, uint32_t &touch) {
          return fw_finish(a, T, P, row, q, f, in, len, touch);
        });
  });
}

// ------------------------------------------------------------- phase B --

// FlowId keys and hashes of the queued LAN misses.
__global__ void fw_miss_keys(FwArgs a, const uint32_t *list, uint32_t n,
                             uint32_t *mkey, uint32_t *mhash) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    GFrame f{a.frames + (size_t)p * a.slot, a.slot};
    const L34 h = parse_l34(f, a.len[p]);
    const uint32_t proto = f.r8(h.ip + 9);
    const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
    const uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
    uint32_t *k = mkey + 4 * (size_t)j;
    fw_key(false, sp, dp, sip, dip, proto, k);
    mhash[j] = fw_hash(a.crc_tab, sp, dp, sip, dip, proto);
  }
}

// Every LAN miss: forwarded to the WAN device whether or not an index was
// free (fw_flowmanager.c:49-53); the first sighting of a key records its
// input device as the flow's int_devices entry (fw_flowmanager.c:61-64).
__global__ void fw_miss_finish(FwArgs a, const uint32_t *list, uint32_t n,
                               const uint32_t *mkey, const uint32_t *scratch,
                               const uint32_t *rep, const uint32_t *assign) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint32_t j0 = scratch[rep[j]];
    const uint32_t idx = assign[j0];
    a.log[p] = idx;
    if (idx != kNone && j0 == j) {
      const uint32_t e = a.t.slot_of[idx];
      a.t.bk[e >> 2].k[e & 3][3] = mkey[4 * (size_t)j + 3] | ((uint32_t)a.in_dev[p] << 8);
    }
    GFrame f{a.frames + (size_t)p * a.slot, a.slot};
    uint32_t mw[3];
    fw_macs(a, a.wan, mw);
    set_macs(f, mw);
    a.out[p] = a.wan;
  }
}

// ------------------------------------------------------------- phase C --
// WAN packets whose reversed FlowId was not in the table at segment start:
// a hit iff a LAN packet before this one (packet order) allocated it.
__global__ void fw_defer_finish(FwArgs a, const uint32_t *list, uint32_t n) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += gridDim.x * blockDim.x) {
    const uint32_t p = list[j];
    const uint64_t q = a.seq_base + p;
    const uint32_t in = a.in_dev[p];
    GFrame f{a.frames + (size_t)p * a.slot, a.slot};
    const L34 h = parse_l34(f, a.len[p]);
    const uint32_t proto = f.r8(h.ip + 9);
    const uint32_t sp = f.r16(h.l4), dp = f.r16(h.l4 + 2);
    const uint32_t sip = f.r32(h.ip + 12), dip = f.r32(h.ip + 16);
    uint32_t key[4];
    fw_key(true, sp, dp, sip, dip, proto, key);
    uint32_t w3 = 0;
    const uint32_t idx =
        tbl_probe<0xFFu>(a.t, fw_hash(a.crc_tab, dp, sp, dip, sip, proto), key, &w3);
    if (idx == kNone || !tbl_allocated_before(a.t, idx, q)) {
      a.out[p] = (uint16_t)in;  // unknown external flow (fw_main.c:56-59)
      a.log[p] = kNone;
      continue;
    }
    a.log[p] = idx;
    const uint32_t dst = w3 >> 8;
    uint32_t mw[3];
    fw_macs(a, dst, mw);
    set_macs(f, mw);
    a.out[p] = (uint16_t)dst;
  }
}

// =============================================================== host ==

// fw_flowmanager.c:66-73: FlowManager.expiration_time is a vigor_time_t, so
// expiration_time * 1000 is computed in 64 bits (no wrap, unlike vignat).
static inline int64_t fw_cutoff(const vp_ctx *c, int64_t t) {
  return (int64_t)((uint64_t)t - (uint64_t)((int64_t)c->fw.expiration_time * 1000));
}

static int fw_segment(vp_ctx *c, const vp_dev_batch *b, const NowSpec &now,
                      uint32_t p0, uint32_t p1, float *ms, int *launches,
                      uint32_t *allocated) {
  FlowTable &t = c->ft;
  Workspace &w = c->ws;
  FwArgs a{};
  a.frames = b->frames;
  a.len = b->len;
  a.in_dev = b->in_dev;
  a.out = b->out_dev;
  a.log = w.log;
  const uint64_t seq0 = c->seq;
  a.seq_base = seq0;
  a.slot = b->slot;
  a.p0 = p0;
  a.p1 = p1;
  a.t = tbl_dev(t);
  a.crc_tab = c->crc_tab;
  a.macw = c->macw;
  a.miss = w.miss;
  a.defer = w.defer;
  a.reprobe = w.reprobe;
  a.wan = c->fw.wan_device;
  a.n_dev = c->fw.n_devices;

  // 64-byte slots: the classify launch also bins its touches (TouchBins)
  const bool tiles64 = p1 > p0 && b->slot == 64 && c->coalesced_io;
  BinsPlan bp{};
  uint32_t grid64 = 0, range64 = 0;
  TileQueue rq{};
  if (tiles64) {
    VP_TRY(tbl_bins_plan(c, t, (const void *)fw_classify64, p0, p1, &bp));
    const uint32_t tiles = (p1 - (p0 & ~63u) + 63) / 64;
    grid64 = resident_grid((const void *)fw_classify64, (tiles + 3) / 4);
    range64 = (tiles + grid64 - 1) / grid64 * 64;
    rq = TileQueue{w.reprobe, w.reprobe_cnt, &t.ctl->reprobe_count};
    a.tileq = 1;
  }
  // (still zero after a segment that queued nothing: no reset launch)
  if (!t.ctl_clean) VP_HIP(hipMemsetAsync(&t.ctl->miss_count, 0, 16, c->stream));  // .. reprobe
  t.ctl_clean = false;
  VP_HIP(ev_record(c->ktime, c->ev0, c->stream));
  if (p1 > p0) {
    if (tiles64) {
      FwArgs a64 = a;
      if (bp.on) a64.log = nullptr;  // touches go to the bins only
      fw_classify64<<<grid64, 256, 0, c->stream>>>(a64, b->n, bp.bins, rq);
    } else {
      fw_classify<<<grid_for(p1 - p0), 256, 0, c->stream>>>(a);
    }
    VP_HIP(hipGetLastError());
  }
  VP_HIP(ev_record(c->ktime, c->ev1, c->stream));
  // phase A's counts, and the fold of its touches behind them; queued
  // packets follow as late touches
  VP_TRY(tbl_fold_read_ctl(c, t, bp, w.log, p0, p1, now, seq0));
  // reprobes come only from the 64-byte tiles (fw_generic_a walks in place)
  const uint32_t nre = t.h_ctl.reprobe_count;
  if (nre) {  // probes past a full home bucket: finish them, patch the fold
    fw_reprobe<<<std::min<uint32_t>(grid64, 2048), 256, 0, c->stream>>>(
        a, w.reprobe, w.reprobe_cnt, nre, range64, grid64, seq0);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_reprobe_stamp(c, t, w.reprobe, w.reprobe_cnt, nre, range64, grid64,
                             w.log, now, seq0));
    VP_TRY(read_ctl(c, t));  // the walk may have found new flows
  }
  const bool ovf = bp.on && t.h_ctl.touch_ovf != 0;
  if (ovf)  // touches that found their bin slice full, logged alone
    VP_TRY(tbl_late_touches(c, t, bp.bins.oent, bp.bins.ocnt, 0, range64, grid64,
                            w.log, now, seq0));
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
    fw_miss_keys<<<grid_for(nmiss), 256, 0, c->stream>>>(a, w.miss_sorted, nmiss,
                                                         w.mkey, w.mhash);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_new_keys(c, t, NewKeys{nmiss, w.miss_sorted}, c->seq, nullptr));
    a.t = tbl_dev(t);  // a rebuild may have moved the buckets
    fw_miss_finish<<<grid_for(nmiss), 256, 0, c->stream>>>(
        a, w.miss_sorted, nmiss, w.mkey, w.scratch, w.rep, w.assign);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_late_touches(c, t, w.miss_sorted, nullptr, nmiss, 256,
                            (nmiss + 255) / 256, w.log, now, seq0));
    *allocated |= 1u;
  }
  if (ndefer) {
    a.t = tbl_dev(t);  // a rebuild during phase B may have changed the layout
    fw_defer_finish<<<grid_for(ndefer), 256, 0, c->stream>>>(a, w.defer, ndefer);
    VP_HIP(hipGetLastError());
    VP_TRY(tbl_late_touches(c, t, w.defer, nullptr, ndefer, 256, (ndefer + 255) / 256,
                            w.log, now, seq0));
  }
  if (nmiss || ndefer) VP_TRY(read_ctl(c, t));
  // steady state: frames and ports complete, only the stamp fold may run
  // (not when it reads the caller's time array)
  c->fold_pending = !b->now && !nre && !nmiss && !ndefer && !ovf;
  t.ctl_clean = !nre && !nmiss && !ndefer && !ovf;
  return 0;
}

int fw_process_device(vp_ctx *c, const vp_dev_batch *b) {
  ExpiringTable tabs[1] = {{&c->ft, fw_cutoff}};
  return run_batch(c, b, tabs, 1, fw_segment);
}

// State by flow index: alloc, ts, FlowId bytes (vigfw/flow.h layout, padding
// zero) and int_devices.
int fw_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys,
            uint32_t *int_dev) {
  const uint32_t cap = c->ft.cap;
  std::vector<uint32_t> k(4ull * cap);
  VP_TRY(tbl_dump(c, c->ft, alloc, ts, k.data()));
  for (uint32_t i = 0; i < cap; i++) {
    const uint32_t *e = &k[4ull * i];
    uint8_t *o = keys + 16ull * i;
    memcpy(o, e, 12);
    o[12] = (uint8_t)e[3];
    o[13] = o[14] = o[15] = 0;
    int_dev[i] = alloc[i] ? e[3] >> 8 : 0;
  }
  return 0;
}

void build_fw_tables(std::vector<uint32_t> &tab) {
  tab.assign(kFwTabs * 256, 0);
  for (uint32_t j = 0; j < kFwTabs; j++)
    build_position_table(&tab[j * 256], kFwPos[j], kFwMsg);
}

}  // namespace vp
