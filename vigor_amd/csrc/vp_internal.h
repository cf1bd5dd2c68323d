// Host-side context shared by the runtime translation units.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>
#include <tuple>
#include <vector>

#include "../../include/vigpath.h"
#include "vp_device.h"

#define VP_HIP(call)                                                      \
  do {                                                                    \
    hipError_t e_ = (call);                                               \
    if (e_ != hipSuccess) return vp::hip_fail(e_, #call, __FILE__, __LINE__); \
  } while (0)

#define VP_TRY(call)          \
  do {                        \
    int rc_ = (call);         \
    if (rc_) return rc_;      \
  } while (0)

namespace vp {

int hip_fail(hipError_t e, const char *what, const char *file, int line);
// Record a VP_ESTATE failure (vp_last_error) and return VP_ESTATE.
int state_fail(const char *fmt, ...);

// Wait for `s` to drain by polling (a packet-processing host thread polls,
// as DPDK's lcores do): a blocking wait adds tens of microseconds of wake-up
// latency to every batch's control-block read-back.
hipError_t stream_wait(hipStream_t s);
hipError_t event_ms(hipEvent_t a, hipEvent_t b, float *ms);
// Per-launch kernel timing (vp_kernel_timing): the classify launch between
// two events, summed into vp_last_kernel_ms. Off by default: the events cost
// a step about 6 us of kernel-boundary time.
inline hipError_t ev_record(bool on, hipEvent_t e, hipStream_t s) {
  return on ? hipEventRecord(e, s) : hipSuccess;
}
inline hipError_t ev_ms(bool on, hipEvent_t a, hipEvent_t b, float *ms) {
  *ms = 0.f;
  return on ? event_ms(a, b, ms) : hipSuccess;
}
// Host-side stage clock (VIGPATH_HOSTPROF=1, diagnostics): hostprof(k)
// stamps stage k of the current call; the call's stamps go to stderr.
void hostprof(int k);
// Launch k with its dispatch's own start and end timestamps in e0 / e1
// (hipExtLaunchKernel: the kernel's AQL packet is timed, as rocprofv3's
// kernel trace times it, not the marker packets around it). e1 completes
// with the kernel.
template <class... P, class... A>
hipError_t launch_timed(void (*k)(P...), dim3 grid, dim3 block, hipStream_t s,
                        hipEvent_t e0, hipEvent_t e1, A... args) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  std::tuple<P...> t{args...};
  void *ptrs[sizeof...(P)];
  std::apply([&](auto &...x) {
    size_t i = 0;
    ((ptrs[i++] = (void *)&x), ...);
  }, t);
  return hipExtLaunchKernel((const void *)k, grid, block, ptrs, 0, s, e0, e1, 0);
}

// 1024-thread vignat tiles (nat_tiles) and their memory-shape probe
// (vp_probe_slots_w): each block's range in VIGPATH_SPLIT (1, 2 or 4)
// contiguous sub-ranges, 16 / split waves interleaved over each.
inline uint32_t tile_split() {
  static const uint32_t s = [] {
    const char *e = getenv("VIGPATH_SPLIT");
    const int v = e ? atoi(e) : 1;
    return v == 2 || v == 4 ? (uint32_t)v : 1u;
  }();
  return s;
}

// One empty kernel per translation unit: launching it makes HIP load the
// unit's device code, which it otherwise does at the unit's first kernel
// launch (5-30 ms for vp_nat.hip's variants): ctx_common pays it once per
// GPU, at context creation (nf_init), not the first batch.
#define VP_PRELOAD_UNIT(name)                                     \
  __global__ void preload_k_##name() {}                           \
  hipError_t preload_##name(hipStream_t s) {                      \
    preload_k_##name<<<1, 64, 0, s>>>();                          \
    return hipGetLastError();                                     \
  }
hipError_t preload_runtime(hipStream_t s);
hipError_t preload_table(hipStream_t s);
hipError_t preload_nat(hipStream_t s);
hipError_t preload_bridge(hipStream_t s);
hipError_t preload_lb(hipStream_t s);
hipError_t preload_fw(hipStream_t s);
hipError_t preload_pol(hipStream_t s);
hipError_t preload_comm(hipStream_t s);
hipError_t preload_mbuf(hipStream_t s);

// Owner-mode phase A stages (vp_last_stage_ms).
constexpr int kStages = 8;
inline constexpr const char *kStageNames[kStages] = {
    "pass1", "offsets", "a2a_keys", "probe", "a2a_answers", "pass2", "fold", "pipeline"};
constexpr int kStageFold = 6, kStagePipeline = 7;

struct Comm;  // vp_comm.hip: collectives between the ranks of one NF
constexpr int kMaxRanks = 64;

enum Kind { KIND_NAT = 1, KIND_BRIDGE = 2, KIND_LB = 3, KIND_FW = 4, KIND_POL = 5 };

// Device control block of one table (dchain + map bookkeeping).
struct Ctl {
  uint32_t stack_top;   // freed indices on the LIFO stack
  uint32_t fresh_next;  // first never-allocated index
  uint32_t n_live;
  uint32_t n_tomb;
  uint32_t miss_count;     // } reset together at the start of a segment
  uint32_t defer_count;    // }
  uint32_t touch_ovf;      // } a touch-bin slice overflowed (TouchBins)
  uint32_t reprobe_count;  // } home bucket full of other keys (vp_nat.hip)
  uint32_t route_ovf;   // } owner mode: some rank's keys for an owner exceeded the
                        //   padded exchange's capacity (the unchunked pipeline:
                        //   all ranks agree, allreduced; the chunked one: this
                        //   rank's own slices, gathered before the fold)
  uint32_t exp_count;
  uint32_t tomb_reused;
  uint64_t min_ts;
  uint32_t new_count;
  uint32_t aux_count;
  uint32_t max_disp;    // longest insert probe (buckets) since last check
  uint32_t disp_count;  // inserts that passed their home bucket (since rebuild)
  uint32_t sh_live;     // entries in this rank's buckets (= n_live unless owner mode)
  uint32_t own_new;     // owner mode: union keys this rank will insert (upper bound)
  uint32_t run_tiles;   // vignat's 64-byte tiles whose 64 touches were one run
                        // (cumulative, never reset: the host takes differences)
  uint32_t last_first;  // unsorted new keys: 1 + the last first sighting's
                        // position in the segment (nku_firsts)
  uint32_t arrive;      // classify blocks finished (tile_publish; 0 between launches)
};

// The control block as a fold kernel (or, one GPU, the classify's last
// block: tile_publish) publishes it into page-locked host memory
// (tbl_fold_read_ctl, vp_table.hip); the host polls `epoch`.
// Multi-GPU: the fold also publishes every rank's segment counters
// (miss, defer, touch_ovf, reprobe: gathered on the device before the fold)
// and, owner mode, this rank's key count per owner.
constexpr int kPubGath = 5;  // words per rank (miss_count .. route_ovf)
struct CtlPub {
  Ctl ctl;
  uint32_t xtra[(kPubGath + 1) * 64];
  uint32_t epoch;
};

// One device table (see vp_table.h).
struct FlowTable {
  Bucket *bk = nullptr;
  uint32_t bmask = 0;  // buckets - 1
  uint32_t cap = 0;
  uint32_t mix = 0;    // home-bucket mode (vp_table.h home_bucket)
  uint64_t ins_since = 0;  // inserts since the last rebuild (mode check)
  uint32_t layout_tries = 0;  // tbl_choose_layout calls so far
  uint64_t rebuilds = 0;      // tbl_rebuild calls so far (vp_table_stats_get)
  // allocation-order layout (mix == kMixLin, vp_table.hip tbl_try_linear):
  // the linear map's four byte tables on the device; lin_ok: the NF's
  // classify kernels stage them (vignat); lin_tried: fitted once already
  // (lin_ok 2: two consecutive indices per bucket, half the buckets)
  uint32_t *lin = nullptr;
  uint32_t lin_ok = 0;
  bool lin_tried = false;
  uint64_t nb_nominal = 0;  // buckets of the CRC-bit layouts
  uint64_t nb_base = 0;     // the power of two >= cap (one bucket per index)
  uint32_t *slot_of = nullptr;
  uint32_t *hash_of = nullptr;
  uint64_t *ts = nullptr;
  uint64_t *tseq = nullptr;
  uint64_t *birth = nullptr;
  uint32_t *stack = nullptr;
  uint32_t *lastg = nullptr;  // touch-reduce partial maxima (small tables)
  Ctl *ctl = nullptr;
  Ctl h_ctl{};                     // last copy read back
  Ctl *h_pin = nullptr;            // page-locked landing buffer for h_ctl
  CtlPub *h_pub = nullptr;         // host-coherent page, written by the fold
  CtlPub *d_pub = nullptr;         // (its device address)
  uint32_t pub_epoch = 0;          // last epoch asked of the fold
  uint32_t *ttotal = nullptr;  // touch-reduce entry count (device)
  uint64_t ts_floor = UINT64_MAX;  // lower bound of min ts over live indices
  // first-sighting cut (vignat, one GPU; run_batch): the packets at the start
  // of a batch that held the last batch's first sightings of new flows when
  // most of its misses were repeats of them; 0: no cut
  uint32_t fs_hint = 0;
  // vignat: the last segment's tiles were mostly runs (Ctl::run_tiles), so
  // the next one takes the 1024-thread tile without staged bin lines
  bool runs_seen = true;
  uint32_t last_run_tiles = 0;
  // the segment counters (miss_count .. reprobe_count) are known to be zero on
  // the device: the next segment needs no reset (vignat steady state)
  bool ctl_clean = false;
  // expiry workspace (sized cap)
  uint64_t *ekey = nullptr, *ekey2 = nullptr;
  uint32_t *eidx = nullptr, *eidx2 = nullptr;
  // owner-sharded mode (vp_shard_mode): this rank's buckets
  // hold only the keys it owns; key by index is replicated in kv
  uint4 *kv = nullptr;
  uint32_t own_n = 0, own_r = 0;  // ranks, this rank (own_n == 0: off)
};

struct Workspace {
  uint32_t cap_n = 0;  // batch capacity these buffers hold
  uint32_t *miss = nullptr;
  uint32_t *miss_sorted = nullptr;
  uint32_t *defer = nullptr;
  uint32_t *reprobe = nullptr;  // packets whose probe continues past the home bucket
  uint32_t *reprobe_cnt = nullptr;  // per classify block (TileQueue)
  uint32_t *missq = nullptr;  // phase-A misses per classify block (the reprobe slices' layout)
  uint32_t *mkey = nullptr;  // 4 words per miss
  uint32_t *pairs = nullptr;  // tbl_touch_reduce's scattered (position, index) words
  uint16_t *in_fill = nullptr;  // a batch's one port as an array (vp_dev_batch.in_port)
  size_t in_fill_n = 0;
  // tbl_new_keys_unsorted: the tagged key set (3 x u64 per slot, never
  // reset: a slot of an older tag is empty), its tag, first-sighting bits
  // per position and their scan, the first sightings' miss ordinals and
  // their count; phase A's per-block key slices (beside missq)
  unsigned long long *nkset = nullptr;
  size_t nkset_n = 0;
  uint32_t nk_tag = 0;
  uint32_t *nkbits = nullptr, *nkpre = nullptr, *nkfirst = nullptr, *nkcnt = nullptr;
  size_t nkbits_n = 0, nkfirst_n = 0;
  uint4 *mkq = nullptr;
  uint32_t *mhq = nullptr;
  uint32_t *mhash = nullptr;
  uint32_t *first = nullptr;
  uint32_t *rank = nullptr;
  uint32_t *rep = nullptr;
  uint32_t *assign = nullptr;
  uint32_t *scratch = nullptr;
  uint32_t *log = nullptr;   // touch log, one entry per packet
  uint32_t *log2 = nullptr;  // second table's touch log (viglb backends)
  uint32_t *defer_sorted = nullptr;
  uint32_t *aux = nullptr, *aux_sorted = nullptr;  // third queue (viglb)
  uint32_t *rlist = nullptr;  // re-classification input (viglb rounds)
  uint32_t *hbl = nullptr;    // viglb: heartbeat positions of a segment
  // multi-GPU: new-flow records exchanged between ranks, union positions/times
  void *sbuf = nullptr, *rbuf = nullptr;
  size_t sbuf_bytes = 0, rbuf_bytes = 0;
  int64_t *unow = nullptr;
  uint32_t *iota = nullptr;  // 0..cap_n-1
  uint32_t *skey = nullptr, *sval = nullptr;
  uint32_t *hist = nullptr, *hoff = nullptr;  // touch-reduce (chunk x span)
  uint64_t hist_cap = 0;
  uint32_t *bins_ent = nullptr, *bins_cnt = nullptr;  // touch bins (TouchBins)
  uint32_t *bins_rtab = nullptr;  // their run words ([block][bin][2])
  size_t bins_rtab_n = 0;
  uint32_t *ovf_q = nullptr, *ovf_cnt = nullptr;  // overflowed touches per block
  // owner mode: per-block slices of descriptors by owner rank, their counts
  // and send offsets, per-packet routes, the exchanged keys and replies
  uint4 *desc = nullptr;
  size_t desc_n = 0;
  uint32_t *dcnt = nullptr, *dbase = nullptr, *dtot = nullptr;
  size_t dcnt_n = 0, dbase_n = 0, dtot_n = 0;
  uint32_t *route = nullptr;
  size_t route_n = 0;
  uint4 *sendk = nullptr, *recvk = nullptr;
  size_t sendk_n = 0, recvk_n = 0;
  uint32_t *reply = nullptr, *rreply = nullptr;
  size_t reply_n = 0, rreply_n = 0;
  uint32_t *h_tot = nullptr;  // pinned landing buffer for dtot
  // padded exchange (owner mode): per-block slice counts by owner (cnt_t)
  // and as received by peer (rcnt_t), each owner's needed chunk size (dneed,
  // published for the next batch's capacity), the global slice-overflow
  // flag; the exact exchange's tight send buffer (xsend)
  uint32_t *cnt_t = nullptr, *rcnt_t = nullptr, *dneed = nullptr;
  size_t cnt_t_n = 0, rcnt_t_n = 0, dneed_n = 0;
  uint4 *xsend = nullptr;
  size_t xsend_n = 0;
  uint64_t *ovf64 = nullptr;
  bool ovf64_clean = false;  // ovf64 is zero (the last exchange did not overflow)
  // the chunked owner pipeline (vp_nat.hip nat_phase_a_owner_chunked): the
  // exchange stream, and per chunk parity the events "pass 1 done" and
  // "answers back"; a second set of the padded exchange's buffers
  hipStream_t xstream = nullptr;
  hipEvent_t ev_p1[2] = {}, ev_ans[2] = {};
  uint4 *sendk2 = nullptr, *recvk2 = nullptr;
  uint32_t *reply2 = nullptr, *rreply2 = nullptr;
  size_t sendk2_n = 0, recvk2_n = 0, reply2_n = 0, rreply2_n = 0;
  uint32_t *lcnt = nullptr;  // leftover exchange: keys past each slice
  size_t lcnt_n = 0;
  // multi-GPU: the ranks' segment counters gathered on the device before a
  // fold (kPubGath words each) and their host copy (gath_ok: this segment's)
  uint32_t *gath = nullptr;
  std::vector<uint32_t> h_gath;
  bool gath_ok = false;
  size_t bins_ent_n = 0, bins_cnt_n = 0;
  void *cub_tmp = nullptr;
  size_t cub_bytes = 0;
  // host staging for the host-batch entry points
  uint8_t *h_frames = nullptr;
  size_t h_frames_bytes = 0;
  uint8_t *d_frames = nullptr;
  size_t d_frames_bytes = 0;
  uint16_t *d_len = nullptr, *d_in = nullptr, *d_out = nullptr;
  int64_t *d_now = nullptr;
  uint32_t d_meta_n = 0;
  // pipelined host batches (vp_process_host): copy stream, per-buffer
  // events, pinned staging of the small per-packet arrays
  hipStream_t cstream = nullptr;  // host -> device copies
  hipStream_t dstream = nullptr;  // device -> host copies (PCIe is full duplex)
  hipEvent_t ev_in[3] = {}, ev_done[3] = {}, ev_out[3] = {};  // per buffer set
  uint8_t *h_meta = nullptr;
  size_t h_meta_bytes = 0;
  // host frames (vp_process_mbufs, vp_mbuf.hip): kMbufSets buffer sets of
  // mb_cap packets each -- mbuf data pointers, 64-byte header slots, tail
  // sums, per-set flags (device; their host copy in h_mbflags) -- and the
  // whole-frame slots of a chunk that needs them (mb_full)
  static constexpr int kMbufSets = 4;
  uint64_t *mb_ptr = nullptr;
  uint8_t *mb_slots = nullptr;
  uint32_t *mb_tail = nullptr, *mb_flags = nullptr, *h_mbflags = nullptr;
  size_t mb_cap = 0;
  uint16_t *mb_len = nullptr, *mb_in = nullptr, *mb_out = nullptr;
  int64_t *mb_now = nullptr;
  uint8_t *mb_full = nullptr;
  size_t mb_full_bytes = 0;
  uint8_t *st_meta = nullptr;  // staged_range's device len / in / out / now
  size_t st_meta_n = 0;
  uint8_t *h_mbmeta = nullptr;  // pinned staging of pageable per-packet arrays
  size_t h_mbmeta_bytes = 0;
  // host-gather mode: pinned header slots and tail sums the host threads
  // fill (kMbufSets sets of mb_hcap packets)
  uint8_t *h_mbslots = nullptr;
  uint32_t *h_mbtail = nullptr;
  size_t mb_hcap = 0;
  hipEvent_t mb_ev_in[kMbufSets] = {}, mb_ev_done[kMbufSets] = {},
             mb_ev_out[kMbufSets] = {};
};

// Host memory registered for direct access by the context's GPU
// (vp_register_host): frames in [hbase, hend) are read and written at
// address + delta by the mbuf kernels (vp_mbuf.hip).
struct HostMap {
  uint64_t hbase, hend;
  int64_t delta;
  bool ours;  // hipHostRegister'ed by the library (unregistered on release)
};
constexpr int kMaxHostMaps = 16;

// vp_process_one's mailbox (vp_nat.hip nat_serve): page-locked, host-coherent
// memory the host and a persistent one-wave kernel poll. The host writes the
// request (below); the kernel writes the rewritten frame to `frame`, then
// sets the answer word.
constexpr uint32_t kServeFrame = 2048;  // longest frame served (others: the batch path)
constexpr uint32_t kServeLeave = 0xFFFFFFFFu;  // message word 0: leave
// The request travels in kServeChunks tagged 16-byte chunks that every poll
// of the server reads whole (one PCIe read per poll, no second round trip for
// the frame): chunk k holds bytes 12k .. 12k + 11 of the message (len |
// in_dev << 16 as 4 bytes -- kServeLeave: leave --, the time as 8, then the
// frame's first kServeInline bytes) and, as its last word, the request
// number. The host writes a chunk's payload before its tag, and a chunk lies
// within one cache line, which a device read sees whole: a chunk whose tag is
// the request's carries the request's bytes. Frames past kServeInline bytes
// also go whole through `frame`, read after the chunks.
constexpr uint32_t kServeChunks = 8;
constexpr uint32_t kServeInline = 12 * kServeChunks - 12;  // 84 frame bytes
struct ServeBox {
  alignas(128) uint32_t msg[kServeChunks][4];  // host: the tagged request chunks
  // device: the answer the same way -- chunk k = bytes 12k .. 12k + 11 of
  // (out | fresh << 16, 8 unused bytes, the rewritten frame's first
  // kServeInline bytes) and the request number; one store instruction, no
  // wait between the frame and the answer word (a longer frame goes through
  // `frame` first, then chunk 0 alone)
  alignas(128) uint32_t amsg[kServeChunks][4];
  uint64_t ans;      // device: request number | (out | fresh << 16) << 32 (relaunch state)
  uint64_t prof[10];  // device: wall-clock stamps of the last request (VIGPATH_SERVE_PROF)
  alignas(16) uint8_t frame[kServeFrame];  // longer frames in; every result out
};
// One packet through the persistent kernel (vignat, one GPU, no expiry due):
// 0 done; 1 not eligible (the caller takes the batch path, the server is
// stopped); < 0 an error.
int nat_process_one(vp_ctx *c, uint16_t in_dev, uint8_t *frame, uint16_t len, int64_t now,
                    uint16_t *out);
// Stop the context's persistent kernel, if it runs (every other entry point
// calls this first: the kernel owns the table while it runs).
int serve_stop(vp_ctx *c);
void serve_free(vp_ctx *c);

}  // namespace vp

struct vp_ctx {
  int kind = 0;
  int gpu = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t evc = nullptr;  // control-block copy (read_ctl_post / _wait)
  // host copy of the current device batch's time array (host_pipeline sets it
  // for the chunk it hands to vp_process_device): the batch driver reads its
  // expiry cuts from it instead of copying the array back
  const int64_t *host_now = nullptr;
  hipEvent_t ev2 = nullptr, ev3 = nullptr;  // owner mode: pass 2 timing
  // The last segment left only its timestamp fold running on `stream`
  // (results complete): run_batch returns without waiting for it.
  bool fold_pending = false;
  bool seg_fs = false;  // the segment run_batch is running is a first-sighting cut
  float last_ms = 0.f;
  // the classification kernel the last vp_process_device call launched last
  // (vp_last_kernel; "" before any)
  const char *last_kernel = "";
  bool ktime = false;  // vp_kernel_timing: events around the classify launch
  // owner mode with ktime: the last call's phase-A stage times (ms, summed
  // over its segments; vp_last_stage_ms)
  float stage_ms[vp::kStages] = {};
  int stage_n = 0;
  int last_launches = 0;
  uint64_t seq = 0;       // packets processed so far (global packet order)
  int64_t last_now = -1;  // time of the last packet processed
  vp_nat_config nat{};
  vp_bridge_config brg{};  // static_rules not kept (built into st_*)
  vp::FlowTable ft;       // vignat/vigfw flows / vigbridge dyn MACs / viglb flows
  vp::FlowTable ft2;      // viglb backends (ip_to_backend_id + dchain)
  vp_lb_config lb{};
  vp_fw_config fw{};
  vp_pol_config pol{};
  uint64_t *pol_size = nullptr;  // vigpol dyn_vals: bucket_size by index
  int64_t *pol_time = nullptr;   //                  bucket_time by index
  uint32_t *pol_cnt = nullptr;   // hits per index in a segment (grouping)
  bool pol_cnt_clean = false;     // pol_cnt is all zero (the replay cleared it)
  uint32_t *pol_off = nullptr;   // exclusive scan of pol_cnt
  uint32_t *pol_runs = nullptr;  // [kRunMax][index] hit positions (grouping;
                                 // allocated by the first grouping segment,
                                 // tables up to 4M indices, else pol_off)
  bool pol_runs_tried = false;   // that allocation was attempted
  uint4 *be_rec = nullptr;  // viglb backends[]: {ip, mac0-3, mac4-5|nic<<16, 0}
  uint32_t *cht = nullptr;  // viglb CHT, cht[bucket * backend_capacity + prio]
  uint32_t *dmacw = nullptr;  // per device: {s_addr[0..1] << 16, s_addr[2..5]}
  vp::Bucket *st_bk = nullptr;  // vigbridge static table (rule number = idx)
  uint32_t st_bmask = 0;
  int32_t *st_val = nullptr;    // rule -> device_to
  uint32_t n_static = 0;
  uint32_t *crc_tab = nullptr;  // CRC position tables (LDS-staged)
  uint32_t *macw = nullptr;     // per device: d_addr|s_addr header words
  uint32_t wan_macw[3] = {0, 0, 0};
  bool coalesced_io = true;  // LDS-staged 64 B frame I/O (VIGPATH_COALESCED=0 off)
  vp::Workspace ws;
  // multi-GPU (vp_attach_*): this rank's collectives, and during a batch the
  // global position of local packet 0 and the per-rank slice sizes
  vp::Comm *comm = nullptr;
  int shard_mode = 0;  // VP_SHARD_REPLICATED / VP_SHARD_OWNER
  uint32_t off = 0;
  // the current segment's global packet range (run_batch_sharded): every rank
  // derives every rank's part of it from rank_n (the chunked owner pipeline's
  // chunk count is the same everywhere)
  uint64_t seg_g0 = 0, seg_g1 = 0;
  // owner mode: keys per peer the padded exchange carries in this batch (0:
  // exact exchange), and this rank's largest per-owner key count last seen
  uint32_t own_cap = 0;
  uint32_t own_maxsend = 0;
  std::vector<uint32_t> rank_n;    // slice sizes of the current batch
  std::vector<uint32_t> rank_cnt;  // new keys per rank of the current segment
  // multi-GPU: this rank broke an invariant (union_sizes); every rank returns
  // VP_ESTATE from the next batch on, decided from the RankInfo gather
  bool estate_pending = false;
  // host memory the GPU reads frames from in place (vp_register_host)
  std::vector<vp::HostMap> hmaps;
  // during vp_process_mbufs: tail sums of the 64-byte header slots the
  // current device batch holds (vp_nat.hip NatArgs::tail), else null
  const uint32_t *hdr_tail = nullptr;
  // vp_process_one (vp_nat.hip): the mailbox, whether nat_serve runs on
  // `stream`, the last request number, and its idle exit (wall-clock ticks)
  vp::ServeBox *sbox = nullptr;
  bool srv_on = false;
  uint32_t srv_req = 0;
  uint64_t srv_idle = 0, srv_idle_ms = 1;
  // held by the thread serving (nat_process_one, serve_stop); another
  // context's server launch on the same GPU stops this one only if it can
  // take it (serve_launch: resident kernels share the hardware queues)
  std::recursive_mutex srv_mu;
  double srv_prof[11] = {};  // VIGPATH_SERVE_PROF: summed stage times (us), counts
};
