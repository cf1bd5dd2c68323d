// C-ABI entry points of libvigpath.so (include/vigpath.h): context
// lifetime, workspace, host<->device batch staging and dispatch per NF.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <mutex>
#include <cstdarg>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "vp_comm.h"
#include "vp_table.h"

namespace vp {

VP_PRELOAD_UNIT(runtime)


// vp_last_error(): the calling thread's last failure
static thread_local char g_last_error[256];

int hip_fail(hipError_t e, const char *what, const char *file, int line) {
  const char *base = strrchr(file, '/');
  snprintf(g_last_error, sizeof g_last_error, "HIP %s (%s) in %s at %s:%d",
           hipGetErrorName(e), hipGetErrorString(e), what, base ? base + 1 : file, line);
  if (getenv("VIGPATH_DEBUG")) fprintf(stderr, "vigpath: %s\n", g_last_error);
  return e == hipErrorOutOfMemory ? VP_ENOMEM : VP_EIO;
}

int state_fail(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof g_last_error, fmt, ap);
  va_end(ap);
  if (getenv("VIGPATH_DEBUG")) fprintf(stderr, "vigpath: %s\n", g_last_error);
  return VP_ESTATE;
}

int nat_process_device(vp_ctx *c, const vp_dev_batch *b);
int nat_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys);
void build_flowid_tables(std::vector<uint32_t> &tab);
int bridge_process_device(vp_ctx *c, const vp_dev_batch *b);
void build_bridge_tables(std::vector<uint32_t> &tab);
int bridge_static_build(const vp_bridge_config *cfg, std::vector<Bucket> &bk,
                        uint32_t *bmask);
int lb_process_device(vp_ctx *c, const vp_dev_batch *b);
void build_lb_tables(std::vector<uint32_t> &tab);
void lb_fill_cht(uint32_t height, uint32_t bcap, std::vector<uint32_t> &cht);
int fw_process_device(vp_ctx *c, const vp_dev_batch *b);
void build_fw_tables(std::vector<uint32_t> &tab);
int fw_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys, uint32_t *int_dev);
int pol_process_device(vp_ctx *c, const vp_dev_batch *b);
void build_pol_tables(std::vector<uint32_t> &tab);
int pol_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint32_t *keys,
             uint64_t *bucket_size, int64_t *bucket_time);
int lb_dump(vp_ctx *c, uint8_t *f_alloc, int64_t *f_ts, uint8_t *f_keys,
            uint32_t *f_backend, uint8_t *b_alloc, int64_t *b_ts, uint32_t *b_ip,
            uint8_t *b_mac, uint16_t *b_nic);

hipError_t stream_wait(hipStream_t s) {
  hipError_t e;
  while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
  }
  return e;
}

// Kernel time between two events of the context's stream. The host may learn
// that the work behind `b` ran (a published control block) before the
// runtime has marked `b` complete, so wait for `b` first.
hipError_t event_ms(hipEvent_t a, hipEvent_t b, float *ms) {
  const hipError_t e = hipEventSynchronize(b);
  return e != hipSuccess ? e : hipEventElapsedTime(ms, a, b);
}

static bool is_pow2(uint32_t v) { return v && !(v & (v - 1)); }

template <class T>
static int dalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void **)p, sizeof(T) * count);
  return e == hipSuccess ? 0 : hip_fail(e, "hipMalloc", __FILE__, __LINE__);
}

__global__ void iota_k(uint32_t *v, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x)
    v[i] = i;
}

static void ws_release(Workspace &w) {
  void *ptrs[] = {w.miss,  w.miss_sorted, w.defer, w.mkey, w.mhash,
                  w.first, w.rank,        w.rep,   w.assign, w.scratch,
                  w.log,   w.iota,        w.skey,  w.sval,
                  w.log2,  w.defer_sorted, w.aux,  w.aux_sorted, w.rlist, w.hbl,
                  w.unow,  w.reprobe,     w.reprobe_cnt, w.ovf_q, w.ovf_cnt, w.missq,
                  w.mkq,   w.mhq,    w.pairs};
  for (void *p : ptrs) hipFree(p);
  w.miss = w.miss_sorted = w.defer = w.mkey = w.mhash = w.first = w.rank =
      w.rep = w.assign = w.scratch = w.log = w.iota = w.skey = w.sval = nullptr;
  w.log2 = w.defer_sorted = w.aux = w.aux_sorted = w.rlist = w.hbl = nullptr;
  w.unow = nullptr;
  w.reprobe = w.reprobe_cnt = nullptr;
  w.ovf_q = w.ovf_cnt = nullptr;
  w.missq = nullptr;
  w.mkq = nullptr;
  w.mhq = nullptr;
  w.pairs = nullptr;
  w.cap_n = 0;
}

// Per-batch scratch sized for the largest batch seen so far.
int ws_reserve(vp_ctx *c, uint32_t n) {
  Workspace &w = c->ws;
  if (n <= w.cap_n) return 0;
  VP_HIP(hipStreamSynchronize(c->stream));
  ws_release(w);
  const uint32_t cap = std::max<uint32_t>(n, 1024);
  const uint64_t ss = next_pow2(2ull * cap);
  VP_TRY(dalloc(&w.miss, cap));
  VP_TRY(dalloc(&w.miss_sorted, cap));
  VP_TRY(dalloc(&w.defer, cap));
  VP_TRY(dalloc(&w.reprobe, cap + 128));  // per-block slices end on tile bounds
  // per classify block: >= any resident grid, and the chunked owner
  // pipeline's virtual blocks (at least one tile each)
  const size_t nblk = std::max<size_t>(4096, cap / 64 + 64);
  VP_TRY(dalloc(&w.reprobe_cnt, nblk));
  VP_TRY(dalloc(&w.ovf_q, cap + 128));     // (the same slices as reprobe)
  VP_TRY(dalloc(&w.missq, cap + 128));
  VP_TRY(dalloc(&w.mkq, cap + 128));  // (phase A's miss keys beside missq)
  VP_TRY(dalloc(&w.mhq, cap + 128));
  VP_TRY(dalloc(&w.pairs, cap));
  VP_TRY(dalloc(&w.ovf_cnt, nblk));
  VP_TRY(dalloc(&w.mkey, 4ull * cap));
  VP_TRY(dalloc(&w.mhash, cap));
  VP_TRY(dalloc(&w.first, cap));
  VP_TRY(dalloc(&w.rank, cap));
  VP_TRY(dalloc(&w.rep, cap));
  VP_TRY(dalloc(&w.assign, cap));
  VP_TRY(dalloc(&w.scratch, ss));
  VP_TRY(dalloc(&w.log, cap));
  if (c->comm) VP_TRY(dalloc(&w.unow, cap));  // multi-GPU union times
  if (c->kind == KIND_LB) {  // second table + round queues
    VP_TRY(dalloc(&w.log2, cap));
    VP_TRY(dalloc(&w.defer_sorted, cap));
    VP_TRY(dalloc(&w.aux, cap));
    VP_TRY(dalloc(&w.aux_sorted, cap));
    VP_TRY(dalloc(&w.rlist, cap));
    VP_TRY(dalloc(&w.hbl, cap));
  }
  if (c->kind == KIND_POL) VP_TRY(dalloc(&w.aux, cap));  // hit ranks (vp_pol.hip)
  VP_TRY(dalloc(&w.iota, cap));
  VP_TRY(dalloc(&w.skey, cap));
  VP_TRY(dalloc(&w.sval, cap));
  iota_k<<<grid_for(cap), 256, 0, c->stream>>>(w.iota, cap);
  VP_HIP(hipGetLastError());
  w.cap_n = cap;
  return 0;
}

static void mac_words(const uint8_t d[6], const uint8_t s[6], uint32_t w[3]) {
  uint8_t b[12];
  memcpy(b, d, 6);
  memcpy(b + 6, s, 6);
  for (int k = 0; k < 3; k++)
    w[k] = b[4 * k] | (b[4 * k + 1] << 8) | (b[4 * k + 2] << 16) |
           ((uint32_t)b[4 * k + 3] << 24);
}

// Every unit's device code loaded on `gpu` (VP_PRELOAD_UNIT), once per
// process and GPU.
static int preload_units(int gpu, hipStream_t s) {
  static std::mutex mu;
  static std::vector<int> done;
  std::lock_guard<std::mutex> g(mu);
  if (std::find(done.begin(), done.end(), gpu) != done.end()) return 0;
  for (auto f : {preload_runtime, preload_table, preload_nat, preload_bridge, preload_lb,
                 preload_fw, preload_pol, preload_comm, preload_mbuf})
    VP_HIP(f(s));
  VP_HIP(hipStreamSynchronize(s));
  done.push_back(gpu);
  return 0;
}

static int ctx_common(vp_ctx *c, int gpu) {
  c->gpu = gpu;
  const char *co = getenv("VIGPATH_COALESCED");
  c->coalesced_io = !co || atoi(co) != 0;  // default on (tools/ablate.py)
  VP_HIP(hipSetDevice(gpu));
  VP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  VP_TRY(preload_units(gpu, c->stream));
  VP_HIP(hipEventCreate(&c->ev0));
  VP_HIP(hipEventCreate(&c->ev1));
  VP_HIP(hipEventCreateWithFlags(&c->evc, hipEventDisableTiming));
  VP_HIP(hipEventCreate(&c->ev2));
  VP_HIP(hipEventCreate(&c->ev3));
  return 0;
}

static void free_all(vp_ctx *c) {
  if (!c) return;
  hipSetDevice(c->gpu);
  serve_free(c);  // (vp_process_one's kernel: stopped first)
  if (c->stream) hipStreamSynchronize(c->stream);
  tbl_free(c->ft);
  tbl_free(c->ft2);
  Workspace &w = c->ws;
  ws_release(w);
  for (const HostMap &h : c->hmaps)  // (registered by vp_register_host)
    if (h.ours) hipHostUnregister(reinterpret_cast<void *>(h.hbase));
  void *mb[] = {w.mb_ptr, w.mb_slots, w.mb_tail, w.mb_flags, w.mb_len, w.mb_in,
                w.mb_out, w.mb_now, w.mb_full, w.st_meta};
  for (void *p : mb) hipFree(p);
  if (w.h_mbflags) hipHostFree(w.h_mbflags);
  if (w.h_mbmeta) hipHostFree(w.h_mbmeta);
  if (w.h_mbslots) hipHostFree(w.h_mbslots);
  if (w.h_mbtail) hipHostFree(w.h_mbtail);
  for (int i = 0; i < Workspace::kMbufSets; i++) {
    if (w.mb_ev_in[i]) hipEventDestroy(w.mb_ev_in[i]);
    if (w.mb_ev_done[i]) hipEventDestroy(w.mb_ev_done[i]);
    if (w.mb_ev_out[i]) hipEventDestroy(w.mb_ev_out[i]);
  }
  void *ptrs[] = {w.hist, w.hoff, w.cub_tmp, w.d_frames, w.d_len,    w.d_in,
                  w.bins_ent, w.bins_cnt, w.bins_rtab,
                  w.d_out,   w.d_now,    c->crc_tab, c->macw,
                  c->st_bk,  c->st_val,  c->be_rec,   c->cht,   c->dmacw,
                  w.sbuf,    w.rbuf,     c->pol_size, c->pol_time,
                  c->pol_cnt, c->pol_off, c->pol_runs, w.desc, w.dcnt, w.dbase, w.dtot,
                  w.route,   w.sendk,    w.recvk,  w.reply,  w.rreply,
                  w.cnt_t,   w.rcnt_t,   w.dneed,  w.xsend, w.sendk2, w.recvk2,
                  w.reply2,  w.rreply2,  w.lcnt, w.nkset, w.nkbits, w.nkpre,
                  w.nkfirst, w.nkcnt, w.in_fill};
  for (void *p : ptrs) hipFree(p);
  for (int i = 0; i < 2; i++) {
    if (w.ev_p1[i]) hipEventDestroy(w.ev_p1[i]);
    if (w.ev_ans[i]) hipEventDestroy(w.ev_ans[i]);
  }
  if (w.xstream) {
    hipStreamSynchronize(w.xstream);
    hipStreamDestroy(w.xstream);
  }
  if (w.h_tot) hipHostFree(w.h_tot);
  if (w.h_frames) hipHostFree(w.h_frames);
  if (w.h_meta) hipHostFree(w.h_meta);
  for (int i = 0; i < 3; i++) {
    if (w.ev_in[i]) hipEventDestroy(w.ev_in[i]);
    if (w.ev_done[i]) hipEventDestroy(w.ev_done[i]);
    if (w.ev_out[i]) hipEventDestroy(w.ev_out[i]);
  }
  if (w.cstream) hipStreamDestroy(w.cstream);
  if (w.dstream) hipStreamDestroy(w.dstream);
  delete c->comm;
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  if (c->evc) hipEventDestroy(c->evc);
  if (c->ev2) hipEventDestroy(c->ev2);
  if (c->ev3) hipEventDestroy(c->ev3);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

static int upload(uint32_t **dst, const std::vector<uint32_t> &v) {
  VP_TRY(dalloc(dst, v.size()));
  VP_HIP(hipMemcpy(*dst, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  return 0;
}

// The allocation-order home-bucket layout (vp_table.hip tbl_try_linear) for
// a table whose indices the dchain hands out in arrival order: VIGPATH_LIN 0
// off, 1 one index per bucket, 2 two per bucket (the default).
static void lin_enable(FlowTable &t) {
  const char *lin = getenv("VIGPATH_LIN");
  t.lin_ok = lin ? (uint32_t)atoi(lin) : 2u;
}

static int nat_init(vp_ctx *c, const vp_nat_config *cfg) {
  c->kind = KIND_NAT;
  c->nat = *cfg;
  VP_TRY(tbl_alloc(c, c->ft, cfg->max_flows));
  lin_enable(c->ft);
  std::vector<uint32_t> tab;
  build_flowid_tables(tab);
  VP_TRY(upload(&c->crc_tab, tab));
  std::vector<uint32_t> mw(3 * VP_MAX_DEVICES, 0);
  for (int d = 0; d < cfg->n_devices; d++)
    mac_words(cfg->endpoint_macs[d], cfg->device_macs[d], &mw[3 * d]);
  memcpy(c->wan_macw, &mw[3 * cfg->wan_device], sizeof c->wan_macw);
  VP_TRY(upload(&c->macw, mw));
  return 0;
}

static int bridge_init(vp_ctx *c, const vp_bridge_config *cfg) {
  c->kind = KIND_BRIDGE;
  c->brg = *cfg;
  c->brg.static_rules = nullptr;
  VP_TRY(tbl_alloc(c, c->ft, cfg->dyn_capacity));
  lin_enable(c->ft);
  std::vector<uint32_t> tab;
  build_bridge_tables(tab);
  VP_TRY(upload(&c->crc_tab, tab));
  std::vector<Bucket> bk;
  VP_TRY(bridge_static_build(cfg, bk, &c->st_bmask));
  VP_TRY(dalloc(&c->st_bk, bk.size()));
  VP_HIP(hipMemcpy(c->st_bk, bk.data(), bk.size() * sizeof(Bucket),
                   hipMemcpyHostToDevice));
  std::vector<int32_t> val(cfg->n_static + 1, 0);
  for (uint32_t r = 0; r < cfg->n_static; r++)
    val[r] = cfg->static_rules[r].device_to;
  VP_TRY(dalloc(&c->st_val, val.size()));
  VP_HIP(hipMemcpy(c->st_val, val.data(), val.size() * 4, hipMemcpyHostToDevice));
  c->n_static = cfg->n_static;
  return 0;
}

static int lb_init(vp_ctx *c, const vp_lb_config *cfg) {
  c->kind = KIND_LB;
  c->lb = *cfg;
  VP_TRY(tbl_alloc(c, c->ft, cfg->flow_capacity));
  lin_enable(c->ft);
  VP_TRY(tbl_alloc(c, c->ft2, cfg->backend_capacity));
  std::vector<uint32_t> tab;
  build_lb_tables(tab);
  VP_TRY(upload(&c->crc_tab, tab));
  std::vector<uint32_t> cht;
  lb_fill_cht(cfg->cht_height, cfg->backend_capacity, cht);
  VP_TRY(upload(&c->cht, cht));
  VP_TRY(dalloc(&c->be_rec, cfg->backend_capacity));
  VP_HIP(hipMemset(c->be_rec, 0, sizeof(uint4) * cfg->backend_capacity));
  std::vector<uint32_t> dm(2 * VP_MAX_DEVICES, 0);
  for (int d = 0; d < cfg->n_devices; d++) {
    const uint8_t *m = cfg->device_macs[d];
    dm[2 * d] = ((uint32_t)m[0] | ((uint32_t)m[1] << 8)) << 16;
    dm[2 * d + 1] = m[2] | (m[3] << 8) | (m[4] << 16) | ((uint32_t)m[5] << 24);
  }
  VP_TRY(upload(&c->dmacw, dm));
  return 0;
}

static int fw_init(vp_ctx *c, const vp_fw_config *cfg) {
  c->kind = KIND_FW;
  c->fw = *cfg;
  VP_TRY(tbl_alloc(c, c->ft, cfg->max_flows));
  lin_enable(c->ft);
  std::vector<uint32_t> tab;
  build_fw_tables(tab);
  VP_TRY(upload(&c->crc_tab, tab));
  std::vector<uint32_t> mw(3 * VP_MAX_DEVICES, 0);
  for (int d = 0; d < cfg->n_devices; d++)
    mac_words(cfg->endpoint_macs[d], cfg->device_macs[d], &mw[3 * d]);
  VP_TRY(upload(&c->macw, mw));
  return 0;
}

static int pol_init(vp_ctx *c, const vp_pol_config *cfg) {
  c->kind = KIND_POL;
  c->pol = *cfg;
  VP_TRY(tbl_alloc(c, c->ft, cfg->dyn_capacity));
  lin_enable(c->ft);
  std::vector<uint32_t> tab;
  build_pol_tables(tab);
  VP_TRY(upload(&c->crc_tab, tab));
  // dyn_vals (DynamicValue_allocate zero-fills, vigpol/dataspec.ml:8)
  VP_TRY(dalloc(&c->pol_size, cfg->dyn_capacity));
  VP_TRY(dalloc(&c->pol_time, cfg->dyn_capacity));
  VP_HIP(hipMemset(c->pol_size, 0, 8ull * cfg->dyn_capacity));
  VP_HIP(hipMemset(c->pol_time, 0, 8ull * cfg->dyn_capacity));
  VP_TRY(dalloc(&c->pol_cnt, cfg->dyn_capacity));
  VP_TRY(dalloc(&c->pol_off, cfg->dyn_capacity));
  // (the run slots of the grouping path, 64 per index, are allocated by the
  // first segment that groups: vp_pol.hip pol_runs_reserve)
  return 0;
}

static bool is_prime(uint32_t v) {
  if (v < 2) return false;
  for (uint32_t d = 2; (uint64_t)d * d <= v; d++)
    if (v % d == 0) return false;
  return true;
}

static int stage_meta(vp_ctx *c, uint32_t n) {
  Workspace &w = c->ws;
  if (n <= w.d_meta_n) return 0;
  hipFree(w.d_len);
  hipFree(w.d_in);
  hipFree(w.d_out);
  hipFree(w.d_now);
  w.d_len = w.d_in = w.d_out = nullptr;
  w.d_now = nullptr;
  w.d_meta_n = 0;
  VP_TRY(dalloc(&w.d_len, n));
  VP_TRY(dalloc(&w.d_in, n));
  VP_TRY(dalloc(&w.d_out, n));
  VP_TRY(dalloc(&w.d_now, n));
  w.d_meta_n = n;
  return 0;
}

// Page-locked (hipHostMalloc'd or hipHostRegister'ed, e.g. a DPDK hugepage
// pool) host memory can be DMA'd directly.
static bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Host batch in chunks of `ch` packets, three buffer sets in HBM: one copy
// stream moves chunks k+1 and k+2 in while another moves chunk k-1 out (PCIe
// carries both directions at once: 48.6 GB/s each way together, 57 GB/s
// alone, tools/pcie_probe.hip) and chunk k is processed (chunks are processed
// in order, so results equal one call on the batch). Chunk k+2's copy is
// enqueued while chunk k is processed, so the host->device engine never
// waits for the host (vp_process_device returns only once phase A's counts
// are known). Page-locked arrays (hipHostMalloc'd or hipHostRegister'ed, e.g. a
// DPDK hugepage mbuf pool) are DMA'd in place; pageable ones go through
// pinned staging. With a time array, the host's copy serves the batch
// driver's expiry cuts (vp_ctx::host_now), so it is not read back; with
// affine time (now == NULL) no time crosses PCIe at all.
static int host_pipeline(vp_ctx *c, const vp_host_batch *hb) {
  Workspace &w = c->ws;
  const uint32_t n = hb->n, slot = hb->slot;
  const char *env = getenv("VIGPATH_HOST_CHUNK");
  uint32_t ch = env ? (uint32_t)atoi(env) : (1u << 20);
  if (ch == 0) ch = 1u << 20;
  ch = std::min(ch, n);
  const uint32_t K = (n + ch - 1) / ch;
  const bool pin_fr = is_pinned(hb->frames), pin_len = is_pinned(hb->len),
             pin_in = is_pinned(hb->in_dev), pin_out = is_pinned(hb->out_dev),
             pin_now = hb->now && is_pinned(hb->now);
  constexpr uint32_t S = 3;  // buffer sets
  VP_TRY(stage_meta(c, S * ch));
  {  // device frames (S chunks); pinned staging only for pageable frames
    const size_t bytes = (size_t)S * ch * slot;
    if (bytes > w.d_frames_bytes) {
      hipFree(w.d_frames);
      w.d_frames = nullptr;
      w.d_frames_bytes = 0;
      VP_HIP(hipMalloc((void **)&w.d_frames, bytes));
      w.d_frames_bytes = bytes;
    }
    if (!pin_fr && bytes > w.h_frames_bytes) {
      if (w.h_frames) hipHostFree(w.h_frames);
      w.h_frames = nullptr;
      w.h_frames_bytes = 0;
      VP_HIP(hipHostMalloc((void **)&w.h_frames, bytes, hipHostMallocDefault));
      w.h_frames_bytes = bytes;
    }
  }
  const size_t meta = 14ull * ch;  // len 2 + in 2 + now 8 + out 2 per packet
  if (S * meta > w.h_meta_bytes) {
    if (w.h_meta) hipHostFree(w.h_meta);
    w.h_meta = nullptr;
    w.h_meta_bytes = 0;
    VP_HIP(hipHostMalloc((void **)&w.h_meta, S * meta, hipHostMallocDefault));
    w.h_meta_bytes = S * meta;
  }
  if (!w.cstream) {
    VP_HIP(hipStreamCreateWithFlags(&w.cstream, hipStreamNonBlocking));
    VP_HIP(hipStreamCreateWithFlags(&w.dstream, hipStreamNonBlocking));
    for (uint32_t i = 0; i < S; i++) {
      VP_HIP(hipEventCreateWithFlags(&w.ev_in[i], hipEventDisableTiming));
      VP_HIP(hipEventCreateWithFlags(&w.ev_done[i], hipEventDisableTiming));
      VP_HIP(hipEventCreateWithFlags(&w.ev_out[i], hipEventDisableTiming));
    }
  }
  auto cnt = [&](uint32_t k) { return std::min(ch, n - k * ch); };
  auto hm = [&](uint32_t k) { return w.h_meta + (k % S) * meta; };
  auto dfr = [&](uint32_t k) { return w.d_frames + (size_t)(k % S) * ch * slot; };
  auto hfr = [&](uint32_t k) {
    return pin_fr ? hb->frames + (size_t)k * ch * slot
                  : w.h_frames + (size_t)(k % S) * ch * slot;
  };
  // where chunk k's out ports land on the host
  auto hout = [&](uint32_t k) {
    return pin_out ? hb->out_dev + (size_t)k * ch
                   : reinterpret_cast<uint16_t *>(hm(k) + 12ull * ch);
  };
  // a per-packet array's chunk k: the caller's page-locked memory itself, or
  // a staged copy at offset `at` of the chunk's meta block
  auto src = [&](const void *arr, bool pinned, size_t esz, size_t at, uint32_t k) {
    const uint8_t *a = static_cast<const uint8_t *>(arr) + (size_t)k * ch * esz;
    if (pinned) return a;
    memcpy(hm(k) + at, a, esz * cnt(k));
    return static_cast<const uint8_t *>(hm(k) + at);
  };
  // chunk k's results back to the caller (after its D2H completed)
  auto retire = [&](uint32_t k) -> int {
    VP_HIP(hipEventSynchronize(w.ev_out[k % S]));
    const uint32_t m = cnt(k);
    if (!pin_fr) memcpy(hb->frames + (size_t)k * ch * slot, hfr(k), (size_t)m * slot);
    if (!pin_out) memcpy(hb->out_dev + (size_t)k * ch, hout(k), 2ull * m);
    return 0;
  };
  auto issue_in = [&](uint32_t k) -> int {
    const uint32_t m = cnt(k), o = k * ch, i = k % S;
    if (k >= S) VP_TRY(retire(k - S));  // frees buffer set k % S
    if (!pin_fr) memcpy(hfr(k), hb->frames + (size_t)o * slot, (size_t)m * slot);
    VP_HIP(hipMemcpyAsync(dfr(k), hfr(k), (size_t)m * slot, hipMemcpyHostToDevice,
                          w.cstream));
    VP_HIP(hipMemcpyAsync(w.d_len + i * ch, src(hb->len, pin_len, 2, 0, k), 2ull * m,
                          hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipMemcpyAsync(w.d_in + i * ch, src(hb->in_dev, pin_in, 2, 2ull * ch, k),
                          2ull * m, hipMemcpyHostToDevice, w.cstream));
    if (hb->now)
      VP_HIP(hipMemcpyAsync(w.d_now + i * ch, src(hb->now, pin_now, 8, 4ull * ch, k),
                            8ull * m, hipMemcpyHostToDevice, w.cstream));
    VP_HIP(hipEventRecord(w.ev_in[i], w.cstream));
    return 0;
  };
  for (uint32_t k = 0; k < std::min(K, S - 1); k++) VP_TRY(issue_in(k));
  for (uint32_t k = 0; k < K; k++) {
    const uint32_t i = k % S, m = cnt(k);
    VP_HIP(hipStreamWaitEvent(c->stream, w.ev_in[i], 0));
    vp_dev_batch b{};
    b.frames = dfr(k);
    b.slot = slot;
    b.n = m;
    b.len = w.d_len + i * ch;
    b.in_dev = w.d_in + i * ch;
    b.now = hb->now ? w.d_now + i * ch : nullptr;
    b.now0 = hb->now0 + (int64_t)k * ch * hb->now_step;
    b.now_step = hb->now_step;
    b.out_dev = w.d_out + i * ch;
    c->host_now = hb->now ? hb->now + (size_t)k * ch : nullptr;
    const int rc = vp_process_device(c, &b, nullptr);
    c->host_now = nullptr;
    VP_TRY(rc);
    VP_HIP(hipEventRecord(w.ev_done[i], c->stream));
    VP_HIP(hipStreamWaitEvent(w.dstream, w.ev_done[i], 0));
    VP_HIP(hipMemcpyAsync(hfr(k), dfr(k), (size_t)m * slot, hipMemcpyDeviceToHost,
                          w.dstream));
    VP_HIP(hipMemcpyAsync(hout(k), w.d_out + i * ch, 2ull * m, hipMemcpyDeviceToHost,
                          w.dstream));
    VP_HIP(hipEventRecord(w.ev_out[i], w.dstream));
    if (k + S - 1 < K) VP_TRY(issue_in(k + S - 1));  // (waits for chunk k-1's results)
  }
  for (uint32_t k = K >= S ? K - S : 0; k < K; k++) VP_TRY(retire(k));
  return 0;
}

}  // namespace vp

using namespace vp;

extern "C" {

const char *vp_version(void) { return "vigpath 0.3 gfx950"; }

int vp_nat_create(const vp_nat_config *cfg, int gpu, vp_ctx **out) {
  if (!cfg || !out) return VP_EINVAL;
  // map.c:73 (CAPACITY_POW2): power-of-two capacity; nat_config.c: devices
  if (!is_pow2(cfg->max_flows) || cfg->n_devices == 0 ||
      cfg->n_devices > VP_MAX_DEVICES || cfg->wan_device >= cfg->n_devices ||
      cfg->max_flows > (1u << 30))
    return VP_EINVAL;
  vp_ctx *c = new vp_ctx();
  int rc = ctx_common(c, gpu);
  if (!rc) rc = nat_init(c, cfg);
  if (rc) {
    free_all(c);
    return rc;
  }
  *out = c;
  return 0;
}

int vp_bridge_create(const vp_bridge_config *cfg, int gpu, vp_ctx **out) {
  if (!cfg || !out || (cfg->n_static && !cfg->static_rules)) return VP_EINVAL;
  // map.c:73 (CAPACITY_POW2); bridge_main.c:150-154: the static map (8192
  // entries, bridge_main.c:293) must stay at most half full
  if (!is_pow2(cfg->dyn_capacity) || cfg->dyn_capacity > (1u << 30) ||
      2ull * cfg->n_static >= 8192)
    return VP_EINVAL;
  vp_ctx *c = new vp_ctx();
  int rc = ctx_common(c, gpu);
  if (!rc) rc = bridge_init(c, cfg);
  if (rc) {
    free_all(c);
    return rc;
  }
  *out = c;
  return 0;
}

int vp_lb_create(const vp_lb_config *cfg, int gpu, vp_ctx **out) {
  if (!cfg || !out) return VP_EINVAL;
  // map.c:73 (CAPACITY_POW2) for both maps; cht_fill_cht's precondition
  // (cht.c:546-553): prime height < MAX_CHT_HEIGHT, 0 < backends < height
  if (!is_pow2(cfg->flow_capacity) || cfg->flow_capacity > (1u << 30) ||
      !is_pow2(cfg->backend_capacity) || cfg->backend_capacity >= cfg->cht_height ||
      cfg->cht_height >= 40000 || !is_prime(cfg->cht_height) ||
      cfg->n_devices == 0 || cfg->n_devices > VP_MAX_DEVICES)
    return VP_EINVAL;
  vp_ctx *c = new vp_ctx();
  int rc = ctx_common(c, gpu);
  if (!rc) rc = lb_init(c, cfg);
  if (rc) {
    free_all(c);
    return rc;
  }
  *out = c;
  return 0;
}

int vp_fw_create(const vp_fw_config *cfg, int gpu, vp_ctx **out) {
  if (!cfg || !out) return VP_EINVAL;
  // map.c:73 (CAPACITY_POW2); fw_config.c:39-75: devices, --wan < devices
  if (!is_pow2(cfg->max_flows) || cfg->max_flows > (1u << 30) ||
      cfg->n_devices == 0 || cfg->n_devices > VP_MAX_DEVICES ||
      cfg->wan_device >= cfg->n_devices)
    return VP_EINVAL;
  vp_ctx *c = new vp_ctx();
  int rc = ctx_common(c, gpu);
  if (!rc) rc = fw_init(c, cfg);
  if (rc) {
    free_all(c);
    return rc;
  }
  *out = c;
  return 0;
}

int vp_pol_create(const vp_pol_config *cfg, int gpu, vp_ctx **out) {
  if (!cfg || !out) return VP_EINVAL;
  // policer_config.c:44-77: devices < rte_eth_dev_count_avail(), rate and
  // burst strictly positive; map.c:73 (CAPACITY_POW2)
  if (!is_pow2(cfg->dyn_capacity) || cfg->dyn_capacity > (1u << 30) ||
      cfg->n_devices == 0 || cfg->n_devices > VP_MAX_DEVICES ||
      cfg->lan_device >= cfg->n_devices || cfg->wan_device >= cfg->n_devices ||
      cfg->rate == 0 || cfg->burst == 0)
    return VP_EINVAL;
  vp_ctx *c = new vp_ctx();
  int rc = ctx_common(c, gpu);
  if (!rc) rc = pol_init(c, cfg);
  if (rc) {
    free_all(c);
    return rc;
  }
  *out = c;
  return 0;
}

void vp_destroy(vp_ctx *ctx) { free_all(ctx); }

extern "C++" {
namespace vp {
// VIGPATH_HOSTPROF=1: each call's stages printed as it returns (us from
// entry); =2: recorded as absolute steady-clock times (CLOCK_MONOTONIC, the
// kernel trace's clock) and printed at exit, so that they line up with a
// rocprofv3 kernel trace of the same run without a print between calls
static const int g_hostprof = [] {
  const char *e = getenv("VIGPATH_HOSTPROF");
  return e ? atoi(e) : 0;
}();
static double g_hp[8];
static std::vector<std::array<double, 8>> g_hp_log;
static void hostprof_dump() {
  for (size_t i = 0; i < g_hp_log.size(); i++) {
    fprintf(stderr, "vigpath hostprof abs %zu:", i);
    for (int k = 0; k < 8; k++) fprintf(stderr, " %.3f", g_hp_log[i][k]);
    fprintf(stderr, " (us, CLOCK_MONOTONIC)\n");
  }
}
void hostprof(int k) {
  if (g_hostprof && k >= 0 && k < 8)
    g_hp[k] = std::chrono::duration<double, std::micro>(
                  std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace vp
}

int vp_process_device(vp_ctx *c, const vp_dev_batch *b, void *stream) {
  if (!c || !b) return VP_EINVAL;
  // (nf_process's device is a uint16_t, nf.h:14: the kernels that read the
  // burst's port directly and the port arrays made below must agree)
  if (!b->in_dev && b->in_port > 0xFFFFu) return VP_EINVAL;
  if (vp::g_hostprof) {
    for (double &x : vp::g_hp) x = 0;
    vp::hostprof(0);
  }
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  hipStream_t user = (hipStream_t)stream;
  hipEvent_t dep = nullptr;
  if (user && user != c->stream) {  // order after the caller's stream
    VP_HIP(hipEventCreateWithFlags(&dep, hipEventDisableTiming));
    VP_HIP(hipEventRecord(dep, user));
    VP_HIP(hipStreamWaitEvent(c->stream, dep, 0));
  }
  // one port for the whole batch (in_dev == NULL): vignat's and viglb's
  // 64-byte slots on one GPU read in_port themselves; elsewhere the port
  // array is made here
  vp_dev_batch one;
  if (!b->in_dev && b->n &&
      ((c->kind != KIND_NAT && c->kind != KIND_LB) || c->comm || b->slot != 64)) {
    Workspace &w = c->ws;
    if (w.in_fill_n < b->n) {
      VP_HIP(hipStreamSynchronize(c->stream));
      hipFree(w.in_fill);
      w.in_fill = nullptr;
      w.in_fill_n = 0;
      VP_HIP(hipMalloc((void **)&w.in_fill, 2ull * b->n));
      w.in_fill_n = b->n;
    }
    VP_HIP(hipMemsetD16Async(w.in_fill, (uint16_t)b->in_port, b->n, c->stream));
    one = *b;
    one.in_dev = w.in_fill;
    b = &one;
  }
  int rc = VP_ENOTSUP;
  switch (c->kind) {
    case KIND_NAT:
      rc = nat_process_device(c, b);
      break;
    case KIND_BRIDGE:
      rc = bridge_process_device(c, b);
      break;
    case KIND_LB:
      rc = lb_process_device(c, b);
      break;
    case KIND_FW:
      rc = fw_process_device(c, b);
      break;
    case KIND_POL:
      rc = pol_process_device(c, b);
      break;
    default:
      break;
  }
  if (dep) {
    hipEventRecord(dep, c->stream);
    hipStreamWaitEvent(user, dep, 0);
    hipEventDestroy(dep);
  }
  if (vp::g_hostprof == 2) {
    vp::hostprof(7);
    if (vp::g_hp_log.empty()) atexit(vp::hostprof_dump);
    std::array<double, 8> r;
    for (int k = 0; k < 8; k++) r[k] = vp::g_hp[k];
    if (vp::g_hp_log.size() < 4096) vp::g_hp_log.push_back(r);
  } else if (vp::g_hostprof) {  // entry -> classify issued -> fold issued -> ctl seen -> exit
    vp::hostprof(7);
    fprintf(stderr, "vigpath hostprof:");
    for (int k = 1; k < 8; k++)
      if (vp::g_hp[k] > 0) fprintf(stderr, " s%d %.1f", k, vp::g_hp[k] - vp::g_hp[0]);
    fprintf(stderr, " us\n");
  }
  return rc;
}

int vp_process_one(vp_ctx *c, uint16_t in_dev, uint8_t *frame, uint16_t len, int64_t now,
                   uint16_t *out_dev) {
  if (!c || !frame || !out_dev) return VP_EINVAL;
  if (c->kind == KIND_NAT) {
    // (no hipSetDevice here: a served packet makes no HIP call; the server's
    // launch and stop set the device themselves)
    const int rc = nat_process_one(c, in_dev, frame, len, now, out_dev);
    if (rc <= 0) return rc;  // (1: not eligible, the batch path below)
    if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  }
  uint8_t *frames[1] = {frame};
  return vp_process_batch(c, 1, &in_dev, frames, &len, &now, out_dev);
}

int vp_process_host_batch(vp_ctx *c, const vp_host_batch *b) {
  if (!c || !b) return VP_EINVAL;
  if (b->n && (!b->in_dev || !b->frames || !b->len || !b->out_dev)) return VP_EINVAL;
  if (b->n == 0) return 0;
  if (b->slot < 64 || (b->slot & 15)) return VP_EINVAL;
  if (!b->now && (b->now_step < 0 || b->now0 < 0)) return VP_ENOTSUP;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  return host_pipeline(c, b);
}

int vp_process_host(vp_ctx *c, uint32_t n, const uint16_t *in_dev,
                    uint8_t *frames, uint32_t slot, const uint16_t *len,
                    const int64_t *now, uint16_t *out_dev) {
  if (!c || (n && !now)) return VP_EINVAL;
  vp_host_batch b{};
  b.frames = frames;
  b.slot = slot;
  b.n = n;
  b.len = len;
  b.in_dev = in_dev;
  b.now = now;
  b.out_dev = out_dev;
  return vp_process_host_batch(c, &b);
}

int vp_nat_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys) {
  if (!c || c->kind != KIND_NAT || !alloc || !ts || !keys) return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  return nat_dump(c, alloc, ts, keys);
}

int vp_bridge_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *macs,
                   uint16_t *port) {
  if (!c || c->kind != KIND_BRIDGE || !alloc || !ts || !macs || !port)
    return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  std::vector<uint32_t> keys(4ull * c->ft.cap);
  VP_TRY(tbl_dump(c, c->ft, alloc, ts, keys.data()));
  for (uint32_t i = 0; i < c->ft.cap; i++) {
    const uint32_t *k = &keys[4ull * i];
    memcpy(macs + 6ull * i, k, 4);
    memcpy(macs + 6ull * i + 4, k + 1, 2);
    port[i] = (uint16_t)k[2];
  }
  return 0;
}

int vp_fw_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint8_t *keys,
               uint32_t *int_dev) {
  if (!c || c->kind != KIND_FW || !alloc || !ts || !keys || !int_dev)
    return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  return fw_dump(c, alloc, ts, keys, int_dev);
}

int vp_pol_dump(vp_ctx *c, uint8_t *alloc, int64_t *ts, uint32_t *keys,
                uint64_t *bucket_size, int64_t *bucket_time) {
  if (!c || c->kind != KIND_POL || !alloc || !ts || !keys || !bucket_size ||
      !bucket_time)
    return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  return pol_dump(c, alloc, ts, keys, bucket_size, bucket_time);
}

int64_t vp_live_count(vp_ctx *c) {
  if (!c) return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  if (hipStreamSynchronize(c->stream) != hipSuccess) return VP_EIO;
  Ctl h{};
  if (hipMemcpy(&h, c->ft.ctl, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)
    return VP_EIO;
  int64_t live = h.n_live;
  if (c->kind == KIND_LB) {
    if (hipMemcpy(&h, c->ft2.ctl, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)
      return VP_EIO;
    live += h.n_live;
  }
  return live;
}

int vp_lb_dump(vp_ctx *c, uint8_t *f_alloc, int64_t *f_ts, uint8_t *f_keys,
               uint32_t *f_backend, uint8_t *b_alloc, int64_t *b_ts,
               uint32_t *b_ip, uint8_t *b_mac, uint16_t *b_nic) {
  if (!c || c->kind != KIND_LB || !f_alloc || !f_ts || !f_keys || !f_backend ||
      !b_alloc || !b_ts || !b_ip || !b_mac || !b_nic)
    return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  return lb_dump(c, f_alloc, f_ts, f_keys, f_backend, b_alloc, b_ts, b_ip, b_mac,
                 b_nic);
}

int vp_table_stats_get(vp_ctx *c, int table, vp_table_stats *out) {
  if (!c || !out || table < 0 || table > 1 || (table == 1 && c->kind != KIND_LB))
    return VP_EINVAL;
  if (hipSetDevice(c->gpu) != hipSuccess) return VP_EIO;
  VP_TRY(serve_stop(c));
  const vp::FlowTable &t = table ? c->ft2 : c->ft;
  VP_HIP(hipStreamSynchronize(c->stream));
  Ctl h{};
  VP_HIP(hipMemcpy(&h, t.ctl, sizeof h, hipMemcpyDeviceToHost));
  *out = vp_table_stats{};
  out->live = h.n_live;
  out->shard_live = h.sh_live;
  out->tombstones = h.n_tomb;
  out->buckets = (uint64_t)t.bmask + 1;
  out->rebuilds = t.rebuilds;
  out->layout = t.mix;
  return 0;
}

const char *vp_last_error(void) { return vp::g_last_error; }

int vp_kernel_timing(vp_ctx *c, int on) {
  if (!c) return VP_EINVAL;
  c->ktime = on != 0;
  return 0;
}

int vp_stage_ms(vp_ctx *c, float *ms, int cap, int *stages) {
  static_assert(kStages == VP_STAGES, "include/vigpath.h VP_STAGES");
  if (!c || !stages || cap < 0 || (cap > 0 && !ms)) return VP_EINVAL;
  for (int i = 0; i < kStages && i < cap; i++) ms[i] = c->stage_ms[i];
  *stages = c->stage_n;
  return 0;
}

// (the 0.2 contract: seven floats; the chunked pipeline's ms[7] only through
// vp_stage_ms)
int vp_last_stage_ms(vp_ctx *c, float *ms, int *stages) {
  const int rc = vp_stage_ms(c, ms, 7, stages);
  if (rc == 0 && *stages > 7) *stages = 7;
  return rc;
}

const char *vp_last_kernel(vp_ctx *c) { return c ? c->last_kernel : ""; }

int vp_last_kernel_ms(vp_ctx *c, float *ms, int *launches) {
  if (!c || !ms || !launches) return VP_EINVAL;
  *ms = c->last_ms;
  *launches = c->last_launches;
  return 0;
}

}  // extern "C"
