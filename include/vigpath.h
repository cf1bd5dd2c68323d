/*
 * vigpath — MI355X-native implementation of Vigor's per-packet receive path
 * (parse -> CRC32C flow hash -> libVig map probe -> state update -> header
 * rewrite + IPv4/L4 checksum) for vignat, vigbridge, viglb, vigfw and vigpol.
 *
 * C ABI only: plain pointers and sizes, no HIP or torch types. Two layers:
 *
 *  1. The reference's own operator surface, nf.h (reference nf.h:8-18):
 *       bool nf_init(void);
 *       int  nf_process(uint16_t device, uint8_t *buffer,
 *                       uint16_t packet_length, vigor_time_t now);
 *       void nf_config_init(int argc, char **argv); nf_config_usage();
 *       nf_config_print(); FLOOD_FRAME
 *     exported by the per-NF shim libraries libvignat_nf.so /
 *     libvigbridge_nf.so / libviglb_nf.so / libvigfw_nf.so /
 *     libvigpol_nf.so (one NF per binary, as the
 *     reference builds one NF per binary, Makefile.dpdk). They link unchanged
 *     against the reference's nf.c (nf.c:143-216). See INTEGRATION.md.
 *
 *  2. The batch interface those shims sit on (libvigpath.so), which is what a
 *     batching caller (nf.c's VIGOR_BATCH_SIZE path, nf.c:178-215, or a GPU
 *     host loop) binds. It replaces the per-packet loop
 *     `for each mbuf: nf_process(...)` (nf.c:150-176) with one call per
 *     batch whose results are identical to calling nf_process on every
 *     packet in order.
 *
 * Error convention: 0 on success, a negative errno-style code on failure;
 * never aborts. "Drop" keeps the reference encoding: out_dev == in_dev.
 */
#ifndef VIGPATH_H
#define VIGPATH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP_FLOOD_FRAME ((uint16_t)-1) /* nf.h:8 FLOOD_FRAME */
#define VP_MAX_DEVICES 32

/* error codes (negated errno values) */
#define VP_OK 0
#define VP_EINVAL (-22)
#define VP_ENOMEM (-12)
#define VP_EIO (-5)       /* HIP runtime failure */
#define VP_ENOTSUP (-95)  /* outside the supported domain */
#define VP_ESTATE (-71)   /* EPROTO: a device-side protocol of the library broke
                           * (e.g. the fold kernel ended without publishing its
                           * control block); distinct from a HIP failure */

typedef struct vp_ctx vp_ctx;

/* ------------------------------------------------------------ configs --
 * Field meanings and units are exactly the reference's struct nf_config. */

/* vignat/nat_config.h:5-31 (+ the device MACs nf_config_init reads through
 * rte_eth_macaddr_get, nat_config.c:34-37). */
typedef struct vp_nat_config {
  uint16_t wan_device;
  uint16_t lan_main_device;
  uint16_t start_port;
  uint32_t external_addr;   /* host-order value, as nf_parse_ipv4addr makes */
  uint32_t expiration_time; /* microseconds */
  uint32_t max_flows;       /* power of two (map.c:73, -DCAPACITY_POW2) */
  uint16_t n_devices;       /* rte_eth_dev_count_avail() */
  uint8_t device_macs[VP_MAX_DEVICES][6];
  uint8_t endpoint_macs[VP_MAX_DEVICES][6];
} vp_nat_config;

/* vigbridge/bridge_config.h:8-18; the --config static table is passed as
 * rules instead of a file name (bridge_main.c:130-230 parses the file into
 * exactly these triples). */
typedef struct vp_bridge_rule {
  uint8_t mac[6];
  int32_t device_from;
  int32_t device_to; /* -2 filters (bridge_main.c:322-325) */
} vp_bridge_rule;
typedef struct vp_bridge_config {
  uint32_t expiration_time; /* microseconds */
  uint32_t dyn_capacity;    /* power of two */
  uint16_t n_devices;
  uint32_t n_static;
  const vp_bridge_rule *static_rules;
} vp_bridge_config;

/* viglb/lb_config.h:8-38 */
typedef struct vp_lb_config {
  uint32_t flow_capacity;           /* power of two */
  uint32_t flow_expiration_time;    /* microseconds */
  uint32_t backend_capacity;        /* power of two, < cht_height */
  uint32_t cht_height;              /* prime */
  uint32_t backend_expiration_time; /* microseconds */
  uint16_t wan_device;
  uint16_t n_devices;
  uint8_t device_macs[VP_MAX_DEVICES][6];
} vp_lb_config;

/* vigfw/fw_config.h:9-24 (+ device MACs, as for vignat). */
typedef struct vp_fw_config {
  uint16_t wan_device;
  uint32_t expiration_time; /* microseconds */
  uint32_t max_flows;       /* power of two (map.c:73, -DCAPACITY_POW2) */
  uint16_t n_devices;       /* rte_eth_dev_count_avail() */
  uint8_t device_macs[VP_MAX_DEVICES][6];
  uint8_t endpoint_macs[VP_MAX_DEVICES][6];
} vp_fw_config;

/* vigpol/policer_config.h:8-24 (policer_config.c:17-93 parses it). */
typedef struct vp_pol_config {
  uint16_t lan_device;
  uint16_t wan_device;
  uint64_t rate;         /* B/s, > 0 */
  uint64_t burst;        /* B, > 0 */
  uint32_t dyn_capacity; /* power of two (map.c:73, -DCAPACITY_POW2) */
  uint16_t n_devices;    /* rte_eth_dev_count_avail() */
} vp_pol_config;

/* Create an NF instance whose state lives in HBM of HIP device `gpu`.
 * Returns 0 and *out, or VP_EINVAL for a configuration the reference's
 * nf_init would reject (non power-of-two capacities, ...). */
int vp_nat_create(const vp_nat_config *cfg, int gpu, vp_ctx **out);
int vp_bridge_create(const vp_bridge_config *cfg, int gpu, vp_ctx **out);
int vp_lb_create(const vp_lb_config *cfg, int gpu, vp_ctx **out);
int vp_fw_create(const vp_fw_config *cfg, int gpu, vp_ctx **out);
int vp_pol_create(const vp_pol_config *cfg, int gpu, vp_ctx **out);
void vp_destroy(vp_ctx *ctx);

/* ------------------------------------------------------------ batches -- */

/* A batch already resident in device memory (all pointers are device
 * pointers). Frames sit `slot` bytes apart from a 16-byte aligned start and
 * are rewritten in place, like the mbuf data nf_process mutates
 * (nf.c:154-156). `slot` must be a multiple of 16 and >= 64 (wider slots:
 * frames up to the slot, e.g. 1518 B in 1536 or mbuf-sized 2048). Bytes past a frame's slot read as 0.
 * Time: if `now` is NULL, packet i has now0 + i * now_step (ns); otherwise
 * now[i]. Times must be non-decreasing (nf.c takes them from
 * CLOCK_MONOTONIC, vigor-time.c:56-66) and >= 0 (nat_flowmanager.c:58). */
typedef struct vp_dev_batch {
  uint8_t *frames;
  uint32_t slot;
  uint32_t n;
  const uint16_t *len;
  const uint16_t *in_dev;
  const int64_t *now;
  int64_t now0;
  int64_t now_step;
  uint16_t *out_dev; /* nf_process's return value, stored as u16 (nf.c:156) */
  /* in_dev == NULL: every packet arrived on port in_port (nf.c receives each
   * burst from one device, nf.c:150-153 / 186-190), and no per-packet port
   * array is read. vp_process_device only; the host entry points need
   * in_dev. A port above 0xFFFF (nf_process's uint16_t device, nf.h:14) is
   * VP_EINVAL. */
  uint32_t in_port;
} vp_dev_batch;

/* Process one device-resident batch on HIP stream `stream` (a hipStream_t,
 * or NULL for the context's own stream). Returns after the results (frames,
 * out_dev) are in device memory; from then on no work of the library reads
 * the caller's buffers, so all of them (the per-packet time array included)
 * may be refilled or freed at once. With affine time (now == NULL) the fold
 * of the flow timestamps, which reads only library workspace, may still be
 * running on the context's stream when it returns; it is ordered before
 * every later call on this context (dumps, counts, the next batch) and
 * before work enqueued on `stream` afterwards. A batch with a time array
 * completes entirely before the call returns. */
int vp_process_device(vp_ctx *ctx, const vp_dev_batch *batch, void *stream);

/* Host memory the GPU may read and write frames in directly: a DPDK mbuf
 * pool's memory (the hugepages rte_pktmbuf_pool_create, nf.c:235-242, lays
 * the mbufs out in), registered once after the pool is created. Page-locked
 * and mapped for the context's GPU (hipHostRegister; memory that is page-
 * locked already, e.g. hipHostMalloc'd, is only mapped). At most 16 ranges,
 * not overlapping. vp_unregister_host takes the base passed to
 * vp_register_host; vp_destroy unregisters what is left. */
int vp_register_host(vp_ctx *ctx, void *base, size_t bytes);
int vp_unregister_host(vp_ctx *ctx, void *base);

/* Host-resident batch shaped like DPDK rx bursts (nf.c:186-214): frames[i]
 * is the data of mbuf i (rte_pktmbuf_mtod, nf.c:154), len[i] its pkt_len,
 * in_dev[i] its port; every frame is rewritten in place and out_dev[i] gets
 * nf_process's return value, as calling nf_process on every packet in order
 * would (nf.c:150-176). Time: now[i], or now0 + i * now_step when now is
 * NULL (nf.c's per-packet loop stamps a polling sweep over the devices with
 * one current_time(), nf.c:56: now_step 0; its batched loop stamps every
 * packet, nf.c:197: a time array, or now_step > 0).
 * Frames inside memory registered with vp_register_host are read and written
 * by the GPU in place, in pipelined chunks: per frame the
 * first 64 bytes and, for vignat, the bytes its L4 checksum covers cross
 * PCIe inbound, and the bytes a rewrite can change (the first min(len, 64)
 * of a frame that is not dropped) outbound. Other frames are gathered and
 * scattered on the host through pinned staging. Bytes past a frame's length
 * read as 0 and are never written. Per-packet arrays in page-locked memory
 * are DMA'd in place. Frames and out_dev hold the results when the call
 * returns. */
typedef struct vp_mbuf_batch {
  uint32_t n;
  uint8_t *const *frames;
  const uint16_t *len;
  const uint16_t *in_dev;
  const int64_t *now;
  int64_t now0;
  int64_t now_step;
  uint16_t *out_dev;
} vp_mbuf_batch;
int vp_process_mbufs(vp_ctx *ctx, const vp_mbuf_batch *batch);

/* The same with a per-packet time array (the batch form of nf_process the
 * nf.h shims call). */
int vp_process_batch(vp_ctx *ctx, uint32_t n, const uint16_t *in_dev,
                     uint8_t *const *frames, const uint16_t *len,
                     const int64_t *now, uint16_t *out_dev);

/* One packet: nf_process (nf.h:14-15, called once per packet by nf.c:150-176;
 * the nf.h shims' nf_process calls this). The frame is rewritten in place and
 * the output port stored in *out_dev; same results as vp_process_batch with
 * n = 1. vignat on one GPU serves it from a persistent kernel that polls a
 * host-coherent mailbox (no launch per packet) while no flow expiry is due at
 * `now`; otherwise, and for the other NFs, it is vp_process_batch with n = 1.
 * The kernel leaves after VIGPATH_SERVE_IDLE_MS (default 20) without a
 * packet, at any other call on the context, and at exit; VIGPATH_SERVE=0
 * turns it off. */
int vp_process_one(vp_ctx *ctx, uint16_t in_dev, uint8_t *frame, uint16_t len,
                   int64_t now, uint16_t *out_dev);

/* Host-resident contiguous batch (frames `slot` bytes apart). */
int vp_process_host(vp_ctx *ctx, uint32_t n, const uint16_t *in_dev,
                    uint8_t *frames, uint32_t slot, const uint16_t *len,
                    const int64_t *now, uint16_t *out_dev);

/* The same with every field of vp_dev_batch, as host pointers: time is
 * now[i], or now0 + i * now_step when now is NULL (nf.c stamps every packet
 * of one polling sweep with one current_time(), nf.c:56: now_step 0). Arrays
 * in page-locked memory (hipHostMalloc / hipHostRegister, e.g. a DPDK
 * hugepage pool) are DMA'd in place, others staged through pinned memory.
 * Frames and out_dev hold the results when the call returns. */
typedef vp_dev_batch vp_host_batch;
int vp_process_host_batch(vp_ctx *ctx, const vp_host_batch *batch);

/* -------------------------------------------------------- multi-GPU -- *
 * One vignat instance over N GPUs (one process and one context per GPU),
 * identical to a single nf.c processing the concatenation of the ranks'
 * slices (rank 0's packets first) of every global batch. The allocator
 * (dchain free list) is replicated; new flows are all-gathered and allocated
 * identically everywhere; timestamps are per-rank partial maxima merged
 * (all-reduce MAX) only where an expiry may happen. The flow dictionary is
 * either replicated (VP_SHARD_REPLICATED, the default: every rank probes
 * locally) or sharded by flow hash (VP_SHARD_OWNER: rank q's buckets hold
 * the keys with owner(FlowId_hash) = q; a LAN packet whose key another rank
 * owns is looked up there through an all-to-all of 16-byte keys and 4-byte
 * replies). After an attach, vp_process_device is a collective: every rank
 * calls it once per global batch with its own slice (n may be 0), in the
 * same order. See DESIGN.md §6. */

/* RCCL over xGMI: rank 0 creates the id, the host distributes it. */
#define VP_COMM_ID_BYTES 128
int vp_comm_unique_id(uint8_t id[VP_COMM_ID_BYTES]);
int vp_attach_rccl(vp_ctx *ctx, const uint8_t id[VP_COMM_ID_BYTES], int nranks,
                   int rank);

/* Host-memory collectives supplied by the caller (e.g. torch.distributed /
 * gloo, or several ranks sharing one GPU). Return 0 on success. */
typedef struct vp_comm_ops {
  void *user;
  /* every rank contributes `bytes`; recv receives nranks * bytes, rank order */
  int (*allgather)(void *user, const void *send, void *recv, size_t bytes);
  /* element-wise maximum over ranks of `count` u64 values (all < 2^63) */
  int (*allreduce_max_u64)(void *user, uint64_t *buf, size_t count);
  /* personalised exchange (VP_SHARD_OWNER only; may be NULL otherwise):
   * this rank sends send_bytes[q] bytes to rank q, the chunks consecutive in
   * `send` in rank order, and receives recv_bytes[q] bytes from rank q into
   * `recv`, laid out the same way */
  int (*alltoallv)(void *user, const void *send, const size_t *send_bytes,
                   void *recv, const size_t *recv_bytes);
} vp_comm_ops;
int vp_attach_comm(vp_ctx *ctx, const vp_comm_ops *ops, int nranks, int rank);

/* Dictionary placement over the attached ranks (collective; call on every
 * rank with the same mode after the attach and before the first batch). */
#define VP_SHARD_REPLICATED 0
#define VP_SHARD_OWNER 1
int vp_shard_mode(vp_ctx *ctx, int mode);

/* Collective: merge the ranks' timestamps so vp_nat_dump is exact on every
 * rank (the dictionary and allocator are identical everywhere already). */
int vp_sync_state(vp_ctx *ctx);

/* Abort this rank's collectives (not collective itself; any thread, also
 * while another thread is inside a vp_* call on the context): the RCCL
 * communicator is aborted (ncclCommAbort), so a rank waiting for a peer that
 * never comes returns instead of spinning; every later vp_* call on the
 * context that needs the ranks fails with VP_EIO. Host transports
 * (vp_attach_comm) have nothing to abort: returns 0. For watchdogs
 * (bench.py --gpus N); the context may only be destroyed afterwards. */
int vp_comm_abort(vp_ctx *ctx);

/* ------------------------------------------------------- observability -- */

/* vignat state by flow index i < max_flows: alloc[i] (dchain allocated?),
 * ts[i] (timestamp, only meaningful when allocated), key[16*i] (the FlowId
 * bytes, vignat/flow.h:3-10 layout, padding zero). */
int vp_nat_dump(vp_ctx *ctx, uint8_t *alloc, int64_t *ts, uint8_t *keys);

/* vigbridge dynamic table by index i < dyn_capacity: alloc[i], ts[i],
 * macs[6*i] (dyn_keys), port[i] (dyn_vals DynamicValue.device). */
int vp_bridge_dump(vp_ctx *ctx, uint8_t *alloc, int64_t *ts, uint8_t *macs,
                   uint16_t *port);

/* viglb state. Flows i < flow_capacity: f_alloc[i], f_ts[i], f_keys[16*i]
 * (LoadBalancedFlow bytes, lb_flow.h:6-12, padding zero), f_backend[i]
 * (flow_id_to_backend_id). Backends b < backend_capacity: b_alloc[b],
 * b_ts[b], and backends[b] (lb_backend.h:7-11) as b_ip[b], b_mac[6*b],
 * b_nic[b]. */
int vp_lb_dump(vp_ctx *ctx, uint8_t *f_alloc, int64_t *f_ts, uint8_t *f_keys,
               uint32_t *f_backend, uint8_t *b_alloc, int64_t *b_ts,
               uint32_t *b_ip, uint8_t *b_mac, uint16_t *b_nic);

/* vigfw state by flow index i < max_flows: alloc[i], ts[i], key[16*i] (the
 * FlowId bytes, vigfw/flow.h:3-9 layout, padding zero), int_dev[i] (the
 * int_devices vector, fw_flowmanager.c:61-64; 0 where not allocated). */
int vp_fw_dump(vp_ctx *ctx, uint8_t *alloc, int64_t *ts, uint8_t *keys,
               uint32_t *int_dev);

/* vigpol state by index i < dyn_capacity: alloc[i], ts[i], keys[i] (dyn_keys:
 * the destination address, raw network-order u32), bucket_size[i] and
 * bucket_time[i] (dyn_vals, vigpol/dynamic_value.h:7-10; meaningful where
 * allocated). */
int vp_pol_dump(vp_ctx *ctx, uint8_t *alloc, int64_t *ts, uint32_t *keys,
                uint64_t *bucket_size, int64_t *bucket_time);

/* Number of live flows / learned MACs / flows+backends. */
int64_t vp_live_count(vp_ctx *ctx);

/* Bookkeeping of one device table: table 0 = the NF's flow table (vignat /
 * vigfw flows, vigbridge dynamic MACs, viglb flows, vigpol destinations),
 * table 1 = viglb's backend table. */
typedef struct vp_table_stats {
  uint64_t live;        /* allocated indices (dchain) */
  uint64_t shard_live;  /* entries in this rank's buckets (= live unless
                         * VP_SHARD_OWNER) */
  uint64_t tombstones;  /* erased entries not yet rebuilt away */
  uint64_t buckets;     /* 64-byte buckets (3 entries each) */
  uint64_t rebuilds;    /* bucket-array rebuilds since creation */
  uint32_t layout;      /* home-bucket mode (vp_table.h kMix*) */
  uint32_t pad;
} vp_table_stats;
int vp_table_stats_get(vp_ctx *ctx, int table, vp_table_stats *out);

/* Why the calling thread's last failing vp_* call failed: the HIP error and
 * the call site for VP_EIO / VP_ENOMEM, the broken invariant for VP_ESTATE
 * ("" if none was recorded). The text stays until the thread's next failure. */
const char *vp_last_error(void);

/* Per-context kernel timing (diagnostics, off by default): with on != 0,
 * every vp_process_device call brackets its classification kernel launches
 * with HIP events on the stream they run on (about 6 us of kernel-boundary
 * time per call). */
int vp_kernel_timing(vp_ctx *ctx, int on);

/* Kernel timing of the last vp_process_device call: time of the dominant
 * classification kernel in ms, summed over its launches (0 while
 * vp_kernel_timing is off), and the number of launches. */
int vp_last_kernel_ms(vp_ctx *ctx, float *ms, int *launches);

/* The name of the tile kernel the last vp_process_device call launched for
 * its 64-byte slots (vignat picks nat_classify64w or nat_classify64ws per
 * segment; viglb lb_classify64[w]); "" when none was. The
 * string is static. */
const char *vp_last_kernel(vp_ctx *ctx);

/* Owner-sharded multi-GPU contexts (VP_SHARD_OWNER) with kernel timing on:
 * the last vp_process_device call's phase-A stage times in ms, summed over
 * its segments, from HIP events between the stages: ms[0] pass 1 (classify,
 * keys routed), ms[1] offsets (counts all-to-all, overflow all-reduce),
 * ms[2] keys all-to-all, ms[3] owner probe, ms[4] answers all-to-all,
 * ms[5] pass 2 (routed packets rewritten, touches binned), ms[6] fold;
 * the chunked pipeline records ms[7], its chunks' passes,
 * exchanges and probes together (they overlap), and ms[6] only.
 * vp_stage_ms writes at most `cap` floats and sets *stages to the number of
 * stages recorded (0..VP_STAGES, may exceed cap). vp_last_stage_ms is the
 * 0.2 entry point: exactly 7 floats (ms[0..6]), *stages at most 7. */
#define VP_STAGES 8
int vp_stage_ms(vp_ctx *ctx, float *ms, int cap, int *stages);
int vp_last_stage_ms(vp_ctx *ctx, float *ms, int *stages);

/* Diagnostics (bench.py): the memory-shape ceiling of the classify tile --
 * n slots of `slot` (64 or 128) bytes at `frames` (device memory, n a
 * multiple of 64) streamed with nat_classify64's grid and access shape, each
 * slot read and, store != 0, written back unchanged (write-through). *ms =
 * the mean duration of `reps` launches, each timed by its own dispatch's
 * timestamps. DESIGN.md §5.1. vp_probe_slots_w: the same with `waves` (4,
 * 8, 12 or 16) waves per block, as many blocks per CU as 16 waves make (16:
 * nat_classify64w's one 1024-thread block per CU, its tile order as
 * VIGPATH_SPLIT sets it); vp_probe_slots is waves = 4. */
int vp_probe_slots(void *frames, uint32_t n, uint32_t slot, int store, int reps, float *ms);
int vp_probe_slots_w(void *frames, uint32_t n, uint32_t slot, int store, int waves, int reps,
                     float *ms);

/* Build identification (e.g. "vigpath gfx950"). */
const char *vp_version(void);

/* Exported by the nf.h shim libraries (libvig*_nf.so), not libvigpath.so:
 * the context nf_init() created, so a batching caller can pass it to
 * vp_process_batch / vp_process_device. NULL before nf_init(). */
vp_ctx *vp_nf_context(void);

#ifdef __cplusplus
}
#endif
#endif
