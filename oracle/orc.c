/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orc.h).
 *
 * NF glue restated from the reference (paths relative to /root/reference):
 *   nf.c:150-176            trace dispatch (orc_run)
 *   nf-util.h:116-162       header "borrow" parse with the packet-io cursor
 *   nf-util.c:21-64         predicates + checksum rewrite
 *   DPDK 20.08 rte_ip.h     rte_raw_cksum / rte_ipv4_cksum / rte_ipv4_phdr_cksum
 *                           / rte_ipv4_udptcp_cksum (not vendored; restated,
 *                           version pinned at setup.sh:94)
 *   vignat/nat_main.c:14-109, nat_flowmanager.c:20-94
 *   vigbridge/bridge_main.c:29-128, 292-329
 *   viglb/lb_main.c:13-68, lb_balancer.c:22-237
 *   vigfw/fw_main.c:21-80, fw_flowmanager.c:38-86
 *   vigpol/policer_main.c:21-145
 *   codegen/main.ml:163-206, 328-401, 444-486 (generated _eq/_hash/_allocate)
 * libVig is reached only through orc_lv.h, so the same glue runs over the
 * restated libVig (liborc.so) or the reference's own (oracle/_ref).
 */
#include "orc.h"

#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

#include "orc_lv.h"

/* ------------------------------------------------------------- CRC32C --
 * `__builtin_ia32_crc32si` (boilerplate-util.h:9): SSE4.2 crc32 r32 =
 * reflected CRC-32C (poly 0x82F63B78) over the 4 LE bytes of the operand, no
 * pre/post inversion. The _ref build uses the hardware instruction itself. */
#ifdef ORC_HW_CRC
uint32_t orc_crc32c_u32(uint32_t crc, uint32_t v) {
  return __builtin_ia32_crc32si(crc, v);
}
#else
static uint32_t crc_tab[256];
static int crc_ready;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    crc_tab[i] = c;
  }
  crc_ready = 1;
}
uint32_t orc_crc32c_u32(uint32_t crc, uint32_t v) {
  if (!crc_ready) crc_init();
  for (int b = 0; b < 4; b++) {
    crc = crc_tab[(crc ^ v) & 0xFFu] ^ (crc >> 8);
    v >>= 8;
  }
  return crc;
}
#endif

const char *orc_impl_name(void) { return lv_impl_name(); }

/* ---------------------------------------------------------- key types -- */
/* vignat/flow.h:3-10 */
struct FlowId {
  uint16_t src_port;
  uint16_t dst_port;
  uint32_t src_ip;
  uint32_t dst_ip;
  uint16_t internal_device;
  uint8_t protocol;
};
/* vigfw/flow.h:3-9 (13 bytes + padding) */
struct FwFlowId {
  uint16_t src_port;
  uint16_t dst_port;
  uint32_t src_ip;
  uint32_t dst_ip;
  uint8_t protocol;
};
/* rte_ether.h model :10-12 */
struct EthAddr {
  uint8_t b[6];
};
/* vigbridge/stat_key.h:7-10 */
struct StaticKey {
  struct EthAddr addr;
  uint16_t device;
};
/* vigbridge/dyn_value.h:6-8 */
struct DynamicValue {
  uint16_t device;
};
/* viglb/lb_flow.h:6-12 */
struct LbFlow {
  uint32_t src_ip;
  uint32_t dst_ip;
  uint16_t src_port;
  uint16_t dst_port;
  uint8_t protocol;
};
/* viglb/lb_backend.h:7-11 */
struct LbBackend {
  uint16_t nic;
  struct EthAddr mac;
  uint32_t ip;
};

/* Generated per codegen/main.ml:328-401: one crc step per field, in
 * declaration order, unsigned fields zero-extended to 32 bits. */
static unsigned FlowId_hash(void *k) {
  struct FlowId *f = k;
  unsigned h = 0;
  h = orc_crc32c_u32(h, f->src_port);
  h = orc_crc32c_u32(h, f->dst_port);
  h = orc_crc32c_u32(h, f->src_ip);
  h = orc_crc32c_u32(h, f->dst_ip);
  h = orc_crc32c_u32(h, f->internal_device);
  h = orc_crc32c_u32(h, f->protocol);
  return h;
}
/* codegen/main.ml:163-206: field-wise equality (padding ignored) */
static bool FlowId_eq(void *a, void *b) {
  struct FlowId *x = a, *y = b;
  return x->src_port == y->src_port && x->dst_port == y->dst_port &&
         x->src_ip == y->src_ip && x->dst_ip == y->dst_ip &&
         x->internal_device == y->internal_device && x->protocol == y->protocol;
}
static void FlowId_allocate(void *k) { memset(k, 0, sizeof(struct FlowId)); }

/* vigfw's generated FlowId_hash / _eq / _allocate (codegen/main.ml:163-206,
 * 328-401, 444-486): five CRC steps in field order. */
static unsigned FwFlowId_hash(void *k) {
  struct FwFlowId *f = k;
  unsigned h = 0;
  h = orc_crc32c_u32(h, f->src_port);
  h = orc_crc32c_u32(h, f->dst_port);
  h = orc_crc32c_u32(h, f->src_ip);
  h = orc_crc32c_u32(h, f->dst_ip);
  h = orc_crc32c_u32(h, f->protocol);
  return h;
}
static bool FwFlowId_eq(void *a, void *b) {
  struct FwFlowId *x = a, *y = b;
  return x->src_port == y->src_port && x->dst_port == y->dst_port &&
         x->src_ip == y->src_ip && x->dst_ip == y->dst_ip &&
         x->protocol == y->protocol;
}
static void FwFlowId_allocate(void *k) { memset(k, 0, sizeof(struct FwFlowId)); }

uint32_t orc_fw_flowid_hash(uint16_t sp, uint16_t dp, uint32_t sip, uint32_t dip,
                            uint8_t proto) {
  struct FwFlowId f = {sp, dp, sip, dip, proto};
  return FwFlowId_hash(&f);
}

uint32_t orc_flowid_hash(uint16_t sp, uint16_t dp, uint32_t sip, uint32_t dip,
                         uint16_t dev, uint8_t proto) {
  struct FlowId f = {sp, dp, sip, dip, dev, proto};
  return FlowId_hash(&f);
}

/* libvig/verified/ether.c:3-21, 61-90: six byte-steps. */
static unsigned Eth_hash(void *k) {
  struct EthAddr *a = k;
  unsigned h = 0;
  for (int i = 0; i < 6; i++) h = orc_crc32c_u32(h, a->b[i]);
  return h;
}
static bool Eth_eq(void *a, void *b) {
  return memcmp(((struct EthAddr *)a)->b, ((struct EthAddr *)b)->b, 6) == 0;
}
static void Eth_allocate(void *k) { memset(k, 0, sizeof(struct EthAddr)); }
uint32_t orc_ether_hash(const uint8_t mac[6]) {
  struct EthAddr a;
  memcpy(a.b, mac, 6);
  return Eth_hash(&a);
}

/* StaticKey: nested struct field hashed by its own hash, then crc'd in. */
static unsigned StaticKey_hash(void *k) {
  struct StaticKey *s = k;
  unsigned h = 0;
  h = orc_crc32c_u32(h, Eth_hash(&s->addr));
  h = orc_crc32c_u32(h, s->device);
  return h;
}
static bool StaticKey_eq(void *a, void *b) {
  struct StaticKey *x = a, *y = b;
  return Eth_eq(&x->addr, &y->addr) && x->device == y->device;
}
static void StaticKey_allocate(void *k) {
  memset(k, 0, sizeof(struct StaticKey));
}
static void DynamicValue_allocate(void *k) {
  memset(k, 0, sizeof(struct DynamicValue));
}

static unsigned LbFlow_hash(void *k) {
  struct LbFlow *f = k;
  unsigned h = 0;
  h = orc_crc32c_u32(h, f->src_ip);
  h = orc_crc32c_u32(h, f->dst_ip);
  h = orc_crc32c_u32(h, f->src_port);
  h = orc_crc32c_u32(h, f->dst_port);
  h = orc_crc32c_u32(h, f->protocol);
  return h;
}
static bool LbFlow_eq(void *a, void *b) {
  struct LbFlow *x = a, *y = b;
  return x->src_ip == y->src_ip && x->dst_ip == y->dst_ip &&
         x->src_port == y->src_port && x->dst_port == y->dst_port &&
         x->protocol == y->protocol;
}
static void LbFlow_allocate(void *k) { memset(k, 0, sizeof(struct LbFlow)); }
/* viglb/ip_addr.h:6-8 */
static unsigned IpAddr_hash(void *k) {
  return orc_crc32c_u32(0, *(uint32_t *)k);
}
static bool IpAddr_eq(void *a, void *b) {
  return *(uint32_t *)a == *(uint32_t *)b;
}
static void U32_init(void *k) { *(uint32_t *)k = 0; } /* null_init */
static void LbBackend_allocate(void *k) {
  memset(k, 0, sizeof(struct LbBackend));
}

/* ------------------------------------------------------------- packet --
 * libvig/verified/packet-io.c:8-111: a read cursor over the frame. The
 * lengths are size_t in the reference; packet_get_unread_length returns the
 * difference truncated to u32 (and nf_then_get_rte_ipv4_header further to
 * u16). */
struct pkt {
  uint8_t *buf;
  uint32_t cap;   /* slot bytes: reads past are 0, writes past dropped */
  uint32_t total; /* global_total_length (= pkt_len) */
  uint32_t read;  /* global_read_length */
};
static inline uint8_t rd8(struct pkt *p, uint32_t o) {
  return o < p->cap ? p->buf[o] : 0;
}
static inline uint16_t rd16(struct pkt *p, uint32_t o) { /* raw LE load */
  return (uint16_t)(rd8(p, o) | (rd8(p, o + 1) << 8));
}
static inline uint32_t rd32(struct pkt *p, uint32_t o) {
  return (uint32_t)rd16(p, o) | ((uint32_t)rd16(p, o + 2) << 16);
}
static inline void wr8(struct pkt *p, uint32_t o, uint8_t v) {
  if (o < p->cap) p->buf[o] = v;
}
static inline void wr16(struct pkt *p, uint32_t o, uint16_t v) {
  wr8(p, o, (uint8_t)v);
  wr8(p, o + 1, (uint8_t)(v >> 8));
}
static inline void wr32(struct pkt *p, uint32_t o, uint32_t v) {
  wr16(p, o, (uint16_t)v);
  wr16(p, o + 2, (uint16_t)(v >> 16));
}
static inline uint32_t borrow(struct pkt *p, uint32_t n) {
  uint32_t at = p->read;
  p->read += n;
  return at;
}
static inline uint32_t unread_u32(struct pkt *p) { return p->total - p->read; }
static inline uint16_t be16(uint16_t raw) {
  return (uint16_t)((raw >> 8) | (raw << 8));
}

/* nf-util.h:122-151. Returns 1 and the IPv4 header offset, or 0. */
static int get_ipv4(struct pkt *p, uint32_t eth, uint32_t *ip_out) {
  uint16_t unread = (uint16_t)unread_u32(p);
  /* nf_has_rte_ipv4_header (nf-util.c:21-23): ether_type == be16(0x0800) */
  bool is_ip = rd16(p, eth + 12) == be16(0x0800);
  if (!is_ip | (unread < 20)) return 0;
  uint32_t ip = borrow(p, 20);
  uint8_t ihl = rd8(p, ip) & 0x0F;
  if ((ihl < 5) | (unread < be16(rd16(p, ip + 2)))) return 0;
  uint16_t opt = (uint16_t)((ihl - 5) * 4);
  if ((opt != 0) & ((size_t)unread - 20 >= opt)) borrow(p, opt);
  *ip_out = ip;
  return 1;
}

/* nf-util.h:153-162 + nf_has_tcpudp_header (nf-util.c:25-31) */
static int get_tcpudp(struct pkt *p, uint32_t ip, uint32_t *l4_out) {
  uint8_t proto = rd8(p, ip + 9);
  if (!((proto == 6) | (proto == 17)) | (unread_u32(p) < 4)) return 0;
  *l4_out = borrow(p, 4);
  return 1;
}

/* DPDK 20.08 __rte_raw_cksum + __rte_raw_cksum_reduce */
static uint16_t raw_cksum(struct pkt *p, uint32_t off, uint32_t len) {
  uint32_t sum = 0;
  uint32_t i = 0;
  for (; i + 1 < len; i += 2) sum += rd16(p, off + i);
  if (len & 1) sum += rd8(p, off + i); /* odd byte as the low byte */
  sum = (sum >> 16) + (sum & 0xFFFF);
  sum = (sum >> 16) + (sum & 0xFFFF);
  return (uint16_t)sum;
}
static uint16_t raw_cksum_bytes(const uint8_t *b, uint32_t len) {
  struct pkt q = {(uint8_t *)b, len, len, 0};
  return raw_cksum(&q, 0, len);
}
/* rte_ipv4_udptcp_cksum: raw sum of total_length-20 L4 bytes + pseudo
 * header {src, dst, 0, proto, be16(total_length-20)}, folded once,
 * inverted; 0 -> 0xFFFF. (The UDP-only form of that last rule is a later
 * DPDK change; the TCP-zero edge is "parity unpinned".) */
static uint16_t udptcp_cksum(struct pkt *p, uint32_t ip, uint32_t l4) {
  uint32_t l3_len = be16(rd16(p, ip + 2));
  if (l3_len < 20) return 0;
  uint32_t l4_len = l3_len - 20;
  uint32_t c = raw_cksum(p, l4, l4_len);
  uint8_t ph[12];
  for (int i = 0; i < 4; i++) ph[i] = rd8(p, ip + 12 + i);
  for (int i = 0; i < 4; i++) ph[4 + i] = rd8(p, ip + 16 + i);
  ph[8] = 0;
  ph[9] = rd8(p, ip + 9);
  ph[10] = (uint8_t)(l4_len >> 8);
  ph[11] = (uint8_t)l4_len;
  c += raw_cksum_bytes(ph, 12);
  c = ((c & 0xFFFF0000u) >> 16) + (c & 0xFFFF);
  c = (~c) & 0xFFFF;
  if (c == 0) c = 0xFFFF;
  return (uint16_t)c;
}
/* rte_ipv4_cksum: over sizeof(struct rte_ipv4_hdr) = 20 bytes */
static uint16_t ipv4_cksum(struct pkt *p, uint32_t ip) {
  return (uint16_t)~raw_cksum(p, ip, 20);
}
/* nf-util.c:45-64 */
static void set_checksums(struct pkt *p, uint32_t ip, uint32_t l4) {
  wr16(p, ip + 10, 0);
  uint8_t proto = rd8(p, ip + 9);
  if (proto == 6) {
    wr16(p, l4 + 16, 0);
    wr16(p, l4 + 16, udptcp_cksum(p, ip, l4));
  } else if (proto == 17) {
    wr16(p, l4 + 6, 0);
    wr16(p, l4 + 6, udptcp_cksum(p, ip, l4));
  }
  wr16(p, ip + 10, ipv4_cksum(p, ip));
}
static void set_macs(struct pkt *p, uint32_t eth, const uint8_t *src,
                     const uint8_t *dst) {
  for (int i = 0; i < 6; i++) wr8(p, eth + 6 + i, src[i]);
  for (int i = 0; i < 6; i++) wr8(p, eth + i, dst[i]);
}

/* ---------------------------------------------------------------- NFs -- */
enum nf_kind { NF_NAT = 1, NF_BRIDGE = 2, NF_LB = 3, NF_FW = 4, NF_POL = 5 };

struct nat_state {
  orc_nat_cfg cfg;
  struct lv_map *fm;
  struct lv_vector *fv;
  struct lv_dchain *heap;
};
/* vigfw/dataspec.ml:5-11: fm, fv, int_devices, heap */
struct fw_state {
  orc_fw_cfg cfg;
  struct lv_map *fm;
  struct lv_vector *fv;
  struct lv_vector *int_devices;
  struct lv_dchain *heap;
};
/* vigpol/dataspec.ml:5-11: dyn_map, dyn_keys, dyn_heap, dyn_vals */
struct pol_state {
  orc_pol_cfg cfg;
  struct lv_map *dyn_map;
  struct lv_vector *dyn_keys;
  struct lv_dchain *dyn_heap;
  struct lv_vector *dyn_vals;
};
/* vigpol/dynamic_value.h:7-10 */
struct PolValue {
  uint64_t bucket_size;
  int64_t bucket_time;
};
static void PolValue_allocate(void *k) { memset(k, 0, sizeof(struct PolValue)); }
struct bridge_state {
  orc_bridge_cfg cfg;
  struct lv_map *dyn_map;
  struct lv_vector *dyn_keys;
  struct lv_vector *dyn_vals;
  struct lv_map *st_map;
  struct lv_vector *st_vec;
  struct lv_dchain *dyn_heap;
};
struct lb_state {
  orc_lb_cfg cfg;
  struct lv_map *flow_to_flow_id;
  struct lv_vector *flow_heap;
  struct lv_dchain *flow_chain;
  struct lv_vector *flow_id_to_backend_id;
  struct lv_map *ip_to_backend_id;
  struct lv_vector *backend_ips;
  struct lv_vector *backends;
  struct lv_dchain *active_backends;
  struct lv_vector *cht;
};

struct orc_nf {
  enum nf_kind kind;
  union {
    struct nat_state nat;
    struct bridge_state br;
    struct lb_state lb;
    struct fw_state fw;
    struct pol_state pol;
  } u;
};

static const uint8_t zero_mac[6];

/* ---- vignat ---- */
orc_nf *orc_nat_create(const orc_nat_cfg *cfg) {
  if (cfg->n_devices == 0 || cfg->n_devices > ORC_MAX_DEV) return NULL;
  orc_nf *nf = calloc(1, sizeof *nf);
  if (!nf) return NULL;
  nf->kind = NF_NAT;
  struct nat_state *s = &nf->u.nat;
  s->cfg = *cfg;
  /* alloc_state(max_flows, start_port, ext_ip, nat_device): vignat/
   * dataspec.ml:5-12, loop_boilerplate_gen.ml:626-710 */
  if (!lv_map_allocate(FlowId_eq, FlowId_hash, cfg->max_flows, &s->fm) ||
      !lv_vector_allocate(sizeof(struct FlowId), cfg->max_flows,
                          FlowId_allocate, &s->fv) ||
      !lv_dchain_allocate((int)cfg->max_flows, &s->heap)) {
    free(nf);
    return NULL;
  }
  return nf;
}

static int nat_process(struct nat_state *s, uint16_t device, struct pkt *p,
                       int64_t now) {
  /* nat_flowmanager.c:57-65: expiration_time (u32 us) * 1000 is computed in
   * unsigned 32-bit arithmetic and so wraps for > 4294967 us. */
  uint32_t exp_ns = s->cfg.expiration_time * 1000u;
  int64_t last_time = (int64_t)((uint64_t)now - exp_ns);
  lv_expire_items_single_map(s->heap, s->fv, s->fm, last_time);

  uint32_t eth = borrow(p, 14);
  uint32_t ip, l4;
  if (!get_ipv4(p, eth, &ip)) return device;
  if (!get_tcpudp(p, ip, &l4)) return device;

  uint16_t dst_device;
  if (device == s->cfg.wan_device) {
    /* nat_flowmanager.c:78-94 */
    int index = (int)rd16(p, l4 + 2) - (int)s->cfg.start_port;
    /* Outside [0, max_flows) the reference reads cells out of range (UB,
     * SURVEY.md §3.4); index -1 is deterministically "not allocated". We
     * define the whole range as not allocated. */
    if (index < 0 || index >= (int)s->cfg.max_flows) return device;
    if (!lv_dchain_is_index_allocated(s->heap, index)) return device;
    struct FlowId *key;
    lv_vector_borrow(s->fv, index, (void **)&key);
    struct FlowId f = *key;
    lv_vector_return(s->fv, index, key);
    lv_dchain_rejuvenate_index(s->heap, index, now);
    /* nat_main.c:55-60 anti-spoofing (non-short-circuit) */
    if ((f.dst_ip != rd32(p, ip + 12)) | (f.dst_port != rd16(p, l4)) |
        (f.protocol != rd8(p, ip + 9)))
      return device;
    wr32(p, ip + 16, f.src_ip);
    wr16(p, l4 + 2, f.src_port);
    dst_device = f.internal_device;
  } else {
    struct FlowId id = {rd16(p, l4), rd16(p, l4 + 2), rd32(p, ip + 12),
                        rd32(p, ip + 16), device, rd8(p, ip + 9)};
    uint16_t ext_port;
    int index;
    if (lv_map_get(s->fm, &id, &index)) { /* nat_flowmanager.c:67-76 */
      ext_port = (uint16_t)(index + s->cfg.start_port);
      lv_dchain_rejuvenate_index(s->heap, index, now);
    } else { /* nat_flowmanager.c:39-55 */
      if (!lv_dchain_allocate_new_index(s->heap, &index, now)) return device;
      ext_port = (uint16_t)(s->cfg.start_port + index);
      struct FlowId *key;
      lv_vector_borrow(s->fv, index, (void **)&key);
      *key = id;
      lv_map_put(s->fm, key, index);
      lv_vector_return(s->fv, index, key);
    }
    wr32(p, ip + 12, s->cfg.external_addr); /* host-order value, raw store */
    wr16(p, l4, ext_port);                  /* raw (host-order) store */
    dst_device = s->cfg.wan_device;
  }
  set_checksums(p, ip, l4);
  const uint8_t *smac = dst_device < s->cfg.n_devices
                            ? s->cfg.device_macs[dst_device] : zero_mac;
  const uint8_t *dmac = dst_device < s->cfg.n_devices
                            ? s->cfg.endpoint_macs[dst_device] : zero_mac;
  set_macs(p, eth, smac, dmac);
  return dst_device;
}

uint32_t orc_nat_flow_count(orc_nf *nf) {
  return nf->kind == NF_NAT ? lv_map_size(nf->u.nat.fm) : 0;
}

void orc_nat_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint8_t *keys) {
  struct nat_state *s = &nf->u.nat;
  int n = (int)s->cfg.max_flows;
  int *order = malloc(sizeof(int) * (size_t)n);
  int *fre = malloc(sizeof(int) * (size_t)n);
  int na, nfree;
  lv_dchain_dump(s->heap, n, order, &na, fre, &nfree, ts);
  for (int i = 0; i < n; i++) {
    alloc[i] = (uint8_t)lv_dchain_is_index_allocated(s->heap, i);
    void *k;
    lv_vector_borrow(s->fv, i, &k);
    memcpy(keys + (size_t)16 * i, k, 16);
  }
  free(order);
  free(fre);
}

/* ---- vigfw ---- */
orc_nf *orc_fw_create(const orc_fw_cfg *cfg) {
  if (cfg->n_devices == 0 || cfg->n_devices > ORC_MAX_DEV) return NULL;
  orc_nf *nf = calloc(1, sizeof *nf);
  if (!nf) return NULL;
  nf->kind = NF_FW;
  struct fw_state *s = &nf->u.fw;
  s->cfg = *cfg;
  /* alloc_state(max_flows, fw_device): vigfw/dataspec.ml:5-11,
   * loop_boilerplate_gen.ml:626-710 (containers in declaration order) */
  if (!lv_map_allocate(FwFlowId_eq, FwFlowId_hash, cfg->max_flows, &s->fm) ||
      !lv_vector_allocate(sizeof(struct FwFlowId), cfg->max_flows,
                          FwFlowId_allocate, &s->fv) ||
      !lv_vector_allocate(sizeof(uint32_t), cfg->max_flows, U32_init,
                          &s->int_devices) ||
      !lv_dchain_allocate((int)cfg->max_flows, &s->heap)) {
    free(nf);
    return NULL;
  }
  return nf;
}

/* vigfw/fw_main.c:21-80 with fw_flowmanager.c:38-86 inlined */
static int fw_process(struct fw_state *s, uint16_t device, struct pkt *p,
                      int64_t now) {
  /* fw_flowmanager.c:66-73: FlowManager.expiration_time is a vigor_time_t,
   * so the us -> ns product is 64-bit (no u32 wrap, unlike vignat). */
  int64_t last_time =
      (int64_t)((uint64_t)now - (uint64_t)((int64_t)s->cfg.expiration_time * 1000));
  lv_expire_items_single_map(s->heap, s->fv, s->fm, last_time);

  uint32_t eth = borrow(p, 14);
  uint32_t ip, l4;
  if (!get_ipv4(p, eth, &ip)) return device;
  if (!get_tcpudp(p, ip, &l4)) return device;

  uint16_t dst_device;
  if (device == s->cfg.wan_device) {
    /* reversed key for the reply flow (fw_main.c:46-53) */
    struct FwFlowId id = {rd16(p, l4 + 2), rd16(p, l4), rd32(p, ip + 16),
                          rd32(p, ip + 12), rd8(p, ip + 9)};
    int index; /* flow_manager_get_refresh_flow (fw_flowmanager.c:75-86) */
    if (!lv_map_get(s->fm, &id, &index)) return device;
    uint32_t *int_dev;
    lv_vector_borrow(s->int_devices, index, (void **)&int_dev);
    uint32_t d = *int_dev;
    lv_vector_return(s->int_devices, index, int_dev);
    lv_dchain_rejuvenate_index(s->heap, index, now);
    dst_device = (uint16_t)d;
  } else {
    struct FwFlowId id = {rd16(p, l4), rd16(p, l4 + 2), rd32(p, ip + 12),
                          rd32(p, ip + 16), rd8(p, ip + 9)};
    /* flow_manager_allocate_or_refresh_flow (fw_flowmanager.c:38-64) */
    int index;
    if (lv_map_get(s->fm, &id, &index)) {
      lv_dchain_rejuvenate_index(s->heap, index, now);
    } else if (lv_dchain_allocate_new_index(s->heap, &index, now)) {
      struct FwFlowId *key;
      lv_vector_borrow(s->fv, index, (void **)&key);
      *key = id;
      lv_map_put(s->fm, key, index);
      lv_vector_return(s->fv, index, key);
      uint32_t *int_dev;
      lv_vector_borrow(s->int_devices, index, (void **)&int_dev);
      *int_dev = device;
      lv_vector_return(s->int_devices, index, int_dev);
    } /* table full: the outgoing packet still goes out */
    dst_device = s->cfg.wan_device;
  }
  const uint8_t *smac = dst_device < s->cfg.n_devices
                            ? s->cfg.device_macs[dst_device] : zero_mac;
  const uint8_t *dmac = dst_device < s->cfg.n_devices
                            ? s->cfg.endpoint_macs[dst_device] : zero_mac;
  set_macs(p, eth, smac, dmac);
  return dst_device;
}

void orc_fw_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint8_t *keys,
                 uint32_t *int_dev) {
  struct fw_state *s = &nf->u.fw;
  int n = (int)s->cfg.max_flows;
  int *order = malloc(sizeof(int) * (size_t)n);
  int *fre = malloc(sizeof(int) * (size_t)n);
  int na, nfree;
  lv_dchain_dump(s->heap, n, order, &na, fre, &nfree, ts);
  for (int i = 0; i < n; i++) {
    alloc[i] = (uint8_t)lv_dchain_is_index_allocated(s->heap, i);
    void *k;
    lv_vector_borrow(s->fv, i, &k);
    memset(keys + (size_t)16 * i, 0, 16);
    memcpy(keys + (size_t)16 * i, k, 13);
    lv_vector_borrow(s->int_devices, i, &k);
    int_dev[i] = alloc[i] ? *(uint32_t *)k : 0;
  }
  free(order);
  free(fre);
}

/* ---- vigpol ---- */
orc_nf *orc_pol_create(const orc_pol_cfg *cfg) {
  if (cfg->n_devices == 0 || cfg->rate == 0 || cfg->burst == 0) return NULL;
  orc_nf *nf = calloc(1, sizeof *nf);
  if (!nf) return NULL;
  nf->kind = NF_POL;
  struct pol_state *s = &nf->u.pol;
  s->cfg = *cfg;
  /* alloc_state(capacity, dev_count): vigpol/dataspec.ml:5-11 */
  if (!lv_map_allocate(IpAddr_eq, IpAddr_hash, cfg->dyn_capacity, &s->dyn_map) ||
      !lv_vector_allocate(sizeof(uint32_t), cfg->dyn_capacity, U32_init,
                          &s->dyn_keys) ||
      !lv_dchain_allocate((int)cfg->dyn_capacity, &s->dyn_heap) ||
      !lv_vector_allocate(sizeof(struct PolValue), cfg->dyn_capacity,
                          PolValue_allocate, &s->dyn_vals)) {
    free(nf);
    return NULL;
  }
  return nf;
}

#define ORC_NS_PER_S 1000000000ul /* VIGOR_TIME_SECONDS_MULTIPLIER, vigor-time.h:10 */

/* policer_check_tb, vigpol/policer_main.c:34-111 (u64 arithmetic as there) */
static int pol_check_tb(struct pol_state *s, uint32_t dst, uint16_t size,
                        int64_t time) {
  int index = -1;
  if (lv_map_get(s->dyn_map, &dst, &index)) {
    lv_dchain_rejuvenate_index(s->dyn_heap, index, time);
    struct PolValue *v;
    lv_vector_borrow(s->dyn_vals, index, (void **)&v);
    uint64_t time_u = (uint64_t)time;
    uint64_t time_diff = time_u - (uint64_t)v->bucket_time;
    if (time_diff < s->cfg.burst * ORC_NS_PER_S / s->cfg.rate) {
      uint64_t added = time_diff * s->cfg.rate / ORC_NS_PER_S;
      v->bucket_size += added;
      if (v->bucket_size > s->cfg.burst) v->bucket_size = s->cfg.burst;
    } else {
      v->bucket_size = s->cfg.burst;
    }
    v->bucket_time = (int64_t)time_u;
    int fwd = 0;
    if (v->bucket_size > size) {
      v->bucket_size -= size;
      fwd = 1;
    }
    lv_vector_return(s->dyn_vals, index, v);
    return fwd;
  }
  if (size > s->cfg.burst) return 0; /* unknown flow larger than burst */
  if (!lv_dchain_allocate_new_index(s->dyn_heap, &index, time)) return 0;
  uint32_t *key;
  struct PolValue *v;
  lv_vector_borrow(s->dyn_keys, index, (void **)&key);
  lv_vector_borrow(s->dyn_vals, index, (void **)&v);
  *key = dst;
  v->bucket_size = s->cfg.burst - size;
  v->bucket_time = time;
  lv_map_put(s->dyn_map, key, index);
  lv_vector_return(s->dyn_keys, index, key);
  lv_vector_return(s->dyn_vals, index, v);
  return 1;
}

/* nf_process, vigpol/policer_main.c:120-145; expiry (policer_expire_entries,
 * :21-32) only after the IPv4 header parsed. */
static int pol_process(struct pol_state *s, uint16_t device, struct pkt *p,
                       uint16_t len, int64_t now) {
  uint32_t eth = borrow(p, 14);
  uint32_t ip;
  if (!get_ipv4(p, eth, &ip)) return device;
  uint64_t exp_time = ORC_NS_PER_S * s->cfg.burst / s->cfg.rate;
  int64_t min_time = (int64_t)((uint64_t)now - exp_time);
  lv_expire_items_single_map(s->dyn_heap, s->dyn_keys, s->dyn_map, min_time);
  if (device == s->cfg.lan_device) return s->cfg.wan_device;
  if (device == s->cfg.wan_device)
    return pol_check_tb(s, rd32(p, ip + 16), len, now) ? s->cfg.lan_device
                                                         : s->cfg.wan_device;
  return device;
}

void orc_pol_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint32_t *keys,
                  uint64_t *bucket_size, int64_t *bucket_time) {
  struct pol_state *s = &nf->u.pol;
  int n = (int)s->cfg.dyn_capacity;
  int *order = malloc(sizeof(int) * (size_t)n);
  int *fre = malloc(sizeof(int) * (size_t)n);
  int na, nfree;
  lv_dchain_dump(s->dyn_heap, n, order, &na, fre, &nfree, ts);
  for (int i = 0; i < n; i++) {
    alloc[i] = (uint8_t)lv_dchain_is_index_allocated(s->dyn_heap, i);
    void *k;
    lv_vector_borrow(s->dyn_keys, i, &k);
    keys[i] = *(uint32_t *)k;
    lv_vector_return(s->dyn_keys, i, k);
    lv_vector_borrow(s->dyn_vals, i, &k);
    bucket_size[i] = ((struct PolValue *)k)->bucket_size;
    bucket_time[i] = ((struct PolValue *)k)->bucket_time;
    lv_vector_return(s->dyn_vals, i, k);
  }
  free(order);
  free(fre);
}

/* Dynamic table by index: dchain allocated?, ts, dyn_keys[i], dyn_vals[i]. */
void orc_bridge_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint8_t *macs,
                     uint16_t *port) {
  struct bridge_state *s = &nf->u.br;
  int n = (int)s->cfg.dyn_capacity;
  int *order = malloc(sizeof(int) * (size_t)n);
  int *fre = malloc(sizeof(int) * (size_t)n);
  int na, nfree;
  lv_dchain_dump(s->dyn_heap, n, order, &na, fre, &nfree, ts);
  for (int i = 0; i < n; i++) {
    alloc[i] = (uint8_t)lv_dchain_is_index_allocated(s->dyn_heap, i);
    void *k;
    lv_vector_borrow(s->dyn_keys, i, &k);
    memcpy(macs + (size_t)6 * i, k, 6);
    lv_vector_return(s->dyn_keys, i, k);
    lv_vector_borrow(s->dyn_vals, i, &k);
    port[i] = ((struct DynamicValue *)k)->device;
    lv_vector_return(s->dyn_vals, i, k);
  }
  free(order);
  free(fre);
}

/* viglb state by index. Flows i < flow_capacity: allocated?, ts, LbFlow
 * bytes (16, padding zero), flow_id_to_backend_id. Backends b <
 * backend_capacity: allocated?, ts, backends[b] as {ip, mac, nic}. */
void orc_lb_dump(orc_nf *nf, uint8_t *f_alloc, int64_t *f_ts, uint8_t *f_keys,
                 uint32_t *f_backend, uint8_t *b_alloc, int64_t *b_ts,
                 uint32_t *b_ip, uint8_t *b_mac, uint16_t *b_nic) {
  struct lb_state *s = &nf->u.lb;
  int nf_ = (int)s->cfg.flow_capacity, nb = (int)s->cfg.backend_capacity;
  int n = nf_ > nb ? nf_ : nb;
  int *order = malloc(sizeof(int) * (size_t)n);
  int *fre = malloc(sizeof(int) * (size_t)n);
  int na, nfree;
  lv_dchain_dump(s->flow_chain, nf_, order, &na, fre, &nfree, f_ts);
  for (int i = 0; i < nf_; i++) {
    f_alloc[i] = (uint8_t)lv_dchain_is_index_allocated(s->flow_chain, i);
    void *k;
    lv_vector_borrow(s->flow_heap, i, &k);
    struct LbFlow *fl = k;
    uint8_t *o = f_keys + (size_t)16 * i;
    memset(o, 0, 16);
    memcpy(o, &fl->src_ip, 4);
    memcpy(o + 4, &fl->dst_ip, 4);
    memcpy(o + 8, &fl->src_port, 2);
    memcpy(o + 10, &fl->dst_port, 2);
    o[12] = fl->protocol;
    lv_vector_return(s->flow_heap, i, k);
    lv_vector_borrow(s->flow_id_to_backend_id, i, &k);
    f_backend[i] = *(uint32_t *)k;
    lv_vector_return(s->flow_id_to_backend_id, i, k);
  }
  lv_dchain_dump(s->active_backends, nb, order, &na, fre, &nfree, b_ts);
  for (int i = 0; i < nb; i++) {
    b_alloc[i] = (uint8_t)lv_dchain_is_index_allocated(s->active_backends, i);
    void *k;
    lv_vector_borrow(s->backends, i, &k);
    struct LbBackend *b = k;
    b_ip[i] = b->ip;
    memcpy(b_mac + (size_t)6 * i, b->mac.b, 6);
    b_nic[i] = b->nic;
    lv_vector_return(s->backends, i, k);
  }
  free(order);
  free(fre);
}

/* ---- vigbridge ---- */
orc_nf *orc_bridge_create(const orc_bridge_cfg *cfg) {
  orc_nf *nf = calloc(1, sizeof *nf);
  if (!nf) return NULL;
  nf->kind = NF_BRIDGE;
  struct bridge_state *s = &nf->u.br;
  s->cfg = *cfg;
  const unsigned stat_capacity = 8192; /* bridge_main.c:293 */
  /* alloc_state(capacity, stat_capacity, dev_count): dataspec.ml:5-15 */
  if (!lv_map_allocate(Eth_eq, Eth_hash, cfg->dyn_capacity, &s->dyn_map) ||
      !lv_vector_allocate(sizeof(struct EthAddr), cfg->dyn_capacity,
                          Eth_allocate, &s->dyn_keys) ||
      !lv_vector_allocate(sizeof(struct DynamicValue), cfg->dyn_capacity,
                          DynamicValue_allocate, &s->dyn_vals) ||
      !lv_map_allocate(StaticKey_eq, StaticKey_hash, stat_capacity,
                       &s->st_map) ||
      !lv_vector_allocate(sizeof(struct StaticKey), stat_capacity,
                          StaticKey_allocate, &s->st_vec) ||
      !lv_dchain_allocate((int)cfg->dyn_capacity, &s->dyn_heap)) {
    free(nf);
    return NULL;
  }
  /* read_static_ft_from_file (bridge_main.c:130-230): rule k goes to st_vec
   * slot k, keyed {mac, device_from}, value device_to. */
  if (cfg->n_static * 2 >= stat_capacity) {
    free(nf);
    return NULL;
  }
  for (uint32_t k = 0; k < cfg->n_static; k++) {
    struct StaticKey *key;
    lv_vector_borrow(s->st_vec, (int)k, (void **)&key);
    memcpy(key->addr.b, cfg->static_macs + 6 * k, 6);
    key->device = (uint16_t)cfg->static_from[k];
    lv_map_put(s->st_map, key, cfg->static_to[k]);
    lv_vector_return(s->st_vec, (int)k, key);
  }
  s->cfg.static_macs = NULL;
  s->cfg.static_from = s->cfg.static_to = NULL;
  return nf;
}

static int bridge_process(struct bridge_state *s, uint16_t device,
                          struct pkt *p, int64_t now) {
  uint32_t eth = borrow(p, 14); /* no length check (bridge_main.c:312) */
  struct EthAddr dst, src;
  for (int i = 0; i < 6; i++) dst.b[i] = rd8(p, eth + i);
  for (int i = 0; i < 6; i++) src.b[i] = rd8(p, eth + 6 + i);

  /* bridge_expire_entries (bridge_main.c:69-76): u32 wrap as in vignat */
  uint32_t exp_ns = s->cfg.expiration_time * 1000u;
  int64_t last_time = (int64_t)((uint64_t)now - exp_ns);
  lv_expire_items_single_map(s->dyn_heap, s->dyn_keys, s->dyn_map, last_time);

  /* bridge_put_update_entry (103-128): a known MAC is only rejuvenated */
  int index = -1;
  if (lv_map_get(s->dyn_map, &src, &index)) {
    lv_dchain_rejuvenate_index(s->dyn_heap, index, now);
  } else if (lv_dchain_allocate_new_index(s->dyn_heap, &index, now)) {
    struct EthAddr *key;
    struct DynamicValue *val;
    lv_vector_borrow(s->dyn_keys, index, (void **)&key);
    lv_vector_borrow(s->dyn_vals, index, (void **)&val);
    *key = src;
    val->device = device;
    lv_map_put(s->dyn_map, key, index);
    lv_vector_return(s->dyn_keys, index, key);
    lv_vector_return(s->dyn_vals, index, val);
  }

  /* bridge_get_device (78-101) */
  int fwd = -1;
  struct StaticKey k;
  memset(&k, 0, sizeof k);
  k.addr = dst;
  k.device = device;
  int v;
  if (lv_map_get(s->st_map, &k, &v)) {
    fwd = v;
  } else if (lv_map_get(s->dyn_map, &dst, &index)) {
    struct DynamicValue *val;
    lv_vector_borrow(s->dyn_vals, index, (void **)&val);
    fwd = val->device;
    lv_vector_return(s->dyn_vals, index, val);
  }
  if (fwd == -1) return ORC_FLOOD;
  if (fwd == -2) return device;
  return fwd;
}

/* ---- viglb ---- */
orc_nf *orc_lb_create(const orc_lb_cfg *cfg) {
  if (cfg->n_devices == 0 || cfg->n_devices > ORC_MAX_DEV) return NULL;
  orc_nf *nf = calloc(1, sizeof *nf);
  if (!nf) return NULL;
  nf->kind = NF_LB;
  struct lb_state *s = &nf->u.lb;
  s->cfg = *cfg;
  /* alloc_state(backend_capacity, flow_capacity, cht_height):
   * viglb/dataspec.ml:5-25 container order */
  uint32_t fc = cfg->flow_capacity, bc = cfg->backend_capacity;
  if (!lv_map_allocate(LbFlow_eq, LbFlow_hash, fc, &s->flow_to_flow_id) ||
      !lv_vector_allocate(sizeof(struct LbFlow), fc, LbFlow_allocate,
                          &s->flow_heap) ||
      !lv_dchain_allocate((int)fc, &s->flow_chain) ||
      !lv_vector_allocate(sizeof(uint32_t), fc, U32_init,
                          &s->flow_id_to_backend_id) ||
      !lv_map_allocate(IpAddr_eq, IpAddr_hash, bc, &s->ip_to_backend_id) ||
      !lv_vector_allocate(sizeof(uint32_t), bc, U32_init, &s->backend_ips) ||
      !lv_vector_allocate(sizeof(struct LbBackend), bc, LbBackend_allocate,
                          &s->backends) ||
      !lv_dchain_allocate((int)bc, &s->active_backends) ||
      !lv_vector_allocate(sizeof(uint32_t), bc * cfg->cht_height, U32_init,
                          &s->cht) ||
      !lv_cht_fill_cht(s->cht, cfg->cht_height, bc)) {
    free(nf);
    return NULL;
  }
  return nf;
}

/* lb_balancer.c:106-181 */
static struct LbBackend lb_get_backend(struct lb_state *s, struct LbFlow *flow,
                                       int64_t now) {
  struct LbBackend backend;
  memset(&backend, 0, sizeof backend);
  int flow_index;
  if (!lv_map_get(s->flow_to_flow_id, flow, &flow_index)) {
    int backend_index = 0;
    int found = lv_cht_find_preferred_available_backend(
        (uint64_t)LbFlow_hash(flow), s->cht, s->active_backends,
        s->cfg.cht_height, s->cfg.backend_capacity, &backend_index);
    if (found) {
      if (lv_dchain_allocate_new_index(s->flow_chain, &flow_index, now)) {
        struct LbFlow *vf;
        uint32_t *vb;
        lv_vector_borrow(s->flow_heap, flow_index, (void **)&vf);
        *vf = *flow;
        lv_vector_borrow(s->flow_id_to_backend_id, flow_index, (void **)&vb);
        *vb = (uint32_t)backend_index;
        lv_vector_return(s->flow_id_to_backend_id, flow_index, vb);
        lv_map_put(s->flow_to_flow_id, vf, flow_index);
        lv_vector_return(s->flow_heap, flow_index, vf);
      }
      struct LbBackend *vb;
      lv_vector_borrow(s->backends, backend_index, (void **)&vb);
      backend = *vb;
      lv_vector_return(s->backends, backend_index, vb);
    } else {
      backend.nic = s->cfg.wan_device; /* drop */
    }
  } else {
    uint32_t *vbi;
    lv_vector_borrow(s->flow_id_to_backend_id, flow_index, (void **)&vbi);
    uint32_t backend_index = *vbi;
    lv_vector_return(s->flow_id_to_backend_id, flow_index, vbi);
    if (!lv_dchain_is_index_allocated(s->active_backends, (int)backend_index)) {
      void *trash;
      struct LbFlow *fk;
      lv_vector_borrow(s->flow_heap, flow_index, (void **)&fk);
      lv_map_erase(s->flow_to_flow_id, flow, &trash);
      lv_dchain_free_index(s->flow_chain, flow_index);
      lv_vector_return(s->flow_heap, flow_index, fk);
      return lb_get_backend(s, flow, now);
    }
    lv_dchain_rejuvenate_index(s->flow_chain, flow_index, now);
    struct LbBackend *vb;
    lv_vector_borrow(s->backends, (int)backend_index, (void **)&vb);
    backend = *vb;
    lv_vector_return(s->backends, (int)backend_index, vb);
  }
  return backend;
}

/* lb_balancer.c:183-215 */
static void lb_heartbeat(struct lb_state *s, struct LbFlow *flow,
                         const struct EthAddr *mac, int nic, int64_t now) {
  int backend_index;
  if (!lv_map_get(s->ip_to_backend_id, &flow->src_ip, &backend_index)) {
    if (lv_dchain_allocate_new_index(s->active_backends, &backend_index,
                                     now)) {
      struct LbBackend *nb;
      lv_vector_borrow(s->backends, backend_index, (void **)&nb);
      nb->ip = flow->src_ip;
      nb->mac = *mac;
      nb->nic = (uint16_t)nic;
      lv_vector_return(s->backends, backend_index, nb);
      uint32_t *ipp;
      lv_vector_borrow(s->backend_ips, backend_index, (void **)&ipp);
      *ipp = flow->src_ip;
      lv_map_put(s->ip_to_backend_id, ipp, backend_index);
      lv_vector_return(s->backend_ips, backend_index, ipp);
    }
  } else {
    lv_dchain_rejuvenate_index(s->active_backends, backend_index, now);
  }
}

static int lb_process(struct lb_state *s, uint16_t device, struct pkt *p,
                      int64_t now) {
  /* lb_expire_flows / lb_expire_backends (lb_balancer.c:217-237): the
   * expiration times are int64 here (lb_main.c:14-18 passes the u32 config
   * into vigor_time_t parameters), so x1000 does not wrap. */
  int64_t fexp = (int64_t)s->cfg.flow_expiration_time;
  int64_t bexp = (int64_t)s->cfg.backend_expiration_time;
  lv_expire_items_single_map(s->flow_chain, s->flow_heap, s->flow_to_flow_id,
                             (int64_t)((uint64_t)now - (uint64_t)(fexp * 1000)));
  lv_expire_items_single_map(s->active_backends, s->backend_ips,
                             s->ip_to_backend_id,
                             (int64_t)((uint64_t)now - (uint64_t)(bexp * 1000)));

  uint32_t eth = borrow(p, 14);
  uint32_t ip, l4;
  if (!get_ipv4(p, eth, &ip)) return device;
  if (!get_tcpudp(p, ip, &l4)) return device;

  struct LbFlow flow;
  memset(&flow, 0, sizeof flow);
  flow.src_ip = rd32(p, ip + 12);
  flow.dst_ip = rd32(p, ip + 16);
  flow.src_port = rd16(p, l4);
  flow.dst_port = rd16(p, l4 + 2);
  flow.protocol = rd8(p, ip + 9);

  if (device != s->cfg.wan_device) {
    struct EthAddr smac;
    for (int i = 0; i < 6; i++) smac.b[i] = rd8(p, eth + 6 + i);
    lb_heartbeat(s, &flow, &smac, device, now);
    return device;
  }
  struct LbBackend b = lb_get_backend(s, &flow, now);
  if (b.nic != s->cfg.wan_device) {
    wr32(p, ip + 16, b.ip);
    const uint8_t *smac =
        b.nic < s->cfg.n_devices ? s->cfg.device_macs[b.nic] : zero_mac;
    for (int i = 0; i < 6; i++) wr8(p, eth + 6 + i, smac[i]);
    for (int i = 0; i < 6; i++) wr8(p, eth + i, b.mac.b[i]);
    set_checksums(p, ip, l4);
  }
  return b.nic;
}

/* ------------------------------------------------------------- driver -- */
void orc_destroy(orc_nf *nf) {
  if (!nf) return;
  switch (nf->kind) {
    case NF_NAT:
      lv_map_free(nf->u.nat.fm);
      lv_vector_free(nf->u.nat.fv);
      lv_dchain_free(nf->u.nat.heap);
      break;
    case NF_BRIDGE:
      lv_map_free(nf->u.br.dyn_map);
      lv_vector_free(nf->u.br.dyn_keys);
      lv_vector_free(nf->u.br.dyn_vals);
      lv_map_free(nf->u.br.st_map);
      lv_vector_free(nf->u.br.st_vec);
      lv_dchain_free(nf->u.br.dyn_heap);
      break;
    case NF_LB:
      lv_map_free(nf->u.lb.flow_to_flow_id);
      lv_vector_free(nf->u.lb.flow_heap);
      lv_dchain_free(nf->u.lb.flow_chain);
      lv_vector_free(nf->u.lb.flow_id_to_backend_id);
      lv_map_free(nf->u.lb.ip_to_backend_id);
      lv_vector_free(nf->u.lb.backend_ips);
      lv_vector_free(nf->u.lb.backends);
      lv_dchain_free(nf->u.lb.active_backends);
      lv_vector_free(nf->u.lb.cht);
      break;
    case NF_FW:
      lv_map_free(nf->u.fw.fm);
      lv_vector_free(nf->u.fw.fv);
      lv_vector_free(nf->u.fw.int_devices);
      lv_dchain_free(nf->u.fw.heap);
      break;
    case NF_POL:
      lv_map_free(nf->u.pol.dyn_map);
      lv_vector_free(nf->u.pol.dyn_keys);
      lv_dchain_free(nf->u.pol.dyn_heap);
      lv_vector_free(nf->u.pol.dyn_vals);
      break;
  }
  free(nf);
}

int orc_process(orc_nf *nf, uint16_t device, uint8_t *frame, uint16_t len,
                uint32_t cap, int64_t now) {
  struct pkt p = {frame, cap, len, 0}; /* packet_state_total_length */
  switch (nf->kind) {
    case NF_NAT:
      return nat_process(&nf->u.nat, device, &p, now);
    case NF_BRIDGE:
      return bridge_process(&nf->u.br, device, &p, now);
    case NF_LB:
      return lb_process(&nf->u.lb, device, &p, now);
    case NF_FW:
      return fw_process(&nf->u.fw, device, &p, now);
    case NF_POL:
      return pol_process(&nf->u.pol, device, &p, len, now);
  }
  return device;
}

void orc_run(orc_nf *nf, uint32_t n, const uint16_t *in_dev, uint8_t *frames,
             uint32_t slot, const uint16_t *len, const int64_t *now,
             uint16_t *out_dev) {
  for (uint32_t i = 0; i < n; i++)
    out_dev[i] = (uint16_t)orc_process(nf, in_dev[i],
                                       frames + (size_t)slot * i, len[i], slot,
                                       now[i]);
}

uint64_t orc_digest(uint32_t n, const uint8_t *frames, uint32_t slot,
                    const uint16_t *len, const uint16_t *out_dev) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t o[2] = {(uint8_t)out_dev[i], (uint8_t)(out_dev[i] >> 8)};
    for (int k = 0; k < 2; k++) h = (h ^ o[k]) * 0x100000001b3ull;
    const uint8_t *f = frames + (size_t)slot * i;
    uint32_t l = len[i] < slot ? len[i] : slot;
    for (uint32_t k = 0; k < l; k++) h = (h ^ f[k]) * 0x100000001b3ull;
  }
  return h;
}

/* ----------------------------------------------- libVig op-stream tests --
 * Drive the lv_* layer directly with a scripted stream so the restated and
 * the reference libVig can be compared call by call. */
enum { OP_ALLOC = 0, OP_REJUV, OP_EXPIRE, OP_FREE, OP_ISALLOC };
/* ops: n x {op, arg, time}; res: one int per op (return value, index for
 * alloc, expired count for expire). Final dchain dump appended by caller. */
int orc_test_dchain(int range, uint32_t n, const int32_t *op, const int32_t *arg,
                    const int64_t *t, int32_t *res, int32_t *alloc_order,
                    int32_t *n_alloc, int32_t *free_order, int32_t *n_free,
                    int64_t *ts) {
  struct lv_dchain *c;
  if (!lv_dchain_allocate(range, &c)) return 0;
  for (uint32_t i = 0; i < n; i++) {
    int idx = -1;
    switch (op[i]) {
      case OP_ALLOC:
        res[i] = lv_dchain_allocate_new_index(c, &idx, t[i]) ? idx : -1;
        break;
      case OP_REJUV:
        res[i] = lv_dchain_rejuvenate_index(c, arg[i], t[i]);
        break;
      case OP_EXPIRE: {
        int k = 0;
        while (lv_dchain_expire_one_index(c, &idx, t[i])) k++;
        res[i] = k;
        break;
      }
      case OP_FREE:
        res[i] = lv_dchain_free_index(c, arg[i]);
        break;
      case OP_ISALLOC:
        res[i] = lv_dchain_is_index_allocated(c, arg[i]);
        break;
      default:
        res[i] = -99;
    }
  }
  lv_dchain_dump(c, range, alloc_order, n_alloc, free_order, n_free, ts);
  lv_dchain_free(c);
  return 1;
}

/* Map over u32 keys kept in a key vector indexed like the NFs do; the hash is
 * a deliberately weak (key % hmod) so probe chains collide. ops: 0 put(key,
 * slot) / 1 get(key) / 2 erase(key at slot). res: get -> value or -1. */
static uint32_t test_hmod = 7;
static unsigned weak_hash(void *k) { return *(uint32_t *)k % test_hmod; }
static bool u32_eq(void *a, void *b) {
  return *(uint32_t *)a == *(uint32_t *)b;
}
int orc_test_map(unsigned cap, uint32_t hmod, uint32_t n, const int32_t *op,
                 const uint32_t *key, const int32_t *val, int32_t *res) {
  struct lv_map *m;
  struct lv_vector *keys;
  test_hmod = hmod ? hmod : 1;
  if (!lv_map_allocate(u32_eq, weak_hash, cap, &m)) return 0;
  if (!lv_vector_allocate(sizeof(uint32_t), cap, U32_init, &keys)) return 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t k = key[i];
    int v = -1;
    switch (op[i]) {
      case 0: {
        void *slot;
        lv_vector_borrow(keys, val[i], &slot);
        *(uint32_t *)slot = k;
        lv_map_put(m, slot, val[i]);
        res[i] = (int)lv_map_size(m);
        break;
      }
      case 1:
        res[i] = lv_map_get(m, &k, &v) ? v : -1;
        break;
      case 2: {
        void *slot, *trash;
        lv_vector_borrow(keys, val[i], &slot);
        lv_map_erase(m, slot, &trash);
        res[i] = (int)lv_map_size(m);
        break;
      }
      default:
        res[i] = -99;
    }
  }
  lv_map_free(m);
  lv_vector_free(keys);
  return 1;
}

/* CHT fill + lookups: table_out gets height*cap entries; for each hash in
 * hashes[], chosen[] gets the backend or -1, with backends in `active_mask`
 * allocated (in index order) in a dchain of range cap. */
int orc_test_cht(uint32_t height, uint32_t cap, uint32_t *table_out,
                 const uint8_t *active_mask, uint32_t nh, const uint64_t *hashes,
                 int32_t *chosen) {
  struct lv_vector *cht;
  struct lv_dchain *act;
  if (!lv_vector_allocate(sizeof(uint32_t), height * cap, U32_init, &cht))
    return 0;
  if (!lv_cht_fill_cht(cht, height, cap)) return 0;
  if (!lv_dchain_allocate((int)cap, &act)) return 0;
  for (uint32_t i = 0; i < height * cap; i++) {
    void *e;
    lv_vector_borrow(cht, (int)i, &e);
    table_out[i] = *(uint32_t *)e;
  }
  /* allocate all, then free the inactive ones */
  for (uint32_t b = 0; b < cap; b++) {
    int idx;
    lv_dchain_allocate_new_index(act, &idx, 0);
  }
  for (uint32_t b = 0; b < cap; b++)
    if (!active_mask[b]) lv_dchain_free_index(act, (int)b);
  for (uint32_t i = 0; i < nh; i++) {
    int c = -1;
    chosen[i] = lv_cht_find_preferred_available_backend(hashes[i], cht, act,
                                                        height, cap, &c)
                    ? c : -1;
  }
  lv_vector_free(cht);
  lv_dchain_free(act);
  return 1;
}
