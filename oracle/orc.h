/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Vigor's per-packet path (nf.c dispatch -> nf_process of
 * vignat / vigbridge / viglb / vigfw / vigpol -> nf-util parse + DPDK 20.08 checksum -> libVig).
 * Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() may
 * load it, and only as the checker (or the timed CPU baseline). The product
 * path (vigor_amd/, include/vigpath.h) never links, loads or calls it.
 *
 * Parity status: the libVig layer is pinned against the reference's own
 * sources (oracle/_ref, tests/test_oracle_ref.py); the CRC32C hash is pinned
 * by the reference's hardware builtin (same) and SURVEY.md's KAT; the
 * end-to-end vignat bytes by SURVEY.md Appendix A's probe KATs. The DPDK
 * 20.08 checksum edges (IHL>5, TCP checksum 0) are "parity unpinned": DPDK is
 * not vendored (setup.sh:94) and no reference test covers checksums
 * (nf-util.c:34-43).
 *
 * Frame buffer convention (both here and in the HIP path): a packet is a slot
 * of `cap` bytes holding `len` valid bytes. The reference reads/writes mbuf
 * memory beyond pkt_len in some malformed-header cases; we read slot bytes
 * there, and treat bytes past the slot as 0 (reads) / discard them (writes).
 */
#ifndef ORC_H
#define ORC_H
#include <stdint.h>

#define ORC_MAX_DEV 32
#define ORC_FLOOD 0xFFFFu

typedef struct orc_nf orc_nf;

/* vignat/nat_config.h:5-31 */
typedef struct {
  uint16_t wan_device;
  uint16_t start_port;
  uint32_t external_addr;   /* host-order value as nf_parse_ipv4addr builds */
  uint32_t expiration_time; /* microseconds (u32; x1000 wraps in u32) */
  uint32_t max_flows;       /* must be a power of two (map.c:73) */
  uint16_t n_devices;
  uint8_t device_macs[ORC_MAX_DEV][6];
  uint8_t endpoint_macs[ORC_MAX_DEV][6];
} orc_nat_cfg;

/* vigbridge/bridge_config.h:8-18; static rules as bridge_main.c:130-230 reads
 * them from the --config file: (mac, device_from, device_to). */
typedef struct {
  uint32_t expiration_time; /* microseconds */
  uint32_t dyn_capacity;    /* power of two */
  uint16_t n_devices;
  uint32_t n_static;
  const uint8_t *static_macs;     /* n_static * 6 */
  const int32_t *static_from;     /* n_static */
  const int32_t *static_to;       /* n_static */
} orc_bridge_cfg;

/* viglb/lb_config.h:8-38 */
typedef struct {
  uint32_t flow_capacity;       /* power of two */
  uint32_t flow_expiration_time;    /* microseconds */
  uint32_t backend_capacity;    /* power of two */
  uint32_t cht_height;          /* prime, > backend_capacity */
  uint32_t backend_expiration_time; /* microseconds */
  uint16_t wan_device;
  uint16_t n_devices;
  uint8_t device_macs[ORC_MAX_DEV][6];
} orc_lb_cfg;

/* vigfw/fw_config.h:9-24 */
typedef struct {
  uint16_t wan_device;
  uint32_t expiration_time; /* microseconds (x1000 in 64 bits) */
  uint32_t max_flows;       /* power of two */
  uint16_t n_devices;
  uint8_t device_macs[ORC_MAX_DEV][6];
  uint8_t endpoint_macs[ORC_MAX_DEV][6];
} orc_fw_cfg;

/* vigpol/policer_config.h:8-24 */
typedef struct {
  uint16_t lan_device;
  uint16_t wan_device;
  uint64_t rate;         /* B/s */
  uint64_t burst;        /* B */
  uint32_t dyn_capacity; /* power of two (map.c:73) */
  uint16_t n_devices;
} orc_pol_cfg;

orc_nf *orc_nat_create(const orc_nat_cfg *cfg);
orc_nf *orc_pol_create(const orc_pol_cfg *cfg);
orc_nf *orc_fw_create(const orc_fw_cfg *cfg);
orc_nf *orc_bridge_create(const orc_bridge_cfg *cfg);
orc_nf *orc_lb_create(const orc_lb_cfg *cfg);
void orc_destroy(orc_nf *nf);

/* One nf_process call (nf.h:13) on a frame buffer of `cap` bytes. */
int orc_process(orc_nf *nf, uint16_t device, uint8_t *frame, uint16_t len,
                uint32_t cap, int64_t now);

/* nf.c:150-176 over a trace: frames are `slot` bytes apart, mutated in place;
 * out_dev[i] = (uint16_t)nf_process(...) (the caller stores it in a u16,
 * nf.c:156): == in_dev -> dropped, 0xFFFF -> flooded, else transmitted. */
void orc_run(orc_nf *nf, uint32_t n, const uint16_t *in_dev, uint8_t *frames,
             uint32_t slot, const uint16_t *len, const int64_t *now,
             uint16_t *out_dev);

/* FNV-1a-64 over out_port (2 B LE) || frame[0:len] for every packet. */
uint64_t orc_digest(uint32_t n, const uint8_t *frames, uint32_t slot,
                    const uint16_t *len, const uint16_t *out_dev);

/* Known-answer helpers. */
uint32_t orc_crc32c_u32(uint32_t crc, uint32_t v);
uint32_t orc_flowid_hash(uint16_t sp, uint16_t dp, uint32_t sip, uint32_t dip,
                         uint16_t dev, uint8_t proto);
uint32_t orc_ether_hash(const uint8_t mac[6]);
uint32_t orc_fw_flowid_hash(uint16_t sp, uint16_t dp, uint32_t sip, uint32_t dip,
                            uint8_t proto);
const char *orc_impl_name(void);

/* Observable state for parity of state (not just outputs). */
uint32_t orc_nat_flow_count(orc_nf *nf);
/* Writes, for index i < max_flows: alloc[i] = allocated?, ts[i] timestamp,
 * key[i] = the 16-byte FlowId stored at that index. */
void orc_nat_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint8_t *keys);
/* vigfw: alloc, ts, FlowId bytes (13 + zero padding), int_devices. */
void orc_fw_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint8_t *keys,
                 uint32_t *int_dev);
/* vigpol: alloc, ts, dyn_keys (u32 dst address, raw), dyn_vals
 * (DynamicValue {bucket_size, bucket_time}, vigpol/dynamic_value.h:7-10). */
void orc_pol_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint32_t *keys,
                  uint64_t *bucket_size, int64_t *bucket_time);
void orc_bridge_dump(orc_nf *nf, uint8_t *alloc, int64_t *ts, uint8_t *macs,
                     uint16_t *port);
void orc_lb_dump(orc_nf *nf, uint8_t *f_alloc, int64_t *f_ts, uint8_t *f_keys,
                 uint32_t *f_backend, uint8_t *b_alloc, int64_t *b_ts,
                 uint32_t *b_ip, uint8_t *b_mac, uint16_t *b_nic);

#endif
