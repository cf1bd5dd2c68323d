/*
 * Shared pieces of the nf.h drop-in shims (vp_nf_<nf>.c -> lib<nf>_nf.so):
 * the DPDK device queries, nf-util's option parsers and the single context
 * nf_init creates. Each shim includes this once; nothing here is exported
 * except vp_nf_context.
 *
 * Device count and MACs come from DPDK's rte_eth_dev_count_avail /
 * rte_eth_macaddr_get when the host process links DPDK (weak references);
 * otherwise from VIGPATH_NB_DEVICES (default 2) and 02:00:00:00:00:<dev>.
 * VIGPATH_GPU selects the HIP device (default 0).
 */
#ifndef VP_NF_COMMON_H
#define VP_NF_COMMON_H

#include <errno.h>
#include <getopt.h>
#include <inttypes.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/vigpath.h"

/* not every shim uses every helper */
#pragma GCC diagnostic ignored "-Wunused-function"

typedef int64_t vigor_time_t; /* libvig/verified/vigor-time.h:7 */

struct rte_ether_addr {
  uint8_t addr_bytes[6];
};

/* DPDK 20.08 (setup.sh:94): present only when the host links DPDK */
extern uint16_t rte_eth_dev_count_avail(void) __attribute__((weak));
extern void rte_eth_macaddr_get(uint16_t port_id, struct rte_ether_addr *mac)
    __attribute__((weak));

void nf_config_usage(void);

static vp_ctx *g_ctx;

/* The context nf_init created, for callers that batch (vp_process_batch). */
vp_ctx *vp_nf_context(void) { return g_ctx; }

static uint16_t nb_devices(void) {
  if (rte_eth_dev_count_avail) return rte_eth_dev_count_avail();
  const char *e = getenv("VIGPATH_NB_DEVICES");
  int n = e ? atoi(e) : 2;
  return (uint16_t)(n > 0 && n <= VP_MAX_DEVICES ? n : 2);
}

static void device_mac(uint16_t d, struct rte_ether_addr *m) {
  if (rte_eth_macaddr_get) {
    rte_eth_macaddr_get(d, m);
    return;
  }
  static const uint8_t base[6] = {0x02, 0, 0, 0, 0, 0};
  memcpy(m->addr_bytes, base, 6);
  m->addr_bytes[5] = (uint8_t)d;
}

static int shim_gpu(void) {
  const char *g = getenv("VIGPATH_GPU");
  return g ? atoi(g) : 0;
}

#define PARSE_ERROR(...)          \
  do {                            \
    nf_config_usage();            \
    fprintf(stderr, __VA_ARGS__); \
    exit(EXIT_FAILURE);           \
  } while (0)

/* nf_util_parse_int (nf-util.c:67-78) */
static intmax_t parse_int(const char *str, const char *name, char next) {
  char *end;
  intmax_t r = strtoimax(str, &end, 10);
  if (end == str || *end != next) {
    fprintf(stderr, "Error while parsing '%s': %s\n", name, str);
    exit(EXIT_FAILURE);
  }
  return r;
}

/* nf_parse_etheraddr (nf-parse.h:9-19) */
static bool parse_mac(const char *s, struct rte_ether_addr *a) {
  return sscanf(s, "%02hhX:%02hhX:%02hhX:%02hhX:%02hhX:%02hhX",
                a->addr_bytes + 0, a->addr_bytes + 1, a->addr_bytes + 2,
                a->addr_bytes + 3, a->addr_bytes + 4, a->addr_bytes + 5) == 6;
}

static void print_mac(const uint8_t *m) {
  printf("%02X:%02X:%02X:%02X:%02X:%02X", m[0], m[1], m[2], m[3], m[4], m[5]);
}

/* One packet through the C-ABI (vp_process_one). The reference has no error
 * path; a device failure here aborts like nf.c's tx failure does
 * (nf.c:167-172). */
static int shim_process_one(uint16_t device, uint8_t *buffer,
                            uint16_t packet_length, vigor_time_t now) {
  uint16_t out = device;
  int rc = vp_process_one(g_ctx, device, buffer, packet_length, now, &out);
  if (rc != VP_OK) {
    fprintf(stderr, "vigpath: nf_process failed (%d)\n", rc);
    abort();
  }
  return out;
}

#endif
