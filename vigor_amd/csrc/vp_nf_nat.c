/*
 * nf.h drop-in for vignat backed by the GPU path (libvignat_nf.so).
 *
 * Exports exactly the operator surface the reference's nf.c links against
 * (nf.h:8-18): nf_init, nf_process, nf_config_init, nf_config_usage,
 * nf_config_print and `struct nf_config config`, with vignat's option names
 * and parse semantics (vignat/nat_config.c:17-106) and struct layout
 * (vignat/nat_config.h:5-31). nf_process runs one packet through the batch
 * C-ABI (vp_process_batch); a batching caller should call vp_process_batch
 * directly (include/vigpath.h).
 *
 * Device count and MACs come from DPDK's rte_eth_dev_count_avail /
 * rte_eth_macaddr_get when the host process links DPDK (weak references);
 * otherwise from VIGPATH_NB_DEVICES (default 2) and 02:00:00:00:00:<dev>.
 * VIGPATH_GPU selects the HIP device (default 0).
 */
#include <errno.h>
#include <getopt.h>
#include <inttypes.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/vigpath.h"

typedef int64_t vigor_time_t; /* libvig/verified/vigor-time.h:7 */

struct rte_ether_addr {
  uint8_t addr_bytes[6];
};

/* vignat/nat_config.h:5-31 */
struct nf_config {
  uint16_t lan_main_device;
  uint16_t wan_device;
  uint32_t external_addr;
  struct rte_ether_addr *device_macs;
  struct rte_ether_addr *endpoint_macs;
  uint16_t start_port;
  uint32_t expiration_time;
  uint32_t max_flows;
};

struct nf_config config;

/* DPDK 20.08 (setup.sh:94): present only when the host links DPDK */
extern uint16_t rte_eth_dev_count_avail(void) __attribute__((weak));
extern void rte_eth_macaddr_get(uint16_t port_id, struct rte_ether_addr *mac)
    __attribute__((weak));

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

void nf_config_usage(void) {
  printf("Usage:\n"
         "[DPDK EAL options] --\n"
         "\t--eth-dest <device>,<mac>: MAC address of the endpoint linked to "
         "a device.\n"
         "\t--expire <time>: flow expiration time (us).\n"
         "\t--extip <ip>: external IP address.\n"
         "\t--lan-dev <device>: set device to be the main LAN device (for "
         "non-NAT).\n"
         "\t--max-flows <n>: flow table capacity.\n"
         "\t--starting-port <n>: start of the port range for external ports.\n"
         "\t--wan <device>: set device to be the external one.\n");
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

/* nf_parse_etheraddr / nf_parse_ipv4addr (nf-parse.h:9-32) */
static bool parse_mac(const char *s, struct rte_ether_addr *a) {
  return sscanf(s, "%02hhX:%02hhX:%02hhX:%02hhX:%02hhX:%02hhX",
                a->addr_bytes + 0, a->addr_bytes + 1, a->addr_bytes + 2,
                a->addr_bytes + 3, a->addr_bytes + 4, a->addr_bytes + 5) == 6;
}
static bool parse_ipv4(const char *s, uint32_t *out) {
  uint8_t a, b, c, d;
  if (sscanf(s, "%hhu.%hhu.%hhu.%hhu", &a, &b, &c, &d) != 4) return false;
  *out = ((uint32_t)a << 24) | ((uint32_t)b << 16) | ((uint32_t)c << 8) | d;
  return true;
}

/* vignat/nat_config.c:17-106 */
void nf_config_init(int argc, char **argv) {
  uint16_t nb = nb_devices();
  struct option long_options[] = {{"eth-dest", required_argument, NULL, 'm'},
                                  {"expire", required_argument, NULL, 't'},
                                  {"extip", required_argument, NULL, 'i'},
                                  {"lan-dev", required_argument, NULL, 'l'},
                                  {"max-flows", required_argument, NULL, 'f'},
                                  {"starting-port", required_argument, NULL, 's'},
                                  {"wan", required_argument, NULL, 'w'},
                                  {NULL, 0, NULL, 0}};
  config.device_macs = calloc(nb, sizeof(struct rte_ether_addr));
  config.endpoint_macs = calloc(nb, sizeof(struct rte_ether_addr));
  for (uint16_t d = 0; d < nb; d++) device_mac(d, &config.device_macs[d]);
  int opt;
  while ((opt = getopt_long(argc, argv, "m:e:t:i:l:f:p:s:w:", long_options,
                            NULL)) != EOF) {
    unsigned device;
    switch (opt) {
      case 'm':
        device = (unsigned)parse_int(optarg, "eth-dest device", ',');
        if (device >= nb)
          PARSE_ERROR("eth-dest: device %d >= nb_devices (%d)\n", device, nb);
        optarg += 2;
        if (!parse_mac(optarg, &config.endpoint_macs[device]))
          PARSE_ERROR("Invalid MAC address: %s\n", optarg);
        break;
      case 't':
        config.expiration_time = (uint32_t)parse_int(optarg, "exp-time", '\0');
        if (config.expiration_time == 0)
          PARSE_ERROR("Expiration time must be strictly positive.\n");
        break;
      case 'i':
        if (!parse_ipv4(optarg, &config.external_addr))
          PARSE_ERROR("Invalid external IP address: %s\n", optarg);
        break;
      case 'l':
        config.lan_main_device = (uint16_t)parse_int(optarg, "lan-dev", '\0');
        if (config.lan_main_device >= nb)
          PARSE_ERROR("Main LAN device does not exist.\n");
        break;
      case 'f':
        config.max_flows = (uint32_t)parse_int(optarg, "max-flows", '\0');
        if (config.max_flows <= 0)
          PARSE_ERROR("Flow table size must be strictly positive.\n");
        break;
      case 's':
        config.start_port = (uint16_t)parse_int(optarg, "start-port", '\0');
        break;
      case 'w':
        config.wan_device = (uint16_t)parse_int(optarg, "wan-dev", '\0');
        if (config.wan_device >= nb) PARSE_ERROR("WAN device does not exist.\n");
        break;
      default:
        PARSE_ERROR("Unknown option.\n");
    }
  }
  optind = 1; /* reset getopt */
}

void nf_config_print(void) {
  uint16_t nb = nb_devices();
  printf("\n--- NAT Config ---\n\n");
  printf("Main LAN device (only relevant for NOP): %" PRIu16 "\n",
         config.lan_main_device);
  printf("WAN device: %" PRIu16 "\n", config.wan_device);
  uint32_t a = config.external_addr;
  printf("External IP: %u.%u.%u.%u\n", a & 0xFF, (a >> 8) & 0xFF,
         (a >> 16) & 0xFF, (a >> 24) & 0xFF); /* nf-util.c:95-111 */
  for (uint16_t d = 0; d < nb; d++) {
    const uint8_t *m = config.device_macs[d].addr_bytes;
    const uint8_t *e = config.endpoint_macs[d].addr_bytes;
    printf("Device %" PRIu16 " own-mac: %02X:%02X:%02X:%02X:%02X:%02X, "
           "end-mac: %02X:%02X:%02X:%02X:%02X:%02X\n",
           d, m[0], m[1], m[2], m[3], m[4], m[5], e[0], e[1], e[2], e[3], e[4],
           e[5]);
  }
  printf("Starting port: %" PRIu16 "\n", config.start_port);
  printf("Expiration time: %" PRIu32 "us\n", config.expiration_time);
  printf("Max flows: %" PRIu32 "\n", config.max_flows);
  printf("\n--- --- ------ ---\n\n");
}

/* nat_main.c:14-20: allocate the flow manager; false on failure */
bool nf_init(void) {
  vp_nat_config c;
  memset(&c, 0, sizeof c);
  uint16_t nb = nb_devices();
  c.wan_device = config.wan_device;
  c.lan_main_device = config.lan_main_device;
  c.start_port = config.start_port;
  c.external_addr = config.external_addr;
  c.expiration_time = config.expiration_time;
  c.max_flows = config.max_flows;
  c.n_devices = nb;
  for (uint16_t d = 0; d < nb && d < VP_MAX_DEVICES; d++) {
    if (config.device_macs) memcpy(c.device_macs[d], config.device_macs[d].addr_bytes, 6);
    if (config.endpoint_macs)
      memcpy(c.endpoint_macs[d], config.endpoint_macs[d].addr_bytes, 6);
  }
  const char *g = getenv("VIGPATH_GPU");
  if (g_ctx) vp_destroy(g_ctx);
  g_ctx = NULL;
  return vp_nat_create(&c, g ? atoi(g) : 0, &g_ctx) == VP_OK;
}

/* nat_main.c:22-109 for one packet. The reference has no error path; a
 * device failure here aborts like nf.c's tx failure does (nf.c:167-172). */
int nf_process(uint16_t device, uint8_t *buffer, uint16_t packet_length,
               vigor_time_t now) {
  uint16_t out = device;
  uint8_t *frames[1] = {buffer};
  int rc = vp_process_batch(g_ctx, 1, &device, frames, &packet_length, &now, &out);
  if (rc != VP_OK) {
    fprintf(stderr, "vigpath: nf_process failed (%d)\n", rc);
    abort();
  }
  return out;
}
