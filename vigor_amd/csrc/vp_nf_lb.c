/*
 * nf.h drop-in for viglb backed by the GPU path (libviglb_nf.so).
 *
 * The nf.h operator surface (nf.h:8-18) with viglb's option names and parse
 * semantics (viglb/lb_config.c:15-86), struct layout (viglb/lb_config.h:8-38)
 * and nf_init (lb_main.c:13-18). Device count, MACs and GPU selection:
 * vp_nf_common.h.
 */
#include "vp_nf_common.h"

/* viglb/lb_config.h:8-38 */
struct nf_config {
  uint16_t backend_count;
  struct rte_ether_addr *device_macs;
  uint32_t flow_capacity;
  uint32_t flow_expiration_time;
  uint32_t backend_capacity;
  uint32_t cht_height;
  uint32_t backend_expiration_time;
  uint16_t wan_device;
};

struct nf_config config;

void nf_config_usage(void) {
  printf("Usage:\n"
         "[DPDK EAL options] --\n"
         "\t--flow-expiration <time>: flow expiration time (us).\n"
         "\t--flow-capacity <n>: flow table capacity.\n"
         "\t--backend-capacity <n>: backend table capacity.\n"
         "\t--cht-height <n>: consistent hashing table height: bigger <n> "
         "generates more smooth distribution.\n"
         "\t--backend-expiration <time>: backend expiration time (us).\n"
         "\t--wan <device>: set device to be the external one.\n");
}

/* viglb/lb_config.c:15-86 */
void nf_config_init(int argc, char **argv) {
  uint16_t nb = nb_devices();
  struct option long_options[] = {
      {"flow-expiration", required_argument, NULL, 'x'},
      {"flow-capacity", required_argument, NULL, 'f'},
      {"backend-capacity", required_argument, NULL, 's'},
      {"cht-height", required_argument, NULL, 'h'},
      {"backend-expiration", required_argument, NULL, 't'},
      {"wan", required_argument, NULL, 'w'},
      {NULL, 0, NULL, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "b:x:f:", long_options, NULL)) != EOF) {
    switch (opt) {
      case 'x':
        config.flow_expiration_time =
            (uint32_t)parse_int(optarg, "flow-expiration", '\0');
        if (config.flow_expiration_time == 0)
          PARSE_ERROR("Flow expiration time must be strictly positive.\n");
        break;
      case 'f':
        config.flow_capacity = (uint32_t)parse_int(optarg, "flow-capacity", '\0');
        if (config.flow_capacity <= 0)
          PARSE_ERROR("Flow capacity must be strictly positive.\n");
        break;
      case 's':
        config.backend_capacity =
            (uint32_t)parse_int(optarg, "backend-capacity", '\0');
        if (config.backend_capacity <= 0)
          PARSE_ERROR("Backend capacity must be strictly positive.\n");
        break;
      case 'h':
        config.cht_height = (uint32_t)parse_int(optarg, "cht-height", '\0');
        if (config.cht_height <= 0)
          PARSE_ERROR("CHT height must be strictly positive.\n");
        break;
      case 't':
        config.backend_expiration_time =
            (uint32_t)parse_int(optarg, "backend-expiration", '\0');
        if (config.backend_expiration_time == 0)
          PARSE_ERROR("Backend expiration time must be strictly positive.\n");
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
  config.device_macs = calloc(nb, sizeof(struct rte_ether_addr));
  for (uint16_t d = 0; d < nb; d++) device_mac(d, &config.device_macs[d]);
}

void nf_config_print(void) {
  printf("\n--- LoadBalancer Config ---\n\n");
  printf("Flow expiration time: %" PRIu32 "\n", config.flow_expiration_time);
  printf("Flow capacity: %" PRIu32 "\n", config.flow_capacity);
  printf("Backend capacity: %" PRIu32 "\n", config.backend_capacity);
  printf("CHT height: %" PRIu32 "\n", config.cht_height);
  printf("Backend expiration time: %" PRIu32 "\n", config.backend_expiration_time);
  printf("WAN device: %" PRIu16 "\n", config.wan_device);
  printf("\n--- --- ------ ---\n\n");
}

/* lb_main.c:13-18 (lb_allocate_balancer); false on failure */
bool nf_init(void) {
  vp_lb_config c;
  memset(&c, 0, sizeof c);
  uint16_t nb = nb_devices();
  c.flow_capacity = config.flow_capacity;
  c.flow_expiration_time = config.flow_expiration_time;
  c.backend_capacity = config.backend_capacity;
  c.cht_height = config.cht_height;
  c.backend_expiration_time = config.backend_expiration_time;
  c.wan_device = config.wan_device;
  c.n_devices = nb;
  for (uint16_t d = 0; d < nb && d < VP_MAX_DEVICES; d++)
    if (config.device_macs) memcpy(c.device_macs[d], config.device_macs[d].addr_bytes, 6);
  if (g_ctx) vp_destroy(g_ctx);
  g_ctx = NULL;
  return vp_lb_create(&c, shim_gpu(), &g_ctx) == VP_OK;
}

/* lb_main.c:20-68 for one packet */
int nf_process(uint16_t device, uint8_t *buffer, uint16_t packet_length,
               vigor_time_t now) {
  return shim_process_one(device, buffer, packet_length, now);
}
