/*
 * nf.h drop-in for vigfw backed by the GPU path (libvigfw_nf.so).
 *
 * The nf.h operator surface (nf.h:8-18) with vigfw's option names and parse
 * semantics (vigfw/fw_config.c:17-82), struct layout (vigfw/fw_config.h:9-24)
 * and nf_init (fw_main.c:14-19). Device count, MACs and GPU selection:
 * vp_nf_common.h.
 */
#include "vp_nf_common.h"

/* vigfw/fw_config.h:9-24 */
struct nf_config {
  uint16_t wan_device;
  struct rte_ether_addr *device_macs;
  struct rte_ether_addr *endpoint_macs;
  uint32_t expiration_time;
  uint32_t max_flows;
};

struct nf_config config;

void nf_config_usage(void) {
  printf("Usage:\n"
         "[DPDK EAL options] --\n"
         "\t--eth-dest <device>,<mac>: MAC address of the endpoint linked to "
         "a device.\n"
         "\t--expire <time>: flow expiration time (us).\n"
         "\t--max-flows <n>: flow table capacity.\n"
         "\t--wan <device>: set device to be the external one.\n");
}

/* vigfw/fw_config.c:17-82 */
void nf_config_init(int argc, char **argv) {
  uint16_t nb = nb_devices();
  struct option long_options[] = {{"eth-dest", required_argument, NULL, 'm'},
                                  {"expire", required_argument, NULL, 't'},
                                  {"max-flows", required_argument, NULL, 'f'},
                                  {"wan", required_argument, NULL, 'w'},
                                  {NULL, 0, NULL, 0}};
  config.device_macs = calloc(nb, sizeof(struct rte_ether_addr));
  config.endpoint_macs = calloc(nb, sizeof(struct rte_ether_addr));
  for (uint16_t d = 0; d < nb; d++) device_mac(d, &config.device_macs[d]);
  int opt;
  while ((opt = getopt_long(argc, argv, "m:t:f:w:", long_options, NULL)) != EOF) {
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
      case 'f':
        config.max_flows = (uint32_t)parse_int(optarg, "max-flows", '\0');
        if (config.max_flows <= 0)
          PARSE_ERROR("Flow table size must be strictly positive.\n");
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

/* vigfw/fw_config.c:94-115 */
void nf_config_print(void) {
  uint16_t nb = nb_devices();
  printf("\n--- FW Config ---\n\n");
  printf("WAN device: %" PRIu16 "\n", config.wan_device);
  for (uint16_t d = 0; d < nb; d++) {
    printf("Device %" PRIu16 " own-mac: ", d);
    print_mac(config.device_macs[d].addr_bytes);
    printf(", end-mac: ");
    print_mac(config.endpoint_macs[d].addr_bytes);
    printf("\n");
  }
  printf("Expiration time: %" PRIu32 "us\n", config.expiration_time);
  printf("Max flows: %" PRIu32 "\n", config.max_flows);
  printf("\n--- --- ------ ---\n\n");
}

/* fw_main.c:14-19: allocate the flow manager; false on failure */
bool nf_init(void) {
  vp_fw_config c;
  memset(&c, 0, sizeof c);
  uint16_t nb = nb_devices();
  c.wan_device = config.wan_device;
  c.expiration_time = config.expiration_time;
  c.max_flows = config.max_flows;
  c.n_devices = nb;
  for (uint16_t d = 0; d < nb && d < VP_MAX_DEVICES; d++) {
    if (config.device_macs) memcpy(c.device_macs[d], config.device_macs[d].addr_bytes, 6);
    if (config.endpoint_macs)
      memcpy(c.endpoint_macs[d], config.endpoint_macs[d].addr_bytes, 6);
  }
  if (g_ctx) vp_destroy(g_ctx);
  g_ctx = NULL;
  return vp_fw_create(&c, shim_gpu(), &g_ctx) == VP_OK;
}

/* fw_main.c:21-80 for one packet */
int nf_process(uint16_t device, uint8_t *buffer, uint16_t packet_length,
               vigor_time_t now) {
  return shim_process_one(device, buffer, packet_length, now);
}
