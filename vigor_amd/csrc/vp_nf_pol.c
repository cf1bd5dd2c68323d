/*
 * nf.h drop-in for vigpol backed by the GPU path (libvigpol_nf.so).
 *
 * The nf.h operator surface (nf.h:8-18) with vigpol's option names, defaults
 * and parse semantics (vigpol/policer_config.c:9-93), struct layout
 * (vigpol/policer_config.h:9-24) and nf_init (policer_main.c:113-117).
 * Device count and GPU selection: vp_nf_common.h.
 */
#include "vp_nf_common.h"

/* vigpol/policer_config.h:9-24 */
struct nf_config {
  uint16_t lan_device;
  uint16_t wan_device;
  uint64_t rate;
  uint64_t burst;
  uint32_t dyn_capacity;
};

struct nf_config config;

/* policer_config.c:9-13 */
static const uint16_t DEFAULT_LAN = 1;
static const uint16_t DEFAULT_WAN = 0;
static const uint64_t DEFAULT_RATE = 1000000;
static const uint64_t DEFAULT_BURST = 100000;
static const uint32_t DEFAULT_CAPACITY = 128;

void nf_config_usage(void) {
  printf("Usage:\n"
         "[DPDK EAL options] --\n"
         "\t--lan <device>: LAN device, default: %" PRIu16 ".\n"
         "\t--wan <device>: WAN device, default: %" PRIu16 ".\n"
         "\t--rate <rate>: policer rate in bytes/s, default: %" PRIu64 ".\n"
         "\t--burst <size>: policer burst size in bytes, default: %" PRIu64 ".\n"
         "\t--capacity <n>: policer table capacity, default: %" PRIu32 ".\n",
         DEFAULT_LAN, DEFAULT_WAN, DEFAULT_RATE, DEFAULT_BURST, DEFAULT_CAPACITY);
}

/* vigpol/policer_config.c:20-93 */
void nf_config_init(int argc, char **argv) {
  config.lan_device = DEFAULT_LAN;
  config.wan_device = DEFAULT_WAN;
  config.rate = DEFAULT_RATE;
  config.burst = DEFAULT_BURST;
  config.dyn_capacity = DEFAULT_CAPACITY;
  unsigned nb = nb_devices();
  struct option long_options[] = {{"lan", required_argument, NULL, 'l'},
                                  {"wan", required_argument, NULL, 'w'},
                                  {"rate", required_argument, NULL, 'r'},
                                  {"burst", required_argument, NULL, 'b'},
                                  {"capacity", required_argument, NULL, 'c'},
                                  {NULL, 0, NULL, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "l:w:r:b:c:", long_options, NULL)) != EOF) {
    switch (opt) {
      case 'l':
        config.lan_device = (uint16_t)parse_int(optarg, "lan", '\0');
        if (config.lan_device >= nb) PARSE_ERROR("Invalid LAN device.\n");
        break;
      case 'w':
        config.wan_device = (uint16_t)parse_int(optarg, "wan", '\0');
        if (config.wan_device >= nb) PARSE_ERROR("Invalid WAN device.\n");
        break;
      case 'r':
        config.rate = (uint64_t)parse_int(optarg, "rate", '\0');
        if (config.rate == 0)
          PARSE_ERROR("Policer rate must be strictly positive.\n");
        break;
      case 'b':
        config.burst = (uint64_t)parse_int(optarg, "burst", '\0');
        if (config.burst == 0)
          PARSE_ERROR("Policer burst size must be strictly positive.\n");
        break;
      case 'c':
        config.dyn_capacity = (uint32_t)parse_int(optarg, "capacity", '\0');
        if (config.dyn_capacity <= 0)
          PARSE_ERROR("Flow table size must be strictly positive.\n");
        break;
      default:
        PARSE_ERROR("Unknown option %c", opt);
    }
  }
  optind = 1; /* reset getopt */
}

/* vigpol/policer_config.c:95-114 */
void nf_config_print(void) {
  printf("\n--- Policer Config ---\n\n");
  printf("LAN Device: %" PRIu16 "\n", config.lan_device);
  printf("WAN Device: %" PRIu16 "\n", config.wan_device);
  printf("Rate: %" PRIu64 "\n", config.rate);
  printf("Burst: %" PRIu64 "\n", config.burst);
  printf("Capacity: %" PRIu32 "\n", config.dyn_capacity);
  printf("\n--- ------ ------ ---\n\n");
}

/* policer_main.c:113-117: allocate the state; false on failure */
bool nf_init(void) {
  vp_pol_config c;
  memset(&c, 0, sizeof c);
  c.lan_device = config.lan_device;
  c.wan_device = config.wan_device;
  c.rate = config.rate;
  c.burst = config.burst;
  c.dyn_capacity = config.dyn_capacity;
  c.n_devices = nb_devices();
  if (g_ctx) vp_destroy(g_ctx);
  g_ctx = NULL;
  return vp_pol_create(&c, shim_gpu(), &g_ctx) == VP_OK;
}

/* policer_main.c:119-145 for one packet */
int nf_process(uint16_t device, uint8_t *buffer, uint16_t packet_length,
               vigor_time_t now) {
  return shim_process_one(device, buffer, packet_length, now);
}
