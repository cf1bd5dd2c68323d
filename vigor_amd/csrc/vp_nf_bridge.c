/*
 * nf.h drop-in for vigbridge backed by the GPU path (libvigbridge_nf.so).
 *
 * The nf.h operator surface (nf.h:8-18) with vigbridge's option names and
 * parse semantics (vigbridge/bridge_config.c:22-66), struct layout
 * (vigbridge/bridge_config.h:8-18), and nf_init (bridge_main.c:253-270)
 * including the static filtering table read from the --config file
 * (read_static_ft_from_file, bridge_main.c:103-194). Device count, MACs and
 * GPU selection: vp_nf_common.h.
 */
#include "vp_nf_common.h"

#define CONFIG_FNAME_LEN 512
#define STAT_CAPACITY 8192 /* bridge_main.c:254 */

/* vigbridge/bridge_config.h:8-18 */
struct nf_config {
  uint32_t expiration_time;
  uint32_t dyn_capacity;
  char static_config_fname[CONFIG_FNAME_LEN];
};

struct nf_config config;

void nf_config_usage(void) {
  printf("Usage:\n"
         "[DPDK EAL options] --\n"
         "\t--expire <time>: flow expiration time (us).\n"
         "\t--capacity <n>: dynamic mac learning table capacity.\n"
         "\t--config <fname>: static filtering table configuration file.\n");
}

/* vigbridge/bridge_config.c:22-66 */
void nf_config_init(int argc, char **argv) {
  config.expiration_time = 300000000; /* DEFAULT_EXP_TIME, bridge_config.c:14 */
  config.dyn_capacity = 128;          /* DEFAULT_CAPACITY, bridge_config.c:15 */
  config.static_config_fname[0] = '\0';
  struct option long_options[] = {{"expire", required_argument, NULL, 't'},
                                  {"capacity", required_argument, NULL, 'c'},
                                  {"config", required_argument, NULL, 'f'},
                                  {NULL, 0, NULL, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "t:c:f:", long_options, NULL)) != EOF) {
    switch (opt) {
      case 't':
        config.expiration_time = (uint32_t)parse_int(optarg, "exp-time", '\0');
        if (config.expiration_time <= 0)
          PARSE_ERROR("Expiration time must be strictly positive.\n");
        break;
      case 'c':
        config.dyn_capacity = (uint32_t)parse_int(optarg, "capacity", '\0');
        if (config.dyn_capacity <= 0)
          PARSE_ERROR("Flow table size must be strictly positive.\n");
        break;
      case 'f':
        strncpy(config.static_config_fname, optarg, CONFIG_FNAME_LEN - 1);
        config.static_config_fname[CONFIG_FNAME_LEN - 1] = '\0';
        break;
      default:
        PARSE_ERROR("Unknown option %c", opt);
    }
  }
  optind = 1; /* reset getopt */
}

void nf_config_print(void) {
  printf("\n--- Bridge Config ---\n\n");
  printf("Expiration time: %" PRIu32 "\n", config.expiration_time);
  printf("Capacity: %" PRIu32 "\n", config.dyn_capacity);
  printf("Static configuration file: %s\n", config.static_config_fname);
  printf("\n--- --- ------ ---\n\n");
}

/* read_static_ft_from_file (bridge_main.c:103-194): whitespace separated
 * `MAC device_from device_to` triples; malformed triples are skipped; the
 * static map must stay at most half full. Returns the rule count, or -1 when
 * the reference would rte_exit. */
static int read_static_rules(vp_bridge_rule **out) {
  *out = NULL;
  if (config.static_config_fname[0] == '\0') return 0;
  FILE *f = fopen(config.static_config_fname, "r");
  if (!f) {
    fprintf(stderr, "Error opening the static config file: %s\n",
            config.static_config_fname);
    return -1;
  }
  unsigned lines = 0;
  for (int ch = fgetc(f); ch != EOF; ch = fgetc(f))
    if (ch == '\n') lines++;
  rewind(f);
  if (STAT_CAPACITY <= lines * 2) {
    fprintf(stderr, "Too many static rules (%u), max: %d\n", lines,
            STAT_CAPACITY / 2);
    fclose(f);
    return -1;
  }
  vp_bridge_rule *r = calloc(lines + 1, sizeof *r);
  int count = 0;
  char mac_s[20], from_s[10], to_s[10];
  while (r && fscanf(f, "%18s", mac_s) == 1) {
    if (fscanf(f, "%9s", from_s) != 1 || fscanf(f, "%9s", to_s) != 1) break;
    struct rte_ether_addr a;
    char *end;
    if (!parse_mac(mac_s, &a)) continue;
    long from = strtol(from_s, &end, 10);
    if (end == from_s || *end != '\0') continue;
    long to = strtol(to_s, &end, 10);
    if (end == to_s || *end != '\0') continue;
    if ((unsigned)count >= lines + 1) break;
    memcpy(r[count].mac, a.addr_bytes, 6);
    r[count].device_from = (int32_t)from;
    r[count].device_to = (int32_t)to;
    count++;
  }
  fclose(f);
  *out = r;
  return count;
}

/* bridge_main.c:253-270 */
bool nf_init(void) {
  vp_bridge_rule *rules;
  int n = read_static_rules(&rules);
  if (n < 0) return false;
  vp_bridge_config c;
  memset(&c, 0, sizeof c);
  c.expiration_time = config.expiration_time;
  c.dyn_capacity = config.dyn_capacity;
  c.n_devices = nb_devices();
  c.n_static = (uint32_t)n;
  c.static_rules = rules;
  if (g_ctx) vp_destroy(g_ctx);
  g_ctx = NULL;
  int rc = vp_bridge_create(&c, shim_gpu(), &g_ctx);
  free(rules);
  return rc == VP_OK;
}

/* bridge_main.c:272-290 for one frame */
int nf_process(uint16_t device, uint8_t *buffer, uint16_t packet_length,
               vigor_time_t now) {
  return shim_process_one(device, buffer, packet_length, now);
}
