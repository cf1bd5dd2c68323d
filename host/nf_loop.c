/*
 * Host-side C driver restating the reference's nf.c worker loop over a trace
 * file instead of DPDK rx/tx queues (reference nf.c:143-216):
 *
 *   per packet:  packet_state_total_length -> dst = nf_process(port, data,
 *                len, now) -> dst == in ? drop : dst == FLOOD_FRAME ? flood
 *                : tx                                      (nf.c:150-176)
 *
 * It links against the nf.h surface only (nf_config_init / nf_init /
 * nf_process), so the same source links against the reference NF objects or
 * against our libvignat_nf.so. With --batch B it instead hands B packets at
 * a time to vp_process_batch (the batched form, nf.c:178-215).
 *
 * usage: nf_loop <trace.in> <trace.out> [--batch B] [--warm W] -- <NF options>
 * --warm W: the first W packets run first, untimed; the rest are timed and
 * the rate is printed on stderr ("timed P packets: S s, U us/packet, K Kpps":
 * the per-packet cost of the drop-in).
 * trace.in:  "VPTR" u32 n u32 slot, u16 in_dev[n], u16 len[n], i64 now[n],
 *            u8 frames[n*slot]
 * trace.out: "VPTO" u32 n u32 slot, u16 out_dev[n], u8 frames[n*slot],
 *            "VPTX" u32 txmask[n]: the ports each packet leaves on, as nf.c
 *            dispatches it. Per-packet path (VIGOR_BATCH_SIZE == 1,
 *            nf.c:158-175): none (drop: dst == in), every port but the input
 *            (flood(mbuf, VIGOR_DEVICES_COUNT), nf.c:83-96, where
 *            VIGOR_DEVICES_COUNT = rte_eth_dev_count_avail(), nf.c:57), or
 *            dst (rte_eth_tx_burst). With --batch and two ports, nf.c's
 *            batched loop (nf.c:186-209): every packet that is not dropped,
 *            floods included, goes to port 1 - in. The reference's batched
 *            loop refuses any other port count (nf.c:179-182); there the
 *            per-packet dispatch is kept. The port count comes from
 *            VIGPATH_NB_DEVICES (default 2), as in the nf.h shims.
 */
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/vigpath.h"

typedef int64_t vigor_time_t;
bool nf_init(void);
int nf_process(uint16_t device, uint8_t *buffer, uint16_t packet_length,
               vigor_time_t now);
void nf_config_init(int argc, char **argv);
void nf_config_print(void);
#define FLOOD_FRAME ((uint16_t)-1)

static void *xread(FILE *f, size_t bytes) {
  void *p = malloc(bytes ? bytes : 1);
  if (!p || fread(p, 1, bytes, f) != bytes) {
    fprintf(stderr, "short trace\n");
    exit(2);
  }
  return p;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s in out [--batch B] -- NF options\n", argv[0]);
    return 2;
  }
  uint32_t batch = 0, warm = 0;
  int nf_argc = 1;
  char **nf_argv = argv + 2; /* argv[2] stands in for the program name */
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--batch") && i + 1 < argc) {
      batch = (uint32_t)atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--warm") && i + 1 < argc) {
      warm = (uint32_t)atoi(argv[++i]);
    } else if (!strcmp(argv[i], "--")) {
      nf_argv = argv + i;
      nf_argc = argc - i;
      break;
    }
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) {
    perror(argv[1]);
    return 2;
  }
  char magic[4];
  uint32_t n, slot;
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "VPTR", 4) ||
      fread(&n, 4, 1, f) != 1 || fread(&slot, 4, 1, f) != 1) {
    fprintf(stderr, "bad trace header\n");
    return 2;
  }
  uint16_t *in_dev = xread(f, 2ull * n);
  uint16_t *len = xread(f, 2ull * n);
  int64_t *now = xread(f, 8ull * n);
  uint8_t *frames = xread(f, (size_t)n * slot);
  fclose(f);

  nf_config_init(nf_argc, nf_argv); /* nf.c:230 */
  if (!nf_init()) {                 /* nf.c:144-146 */
    fprintf(stderr, "Error initializing NF\n");
    return 1;
  }
  uint16_t *out = calloc(n ? n : 1, 2);
  uint64_t drops = 0, floods = 0, tx = 0;
  if (warm > n) warm = n;
  struct timespec t0 = {0, 0}, t1;
  if (batch == 0) {
    for (uint32_t i = 0; i < n; i++) { /* nf.c:150-176 */
      if (i == warm) clock_gettime(CLOCK_MONOTONIC, &t0);
      out[i] = (uint16_t)nf_process(in_dev[i], frames + (size_t)i * slot, len[i],
                                    now[i]);
    }
  } else {
    extern vp_ctx *vp_nf_context(void);
    uint8_t **ptrs = malloc(sizeof(uint8_t *) * batch);
    for (uint32_t a = 0; a < warm; a += batch) {  /* untimed */
      uint32_t m = warm - a < batch ? warm - a : batch;
      for (uint32_t i = 0; i < m; i++) ptrs[i] = frames + (size_t)(a + i) * slot;
      if (vp_process_batch(vp_nf_context(), m, in_dev + a, ptrs, len + a,
                           now + a, out + a) != VP_OK) {
        fprintf(stderr, "vp_process_batch failed\n");
        return 1;
      }
    }
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint32_t a = warm; a < n; a += batch) {
      uint32_t m = n - a < batch ? n - a : batch;
      for (uint32_t i = 0; i < m; i++) ptrs[i] = frames + (size_t)(a + i) * slot;
      if (vp_process_batch(vp_nf_context(), m, in_dev + a, ptrs, len + a,
                           now + a, out + a) != VP_OK) {
        fprintf(stderr, "vp_process_batch failed\n");
        return 1;
      }
    }
    free(ptrs);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (n > warm) {
    const double el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    fprintf(stderr, "timed %u packets: %.6f s, %.3f us/packet, %.2f Kpps\n", n - warm, el,
            1e6 * el / (n - warm), (n - warm) / el / 1e3);
  }
  const char *nd = getenv("VIGPATH_NB_DEVICES");
  const uint32_t nb_devices = nd ? (uint32_t)atoi(nd) : 2u;
  uint32_t *txmask = calloc(n ? n : 1, 4);
  const bool batch_dispatch = batch != 0 && nb_devices == 2;  /* nf.c:186-209 */
  for (uint32_t i = 0; i < n; i++) {  /* nf.c:158-175 */
    if (out[i] == in_dev[i]) {
      drops++;
    } else if (batch_dispatch) {  /* mbufs_to_send -> tx_burst(1 - VIGOR_DEVICE) */
      if (out[i] == FLOOD_FRAME) floods++; else tx++;
      if (in_dev[i] < 2) txmask[i] = 1u << (1 - in_dev[i]);
    } else if (out[i] == FLOOD_FRAME) {  /* flood(): nf.c:83-96 */
      floods++;
      for (uint32_t d = 0; d < nb_devices && d < 32; d++)
        if (d != in_dev[i]) txmask[i] |= 1u << d;
    } else {
      tx++;
      if (out[i] < 32) txmask[i] = 1u << out[i];
    }
  }
  FILE *o = fopen(argv[2], "wb");
  if (!o) {
    perror(argv[2]);
    return 2;
  }
  fwrite("VPTO", 1, 4, o);
  fwrite(&n, 4, 1, o);
  fwrite(&slot, 4, 1, o);
  fwrite(out, 2, n, o);
  fwrite(frames, 1, (size_t)n * slot, o);
  fwrite("VPTX", 1, 4, o);
  fwrite(txmask, 4, n, o);
  fclose(o);
  printf("packets %u tx %llu drop %llu flood %llu\n", n, (unsigned long long)tx,
         (unsigned long long)drops, (unsigned long long)floods);
  return 0;
}
