/* The bench's timed loop in C: n prepared vp_process_device calls in order,
 * as nf.c's main loop (nf.c:178-215) makes one call per burst with no
 * interpreter between them. bench.py builds the descriptors (one per
 * batch buffer, its time stamps set) and times this call; Python's per-call
 * overhead (ctypes, the loop) would otherwise sit on the step's critical path
 * while the fold of the previous batch runs. Not part of the
 * C-ABI: test and measurement infrastructure (libvp_steps.so). */
#include <stdint.h>

#include "../include/vigpath.h"

/* 0, or the first failing call's return code (*done: the calls made). */
int vp_steps_device(vp_ctx *ctx, const vp_dev_batch *b, int n, int *done) {
  int k = 0, rc = 0;
  for (; k < n; k++) {
    rc = vp_process_device(ctx, &b[k], 0);
    if (rc) break;
  }
  if (done) *done = k;
  return rc;
}
