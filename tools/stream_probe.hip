// Diagnostic microbenchmark (not product code): the ceiling of the classify
// kernel's memory shape on MI355X. A batch of 2^24 64-byte slots (1 GiB) is
// streamed the way frames64_tiles streams it (each wave instruction moves
// 1 KiB contiguous, a wave owns 64 consecutive slots, persistent grid, each
// block a contiguous range of tiles) in these variants:
//   read        load every slot (no stores)
//   copy        load slot, store it to a second buffer
//   rmw64       load slot, store all 64 bytes back in place
//   rmw48       load slot, store bytes 0-47 back in place (UDP rewrite shape)
//   rmw64+row   rmw64 plus one 64-byte row of a 32 MB table per slot, its
//               index taken from the slot (a dependent random read, gathered
//               4 lanes per row as the classify kernel does)
// with DEPTH tiles in flight per wave (register double/triple buffering).
// Reported: Gslots/s and streamed TB/s (64 B read + 64 or 48 B written).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

enum Mode { kRead = 0, kCopy = 1, kRmw64 = 2, kRmw48 = 3, kRow64 = 4, kRow48 = 5,
            kSide = 6, kSideNoRow = 7 };
// kSide: kRow64 plus the classify kernel's side streams per slot: two u16
// inputs (len, in_dev), one u16 output (out port) and one u32 log entry.
// kSideNoRow: the same without the row.
__device__ uint16_t *g_len, *g_dev, *g_out;
__device__ uint32_t *g_log;

template <int MODE, int DEPTH, int BPC>
__global__ __launch_bounds__(256, BPC) void stream(uint4 *__restrict__ buf,
                                                   uint4 *__restrict__ dst,
                                                   const uint4 *__restrict__ table,
                                                   uint32_t rows_mask, uint32_t tiles,
                                                   uint4 *__restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t per_b = (tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t t0 = blockIdx.x * per_b, t1 = min(tiles, t0 + per_b);
  uint4 r[DEPTH][4];
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint32_t tile = t0 + wv;
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    const uint32_t tt = tile + 4 * d;
    if (tt < t1) {
#pragma unroll
      for (int j = 0; j < 4; j++) r[d][j] = buf[(size_t)tt * 256 + 64 * j + lane];
    }
  }
  for (; tile < t1; tile += 4 * DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      const uint32_t tt = tile + 4 * d;
      if (tt >= t1) break;
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = r[d][j];
      const uint32_t nt = tt + 4 * DEPTH;
      uint32_t side = 0;
      if (MODE == kSide || MODE == kSideNoRow) side = g_len[(size_t)tt * 64 + lane] + g_dev[(size_t)tt * 64 + lane];
      if (MODE == kRow64 || MODE == kRow48 || MODE == kSide) {
        // lane L fetches part L%4 of the row of slot 16j + L/4
        uint4 q[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          // v[j] of lane L is part L%4 of slot 16j + L/4: its word 1 (part 0)
          const uint32_t row = __shfl(v[j].y, lane & ~3u) & rows_mask;
          q[j] = table[(size_t)row * 4 + (lane & 3)];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
          v[j].x ^= q[j].x;
          v[j].z += q[j].z;
        }
      }
      if (nt < t1) {
#pragma unroll
        for (int j = 0; j < 4; j++) r[d][j] = buf[(size_t)nt * 256 + 64 * j + lane];
      }
      if (MODE == kSide || MODE == kSideNoRow) {
        g_out[(size_t)tt * 64 + lane] = (uint16_t)(side + v[0].x);
        g_log[(size_t)tt * 64 + lane] = side ^ v[1].y;
      }
      if (MODE == kRead) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          acc.x ^= v[j].x;
          acc.y += v[j].y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t c = 64 * j + lane;
          v[j].w += 1;
          if (MODE == kCopy)
            dst[(size_t)tt * 256 + c] = v[j];
          else if (MODE == kRmw64 || MODE == kRow64 || MODE == kSide || MODE == kSideNoRow ||
                   (c & 3) != 3)
            buf[(size_t)tt * 256 + c] = v[j];
        }
      }
    }
  }
  if ((acc.x ^ acc.y) == 0x12345678u) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE, int DEPTH, int BPC>
static void run(const char *name, uint4 *buf, uint4 *dst, const uint4 *table,
                uint32_t rows_mask, uint32_t tiles, uint4 *sink, int cus) {
  const int blocks = cus * BPC;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f, sum = 0.f;
  const int reps = 8;
  for (int rep = 0; rep < reps; rep++) {
    CK(hipEventRecord(e0));
    stream<MODE, DEPTH, BPC><<<blocks, 256>>>(buf, dst, table, rows_mask, tiles, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0) {
      sum += ms;
      if (ms < best) best = ms;
    }
  }
  const double slots = (double)tiles * 64;
  const double wr = MODE == kRead ? 0 : (MODE == kRmw48 || MODE == kRow48) ? 48 : 64;
  printf("%-10s depth %d bpc %d : %7.3f ms (mean %7.3f)  %6.2f Gslots/s  %5.2f TB/s streamed\n",
         name, DEPTH, BPC, best, sum / (reps - 1), slots / best / 1e6,
         slots * (64 + wr) / best / 1e9);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const uint32_t slots = 1u << 24, tiles = slots / 64;
  const size_t bytes = (size_t)slots * 64, tbytes = 32u << 20;
  int cus = 256;
  {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    cus = p.multiProcessorCount;
  }
  uint4 *buf, *dst, *table, *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&table, tbytes));
  CK(hipMalloc(&sink, (size_t)cus * 8 * 256 * sizeof(uint4)));
  CK(hipMemset(table, 3, tbytes));
  // slot word 1 = a spread row index (the "hash")
  {
    uint32_t *h = (uint32_t *)malloc(bytes);
    for (size_t i = 0; i < bytes / 4; i++) h[i] = (uint32_t)(i * 2654435761u);
    CK(hipMemcpy(buf, h, bytes, hipMemcpyHostToDevice));
    free(h);
  }
  const uint32_t rmask = (uint32_t)(tbytes / 64) - 1;
  {
    uint16_t *l, *d, *o;
    uint32_t *lg;
    CK(hipMalloc(&l, slots * 2));
    CK(hipMalloc(&d, slots * 2));
    CK(hipMalloc(&o, slots * 2));
    CK(hipMalloc(&lg, slots * 4));
    CK(hipMemset(l, 0, slots * 2));
    CK(hipMemset(d, 0, slots * 2));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_len), &l, sizeof(l)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_dev), &d, sizeof(d)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), &o, sizeof(o)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_log), &lg, sizeof(lg)));
  }
  run<kRead, 1, 4>("read", buf, dst, table, rmask, tiles, sink, cus);
  run<kRead, 2, 4>("read", buf, dst, table, rmask, tiles, sink, cus);
  run<kCopy, 1, 4>("copy", buf, dst, table, rmask, tiles, sink, cus);
  run<kCopy, 2, 4>("copy", buf, dst, table, rmask, tiles, sink, cus);
  run<kRmw64, 1, 4>("rmw64", buf, dst, table, rmask, tiles, sink, cus);
  run<kRmw64, 2, 4>("rmw64", buf, dst, table, rmask, tiles, sink, cus);
  run<kRmw64, 3, 4>("rmw64", buf, dst, table, rmask, tiles, sink, cus);
  run<kRmw64, 2, 2>("rmw64", buf, dst, table, rmask, tiles, sink, cus);
  run<kRmw48, 1, 4>("rmw48", buf, dst, table, rmask, tiles, sink, cus);
  run<kRmw48, 2, 4>("rmw48", buf, dst, table, rmask, tiles, sink, cus);
  run<kRow64, 1, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus);
  run<kRow64, 2, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus);
  run<kRow64, 3, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus);
  run<kRow48, 2, 4>("rmw48+row", buf, dst, table, rmask, tiles, sink, cus);
  run<kSideNoRow, 1, 4>("rmw64+side", buf, dst, table, rmask, tiles, sink, cus);
  run<kSide, 1, 4>("row+side", buf, dst, table, rmask, tiles, sink, cus);
  run<kSide, 2, 4>("row+side", buf, dst, table, rmask, tiles, sink, cus);
  run<kRow64, 1, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus);
  CK(hipFree(buf));
  CK(hipFree(dst));
  CK(hipFree(table));
  CK(hipFree(sink));
  return 0;
}
