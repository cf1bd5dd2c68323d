// Diagnostic microbenchmark (not product code): what does one random read
// of a table row cost on MI355X, by row size? Decides the flow table's
// bucket size.
//
// Each group of g lanes (g = 1, 2, 4, 8) reads one random, 16g-byte-aligned
// row of 16g bytes as g uint4 (one wave instruction per row set, rows in
// flight = 64 / g per wave instruction, `depth` independent instructions per
// lane). Reported: rows per second and requested GB/s per table size. If a
// 32-B or 64-B row costs the same as a 128-B one, the fabric moves whole
// 128-B lines and a bucket should be one line.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/gran_probe tools/gran_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// rows_mask: number of rows - 1 (power of two); total_sets: wave-level
// iterations over the whole grid.
template <int G, int DEPTH>
__global__ __launch_bounds__(256) void gather(const uint4 *__restrict__ t,
                                              uint32_t rows_mask,
                                              uint32_t iters, uint32_t seed,
                                              uint4 *__restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t gid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t grp = lane / G, part = lane % G;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t it = 0; it < iters; it++) {
    uint4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      const uint32_t r =
          mix32(seed ^ (gid * 0x9E3779B9u) ^ ((it * DEPTH + d) * 0x85EBCA6Bu) ^
                (grp * 0xC2B2AE35u)) & rows_mask;
      v[d] = t[(size_t)r * G + part];
    }
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      acc.x ^= v[d].x;
      acc.y += v[d].y;
      acc.z ^= v[d].z;
      acc.w += v[d].w;
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int G>
static void run(const uint4 *t, size_t table_bytes, uint4 *sink, int blocks) {
  const uint32_t rows = (uint32_t)(table_bytes / (16 * G));
  const uint32_t iters = 64;
  constexpr int DEPTH = 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CK(hipEventRecord(e0));
    gather<G, DEPTH><<<blocks, 256>>>(t, rows - 1, iters, 17u + rep, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double row_reads = (double)blocks * 256 / G * iters * DEPTH;
  printf("table %6zu MB  row %3d B : %8.3f ms  %7.2f Grows/s  %6.2f TB/s requested\n",
         table_bytes >> 20, 16 * G, best, row_reads / best / 1e6,
         row_reads * 16 * G / best / 1e9);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  const size_t sizes[] = {32u << 20, 64u << 20, 1024u << 20};
  const int blocks = 256 * 8;  // 8 workgroups (32 waves) per CU
  uint4 *sink;
  CK(hipMalloc(&sink, (size_t)blocks * 256 * sizeof(uint4)));
  for (size_t sz : sizes) {
    uint4 *t;
    CK(hipMalloc(&t, sz));
    CK(hipMemset(t, 1, sz));
    CK(hipDeviceSynchronize());
    run<1>(t, sz, sink, blocks);
    run<2>(t, sz, sink, blocks);
    run<4>(t, sz, sink, blocks);
    run<8>(t, sz, sink, blocks);
    CK(hipFree(t));
  }
  CK(hipFree(sink));
  return 0;
}
