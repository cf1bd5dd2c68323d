// Diagnostic microbenchmark (not product code): the memory ceiling of the
// 128-byte-slot classify tile's shape (nat_classify128, vp_nat.hip). 2^24
// slots of SLOT bytes are streamed as the kernel streams them: a persistent
// grid (4 blocks of 256 threads per CU), each block a contiguous range of
// 64-slot tiles, its four waves interleaved over it, each load instruction
// 1 KiB contiguous. Variants:
//   read     load every slot
//   hdr      load every slot, store its first 64 bytes back in place
//            (what a NAT rewrite stores)
//   whole    load every slot, store all of it back in place
// each with write-through (sc1) or default stores. Reported: Gslots/s and
// the TB/s of bytes moved (slot read + bytes stored).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/slot_probe tools/slot_probe.hip
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

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// N = 16-byte chunks per slot (4: 64-byte slots, 8: 128-byte slots);
// ST = 0 none, 1 the first 64 bytes, 2 all; WT = write-through stores
template <uint32_t N, uint32_t ST, bool WT>
__global__ __launch_bounds__(256, 4) void slots(uint4 *buf, uint32_t tiles, uint4 *sink) {
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t per_b = (tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t tend = min(tiles, blockIdx.x * per_b + per_b);
  v4u acc = {0, 0, 0, 0};
  for (uint32_t tile = blockIdx.x * per_b + wv; tile < tend; tile += 4) {
    uint4 *g = buf + (size_t)tile * 64 * N;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(g, 0, 64 * N * 16, 0x00020000);
    v4u d[N];
#pragma unroll
    for (uint32_t j = 0; j < N; j++)
      d[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((64 * j + lane) * 16), 0, 0);
#pragma unroll
    for (uint32_t j = 0; j < N; j++) {
      acc += d[j];
      d[j].x += 1;
    }
    if constexpr (ST != 0) {
#pragma unroll
      for (uint32_t j = 0; j < N; j++) {
        // chunk 64 j + lane is part (64 j + lane) % N of its slot
        const bool hdr = ((64 * j + lane) % N) < 4;
        if (ST == 2 || hdr)
          __builtin_amdgcn_raw_buffer_store_b128(d[j], rs, (int)((64 * j + lane) * 16), 0,
                                                 WT ? 16 : 0);
      }
    }
  }
  if (acc.x == 0x12345678u) sink[blockIdx.x * 256 + threadIdx.x] = make_uint4(acc.x, acc.y, acc.z, acc.w);
}

template <uint32_t N, uint32_t ST, bool WT>
static void run(uint4 *buf, uint32_t slots_n, int grid, uint4 *sink, const char *name) {
  const uint32_t tiles = slots_n / 64;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; i++) slots<N, ST, WT><<<grid, 256>>>(buf, tiles, sink);
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) slots<N, ST, WT><<<grid, 256>>>(buf, tiles, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double per = 16.0 * N + (ST == 0 ? 0 : ST == 1 ? 64 : 16.0 * N);
  printf("slot %3u %-6s %-3s %.4f ms  %.2f Gslots/s  %.2f TB/s\n", 16 * N, name,
         WT ? "wt" : "wb", ms, slots_n / ms / 1e6, slots_n * per / ms / 1e9);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  const uint32_t n = 1u << 24;
  int cus = 256;
  {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    cus = p.multiProcessorCount;
  }
  const int grid = 4 * cus;
  uint4 *buf, *sink;
  CK(hipMalloc(&buf, (size_t)n * 128));
  CK(hipMalloc(&sink, (size_t)grid * 256 * sizeof(uint4)));
  CK(hipMemset(buf, 1, (size_t)n * 128));
  for (int r = 0; r < 2; r++) {
    run<4, 0, true>(buf, n, grid, sink, "read");
    run<4, 2, true>(buf, n, grid, sink, "whole");
    run<8, 0, true>(buf, n, grid, sink, "read");
    run<8, 1, true>(buf, n, grid, sink, "hdr");
    run<8, 1, false>(buf, n, grid, sink, "hdr");
    run<8, 2, true>(buf, n, grid, sink, "whole");
    run<8, 2, false>(buf, n, grid, sink, "whole");
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
