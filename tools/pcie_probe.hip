// Diagnostic microbenchmark (not product code): how fast can frames that
// start and end in page-locked host memory (nf.c's mbufs, nf.c:153,166) reach
// the GPU and come back on MI355X?
//   copy H2D / D2H          hipMemcpyAsync of 1 GiB, one direction
//   copy H2D + D2H          both at once on two streams (full duplex?)
//   kernel rd / wr / rmw    a kernel streaming 64-byte slots straight from
//                           host memory (zero-copy: loads and stores cross
//                           PCIe, no staging), 1 KiB contiguous per wave
//                           instruction as in the classify kernel
// Reported: GB/s and, for the kernels, Gslots/s (= Gpackets/s of 64 B).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/pcie_probe tools/pcie_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

enum { kRd = 0, kWr = 1, kRmw = 2 };

template <int MODE>
__global__ __launch_bounds__(256) void host_stream(uint4 *buf, uint32_t tiles,
                                                  uint4 *sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t t = wid; t < tiles; t += nw) {
    uint4 v[4];
    if (MODE != kWr) {
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = buf[(size_t)t * 256 + 64 * j + lane];
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = make_uint4(t, j, lane, 7);
    }
    if (MODE == kRd) {
#pragma unroll
      for (int j = 0; j < 4; j++) acc.x ^= v[j].x + v[j].w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        v[j].y += 1;
        buf[(size_t)t * 256 + 64 * j + lane] = v[j];
      }
    }
  }
  if (acc.x == 0x12345678u) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int MODE>
static void run_kernel(const char *name, uint4 *dptr, uint32_t tiles, uint4 *sink,
                       int blocks) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    CK(hipEventRecord(e0));
    host_stream<MODE><<<blocks, 256>>>(dptr, tiles, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double slots = (double)tiles * 64;
  const double bytes = slots * 64 * (MODE == kRmw ? 2 : 1);
  printf("kernel %-4s blocks %5d : %8.3f ms  %6.2f GB/s  %6.3f Gslots/s\n", name, blocks,
         best, bytes / best / 1e6, slots / best / 1e6);
}

int main() {
  const size_t bytes = 1ull << 30;
  const uint32_t tiles = (uint32_t)(bytes / 4096);
  uint8_t *h, *h2, *d, *d2;
  CK(hipHostMalloc((void **)&h, bytes, hipHostMallocDefault));
  CK(hipHostMalloc((void **)&h2, bytes, hipHostMallocDefault));
  CK(hipMalloc((void **)&d, bytes));
  CK(hipMalloc((void **)&d2, bytes));
  memset(h, 1, bytes);
  memset(h2, 2, bytes);
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto wall = [](auto fn) {
    const auto t0 = std::chrono::steady_clock::now();
    fn();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  };
  for (int rep = 0; rep < 2; rep++) {
    const double t_h2d = wall([&] {
      CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1));
      CK(hipStreamSynchronize(s1));
    });
    const double t_d2h = wall([&] {
      CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
      CK(hipStreamSynchronize(s2));
    });
    const double t_both = wall([&] {
      CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1));
      CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
      CK(hipStreamSynchronize(s1));
      CK(hipStreamSynchronize(s2));
    });
    printf("copy H2D %.1f GB/s  D2H %.1f GB/s  H2D+D2H together %.1f GB/s each way\n",
           bytes / t_h2d / 1e9, bytes / t_d2h / 1e9, bytes / t_both / 1e9);
  }
  uint4 *dh = nullptr, *sink;
  CK(hipHostGetDevicePointer((void **)&dh, h, 0));
  CK(hipMalloc((void **)&sink, 4096ull * 256 * sizeof(uint4)));
  int cus = 256;
  {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    cus = p.multiProcessorCount;
  }
  for (int bpc : {2, 4, 8}) {
    run_kernel<kRd>("rd", dh, tiles, sink, cus * bpc);
    run_kernel<kWr>("wr", dh, tiles, sink, cus * bpc);
    run_kernel<kRmw>("rmw", dh, tiles, sink, cus * bpc);
  }
  CK(hipHostFree(h));
  CK(hipHostFree(h2));
  CK(hipFree(d));
  CK(hipFree(d2));
  CK(hipFree(sink));
  return 0;
}
