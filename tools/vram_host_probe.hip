// Can the host write device memory directly (large BAR)? Allocates
// fine-grained device memory, prints what hipPointerGetAttributes says about
// host access, and only if it names a host pointer writes through it and
// checks the words from a kernel. Diagnostic for vp_process_one's mailbox
// (DESIGN.md §5.3).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void sum_words(const unsigned *p, unsigned n, unsigned *out) {
  unsigned s = 0;
  for (unsigned i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  atomicAdd(out, s);
}

int main() {
  void *d = nullptr;
  hipError_t e = hipExtMallocWithFlags(&d, 4096, hipDeviceMallocFinegrained);
  printf("hipExtMallocWithFlags(fine-grained): %s %p\n", hipGetErrorString(e), d);
  if (e != hipSuccess) return 1;
  hipPointerAttribute_t a{};
  e = hipPointerGetAttributes(&a, d);
  printf("attributes: %s type %d device %p host %p isManaged %d\n", hipGetErrorString(e),
         (int)a.type, a.devicePointer, a.hostPointer, (int)a.isManaged);
  int lb = 0;
  hipDeviceGetAttribute(&lb, hipDeviceAttributeHostNativeAtomicSupported, 0);
  printf("host native atomics: %d\n", lb);
  if (!a.hostPointer) {
    printf("no host pointer: not host-accessible\n");
    return 0;
  }
  unsigned *h = (unsigned *)a.hostPointer;
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0; i < 1024; i++) h[i] = i;
  auto t1 = std::chrono::steady_clock::now();
  unsigned *out = nullptr;
  hipMalloc(&out, 4);
  hipMemset(out, 0, 4);
  sum_words<<<1, 256>>>((const unsigned *)d, 1024, out);
  unsigned got = 0;
  hipMemcpy(&got, out, 4, hipMemcpyDeviceToHost);
  printf("host wrote 4 KiB in %.2f us; kernel sum %u (expect %u)\n",
         std::chrono::duration<double, std::micro>(t1 - t0).count(), got, 1023u * 1024u / 2u);
  volatile unsigned x = h[5];
  printf("host read back %u\n", x);
  return 0;
}
