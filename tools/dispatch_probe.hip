// Dispatch-cost probe (measurement tool, not product): what a step of two
// dependent kernels costs the host and the GPU between kernels, launched
// through HIP (<<<>>> on one stream) and through AQL packets written straight
// into an HSA queue of our own (the kernels' code objects as HIP loaded them,
// found through the AMD loader extension), with system- or agent-scope
// packet fences.
// A step: `heavy` (a ~0.4 ms HBM copy, 256 x 1024 threads) then `tiny`
// (writes the step's epoch into host memory); the host spins on the epoch,
// then issues the next step -- the shape of vignat's classify + fold +
// control-block wait.
// Build: hipcc --offload-arch=gfx950 -O2 tools/dispatch_probe.hip
//        -o tools/dispatch_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)
#define HK(x)                                                                \
  do {                                                                       \
    hsa_status_t s_ = (x);                                                   \
    if (s_ != HSA_STATUS_SUCCESS) {                                          \
      fprintf(stderr, "%s:%d hsa status 0x%x\n", __FILE__, __LINE__, s_);     \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

struct HeavyArgs {
  const uint4 *src;
  uint4 *dst;
  uint64_t n;  // uint4 elements
  uint32_t nthreads;
};
struct TinyArgs {
  uint32_t *flag;
  uint32_t epoch;
};

__global__ __launch_bounds__(1024) void heavy(HeavyArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  for (uint64_t i = t; i < a.n; i += a.nthreads) a.dst[i] = a.src[i];
}
__global__ __launch_bounds__(64) void tiny(TinyArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Sym {
  const char *want;
  uint64_t kobj = 0;
  uint32_t karg = 0, group = 0, priv = 0;
};
static hsa_agent_t g_gpu{};
static hsa_status_t find_gpu(hsa_agent_t a, void *) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t sym_cb(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t s, void *d) {
  Sym *w = (Sym *)d;
  hsa_symbol_kind_t k;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &k);
  if (k != HSA_SYMBOL_KIND_KERNEL) return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
  std::string name(len, '\0');
  hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]);
  for (Sym *x = w; x->want; x++) {
    if (name.find(x->want) == std::string::npos) continue;
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &x->kobj);
    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE,
                                   &x->karg);
    hsa_executable_symbol_get_info(
        s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &x->group);
    hsa_executable_symbol_get_info(
        s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &x->priv);
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_ven_amd_loader_1_03_pfn_t g_ld;
static hsa_status_t exec_cb(hsa_executable_t e, void *d) {
  hsa_executable_iterate_agent_symbols(e, g_gpu, sym_cb, d);
  return HSA_STATUS_SUCCESS;
}

struct Q {
  hsa_queue_t *q;
  uint8_t *karg;  // ring of 1 KiB kernarg slots (pinned host memory)
  uint32_t slot = 0;
  hsa_signal_t done;
};

static void dispatch(Q &q, const Sym &k, const void *args, size_t asz, uint32_t blocks,
                     uint32_t wg, hsa_fence_scope_t acq, hsa_fence_scope_t rel, bool sig) {
  uint8_t *ka = q.karg + 1024 * (q.slot++ % 64);
  memcpy(ka, args, asz);
  const uint64_t idx = hsa_queue_add_write_index_relaxed(q.q, 1);
  while (idx - hsa_queue_load_read_index_scacquire(q.q) >= q.q->size) {
  }
  auto *p = (hsa_kernel_dispatch_packet_t *)q.q->base_address + (idx & (q.q->size - 1));
  p->workgroup_size_x = (uint16_t)wg;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->grid_size_x = blocks * wg;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = k.priv;
  p->group_segment_size = k.group;
  p->kernel_object = k.kobj;
  p->kernarg_address = ka;
  p->completion_signal = sig ? q.done : hsa_signal_t{0};
  p->reserved0 = 0;
  p->reserved2 = 0;
  const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                       (1 << HSA_PACKET_HEADER_BARRIER) |
                       (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                       (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n((uint32_t *)p, (uint32_t)hdr | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  hsa_signal_store_relaxed(q.q->doorbell_signal, (hsa_signal_value_t)idx);
}

int main(int argc, char **argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 40;
  const uint64_t bytes = 1ull << 30;
  uint4 *src, *dst;
  uint32_t *flag;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMemset(src, 1, bytes));
  CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  *flag = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  HeavyArgs ha{src, dst, bytes / 16, 256 * 1024};
  // (the first launches load the code objects)
  heavy<<<256, 1024, 0, s>>>(ha);
  tiny<<<1, 64, 0, s>>>(TinyArgs{flag, 0});
  CK(hipStreamSynchronize(s));

  // -- HIP: <<<>>> on one stream
  double l_h = 0, l_t = 0;
  uint32_t ep = 0;
  for (int pass = 0; pass < 2; pass++) {
    l_h = l_t = 0;
    const double t0 = now_us();
    for (int i = 0; i < steps; i++) {
      ++ep;
      const double a = now_us();
      heavy<<<256, 1024, 0, s>>>(ha);
      const double b = now_us();
      tiny<<<1, 64, 0, s>>>(TinyArgs{flag, ep});
      const double c = now_us();
      l_h += b - a;
      l_t += c - b;
      while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != ep) {
      }
    }
    const double t1 = now_us();
    CK(hipStreamSynchronize(s));
    if (pass)
      printf("{\"path\": \"hip\", \"us_per_step\": %.2f, \"launch_heavy_us\": %.2f, "
             "\"launch_tiny_us\": %.2f}\n",
             (t1 - t0) / steps, l_h / steps, l_t / steps);
  }
  // heavy alone, back to back on the stream (no host wait): its own time
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < steps; i++) heavy<<<256, 1024, 0, s>>>(ha);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"path\": \"hip heavy back to back\", \"us_per_kernel\": %.2f}\n",
           ms * 1e3 / steps);
  }

  // -- HSA: our own queue, AQL packets written here
  HK(hsa_init());
  HK(hsa_iterate_agents(find_gpu, nullptr));
  HK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(g_ld), &g_ld));
  Sym syms[3] = {{"5heavy"}, {"4tiny"}, {nullptr}};
  HK(g_ld.hsa_ven_amd_loader_iterate_executables(exec_cb, syms));
  if (!syms[0].kobj || !syms[1].kobj) {
    fprintf(stderr, "kernel objects not found\n");
    return 1;
  }
  printf("{\"heavy_kernarg\": %u, \"tiny_kernarg\": %u, \"heavy_group\": %u}\n", syms[0].karg,
         syms[1].karg, syms[0].group);
  Q q;
  HK(hsa_queue_create(g_gpu, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX,
                      UINT32_MAX, &q.q));
  CK(hipHostMalloc((void **)&q.karg, 1024 * 64, hipHostMallocCoherent | hipHostMallocMapped));
  memset(q.karg, 0, 1024 * 64);
  HK(hsa_signal_create(1, 0, nullptr, &q.done));
  const hsa_fence_scope_t SYS = HSA_FENCE_SCOPE_SYSTEM, AG = HSA_FENCE_SCOPE_AGENT;
  struct Mode {
    const char *name;
    hsa_fence_scope_t acq, rel;
  } modes[2] = {{"hsa system fences", SYS, SYS}, {"hsa agent fences", AG, AG}};
  for (const Mode &m : modes) {
    for (int pass = 0; pass < 2; pass++) {
      l_h = l_t = 0;
      hsa_signal_store_relaxed(q.done, 1);
      const double t0 = now_us();
      for (int i = 0; i < steps; i++) {
        ++ep;
        const double a = now_us();
        dispatch(q, syms[0], &ha, sizeof(ha), 256, 1024, m.acq, m.rel, false);
        const double b = now_us();
        const TinyArgs ta{flag, ep};
        dispatch(q, syms[1], &ta, sizeof(ta), 1, 64, m.acq, m.rel, i == steps - 1);
        const double c = now_us();
        l_h += b - a;
        l_t += c - b;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != ep) {
        }
      }
      const double t1 = now_us();
      hsa_signal_wait_scacquire(q.done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                HSA_WAIT_STATE_ACTIVE);
      if (pass)
        printf("{\"path\": \"%s\", \"us_per_step\": %.2f, \"launch_heavy_us\": %.2f, "
               "\"launch_tiny_us\": %.2f}\n",
               m.name, (t1 - t0) / steps, l_h / steps, l_t / steps);
    }
  }
  hsa_queue_destroy(q.q);
  hsa_signal_destroy(q.done);
  return 0;
}
