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
            kSide = 6, kSideNoRow = 7, kPf = 8 };
// kPf: kRow64 with the per-packet side streams chosen by SIDE bits, the
// loads prefetched with the next tile's frames as the classify kernel does:
enum Side { sIn16 = 1,    // two u16 loads (len, in_dev)
            sIn32 = 2,    // one u32 descriptor load (len | in_dev << 16)
            sOut16 = 4,   // u16 out-port store
            sOut32 = 8,   // u32 descriptor store in place (len | out << 16)
            sLog = 16,    // u32 log store
            sOutWT = 32, sLogWT = 64,    // those stores write-through (sc1)
            sOutNT = 128, sLogNT = 256 };  // those stores non-temporal
__device__ __forceinline__ void st16(uint16_t *p, uint16_t v, int pol) {
  if (pol == 1) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 2, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b16(v, rs, 0, 0, 16);
  } else if (pol == 2) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}
__device__ __forceinline__ void st32(uint32_t *p, uint32_t v, int pol) {
  if (pol == 1) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 4, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(v, rs, 0, 0, 16);
  } else if (pol == 2) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}
// kSide: kRow64 plus the classify kernel's side streams per slot: two u16
// inputs (len, in_dev), one u16 output (out port) and one u32 log entry.
// kSideNoRow: the same without the row.
__device__ uint16_t *g_len, *g_dev, *g_out;
__device__ uint32_t *g_log, *g_desc;

template <int MODE, int DEPTH, int BPC, int SIDE = 0>
__global__ __launch_bounds__(256, BPC) void stream(uint4 *__restrict__ buf,
                                                   uint4 *__restrict__ dst,
                                                   const uint4 *__restrict__ table,
                                                   uint32_t rows_mask, uint32_t tiles,
                                                   uint4 *__restrict__ sink, int order) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // order 0: each block a contiguous range of tiles, its waves interleaved;
  // order 1/2: grid-stride over all waves (2: one tile per wave, grid = tiles / 4)
  const uint32_t per_b = (tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t t0 = order ? blockIdx.x * 4 : blockIdx.x * per_b;
  const uint32_t t1 = order ? tiles : min(tiles, t0 + per_b);
  const uint32_t TS = order ? gridDim.x * 4 : 4;
  uint4 r[DEPTH][4];
  uint32_t sd[DEPTH] = {};
  auto side_ld = [&](uint32_t tt) -> uint32_t {
    uint32_t x = 0;
    if (SIDE & sIn16) x = g_len[(size_t)tt * 64 + lane] + (g_dev[(size_t)tt * 64 + lane] << 16);
    if (SIDE & sIn32) x = g_desc[(size_t)tt * 64 + lane];
    return x;
  };
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint32_t tile = t0 + wv;
#pragma unroll
  for (int d = 0; d < DEPTH; d++) {
    const uint32_t tt = tile + TS * d;
    if (tt < t1) {
#pragma unroll
      for (int j = 0; j < 4; j++) r[d][j] = buf[(size_t)tt * 256 + 64 * j + lane];
      if (MODE == kPf) sd[d] = side_ld(tt);
    }
  }
  for (; tile < t1; tile += TS * DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      const uint32_t tt = tile + TS * d;
      if (tt >= t1) break;
      uint4 v[4];
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = r[d][j];
      const uint32_t nt = tt + TS * DEPTH;
      uint32_t side = 0;
      if (MODE == kSide || MODE == kSideNoRow) side = g_len[(size_t)tt * 64 + lane] + g_dev[(size_t)tt * 64 + lane];
      if (MODE == kPf) side = sd[d];
      if (MODE == kRow64 || MODE == kRow48 || MODE == kSide || MODE == kPf) {
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
        if (MODE == kPf) sd[d] = side_ld(nt);
      }
      if (MODE == kPf) {
        if (SIDE & sOut16)
          st16(g_out + (size_t)tt * 64 + lane, (uint16_t)(side + v[0].x),
               (SIDE & sOutWT) ? 1 : (SIDE & sOutNT) ? 2 : 0);
        if (SIDE & sOut32) g_desc[(size_t)tt * 64 + lane] = (side & 0xFFFF) | ((side + v[0].x) << 16);
        if (SIDE & sLog)
          st32(g_log + (size_t)tt * 64 + lane, side ^ v[1].y,
               (SIDE & sLogWT) ? 1 : (SIDE & sLogNT) ? 2 : 0);
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
          else if (MODE == kRmw64 || MODE == kRow64 || MODE == kSide || MODE == kSideNoRow || MODE == kPf ||
                   (c & 3) != 3)
            buf[(size_t)tt * 256 + c] = v[j];
        }
      }
    }
  }
  if ((acc.x ^ acc.y) == 0x12345678u) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

// Tile schedules for the full classify shape (FULL: row + in16 + out16 +
// log) or rmw64 alone. SCHED 0: static contiguous block ranges; 1: static
// grid-stride over waves; 2: dynamic, each wave claims its next tile from one
// counter (atomicAdd); 3: dynamic, per-XCD-slot counters (block b uses
// counter b % 8 over tiles = 8 k + b % 8). PF: the next tile's loads are
// issued before the current tile is processed.
__device__ uint32_t g_ctr[8 * 64];
template <int SCHED, bool PF, bool FULL>
__global__ __launch_bounds__(256, 4) void stream2(uint4 *__restrict__ buf,
                                                  const uint4 *__restrict__ table,
                                                  uint32_t rows_mask, uint32_t tiles) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t per_b = (tiles + gridDim.x - 1) / gridDim.x;
  const uint32_t x = blockIdx.x & 7;
  uint32_t k = 0;  // static schedules: this wave's k-th tile
  auto next = [&]() -> uint32_t {
    uint32_t t;
    if (SCHED == 0) {
      t = blockIdx.x * per_b + wv + 4 * k;
      if (t >= min(tiles, blockIdx.x * per_b + per_b)) t = ~0u;
    } else if (SCHED == 1) {
      t = (blockIdx.x + gridDim.x * k) * 4 + wv;
    } else if (SCHED == 2) {
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(&g_ctr[0], 1u);
      t = __shfl(c, 0);
    } else {
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(&g_ctr[x * 64], 1u);
      t = __shfl(c, 0) * 8 + x;
    }
    k++;
    return t < tiles ? t : ~0u;
  };
  uint4 r[4];
  uint32_t sd = 0;
  auto load = [&](uint32_t t) {
#pragma unroll
    for (int j = 0; j < 4; j++) r[j] = buf[(size_t)t * 256 + 64 * j + lane];
    if (FULL) sd = g_len[(size_t)t * 64 + lane] + (g_dev[(size_t)t * 64 + lane] << 16);
  };
  uint32_t t = next();
  if (PF && t != ~0u) load(t);
  while (t != ~0u) {
    if (!PF) load(t);
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = r[j];
    const uint32_t side = sd;
    const uint32_t nt = next();
    if (FULL) {
      uint4 q[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t row = __shfl(v[j].y, lane & ~3u) & rows_mask;
        q[j] = table[(size_t)row * 4 + (lane & 3)];
      }
      if (PF && nt != ~0u) load(nt);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        v[j].x ^= q[j].x;
        v[j].z += q[j].z;
      }
      g_out[(size_t)t * 64 + lane] = (uint16_t)(side + v[0].x);
      g_log[(size_t)t * 64 + lane] = side ^ v[1].y;
    } else if (PF && nt != ~0u) {
      load(nt);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j].w += 1;
      buf[(size_t)t * 256 + 64 * j + lane] = v[j];
    }
    t = nt;
  }
}
template <int SCHED, bool PF, bool FULL>
static void run2(const char *name, uint4 *buf, const uint4 *table, uint32_t rows_mask,
                 uint32_t tiles, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t *ctr;
  CK(hipGetSymbolAddress((void **)&ctr, HIP_SYMBOL(g_ctr)));
  float best = 1e30f, sum = 0.f;
  for (int rep = 0; rep < 8; rep++) {
    CK(hipMemset(ctr, 0, sizeof(uint32_t) * 8 * 64));
    CK(hipEventRecord(e0));
    stream2<SCHED, PF, FULL><<<cus * 4, 256>>>(buf, table, rows_mask, tiles);
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
  printf("%-20s sched %d pf %d : %7.3f ms (mean %7.3f)  %6.2f Gslots/s\n", name, SCHED,
         (int)PF, best, sum / 7, slots / best / 1e6);
}

// One tile per wave, grid over all tiles (dispatch order), the full shape
// plus the per-block costs a classify kernel in that shape would carry:
// TLOAD 1/2: a 4 KB / 15 KB lookup table staged into LDS per block (and
// four lookups per lane); BINS 1: the log entries go to (slice, bin) runs
// reserved by one returning atomicAdd per wave on a global cursor
// (slice = 256 tiles, bin = tile % 256, the bench's pattern).
__device__ uint32_t *g_tab, *g_cur, *g_ent;
template <int TLOAD, int BINS>
__global__ __launch_bounds__(256, 4) void stream3(uint4 *__restrict__ buf,
                                                  const uint4 *__restrict__ table,
                                                  uint32_t rows_mask, uint32_t tiles) {
  __shared__ uint32_t T[TLOAD ? (TLOAD == 1 ? 1024 : 15 * 256) : 1];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t t = blockIdx.x * 4 + wv;
  uint4 r[4];
#pragma unroll
  for (int j = 0; j < 4; j++) r[j] = buf[(size_t)t * 256 + 64 * j + lane];
  const uint32_t side = g_len[(size_t)t * 64 + lane] + (g_dev[(size_t)t * 64 + lane] << 16);
  uint32_t h = 0;
  if (TLOAD) {
    const uint32_t nw = TLOAD == 1 ? 1024 : 15 * 256;
    for (uint32_t i = threadIdx.x * 4; i < nw; i += 1024)
      *reinterpret_cast<uint4 *>(&T[i]) = *reinterpret_cast<const uint4 *>(&g_tab[i]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++) h ^= T[(r[j].x >> (8 * j)) & (nw - 1)];
  }
  uint4 v[4];
#pragma unroll
  for (int j = 0; j < 4; j++) v[j] = r[j];
  uint4 q[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t row = (__shfl(v[j].y, lane & ~3u) ^ (h & 1)) & rows_mask;
    q[j] = table[(size_t)row * 4 + (lane & 3)];
  }
  uint32_t base = 0;
  if (BINS) {
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&g_cur[t], 64u);  // slice (t >> 8), bin (t & 255)
    base = __shfl(c, 0);
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    v[j].x ^= q[j].x;
    v[j].z += q[j].z;
  }
  g_out[(size_t)t * 64 + lane] = (uint16_t)(side + v[0].x);
  if (BINS)
    g_ent[(size_t)t * 128 + (base & 127) + lane] = side ^ v[1].y;
  else
    g_log[(size_t)t * 64 + lane] = side ^ v[1].y;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    v[j].w += 1;
    buf[(size_t)t * 256 + 64 * j + lane] = v[j];
  }
}
template <int TLOAD, int BINS>
static void run3(const char *name, uint4 *buf, const uint4 *table, uint32_t rows_mask,
                 uint32_t tiles) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t *cur;
  CK(hipMemcpyFromSymbol(&cur, HIP_SYMBOL(g_cur), sizeof(cur)));
  float best = 1e30f, sum = 0.f;
  for (int rep = 0; rep < 8; rep++) {
    CK(hipMemset(cur, 0, tiles * 4));
    CK(hipEventRecord(e0));
    stream3<TLOAD, BINS><<<tiles / 4, 256>>>(buf, table, rows_mask, tiles);
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
  printf("%-20s tload %d bins %d : %7.3f ms (mean %7.3f)  %6.2f Gslots/s\n", name, TLOAD,
         BINS, best, sum / 7, slots / best / 1e6);
}

// TPW tiles per wave: block b owns tiles [4 TPW b, 4 TPW (b + 1)), wave w
// the tiles 4 TPW b + w + 4 k, the next one prefetched (PF); the block
// stages a 15 KB table in LDS (TLOAD) and reserves its log runs by atomics.
template <int TPW, bool PF, bool TLOAD>
__global__ __launch_bounds__(256, 4) void stream4(uint4 *__restrict__ buf,
                                                  const uint4 *__restrict__ table,
                                                  uint32_t rows_mask, uint32_t tiles) {
  __shared__ uint32_t T[15 * 256];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t tb0 = blockIdx.x * 4 * TPW + wv;
  uint4 r[4];
  uint32_t sd = 0;
  auto load = [&](uint32_t t) {
#pragma unroll
    for (int j = 0; j < 4; j++) r[j] = buf[(size_t)t * 256 + 64 * j + lane];
    sd = g_len[(size_t)t * 64 + lane] + (g_dev[(size_t)t * 64 + lane] << 16);
  };
  if (PF) load(tb0);
  if (TLOAD) {
    for (uint32_t i = threadIdx.x * 4; i < 15 * 256; i += 1024)
      *reinterpret_cast<uint4 *>(&T[i]) = *reinterpret_cast<const uint4 *>(&g_tab[i]);
    __syncthreads();
  }
  for (int k = 0; k < TPW; k++) {
    const uint32_t t = tb0 + 4 * k;
    if (!PF) load(t);
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = r[j];
    const uint32_t side = sd;
    uint32_t h = 0;
    if (TLOAD) {
#pragma unroll
      for (int j = 0; j < 4; j++) h ^= T[(v[j].x >> (8 * j)) & 4095];
    }
    uint4 q[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t row = (__shfl(v[j].y, lane & ~3u) ^ (h & 1)) & rows_mask;
      q[j] = table[(size_t)row * 4 + (lane & 3)];
    }
    if (PF && k + 1 < TPW) load(t + 4);
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&g_cur[t], 64u);
    const uint32_t base = __shfl(c, 0);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j].x ^= q[j].x;
      v[j].z += q[j].z;
    }
    g_out[(size_t)t * 64 + lane] = (uint16_t)(side + v[0].x);
    g_ent[(size_t)t * 128 + (base & 127) + lane] = side ^ v[1].y;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j].w += 1;
      buf[(size_t)t * 256 + 64 * j + lane] = v[j];
    }
  }
}
template <int TPW, bool PF, bool TLOAD>
static void run4(uint4 *buf, const uint4 *table, uint32_t rows_mask, uint32_t tiles) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t *cur;
  CK(hipMemcpyFromSymbol(&cur, HIP_SYMBOL(g_cur), sizeof(cur)));
  float best = 1e30f, sum = 0.f;
  for (int rep = 0; rep < 8; rep++) {
    CK(hipMemset(cur, 0, tiles * 4));
    CK(hipEventRecord(e0));
    stream4<TPW, PF, TLOAD><<<tiles / 4 / TPW, 256>>>(buf, table, rows_mask, tiles);
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
  printf("tpw %2d pf %d tload %d : %7.3f ms (mean %7.3f)  %6.2f Gslots/s\n", TPW, (int)PF,
         (int)TLOAD, best, sum / 7, slots / best / 1e6);
}

// The guide's float4 copy shape: one 16-byte chunk per thread, a grid over
// the whole buffer (in place: rmw).
template <bool INPLACE>
__global__ __launch_bounds__(256) void simple(uint4 *__restrict__ buf, uint4 *__restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  uint4 v = buf[i];
  v.w += 1;
  (INPLACE ? buf : dst)[i] = v;
}
template <bool INPLACE>
static void run_simple(const char *name, uint4 *buf, uint4 *dst, uint32_t tiles) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 8; rep++) {
    CK(hipEventRecord(e0));
    simple<INPLACE><<<tiles, 256>>>(buf, dst);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double slots = (double)tiles * 64;
  printf("%-20s    : %7.3f ms  %6.2f Gslots/s  %5.2f TB/s streamed\n", name, best,
         slots / best / 1e6, slots * 128 / best / 1e9);
}

template <int MODE, int DEPTH, int BPC, int SIDE = 0>
static void run(const char *name, uint4 *buf, uint4 *dst, const uint4 *table,
                uint32_t rows_mask, uint32_t tiles, uint4 *sink, int cus, int order = 0) {
  const int blocks = order == 2 ? (int)(tiles / 4) : cus * BPC;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f, sum = 0.f;
  const int reps = 8;
  for (int rep = 0; rep < reps; rep++) {
    CK(hipEventRecord(e0));
    stream<MODE, DEPTH, BPC, SIDE><<<blocks, 256>>>(buf, dst, table, rows_mask, tiles, sink, order);
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
  printf("%-20s o%d depth %d bpc %d : %7.3f ms (mean %7.3f)  %6.2f Gslots/s  %5.2f TB/s streamed\n",
         name, order, DEPTH, BPC, best, sum / (reps - 1), slots / best / 1e6,
         slots * (64 + wr) / best / 1e9);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
  const bool side_only = argc > 1 && argv[1][0] == 's';  // only the side-stream variants
  const bool order_only = argc > 1 && argv[1][0] == 'o';  // tile orders
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
    uint32_t *lg, *ds;
    CK(hipMalloc(&l, slots * 2));
    CK(hipMalloc(&d, slots * 2));
    CK(hipMalloc(&o, slots * 2));
    CK(hipMalloc(&lg, slots * 4));
    CK(hipMalloc(&ds, slots * 4));
    CK(hipMemset(ds, 0, slots * 4));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_desc), &ds, sizeof(ds)));
    CK(hipMemset(l, 0, slots * 2));
    CK(hipMemset(d, 0, slots * 2));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_len), &l, sizeof(l)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_dev), &d, sizeof(d)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), &o, sizeof(o)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_log), &lg, sizeof(lg)));
  }
  if (argc > 1 && argv[1][0] == 'r') {  // uniformly random rows (SURVEY §8(d) uniform order)
    // slot word 1 = splitmix64(slot) (bits unrelated between neighbours), the
    // row index the kRow64 / kSide shapes fetch: the memory shape of vignat
    // under uniform packet order, one random 64-byte row of a 32 MB table per
    // slot, against the stride-spread index of the default runs
    for (int rep = 0; rep < 2; rep++) {
      for (int mode = 0; mode < 2; mode++) {
        uint32_t *h = (uint32_t *)malloc(bytes);
        for (size_t i = 0; i < bytes / 4; i++) {
          uint64_t z = (i >> 4) + (mode ? 0x9E3779B97F4A7C15ull : 0);
          if (mode) {
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
          }
          h[i] = mode ? (uint32_t)z : (uint32_t)(i * 2654435761u);
        }
        CK(hipMemcpy(buf, h, bytes, hipMemcpyHostToDevice));
        free(h);
        printf("row index: %s\n", mode ? "splitmix64 (uniform)" : "stride spread (default)");
        run<kRow64, 1, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus);
        run<kSide, 1, 4>("row+side", buf, dst, table, rmask, tiles, sink, cus);
      }
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'g') {  // one tile per wave + per-block costs
    uint32_t *tb, *cu, *en;
    CK(hipMalloc(&tb, 15 * 256 * 4));
    CK(hipMemset(tb, 1, 15 * 256 * 4));
    CK(hipMalloc(&cu, tiles * 4));
    CK(hipMalloc(&en, (size_t)tiles * 128 * 4));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &tb, sizeof(tb)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_cur), &cu, sizeof(cu)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ent), &en, sizeof(en)));
    for (int rep = 0; rep < 2; rep++) {
      run<kPf, 1, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus, 2);
      run3<0, 0>("o2", buf, table, rmask, tiles);
      run3<1, 0>("o2", buf, table, rmask, tiles);
      run3<2, 0>("o2", buf, table, rmask, tiles);
      run3<0, 1>("o2", buf, table, rmask, tiles);
      run3<1, 1>("o2", buf, table, rmask, tiles);
      run3<2, 1>("o2", buf, table, rmask, tiles);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus, 0);
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 't') {  // tiles per wave
    uint32_t *tb, *cu, *en;
    CK(hipMalloc(&tb, 15 * 256 * 4));
    CK(hipMemset(tb, 1, 15 * 256 * 4));
    CK(hipMalloc(&cu, tiles * 4));
    CK(hipMalloc(&en, (size_t)tiles * 128 * 4));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &tb, sizeof(tb)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_cur), &cu, sizeof(cu)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ent), &en, sizeof(en)));
    for (int rep = 0; rep < 2; rep++) {
      run4<1, false, true>(buf, table, rmask, tiles);
      run4<1, false, false>(buf, table, rmask, tiles);
      run4<2, true, true>(buf, table, rmask, tiles);
      run4<2, false, true>(buf, table, rmask, tiles);
      run4<4, true, true>(buf, table, rmask, tiles);
      run4<4, false, true>(buf, table, rmask, tiles);
      run4<8, true, true>(buf, table, rmask, tiles);
      run4<16, true, true>(buf, table, rmask, tiles);
      run4<64, true, true>(buf, table, rmask, tiles);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus, 0);
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'q') {  // schedules
    for (int rep = 0; rep < 2; rep++) {
      run2<0, true, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<0, false, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<1, true, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<1, false, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<2, true, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<2, false, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<3, true, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<3, false, false>("rmw64", buf, table, rmask, tiles, cus);
      run2<0, true, true>("full", buf, table, rmask, tiles, cus);
      run2<0, false, true>("full", buf, table, rmask, tiles, cus);
      run2<1, true, true>("full", buf, table, rmask, tiles, cus);
      run2<1, false, true>("full", buf, table, rmask, tiles, cus);
      run2<2, true, true>("full", buf, table, rmask, tiles, cus);
      run2<2, false, true>("full", buf, table, rmask, tiles, cus);
      run2<3, true, true>("full", buf, table, rmask, tiles, cus);
      run2<3, false, true>("full", buf, table, rmask, tiles, cus);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus, 2);
    }
    return 0;
  }
  if (order_only) {
    run_simple<false>("simple copy", buf, dst, tiles);
    run_simple<true>("simple rmw", buf, dst, tiles);
    for (int o = 0; o < 3; o++) {
      run<kCopy, 1, 4>("copy", buf, dst, table, rmask, tiles, sink, cus, o);
      run<kRmw64, 1, 4>("rmw64", buf, dst, table, rmask, tiles, sink, cus, o);
      run<kRmw64, 2, 4>("rmw64", buf, dst, table, rmask, tiles, sink, cus, o);
      run<kRmw64, 1, 2>("rmw64", buf, dst, table, rmask, tiles, sink, cus, o);
      run<kRow64, 1, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus, o);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus, o);
      run<kPf, 2, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus, o);
    }
    return 0;
  }
  if (side_only) {
    for (int rep = 0; rep < 2; rep++) {
      run<kRow64, 1, 4>("rmw64+row", buf, dst, table, rmask, tiles, sink, cus);
      run<kSide, 1, 4>("row+side", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog>("pf:in16+out16+log", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog | sOutWT | sLogWT>("pf:..+out/log wt", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog | sOutWT>("pf:..+out wt", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog | sLogWT>("pf:..+log wt", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16 | sOut16 | sLog | sOutNT | sLogNT>("pf:..+out/log nt", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16 | sOut16>("pf:in16+out16", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn16>("pf:in16", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sOut16>("pf:out16", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sLog>("pf:log", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn32 | sOut16 | sLog>("pf:in32+out16+log", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn32 | sOut32 | sLog>("pf:desc32rw+log", buf, dst, table, rmask, tiles, sink, cus);
      run<kPf, 1, 4, sIn32 | sOut32>("pf:desc32rw", buf, dst, table, rmask, tiles, sink, cus);
    }
    return 0;
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
