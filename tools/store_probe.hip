// store_probe.hip -- diagnostics: HBM store rate of the trace write patterns a fill kernel can
// use, on the real 2^18 x 12-round trace shape (11 u32 columns, 5,220 rows per instance).
//   tile  : 1024-row tiles dealt round-robin to persistent workgroups (the fill kernel's order)
//   wave  : every wave owns whole instances (dynamic: a global counter), writing an instance's
//           rows in steps of STEP quads (52 = one half-round of 4 G's) from row 0 to its end
//   wavesI: the same with a static interleave (wave w takes instances w, w + W, ...)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void __launch_bounds__(256) tile_store(uint32_t* adv, uint64_t total_rows, uint64_t n_tiles) {
  const uint64_t total_quads = total_rows >> 2;
  for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const uint64_t gq = t * 256 + threadIdx.x;
    if (gq >= total_quads) continue;
    const u32x4 v = {(uint32_t)gq, 1u, 2u, 3u};
#pragma unroll
    for (int c = 0; c < 11; c++)
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + 4 * gq));
  }
}

template <int STEP, bool DYN>
__global__ void __launch_bounds__(256) wave_store(uint32_t* adv, uint64_t total_rows, uint32_t n,
                                                  uint32_t rows_per, unsigned* counter) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  const uint32_t quads = rows_per / 4;
  for (uint32_t k = 0;; k++) {
    uint32_t i;
    if (DYN) {
      uint32_t v = 0;
      if (lane == 0) v = atomicAdd(counter, 1u);
      i = __builtin_amdgcn_readfirstlane(v);
    } else {
      i = wid + k * nw;
    }
    if (i >= n) break;
    const uint64_t o = (uint64_t)i * rows_per;
    for (uint32_t q0 = 0; q0 < quads; q0 += STEP) {
      const uint32_t q = q0 + lane;
      if (lane < STEP && q < quads) {
        const u32x4 v = {q, i, 2u, 3u};
#pragma unroll
        for (int c = 0; c < 11; c++)
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + o + 4 * q));
      }
    }
  }
}

// wave-granular round robin: wave w writes tiles w, w + W, ... of STEP quads each (rows 4 STEP t
// onwards): the order a wave-per-tile fused kernel writes in
template <int STEP>
__global__ void __launch_bounds__(256) wave_rr_store(uint32_t* adv, uint64_t total_rows) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    if (lane < STEP && q < total_quads) {
      const u32x4 v = {(uint32_t)q, 1u, 2u, 3u};
#pragma unroll
      for (int c = 0; c < 11; c++)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + 4 * q));
    }
  }
}

// wave_rr_store with the columns `stride` words apart (stride >= total_rows): column padding
template <int STEP>
__global__ void __launch_bounds__(256) wave_rr_pad(uint32_t* adv, uint64_t total_rows, uint64_t stride, int work) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  uint32_t h = lane;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    h ^= (uint32_t)q;
    for (int k = 0; k < work; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
    if (lane < STEP && q < total_quads) {
#pragma unroll
      for (int c = 0; c < 11; c++)
        __builtin_nontemporal_store(u32x4{h + c, h ^ c, h * c, h - c},
                                    reinterpret_cast<u32x4*>(adv + (uint64_t)c * stride + 4 * q));
    }
  }
}

// the same order with per-tile work in front of the stores: `work` rounds of a dependent
// integer hash per lane (~4 VALU each), optionally staged through LDS and read back (STAGE), and
// stored with raw buffer stores (BUF) instead of global stores
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ void probe_buffer_store(i32x4 data, i32x4 rsrc, int voffset, int soffset,
                                   int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
template <int STEP, bool STAGE, bool BUF, int POL = 2, bool XCD = false>
__global__ void __launch_bounds__(256) wave_rr_work(uint32_t* adv, uint64_t total_rows, int work) {
  __shared__ __attribute__((aligned(16))) uint32_t L[4 * 11 * 256];
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t* S = L + (threadIdx.x >> 6) * 11 * 256;
  // XCD: the fused kernel's deal (workgroups go to the 8 XCDs round-robin; XCD x takes the x-th
  // eighth of every round as one contiguous run, so neighbouring tiles share an L2)
  const uint64_t bx = XCD ? (uint64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
  const uint64_t wid = bx * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    uint32_t h = (uint32_t)q;
    for (int k = 0; k < work; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
    u32x4 v[11];
#pragma unroll
    for (int c = 0; c < 11; c++) v[c] = u32x4{h + c, h ^ c, h * c, h - c};
    if (STAGE) {
#pragma unroll
      for (int c = 0; c < 11; c++) *reinterpret_cast<u32x4*>(S + c * 256 + 4 * lane) = v[c];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = 0; c < 11; c++) v[c] = *reinterpret_cast<const u32x4*>(S + c * 256 + 4 * lane);
    }
    const uint32_t nq = (uint32_t)(total_quads - t * STEP < STEP ? total_quads - t * STEP : STEP);
#pragma unroll
    for (int c = 0; c < 11; c++) {
      uint32_t* base = adv + (uint64_t)c * total_rows + 4 * t * STEP;
      if (BUF) {
        const uint64_t a = reinterpret_cast<uint64_t>(base);
        const i32x4 rsrc = {(int32_t)(uint32_t)a, (int32_t)(uint32_t)(a >> 32), (int32_t)(nq * 16u), 0x00020000};
        probe_buffer_store(i32x4{(int32_t)v[c].x, (int32_t)v[c].y, (int32_t)v[c].z, (int32_t)v[c].w}, rsrc, (int)(16 * lane), 0, POL);
      } else if (lane < nq) {
        __builtin_nontemporal_store(v[c], reinterpret_cast<u32x4*>(base + 4 * lane));
      }
    }
    if (STAGE) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// the fused kernel's 52-quad tiles with the lines they share with a neighbouring tile (a partial
// 128-byte line at each end) stored non-temporal and the whole lines with the default policy:
// two buffer stores per column, every lane in both, each lane's 16 bytes kept in range by exactly
// one of them (the other's offset points past the range and is dropped)
template <int STEP, bool XCD>
__global__ void __launch_bounds__(256) wave_rr_mixed(uint32_t* adv, uint64_t total_rows, int work) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t bx = XCD ? (uint64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
  const uint64_t wid = bx * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    uint32_t h = (uint32_t)q;
    for (int k = 0; k < work; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
    const uint32_t nq = (uint32_t)(total_quads - t * STEP < STEP ? total_quads - t * STEP : STEP);
#pragma unroll
    for (int c = 0; c < 11; c++) {
      uint32_t* base = adv + (uint64_t)c * total_rows + 4 * t * STEP;
      const uint64_t a = reinterpret_cast<uint64_t>(base);
      const uint32_t lo = (uint32_t)((128 - (a & 127)) & 127);          // bytes before the first whole line
      const uint32_t hi = nq * 16u - (uint32_t)((a + nq * 16u) & 127);  // bytes up to the last whole line
      const uint32_t off = 16 * lane;
      const bool whole = off >= lo && off + 16 <= hi;
      const i32x4 rsrc = {(int32_t)(uint32_t)a, (int32_t)(uint32_t)(a >> 32), (int32_t)(nq * 16u), 0x00020000};
      const i32x4 v = {(int32_t)(h + c), (int32_t)(h ^ c), (int32_t)(h * c), (int32_t)(h - c)};
      probe_buffer_store(v, rsrc, whole ? (int)off : 0x7ffffff0, 0, 0);
      probe_buffer_store(v, rsrc, whole ? 0x7ffffff0 : (int)off, 0, 2);
    }
  }
}

// interleaved: the tile's work split into 11 parts, each followed by its column's store;
// STAGGER: wave w of a workgroup first runs (w % 4) / 4 of a tile's work, so the waves of a SIMD
// are out of phase
template <int STEP, bool STAGGER>
__global__ void __launch_bounds__(256) wave_rr_inter(uint32_t* adv, uint64_t total_rows, int work) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  uint32_t h = lane;
  if (STAGGER)
    for (int k = 0; k < (int)(wid & 3) * work / 4; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    h ^= (uint32_t)q;
#pragma unroll
    for (int c = 0; c < 11; c++) {
      for (int k = 0; k < work / 11; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
      if (lane < STEP && q < total_quads)
        __builtin_nontemporal_store(u32x4{h, h + 1, h + 2, h + 3},
                                    reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + 4 * q));
    }
  }
}
template <int STEP>
__global__ void __launch_bounds__(256) wave_rr_stagger(uint32_t* adv, uint64_t total_rows, int work) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  uint32_t h = lane;
  for (int k = 0; k < (int)(wid & 3) * work / 4; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    h ^= (uint32_t)q;
    for (int k = 0; k < work; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
    if (lane < STEP && q < total_quads) {
#pragma unroll
      for (int c = 0; c < 11; c++)
        __builtin_nontemporal_store(u32x4{h + c, h ^ c, h * c, h - c},
                                    reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + 4 * q));
    }
  }
}
template <int STEP>
__global__ void __launch_bounds__(256) wave_rr_nostore(uint32_t* adv, uint64_t total_rows, int work) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  uint32_t h = lane;
  for (uint64_t t = wid; t < n_t; t += nw) {
    h ^= (uint32_t)(t * STEP + lane);
    for (int k = 0; k < work; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
  }
  if (h == 0x12345678u) adv[lane] = h;
}

// the same order with LDS-latency-bound work in front of the stores: `work` dependent LDS round
// trips per tile (write, wait, read a neighbour lane's word), the shape of a tile whose phases
// hand data between lanes through LDS; NOSTORE: the work alone
template <int STEP, bool NOSTORE>
__global__ void __launch_bounds__(256) wave_rr_ldswork(uint32_t* adv, uint64_t total_rows, int work) {
  __shared__ uint32_t L[256];
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t* S = L + (threadIdx.x & ~63u);
  const uint64_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  uint32_t h = lane;
  for (uint64_t t = wid; t < n_t; t += nw) {
    const uint64_t q = t * STEP + lane;
    h ^= (uint32_t)q;
    for (int k = 0; k < work; k++) {
      S[lane] = h;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      h = S[(lane + 7u) & 63u] * 0x9E3779B1u + (uint32_t)k;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    if (!NOSTORE && lane < STEP && q < total_quads) {
#pragma unroll
      for (int c = 0; c < 11; c++)
        __builtin_nontemporal_store(u32x4{h + c, h ^ c, h * c, h - c},
                                    reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + 4 * q));
    }
  }
  if (NOSTORE && h == 0x12345678u) adv[lane] = h;
}


// wave-specialised: NC compute waves per workgroup produce tiles (the work120 hash, 11 columns x
// 52 quads) into NSLOT LDS slots each; one store wave per workgroup drains the slots in tile
// order and issues the 11 column stores. Slot handshake by LDS counters: compute waits for the
// slot's drain count, fills it, bumps its fill count; the store wave waits for the fill count,
// reads the slot into registers, bumps the drain count, stores. NOSTORE: drain without storing.
template <int NC, int NSLOT, bool NOSTORE>
__global__ void __launch_bounds__((NC + 1) * 64) wave_spec(uint32_t* adv, uint64_t total_rows, int work) {
  constexpr int STEP = 52, SW = 11 * STEP * 4;
  __shared__ __attribute__((aligned(16))) uint32_t L[NC * NSLOT * SW];
  __shared__ uint32_t Fc[NC * NSLOT], Dc[NC * NSLOT];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t n_t = (total_quads + STEP - 1) / STEP;
  const uint64_t ncw = (uint64_t)gridDim.x * NC;
  if (threadIdx.x < NC * NSLOT) {
    Fc[threadIdx.x] = 0;
    Dc[threadIdx.x] = 0;
  }
  __syncthreads();
  volatile uint32_t* vF = Fc;
  volatile uint32_t* vD = Dc;
  if (w < NC) {
    uint32_t h = lane;
    uint32_t r = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * NC + w; t < n_t; t += ncw, r++) {
      const uint64_t q = t * STEP + lane;
      h ^= (uint32_t)q;
      for (int k = 0; k < work; k++) h = (h ^ (h >> 7)) * 0x9E3779B1u + (uint32_t)k;
      const uint32_t sl = w * NSLOT + r % NSLOT, seq = r / NSLOT;
      while (__builtin_amdgcn_readfirstlane(vD[sl]) != seq) __builtin_amdgcn_s_sleep(1);
      uint32_t* S = L + sl * SW;
      if (lane < STEP) {
#pragma unroll
        for (int c = 0; c < 11; c++)
          *reinterpret_cast<u32x4*>(S + c * STEP * 4 + 4 * lane) = u32x4{h + c, h ^ c, h * c, h - c};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) vF[sl] = seq + 1;
    }
  } else {
    for (uint32_t r = 0;; r++) {
      const uint64_t t0 = (uint64_t)blockIdx.x * NC + (uint64_t)r * ncw;
      if (t0 >= n_t) break;
      for (int cw = 0; cw < NC; cw++) {
        const uint64_t t = t0 + cw;
        if (t >= n_t) break;
        const uint32_t sl = cw * NSLOT + r % NSLOT, seq = r / NSLOT;
        while (__builtin_amdgcn_readfirstlane(vF[sl]) != seq + 1) __builtin_amdgcn_s_sleep(1);
        const uint32_t* S = L + sl * SW;
        u32x4 v[11];
#pragma unroll
        for (int c = 0; c < 11; c++) v[c] = *reinterpret_cast<const u32x4*>(S + c * STEP * 4 + 4 * (lane < STEP ? lane : 0));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) vD[sl] = seq + 1;
        const uint64_t q = t * STEP + lane;
        if (!NOSTORE && lane < STEP && q < total_quads) {
#pragma unroll
          for (int c = 0; c < 11; c++)
            __builtin_nontemporal_store(v[c], reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + 4 * q));
        } else if (NOSTORE && v[3].x == 0x12345678u && v[5].y == 7u) {
          adv[lane] = v[0].x;
        }
      }
    }
  }
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? atoi(argv[1]) : (1u << 18);
  const uint32_t rows_per = 228 + 416 * 12;
  const uint64_t total = (uint64_t)n * rows_per;
  uint32_t* adv;
  unsigned* ctr;
  CHK(hipMalloc(&adv, total * 11 * 4));
  CHK(hipMalloc(&ctr, 4));
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const double bytes = (double)total * 44;
  auto run = [&](const char* name, auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHK(hipMemset(ctr, 0, 4));
      CHK(hipEventRecord(a));
      launch();
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (rep && ms < best) best = ms;
    }
    printf("{\"pattern\": \"%s\", \"ms\": %.3f, \"TBs\": %.3f}\n", name, best, bytes / best / 1e9);
    fflush(stdout);
  };
  const uint64_t nt = (total + 1023) / 1024;
  if (argc > 2 && argv[2][0] == 's') {  // wave-specialised store waves vs the burst pattern
    for (int work : {0, 120, 240}) {
      char nm[96];
      snprintf(nm, sizeof nm, "work%d_burst", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, false>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "work%d_nostore", work);
      run(nm, [&] { hipLaunchKernelGGL(wave_rr_nostore<52>, dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
#define SPEC(NC, NS, WG)                                                                          \
      snprintf(nm, sizeof nm, "work%d_spec_c%d_s%d_wg%d", work, NC, NS, WG);                     \
      run(nm, [&] { hipLaunchKernelGGL((wave_spec<NC, NS, false>), dim3(cus * WG), dim3((NC + 1) * 64), 0, 0, adv, total, work); }); \
      snprintf(nm, sizeof nm, "work%d_spec_c%d_s%d_wg%d_nostore", work, NC, NS, WG);             \
      run(nm, [&] { hipLaunchKernelGGL((wave_spec<NC, NS, true>), dim3(cus * WG), dim3((NC + 1) * 64), 0, 0, adv, total, work); });
      SPEC(4, 2, 2)
      SPEC(2, 2, 4)
      SPEC(3, 2, 2)
      SPEC(7, 1, 2)
      SPEC(4, 3, 1)
#undef SPEC
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'a') {  // tile alignment: 52-quad (832 B, lines split between
                                        // neighbouring tiles) vs 64-quad (1 KiB, whole lines)
    // tiles, against the fill kernel's 1024-row workgroup tiles, on this box
    for (int w : {8}) {
      char nm[64];
      snprintf(nm, sizeof nm, "tile_rr_%dwg", w);
      run(nm, [&] { hipLaunchKernelGGL(tile_store, dim3(cus * w), dim3(256), 0, 0, adv, total, nt); });
    }
    for (int w : {2, 4, 8}) {
      char nm[64];
      snprintf(nm, sizeof nm, "wave_rr_q52_%dwg", w);
      run(nm, [&] { hipLaunchKernelGGL(wave_rr_store<52>, dim3(cus * w), dim3(256), 0, 0, adv, total); });
      snprintf(nm, sizeof nm, "wave_rr_q64_%dwg", w);
      run(nm, [&] { hipLaunchKernelGGL(wave_rr_store<64>, dim3(cus * w), dim3(256), 0, 0, adv, total); });
    }
    for (int work : {0, 120}) {
      char nm[64];
      snprintf(nm, sizeof nm, "buf_pol0_q52_xcd_work%d_2wg", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, true, 0, true>), dim3(cus * 2), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "buf_pol0_q64_xcd_work%d_2wg", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<64, false, true, 0, true>), dim3(cus * 2), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "buf_mixed_q52_xcd_work%d_2wg", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_mixed<52, true>), dim3(cus * 2), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "buf_pol0_q52_work%d_2wg", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, true, 0>), dim3(cus * 2), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "buf_pol0_q64_work%d_2wg", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<64, false, true, 0>), dim3(cus * 2), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "buf_pol2_q52_work%d_2wg", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, true, 2>), dim3(cus * 2), dim3(256), 0, 0, adv, total, work); });
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'p') {  // column stride padding (words), 2 workgroups per CU
    CHK(hipFree(adv));
    const uint64_t maxpad = 1ull << 20;
    CHK(hipMalloc(&adv, (total + maxpad) * 11 * 4));
    for (int work : {0, 120}) {
      for (uint64_t pad : {0ull, 64ull, 256ull, 1024ull, 4096ull, 16384ull, 65536ull, 3ull * 65536ull + 1024ull,
                           1ull << 20}) {
        for (int w : {2, 4}) {
          char nm[96];
          snprintf(nm, sizeof nm, "pad%llu_work%d_%dwg", (unsigned long long)pad, work, w);
          run(nm, [&] { hipLaunchKernelGGL(wave_rr_pad<52>, dim3(cus * w), dim3(256), 0, 0, adv, total, total + pad, work); });
        }
      }
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'i') {  // instance-per-wave orders vs the half-round round robin
    for (int w : {4, 8}) {
      char nm[64];
      snprintf(nm, sizeof nm, "wave_rr_q52_%dwg", w);
      run(nm, [&] { hipLaunchKernelGGL(wave_rr_store<52>, dim3(cus * w), dim3(256), 0, 0, adv, total); });
      snprintf(nm, sizeof nm, "wave_dyn_step52_%dwg", w);
      run(nm, [&] { hipLaunchKernelGGL((wave_store<52, true>), dim3(cus * w), dim3(256), 0, 0, adv, total, n, rows_per, ctr); });
      snprintf(nm, sizeof nm, "wave_static_step52_%dwg", w);
      run(nm, [&] { hipLaunchKernelGGL((wave_store<52, false>), dim3(cus * w), dim3(256), 0, 0, adv, total, n, rows_per, ctr); });
    }
    return 0;
  }
  if (argc > 2 && argv[2][0] == 'l') {  // LDS-latency work vs VALU work, with and without stores
    for (int work : {120}) {
      char nm[96];
      snprintf(nm, sizeof nm, "work%d_nostore", work);
      run(nm, [&] { hipLaunchKernelGGL(wave_rr_nostore<52>, dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "work%d_burst", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, false>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    }
    for (int work : {4, 8, 16}) {
      char nm[96];
      snprintf(nm, sizeof nm, "ldswork%d_nostore", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_ldswork<52, true>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
      snprintf(nm, sizeof nm, "ldswork%d_burst", work);
      run(nm, [&] { hipLaunchKernelGGL((wave_rr_ldswork<52, false>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    }
    return 0;
  }
  for (int w : {8, 4}) {
    char nm[64];
    snprintf(nm, sizeof nm, "tile_rr_%dwg", w);
    run(nm, [&] { hipLaunchKernelGGL(tile_store, dim3(cus * w), dim3(256), 0, 0, adv, total, nt); });
  }
  for (int work : {120, 240}) {
    char nm[96];
    snprintf(nm, sizeof nm, "work%d_nostore", work);
    run(nm, [&] { hipLaunchKernelGGL(wave_rr_nostore<52>, dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    snprintf(nm, sizeof nm, "work%d_burst", work);
    run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, false>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    snprintf(nm, sizeof nm, "work%d_burst_stagger", work);
    run(nm, [&] { hipLaunchKernelGGL(wave_rr_stagger<52>, dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    snprintf(nm, sizeof nm, "work%d_interleaved", work);
    run(nm, [&] { hipLaunchKernelGGL((wave_rr_inter<52, false>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    snprintf(nm, sizeof nm, "work%d_interleaved_stagger", work);
    run(nm, [&] { hipLaunchKernelGGL((wave_rr_inter<52, true>), dim3(cus * 4), dim3(256), 0, 0, adv, total, work); });
    snprintf(nm, sizeof nm, "work%d_burst_8wg", work);
    run(nm, [&] { hipLaunchKernelGGL((wave_rr_work<52, false, false>), dim3(cus * 8), dim3(256), 0, 0, adv, total, work); });
  }
  for (int w : {4}) {
    char nm[64];
    snprintf(nm, sizeof nm, "wave_rr_q52_%dwg", w);
    run(nm, [&] { hipLaunchKernelGGL(wave_rr_store<52>, dim3(cus * w), dim3(256), 0, 0, adv, total); });
    snprintf(nm, sizeof nm, "wave_rr_q64_%dwg", w);
    run(nm, [&] { hipLaunchKernelGGL(wave_rr_store<64>, dim3(cus * w), dim3(256), 0, 0, adv, total); });
  }
  for (int w : {4, 8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "wave_dyn_step52_%dwg", w);
    run(nm, [&] { hipLaunchKernelGGL((wave_store<52, true>), dim3(cus * w), dim3(256), 0, 0, adv, total, n, rows_per, ctr); });
    snprintf(nm, sizeof nm, "wave_static_step52_%dwg", w);
    run(nm, [&] { hipLaunchKernelGGL((wave_store<52, false>), dim3(cus * w), dim3(256), 0, 0, adv, total, n, rows_per, ctr); });
    snprintf(nm, sizeof nm, "wave_dyn_step64_%dwg", w);
    run(nm, [&] { hipLaunchKernelGGL((wave_store<64, true>), dim3(cus * w), dim3(256), 0, 0, adv, total, n, rows_per, ctr); });
  }
  CHK(hipFree(adv));
  return 0;
}
