// Access-pattern probe for the fused fp8 verify+unpack walk (crc32c.hip):
// which part of its shape - persistent 16-wave workgroups, one 16 KiB segment
// of packed input and one 32 KiB region of bf16 output per wave at a time -
// costs HBM throughput. Every kernel moves the same bytes as the fused kernel
// on 512 MiB of bf16 (264 MiB read, 512 MiB written), with no math:
//
//   rd_seg    persistent walk, loads only (16 KiB per wave in 16 x 1 KiB loads)
//   wr_seg    persistent walk, stores only (32 KiB per wave in 32 x 1 KiB stores)
//   rw_seg    both, as the fused walk issues them (loads of segment g+1 behind
//             the stores of segment g)
//   wr_il     persistent, stores interleaved across waves (wave w writes KiB
//             w, w + nwaves, ...: every instant the chip writes one contiguous run)
//   rw_il     loads and stores interleaved the same way
//   rw_grid   one-shot grid of 256-thread workgroups (the plain unpack's shape)
//
//   bin/walkprobe [MiB of output, default 512] [reps, default 20]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

using u4 = uint4;
constexpr int kThreads = 1024, kWaves = 16;

using v4u = unsigned int __attribute__((ext_vector_type(4)));
// the fused walk's loads are nontemporal (buffer loads with aux = 2)
__device__ __forceinline__ u4 ld_nt(const u4* p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ int wave_id(int waves_per_wg) {
  return __builtin_amdgcn_readfirstlane(int(blockIdx.x * waves_per_wg + (threadIdx.x >> 6)));
}

// segment walk: wave w takes segments w, w + nwaves, ...; segment g = 16 KiB in, 32 KiB out.
// With both loads and stores it issues as the fused walk does: block b's 4
// words are stored (8 KiB out), then the next segment's block b is loaded.
template <bool RD, bool WR>
__global__ void __launch_bounds__(kThreads) seg_walk(const u4* __restrict__ in, u4* __restrict__ out, int64_t segs) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = int64_t(gridDim.x) * kWaves;
  u4 acc = make_uint4(0, 0, 0, 0);
  int64_t g = wave_id(kWaves);
  if (g >= segs) return;
  u4 w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    w[i] = RD ? ld_nt(&in[g * 1024 + i * 64 + lane]) : make_uint4(uint32_t(g), i, lane, 1);
  for (; g < segs; g += nw) {
    const int64_t gn = g + nw < segs ? g + nw : g;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * b + j;
        if (WR) {
          out[g * 2048 + (2 * i) * 64 + lane] = w[i];
          out[g * 2048 + (2 * i + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
        } else {
          acc.x ^= w[i].x ^ w[i].y ^ w[i].z ^ w[i].w;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * b + j;
        w[i] = RD ? ld_nt(&in[gn * 1024 + i * 64 + lane]) : make_uint4(uint32_t(gn), i, lane, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (!WR && acc.x == 0x12345678u) out[lane] = acc;  // keep the loads
}

// The same walk with the next segment's loads issued AHEAD of the current
// segment's stores (ahead = 1: per block, the next block's 4 loads go out
// into temporaries before this block's stores; ahead = 2: the whole next
// segment at the top, a full second register set). vmcnt counts loads and
// stores in one in-order counter on gfx9: a load issued behind stores cannot
// be waited for without waiting for those stores too.
template <int AHEAD>
__global__ void __launch_bounds__(kThreads) seg_walk_ahead(const u4* __restrict__ in, u4* __restrict__ out,
                                                           int64_t segs) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = int64_t(gridDim.x) * kWaves;
  int64_t g = wave_id(kWaves);
  if (g >= segs) return;
  u4 w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = ld_nt(&in[g * 1024 + i * 64 + lane]);
  for (; g < segs; g += nw) {
    const int64_t gn = g + nw < segs ? g + nw : g;
    if constexpr (AHEAD == 2) {
      u4 nx[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) nx[i] = ld_nt(&in[gn * 1024 + i * 64 + lane]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        out[g * 2048 + (2 * i) * 64 + lane] = w[i];
        out[g * 2048 + (2 * i + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = nx[i];
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        u4 t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = ld_nt(&in[gn * 1024 + (4 * b + j) * 64 + lane]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * b + j;
          out[g * 2048 + (2 * i) * 64 + lane] = w[i];
          out[g * 2048 + (2 * i + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) w[4 * b + j] = t[j];
      }
    }
  }
}

// Non-persistent: every wave exactly one segment (SPW = segments per wave in
// sequence), the grid as large as the work - the hardware refills a CU with
// new workgroups as old ones retire, as it does for the plain unpack.
template <int SPW>
__global__ void __launch_bounds__(kThreads) seg_once(const u4* __restrict__ in, u4* __restrict__ out, int64_t segs) {
  const int lane = threadIdx.x & 63;
  for (int k = 0; k < SPW; ++k) {
    const int64_t g = int64_t(wave_id(kWaves)) * SPW + k;
    if (g >= segs) return;
    u4 w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = ld_nt(&in[g * 1024 + i * 64 + lane]);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      out[g * 2048 + (2 * i) * 64 + lane] = w[i];
      out[g * 2048 + (2 * i + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
    }
  }
}

// One segment per wave with the fused kernel's per-workgroup LDS table fill
// (LDSB bytes written from a small global source before any wave works on
// its segment; the segment's loads go out first). THREADS = 1024 with 144 KiB
// (one workgroup per CU, as today) or 512 with 72 KiB (16 table replicas:
// two workgroups per CU, so one fills while the other streams).
template <int THREADS, int LDSB>
__global__ void __launch_bounds__(THREADS) seg_once_lds(const u4* __restrict__ in, u4* __restrict__ out,
                                                        const u4* __restrict__ tab, int64_t segs) {
  __shared__ u4 lds[LDSB / 16];
  const int lane = threadIdx.x & 63;
  const int64_t g = int64_t(wave_id(THREADS / 64));
  u4 w[16];
  if (g < segs) {
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = ld_nt(&in[g * 1024 + i * 64 + lane]);
  }
  for (int i = threadIdx.x; i < LDSB / 16; i += THREADS) lds[i] = tab[i & 255];
  __syncthreads();
  if (g >= segs) return;
  const u4 z = lds[(lane * 37) & (LDSB / 16 - 1)];  // one read of the table (keeps the fill)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    out[g * 2048 + (2 * i) * 64 + lane] = make_uint4(w[i].x ^ z.x, w[i].y, w[i].z, w[i].w);
    out[g * 2048 + (2 * i + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
  }
}

// Persistent with half segments (8 KiB in per wave at a time): fewer VGPRs,
// two workgroups per CU.
__global__ void __launch_bounds__(kThreads) half_walk(const u4* __restrict__ in, u4* __restrict__ out, int64_t halves) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = int64_t(gridDim.x) * kWaves;
  for (int64_t g = wave_id(kWaves); g < halves; g += nw) {
    u4 w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = ld_nt(&in[g * 512 + i * 64 + lane]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      out[g * 1024 + (2 * i) * 64 + lane] = w[i];
      out[g * 1024 + (2 * i + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
    }
  }
}

// interleaved: KiB k of the input and KiBs 2k, 2k+1 of the output go to wave k mod nwaves
template <bool RD>
__global__ void __launch_bounds__(kThreads) il_walk(const u4* __restrict__ in, u4* __restrict__ out, int64_t kibs) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = int64_t(gridDim.x) * kWaves;
  for (int64_t k0 = wave_id(kWaves); k0 < kibs; k0 += 16 * nw) {
    u4 w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t k = k0 + i * nw;
      w[i] = RD ? (k < kibs ? in[k * 64 + lane] : make_uint4(0, 0, 0, 0)) : make_uint4(uint32_t(k), i, lane, 1);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int64_t k = k0 + i * nw;
      if (k < kibs) {
        out[(2 * k) * 64 + lane] = w[i];
        out[(2 * k + 1) * 64 + lane] = make_uint4(w[i].y, w[i].x, w[i].w, w[i].z);
      }
    }
  }
}

// the plain unpack's shape: every thread 8 B in, 16 B out, one-shot grid
__global__ void __launch_bounds__(256) rw_grid(const uint2* __restrict__ in, u4* __restrict__ out, int64_t n) {
  const int64_t t = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (t >= n) return;
  const uint2 v = in[t];
  out[t] = make_uint4(v.x, v.y, v.x ^ v.y, v.y + 1);
}

int main(int argc, char** argv) {
  const int64_t out_mib = argc > 1 ? atoll(argv[1]) : 512;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int64_t out_bytes = out_mib << 20, in_bytes = out_bytes / 2;
  const int64_t segs = in_bytes / 16384;
  u4 *in, *out;
  CK(hipMalloc(&in, in_bytes));
  CK(hipMalloc(&out, out_bytes));
  CK(hipMemset(in, 1, in_bytes));
  CK(hipMemset(out, 0, out_bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](const char* name, int64_t rbytes, int64_t wbytes, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    printf("{\"kernel\": \"%s\", \"us\": %.1f, \"GBps\": %.1f, \"read_MiB\": %lld, \"write_MiB\": %lld}\n", name, us,
           double(rbytes + wbytes) / (us * 1e-6) / 1e9, (long long)(rbytes >> 20), (long long)(wbytes >> 20));
    fflush(stdout);
  };
  // as the fused kernel picks its grid: fewest rounds of 16 segments per workgroup, then fewest workgroups
  const int64_t rounds = (segs + int64_t(cus) * kWaves - 1) / (int64_t(cus) * kWaves);
  const int wgs = int((segs + kWaves * rounds - 1) / (kWaves * rounds));
  for (int g : {wgs, cus, 2 * cus}) {
    char nm[64];
    snprintf(nm, sizeof nm, "rd_seg/%d", g);
    time(nm, in_bytes, 0, [&] { seg_walk<true, false><<<g, kThreads>>>(in, out, segs); });
    snprintf(nm, sizeof nm, "wr_seg/%d", g);
    time(nm, 0, out_bytes, [&] { seg_walk<false, true><<<g, kThreads>>>(in, out, segs); });
    snprintf(nm, sizeof nm, "rw_seg/%d", g);
    time(nm, in_bytes, out_bytes, [&] { seg_walk<true, true><<<g, kThreads>>>(in, out, segs); });
    snprintf(nm, sizeof nm, "rw_ahead1/%d", g);
    time(nm, in_bytes, out_bytes, [&] { seg_walk_ahead<1><<<g, kThreads>>>(in, out, segs); });
    snprintf(nm, sizeof nm, "rw_ahead2/%d", g);
    time(nm, in_bytes, out_bytes, [&] { seg_walk_ahead<2><<<g, kThreads>>>(in, out, segs); });
    snprintf(nm, sizeof nm, "wr_il/%d", g);
    time(nm, 0, out_bytes, [&] { il_walk<false><<<g, kThreads>>>(in, out, in_bytes / 1024); });
    snprintf(nm, sizeof nm, "rw_il/%d", g);
    time(nm, in_bytes, out_bytes, [&] { il_walk<true><<<g, kThreads>>>(in, out, in_bytes / 1024); });
  }
  for (int spw : {1, 2, 4}) {
    char nm[64];
    snprintf(nm, sizeof nm, "rw_once_spw%d", spw);
    const unsigned grid = unsigned((segs + int64_t(kWaves) * spw - 1) / (int64_t(kWaves) * spw));
    if (spw == 1) time(nm, in_bytes, out_bytes, [&] { seg_once<1><<<grid, kThreads>>>(in, out, segs); });
    if (spw == 2) time(nm, in_bytes, out_bytes, [&] { seg_once<2><<<grid, kThreads>>>(in, out, segs); });
    if (spw == 4) time(nm, in_bytes, out_bytes, [&] { seg_once<4><<<grid, kThreads>>>(in, out, segs); });
  }
  {
    u4* tab;
    CK(hipMalloc(&tab, 4096));
    CK(hipMemset(tab, 3, 4096));
    time("rw_once_lds144k_1024t", in_bytes, out_bytes, [&] {
      seg_once_lds<1024, 147456><<<unsigned((segs + 15) / 16), 1024>>>(in, out, tab, segs);
    });
    time("rw_once_lds72k_512t", in_bytes, out_bytes, [&] {
      seg_once_lds<512, 73728><<<unsigned((segs + 7) / 8), 512>>>(in, out, tab, segs);
    });
    time("rw_once_lds48k_256t", in_bytes, out_bytes, [&] {
      seg_once_lds<256, 49152><<<unsigned((segs + 3) / 4), 256>>>(in, out, tab, segs);
    });
    CK(hipFree(tab));
  }
  for (int g : {cus, 2 * cus}) {
    char nm[64];
    snprintf(nm, sizeof nm, "rw_half/%d", g);
    time(nm, in_bytes, out_bytes, [&] { half_walk<<<g, kThreads>>>(in, out, 2 * segs); });
  }
  const int64_t n = in_bytes / 8;
  time("rw_grid", in_bytes, out_bytes,
       [&] { rw_grid<<<unsigned((n + 255) / 256), 256>>>(reinterpret_cast<const uint2*>(in), out, n); });
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
