// h2dbench: what is the fastest way to move pinned host bytes into HBM on this
// GPU? The staging step (host tier -> HBM) bounds the 1-GPU headline and, at 8
// GPUs, each GPU's share of the layers that must cross PCIe once.
//
//   bin/h2dbench [-gib N] [-device D]
//
// Compares, over N GiB of pinned host memory (hipHostMalloc):
//  * hipMemcpyAsync (SDMA copy engine) in chunks of 4-256 MiB on 1, 2 and 4 streams;
//  * a gfx950 copy kernel that reads the host buffer directly over PCIe
//    (host-mapped pointer, 16 B per lane, non-temporal), at several grid sizes;
//  * SDMA + kernel together (half the chunks each).
// Prints one JSON line per configuration.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t err_ = (x);                                             \
    if (err_ != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(err_)); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

// Grid-stride copy, 16 B per lane; reads cross PCIe (host-mapped source).
__global__ void __launch_bounds__(256) pull_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                   int64_t n16) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  // 4 loads in flight per lane before the stores.
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(src + i);
    u32x4 b = __builtin_nontemporal_load(src + i + stride);
    u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + stride);
    __builtin_nontemporal_store(c, dst + i + 2 * stride);
    __builtin_nontemporal_store(d, dst + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  int64_t gib = 4;
  int device = 0;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "-gib") gib = atoll(argv[i + 1]);
    else if (a == "-device") device = atoi(argv[i + 1]);
  }
  CHECK(hipSetDevice(device));
  const int64_t n = gib << 30;
  uint8_t *host = nullptr, *dev = nullptr, *hdev = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&host), size_t(n), hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), host, 0));
  CHECK(hipMalloc(&dev, size_t(n)));
  for (int64_t i = 0; i < n; i += 4096) host[i] = uint8_t(i >> 12);
  std::vector<hipStream_t> st(4);
  for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  auto report = [&](const char* what, int64_t chunk_mib, int streams, int blocks, double sec) {
    printf("{\"path\": \"%s\", \"chunk_mib\": %lld, \"streams\": %d, \"blocks\": %d, \"GBps\": %.2f}\n", what,
           (long long)chunk_mib, streams, blocks, double(n) / sec / 1e9);
    fflush(stdout);
  };
  auto sync_all = [&] {
    for (auto& s : st) CHECK(hipStreamSynchronize(s));
  };
  auto best_of = [&](auto&& run) {
    run();  // warm
    sync_all();
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      double t0 = now();
      run();
      sync_all();
      best = std::min(best, now() - t0);
    }
    return best;
  };

  for (int64_t cm : {4, 16, 64, 256}) {
    for (int ns : {1, 2, 4}) {
      const int64_t chunk = cm << 20;
      double t = best_of([&] {
        int k = 0;
        for (int64_t off = 0; off < n; off += chunk, ++k)
          CHECK(hipMemcpyAsync(dev + off, host + off, size_t(std::min(chunk, n - off)), hipMemcpyHostToDevice,
                               st[size_t(k % ns)]));
      });
      report("sdma", cm, ns, 0, t);
    }
  }
  for (int blocks : {64, 128, 256, 512, 1024, 2048}) {
    double t = best_of([&] {
      pull_kernel<<<blocks, 256, 0, st[0]>>>(reinterpret_cast<const u32x4*>(hdev), reinterpret_cast<u32x4*>(dev),
                                             n / 16);
      CHECK(hipGetLastError());
    });
    report("kernel_pull", 0, 1, blocks, t);
  }
  for (int blocks : {128, 512}) {
    // Interleaved 64 MiB chunks: even ones on SDMA, odd ones pulled by the kernel.
    const int64_t chunk = 64ll << 20;
    double t = best_of([&] {
      int k = 0;
      for (int64_t off = 0; off < n; off += chunk, ++k) {
        const int64_t len = std::min(chunk, n - off);
        if (k % 2 == 0) {
          CHECK(hipMemcpyAsync(dev + off, host + off, size_t(len), hipMemcpyHostToDevice, st[1]));
        } else {
          pull_kernel<<<blocks, 256, 0, st[0]>>>(reinterpret_cast<const u32x4*>(hdev + off),
                                                 reinterpret_cast<u32x4*>(dev + off), len / 16);
          CHECK(hipGetLastError());
        }
      }
    });
    report("sdma+kernel", 64, 2, blocks, t);
  }
  // Check the bytes arrived.
  std::vector<uint8_t> back(4096);
  CHECK(hipMemcpy(back.data(), dev + (n - 4096), 4096, hipMemcpyDeviceToHost));
  if (back[0] != uint8_t((n - 4096) >> 12)) {
    fprintf(stderr, "data mismatch\n");
    return 1;
  }
  return 0;
}
