// contention: does a burst of verify kernels delay an RCCL-like kernel launched
// on another stream, and does reserving CUs on the verify stream fix it?
//
//   bin/contention [-trials N] [-reserve R]
//
// In the planned engine a P2P group lands up to 7 chunks at once; their CRC
// (one batched launch; one 144 KiB-LDS workgroup per CU) runs on the verify
// stream while the next RCCL group kernel waits to launch on the comm stream.
// The probe here stands in for that kernel: 28 workgroups x 256 threads, 16 KiB
// of LDS each, ~20 us of work. For each trial we enqueue the batched CRC of 7
// 64 MiB chunks on the verify stream, then the probe, and time the probe from
// its enqueue to its end (HIP events on its own idle stream), and the burst.
// Verify stream without a CU mask vs one created with R CUs left free, with
// the CRC grid at 256 workgroups or capped at the stream's 256 - R CUs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kernels/kernels.h"

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t err_ = (x);                                             \
    if (err_ != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(err_)); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ void __launch_bounds__(256) probe_kernel(uint32_t* out, uint64_t ticks) {
  __shared__ uint32_t lds[4096];  // 16 KiB, like a comm kernel's staging space
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
  uint32_t acc = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) acc += lds[(acc + threadIdx.x) & 4095];
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

static hipStream_t make_stream(int reserve) {
  hipStream_t s = nullptr;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (reserve <= 0) {
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
  for (int cu = 0; cu < cus - reserve; ++cu) mask[size_t(cu / 32)] |= 1u << (cu % 32);
  CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return s;
}

int main(int argc, char** argv) {
  int trials = 40, reserve = 32;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "-trials") trials = atoi(argv[i + 1]);
    else if (a == "-reserve") reserve = atoi(argv[i + 1]);
  }
  CHECK(hipSetDevice(0));
  const int64_t chunk = 64ll << 20, nchunks = 7;
  uint8_t* buf = nullptr;
  CHECK(hipMalloc(&buf, size_t(chunk * nchunks)));
  CHECK(dissem::kern::fill_random(buf, chunk * nchunks, 42, nullptr));
  void* ws = nullptr;
  CHECK(hipMalloc(&ws, dissem::kern::crc32c_batch_workspace_bytes(chunk, int(nchunks))));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *crc = nullptr, *probe_out = nullptr;
  CHECK(hipMalloc(&crc, 64 * sizeof(uint32_t)));
  CHECK(hipMalloc(&probe_out, 64 * sizeof(uint32_t)));
  hipStream_t comm;
  CHECK(hipStreamCreateWithFlags(&comm, hipStreamNonBlocking));
  hipEvent_t e0, e1, v0, v1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreate(&v0));
  CHECK(hipEventCreate(&v1));
  const uint64_t ticks = 2000;  // 20 us

  // Probe alone: its own launch + run time.
  std::vector<float> alone;
  for (int t = 0; t < trials; ++t) {
    CHECK(hipEventRecord(e0, comm));
    probe_kernel<<<28, 256, 0, comm>>>(probe_out, ticks);
    CHECK(hipEventRecord(e1, comm));
    CHECK(hipStreamSynchronize(comm));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    alone.push_back(ms * 1e3f);
  }
  auto pct = [](std::vector<float> v, double q) {
    std::sort(v.begin(), v.end());
    return v[size_t(q * double(v.size() - 1))];
  };
  printf("{\"case\": \"probe_alone\", \"p50_us\": %.1f, \"max_us\": %.1f}\n", pct(alone, 0.5), pct(alone, 1.0));

  // The 7 chunks as the engine verifies a landed P2P group: one batched launch
  // on the verify stream, unmasked, masked with the full 256-workgroup grid, and
  // masked with the grid capped at the stream's CUs (what HipBackend does).
  dissem::kern::CrcItem items[nchunks];
  for (int64_t c = 0; c < nchunks; ++c) items[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + c};
  const std::pair<int, int> cases[] = {{0, 0}, {reserve, 0}, {reserve, cus - reserve}};
  for (auto [r, cap] : cases) {
    hipStream_t verify = make_stream(r);
    std::vector<float> lat, burst;
    for (int t = 0; t < trials + 2; ++t) {
      CHECK(hipEventRecord(v0, verify));
      CHECK(dissem::kern::crc32c_batch(items, int(nchunks), ws, verify, cap));
      CHECK(hipEventRecord(v1, verify));
      CHECK(hipEventRecord(e0, comm));
      probe_kernel<<<28, 256, 0, comm>>>(probe_out, ticks);
      CHECK(hipEventRecord(e1, comm));
      CHECK(hipStreamSynchronize(comm));
      CHECK(hipStreamSynchronize(verify));
      float ms = 0, vms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipEventElapsedTime(&vms, v0, v1));
      if (t >= 2) {  // first trials build the CRC tables
        lat.push_back(ms * 1e3f);
        burst.push_back(vms * 1e3f);
      }
    }
    printf("{\"case\": \"probe_during_7_crc64MiB\", \"reserved_cus\": %d, \"crc_grid_cap\": %d, "
           "\"probe_p50_us\": %.1f, \"probe_p90_us\": %.1f, \"probe_max_us\": %.1f, \"crc_burst_p50_us\": %.1f}\n",
           r, cap, pct(lat, 0.5), pct(lat, 0.9), pct(lat, 1.0), pct(burst, 0.5));
    CHECK(hipStreamDestroy(verify));
  }
  return 0;
}
