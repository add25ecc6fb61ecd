// diskspeed: calibrate the NVMe -> pinned host -> HBM staging path
// (reference: diskspeed/main.go, which only times a buffered ReadAt into RAM).
//
//   bin/diskspeed -path FILE [-chunk MiB] [-depth N] [-device D] [-no-direct]
//
// Reports three rates: file -> pinned host (O_DIRECT preads on `depth` reader
// threads), pinned host -> HBM (hipMemcpyAsync), and the overlapped pipeline
// file -> pinned ring -> HBM, which is what the disk tier of the data engine
// does. Use the numbers as `Sources` rates in a topology config.
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t err_ = (x);                                                           \
    if (err_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(err_));               \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  std::string path;
  int64_t chunk = 64ll << 20;
  int depth = 4, device = 0;
  bool direct = true;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-path" && i + 1 < argc) path = argv[++i];
    else if (a == "-chunk" && i + 1 < argc) chunk = atoll(argv[++i]) << 20;
    else if (a == "-depth" && i + 1 < argc) depth = atoi(argv[++i]);
    else if (a == "-device" && i + 1 < argc) device = atoi(argv[++i]);
    else if (a == "-no-direct") direct = false;
  }
  if (path.empty()) {
    printf("usage: -path [file path] [-chunk MiB] [-depth N] [-device D] [-no-direct]\n");
    return 0;
  }
  struct stat st;
  if (stat(path.c_str(), &st) != 0) {
    perror("stat");
    return 1;
  }
  const int64_t size = st.st_size;
  int fd = open(path.c_str(), O_RDONLY | (direct ? O_DIRECT : 0));
  if (fd < 0 && direct) {
    fprintf(stderr, "O_DIRECT not supported here, falling back to buffered reads\n");
    direct = false;
    fd = open(path.c_str(), O_RDONLY);
  }
  if (fd < 0) {
    perror("open");
    return 1;
  }
  CHECK(hipSetDevice(device));
  std::vector<void*> ring(static_cast<size_t>(depth));
  for (auto& p : ring) CHECK(hipHostMalloc(&p, size_t(chunk), hipHostMallocDefault));
  void* dev = nullptr;
  CHECK(hipMalloc(&dev, size_t(size)));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const int64_t n = (size + chunk - 1) / chunk;

  auto read_chunk = [&](int64_t c, void* buf) {
    int64_t off = c * chunk, len = std::min(chunk, size - off);
    int64_t want = direct ? ((len + 4095) / 4096) * 4096 : len;
    int64_t got = 0;
    while (got < len) {
      ssize_t r = pread(fd, static_cast<char*>(buf) + got, size_t(want - got), off + got);
      if (r <= 0) break;
      got += r;
    }
    return len;
  };

  // 1) file -> pinned host, `depth` readers
  double t0 = now();
  std::atomic<int64_t> next{0};
  std::vector<std::thread> th;
  for (int r = 0; r < depth; ++r)
    th.emplace_back([&, r] {
      for (int64_t c; (c = next++) < n;) read_chunk(c, ring[size_t(r)]);
    });
  for (auto& t : th) t.join();
  double t_read = now() - t0;

  // 2) pinned host -> HBM
  t0 = now();
  for (int64_t c = 0; c < n; ++c) {
    int64_t off = c * chunk, len = std::min(chunk, size - off);
    CHECK(hipMemcpyAsync(static_cast<char*>(dev) + off, ring[size_t(c % depth)], size_t(len), hipMemcpyHostToDevice, s));
  }
  CHECK(hipStreamSynchronize(s));
  double t_h2d = now() - t0;

  // 3) overlapped: read chunk c+1.. while chunk c copies (ring of `depth` pinned buffers)
  std::vector<hipEvent_t> ev(static_cast<size_t>(depth));
  for (auto& e : ev) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  t0 = now();
  for (int64_t c = 0; c < n; ++c) {
    int slot = int(c % depth);
    if (c >= depth) CHECK(hipEventSynchronize(ev[size_t(slot)]));
    int64_t len = read_chunk(c, ring[size_t(slot)]);
    CHECK(hipMemcpyAsync(static_cast<char*>(dev) + c * chunk, ring[size_t(slot)], size_t(len), hipMemcpyHostToDevice, s));
    CHECK(hipEventRecord(ev[size_t(slot)], s));
  }
  CHECK(hipStreamSynchronize(s));
  double t_pipe = now() - t0;

  const double mib = double(size) / (1 << 20);
  printf("File size: %lld\n", (long long)size);
  printf("Time to load: %.3fs\n", t_read);
  printf("Throughput: %.2f MiB/s (file -> pinned host, %s, depth %d)\n", mib / t_read, direct ? "O_DIRECT" : "buffered",
         depth);
  printf("H2D: %.2f MiB/s (pinned -> HBM)\n", mib / t_h2d);
  printf("Pipeline: %.2f MiB/s (file -> pinned ring -> HBM)\n", mib / t_pipe);
  printf("{\"bytes\": %lld, \"read_MiBps\": %.1f, \"h2d_MiBps\": %.1f, \"pipeline_MiBps\": %.1f}\n", (long long)size,
         mib / t_read, mib / t_h2d, mib / t_pipe);
  close(fd);
  return 0;
}
