// diskspeed: calibrate the NVMe -> pinned host -> HBM staging path
// (reference: diskspeed/main.go, which only times a buffered ReadAt into RAM).
//
//   bin/diskspeed -path FILE [-path FILE ...] [-chunk MiB] [-depth N] [-device D] [-no-direct]
//
// Every -path adds a file (e.g. all layer files of a bench run: the rate over
// tens of GiB, not the ramp of one file). Reports three rates over all of
// them: file -> pinned host (O_DIRECT preads on `depth` reader threads),
// pinned host -> HBM (hipMemcpyAsync), and the overlapped pipeline
// file -> pinned ring -> HBM with `depth` readers, each handing its chunk to
// the copy stream - what the disk tier of the data engine does (its reader
// threads and bounce ring, planned_stage.cc). Evict the files from the page
// cache first (bench.py does; Runtime.drop_disk_cache) or the first pass
// reads memory. Use the numbers as `Sources` rates in a topology config.
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
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

struct Chunk {
  int file;
  int64_t off, len;
};

int main(int argc, char** argv) {
  std::vector<std::string> paths;
  int64_t chunk = 64ll << 20;
  int depth = 4, device = 0;
  bool direct = true;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-path" && i + 1 < argc) paths.push_back(argv[++i]);
    else if (a == "-chunk" && i + 1 < argc) chunk = atoll(argv[++i]) << 20;
    else if (a == "-depth" && i + 1 < argc) depth = atoi(argv[++i]);
    else if (a == "-device" && i + 1 < argc) device = atoi(argv[++i]);
    else if (a == "-no-direct") direct = false;
  }
  if (paths.empty() || depth < 1 || chunk <= 0) {
    printf("usage: -path [file path] [-path ...] [-chunk MiB] [-depth N] [-device D] [-no-direct]\n");
    return 0;
  }
  std::vector<int> fds;
  std::vector<Chunk> chunks;
  int64_t total = 0;
  for (size_t f = 0; f < paths.size(); ++f) {
    struct stat st;
    if (stat(paths[f].c_str(), &st) != 0) {
      perror(paths[f].c_str());
      return 1;
    }
    int fd = open(paths[f].c_str(), O_RDONLY | (direct ? O_DIRECT : 0));
    if (fd < 0 && direct) {
      fprintf(stderr, "O_DIRECT not supported here, falling back to buffered reads\n");
      direct = false;
      fd = open(paths[f].c_str(), O_RDONLY);
    }
    if (fd < 0) {
      perror("open");
      return 1;
    }
    fds.push_back(fd);
    for (int64_t off = 0; off < st.st_size; off += chunk)
      chunks.push_back(Chunk{int(f), off, std::min<int64_t>(chunk, st.st_size - off)});
    total += st.st_size;
  }
  CHECK(hipSetDevice(device));
  const int ring_n = 2 * depth;  // pinned bounce buffers (the engine's disk_ring)
  std::vector<void*> ring(static_cast<size_t>(ring_n));
  for (auto& p : ring) CHECK(hipHostMalloc(&p, size_t(chunk), hipHostMallocDefault));
  const int dev_slots = 64;  // HBM destination: a 4 GiB ring at 64 MiB chunks, whatever the file sizes
  void* dev = nullptr;
  CHECK(hipMalloc(&dev, size_t(chunk) * dev_slots));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const int64_t n = int64_t(chunks.size());

  auto read_chunk = [&](int64_t c, void* buf) {
    const Chunk& k = chunks[size_t(c)];
    int64_t want = direct ? ((k.len + 4095) / 4096) * 4096 : k.len;
    int64_t got = 0;
    while (got < k.len) {
      ssize_t r = pread(fds[size_t(k.file)], static_cast<char*>(buf) + got, size_t(want - got), k.off + got);
      if (r <= 0) break;
      got += r;
    }
    return k.len;
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
  const double t_read = now() - t0;

  // 2) pinned host -> HBM (the same number of chunks, from the ring)
  t0 = now();
  for (int64_t c = 0; c < n; ++c)
    CHECK(hipMemcpyAsync(static_cast<char*>(dev) + (c % dev_slots) * chunk, ring[size_t(c % ring_n)],
                         size_t(chunks[size_t(c)].len), hipMemcpyHostToDevice, s));
  CHECK(hipStreamSynchronize(s));
  const double t_h2d = now() - t0;

  // 3) overlapped, as the engine's disk tier runs it (planned_stage.cc): a
  // free list of pinned bounce buffers, `depth` readers each taking the next
  // chunk and any free buffer, the H2D copy enqueued on two alternating
  // streams (the engine's two copy queues), and the main thread returning a
  // buffer to the free list once the event behind its copy has fired.
  hipStream_t s2;
  CHECK(hipStreamCreate(&s2));
  std::vector<hipEvent_t> ev(static_cast<size_t>(ring_n));
  for (auto& e : ev) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> free_slots, busy;
  for (int i = 0; i < ring_n; ++i) free_slots.push_back(i);
  int64_t copies = 0, landed = 0;
  next = 0;
  th.clear();
  t0 = now();
  for (int r = 0; r < depth; ++r)
    th.emplace_back([&] {
      for (int64_t c; (c = next++) < n;) {
        int slot;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return !free_slots.empty(); });
          slot = free_slots.back();
          free_slots.pop_back();
        }
        const int64_t len = read_chunk(c, ring[size_t(slot)]);
        std::lock_guard<std::mutex> lk(mu);
        hipStream_t cs = (copies++ & 1) ? s2 : s;
        CHECK(hipMemcpyAsync(static_cast<char*>(dev) + (c % dev_slots) * chunk, ring[size_t(slot)], size_t(len),
                             hipMemcpyHostToDevice, cs));
        CHECK(hipEventRecord(ev[size_t(slot)], cs));
        busy.push_back(slot);
      }
    });
  while (true) {  // reclaim buffers whose copy landed
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = 0; i < busy.size();) {
        if (hipEventQuery(ev[size_t(busy[i])]) == hipSuccess) {
          free_slots.push_back(busy[i]);
          busy[i] = busy.back();
          busy.pop_back();
          ++landed;
        } else {
          ++i;
        }
      }
      if (landed == n) break;
    }
    cv.notify_all();
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  for (auto& t : th) t.join();
  CHECK(hipStreamSynchronize(s));
  CHECK(hipStreamSynchronize(s2));
  const double t_pipe = now() - t0;

  const double mib = double(total) / (1 << 20);
  printf("Files: %zu, bytes: %lld\n", paths.size(), (long long)total);
  printf("Time to load: %.3fs\n", t_read);
  printf("Throughput: %.2f MiB/s (file -> pinned host, %s, depth %d)\n", mib / t_read, direct ? "O_DIRECT" : "buffered",
         depth);
  printf("H2D: %.2f MiB/s (pinned -> HBM)\n", mib / t_h2d);
  printf("Pipeline: %.2f MiB/s (file -> pinned ring -> HBM, %d readers)\n", mib / t_pipe, depth);
  printf("{\"files\": %zu, \"bytes\": %lld, \"direct\": %s, \"depth\": %d, \"read_GBps\": %.2f, \"h2d_GBps\": %.2f, "
         "\"pipeline_GBps\": %.2f}\n",
         paths.size(), (long long)total, direct ? "true" : "false", depth, double(total) / t_read / 1e9,
         double(total) / t_h2d / 1e9, double(total) / t_pipe / 1e9);
  for (int fd : fds) close(fd);
  return 0;
}
