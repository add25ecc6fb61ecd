// One read budget shared by every process of a node (BASELINE config #4: all
// ranks of an MI355X node stage their disk tiers from the same NVMe).
//
// A virtual-time pacer in POSIX shared memory: one 64-bit "next free start"
// timestamp (CLOCK_MONOTONIC ns, system-wide) that every reader of every
// process advances with a CAS by the time its read occupies the device at the
// node rate (bytes / rate); the reader then sleeps until its slot. Reads thus
// start no faster than the device can serve them, in arrival order across the
// processes, with no burst (the device queue stays about rate x one read
// deep). Unpaced, 8 processes x 4 readers would keep 32 reads in flight and
// serve them in whatever order the device picks, so the chunks a rank needs
// first wait behind other ranks' later ones.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <thread>

#include "core/vclock.h"

namespace dissem {

class NodePacer {
 public:
  // `key`: names the shared segment (same on every process of the node);
  // `rate`: node read budget in bytes/s (> 0).
  NodePacer(const std::string& key, int64_t rate) : rate_(rate) {
    if (rate <= 0) throw std::runtime_error("NodePacer: rate must be > 0");
    name_ = "/dld_pacer_" + key;
    int fd = shm_open(name_.c_str(), O_RDWR | O_CREAT, 0600);
    if (fd < 0) throw std::runtime_error("NodePacer: shm_open " + name_ + " failed");
    if (ftruncate(fd, 4096) != 0) {
      close(fd);
      throw std::runtime_error("NodePacer: ftruncate failed");
    }
    void* p = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("NodePacer: mmap failed");
    next_ = static_cast<std::atomic<int64_t>*>(p);  // zero-filled on creation: "free now"
    static_assert(std::atomic<int64_t>::is_always_lock_free, "the shared counter must be lock-free");
  }
  ~NodePacer() {
    if (next_) munmap(static_cast<void*>(next_), 4096);
  }
  NodePacer(const NodePacer&) = delete;
  NodePacer& operator=(const NodePacer&) = delete;

  static int64_t now_ns() {
    if (vclock::enabled()) return int64_t(vclock::now() * 1e9);  // simulated node: model time
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return int64_t(ts.tv_sec) * 1000000000ll + ts.tv_nsec;
  }

  // Reserve the device for `bytes` and sleep until the reservation starts.
  // Returns the ns this caller waited.
  int64_t acquire(int64_t bytes) {
    const int64_t dur = int64_t(double(bytes) * 1e9 / double(rate_));
    int64_t now = now_ns();
    int64_t cur = next_->load(std::memory_order_relaxed), start;
    do {
      start = cur > now ? cur : now;
    } while (!next_->compare_exchange_weak(cur, start + dur, std::memory_order_acq_rel, std::memory_order_relaxed));
    const int64_t wait = start - now;
    // A simulated node has no device to serve the read: the reader holds the
    // bytes only at the end of its slot, as a real pread returns then.
    const int64_t until = vclock::enabled() ? wait + dur : wait;
    if (until > 0) vclock::sleep_for(double(until) * 1e-9);
    return wait > 0 ? wait : 0;
  }

  // Remove the segment name (the last process of a run; mapped segments stay valid).
  static void unlink(const std::string& key) { shm_unlink(("/dld_pacer_" + key).c_str()); }

 private:
  int64_t rate_;
  std::string name_;
  std::atomic<int64_t>* next_ = nullptr;
};

}  // namespace dissem
