// Token-bucket pacing (reference: golang.org/x/time/rate with a 256 KiB bucket,
// transport.go:407-424, node.go:1615-1624). Differences by design:
//  * rate <= 0 means unlimited (quirk Q1: the reference's rate 0 admits only the
//    initial burst on the send path while mode 2 treats 0 as infinite);
//  * one pacer is used for every source tier (quirk Q2: the reference's disk path
//    ignores LimitRate).
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <thread>

#include "core/vclock.h"

namespace dissem {

// The bucket's clock: the process clock (real time, or the simulator's model
// time when core/vclock.h is on), or a private virtual clock whose sleep
// advances it (unit tests: exact, host-load independent).
struct SteadyClock {
  double now() const { return vclock::now(); }
  void sleep(double secs) { vclock::sleep_for(secs); }
};
struct VirtualClock {
  double t = 0;
  double now() const { return t; }
  void sleep(double secs) { t += secs; }
};

template <class Clock = SteadyClock>
class BasicTokenBucket {
 public:
  static constexpr int64_t kDefaultBurst = 256 * 1024;

  explicit BasicTokenBucket(int64_t rate_bps, int64_t burst = kDefaultBurst, Clock clock = Clock())
      : rate_(rate_bps), burst_(std::max<int64_t>(burst, 1)), tokens_(double(burst_)), clock_(clock),
        last_(clock_.now()) {}

  bool unlimited() const { return rate_ <= 0; }
  int64_t burst() const { return burst_; }
  int64_t rate() const { return rate_; }
  const Clock& clock() const { return clock_; }

  // Blocks until n bytes may pass (n <= burst is the intended use).
  void wait(int64_t n) {
    if (rate_ <= 0) return;
    refill();
    tokens_ -= double(n);
    if (tokens_ < 0) {
      clock_.sleep(-tokens_ / double(rate_));
      refill();
    }
  }

  // Calls fn(offset, len) over [0, total) in burst-sized pieces, pacing each.
  template <class F>
  void paced(int64_t total, F&& fn) {
    int64_t step = rate_ <= 0 ? total : burst_;
    if (step <= 0) step = total;
    for (int64_t off = 0; off < total;) {
      int64_t n = std::min(step, total - off);
      wait(n);
      fn(off, n);
      off += n;
    }
  }

 private:
  void refill() {
    const double now = clock_.now();
    const double dt = now - last_;
    last_ = now;
    tokens_ = std::min(double(burst_), tokens_ + dt * double(rate_));
  }
  int64_t rate_;
  int64_t burst_;
  double tokens_;
  Clock clock_;
  double last_;
};

using TokenBucket = BasicTokenBucket<>;

}  // namespace dissem
