// Blocking MPSC/MPMC queue used as a node inbox (the reference's buffered Go
// channel `incomingMsgChan`, transport.go:31). Close() wakes every waiter
// instead of panicking senders (reference quirk: Close closes a channel that
// senders may still use, transport.go:625-631).
#pragma once

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <optional>

#include "core/vclock.h"

namespace dissem {

// Timed condition wait on a system_clock deadline. libstdc++ lowers
// steady_clock waits to pthread_cond_clockwait, which GCC 11's ThreadSanitizer
// does not intercept (it then reports false double locks and races); the
// system_clock form uses pthread_cond_timedwait, which it does.
template <class Lock, class Pred>
bool cv_wait_for(std::condition_variable& cv, Lock& lk, double seconds, Pred pred) {
  auto dl = std::chrono::system_clock::now() +
            std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::duration<double>(seconds));
  return cv.wait_until(lk, dl, pred);
}
// The same on a CondVar (model time when the virtual clock is on).
template <class Pred>
bool cv_wait_for(CondVar& cv, std::unique_lock<std::mutex>& lk, double seconds, Pred pred) {
  return cv.wait_for_s(lk, seconds, pred);
}

template <class T>
class BlockingQueue {
 public:
  // Returns false if the queue is closed.
  bool push(T v) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (closed_) return false;
      q_.push_back(std::move(v));
    }
    cv_.notify_one();
    return true;
  }
  // Blocks until an item is available or the queue is closed and drained.
  std::optional<T> pop() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !q_.empty() || closed_; });
    if (q_.empty()) return std::nullopt;
    T v = std::move(q_.front());
    q_.pop_front();
    return v;
  }
  std::optional<T> pop_for(double seconds) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!cv_wait_for(cv_, lk, seconds, [&] { return !q_.empty() || closed_; })) return std::nullopt;
    if (q_.empty()) return std::nullopt;
    T v = std::move(q_.front());
    q_.pop_front();
    return v;
  }
  std::optional<T> try_pop() {
    std::lock_guard<std::mutex> lk(mu_);
    if (q_.empty()) return std::nullopt;
    T v = std::move(q_.front());
    q_.pop_front();
    return v;
  }
  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      closed_ = true;
    }
    cv_.notify_all();
  }
  bool closed() const {
    std::lock_guard<std::mutex> lk(mu_);
    return closed_;
  }
  size_t size() const {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
  }

 private:
  mutable std::mutex mu_;
  CondVar cv_;
  std::deque<T> q_;
  bool closed_ = false;
};

}  // namespace dissem
