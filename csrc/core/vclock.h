// Virtual clock for the simulated fabric: a discrete-event mode in which no
// participating thread ever sleeps on the wall clock.
//
// Off (the default, every real run): now() is the steady clock, sleeps are
// real sleeps and CondVar is a std::condition_variable.
//
// On (vclock::enable(true), CPU simulations only): time is a number that
// advances only when every PARTICIPATING thread is blocked - in a CondVar
// wait, a sleep or a BlockingQueue pop - and then jumps straight to the
// earliest deadline any of them waits for. A participating thread is one the
// clock counts: threads started with vclock::spawn (the engine's issue,
// monitor and disk-reader threads, the node's event loop, the sim backend's
// lane / copy / verify queues), and caller threads that adopted a reservation
// (vclock::reserve + adopt: the Python threads that run a session's ranks).
// Everything a schedule does at one instant therefore happens before the
// clock moves, whatever the host's load: modeled transfers, staging copies,
// token buckets and the engine's 20 us polls all advance model time, and a
// session's makespan is a property of the schedule, not of the simulator's
// own threads.
//
// Rules for code that runs on participating threads: block only through
// CondVar / vclock::sleep_* (std::mutex critical sections are fine, they do
// not wait on time); a CondVar's predicate state changes under the mutex the
// waiter holds (the std::condition_variable discipline).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dissem {

class CondVar;

namespace vclock {

constexpr double kNever = std::numeric_limits<double>::infinity();

bool enabled();
// Switch modes; only while no participating thread exists (between runs).
// Switching off wakes every virtual waiter (they re-wait on the real clock).
void enable(bool on);
double now();  // seconds: model time when enabled, else the steady clock
inline int64_t now_us() { return int64_t(now() * 1e6); }
void sleep_until(double t);
inline void sleep_for(double secs) { sleep_until(now() + secs); }

// A thread counted by the clock (a plain std::thread when the clock is off).
std::thread spawn(std::function<void()> fn, const char* name = "");
// Count n threads that are about to adopt (caller side), so the clock cannot
// move between their creation and their first wait.
void reserve(int n);
void adopt(const char* name = "");  // this thread takes one reservation
void release();                     // this thread stops being counted
bool attached();

struct Stats {
  double t = 0;
  int64_t busy = 0;      // counted threads not blocked (reservations included)
  int64_t blocked = 0;   // threads blocked in a virtual wait
  int64_t timers = 0;
  int64_t advances = 0;  // clock jumps since the process started
};
Stats stats();
std::string describe();  // names of the counted threads that are running (a stuck clock's suspects)

namespace detail {
// Block the calling thread until woken or the deadline passes (model time).
// `lk` (may be null) is released while blocked and re-acquired after.
void block(CondVar* cv, std::unique_lock<std::mutex>* lk, double deadline);
}  // namespace detail

}  // namespace vclock

// Drop-in for std::condition_variable on the paths the simulator drives.
// Deadlines are in vclock::now() seconds.
class CondVar {
 public:
  void notify_one() { notify(false); }
  void notify_all() { notify(true); }

  template <class Pred>
  void wait(std::unique_lock<std::mutex>& lk, Pred pred) {
    (void)wait_until_s(lk, vclock::kNever, pred);
  }
  // Returns pred() (false: the deadline passed first).
  template <class Pred>
  bool wait_until_s(std::unique_lock<std::mutex>& lk, double deadline, Pred pred) {
    while (!pred()) {
      if (vclock::enabled()) {
        if (deadline <= vclock::now()) return pred();
        vclock::detail::block(this, &lk, deadline);
        continue;
      }
      if (deadline == vclock::kNever) {
        cv_.wait(lk);
        continue;
      }
      const double left = deadline - vclock::now();
      if (left <= 0) return pred();
      // system_clock deadline: libstdc++ lowers steady_clock waits to
      // pthread_cond_clockwait, which GCC 11's ThreadSanitizer does not intercept
      cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                                                std::chrono::duration<double>(left)));
    }
    return true;
  }
  template <class Pred>
  bool wait_for_s(std::unique_lock<std::mutex>& lk, double secs, Pred pred) {
    return wait_until_s(lk, vclock::now() + secs, pred);
  }

 private:
  friend void vclock::detail::block(CondVar*, std::unique_lock<std::mutex>*, double);
  void notify(bool all);
  std::condition_variable cv_;
  std::vector<void*> waiters_;        // virtual waiters (guarded by the clock's mutex)
  std::atomic<int> nwaiters_{0};
};

}  // namespace dissem
