#include "core/vclock.h"

#include <algorithm>
#include <map>
#include <set>
#include <sstream>

namespace dissem {
namespace vclock {

namespace {

struct Waiter {
  std::condition_variable cv;
  bool woken = false;
  bool counted = false;  // the clock counts this thread (busy drops while it waits)
  bool timed = false;
  std::multimap<double, Waiter*>::iterator tit;
  const char* name = "";
};

struct Participant {
  const char* name = "";
  bool blocked = false;
};

struct State {
  std::mutex mu;
  std::atomic<bool> on{false};
  std::atomic<double> t{0.0};
  int64_t busy = 0;
  int64_t advances = 0;
  std::multimap<double, Waiter*> timers;
  std::set<Waiter*> blocked;
  std::set<Participant*> parts;
};

State& S() {
  static State* s = new State();  // never destroyed: threads may outlive static teardown
  return *s;
}

thread_local Participant* tl_part = nullptr;

double steady_now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void wake_locked(State& s, Waiter* w) {
  if (w->woken) return;
  w->woken = true;
  if (w->counted) ++s.busy;
  if (w->timed) {
    s.timers.erase(w->tit);
    w->timed = false;
  }
  w->cv.notify_one();
}

// Every counted thread waits: jump to the earliest deadline and wake its
// waiters. A jump that wakes only uncounted waiters (threads the clock does
// not count) leaves busy at 0, so the clock keeps going to the next one.
void advance_locked(State& s) {
  while (s.busy <= 0 && !s.timers.empty()) {
    const double next = s.timers.begin()->first;
    if (next > s.t.load(std::memory_order_relaxed)) s.t.store(next, std::memory_order_release);
    ++s.advances;
    while (!s.timers.empty() && s.timers.begin()->first <= next) wake_locked(s, s.timers.begin()->second);
  }
}

void drop_participant_locked(State& s) {
  if (!tl_part) return;
  s.parts.erase(tl_part);
  delete tl_part;
  tl_part = nullptr;
  --s.busy;
  advance_locked(s);
}

}  // namespace

bool enabled() { return S().on.load(std::memory_order_acquire); }

void enable(bool on) {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  if (s.on.load() == on) return;
  s.on.store(on, std::memory_order_release);
  s.busy = int64_t(s.parts.size());
  for (auto* p : s.parts) s.busy -= p->blocked ? 1 : 0;
  if (!on) {
    // Wake every virtual waiter: each re-checks its predicate and, still
    // unsatisfied, waits again on the real clock.
    std::vector<Waiter*> all(s.blocked.begin(), s.blocked.end());
    for (auto* w : all) wake_locked(s, w);
  }
}

double now() {
  State& s = S();
  return s.on.load(std::memory_order_acquire) ? s.t.load(std::memory_order_acquire) : steady_now();
}

void sleep_until(double t) {
  if (!enabled()) {
    const double left = t - steady_now();
    if (left > 0) std::this_thread::sleep_for(std::chrono::duration<double>(left));
    return;
  }
  detail::block(nullptr, nullptr, t);
}

std::thread spawn(std::function<void()> fn, const char* name) {
  if (!enabled()) return std::thread(std::move(fn));
  reserve(1);
  return std::thread([fn = std::move(fn), name] {
    adopt(name);
    fn();
    release();
  });
}

void reserve(int n) {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  s.busy += n;
}

void adopt(const char* name) {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  if (tl_part) {  // already counted: hand the reservation back
    --s.busy;
    advance_locked(s);
    return;
  }
  tl_part = new Participant{name, false};
  s.parts.insert(tl_part);
}

void release() {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  drop_participant_locked(s);
}

bool attached() { return tl_part != nullptr; }

Stats stats() {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  Stats out;
  out.t = s.t.load();
  out.busy = s.busy;
  out.blocked = int64_t(s.blocked.size());
  out.timers = int64_t(s.timers.size());
  out.advances = s.advances;
  return out;
}

std::string describe() {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  std::ostringstream o;
  o << "t=" << s.t.load() << " busy=" << s.busy << " timers=" << s.timers.size() << " running:";
  for (auto* p : s.parts)
    if (!p->blocked) o << " " << (p->name && *p->name ? p->name : "?");
  return o.str();
}

namespace detail {

void block(CondVar* cv, std::unique_lock<std::mutex>* lk, double deadline) {
  State& s = S();
  Waiter w;
  std::unique_lock<std::mutex> g(s.mu);
  if (!s.on.load()) return;  // switched off meanwhile: the caller re-checks on the real clock
  if (deadline <= s.t.load()) return;
  w.counted = tl_part != nullptr;
  if (cv) {
    cv->waiters_.push_back(&w);
    cv->nwaiters_.fetch_add(1, std::memory_order_acq_rel);
  }
  if (deadline != kNever) {
    w.timed = true;
    w.tit = s.timers.emplace(deadline, &w);
  }
  s.blocked.insert(&w);
  if (w.counted) {
    tl_part->blocked = true;
    --s.busy;
  }
  advance_locked(s);
  if (lk) lk->unlock();
  w.cv.wait(g, [&] { return w.woken; });
  s.blocked.erase(&w);
  if (w.counted) tl_part->blocked = false;
  if (cv) {
    auto& v = cv->waiters_;
    auto it = std::find(v.begin(), v.end(), static_cast<void*>(&w));
    if (it != v.end()) {
      v.erase(it);
      cv->nwaiters_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  g.unlock();
  if (lk) lk->lock();
}

}  // namespace detail

}  // namespace vclock

void CondVar::notify(bool all) {
  if (all) cv_.notify_all();
  else cv_.notify_one();
  if (nwaiters_.load(std::memory_order_acquire) == 0) return;
  auto& s = vclock::S();
  std::lock_guard<std::mutex> g(s.mu);
  for (auto it = waiters_.begin(); it != waiters_.end();) {
    auto* w = static_cast<vclock::Waiter*>(*it);
    if (w->woken) {
      ++it;
      continue;
    }
    vclock::wake_locked(s, w);
    it = waiters_.erase(it);
    nwaiters_.fetch_sub(1, std::memory_order_acq_rel);
    if (!all) break;
  }
}

}  // namespace dissem
