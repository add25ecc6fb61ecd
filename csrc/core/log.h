// JSON-lines logger with the reference's field names.
//
// The reference logs zerolog JSON lines on stderr: {"level","time"(unix ms),
// "node",...fields...,"message"} (cmd/main.go:35-44). conf/collect_logs.sh merges
// per-node logs by `time` and rebases on the "timer start" event, so keeping the
// same field names and event strings lets the same tooling (scripts/collect_logs.py)
// work on our logs.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>

namespace dissem {
namespace log {

enum Level : int { Debug = 0, Info = 1, Warn = 2, Error = 3, Off = 4 };

void set_level(int level);
int level();
// Redirect output: empty path = stderr.
void set_file(const std::string& path);
int64_t now_ms();
int64_t now_us();

class Event {
 public:
  Event(Level lvl, int64_t node);
  Event(const Event&) = delete;
  ~Event();
  Event& i(const char* k, int64_t v);
  Event& u(const char* k, uint64_t v);
  Event& f(const char* k, double v);
  Event& s(const char* k, const std::string& v);
  Event& b(const char* k, bool v);
  void msg(const std::string& m);  // emits the line
  void send() { msg(""); }

 private:
  bool on_;
  bool done_ = false;
  std::string buf_;
};

inline Event debug(int64_t node) { return Event(Debug, node); }
inline Event info(int64_t node) { return Event(Info, node); }
inline Event warn(int64_t node) { return Event(Warn, node); }
inline Event error(int64_t node) { return Event(Error, node); }

}  // namespace log
}  // namespace dissem
