#include "core/log.h"

#include <chrono>
#include <cstdio>
#include <mutex>

#include "core/json.h"

namespace dissem {
namespace log {

namespace {
std::atomic<int> g_level{Info};
std::mutex g_mu;
FILE* g_out = nullptr;  // nullptr = stderr
const char* kNames[] = {"debug", "info", "warn", "error", "off"};
}  // namespace

void set_level(int lvl) { g_level.store(lvl); }
int level() { return g_level.load(); }

void set_file(const std::string& path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_out) fclose(g_out);
  g_out = path.empty() ? nullptr : fopen(path.c_str(), "a");
}

int64_t now_ms() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count();
}
int64_t now_us() {
  using namespace std::chrono;
  return duration_cast<microseconds>(steady_clock::now().time_since_epoch()).count();
}

Event::Event(Level lvl, int64_t node) : on_(lvl >= g_level.load()) {
  if (!on_) return;
  buf_.reserve(160);
  buf_ += "{\"level\":\"";
  buf_ += kNames[lvl];
  buf_ += "\",\"time\":";
  buf_ += std::to_string(now_ms());
  buf_ += ",\"node\":";
  buf_ += std::to_string(node);
}

Event::~Event() {
  if (on_ && !done_) send();
}

Event& Event::i(const char* k, int64_t v) {
  if (on_) { buf_ += ",\""; buf_ += k; buf_ += "\":"; buf_ += std::to_string(v); }
  return *this;
}
Event& Event::u(const char* k, uint64_t v) {
  if (on_) { buf_ += ",\""; buf_ += k; buf_ += "\":"; buf_ += std::to_string(v); }
  return *this;
}
Event& Event::f(const char* k, double v) {
  if (on_) { buf_ += ",\""; buf_ += k; buf_ += "\":"; Json(v).dump_to(buf_); }
  return *this;
}
Event& Event::s(const char* k, const std::string& v) {
  if (on_) { buf_ += ",\""; buf_ += k; buf_ += "\":"; Json(v).dump_to(buf_); }
  return *this;
}
Event& Event::b(const char* k, bool v) {
  if (on_) { buf_ += ",\""; buf_ += k; buf_ += "\":"; buf_ += v ? "true" : "false"; }
  return *this;
}
void Event::msg(const std::string& m) {
  if (!on_ || done_) return;
  done_ = true;
  if (!m.empty()) {
    buf_ += ",\"message\":";
    Json(m).dump_to(buf_);
  }
  buf_ += "}\n";
  std::lock_guard<std::mutex> lk(g_mu);
  FILE* out = g_out ? g_out : stderr;
  fwrite(buf_.data(), 1, buf_.size(), out);
  fflush(out);
}

}  // namespace log
}  // namespace dissem
