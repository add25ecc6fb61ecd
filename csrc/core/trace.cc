#include "core/trace.h"

#include <dlfcn.h>

#include <mutex>

namespace dissem {
namespace trace {

namespace {

struct Roctx {
  uint64_t (*start)(const char*) = nullptr;
  void (*stop)(uint64_t) = nullptr;
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
};

const Roctx& api() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                           "librocprofiler-sdk-roctx.so"};
    void* h = nullptr;
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) return;
    r.start = reinterpret_cast<uint64_t (*)(const char*)>(dlsym(h, "roctxRangeStartA"));
    r.stop = reinterpret_cast<void (*)(uint64_t)>(dlsym(h, "roctxRangeStop"));
    r.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    r.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    r.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
  });
  return r;
}

}  // namespace

bool available() { return api().push != nullptr; }

uint64_t start(const char* name) {
  auto& r = api();
  return r.start ? r.start(name) : 0;
}
void stop(uint64_t id) {
  auto& r = api();
  if (r.stop && id) r.stop(id);
}
void push(const char* name) {
  auto& r = api();
  if (r.push) r.push(name);
}
void pop() {
  auto& r = api();
  if (r.pop) r.pop();
}
void mark(const char* name) {
  auto& r = api();
  if (r.mark) r.mark(name);
}

}  // namespace trace
}  // namespace dissem
