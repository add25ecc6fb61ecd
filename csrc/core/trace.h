// roctx ranges and marks for rocprofv3 (`rocprofv3 --marker-trace ...`, SURVEY
// §5.1). The reference has no tracing; here the control plane (announce, plan,
// batch dispatch, startup) and the data engine (group issue, staging, CRC
// failures) are annotated so host-side scheduling lines up with the kernel and
// copy timeline.
//
// The core links librocprofiler-sdk-roctx (host-only; also in the sanitizer
// builds); without a profiler attached the calls return immediately.
#pragma once

#include <cstdint>

namespace dissem {
namespace trace {

uint64_t start(const char* name);  // process-wide range (may end on another thread)
void stop(uint64_t id);
void push(const char* name);  // thread-local nested range
void pop();
void mark(const char* name);
bool available();

class Scoped {
 public:
  explicit Scoped(const char* name) { push(name); }
  ~Scoped() { pop(); }
  Scoped(const Scoped&) = delete;
  Scoped& operator=(const Scoped&) = delete;
};

}  // namespace trace
}  // namespace dissem
