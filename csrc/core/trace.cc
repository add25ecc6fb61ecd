#include "core/trace.h"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace dissem {
namespace trace {

// Linked against librocprofiler-sdk-roctx (a plain host library): without a
// profiler attached its entry points return immediately.
bool available() { return true; }
uint64_t start(const char* name) { return roctxRangeStartA(name); }
void stop(uint64_t id) {
  if (id) roctxRangeStop(id);
}
void push(const char* name) { roctxRangePushA(name); }
void pop() { roctxRangePop(); }
void mark(const char* name) { roctxMarkA(name); }

}  // namespace trace
}  // namespace dissem
