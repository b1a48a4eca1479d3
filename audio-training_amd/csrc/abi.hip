// ABI utilities: version, thread-local last-error string.
#include "common.h"
#include <cstdio>

namespace acfe {
static thread_local char g_err[256] = "";
void set_error(hipError_t e, const char* where) {
  std::snprintf(g_err, sizeof(g_err), "%s: %s (%d)", where, hipGetErrorString(e), (int)e);
}
}  // namespace acfe

ACFE_API int acfe_version(void) { return 100; }
ACFE_API const char* acfe_last_error(void) { return acfe::g_err; }
