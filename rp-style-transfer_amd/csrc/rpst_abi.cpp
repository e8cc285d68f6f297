// Library-wide C ABI pieces: version and thread-local error reporting.
#include <cstdarg>
#include <cstdio>

#include "rpst_common.h"

namespace rpst {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace rpst

extern "C" int rpst_version(void) { return 100; }  // 0.1.0

extern "C" const char* rpst_last_error(void) { return rpst::g_err; }
