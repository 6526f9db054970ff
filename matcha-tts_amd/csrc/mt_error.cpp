// Thread-local last-error string for the C ABI (mt_last_error()).
#include <stdarg.h>
#include <stdio.h>

namespace mt {
static thread_local char g_err[1024] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }
}  // namespace mt
