// Library-wide C ABI plumbing: version and the thread-local last-error message.
#include <stdarg.h>
#include <stdio.h>

#include "dna_amd.h"

namespace dna {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace dna

extern "C" int dna_abi_version(void) { return DNA_AMD_ABI_VERSION; }
extern "C" const char* dna_last_error(void) { return dna::g_err; }
