// Host-side diagnostic overrides: DCR_DEBUG="key=value,key=value" (docs/DESIGN.md "Knobs").
// The one environment variable the kernels' host code reads; each key forces a choice the
// launcher otherwise makes from measurements (test and A/B use only).
#pragma once
#include <stdlib.h>
#include <string.h>

namespace dcr {

// integer value of `key` in DCR_DEBUG, or `dflt` when absent
inline int debug_int(const char* key, int dflt) {
  const char* e = getenv("DCR_DEBUG");
  if (!e) return dflt;
  const size_t n = strlen(key);
  for (const char* p = e; *p;) {
    if (strncmp(p, key, n) == 0 && p[n] == '=') return atoi(p + n + 1);
    const char* c = strchr(p, ',');
    if (!c) break;
    p = c + 1;
  }
  return dflt;
}

}  // namespace dcr
