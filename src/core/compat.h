// Reference-equivalent timing (BASELINE.md "How the rebuild will be compared"): with
// DEVSPACE_REFERENCE_TIMING=1 the CLI reproduces the reference's waiting behaviour so the
// bench can report a same-box reference column for `devspace deploy` / `devspace dev`:
//   - pod discovery sleeps 1 s before every list (kubectl/client.go:183-217),
//   - rollout / readiness waits poll every 5 s instead of following a watch
//     (helm/tiller.go:101-102, builder/kaniko/kaniko.go:177-178),
//   - no kept-alive API connections (one TCP+TLS handshake per request).
// The sync protocol of that column is chosen separately (DEVSPACE_SYNC_MODE=compat).
#pragma once

#include <cstdlib>
#include <cstring>

namespace ds {

inline bool reference_timing() {
  static const bool on = [] {
    const char* v = std::getenv("DEVSPACE_REFERENCE_TIMING");
    return v && *v && std::strcmp(v, "0") != 0;
  }();
  return on;
}

}  // namespace ds
