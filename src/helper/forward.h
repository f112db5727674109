// `devspace-helper forward` (src/helper/forward.cc; protocol: src/sync/fwd_proto.h).
#pragma once

namespace ds {
namespace helper {

// Serves forwarded connections on stdin/stdout until stdin closes. Returns the exit code.
int forward_main();

}  // namespace helper
}  // namespace ds
