// ab_env.hpp — the library's A/B switches. Tuning studies pick kernels,
// thresholds and pack modes through DLSIM_* environment variables
// (INTEGRATION.md §4); the library reads them only when
// DLSIM_AB=1 is set as well, so a stray variable in a user's environment
// cannot change which kernel runs or how a task is packed. Host code only.
#pragma once

#include <cstdlib>
#include <cstring>

namespace dlsim {

// DLSIM_AB=1 (read per call: the per-call knobs follow it; the read-once
// knobs cache what they saw on their first read)
inline bool ab_enabled() {
  const char* e = std::getenv("DLSIM_AB");
  return e && std::strcmp(e, "1") == 0;
}

// getenv(name) under DLSIM_AB=1, else nullptr (every knob's default)
inline const char* ab_getenv(const char* name) { return ab_enabled() ? std::getenv(name) : nullptr; }

}  // namespace dlsim
