// Shared helpers for liboflow (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/oflow.h"

namespace oflow {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
// Check the launch that was just issued; converts a HIP error into OF_EHIP.
int check_launch(const char* what);

// Conv launch timing (bench instrumentation), see of_timing_enable().
bool timing_on();
void timing_begin(hipStream_t s);
void timing_end(hipStream_t s, int kind, double flops);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return cdiv(a, b) * b; }

constexpr int kWave = 64;

}  // namespace oflow

#define OF_CHECK_ARG(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) return ::oflow::fail(OF_EINVAL, (msg));          \
  } while (0)
