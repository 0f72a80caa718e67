// Shared helpers for the RAFT HIP kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "raft_hip.h"

namespace raft {

// Last-error message, per host thread (raft_hip_last_error()).
char* last_error_buf();

inline int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(last_error_buf(), 512, fmt, ap);
  va_end(ap);
  return code;
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error((int)e, "%s: launch failed: %s", what, hipGetErrorString(e));
  last_error_buf()[0] = 0;
  return 0;
}

#define RAFT_REQUIRE(cond, ...)                              \
  do {                                                       \
    if (!(cond)) return ::raft::set_error(RAFT_E_INVALID, __VA_ARGS__); \
  } while (0)

inline hipStream_t as_stream(raft_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline int round_up(int a, int b) { return cdiv(a, b) * b; }
__host__ __device__ inline long cdiv_l(long a, long b) { return (a + b - 1) / b; }

// XCD-aware tile order.  The dispatcher deals work-groups round-robin over the
// 8 XCDs (work-group L -> XCD L % 8), each with its own L2; hand XCD c a
// contiguous run of the logical tile order so tiles that share operand rows
// (and neighbouring pixels under a conv's taps) hit the same L2.
__device__ inline int xcd_tile(int L, int T) {
  const int c = L & 7, slot = L >> 3;
  const int per = T >> 3, rem = T & 7;
  return c * per + (c < rem ? c : rem) + slot;
}

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

}  // namespace raft
