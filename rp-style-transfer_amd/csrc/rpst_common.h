// Shared helpers for the rpst HIP kernels (gfx950 / CDNA4 only).
//
// Every extern "C" entry point returns RPST_OK (0) or a negative status and records a
// message retrievable with rpst_last_error() (thread-local). Kernels are stateless,
// stream-ordered on the caller's stream and never synchronise the device.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>

#include "../../include/rpst.h"

namespace rpst {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(rpst_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch that was just issued.
inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return RPST_EHIP;
  }
  return RPST_OK;
}

constexpr int kWave = 64;

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef double doublex4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ReflectionPad2d index map for pad = 1 (PyTorch semantics: -1 -> 1, n -> n-2).
// Indices further out only occur for tile overhang whose results are discarded; clamp them.
__device__ __forceinline__ int reflect1(int i, int n) {
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * n - 2 - i : i;
  return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

// ---- WCT colour transform (rpst_wct.hip), used by rpst_conv2d_mix's fallback ----------
// z[b] = T[b] x[b] + c[b] for fp32 x (n, C, HW), fp64 T (n, C, C) and c (n, C); scratch:
// wct_apply_scratch_floats(n, C) floats
size_t wct_apply_scratch_floats(int n, int C);
int wct_apply_f32(const double* T, const double* c, const float* x, float* z, int n, int C,
                  int64_t HW, float* scratch, hipStream_t st);

}  // namespace rpst

#define RPST_REQUIRE(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::rpst::set_error(__VA_ARGS__);    \
      return RPST_EINVAL;                \
    }                                    \
  } while (0)
