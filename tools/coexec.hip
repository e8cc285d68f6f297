// Co-execution microbenchmark (gfx950): can one wave's v_fma_f32 stream run beside its SIMD
// partner's v_mfma_f32_16x16x4_f32 stream (512-thread blocks = two waves per SIMD)?
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/coexec.hip -o /tmp/coexec
// Modes (waves 0-3 = "A", waves 4-7 = "B", wave w and w + 4 share a SIMD):
//   0: A MFMA, B idle   1: A VALU, B idle   2: A MFMA, B VALU   3: A MFMA, B MFMA
//   4: every wave MFMA and VALU interleaved in one stream (the Winograd kernel's pattern)
//   5: A 32x32x2 f32 MFMA, B idle   6: A 32x32x2 f32 MFMA, B VALU
//   7: A 16x16x32 bf16 MFMA, B idle   8: A 16x16x32 bf16 MFMA, B VALU
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(512, 1) void coexec(float* out, int iters, float a, float b) {
  const int wave = threadIdx.x >> 6;
  const bool A = wave < 4;
  const bool do_mfma = MODE == 4 || (A && (MODE == 0 || MODE == 2 || MODE == 3)) || (!A && MODE == 3);
  const bool do_valu = MODE == 4 || (A && MODE == 1) || (!A && (MODE == 2 || MODE == 6 || MODE == 8));
  const bool do_m32 = A && (MODE == 5 || MODE == 6);
  const bool do_bf = A && (MODE == 7 || MODE == 8);
  f4v acc[8];
  float x[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = a * (float)(threadIdx.x + i);
  f16v acc32[2];
  acc32[0] = acc32[1] = f16v{};
  bf8v av, bv;
#pragma unroll
  for (int i = 0; i < 8; ++i) av[i] = bv[i] = (__bf16)(a * (float)i);
  if (do_m32) {
    // 4 x 32x32x2 f32 per iteration: the same 256 cycles as 8 x 16x16x4
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc32[i & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc32[i & 1], 0, 0, 0);
  } else if (do_bf) {
    // 16 x 16x16x32 bf16 (16 cycles each) per iteration
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[i & 7], 0, 0, 0);
  } else if (do_mfma && do_valu) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[i], acc[i], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 16; j += 2) x[j + (i & 1)] = fmaf(x[j + (i & 1)], a, b);
      }
    }
  } else if (do_mfma) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  } else if (do_valu) {
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 16; j += 2) x[j + (i & 1)] = fmaf(x[j + (i & 1)], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i];
  s += acc32[0][0] + acc32[1][5];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  const int blocks = 256, iters = 200000;
  float* o;
  hipMalloc(&o, blocks * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"A mfma, B idle", "A valu, B idle", "A mfma, B valu", "A mfma, B mfma",
                         "all: mfma+valu interleaved", "A mfma32x32x2, B idle",
                         "A mfma32x32x2, B valu", "A bf16 16x16x32, B idle", "A bf16, B valu"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 9; ++m) {
      hipEventRecord(e0);
      switch (m) {
        case 0: coexec<0><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 1: coexec<1><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 2: coexec<2><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 3: coexec<3><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 4: coexec<4><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 5: coexec<5><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 6: coexec<6><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        case 7: coexec<7><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
        default: coexec<8><<<blocks, 512>>>(o, iters, 1.0001f, 0.9999f); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // per wave and iteration: 8 MFMAs (32 cyc each = 256) and/or 64 v_fma_f32
      printf("mode %d %-28s %8.3f ms  %.1f ns/iter\n", m, names[m], ms, ms * 1e6 / iters);
    }
  return 0;
}
