// MFMA throughput microbenchmark (gfx950): back-to-back independent MFMAs in registers.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
// fp64 leg (the round-4 form read 49.2 TF/s while cov_syrk16_kernel
// already ran 62.8 on its SYRK count -- the loop was measuring accumulator copies): sweeps
// the independent accumulator chains per wave (ACC) and the waves per SIMD (blocks per CU),
// on per-lane operands that are not constants (the clock holds higher on trivial data,
// MI355X_MICROARCH.md DVFS item 1), and reports the best sustained rate of each form.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f16v __attribute__((ext_vector_type(16)));
typedef double d4v __attribute__((ext_vector_type(4)));

template <int ACC>
__global__ __launch_bounds__(256) void f32_loop(float* out, int iters, float a, float b) {
  f16v acc[ACC];
  for (int i = 0; i < ACC; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  const float av = a + 1e-3f * (threadIdx.x & 7), bv = b - 1e-3f * (threadIdx.x >> 5);
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i], 0, 0, 0);
  float s = 0.f;
  for (int i = 0; i < ACC; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int ACC>
__global__ __launch_bounds__(256) void f64_loop(double* out, int iters, double a, double b) {
  d4v acc[ACC];
  for (int i = 0; i < ACC; ++i) acc[i] = d4v{0, 0, 0, 0};
  // two operand pairs per lane, alternated between chains (not one broadcast constant)
  const double a0 = a + 1e-3 * (threadIdx.x & 7), a1 = a - 1e-3 * (threadIdx.x & 3);
  const double b0 = b - 1e-3 * (threadIdx.x >> 5), b1 = b + 2e-3 * (threadIdx.x >> 4);
  // tied in-place asm MFMA: the builtin's untied form made this loop copy every accumulator
  // VGPR -> AGPR -> VGPR around the MFMAs each iteration (64 VALU moves per 4 MFMAs: the
  // round-4 "ceiling" of 49.2 TF/s measured those moves); 12 + s_nop before the reads
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < ACC; ++i)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0"
                   : "+v"(acc[i]) : "v"((i & 1) ? a1 : a0), "v"((i & 2) ? b1 : b0));
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  double s = 0;
  for (int i = 0; i < ACC; ++i) for (int r = 0; r < 4; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int ACC>
static double run_f64(double* od, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f64_loop<ACC><<<blocks, 256>>>(od, iters / 10, 1.0001, 0.9999);  // warm-up
  hipEventRecord(e0);
  f64_loop<ACC><<<blocks, 256>>>(od, iters, 1.0001, 0.9999);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double fl = 2.0 * 16 * 16 * 4 * ACC * (double)iters * (blocks * 4.0);
  return fl / ms / 1e9;
}

int main() {
  int blocks = 256 * 8, iters = 20000;
  float* o;
  double* od;
  hipMalloc(&o, blocks * 256 * 4);
  hipMalloc(&od, (size_t)256 * 32 * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    f32_loop<4><<<blocks, 256>>>(o, iters, 1.0001f, 0.9999f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 32 * 32 * 2 * 4.0 * iters * (blocks * 4);
    printf("f32 32x32x2: %.1f TFLOP/s\n", fl / ms / 1e9);
  }
  // fp64 16x16x4: chains per wave x waves per SIMD (= 256-thread blocks per CU)
  double best = 0;
  for (int wps : {1, 2, 4, 8}) {
    const int nb = 256 * wps;
    const double t4 = run_f64<4>(od, nb, iters), t8 = run_f64<8>(od, nb, iters),
                 t16 = run_f64<16>(od, nb, iters);
    printf("f64 16x16x4: %d wave(s)/SIMD: 4 chains %.1f, 8 chains %.1f, 16 chains %.1f TFLOP/s\n",
           wps, t4, t8, t16);
    best = best > t4 ? best : t4;
    best = best > t8 ? best : t8;
    best = best > t16 ? best : t16;
  }
  printf("f64 16x16x4 best: %.1f TFLOP/s\n", best);
  return 0;
}
