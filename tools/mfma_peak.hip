// MFMA throughput microbenchmark (gfx950): back-to-back independent MFMAs in registers.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f16v __attribute__((ext_vector_type(16)));
typedef double d4v __attribute__((ext_vector_type(4)));

template <int ACC>
__global__ __launch_bounds__(256) void f32_loop(float* out, int iters, float a, float b) {
  f16v acc[ACC];
  for (int i = 0; i < ACC; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  float s = 0.f;
  for (int i = 0; i < ACC; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int ACC>
__global__ __launch_bounds__(256) void f64_loop(double* out, int iters, double a, double b) {
  d4v acc[ACC];
  for (int i = 0; i < ACC; ++i) acc[i] = d4v{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  double s = 0;
  for (int i = 0; i < ACC; ++i) for (int r = 0; r < 4; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int blocks = 256 * 8, iters = 20000;
  float* o; double* od;
  hipMalloc(&o, blocks * 256 * 4); hipMalloc(&od, blocks * 256 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    f32_loop<4><<<blocks, 256>>>(o, iters, 1.0001f, 0.9999f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 32 * 32 * 2 * 4.0 * iters * (blocks * 4);
    printf("f32 32x32x2: %.1f TFLOP/s\n", fl / ms / 1e9);
    hipEventRecord(e0);
    f64_loop<4><<<blocks, 256>>>(od, iters, 1.0001, 0.9999);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    fl = 2.0 * 16 * 16 * 4 * 4.0 * iters * (blocks * 4);
    printf("f64 16x16x4: %.1f TFLOP/s\n", fl / ms / 1e9);
  }
  return 0;
}
