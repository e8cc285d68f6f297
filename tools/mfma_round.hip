// Rounding of fp32 MFMA accumulation chains (gfx950): C (16 x 16) = sum over K of A B on a
// chain of v_mfma_f32_16x16x4_f32 (K = 4 per MFMA), against the same sums as a VALU fmaf
// chain in k order and a float64 host reference: mean signed error (bias) and RMS error,
// relative to |C|, for mixed-sign and all-positive products (a truncating accumulator shows
// as a bias on the latter).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_round.hip -o /tmp/mfma_round && /tmp/mfma_round
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
typedef float f4v __attribute__((ext_vector_type(4)));

// A: [K][16] (m fastest), B: [K][16] (n fastest); one wave per 16 x 16 problem
__global__ __launch_bounds__(64) void chain(const float* A, const float* B, float* Cm, float* Cv,
                                            int K) {
  const int l = threadIdx.x, m = l & 15, kq = l >> 4;
  const float* a = A + (size_t)blockIdx.x * K * 16;
  const float* b = B + (size_t)blockIdx.x * K * 16;
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 4)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(k0 + kq) * 16 + m], b[(k0 + kq) * 16 + m], acc,
                                               0, 0, 0);
  for (int r = 0; r < 4; ++r) Cm[(size_t)blockIdx.x * 256 + (4 * kq + r) * 16 + m] = acc[r];
  // VALU: lane l computes C[mm][n] for mm = 4 kq + r, n = m, k in order
  for (int r = 0; r < 4; ++r) {
    const int mm = 4 * kq + r;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = fmaf(a[k * 16 + mm], b[k * 16 + m], s);
    Cv[(size_t)blockIdx.x * 256 + mm * 16 + m] = s;
  }
}

int main() {
  const int P = 256;  // problems
  for (int pos = 0; pos < 2; ++pos)
    for (int K : {64, 512, 4608}) {
      std::mt19937 rng(K + pos);
      std::uniform_real_distribution<float> u(pos ? 0.f : -1.f, 1.f);
      std::vector<float> A((size_t)P * K * 16), B((size_t)P * K * 16);
      for (auto& v : A) v = u(rng);
      for (auto& v : B) v = u(rng);
      float *dA, *dB, *dM, *dV;
      hipMalloc(&dA, A.size() * 4);
      hipMalloc(&dB, B.size() * 4);
      hipMalloc(&dM, (size_t)P * 256 * 4);
      hipMalloc(&dV, (size_t)P * 256 * 4);
      hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
      chain<<<P, 64>>>(dA, dB, dM, dV, K);
      std::vector<float> M((size_t)P * 256), V((size_t)P * 256);
      hipMemcpy(M.data(), dM, M.size() * 4, hipMemcpyDeviceToHost);
      hipMemcpy(V.data(), dV, V.size() * 4, hipMemcpyDeviceToHost);
      double bm = 0, bv = 0, rm = 0, rv = 0, nrm = 0;
      for (int p = 0; p < P; ++p)
        for (int mm = 0; mm < 16; ++mm)
          for (int n = 0; n < 16; ++n) {
            double ex = 0;
            for (int k = 0; k < K; ++k)
              ex += (double)A[((size_t)p * K + k) * 16 + mm] * B[((size_t)p * K + k) * 16 + n];
            const size_t o = (size_t)p * 256 + mm * 16 + n;
            bm += M[o] - ex;
            bv += V[o] - ex;
            rm += (M[o] - ex) * (M[o] - ex);
            rv += (V[o] - ex) * (V[o] - ex);
            nrm += ex * ex;
          }
      const double cnt = (double)P * 256, rmsC = std::sqrt(nrm / cnt);
      printf("%s K=%5d  MFMA bias %+.2e rms %.2e | VALU fmaf bias %+.2e rms %.2e  (rel. to rms|C|)\n",
             pos ? "positive" : "mixed   ", K, bm / cnt / rmsC, std::sqrt(rm / cnt) / rmsC,
             bv / cnt / rmsC, std::sqrt(rv / cnt) / rmsC);
      hipFree(dA);
      hipFree(dB);
      hipFree(dM);
      hipFree(dV);
    }
  return 0;
}
