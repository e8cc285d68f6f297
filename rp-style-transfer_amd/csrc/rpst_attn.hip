// SANet style attention (network/sanet.py:82-99) on fp32 MFMA, gfx950.
//
//   F = f(mvn(c)), G = g(mvn(s)), H = h(s)       (1x1 convs: rpst_conv.hip)
//   S = F^T G                  (B, HW, HW)        gemm #1  M=HW, N=HW, K=C
//   m_i = max_j S_ij, l_i = sum_j exp(S_ij - m_i)  rowstats (one wave per query row)
//   O = H softmax(S)^T         (B, C, HW)         gemm #2  M=C, N=HW, K=HW, with
//       exp(S_ij - m_i) applied while the B operand is staged into LDS and the 1/l_i
//       column scale applied in the epilogue: the probability matrix is never stored.
// No 1/sqrt(d) scaling (sanet.py:90-91). With C = 512 the QK^T operand per query is
// 2 KB, so materialising S (64 MiB per image at HW = 4096, 288 GB of HBM available)
// and streaming it twice costs ~20% of the MFMA time, far less than a flash-style
// kernel would lose to a 512-wide fp32 O accumulator per query tile.
//
// GEMM tile: 128 x 128 x 32, 256 threads = 2 x 2 waves of 64 x 64, v_mfma_f32_32x32x2_f32.
// Operands are staged k-major in LDS (As[k][m], Bs[k][n]) so the MFMA fragment reads
// are lane-contiguous; global tiles are loaded with 16-B loads along whichever dim is
// contiguous (RK: row-major rows with k contiguous; KR: k-rows with m/n contiguous).
// Register prefetch of tile t+1 overlaps the MFMAs of tile t.
#include "rpst_common.h"

namespace rpst {

enum { LAY_RK = 0, LAY_KR = 1 };

constexpr int kGBM = 128, kGBN = 128, kGBK = 32, kGPad = 4;

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* rowmax;    // EXPB: per-n max (B operand row index n)
  const float* colscale;  // optional per-n multiplier in the epilogue
  int M, N, K, lda, ldb, ldc;
  int64_t sA, sB, sC, sV;  // batch strides (elements); sV for rowmax / colscale
};

// Stage a kGBK x 128 tile of operand X (rows r0.., k0..) into registers.
template <int LAY, bool EXP, bool VEC>
__device__ __forceinline__ void g_load(float (&reg)[16], const float* __restrict__ X, int ld,
                                       int r0, int k0, int R, int K,
                                       const float* __restrict__ rmax, int tid) {
  if (LAY == LAY_KR) {
    // thread -> (k = tid>>5 + 8p, r4 = (tid&31)*4), 4 passes of 8 k-rows
    const int kk = tid >> 5, r = r0 + (tid & 31) * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int k = k0 + kk + 8 * p;
      if (VEC) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < K && r < R) v = *reinterpret_cast<const float4*>(X + (int64_t)k * ld + r);
        reg[4 * p + 0] = v.x;
        reg[4 * p + 1] = v.y;
        reg[4 * p + 2] = v.z;
        reg[4 * p + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          reg[4 * p + e] = (k < K && r + e < R) ? X[(int64_t)k * ld + r + e] : 0.f;
      }
    }
  } else {
    // thread -> (r = tid>>3 + 32p, k4 = (tid&7)*4), 4 passes of 32 rows
    const int rr = tid >> 3, k = k0 + (tid & 7) * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = r0 + rr + 32 * p;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (VEC) {
        if (r < R && k < K) {
          float4 q = *reinterpret_cast<const float4*>(X + (int64_t)r * ld + k);
          v[0] = q.x;
          v[1] = q.y;
          v[2] = q.z;
          v[3] = q.w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (r < R && k + e < K) ? X[(int64_t)r * ld + k + e] : 0.f;
      }
      if (EXP) {
        const float mx = r < R ? rmax[r] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (r < R && k + e < K) ? expf(v[e] - mx) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) reg[4 * p + e] = v[e];
    }
  }
}

template <int LAY>
__device__ __forceinline__ void g_store(float* __restrict__ Xs, const float (&reg)[16], int tid) {
  constexpr int LD = 128 + kGPad;
  if (LAY == LAY_KR) {
    const int kk = tid >> 5, r4 = (tid & 31) * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      *reinterpret_cast<float4*>(Xs + (kk + 8 * p) * LD + r4) =
          make_float4(reg[4 * p], reg[4 * p + 1], reg[4 * p + 2], reg[4 * p + 3]);
  } else {
    const int rr = tid >> 3, k4 = (tid & 7) * 4;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int e = 0; e < 4; ++e) Xs[(k4 + e) * LD + rr + 32 * p] = reg[4 * p + e];
  }
}

template <int ALAY, int BLAY, bool EXPB, bool VECA, bool VECB>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs g) {
  constexpr int LD = 128 + kGPad;
  __shared__ float As[kGBK * LD];
  __shared__ float Bs[kGBK * LD];
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * kGBM, n0 = blockIdx.x * kGBN;
  const float* A = g.A + b * g.sA;
  const float* B = g.B + b * g.sB;
  float* C = g.C + b * g.sC;
  const float* rmax = EXPB ? g.rowmax + b * g.sV : nullptr;
  const float* cscale = g.colscale ? g.colscale + b * g.sV : nullptr;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, j = lane & 31;

  floatx16 acc[2][2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  float ra[16], rb[16];
  const int ktiles = (g.K + kGBK - 1) / kGBK;
  g_load<ALAY, false, VECA>(ra, A, g.lda, m0, 0, g.M, g.K, nullptr, tid);
  g_load<BLAY, EXPB, VECB>(rb, B, g.ldb, n0, 0, g.N, g.K, rmax, tid);
  for (int kt = 0; kt < ktiles; ++kt) {
    g_store<ALAY>(As, ra, tid);
    g_store<BLAY>(Bs, rb, tid);
    __syncthreads();
    if (kt + 1 < ktiles) {
      g_load<ALAY, false, VECA>(ra, A, g.lda, m0, (kt + 1) * kGBK, g.M, g.K, nullptr, tid);
      g_load<BLAY, EXPB, VECB>(rb, B, g.ldb, n0, (kt + 1) * kGBK, g.N, g.K, rmax, tid);
    }
#pragma unroll
    for (int kk = 0; kk < kGBK / 2; ++kk) {
      float av[2], bv[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) av[mt] = As[(2 * kk + h) * LD + wm * 64 + mt * 32 + j];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) bv[nt] = Bs[(2 * kk + h) * LD + wn * 64 + nt * 32 + j];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mt], bv[nt], acc[mt][nt], 0, 0, 0);
    }
    __syncthreads();
  }

#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = n0 + wn * 64 + nt * 32 + j;
    if (n >= g.N) continue;
    const float cs = cscale ? cscale[n] : 1.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < g.M) C[(int64_t)m * g.ldc + n] = acc[mt][nt][r] * cs;
      }
  }
}

// Row max and 1 / sum exp(x - max) of `rows` rows of length L (one wave per row).
__global__ __launch_bounds__(256) void rowstats_kernel(const float* __restrict__ S,
                                                       float* __restrict__ rmax,
                                                       float* __restrict__ rinv, int64_t rows,
                                                       int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * L;
  float mx = -INFINITY;
  if ((L & 3) == 0) {
    for (int i = lane * 4; i < L; i += 256) {
      float4 v = *reinterpret_cast<const float4*>(s + i);
      mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
  } else {
    for (int i = lane; i < L; i += 64) mx = fmaxf(mx, s[i]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  if ((L & 3) == 0) {
    for (int i = lane * 4; i < L; i += 256) {
      float4 v = *reinterpret_cast<const float4*>(s + i);
      sum += (expf(v.x - mx) + expf(v.y - mx)) + (expf(v.z - mx) + expf(v.w - mx));
    }
  } else {
    for (int i = lane; i < L; i += 64) sum += expf(s[i] - mx);
  }
  sum = wave_sum(sum);
  if (lane == 0) {
    rmax[row] = mx;
    rinv[row] = 1.f / sum;
  }
}

template <int ALAY, int BLAY, bool EXPB>
static void launch_gemm(const GemmArgs& g, int batch, hipStream_t st) {
  dim3 grid((g.N + kGBN - 1) / kGBN, (g.M + kGBM - 1) / kGBM, batch);
  auto aligned = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // 16-B loads need the contiguous dim, the leading dim and the batch stride % 4 == 0
  const bool va = aligned(g.A) && (g.lda % 4 == 0) && (g.sA % 4 == 0) &&
                  ((ALAY == LAY_KR) ? (g.M % 4 == 0) : (g.K % 4 == 0));
  const bool vb = aligned(g.B) && (g.ldb % 4 == 0) && (g.sB % 4 == 0) &&
                  ((BLAY == LAY_KR) ? (g.N % 4 == 0) : (g.K % 4 == 0));
  if (va && vb)
    gemm_f32_kernel<ALAY, BLAY, EXPB, true, true><<<grid, 256, 0, st>>>(g);
  else
    gemm_f32_kernel<ALAY, BLAY, EXPB, false, false><<<grid, 256, 0, st>>>(g);
}

}  // namespace rpst

using namespace rpst;

extern "C" size_t rpst_sanet_attention_workspace_size(int B, int HW) {
  if (B <= 0 || HW <= 0) return 0;
  return sizeof(float) * ((size_t)B * HW * HW + 2 * (size_t)B * HW);
}

extern "C" int rpst_sanet_attention(const float* F, const float* G, const float* H, float* O,
                                    int B, int C, int HW, void* workspace,
                                    size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(F && G && H && O, "sanet_attention: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HW > 0, "sanet_attention: bad shape B=%d C=%d HW=%d", B, C, HW);
  RPST_REQUIRE(B <= 65535, "sanet_attention: batch too large");
  if (!workspace || workspace_bytes < rpst_sanet_attention_workspace_size(B, HW)) {
    set_error("sanet_attention: workspace %zu < %zu bytes", workspace_bytes,
              rpst_sanet_attention_workspace_size(B, HW));
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* S = static_cast<float*>(workspace);
  float* rmax = S + (size_t)B * HW * HW;
  float* rinv = rmax + (size_t)B * HW;
  const int64_t fhw = (int64_t)C * HW;
  // S[b][i][j] = sum_c F[b][c][i] G[b][c][j]
  GemmArgs g1{F, G, S, nullptr, nullptr, HW, HW, C, HW, HW, HW, fhw, fhw, (int64_t)HW * HW, 0};
  launch_gemm<LAY_KR, LAY_KR, false>(g1, B, st);
  if (int e = launch_status("gemm_f32_kernel(S=F^T G)")) return e;
  const int64_t rows = (int64_t)B * HW;
  rowstats_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(S, rmax, rinv, rows, HW);
  if (int e = launch_status("rowstats_kernel")) return e;
  // O[b][c][i] = (1/l_i) sum_j H[b][c][j] exp(S[b][i][j] - m_i)
  GemmArgs g2{H, S, O, rmax, rinv, C, HW, HW, HW, HW, HW, fhw, (int64_t)HW * HW, fhw, HW};
  launch_gemm<LAY_RK, LAY_RK, true>(g2, B, st);
  return launch_status("gemm_f32_kernel(O=H P^T)");
}
