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
#include <algorithm>
#include <cstdlib>

#include "rpst_common.h"

namespace rpst {

// flash-style forward attention (rpst_flash.hip)
bool sanet_flash_ok(int C, int HW);
int sanet_flash(const float* F, const float* G, const float* H, float* O, int B, int C, int HW,
                hipStream_t st);
int adaptive_flash_stats(const float* F, const float* G, int B, int C, int HW, float* rm,
                         float* rinv, hipStream_t st);
int adaptive_flash_apply(const float* F, const float* G, const float* H, float* O, int B, int C,
                         int HW, const float* rm, const float* rinv, const float* clamp, int mode,
                         float scale, hipStream_t st);

enum { LAY_RK = 0, LAY_KR = 1 };

constexpr int kGBN = 128, kGBK = 32, kGPad = 4;  // M tile: 128 * MW (gemm_f32_kernel)

// B-operand staging transforms (applied to S while it is staged; row r = query index):
//   BX_NONE   v
//   BX_EXP    exp(v - m_r)                                  softmax numerator (SANet)
//   BX_AEA    sigmoid(scale (exp(v - m_r) inv_r - c_r))     AEAModule clamp (sanet.py:45-47)
//   BX_AEAR   exp(relu(exp(v - m_r) inv_r - c_r) - m2_r)    AEALReluModule (sanet.py:66-69),
//             numerator of softmax(relu(P - c)); 1/l2_r is the epilogue column scale
//   BX_PROB   exp(v - m_r) inv_r                            softmax probability (attention
//             backward: dH = dO P with P formed while S is staged, never stored)
//   BX_AEARQ  BX_AEAR * inv2_r                              the normalised AEALRelu attention
//             (AdaptiveSANet backward: dH = dO Q)
enum { BX_NONE = 0, BX_EXP = 1, BX_AEA = 2, BX_AEAR = 3, BX_PROB = 4, BX_AEARQ = 5 };
template <int BX> constexpr bool bx_inv() { return BX == BX_AEA || BX == BX_AEAR || BX == BX_PROB || BX == BX_AEARQ; }
template <int BX> constexpr bool bx_clamp() { return BX == BX_AEA || BX == BX_AEAR || BX == BX_AEARQ; }
template <int BX> constexpr bool bx_m2() { return BX == BX_AEAR || BX == BX_AEARQ; }

// Per-row vectors of the B operand's transform (each indexed batch * sV + r).
struct RowVec {
  const float* m;      // row max of S
  const float* inv;    // 1 / sum exp(S - m)
  const float* clamp;  // AEA threshold per query row
  const float* m2;     // BX_AEAR: row max of relu(P - c)
  float scale;         // BX_AEA: sigmoid slope (scale_value)
  const float* inv2;   // BX_AEARQ: 1 / sum exp(relu(P - c) - m2)
};

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  RowVec rv;              // B-operand transform vectors (BX_* != BX_NONE)
  const float* colscale;  // optional per-n multiplier in the epilogue
  const float* colbias;   // optional per-n bias added after the scale (nn.Linear bias)
  int act;                // epilogue activation: 0 none, 1 LeakyReLU(0.2)
  int M, N, K, lda, ldb, ldc;
  int64_t sA, sB, sC, sV;  // batch strides (elements); sV for the row / column vectors
  // In-kernel split-K (BX_NONE only): grid z = batch * ks, z -> (batch z / ks, K chunk z % ks
  // of kc elements); C advances by sC per z, so each chunk writes its own partial.
  int ks = 1, kc = 0;
  int accum = 0;  // epilogue adds to C (a sum over launches, in launch order)
};

template <int BX>
__device__ __forceinline__ float bx_apply(float v, float m, float inv, float c, float m2,
                                          float scale, float inv2 = 1.f) {
  if (BX == BX_EXP) return expf(v - m);
  if (BX == BX_AEA) {
    const float p = expf(v - m) * inv;
    return 1.f / (1.f + expf(-(scale * (p - c))));
  }
  if (BX == BX_AEAR) {
    const float p = expf(v - m) * inv;
    return expf(fmaxf(p - c, 0.f) - m2);
  }
  if (BX == BX_PROB) return expf(v - m) * inv;
  if (BX == BX_AEARQ) {
    const float p = expf(v - m) * inv;
    return expf(fmaxf(p - c, 0.f) - m2) * inv2;
  }
  return v;
}

// Stage a kGBK x 128 tile of operand X (rows r0.., k0..) into registers.
template <int LAY, int BX, bool VEC>
__device__ __forceinline__ void g_load(float (&reg)[16], const float* __restrict__ X, int ld,
                                       int r0, int k0, int R, int K, const RowVec& rv,
                                       int64_t voff, int tid) {
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
      if (BX != BX_NONE) {  // KR staging: the row of S (the query) is the k index
        const int64_t q = voff + (k < K ? k : 0);
        const float mx = rv.m[q];
        const float inv = bx_inv<BX>() ? rv.inv[q] : 0.f;
        const float cl = bx_clamp<BX>() ? rv.clamp[q] : 0.f;
        const float m2 = bx_m2<BX>() ? rv.m2[q] : 0.f;
        const float i2 = BX == BX_AEARQ ? rv.inv2[q] : 1.f;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          reg[4 * p + e] = (k < K && r + e < R)
                               ? bx_apply<BX>(reg[4 * p + e], mx, inv, cl, m2, rv.scale, i2)
                               : 0.f;
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
      if (BX != BX_NONE) {
        const int64_t q = voff + (r < R ? r : 0);
        const float mx = rv.m[q];
        const float inv = bx_inv<BX>() ? rv.inv[q] : 0.f;
        const float cl = bx_clamp<BX>() ? rv.clamp[q] : 0.f;
        const float m2 = bx_m2<BX>() ? rv.m2[q] : 0.f;
        const float i2 = BX == BX_AEARQ ? rv.inv2[q] : 1.f;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[e] = (r < R && k + e < K) ? bx_apply<BX>(v[e], mx, inv, cl, m2, rv.scale, i2) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) reg[4 * p + e] = v[e];
    }
  }
}

// LDS row stride of a staged operand: RK tiles are written transposed (4 k of one row per
// thread), so their stride is odd (129: 2-way bank conflicts on those scalar stores instead
// of 4-way at 132); KR tiles keep 132 for their 16-B stores. (Measured: S = F^T G + O at
// B = 32, C = 512, HW = 4096: 10.54 -> 10.33 ms, tools/bench_attn.py; a 64-deep k tile
// (11.2 ms) and double-buffered LDS with the exp applied at the LDS store (11.2 ms) were
// slower.)
template <int LAY, int W = 128>
constexpr int g_ld() { return LAY == LAY_RK ? W + 1 : W + kGPad; }

template <int LAY, int LD = g_ld<LAY>()>
__device__ __forceinline__ void g_store(float* __restrict__ Xs, const float (&reg)[16], int tid) {
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

// MW = 2: 256-row M tiles (each wave 128 x 64): the B tile (and, for the attention, its
// exp / AEA transform) is staged once per 256 rows of A instead of per 128
template <int ALAY, int BLAY, int BX, bool VECA, bool VECB, int MW>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs g) {
  constexpr int BMT = 128 * MW;
  constexpr int LDA = g_ld<ALAY, BMT>(), LDB = g_ld<BLAY>();
  __shared__ float As[kGBK * LDA];
  __shared__ float Bs[kGBK * LDB];
  int b = blockIdx.z, K = g.K;
  int64_t koA = 0, koB = 0;
  if (g.ks > 1) {
    const int kb = (b % g.ks) * g.kc;
    b /= g.ks;
    K = min(g.kc, g.K - kb);
    koA = ALAY == LAY_RK ? kb : (int64_t)kb * g.lda;
    koB = BLAY == LAY_RK ? kb : (int64_t)kb * g.ldb;
  }
  const int m0 = blockIdx.y * BMT, n0 = blockIdx.x * kGBN;
  const float* A = g.A + b * g.sA + koA;
  const float* B = g.B + b * g.sB + koB;
  float* C = g.C + (int64_t)blockIdx.z * g.sC;
  const int64_t voff = (int64_t)b * g.sV;
  const float* cscale = g.colscale ? g.colscale + voff : nullptr;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, j = lane & 31;

  floatx16 acc[2 * MW][2];
#pragma unroll
  for (int mt = 0; mt < 2 * MW; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  float ra[MW][16], rb[16];
  const int ktiles = (K + kGBK - 1) / kGBK;
#pragma unroll
  for (int i = 0; i < MW; ++i)
    g_load<ALAY, BX_NONE, VECA>(ra[i], A, g.lda, m0 + 128 * i, 0, g.M, K, g.rv, 0, tid);
  g_load<BLAY, BX, VECB>(rb, B, g.ldb, n0, 0, g.N, K, g.rv, voff, tid);
  for (int kt = 0; kt < ktiles; ++kt) {
#pragma unroll
    for (int i = 0; i < MW; ++i) g_store<ALAY, LDA>(As + 128 * i, ra[i], tid);
    g_store<BLAY, LDB>(Bs, rb, tid);
    __syncthreads();
    if (kt + 1 < ktiles) {
#pragma unroll
      for (int i = 0; i < MW; ++i)
        g_load<ALAY, BX_NONE, VECA>(ra[i], A, g.lda, m0 + 128 * i, (kt + 1) * kGBK, g.M, K,
                                    g.rv, 0, tid);
      g_load<BLAY, BX, VECB>(rb, B, g.ldb, n0, (kt + 1) * kGBK, g.N, K, g.rv, voff, tid);
    }
#pragma unroll
    for (int kk = 0; kk < kGBK / 2; ++kk) {
      float av[2 * MW], bv[2];
#pragma unroll
      for (int mt = 0; mt < 2 * MW; ++mt)
        av[mt] = As[(2 * kk + h) * LDA + wm * 64 * MW + mt * 32 + j];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) bv[nt] = Bs[(2 * kk + h) * LDB + wn * 64 + nt * 32 + j];
#pragma unroll
      for (int mt = 0; mt < 2 * MW; ++mt)
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
    const float cb = g.colbias ? g.colbias[n] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 2 * MW; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 * MW + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float v = acc[mt][nt][r] * cs;
        if (g.colbias) v += cb;
        if (g.act == 1) v = v > 0.f ? v : 0.2f * v;
        if (m < g.M) {
          float* cp = C + (int64_t)m * g.ldc + n;
          *cp = g.accum ? *cp + v : v;
        }
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

template <int ALAY, int BLAY, int BX>
static void launch_gemm(const GemmArgs& g, int batch, hipStream_t st) {
  static const int mw_env = [] {
    const char* e = std::getenv("RPST_GEMM_MW");  // A/B: 1 = 128-row tiles everywhere
    return e && *e ? std::atoi(e) : 0;
  }();
  const int mw = mw_env == 1 ? 1 : (g.M >= 256 ? 2 : 1);
  dim3 grid((g.N + kGBN - 1) / kGBN, (g.M + 128 * mw - 1) / (128 * mw), batch * g.ks);
  auto aligned = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // 16-B loads need the contiguous dim, the leading dim and the batch stride % 4 == 0
  const bool va = aligned(g.A) && (g.lda % 4 == 0) && (g.sA % 4 == 0) && (g.kc % 4 == 0) &&
                  ((ALAY == LAY_KR) ? (g.M % 4 == 0) : (g.K % 4 == 0));
  const bool vb = aligned(g.B) && (g.ldb % 4 == 0) && (g.sB % 4 == 0) && (g.kc % 4 == 0) &&
                  ((BLAY == LAY_KR) ? (g.N % 4 == 0) : (g.K % 4 == 0));
  if (mw == 2) {
    if (va && vb) gemm_f32_kernel<ALAY, BLAY, BX, true, true, 2><<<grid, 256, 0, st>>>(g);
    else gemm_f32_kernel<ALAY, BLAY, BX, false, false, 2><<<grid, 256, 0, st>>>(g);
  } else {
    if (va && vb) gemm_f32_kernel<ALAY, BLAY, BX, true, true, 1><<<grid, 256, 0, st>>>(g);
    else gemm_f32_kernel<ALAY, BLAY, BX, false, false, 1><<<grid, 256, 0, st>>>(g);
  }
}


// ---- SANet attention backward (sanet.py:86-94 under autograd) ---------------------------
// dS = P (dP - rowsum(dP P)) with P = exp(S - m) inv formed from the logits (P is never
// stored); in place over dP. One wave per row, fixed-order sums. rowsum(dP P) is divided by
// the row's own sum of P (1 up to fp32 rounding), so each row of dS sums to zero to fp32
// rounding: the softmax's shift invariance (the SANet g.bias gradient is exactly zero in exact
// arithmetic) survives the recomputed P.
__global__ __launch_bounds__(256) void softmax_bwd_logits_kernel(const float* __restrict__ S,
                                                                 const float* __restrict__ rmax,
                                                                 const float* __restrict__ rinv,
                                                                 float* __restrict__ dP,
                                                                 int64_t rows, int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * L;
  float* d = dP + row * L;
  const float m = rmax[row], inv = rinv[row];
  float dot = 0.f, psum = 0.f;
  for (int i = lane; i < L; i += 64) {
    const float p = expf(s[i] - m) * inv;
    dot = fmaf(d[i], p, dot);
    psum += p;
  }
  dot = wave_sum(dot) / wave_sum(psum);
  for (int i = lane; i < L; i += 64) d[i] = expf(s[i] - m) * inv * (d[i] - dot);
}

// out[i] = sum_b in[b][i] (fixed order over b)
__global__ void batch_sum_kernel(const float* __restrict__ in, float* __restrict__ out,
                                 int64_t per, int nb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += in[(int64_t)b * per + i];
  out[i] = s;
}

// db[c] = sum_{b, p} dy[b][c][p]: one block per channel (a launch of C blocks fills the chip
// at the SANet's 512 channels; one wave per channel ran 88 us for a 64 MB read), 16-B loads
// when the planes allow, fixed order: per-thread strided sums, wave sums, then the four
// waves in order
__global__ __launch_bounds__(256) void channel_sum_kernel(const float* __restrict__ dy,
                                                          float* __restrict__ db, int nb, int C,
                                                          int64_t HW) {
  __shared__ float part[4];
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const bool vec = (HW & 3) == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) {
    const float* p = dy + ((int64_t)b * C + c) * HW;
    if (vec) {
      for (int64_t i = 4 * tid; i < HW; i += 1024) {
        const float4 v = *reinterpret_cast<const float4*>(p + i);
        s += (v.x + v.y) + (v.z + v.w);
      }
    } else {
      for (int64_t i = tid; i < HW; i += 256) s += p[i];
    }
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) part[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) db[c] = ((part[0] + part[1]) + part[2]) + part[3];
}

// chunk-local row vectors of a query chunk: dst[b][i] = src[b][q0 + i] and back
__global__ void rows_gather_kernel(const float* __restrict__ src, float* __restrict__ dst, int B,
                                   int HW, int q0, int n) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * n) return;
  const int64_t b = t / n;
  dst[t] = src[b * HW + q0 + (t - b * n)];
}
__global__ void rows_scatter_kernel(const float* __restrict__ src, float* __restrict__ dst, int B,
                                    int HW, int q0, int n) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)B * n) return;
  const int64_t b = t / n;
  dst[b * HW + q0 + (t - b * n)] = src[t];
}

// ---- AdaptiveSANet backward (sanet.py:100-138 under autograd; train.py:118-119 trains it) --
// Row pass from dQ (the gradient at the clamped attention) to dS (the gradient at the logits,
// in place over dQ) and dc (at the per-query clamp value):
//   aea  Q = sigmoid(scale (P - c)):      dP = dQ scale Q (1 - Q)
//   relu Q = softmax(relu(P - c)):        dR = Q (dQ - rowsum(dQ Q)), dP = dR [P > c]
//   dc = -sum_j dP, dS = P (dP - rowsum(dP P))   (P = softmax(S), from the logits)
// One wave per row; the row sums are divided by the row's own sum of P / Q (1 to rounding) as
// in softmax_bwd_logits_kernel.
__global__ __launch_bounds__(256) void aea_bwd_rows_kernel(const float* __restrict__ S,
                                                           RowVec rv, float* __restrict__ dQ,
                                                           float* __restrict__ dc, int mode,
                                                           int64_t rows, int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * L;
  float* d = dQ + row * L;
  const float m = rv.m[row], inv = rv.inv[row], c = rv.clamp[row], scale = rv.scale;
  const float m2 = mode == 1 ? rv.m2[row] : 0.f, i2 = mode == 1 ? rv.inv2[row] : 0.f;
  float dq_dot = 0.f;  // relu: rowsum(dQ Q) / rowsum(Q)
  if (mode == 1) {
    float dot = 0.f, qs = 0.f;
    for (int i = lane; i < L; i += 64) {
      const float p = expf(s[i] - m) * inv;
      const float q = expf(fmaxf(p - c, 0.f) - m2) * i2;
      dot = fmaf(d[i], q, dot);
      qs += q;
    }
    dq_dot = wave_sum(dot) / wave_sum(qs);
  }
  auto dp_of = [&](float p, float g) {
    if (mode == 0) {
      const float q = 1.f / (1.f + expf(-(scale * (p - c))));
      return g * scale * q * (1.f - q);
    }
    const float q = expf(fmaxf(p - c, 0.f) - m2) * i2;
    return p - c > 0.f ? q * (g - dq_dot) : 0.f;
  };
  float dot = 0.f, ps = 0.f, dcs = 0.f;
  for (int i = lane; i < L; i += 64) {
    const float p = expf(s[i] - m) * inv;
    const float dp = dp_of(p, d[i]);
    dot = fmaf(dp, p, dot);
    ps += p;
    dcs += dp;
  }
  dot = wave_sum(dot) / wave_sum(ps);
  dcs = wave_sum(dcs);
  for (int i = lane; i < L; i += 64) {
    const float p = expf(s[i] - m) * inv;
    d[i] = p * (dp_of(p, d[i]) - dot);
  }
  if (lane == 0) dc[row] = -dcs;
}

// f_psi backward, per query row k (= b * HW + i): t = Z_k . w2 + b2 recomputed in the order
// clamp_head_kernel used; dt = dc * head'(t) (aea: interval sigmoid'(t), relu: (1 - tanh^2)/2);
// du[k][n] = dt w2[n] LeakyReLU'(Z[k][n]) (Z = LeakyReLU(u): u > 0 iff Z > 0). One wave per row.
__global__ __launch_bounds__(256) void fpsi_bwd_rows_kernel(const float* __restrict__ Z,
                                                            const float* __restrict__ w2,
                                                            const float* __restrict__ b2,
                                                            const float* __restrict__ dc,
                                                            float* __restrict__ dt,
                                                            float* __restrict__ du, int64_t rows,
                                                            int hid, int mode, float interval) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* z = Z + row * hid;
  float acc = 0.f;
  for (int n = lane; n < hid; n += 64) acc = fmaf(z[n], w2[n], acc);
  acc = wave_sum(acc);
  const float t = acc + b2[0];
  float g;
  if (mode == 0) {
    const float sg = 1.f / (1.f + expf(-t));
    g = dc[row] * interval * sg * (1.f - sg);
  } else {
    const float th = tanhf(t);
    g = dc[row] * 0.5f * (1.f - th * th);
  }
  float* u = du + row * hid;
  for (int n = lane; n < hid; n += 64) u[n] = g * w2[n] * (z[n] > 0.f ? 1.f : 0.2f);
  if (lane == 0) dt[row] = g;
}

// Column sums of the f_psi backward over all B * HW query rows, in two fixed-order passes:
// part[(c * 3 + s) * (hid + 1) + n] over the 128-row chunk c (s = 0: sum dt Z[.][n] -> dw2,
// s = 1: sum du[.][n] -> db1, column hid of s = 2: sum dt -> db2), then the chunks in order.
// (The single-pass form ran 257 threads over all rows: latency-bound on two CUs.)
constexpr int kColChunk = 128;
__global__ __launch_bounds__(256) void fpsi_colsum_part_kernel(
    const float* __restrict__ Z, const float* __restrict__ du, const float* __restrict__ dt,
    float* __restrict__ part, int64_t rows, int hid) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (n > hid) return;
  const int64_t k0 = (int64_t)c * kColChunk;
  const int64_t k1 = rows < k0 + kColChunk ? rows : k0 + kColChunk;
  float a = 0.f, b = 0.f;
  if (n == hid) {
    for (int64_t k = k0; k < k1; ++k) a += dt[k];
  } else {
    for (int64_t k = k0; k < k1; ++k) {
      a = fmaf(dt[k], Z[k * hid + n], a);
      b += du[k * hid + n];
    }
  }
  float* p = part + (int64_t)c * 3 * (hid + 1);
  if (n == hid) {
    p[2 * (hid + 1) + n] = a;
  } else {
    p[n] = a;
    p[(hid + 1) + n] = b;
  }
}

__global__ void fpsi_colsum_final_kernel(const float* __restrict__ part, float* __restrict__ dw2,
                                         float* __restrict__ db1, float* __restrict__ db2,
                                         int chunks, int hid) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n > hid) return;
  float a = 0.f, b = 0.f;
  for (int c = 0; c < chunks; ++c) {
    const float* p = part + (int64_t)c * 3 * (hid + 1);
    if (n == hid) {
      a += p[2 * (hid + 1) + n];
    } else {
      a += p[n];
      b += p[(hid + 1) + n];
    }
  }
  if (n == hid) {
    db2[0] = a;
  } else {
    dw2[n] = a;
    db1[n] = b;
  }
}

// ---- AdaptiveSANet (sanet.py:12-18, 26-71, 100-138) -----------------------------------
// functional.normalize(x, dim=1): x / max(||x||_2 over channels, 1e-12), per position.
// Block = 64 consecutive positions (of one image) x 4 channel quarters (one wave each; a
// wave reads 64 consecutive positions of one channel row per load: coalesced); each lane
// sums its quarter's squares in fp64 over 4 interleaved chains, the quarters are combined in
// order through LDS, and every lane scales its quarter by the one reciprocal of the norm (one
// rounding more than the division: <= 1 ulp). (The thread-per-position form with a serial
// fp64 chain and a division per element took 0.49 ms per call at B = 32, C = 512, HW = 4096.)
__global__ __launch_bounds__(256) void colnorm_kernel(const float* __restrict__ x,
                                                      float* __restrict__ out, int B, int C,
                                                      int HW) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, qtr = threadIdx.x >> 6;
  const int pblocks = (HW + 63) / 64;
  const int64_t b = blockIdx.x / pblocks;
  const int i = (int)(blockIdx.x - b * pblocks) * 64 + lane;
  const bool ok = i < HW;
  const int c0 = (int)((int64_t)C * qtr / 4), c1 = (int)((int64_t)C * (qtr + 1) / 4);
  const float* xp = x + b * C * (int64_t)HW + (ok ? i : 0);
  double ss[4] = {0.0, 0.0, 0.0, 0.0};
  if (ok) {
    int c = c0;
    for (; c + 4 <= c1; c += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double v = xp[(int64_t)(c + u) * HW];
        ss[u] = fma(v, v, ss[u]);
      }
    }
    for (; c < c1; ++c) {
      const double v = xp[(int64_t)c * HW];
      ss[0] = fma(v, v, ss[0]);
    }
  }
  part[qtr][lane] = (ss[0] + ss[1]) + (ss[2] + ss[3]);
  __syncthreads();
  if (!ok) return;
  const double tot = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
  const float r = 1.f / fmaxf((float)sqrt(tot), 1e-12f);
  float* op = out + b * C * (int64_t)HW + i;
  for (int c = c0; c < c1; ++c) op[(int64_t)c * HW] = xp[(int64_t)c * HW] * r;
}

// f_psi's last Linear(hid -> 1) + head: AEA  clamp = sigmoid(t) * interval + from
// (sanet.py:45); AEALRelu  clamp = (tanh(t) + 1) / 2 (sanet.py:66). One wave per row.
__global__ __launch_bounds__(256) void clamp_head_kernel(const float* __restrict__ Z,
                                                         const float* __restrict__ w2,
                                                         const float* __restrict__ b2,
                                                         float* __restrict__ clamp,
                                                         int64_t rows, int hid, int mode,
                                                         float from, float interval) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* z = Z + row * hid;
  float acc = 0.f;
  for (int n = lane; n < hid; n += 64) acc = fmaf(z[n], w2[n], acc);
  acc = wave_sum(acc);
  if (lane == 0) {
    const float t = acc + b2[0];
    clamp[row] = mode == 0 ? (1.f / (1.f + expf(-t))) * interval + from : (tanhf(t) + 1.f) / 2.f;
  }
}

// AEALRelu second softmax: per row, m2 = max_j relu(P_ij - c_i), inv2 = 1 / sum_j
// exp(relu(P_ij - c_i) - m2), with P_ij = exp(S_ij - m_i) inv_i formed exactly as the
// GEMM staging forms it. One wave per row.
__global__ __launch_bounds__(256) void rowstats_relu_kernel(
    const float* __restrict__ S, const float* __restrict__ rmax, const float* __restrict__ rinv,
    const float* __restrict__ clamp, float* __restrict__ m2, float* __restrict__ inv2,
    int64_t rows, int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * L;
  const float m = rmax[row], inv = rinv[row], c = clamp[row];
  float mx = -INFINITY;
  for (int i = lane; i < L; i += 64) mx = fmaxf(mx, fmaxf(expf(s[i] - m) * inv - c, 0.f));
  mx = wave_max(mx);
  float sum = 0.f;
  for (int i = lane; i < L; i += 64) sum += expf(fmaxf(expf(s[i] - m) * inv - c, 0.f) - mx);
  sum = wave_sum(sum);
  if (lane == 0) {
    m2[row] = mx;
    inv2[row] = 1.f / sum;
  }
}

// Materialise P = softmax(S) (claim_before) and/or the clamped attention (claim_after)
// for callers that keep them (AdaptiveSANet.claim_before / claim_after).
// (S may be one of the outputs: the flash path forms S in the caller's claim buffer, and each
// element is read before it is overwritten)
__global__ __launch_bounds__(256) void claim_maps_kernel(
    const float* S, RowVec rv, const float* __restrict__ inv2, int mode, float* before,
    float* after, int64_t rows, int L) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * L) return;
  const int64_t r = idx / L;
  const float v = S[idx];
  const float p = expf(v - rv.m[r]) * rv.inv[r];
  if (before) before[idx] = p;
  if (after) {
    after[idx] = mode == 0
                     ? bx_apply<BX_AEA>(v, rv.m[r], rv.inv[r], rv.clamp[r], 0.f, rv.scale)
                     : bx_apply<BX_AEAR>(v, rv.m[r], rv.inv[r], rv.clamp[r], rv.m2[r], 0.f) *
                           inv2[r];
  }
}

// Elementwise AEA transform of a given attention matrix fx (AEAModule.forward's second
// half, for the function-level module API): out = f(fx, clamp_row).
__global__ __launch_bounds__(256) void aea_apply_kernel(const float* __restrict__ fx,
                                                        const float* __restrict__ clamp,
                                                        const float* __restrict__ m2,
                                                        const float* __restrict__ inv2,
                                                        float* __restrict__ out, int64_t rows,
                                                        int L, int mode, float scale) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * L) return;
  const int64_t r = idx / L;
  const float d = fx[idx] - clamp[r];
  out[idx] = mode == 0 ? 1.f / (1.f + expf(-(scale * d))) : expf(fmaxf(d, 0.f) - m2[r]) * inv2[r];
}

// Row max / inverse sum of exp(relu(fx - c) - max) for aea_apply_kernel's mode 1.
__global__ __launch_bounds__(256) void rowstats_relu_plain_kernel(
    const float* __restrict__ fx, const float* __restrict__ clamp, float* __restrict__ m2,
    float* __restrict__ inv2, int64_t rows, int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = fx + row * L;
  const float c = clamp[row];
  float mx = -INFINITY;
  for (int i = lane; i < L; i += 64) mx = fmaxf(mx, fmaxf(s[i] - c, 0.f));
  mx = wave_max(mx);
  float sum = 0.f;
  for (int i = lane; i < L; i += 64) sum += expf(fmaxf(s[i] - c, 0.f) - mx);
  sum = wave_sum(sum);
  if (lane == 0) {
    m2[row] = mx;
    inv2[row] = 1.f / sum;
  }
}

// clamp[b, i] = head(LeakyReLU(A[b, i, :] W1^T + b1)) (AEAModule.f_psi over affinity rows)
static int clamp_values(const float* A, const float* w1, const float* b1, const float* w2,
                        const float* b2, int hid, int mode, float from, float interval,
                        float* Z, float* clamp, int B, int HW, hipStream_t st) {
  // Z[b][i][n] = sum_j A[b][i][j] W1[n][j] + b1[n]: M = HW (i), N = hid (n), K = HW (j)
  GemmArgs gz{A, w1, Z, {}, nullptr, b1, 1, HW, hid, HW, HW, HW, hid,
              (int64_t)HW * HW, 0, (int64_t)HW * hid, 0};
  launch_gemm<LAY_RK, LAY_RK, BX_NONE>(gz, B, st);
  if (int e = launch_status("gemm_f32_kernel(Z=A W1^T)")) return e;
  const int64_t rows = (int64_t)B * HW;
  clamp_head_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Z, w2, b2, clamp, rows, hid,
                                                               mode, from, interval);
  return launch_status("clamp_head_kernel");
}

// K chunks of T = sn W1^T (C x hidden per image, K = HW): its grid is C/256 x hidden/128
// tiles per image (2 x 2 at C = 512, HW = 4096), so the pixels are split 4 ways once HW >=
// 2048 (128 -> 512 workgroups at B = 32; 0.58 ms per call before); the partials sum in order
static int clamp_t_ks(int HW) { return HW >= 2048 ? 4 : 1; }
// floats of the T region: T itself and, when split, its ks partials
static size_t clamp_t_floats(int B, int C, int HW, int hidden) {
  const int ks = clamp_t_ks(HW);
  return (size_t)B * C * hidden * (ks > 1 ? 1 + ks : 1);
}
// out[b][i] = sum_j part[b * ks + j][i] (fixed order over j)
__global__ void ksum_kernel(const float* __restrict__ part, float* __restrict__ out,
                            int64_t per, int ks, int B) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= per * B) return;
  const int64_t b = t / per, i = t - b * per;
  const float* p = part + b * ks * per + i;
  float acc = p[0];
  for (int j = 1; j < ks; ++j) acc += p[j * per];
  out[t] = acc;
}

// The clamp values without the affinity matrix: f_psi's first Linear only ever sees
// A = cn^T sn through Z = A W1^T, and Z = cn^T (sn W1^T) (sanet.py:45-66, 110): T = sn W1^T
// (C x hid per image, K = HW), then Z = cn^T T + b1 (K = C): 2 x 2 C hid HW FLOP per image
// instead of 2 HW^2 (C + hid), and the B x HW x HW affinity is never written or read (the
// same sums in another association: ~1e-7 relative from the two-GEMM form).
// T: clamp_t_floats(B, C, HW, hid) floats of scratch (T, then its K-chunk partials).
static int clamp_values_factored(const float* cn, const float* sn, const float* w1,
                                 const float* b1, const float* w2, const float* b2, int hid,
                                 int mode, float from, float interval, float* T, float* Z,
                                 float* clamp, int B, int C, int HW, hipStream_t st) {
  const int ks = clamp_t_ks(HW);
  const int64_t per = (int64_t)C * hid;
  GemmArgs gt{sn, w1, ks > 1 ? T + (size_t)B * per : T, {}, nullptr, nullptr, 0, C, hid, HW,
              HW, HW, hid, (int64_t)C * HW, 0, per, 0};
  if (ks > 1) {
    gt.ks = ks;
    gt.kc = (HW + ks - 1) / ks;
    gt.kc = (gt.kc + 31) / 32 * 32;
  }
  launch_gemm<LAY_RK, LAY_RK, BX_NONE>(gt, B, st);
  if (int e = launch_status("gemm_f32_kernel(T=sn W1^T)")) return e;
  if (ks > 1) {
    ksum_kernel<<<(unsigned)((per * B + 255) / 256), 256, 0, st>>>(T + (size_t)B * per, T, per,
                                                                   ks, B);
    if (int e = launch_status("ksum_kernel(T)")) return e;
  }
  GemmArgs gz{cn, T, Z, {}, nullptr, b1, 1, HW, hid, C, HW, hid, hid,
              (int64_t)C * HW, (int64_t)C * hid, (int64_t)HW * hid, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(gz, B, st);
  if (int e = launch_status("gemm_f32_kernel(Z=cn^T T)")) return e;
  const int64_t rows = (int64_t)B * HW;
  clamp_head_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Z, w2, b2, clamp, rows, hid,
                                                               mode, from, interval);
  return launch_status("clamp_head_kernel");
}

static int col_norms(const float* c, const float* s, float* cn, float* sn, int B, int C, int HW,
                     hipStream_t st) {
  const unsigned nb = (unsigned)((int64_t)B * ((HW + 63) / 64));
  colnorm_kernel<<<nb, 256, 0, st>>>(c, cn, B, C, HW);
  colnorm_kernel<<<nb, 256, 0, st>>>(s, sn, B, C, HW);
  return launch_status("colnorm_kernel");
}

static int affinity(const float* c, const float* s, float* out, float* cn, float* sn, int B,
                    int C, int HW, hipStream_t st) {
  const unsigned nb = (unsigned)((int64_t)B * ((HW + 63) / 64));
  colnorm_kernel<<<nb, 256, 0, st>>>(c, cn, B, C, HW);
  colnorm_kernel<<<nb, 256, 0, st>>>(s, sn, B, C, HW);
  if (int e = launch_status("colnorm_kernel")) return e;
  const int64_t fhw = (int64_t)C * HW;
  // A[b][i][j] = sum_c cn[b][c][i] sn[b][c][j]
  GemmArgs ga{cn, sn, out, {}, nullptr, nullptr, 0, HW, HW, C, HW, HW, HW,
              fhw, fhw, (int64_t)HW * HW, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(ga, B, st);
  return launch_status("gemm_f32_kernel(A=cn^T sn)");
}

}  // namespace rpst

using namespace rpst;

extern "C" size_t rpst_sanet_attention_workspace_size(int B, int HW) {
  if (B <= 0 || HW <= 0) return 0;
  return sizeof(float) * ((size_t)B * HW * HW + 2 * (size_t)B * HW);
}

extern "C" size_t rpst_sanet_attention_workspace_size_c(int B, int C, int HW) {
  if (B <= 0 || C <= 0 || HW <= 0) return 0;
  return sanet_flash_ok(C, HW) ? 0 : rpst_sanet_attention_workspace_size(B, HW);
}

extern "C" int rpst_sanet_attention(const float* F, const float* G, const float* H, float* O,
                                    int B, int C, int HW, void* workspace,
                                    size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(F && G && H && O, "sanet_attention: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HW > 0, "sanet_attention: bad shape B=%d C=%d HW=%d", B, C, HW);
  RPST_REQUIRE(B <= 65535, "sanet_attention: batch too large");
  if (sanet_flash_ok(C, HW)) return sanet_flash(F, G, H, O, B, C, HW, as_stream(stream));
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
  GemmArgs g1{F, G, S, {}, nullptr, nullptr, 0, HW, HW, C, HW, HW, HW,
               fhw, fhw, (int64_t)HW * HW, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(g1, B, st);
  if (int e = launch_status("gemm_f32_kernel(S=F^T G)")) return e;
  const int64_t rows = (int64_t)B * HW;
  rowstats_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(S, rmax, rinv, rows, HW);
  if (int e = launch_status("rowstats_kernel")) return e;
  // O[b][c][i] = (1/l_i) sum_j H[b][c][j] exp(S[b][i][j] - m_i)
  GemmArgs g2{H, S, O, {rmax, nullptr, nullptr, nullptr, 0.f}, rinv, nullptr, 0,
               C, HW, HW, HW, HW, HW, fhw, (int64_t)HW * HW, fhw, HW};
  launch_gemm<LAY_RK, LAY_RK, BX_EXP>(g2, B, st);
  return launch_status("gemm_f32_kernel(O=H P^T)");
}

extern "C" size_t rpst_cosine_affinity_workspace_size(int B, int C, int HW) {
  if (B <= 0 || C <= 0 || HW <= 0) return 0;
  return sizeof(float) * 2 * (size_t)B * C * HW;
}

extern "C" int rpst_cosine_affinity(const float* content, const float* style, float* out,
                                    int B, int C, int HW, void* workspace,
                                    size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(content && style && out, "cosine_affinity: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HW > 0 && B <= 65535, "cosine_affinity: bad shape");
  if (!workspace || workspace_bytes < rpst_cosine_affinity_workspace_size(B, C, HW)) {
    set_error("cosine_affinity: workspace too small");
    return RPST_EWORKSPACE;
  }
  float* cn = static_cast<float*>(workspace);
  return affinity(content, style, out, cn, cn + (size_t)B * C * HW, B, C, HW,
                  as_stream(stream));
}

extern "C" size_t rpst_aea_clamp_workspace_size(int B, int HW, int hidden) {
  if (B <= 0 || HW <= 0 || hidden <= 0) return 0;
  return sizeof(float) * ((size_t)B * HW * hidden + 2 * (size_t)B * HW);
}

extern "C" int rpst_aea_clamp(const float* x, const float* fx, const float* w1,
                              const float* b1, const float* w2, const float* b2, int hidden,
                              int mode, float scale, float from, float interval, float* out_fx,
                              float* out_clamp, int B, int HW, void* workspace,
                              size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(x && fx && w1 && b1 && w2 && b2 && out_fx && out_clamp, "aea_clamp: null pointer");
  RPST_REQUIRE(B > 0 && HW > 0 && hidden > 0 && B <= 65535, "aea_clamp: bad shape");
  RPST_REQUIRE(mode == 0 || mode == 1, "aea_clamp: mode must be 0 (aea) or 1 (relu)");
  if (!workspace || workspace_bytes < rpst_aea_clamp_workspace_size(B, HW, hidden)) {
    set_error("aea_clamp: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* Z = static_cast<float*>(workspace);
  float* m2 = Z + (size_t)B * HW * hidden;
  float* inv2 = m2 + (size_t)B * HW;
  if (int e = clamp_values(x, w1, b1, w2, b2, hidden, mode, from, interval, Z, out_clamp, B,
                           HW, st))
    return e;
  const int64_t rows = (int64_t)B * HW;
  if (mode == 1) {
    rowstats_relu_plain_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(fx, out_clamp, m2,
                                                                           inv2, rows, HW);
    if (int e = launch_status("rowstats_relu_plain_kernel")) return e;
  }
  const int64_t n = rows * HW;
  aea_apply_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(fx, out_clamp, m2, inv2, out_fx,
                                                                rows, HW, mode, scale);
  return launch_status("aea_apply_kernel");
}

// the logits' region first holds T = sn W1^T (C x hidden per image): whichever is larger.
// On the flash path (sanet_flash_ok) S is never formed: T only.
static size_t sq_or_t(int B, int C, int HW, int hidden) {
  if (sanet_flash_ok(C, HW)) return clamp_t_floats(B, C, HW, hidden);
  return std::max((size_t)B * HW * HW, clamp_t_floats(B, C, HW, hidden));
}

extern "C" size_t rpst_adaptive_attention_workspace_size(int B, int C, int HW, int hidden) {
  if (B <= 0 || C <= 0 || HW <= 0 || hidden <= 0) return 0;
  return sizeof(float) * (sq_or_t(B, C, HW, hidden) + (size_t)B * HW * hidden +
                          2 * (size_t)B * C * HW + 7 * (size_t)B * HW);
}

extern "C" int rpst_adaptive_attention(const float* F, const float* G, const float* H,
                                       const float* content, const float* style,
                                       const float* w1, const float* b1, const float* w2,
                                       const float* b2, int hidden, int mode, float scale,
                                       float from, float interval, float* O, float* claim_value,
                                       float* claim_before, float* claim_after, int B, int C,
                                       int HW, void* workspace, size_t workspace_bytes,
                                       rpst_stream_t stream) {
  RPST_REQUIRE(F && G && H && content && style && w1 && b1 && w2 && b2 && O,
               "adaptive_attention: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HW > 0 && hidden > 0 && B <= 65535,
               "adaptive_attention: bad shape B=%d C=%d HW=%d hidden=%d", B, C, HW, hidden);
  RPST_REQUIRE(mode == 0 || mode == 1, "adaptive_attention: mode must be 0 (aea) or 1 (relu)");
  if (!workspace ||
      workspace_bytes < rpst_adaptive_attention_workspace_size(B, C, HW, hidden)) {
    set_error("adaptive_attention: workspace %zu < %zu bytes", workspace_bytes,
              rpst_adaptive_attention_workspace_size(B, C, HW, hidden));
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* S = static_cast<float*>(workspace);  // T = sn W1^T first, then the logits
  float* Z = S + sq_or_t(B, C, HW, hidden);
  float* cn = Z + (size_t)B * HW * hidden;
  float* sn = cn + (size_t)B * C * HW;
  float* rmax = sn + (size_t)B * C * HW;
  float* rinv = rmax + (size_t)B * HW;
  float* clamp = rinv + (size_t)B * HW;
  float* m2 = clamp + (size_t)B * HW;
  float* inv2 = m2 + (size_t)B * HW;
  // 1. clamp values from the cosine affinity of the raw features (sanet.py:110, 45 / 66), the
  //    affinity folded into f_psi's first Linear (T in the logits' buffer, not yet written)
  if (int e = col_norms(content, style, cn, sn, B, C, HW, st)) return e;
  if (int e = clamp_values_factored(cn, sn, w1, b1, w2, b2, hidden, mode, from, interval, S, Z,
                                    clamp, B, C, HW, st))
    return e;
  const int64_t fhw = (int64_t)C * HW;
  const int64_t rows = (int64_t)B * HW;
  if (sanet_flash_ok(C, HW)) {
    // 2. pass 1: softmax row statistics of S = F^T G, S never written (rpst_flash.hip)
    if (int e = adaptive_flash_stats(F, G, B, C, HW, rmax, rinv, st)) return e;
    if (claim_before || claim_after) {
      // the maps the caller keeps: S formed in its own (B, HW, HW) buffer and transformed in
      // place, with pass 1's statistics
      // (row statistics of this S itself: pass 1's, from the flash kernel's summation order,
      // would put the maps ~1e-5 off the logits they transform, amplified by the slope-50
      // sigmoid)
      float* Sx = claim_before ? claim_before : claim_after;
      float* cmax = inv2 + (size_t)B * HW;
      float* cinv = cmax + (size_t)B * HW;
      GemmArgs g1{F, G, Sx, {}, nullptr, nullptr, 0, HW, HW, C, HW, HW, HW,
                  fhw, fhw, (int64_t)HW * HW, 0};
      launch_gemm<LAY_KR, LAY_KR, BX_NONE>(g1, B, st);
      if (int e = launch_status("gemm_f32_kernel(S=F^T G, claims)")) return e;
      rowstats_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Sx, cmax, cinv, rows, HW);
      if (int e = launch_status("rowstats_kernel")) return e;
      if (mode == 1) {
        rowstats_relu_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Sx, cmax, cinv, clamp,
                                                                         m2, inv2, rows, HW);
        if (int e = launch_status("rowstats_relu_kernel")) return e;
      }
      const RowVec rv{cmax, cinv, clamp, m2, scale};
      const int64_t n = rows * HW;
      claim_maps_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(Sx, rv, inv2, mode,
                                                                     claim_before, claim_after,
                                                                     rows, HW);
      if (int e = launch_status("claim_maps_kernel")) return e;
    }
    if (claim_value &&
        hipMemcpyAsync(claim_value, clamp, sizeof(float) * rows, hipMemcpyDeviceToDevice, st) !=
            hipSuccess) {
      set_error("adaptive_attention: claim_value copy failed");
      return RPST_EHIP;
    }
    // 3. pass 2: S recomputed per key block, Q formed in registers, O = H Q^T
    return adaptive_flash_apply(F, G, H, O, B, C, HW, rmax, rinv, clamp, mode, scale, st);
  }
  // 2. logits S = F^T G and softmax row statistics (sanet.py:114-117)
  GemmArgs g1{F, G, S, {}, nullptr, nullptr, 0, HW, HW, C, HW, HW, HW,
              fhw, fhw, (int64_t)HW * HW, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(g1, B, st);
  if (int e = launch_status("gemm_f32_kernel(S=F^T G)")) return e;
  rowstats_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(S, rmax, rinv, rows, HW);
  if (int e = launch_status("rowstats_kernel")) return e;
  RowVec rv{rmax, rinv, clamp, m2, scale};
  if (mode == 1) {
    rowstats_relu_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(S, rmax, rinv, clamp, m2,
                                                                     inv2, rows, HW);
    if (int e = launch_status("rowstats_relu_kernel")) return e;
  }
  if (claim_before || claim_after) {
    const int64_t n = rows * HW;
    claim_maps_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(S, rv, inv2, mode,
                                                                   claim_before, claim_after,
                                                                   rows, HW);
    if (int e = launch_status("claim_maps_kernel")) return e;
  }
  if (claim_value) {
    if (hipMemcpyAsync(claim_value, clamp, sizeof(float) * rows, hipMemcpyDeviceToDevice, st) !=
        hipSuccess) {
      set_error("adaptive_attention: claim_value copy failed");
      return RPST_EHIP;
    }
  }
  // 3. O[b][c][i] = sum_j H[b][c][j] Q[b][i][j], Q formed while S is staged (sanet.py:122-124)
  if (mode == 0) {
    GemmArgs g2{H, S, O, rv, nullptr, nullptr, 0, C, HW, HW, HW, HW, HW,
                fhw, (int64_t)HW * HW, fhw, HW};
    launch_gemm<LAY_RK, LAY_RK, BX_AEA>(g2, B, st);
  } else {
    GemmArgs g2{H, S, O, rv, inv2, nullptr, 0, C, HW, HW, HW, HW, HW,
                fhw, (int64_t)HW * HW, fhw, HW};
    launch_gemm<LAY_RK, LAY_RK, BX_AEAR>(g2, B, st);
  }
  return launch_status("gemm_f32_kernel(O=H Q^T)");
}

extern "C" size_t rpst_sanet_attention_backward_workspace_size(int B, int HWc, int HWs) {
  if (B <= 0 || HWc <= 0 || HWs <= 0) return 0;
  return sizeof(float) * (2 * (size_t)B * HWc * HWs + 2 * (size_t)B * HWc);
}

extern "C" int rpst_sanet_attention_backward(const float* F, const float* G, const float* H,
                                             const float* dO, float* dF, float* dG, float* dH,
                                             int B, int C, int HWc, int HWs, void* workspace,
                                             size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(F && G && H && dO && dF && dG && dH, "sanet_attention_backward: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HWc > 0 && HWs > 0 && B <= 65535,
               "sanet_attention_backward: bad shape B=%d C=%d HW=%d/%d", B, C, HWc, HWs);
  if (!workspace ||
      workspace_bytes < rpst_sanet_attention_backward_workspace_size(B, HWc, HWs)) {
    set_error("sanet_attention_backward: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t ss = (int64_t)HWc * HWs, fc = (int64_t)C * HWc, fs = (int64_t)C * HWs;
  float* S = static_cast<float*>(workspace);
  float* dP = S + (size_t)B * ss;
  float* rmax = dP + (size_t)B * ss;
  float* rinv = rmax + (size_t)B * HWc;
  // S = F^T G; row statistics of the softmax
  GemmArgs g1{F, G, S, {}, nullptr, nullptr, 0, HWc, HWs, C, HWc, HWs, HWs, fc, fs, ss, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(g1, B, st);
  if (int e = launch_status("gemm_f32_kernel(S=F^T G)")) return e;
  const int64_t rows = (int64_t)B * HWc;
  rowstats_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(S, rmax, rinv, rows, HWs);
  if (int e = launch_status("rowstats_kernel")) return e;
  // dH = dO P: P formed from S while staged (KR: the row of P is the k index)
  GemmArgs gh{dO, S, dH, {rmax, rinv, nullptr, nullptr, 0.f}, nullptr, nullptr, 0,
              C, HWs, HWc, HWc, HWs, HWs, fc, ss, fs, HWc};
  launch_gemm<LAY_RK, LAY_KR, BX_PROB>(gh, B, st);
  if (int e = launch_status("gemm_f32_kernel(dH=dO P)")) return e;
  // dP = dO^T H, then dS = P (dP - rowsum(dP P)) in place
  GemmArgs gp{dO, H, dP, {}, nullptr, nullptr, 0, HWc, HWs, C, HWc, HWs, HWs, fc, fs, ss, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(gp, B, st);
  if (int e = launch_status("gemm_f32_kernel(dP=dO^T H)")) return e;
  softmax_bwd_logits_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(S, rmax, rinv, dP, rows,
                                                                        HWs);
  if (int e = launch_status("softmax_bwd_logits_kernel")) return e;
  // dF = G dS^T, dG = F dS
  GemmArgs gf{G, dP, dF, {}, nullptr, nullptr, 0, C, HWc, HWs, HWs, HWs, HWc, fs, ss, fc, 0};
  launch_gemm<LAY_RK, LAY_RK, BX_NONE>(gf, B, st);
  if (int e = launch_status("gemm_f32_kernel(dF=G dS^T)")) return e;
  GemmArgs gg{F, dP, dG, {}, nullptr, nullptr, 0, C, HWs, HWc, HWc, HWs, HWs, fc, ss, fs, 0};
  launch_gemm<LAY_RK, LAY_KR, BX_NONE>(gg, B, st);
  return launch_status("gemm_f32_kernel(dG=F dS)");
}

// ---- SANet attention backward over query chunks (no B x HW x HW workspace) -------------
// The same gradients with S and dP formed for attn_qc() = 2048 queries (full rows) at a time:
// per chunk S_q = F_q^T G, the row statistics, dH += dO_q P_q (P formed while S_q is staged),
// dP_q = dO_q^T H, dS_q = P (dP - rowsum(dP P)) in place (softmax_bwd_logits_kernel: whole
// rows, so every row of dS sums to zero to rounding as in the single pass), dF_q = G dS_q^T,
// dG += F_q dS_q; dH and dG sum the chunks in order. S, its statistics and dS are the single
// pass's bit for bit (the GEMM's k order does not depend on M); 10 HW^2 C FLOP per image like
// the single pass. Workspace: S_q and dP_q (2 B qc HWs) + 2 B qc row vectors. (2048: the dF_q
// GEMM's grid is C/256 x qc/128 tiles per image -- at 1024 queries, C = 512 and B = 8 only 128
// workgroups, and the SAModel training step ran 2.8 % slower than the single pass; at 2048
// 0.6 %, profiles/r05/attn_bwd_qc.log.)
// (RPST_ATTN_QC overrides the chunk: A/B against the single pass, tests.)
static int attn_qc() {
  static const int qc = [] {
    const char* e = std::getenv("RPST_ATTN_QC");
    const int v = (e && *e) ? std::atoi(e) : 2048;
    return v >= 16 ? v / 4 * 4 : 2048;
  }();
  return qc;
}

extern "C" size_t rpst_sanet_attention_backward_chunked_workspace_size(int B, int C, int HWc,
                                                                       int HWs) {
  if (B <= 0 || C <= 0 || HWc <= 0 || HWs <= 0) return 0;
  const size_t qc = (size_t)std::min(HWc, attn_qc());
  return sizeof(float) * (2 * (size_t)B * qc * HWs + 2 * (size_t)B * qc);
}

extern "C" int rpst_sanet_attention_backward_chunked(const float* F, const float* G,
                                                     const float* H, const float* dO, float* dF,
                                                     float* dG, float* dH, int B, int C, int HWc,
                                                     int HWs, void* workspace,
                                                     size_t workspace_bytes,
                                                     rpst_stream_t stream) {
  RPST_REQUIRE(F && G && H && dO && dF && dG && dH,
               "sanet_attention_backward_chunked: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HWc > 0 && HWs > 0 && B <= 65535,
               "sanet_attention_backward_chunked: bad shape B=%d C=%d HW=%d/%d", B, C, HWc, HWs);
  if (!workspace ||
      workspace_bytes < rpst_sanet_attention_backward_chunked_workspace_size(B, C, HWc, HWs)) {
    set_error("sanet_attention_backward_chunked: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int qc = std::min(HWc, attn_qc());
  const int64_t fc = (int64_t)C * HWc, fs = (int64_t)C * HWs, sq = (int64_t)qc * HWs;
  float* Sq = static_cast<float*>(workspace);
  float* dPq = Sq + (size_t)B * sq;
  float* rmax = dPq + (size_t)B * sq;
  float* rinv = rmax + (size_t)B * qc;
  for (int q0 = 0; q0 < HWc; q0 += qc) {
    const int n = std::min(qc, HWc - q0);
    const int64_t sn = (int64_t)n * HWs, rows = (int64_t)B * n;
    GemmArgs g1{F + q0, G, Sq, {}, nullptr, nullptr, 0, n, HWs, C, HWc, HWs, HWs, fc, fs, sn, 0};
    launch_gemm<LAY_KR, LAY_KR, BX_NONE>(g1, B, st);
    if (int e = launch_status("gemm_f32_kernel(S_q=F_q^T G)")) return e;
    rowstats_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Sq, rmax, rinv, rows, HWs);
    if (int e = launch_status("rowstats_kernel")) return e;
    GemmArgs gh{dO + q0, Sq, dH, {rmax, rinv, nullptr, nullptr, 0.f}, nullptr, nullptr, 0,
                C, HWs, n, HWc, HWs, HWs, fc, sn, fs, n};
    gh.accum = q0 > 0;
    launch_gemm<LAY_RK, LAY_KR, BX_PROB>(gh, B, st);
    if (int e = launch_status("gemm_f32_kernel(dH+=dO_q P_q)")) return e;
    GemmArgs gp{dO + q0, H, dPq, {}, nullptr, nullptr, 0, n, HWs, C, HWc, HWs, HWs, fc, fs, sn, 0};
    launch_gemm<LAY_KR, LAY_KR, BX_NONE>(gp, B, st);
    if (int e = launch_status("gemm_f32_kernel(dP_q=dO_q^T H)")) return e;
    softmax_bwd_logits_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Sq, rmax, rinv, dPq,
                                                                          rows, HWs);
    if (int e = launch_status("softmax_bwd_logits_kernel")) return e;
    GemmArgs gf{G, dPq, dF + q0, {}, nullptr, nullptr, 0, C, n, HWs, HWs, HWs, HWc, fs, sn, fc, 0};
    launch_gemm<LAY_RK, LAY_RK, BX_NONE>(gf, B, st);
    if (int e = launch_status("gemm_f32_kernel(dF_q=G dS_q^T)")) return e;
    GemmArgs gg{F + q0, dPq, dG, {}, nullptr, nullptr, 0, C, HWs, n, HWc, HWs, HWs, fc, sn, fs, 0};
    gg.accum = q0 > 0;
    launch_gemm<LAY_RK, LAY_KR, BX_NONE>(gg, B, st);
    if (int e = launch_status("gemm_f32_kernel(dG+=F_q dS_q)")) return e;
  }
  return RPST_OK;
}

// K (pixel) chunks per image of the 1x1 weight gradient: the per-image GEMM has only
// ceil(Cout/256) x ceil(Cin/128) tiles (8 for the SANet's 512 x 512 convs, 64 workgroups at
// N = 8), so the pixels are split until the launch has ~512 workgroups (two per CU). A
// function of the shape only: the fixed-order partial sum stays deterministic.
static int wgrad1x1_ks(int N, int Cin, int Cout) {
  const int64_t tiles = (int64_t)((Cout + 255) / 256) * ((Cin + 127) / 128) * N;
  const int64_t ks = (512 + tiles - 1) / tiles;
  return (int)std::max<int64_t>(1, std::min<int64_t>(ks, 16));
}

extern "C" size_t rpst_conv1x1_wgrad_workspace_size(int N, int Cin, int Cout) {
  if (N <= 0 || Cin <= 0 || Cout <= 0) return 0;
  return sizeof(float) * (size_t)N * wgrad1x1_ks(N, Cin, Cout) * Cin * Cout;
}

extern "C" int rpst_conv1x1_wgrad(const float* x, const float* dy, float* dw, float* db, int N,
                                  int Cin, int64_t HW, int Cout, void* workspace,
                                  size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(x && dy && dw, "conv1x1_wgrad: null pointer");
  RPST_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && HW > 0 && HW <= 0x7fffffffLL && N <= 65535,
               "conv1x1_wgrad: bad shape");
  if (!workspace || workspace_bytes < rpst_conv1x1_wgrad_workspace_size(N, Cin, Cout)) {
    set_error("conv1x1_wgrad: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  // part[n][co][ci] = sum_p dy[n][co][p] x[n][ci][p]
  // part[n * ks + j][co][ci] = sum over pixel chunk j of dy[n][co][p] x[n][ci][p]; chunks of
  // kc pixels (a multiple of 64, so at most ks of them and 16-B aligned)
  const int ksmax = wgrad1x1_ks(N, Cin, Cout);
  const int64_t kc = std::max<int64_t>(64, ((HW + ksmax - 1) / ksmax + 63) / 64 * 64);
  const int ks = (int)((HW + kc - 1) / kc);
  GemmArgs g{dy, x, part, {}, nullptr, nullptr, 0, Cout, Cin, (int)HW, (int)HW, (int)HW, Cin,
             (int64_t)Cout * HW, (int64_t)Cin * HW, (int64_t)Cout * Cin, 0, ks, (int)kc};
  launch_gemm<LAY_RK, LAY_RK, BX_NONE>(g, N, st);
  if (int e = launch_status("gemm_f32_kernel(dW=dY X^T)")) return e;
  const int64_t per = (int64_t)Cout * Cin;
  batch_sum_kernel<<<(unsigned)((per + 255) / 256), 256, 0, st>>>(part, dw, per, N * ks);
  if (int e = launch_status("batch_sum_kernel")) return e;
  if (db) {
    channel_sum_kernel<<<Cout, 256, 0, st>>>(dy, db, N, Cout, HW);
    return launch_status("channel_sum_kernel");
  }
  return RPST_OK;
}

extern "C" size_t rpst_adaptive_attention_backward_workspace_size(int B, int C, int HW,
                                                                  int hidden) {
  if (B <= 0 || C <= 0 || HW <= 0 || hidden <= 0) return 0;
  const size_t qc = (size_t)std::min(HW, attn_qc());
  const size_t chunks = ((size_t)B * HW + kColChunk - 1) / kColChunk;
  // (the first region holds T and then R, C x hidden per image, never the affinity) + S and
  // dQ of one query chunk + the per-image dW1 partials and the column-sum chunk partials
  return sizeof(float) * (clamp_t_floats(B, C, HW, hidden) + 2 * (size_t)B * qc * HW +
                          2 * (size_t)B * HW * hidden + 2 * (size_t)B * C * HW +
                          3 * (size_t)B * HW + 6 * (size_t)B * qc + (size_t)B * hidden * HW +
                          3 * (size_t)(hidden + 1) * chunks);
}

extern "C" int rpst_adaptive_attention_backward(
    const float* F, const float* G, const float* H, const float* content, const float* style,
    const float* w1, const float* b1, const float* w2, const float* b2, int hidden, int mode,
    float scale, float from, float interval, const float* dO, float* dF, float* dG, float* dH,
    float* dw1, float* db1, float* dw2, float* db2, int B, int C, int HW, void* workspace,
    size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(F && G && H && content && style && w1 && b1 && w2 && b2 && dO && dF && dG &&
                   dH && dw1 && db1 && dw2 && db2,
               "adaptive_attention_backward: null pointer");
  RPST_REQUIRE(B > 0 && C > 0 && HW > 0 && hidden > 0 && B <= 65535 &&
                   (int64_t)B * HW <= 0x7fffffffLL,
               "adaptive_attention_backward: bad shape B=%d C=%d HW=%d hidden=%d", B, C, HW,
               hidden);
  RPST_REQUIRE(mode == 0 || mode == 1, "adaptive_attention_backward: mode must be 0 or 1");
  if (!workspace ||
      workspace_bytes < rpst_adaptive_attention_backward_workspace_size(B, C, HW, hidden)) {
    set_error("adaptive_attention_backward: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  const int qc = std::min(HW, attn_qc());
  const int64_t fhw = (int64_t)C * HW, rows = (int64_t)B * HW, sq = (int64_t)qc * HW;
  float* Aff = static_cast<float*>(workspace);  // T, then R (C x hidden per image)
  float* Sq = Aff + clamp_t_floats(B, C, HW, hidden);  // S and dQ of one query chunk
  float* dQq = Sq + (size_t)B * sq;
  float* Z = dQq + (size_t)B * sq;
  float* du = Z + (size_t)rows * hidden;
  float* cn = du + (size_t)rows * hidden;
  float* sn = cn + (size_t)B * fhw;
  float* clamp = sn + (size_t)B * fhw;
  float* dc = clamp + rows;
  float* dt = dc + rows;
  float* rmax = dt + rows;  // per query chunk: [B][qc] each
  float* rinv = rmax + (size_t)B * qc;
  float* clq = rinv + (size_t)B * qc;
  float* m2 = clq + (size_t)B * qc;
  float* inv2 = m2 + (size_t)B * qc;
  float* dcq = inv2 + (size_t)B * qc;
  float* w1part = dcq + (size_t)B * qc;                    // [B][hidden][HW]
  float* cpart = w1part + (size_t)B * hidden * HW;         // [chunks][3][hidden + 1]
  // forward quantities: clamp (and Z) as the forward forms them (the affinity folded into
  // f_psi's first Linear; T in the Aff region), logits, softmax / relu-softmax statistics
  if (int e = col_norms(content, style, cn, sn, B, C, HW, st)) return e;
  if (int e = clamp_values_factored(cn, sn, w1, b1, w2, b2, hidden, mode, from, interval, Aff,
                                    Z, clamp, B, C, HW, st))
    return e;
  // attention part over query chunks of whole rows (as rpst_sanet_attention_backward_chunked):
  // S_q, its softmax / relu-softmax statistics, dH += dO_q Q_q, dQ_q = dO_q^T H -> dS_q and
  // dc (aea_bwd_rows_kernel on whole rows), dF_q = G dS_q^T, dG += F_q dS_q
  for (int q0 = 0; q0 < HW; q0 += qc) {
    const int n = std::min(qc, HW - q0);
    const int64_t sn_ = (int64_t)n * HW, rq = (int64_t)B * n;
    const unsigned rb = (unsigned)((rq + 255) / 256), wb = (unsigned)((rq + 3) / 4);
    GemmArgs g1{F + q0, G, Sq, {}, nullptr, nullptr, 0, n, HW, C, HW, HW, HW, fhw, fhw, sn_, 0};
    launch_gemm<LAY_KR, LAY_KR, BX_NONE>(g1, B, st);
    if (int e = launch_status("gemm_f32_kernel(S_q=F_q^T G)")) return e;
    rowstats_kernel<<<wb, 256, 0, st>>>(Sq, rmax, rinv, rq, HW);
    if (int e = launch_status("rowstats_kernel")) return e;
    rows_gather_kernel<<<rb, 256, 0, st>>>(clamp, clq, B, HW, q0, n);
    if (int e = launch_status("rows_gather_kernel")) return e;
    if (mode == 1) {
      rowstats_relu_kernel<<<wb, 256, 0, st>>>(Sq, rmax, rinv, clq, m2, inv2, rq, HW);
      if (int e = launch_status("rowstats_relu_kernel")) return e;
    }
    RowVec rv{rmax, rinv, clq, m2, scale, inv2};
    GemmArgs gh{dO + q0, Sq, dH, rv, nullptr, nullptr, 0, C, HW, n, HW, HW, HW, fhw, sn_, fhw, n};
    gh.accum = q0 > 0;
    if (mode == 0) launch_gemm<LAY_RK, LAY_KR, BX_AEA>(gh, B, st);
    else launch_gemm<LAY_RK, LAY_KR, BX_AEARQ>(gh, B, st);
    if (int e = launch_status("gemm_f32_kernel(dH+=dO_q Q_q)")) return e;
    GemmArgs gq{dO + q0, H, dQq, {}, nullptr, nullptr, 0, n, HW, C, HW, HW, HW, fhw, fhw, sn_, 0};
    launch_gemm<LAY_KR, LAY_KR, BX_NONE>(gq, B, st);
    if (int e = launch_status("gemm_f32_kernel(dQ_q=dO_q^T H)")) return e;
    aea_bwd_rows_kernel<<<wb, 256, 0, st>>>(Sq, rv, dQq, dcq, mode, rq, HW);
    if (int e = launch_status("aea_bwd_rows_kernel")) return e;
    rows_scatter_kernel<<<rb, 256, 0, st>>>(dcq, dc, B, HW, q0, n);
    if (int e = launch_status("rows_scatter_kernel")) return e;
    GemmArgs gf{G, dQq, dF + q0, {}, nullptr, nullptr, 0, C, n, HW, HW, HW, HW, fhw, sn_, fhw, 0};
    launch_gemm<LAY_RK, LAY_RK, BX_NONE>(gf, B, st);
    if (int e = launch_status("gemm_f32_kernel(dF_q=G dS_q^T)")) return e;
    GemmArgs gg{F + q0, dQq, dG, {}, nullptr, nullptr, 0, C, HW, n, HW, HW, HW, fhw, sn_, fhw, 0};
    gg.accum = q0 > 0;
    launch_gemm<LAY_RK, LAY_KR, BX_NONE>(gg, B, st);
    if (int e = launch_status("gemm_f32_kernel(dG+=F_q dS_q)")) return e;
  }
  // f_psi: dt, du, then dW1 = du^T Aff over all B * HW query rows (one GEMM), the column sums
  fpsi_bwd_rows_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(Z, w2, b2, dc, dt, du, rows,
                                                                   hidden, mode, interval);
  if (int e = launch_status("fpsi_bwd_rows_kernel")) return e;
  // dW1 = du^T A per image with A = cn^T sn never formed: R = cn du (C x hidden, K = HW),
  // then dW1_b = R^T sn (K = C), then the B partials summed in order
  float* R = Aff;
  GemmArgs gr{cn, du, R, {}, nullptr, nullptr, 0, C, hidden, HW, HW, hidden, hidden,
              fhw, (int64_t)HW * hidden, (int64_t)C * hidden, 0};
  launch_gemm<LAY_RK, LAY_KR, BX_NONE>(gr, B, st);
  if (int e = launch_status("gemm_f32_kernel(R_b=cn_b du_b)")) return e;
  GemmArgs gw{R, sn, w1part, {}, nullptr, nullptr, 0, hidden, HW, C, hidden, HW, HW,
              (int64_t)C * hidden, fhw, (int64_t)hidden * HW, 0};
  launch_gemm<LAY_KR, LAY_KR, BX_NONE>(gw, B, st);
  if (int e = launch_status("gemm_f32_kernel(dW1_b=R_b^T sn_b)")) return e;
  const int64_t nw1 = (int64_t)hidden * HW;
  batch_sum_kernel<<<(unsigned)((nw1 + 255) / 256), 256, 0, st>>>(w1part, dw1, nw1, B);
  if (int e = launch_status("batch_sum_kernel(dW1)")) return e;
  const int chunks = (int)((rows + kColChunk - 1) / kColChunk);
  fpsi_colsum_part_kernel<<<dim3((unsigned)((hidden + 1 + 255) / 256), (unsigned)chunks), 256, 0,
                            st>>>(Z, du, dt, cpart, rows, hidden);
  if (int e = launch_status("fpsi_colsum_part_kernel")) return e;
  fpsi_colsum_final_kernel<<<(hidden + 1 + 255) / 256, 256, 0, st>>>(cpart, dw2, db1, db2, chunks,
                                                                    hidden);
  return launch_status("fpsi_colsum_final_kernel");
}
