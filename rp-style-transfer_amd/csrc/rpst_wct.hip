// Closed-form WCT (Lu et al.) in fp64 on gfx950 — network/wct_rp.py:7-40, 82-114, 157-166.
//
// Per image (cF, sF: C x HW features, read as fp32 and widened to fp64 in registers,
// exactly like the reference's `.double()`):
//   mu_c, mu_s                       row means (fp64)                      wct_rp.py:85,92
//   Cc = (cF-mu)(cF-mu)^T/(n-1) + I  fp64 MFMA "SYRK": only upper-triangular tiles,
//   Cs = (sF-mu)(sF-mu)^T/(n-1)      split-K partials + fixed-order reduce  wct_rp.py:89,94
//   Sc = (Cc+1e-4 I)^(1/2), Ic = (Cc+1e-4 I)^(-1/2)                       wct_rp.py:104-105
//   Mid = (Sc Cs Sc + 1e-4 I)^(1/2)                                         wct_rp.py:107
//   T = Ic Mid Ic ; out = T (cF - mu_c) + mu_s  -> fp32                     wct_rp.py:109-113
//   (the last product on the fp32 MFMA for fp32 features, T rounded once; see below)
// The covariances of fp32 features with C <= 256 come from cov_syrk_kernel and the matrix
// functions (Newton-Schulz square roots, Sc Cs Sc, Ic Mid Ic, mu_s - T mu_c) from the
// persistent matfun_kernel (rpst_wct_mat.hip); this file keeps the generic tiled fp64 GEMM
// (covariances for C > 256 or fp64 features, the fp64 colour transform) and the entry points.
//
// GEMM: v_mfma_f64_16x16x4_f64 (A[l&15][k=l>>4], B[k=l>>4][l&15], D col=l&15,
// row=(l>>4)+4r). Tiles BT x BT (64 or 128) x 16, 256 threads = 2x2 waves, operands
// staged k-major in LDS with a 16-double pad (conflict-free ds_read_b64 halves).
#include "rpst_common.h"
#include "rpst_wct.h"

#include <cstdlib>

namespace rpst {

#ifndef RPST_WCT_BK
#define RPST_WCT_BK 32  // k depth of a staged fp64 GEMM tile (16: wct_params 17.77 vs 16.86 ms)
#endif

// plain fp64 / centered fp64 / centered fp32 / plain fp32
enum { SRC_F64 = 0, SRC_F64C = 1, SRC_F32C = 2, SRC_F32 = 3 };
constexpr bool src_f32(int s) { return s == SRC_F32C || s == SRC_F32; }
constexpr bool src_centred(int s) { return s == SRC_F64C || s == SRC_F32C; }
enum { B_KN = 0, B_NK = 1 };
enum { OUT_F64 = 0, OUT_PARTIAL = 1, OUT_F32_BIAS = 2, OUT_F64_BIAS = 3 };

struct G64Args {
  const void* A;
  const void* B;
  void* C;
  const double* amean;  // per-m mean (A centering), batch stride sMean
  const double* bmean;  // per-k (B_KN) or per-n (B_NK) mean, batch stride sMean
  const double* bias;   // per-m bias (OUT_*_BIAS), batch stride sMean
  const double* avec;   // optional per-batch alpha multiplier
  double alpha, beta_diag;
  int M, N, K, lda, ldb, ldc;
  int64_t sA, sB, sC, sMean;
  int ksplit;           // split-K factor (OUT_PARTIAL)
  int sym;              // only upper-triangular tiles (blockIdx.x enumerates them)
  int tiles_n;
  // dual launch: batch entries z >= dual run C2 = A2 B2 (same shape / strides; ksplit 1),
  // so two independent products share one launch (0 = off)
  const void* A2;
  const void* B2;
  void* C2;
  int dual;
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned kOOB = 0x80000000u;  // out-of-range buffer offset: loads return 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Load N consecutive elements (contiguous dim) starting at element index e of a SRC-typed
// buffer, widened to fp64. VEC: 16-B loads whose validity is all-or-nothing (host checks
// the alignment of sizes / leading dims); else one load per element. ok(i) -> element i
// is inside the logical operand; invalid elements read 0 (buffer out-of-range).
template <int SRC, int N, bool VEC, typename OK>
__device__ __forceinline__ void load_run(double (&v)[N], __amdgpu_buffer_rsrc_t r, unsigned e,
                                         OK ok) {
  if (src_f32(SRC)) {
    if (VEC) {
#pragma unroll
      for (int q = 0; q < N / 4; ++q) {
        const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(
            r, (int)(ok(4 * q) ? (e + 4 * q) * 4u : kOOB), 0, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[4 * q + t] = (double)__uint_as_float(w[t]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        v[i] = (double)__uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(r, (int)(ok(i) ? (e + i) * 4u : kOOB), 0, 0));
    }
  } else {
    if (VEC) {
#pragma unroll
      for (int q = 0; q < N / 2; ++q) {
        const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(
            r, (int)(ok(2 * q) ? (e + 2 * q) * 8u : kOOB), 0, 0);
        v[2 * q] = __hiloint2double((int)w[1], (int)w[0]);
        v[2 * q + 1] = __hiloint2double((int)w[3], (int)w[2]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(ok(i) ? (e + i) * 8u : kOOB), 0, 0);
        v[i] = __hiloint2double((int)w[1], (int)w[0]);
      }
    }
  }
}

template <int BT, int SRCA, int SRCB, int BLAY, int OUT, bool VEC>
__global__ __launch_bounds__(256) void gemm_f64_kernel(G64Args g) {
  constexpr int BK = RPST_WCT_BK, LD = BT + 16, WT = BT / 2, MT = WT / 16;
  constexpr int EPT = BT * BK / 256;  // elements staged per thread per operand
  __shared__ double As[BK * LD];
  __shared__ double Bs[BK * LD];

  // tile decode
  int ti, tj;
  if (g.sym) {  // upper-triangular enumeration of tiles_n x tiles_n
    int t = blockIdx.x, r = 0;
    while (t >= g.tiles_n - r) {
      t -= g.tiles_n - r;
      ++r;
    }
    ti = r;
    tj = r + t;
  } else {
    ti = blockIdx.y;
    tj = blockIdx.x;
  }
  const int z = blockIdx.z;
  int b = z / g.ksplit;
  const int split = z - b * g.ksplit;
  const void* gA = g.A;
  const void* gB = g.B;
  void* gC = g.C;
  if (g.dual && b >= g.dual) {
    b -= g.dual;
    gA = g.A2;
    gB = g.B2;
    gC = g.C2;
  }
  const int m0 = ti * BT, n0 = tj * BT;
  // split-K ranges are whole BK tiles
  const int kper = ((g.K + g.ksplit - 1) / g.ksplit + BK - 1) / BK * BK;
  const int kbeg = split * kper;
  const int kend = min(g.K, kbeg + kper);

  constexpr unsigned ESA = src_f32(SRCA) ? 4u : 8u, ESB = src_f32(SRCB) ? 4u : 8u;
  const char* Ab = static_cast<const char*>(gA) + (int64_t)b * g.sA * ESA;
  const char* Bb = static_cast<const char*>(gB) + (int64_t)b * g.sB * ESB;
  const __amdgpu_buffer_rsrc_t ra = rsrc(Ab, (unsigned)g.M * g.lda * ESA);
  const __amdgpu_buffer_rsrc_t rb =
      rsrc(Bb, BLAY == B_NK ? (unsigned)g.N * g.ldb * ESB : (unsigned)g.K * g.ldb * ESB);
  const double* amean = g.amean ? g.amean + (int64_t)b * g.sMean : nullptr;
  const double* bmean = g.bmean ? g.bmean + (int64_t)b * g.sMean : nullptr;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lk = lane >> 4;

  doublex4 acc[MT][MT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jn = 0; jn < MT; ++jn) acc[i][jn] = doublex4{0.0, 0.0, 0.0, 0.0};

  // row-major [r][k] staging: thread -> (row sr = tid / TPR, k-run sk .. sk+EPT)
  constexpr int TPR = BK / EPT;
  const int sr = tid / TPR, sk = (tid % TPR) * EPT;
  // [k][n] staging: thread -> (k = kk_, n-run sn .. sn+EPT)
  constexpr int TPK = BT / EPT;
  const int kk_ = tid / TPK, sn = (tid % TPK) * EPT;

  const int am = m0 + sr;
  const bool am_ok = am < g.M;
  const double amu = (src_centred(SRCA) && am_ok) ? amean[am] : 0.0;
  const int bn = n0 + sr;  // B_NK row
  const bool bn_ok = bn < g.N;
  const double bmu_nk = (BLAY == B_NK && src_centred(SRCB) && bn_ok) ? bmean[bn] : 0.0;

  double ra_[EPT], rb_[EPT];
  auto load = [&](int k0) {
    {
      const int k = k0 + sk;
      load_run<SRCA, EPT, VEC>(ra_, ra, (unsigned)(am * g.lda + k),
                               [&](int i) { return am_ok && k + i < kend; });
#pragma unroll
      for (int i = 0; i < EPT; ++i) ra_[i] = (am_ok && k + i < kend) ? ra_[i] - amu : 0.0;
    }
    if (BLAY == B_NK) {
      const int k = k0 + sk;
      load_run<SRCB, EPT, VEC>(rb_, rb, (unsigned)(bn * g.ldb + k),
                               [&](int i) { return bn_ok && k + i < kend; });
#pragma unroll
      for (int i = 0; i < EPT; ++i) rb_[i] = (bn_ok && k + i < kend) ? rb_[i] - bmu_nk : 0.0;
    } else {
      const int k = k0 + kk_;
      const bool kok = k < kend;
      const double mu = (src_centred(SRCB) && kok) ? bmean[k] : 0.0;
      const int n = n0 + sn;
      load_run<SRCB, EPT, VEC>(rb_, rb, (unsigned)(k * g.ldb + n),
                               [&](int i) { return kok && n + i < g.N; });
#pragma unroll
      for (int i = 0; i < EPT; ++i) rb_[i] = (kok && n + i < g.N) ? rb_[i] - mu : 0.0;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < EPT; ++e) As[(sk + e) * LD + sr] = ra_[e];
    if (BLAY == B_NK) {
#pragma unroll
      for (int e = 0; e < EPT; ++e) Bs[(sk + e) * LD + sr] = rb_[e];
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e) Bs[kk_ * LD + sn + e] = rb_[e];
    }
  };

  const int ktiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (ktiles > 0) load(kbeg);
  for (int kt = 0; kt < ktiles; ++kt) {
    store();
    __syncthreads();
    if (kt + 1 < ktiles) load(kbeg + (kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      double av[MT], bv[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) av[i] = As[(ks * 4 + lk) * LD + wm * WT + i * 16 + lr];
#pragma unroll
      for (int i = 0; i < MT; ++i) bv[i] = Bs[(ks * 4 + lk) * LD + wn * WT + i * 16 + lr];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jn = 0; jn < MT; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[jn], acc[i][jn], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: D col = lane&15, row = (lane>>4) + 4r
  const double alpha = g.alpha * (g.avec ? g.avec[b] : 1.0);
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * WT + i * 16 + lk + 4 * r;
      if (m >= g.M) continue;
      const double bias = (OUT == OUT_F32_BIAS || OUT == OUT_F64_BIAS) ? g.bias[b * g.sMean + m] : 0.0;
#pragma unroll
      for (int jn = 0; jn < MT; ++jn) {
        const int n = n0 + wn * WT + jn * 16 + lr;
        if (n >= g.N) continue;
        const double v = acc[i][jn][r];
        if (OUT == OUT_PARTIAL) {
          static_cast<double*>(gC)[(int64_t)z * g.sC + (int64_t)m * g.ldc + n] = v;
        } else if (OUT == OUT_F64) {
          static_cast<double*>(gC)[b * g.sC + (int64_t)m * g.ldc + n] =
              alpha * v + (m == n ? g.beta_diag : 0.0);
        } else if (OUT == OUT_F32_BIAS) {
          static_cast<float*>(gC)[b * g.sC + (int64_t)m * g.ldc + n] = (float)(v + bias);
        } else {
          static_cast<double*>(gC)[b * g.sC + (int64_t)m * g.ldc + n] = v + bias;
        }
      }
    }
  }
}

// ---- WCT colour transform in fp32: out = T (cF - mu_c) + mu_s (wct_rp.py:109-113) ----
// T is computed in fp64 and rounded once; the product is a K = C GEMM over the fp32
// features, so it runs on the fp32 MFMA (2x the fp64 rate). Centering in fp32 and fp32
// accumulation over C = 256 terms: ~1.5e-7 rel-L2 vs the fp64 product on encoder features
// with |T| up to 100 (the fp32 output itself rounds at 6e-8).
__global__ __launch_bounds__(256) void wct_f32_prep_kernel(const double* __restrict__ T,
                                                           const double* __restrict__ mu,
                                                           float* __restrict__ Tf,
                                                           float* __restrict__ muf, int64_t nT,
                                                           int64_t nmu, int C) {
  // Tf = T^T per image ([k][m], output channels contiguous) so both GEMM operands stage
  // with 16-B loads and 16-B LDS stores
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nT) {
    const int64_t cc = (int64_t)C * C, b = i / cc, r = i - b * cc;
    const int m = (int)(r / C), k = (int)(r - (int64_t)m * C);
    Tf[b * cc + (int64_t)k * C + m] = (float)T[i];
  }
  if (i < nmu) muf[i] = (float)mu[i];
}

// Block tile 128 (m = output channel) x 128 (n = pixel), K = C in steps of 32, 4 waves of
// 64 x 64 on v_mfma_f32_32x32x2f32; register-prefetched staging of the next K step.
// A = T^T [n][C(k)][C(m)] (m contiguous), B = cF [n][C][HW] (pixels contiguous) centred by mu_c[k]
// while staged, epilogue adds mu_s[m]. VEC: 16-B loads (HW % 4 == 0, C % 4 == 0).
template <bool VEC>
__global__ __launch_bounds__(256, 2) void wct_transform_f32_kernel(
    const float* __restrict__ Tf, const float* __restrict__ X, const float* __restrict__ muc,
    const float* __restrict__ mus, float* __restrict__ out, int C, int HW) {
  constexpr int BK = 32, LD = 128 + 4;
  __shared__ float As[BK * LD];
  __shared__ float Bs[BK * LD];
  const int b = blockIdx.z;
  const int m0 = blockIdx.y * 128, n0 = blockIdx.x * 128;
  const float* A = Tf + (int64_t)b * C * C;
  const float* B = X + (int64_t)b * C * HW;
  const float* mc = muc + (int64_t)b * C;
  const float* ms = mus + (int64_t)b * C;
  float* O = out + (int64_t)b * C * HW;

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

  // staging of both operands: thread -> (k-row bk + 8p, run bn..bn+3 of m or n)
  const int bk = tid >> 5, bn = (tid & 31) * 4;
  float ra[16], rb[16];
  auto load = [&](int k0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int k = k0 + bk + 8 * p, m = m0 + bn;
      if (VEC) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < C && m < C) v = *reinterpret_cast<const float4*>(A + (int64_t)k * C + m);
        ra[4 * p] = v.x; ra[4 * p + 1] = v.y; ra[4 * p + 2] = v.z; ra[4 * p + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) ra[4 * p + e] = (k < C && m + e < C) ? A[(int64_t)k * C + m + e] : 0.f;
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int k = k0 + bk + 8 * p, n = n0 + bn;
      const float mu = k < C ? mc[k] : 0.f;
      if (VEC) {
        float4 v = make_float4(mu, mu, mu, mu);
        if (k < C && n < HW) v = *reinterpret_cast<const float4*>(B + (int64_t)k * HW + n);
        rb[4 * p] = v.x - mu; rb[4 * p + 1] = v.y - mu; rb[4 * p + 2] = v.z - mu; rb[4 * p + 3] = v.w - mu;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          rb[4 * p + e] = (k < C && n + e < HW) ? B[(int64_t)k * HW + n + e] - mu : 0.f;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int p = 0; p < 4; ++p)
      *reinterpret_cast<float4*>(As + (bk + 8 * p) * LD + bn) =
          make_float4(ra[4 * p], ra[4 * p + 1], ra[4 * p + 2], ra[4 * p + 3]);
#pragma unroll
    for (int p = 0; p < 4; ++p)
      *reinterpret_cast<float4*>(Bs + (bk + 8 * p) * LD + bn) =
          make_float4(rb[4 * p], rb[4 * p + 1], rb[4 * p + 2], rb[4 * p + 3]);
  };

  const int ktiles = (C + BK - 1) / BK;
  load(0);
  for (int kt = 0; kt < ktiles; ++kt) {
    store();
    __syncthreads();
    if (kt + 1 < ktiles) load((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
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

  // D: col n = lane & 31, row m = (r & 3) + 8 (r >> 2) + 4 h
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= C) continue;
      const float bias = ms[m];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int n = n0 + wn * 64 + nt * 32 + j;
        if (n < HW) O[(int64_t)m * HW + n] = acc[mt][nt][r] + bias;
      }
    }
}

// out = Tf^T-staged product: out[b] = T[b] (X[b] - muc[b]) + mus[b] for fp32 features
static int wct_transform_f32(const float* Tf, const float* X, const float* muc, const float* mus,
                             float* out, int n, int C, int64_t HW, hipStream_t st) {
  dim3 grid((unsigned)((HW + 127) / 128), (C + 127) / 128, n);
  const bool vec = (HW % 4 == 0) && (C % 4 == 0) && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  if (vec)
    wct_transform_f32_kernel<true><<<grid, 256, 0, st>>>(Tf, X, muc, mus, out, C, (int)HW);
  else
    wct_transform_f32_kernel<false><<<grid, 256, 0, st>>>(Tf, X, muc, mus, out, C, (int)HW);
  return launch_status("wct_transform_f32_kernel");
}

// Tf[b][k][m] = T[b][m][k] (fp32), muc = 0, mus = c (fp32): the operands of wct_transform_f32
// for z = T x + c
__global__ void wct_apply_prep_kernel(const double* __restrict__ T, const double* __restrict__ c,
                                      float* __restrict__ Tf, float* __restrict__ muc,
                                      float* __restrict__ mus, int64_t nT, int64_t nc, int C) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nT) {
    const int64_t cc = (int64_t)C * C, b = i / cc, r = i - b * cc;
    const int m = (int)(r / C), k = (int)(r - (int64_t)m * C);
    Tf[b * cc + (int64_t)k * C + m] = (float)T[i];
  }
  if (i < nc) {
    muc[i] = 0.f;
    mus[i] = (float)c[i];
  }
}

size_t wct_apply_scratch_floats(int n, int C) {
  return (size_t)n * C * C + 2 * (size_t)n * C + 64;
}

int wct_apply_f32(const double* T, const double* c, const float* x, float* z, int n, int C,
                  int64_t HW, float* scratch, hipStream_t st) {
  float* Tf = scratch;
  float* muc = Tf + (size_t)n * C * C;
  float* mus = muc + (size_t)n * C;
  const int64_t nT = (int64_t)n * C * C, nc = (int64_t)n * C;
  wct_apply_prep_kernel<<<(unsigned)((std::max(nT, nc) + 255) / 256), 256, 0, st>>>(
      T, c, Tf, muc, mus, nT, nc, C);
  if (int e = launch_status("wct_apply_prep_kernel")) return e;
  return wct_transform_f32(Tf, x, muc, mus, z, n, C, HW, st);
}

// Row means in fp64 of `rows` rows of length L (one workgroup per row).
template <typename T>
__global__ __launch_bounds__(256) void rowmean_kernel(const T* __restrict__ x0,
                                                      const T* __restrict__ x1, int rows0,
                                                      int64_t L, double* __restrict__ mean) {
  const int r = blockIdx.x;
  const T* x = (r < rows0 ? x0 + (int64_t)r * L : x1 + (int64_t)(r - rows0) * L);
  double s = 0.0;
  constexpr int V = 16 / sizeof(T);
  if ((L % V) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int64_t nv = L / V;
    int64_t i = threadIdx.x;
    for (; i + 256 < nv; i += 512) {  // two 16-B loads in flight per lane
      T a[V], c[V];
      *reinterpret_cast<u32x4*>(a) = reinterpret_cast<const u32x4*>(x)[i];
      *reinterpret_cast<u32x4*>(c) = reinterpret_cast<const u32x4*>(x)[i + 256];
#pragma unroll
      for (int t = 0; t < V; ++t) s += (double)a[t] + (double)c[t];
    }
    for (; i < nv; i += 256) {
      T a[V];
      *reinterpret_cast<u32x4*>(a) = reinterpret_cast<const u32x4*>(x)[i];
#pragma unroll
      for (int t = 0; t < V; ++t) s += (double)a[t];
    }
  } else {
    for (int64_t i = threadIdx.x; i < L; i += 256) s += (double)x[i];
  }
  s = wave_sum(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) mean[r] = ((red[0] + red[1]) + (red[2] + red[3])) / (double)L;
}

// C[b] = (sum_s P[b][s]) * scale + diag*I, symmetric fill from upper-triangular tiles.
__global__ void cov_reduce_kernel(const double* __restrict__ P, double* __restrict__ C, int n,
                                  int ksplit, int BT, double scale, double diag, int batch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)batch * n * n) return;
  const int b = (int)(i / ((int64_t)n * n));
  const int rem = (int)(i - (int64_t)b * n * n);
  int r = rem / n, c = rem - (rem / n) * n;
  if (r / BT > c / BT) {  // lower tile: read the transposed upper tile
    const int t = r;
    r = c;
    c = t;
  }
  double s = 0.0;
  for (int k = 0; k < ksplit; ++k) s += P[((int64_t)b * ksplit + k) * n * n + (int64_t)r * n + c];
  C[i] = s * scale + (r == c ? diag : 0.0);
}

// ---- host-side pipeline ------------------------------------------------------------
template <int BT, int SRCA, int SRCB, int BLAY, int OUT>
static void gemm64(const G64Args& g, dim3 grid, hipStream_t st) {
  // 16-B loads need every contiguous run to start on a 16-B boundary: sizes and leading
  // dims in whole vectors (4 floats / 2 doubles), split-K ranges are whole BK tiles.
  const int va = src_f32(SRCA) ? 4 : 2, vb = src_f32(SRCB) ? 4 : 2;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool vec = al(g.A) && al(g.B) && g.lda % va == 0 && g.ldb % vb == 0 && g.K % va == 0 &&
             g.sA % va == 0 && g.sB % vb == 0;
  if (g.dual) vec = vec && al(g.A2) && al(g.B2);
  if (BLAY == B_NK) vec = vec && g.K % vb == 0;
  else vec = vec && g.N % vb == 0;
  if (vec)
    gemm_f64_kernel<BT, SRCA, SRCB, BLAY, OUT, true><<<grid, 256, 0, st>>>(g);
  else
    gemm_f64_kernel<BT, SRCA, SRCB, BLAY, OUT, false><<<grid, 256, 0, st>>>(g);
}

static int env_int(const char* name, int dflt);

static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}

// Split-K of the covariance SYRK: a function of the per-image K only, so an image's
// summation order (and its bits) never depend on how many images share the launch (the
// per-image multi-GPU split relies on that). K >= kmin per split, at most 128 splits:
// at 512^2, 64 splits of 4096 (profiles/r01_wct_blocks.log: ~8192 workgroups at n = 16,
// 27.6 ms vs 28.9 at 4096 for the whole fuse).
static int pick_ksplit(int64_t K) {
  const int64_t kmin = env_int("RPST_WCT_KMIN", 4096);
  const int64_t s = K / kmin;
  return s < 1 ? 1 : (s > 128 ? 128 : (int)s);
}

struct WctLayout {
  int n, C, ksplit, BT, tiles, symtiles;
  bool v2;  // fp32 features with C <= 256: cov_syrk_kernel (rpst_wct_mat.hip)
  int64_t HW;
  // offsets in doubles
  size_t mu_c, mu_s, mu32, part, cc, cs, tm, off, tf, mf, orig;
  size_t total;
};

// src_f32: the features are fp32 (the v2 covariance applies for C <= 256)
static WctLayout wct_layout(int n, int C, int64_t HW, bool src_f32) {
  WctLayout L{};
  L.n = n;
  L.C = C;
  L.HW = HW;
  L.v2 = src_f32 && cov_v2_supported(C) && env_int("RPST_WCT_COV_V2", 1) != 0;
  L.BT = (C >= 128 && env_int("RPST_WCT_COV_BT", 128) == 128) ? 128 : 64;
  L.tiles = (C + L.BT - 1) / L.BT;
  L.symtiles = L.tiles * (L.tiles + 1) / 2;
  L.ksplit = pick_ksplit(HW);
  const size_t cc = (size_t)C * C * n;
  size_t o = 0;
  L.mu_c = o; o += (size_t)n * C;
  L.mu_s = o; o += (size_t)n * C;
  L.mu32 = o; o += ((size_t)2 * n * C + 1) / 2;  // fp32 centring means (v2 without `means`)
  L.part = o; o += L.v2 ? cov_v2_work_doubles(n, C, HW) : (size_t)2 * n * L.ksplit * C * C;
  L.cc = o; o += cc;
  L.cs = o; o += cc;
  L.tm = o; o += cc;
  L.off = o; o += (size_t)n * C;
  L.tf = o; o += cc / 2 + (size_t)n * C + 2;  // fp32 transform operands (wct_run)
  L.mf = o; o += matfun_wct_work_doubles(n, C);
  // whiten_and_color(method='original') (fp64 features, n = 1): (Cc + 1e-4 I)^(-1/2) and
  // (Cs + 1e-4 I)^(1/2) in SVD form, then the matrix-power workspace
  L.orig = o;
  if (!src_f32) o += (size_t)2 * n * C * C + matfun_power_work_doubles(C, n);
  L.total = o;
  return L;
}

// means (fp32, e.g. from the encoder's statistics epilogue: content rows then style rows,
// 2n x C) widened to fp64
__global__ void widen_means_kernel(const float* __restrict__ m, double* __restrict__ out,
                                   int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = (double)m[i];
}

__global__ void narrow_means_kernel(const double* __restrict__ m, float* __restrict__ out,
                                    int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = (float)m[i];
}

// WCT matrices of every image (wct_rp.py:85-109): fp64 means (mu_c, mu_s in the workspace),
// covariances, then T = Ic Mid Ic and offset = mu_s - T mu_c from the persistent matfun
// launch (original: T = (Cs + 1e-4 I)^(1/2) (Cc + 1e-4 I)^(-1/2) in the reference's SVD form,
// Li et al., wct_rp.py:96-101; offset unused). SRC is SRC_F32C (fp32 features) or SRC_F64C (fp64). means: optional fp32 (2n x C)
// row means (content rows then style rows), used to centre; residual (2n, optional): final
// Newton-Schulz residuals of (Cc + 1e-4 I) and of Mid's argument. T / offset: n x C x C / n x C.
// phase timing (rpst_wct_phase_timing / rpst_wct_phase_ms): events before the means, before
// the matrix-function launch and after it, on the closed-form path
static bool g_phase_on = false, g_phase_done = false;
static hipEvent_t g_phase_ev[3];
static void phase_mark(int i, hipStream_t st) {
  if (!g_phase_on) return;
  static const bool made = [] {
    for (auto& e : g_phase_ev) (void)hipEventCreate(&e);
    return true;
  }();
  (void)made;
  (void)hipEventRecord(g_phase_ev[i], st);
  if (i == 2) g_phase_done = true;
}

template <int SRC>
static int wct_matrices_impl(const void* cF, const void* sF, const float* means, int n, int C,
                        int64_t HW, const WctLayout& L, double* ws, double* T, double* offset,
                        double* residual, hipStream_t st, bool original = false) {
  double *mu_c = ws + L.mu_c, *part = ws + L.part;
  double *Cc = ws + L.cc, *Cs = ws + L.cs;
  const int64_t cnt = (int64_t)2 * n * C;
  if (SRC == SRC_F32C && L.v2) {
    // centre on fp32 means (given, or the fp64 row means rounded); cov_v2 recovers the exact
    // fp64 means and covariances from the centred row sums
    const float* mu32 = means;
    if (!mu32) {
      rowmean_kernel<float><<<2 * n * C, 256, 0, st>>>(static_cast<const float*>(cF),
                                                      static_cast<const float*>(sF), n * C, HW, mu_c);
      float* m32 = reinterpret_cast<float*>(ws + L.mu32);
      narrow_means_kernel<<<(unsigned)((cnt + 255) / 256), 256, 0, st>>>(mu_c, m32, cnt);
      if (int e = launch_status("rowmean_kernel")) return e;
      mu32 = m32;
    }
    if (int e = cov_v2(static_cast<const float*>(cF), static_cast<const float*>(sF), mu32, n, C,
                       HW, Cc, Cs, mu_c, part, st))
      return e;
  } else {
    // 1. means (content rows then style rows; mu_s follows mu_c in the workspace)
    if (means) {
      widen_means_kernel<<<(unsigned)((cnt + 255) / 256), 256, 0, st>>>(means, mu_c, cnt);
      if (int e = launch_status("widen_means_kernel")) return e;
    } else {
      if (SRC == SRC_F32C)
        rowmean_kernel<float><<<2 * n * C, 256, 0, st>>>(static_cast<const float*>(cF),
                                                        static_cast<const float*>(sF), n * C, HW, mu_c);
      else
        rowmean_kernel<double><<<2 * n * C, 256, 0, st>>>(static_cast<const double*>(cF),
                                                         static_cast<const double*>(sF), n * C, HW, mu_c);
      if (int e = launch_status("rowmean_kernel")) return e;
    }
    double* mu_s = ws + L.mu_s;
    // 2. covariances: upper-triangular tiles, split-K partials, fixed-order reduce
    for (int which = 0; which < 2; ++which) {
      G64Args g{};
      g.A = g.B = which == 0 ? cF : sF;
      g.C = part + (size_t)which * n * L.ksplit * C * C;
      g.amean = g.bmean = which == 0 ? mu_c : mu_s;
      g.sMean = C;
      g.M = g.N = C;
      g.K = (int)HW;
      g.lda = g.ldb = (int)HW;
      g.ldc = C;
      g.sA = g.sB = (int64_t)C * HW;
      g.sC = (int64_t)C * C;
      g.ksplit = L.ksplit;
      g.sym = 1;
      g.tiles_n = L.tiles;
      dim3 grid(L.symtiles, 1, n * L.ksplit);
      if (L.BT == 128)
        gemm64<128, SRC, SRC, B_NK, OUT_PARTIAL>(g, grid, st);
      else
        gemm64<64, SRC, SRC, B_NK, OUT_PARTIAL>(g, grid, st);
      if (int e = launch_status("gemm_f64_kernel(cov)")) return e;
    }
    const int64_t nel = (int64_t)n * C * C;
    const unsigned rb = (unsigned)((nel + 255) / 256);
    cov_reduce_kernel<<<rb, 256, 0, st>>>(part, Cc, C, L.ksplit, L.BT, 1.0 / (double)(HW - 1), 1.0, n);
    cov_reduce_kernel<<<rb, 256, 0, st>>>(part + (size_t)n * L.ksplit * C * C, Cs, C, L.ksplit, L.BT,
                                          1.0 / (double)(HW - 1), 0.0, n);
    if (int e = launch_status("cov_reduce_kernel")) return e;
  }
  if (original) {
    // 3'. Li et al.: cF_inv_sqrt = matrix_inv_sqrt(Cc), sF_sqrt = matrix_sqrt(Cs) (each the
    //     SVD form with the 1e-5 truncation: Newton-Schulz, Jacobi where it could differ),
    //     T = sF_sqrt cF_inv_sqrt; sF_sqrt (cF_inv_sqrt cF) of wct_rp.py:101 is the same
    //     product up to fp64 association. No barrier-timeout state is left in L.mf: flagged
    //     matrices are recomputed by the Jacobi kernel.
    double* Ai = ws + L.orig;
    double* Bs = Ai + (size_t)n * C * C;
    double* pw = Bs + (size_t)n * C * C;
    if (int e = matfun_power(Cc, Ai, C, n, 1, nullptr, pw, st)) return e;
    if (int e = matfun_power(Cs, Bs, C, n, 0, nullptr, pw, st)) return e;
    if (int e = matfun_wct_clear_status(ws + L.mf, n, C, st)) return e;
    G64Args g{};
    g.A = Bs;
    g.B = Ai;
    g.C = T;
    g.alpha = 1.0;
    g.M = g.N = g.K = C;
    g.lda = g.ldb = g.ldc = C;
    g.sA = g.sB = g.sC = (int64_t)C * C;
    g.ksplit = 1;
    dim3 grid((unsigned)((C + 63) / 64), (unsigned)((C + 63) / 64), n);
    gemm64<64, SRC_F64, SRC_F64, B_KN, OUT_F64>(g, grid, st);
    return launch_status("gemm_f64_kernel(original T)");
  }
  // 3. Sc, Ic = (Cc + 1e-4 I)^(+-1/2); Mid = (Sc Cs Sc + 1e-4 I)^(1/2); T = Ic Mid Ic;
  //    offset = mu_s - T mu_c: one persistent launch
  phase_mark(1, st);
  return matfun_wct(Cc, Cs, mu_c, T, offset, residual, n, C, ws + L.mf, st);
}

template <int SRC>
static int wct_matrices(const void* cF, const void* sF, const float* means, int n, int C,
                        int64_t HW, const WctLayout& L, double* ws, double* T, double* offset,
                        double* residual, hipStream_t st, bool original = false) {
  if (!original) phase_mark(0, st);
  const int e = wct_matrices_impl<SRC>(cF, sF, means, n, C, HW, L, ws, T, offset, residual, st,
                                       original);
  if (!original && !e) phase_mark(2, st);
  return e;
}

// Shared WCT body: the matrices, then out = T (cF - mu_c) + mu_s.
template <int SRC, int OUTM>
static int wct_run(const void* cF, const void* sF, void* out, int n, int C, int64_t HW,
                   void* workspace, double* residual, hipStream_t st, bool original = false) {
  const WctLayout L = wct_layout(n, C, HW, SRC == SRC_F32C);
  double* ws = static_cast<double*>(workspace);
  double *mu_c = ws + L.mu_c, *mu_s = ws + L.mu_s, *Tm = ws + L.tm;
  if (int e = wct_matrices<SRC>(cF, sF, nullptr, n, C, HW, L, ws, Tm, ws + L.off, residual, st,
                                original))
    return e;

  // out = T (cF - mu_c) + mu_s; fp32 features -> fp32 MFMA (RPST_WCT_T_F64=1: fp64)
  if (SRC == SRC_F32C && OUTM == OUT_F32_BIAS && !env_int("RPST_WCT_T_F64", 0)) {
    float* Tf = reinterpret_cast<float*>(ws + L.tf);
    float* muf = Tf + (size_t)n * C * C;
    const int64_t nT = (int64_t)n * C * C, nmu = (int64_t)2 * n * C;  // mu_c, mu_s adjacent
    wct_f32_prep_kernel<<<(unsigned)((std::max(nT, nmu) + 255) / 256), 256, 0, st>>>(Tm, mu_c, Tf, muf, nT, nmu, C);
    if (int e = launch_status("wct_f32_prep_kernel")) return e;
    return wct_transform_f32(Tf, static_cast<const float*>(cF), muf, muf + (size_t)n * C,
                             static_cast<float*>(out), n, C, HW, st);
  }
  G64Args g{};
  g.A = Tm;
  g.B = cF;
  g.C = out;
  g.bmean = mu_c;
  g.bias = mu_s;
  g.sMean = C;
  g.M = C;
  g.N = (int)HW;
  g.K = C;
  g.lda = C;
  g.ldb = (int)HW;
  g.ldc = (int)HW;
  g.sA = (int64_t)C * C;
  g.sB = (int64_t)C * HW;
  g.sC = (int64_t)C * HW;
  g.ksplit = 1;
  if (env_int("RPST_WCT_T_BT", 64) == 128) {
    dim3 grid((unsigned)((HW + 127) / 128), (C + 127) / 128, n);
    gemm64<128, SRC_F64, SRC, B_KN, OUTM>(g, grid, st);
  } else {
    dim3 grid((unsigned)((HW + 63) / 64), (C + 63) / 64, n);
    gemm64<64, SRC_F64, SRC, B_KN, OUTM>(g, grid, st);
  }
  return launch_status("gemm_f64_kernel(transform)");
}

// out[n] = W T[n]: W (rows x K) fp32 shared by the batch, T[n] (K x K) fp64 -> fp64 (rows x K);
// the per-image folded weights W T_n of rpst_conv2d_mix (rpst_wino4.hip) on the fp64 MFMA
int gemm_f32w_f64(const float* W, const double* T, double* out, int n, int rows, int K,
                  hipStream_t st) {
  G64Args g{};
  g.A = W;
  g.B = T;
  g.C = out;
  g.alpha = 1.0;
  g.M = rows;
  g.N = K;
  g.K = K;
  g.lda = K;
  g.ldb = K;
  g.ldc = K;
  g.sA = 0;
  g.sB = (int64_t)K * K;
  g.sC = (int64_t)rows * K;
  g.ksplit = 1;
  dim3 grid((unsigned)((K + 63) / 64), (unsigned)((rows + 63) / 64), n);
  gemm64<64, SRC_F32, SRC_F64, B_KN, OUT_F64>(g, grid, st);
  return launch_status("gemm_f64_kernel(mix weights)");
}

}  // namespace rpst

using namespace rpst;

extern "C" size_t rpst_wct_workspace_size(int n, int C, int64_t HW) {
  if (n <= 0 || C <= 0 || HW <= 1) return 0;
  // the larger of the fp32-feature and fp64-feature layouts (one size for every entry point)
  const size_t a = wct_layout(n, C, HW, true).total, b = wct_layout(n, C, HW, false).total;
  return (a > b ? a : b) * sizeof(double);
}

extern "C" int rpst_wct_fuse(const float* content, const float* style, float* out, int n, int C,
                             int64_t HW, double* residual, void* workspace,
                             size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(content && style && out, "wct_fuse: null pointer");
  RPST_REQUIRE(n > 0 && C > 0 && HW > 1, "wct_fuse: bad shape n=%d C=%d HW=%lld", n, C, (long long)HW);
  RPST_REQUIRE(HW <= 0x7fffffffLL && n <= 32767 && C <= 1024, "wct_fuse: shape too large");
  if (!workspace || workspace_bytes < rpst_wct_workspace_size(n, C, HW)) {
    set_error("wct_fuse: workspace %zu < %zu bytes", workspace_bytes, rpst_wct_workspace_size(n, C, HW));
    return RPST_EWORKSPACE;
  }
  return wct_run<SRC_F32C, OUT_F32_BIAS>(content, style, out, n, C, HW, workspace, residual,
                                         as_stream(stream));
}

extern "C" int rpst_wct_params(const float* content, const float* style, const float* means,
                               double* T, double* offset, int n, int C, int64_t HW,
                               double* residual, void* workspace, size_t workspace_bytes,
                               rpst_stream_t stream) {
  RPST_REQUIRE(content && style && T && offset, "wct_params: null pointer");
  RPST_REQUIRE(n > 0 && C > 0 && HW > 1, "wct_params: bad shape n=%d C=%d HW=%lld", n, C,
               (long long)HW);
  RPST_REQUIRE(HW <= 0x7fffffffLL && n <= 65535, "wct_params: shape too large");
  if (!workspace || workspace_bytes < rpst_wct_workspace_size(n, C, HW)) {
    set_error("wct_params: workspace %zu < %zu bytes", workspace_bytes,
              rpst_wct_workspace_size(n, C, HW));
    return RPST_EWORKSPACE;
  }
  RPST_REQUIRE(C <= 1024, "wct_params: C=%d > 1024", C);
  hipStream_t st = as_stream(stream);
  const WctLayout L = wct_layout(n, C, HW, true);
  return wct_matrices<SRC_F32C>(content, style, means, n, C, HW, L, static_cast<double*>(workspace),
                                T, offset, residual, st);
}

extern "C" int rpst_whiten_and_color_f64(const double* cF, const double* sF, double* out, int C,
                                         int64_t HW, double* residual, void* workspace,
                                         size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(cF && sF && out, "whiten_and_color: null pointer");
  RPST_REQUIRE(C > 0 && C <= 1024 && HW > 1 && HW <= 0x7fffffffLL, "whiten_and_color: bad shape");
  if (!workspace || workspace_bytes < rpst_wct_workspace_size(1, C, HW)) {
    set_error("whiten_and_color: workspace too small");
    return RPST_EWORKSPACE;
  }
  return wct_run<SRC_F64C, OUT_F64_BIAS>(cF, sF, out, 1, C, HW, workspace, residual,
                                         as_stream(stream));
}

extern "C" int rpst_whiten_and_color_original_f64(const double* cF, const double* sF,
                                                  double* out, int C, int64_t HW, void* workspace,
                                                  size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(cF && sF && out, "whiten_and_color(original): null pointer");
  RPST_REQUIRE(C > 0 && C <= 1024 && HW > 1 && HW <= 0x7fffffffLL,
               "whiten_and_color(original): bad shape");
  if (!workspace || workspace_bytes < rpst_wct_workspace_size(1, C, HW)) {
    set_error("whiten_and_color(original): workspace too small");
    return RPST_EWORKSPACE;
  }
  return wct_run<SRC_F64C, OUT_F64_BIAS>(cF, sF, out, 1, C, HW, workspace, nullptr,
                                         as_stream(stream), true);
}

extern "C" int rpst_wct_status(const void* workspace, int n, int C, int64_t HW, int* status,
                               rpst_stream_t stream) {
  RPST_REQUIRE(workspace && status, "wct_status: null pointer");
  RPST_REQUIRE(n > 0 && C > 0 && C <= 1024 && HW > 1, "wct_status: bad shape");
  // rpst_wct_fuse / rpst_wct_params lay the workspace out for fp32 features
  const WctLayout L = wct_layout(n, C, HW, true);
  double* ws = static_cast<double*>(const_cast<void*>(workspace));
  return matfun_wct_status(ws + L.mf, n, C, status, as_stream(stream));
}

extern "C" int rpst_wct_phase_timing(int on) {
  const int old = g_phase_on;
  g_phase_on = on != 0;
  if (on) g_phase_done = false;
  return old;
}

extern "C" int rpst_wct_phase_ms(float* cov_ms, float* matfun_ms) {
  RPST_REQUIRE(cov_ms && matfun_ms, "wct_phase_ms: null pointer");
  RPST_REQUIRE(g_phase_done, "wct_phase_ms: no call recorded while armed");
  if (hipEventSynchronize(g_phase_ev[2]) != hipSuccess ||
      hipEventElapsedTime(cov_ms, g_phase_ev[0], g_phase_ev[1]) != hipSuccess ||
      hipEventElapsedTime(matfun_ms, g_phase_ev[1], g_phase_ev[2]) != hipSuccess) {
    set_error("wct_phase_ms: event query failed");
    return RPST_EHIP;
  }
  return RPST_OK;
}

extern "C" int rpst_whiten_and_color_status(const void* workspace, int C, int64_t HW, int* status,
                                            rpst_stream_t stream) {
  RPST_REQUIRE(workspace && status, "whiten_and_color_status: null pointer");
  RPST_REQUIRE(C > 0 && C <= 1024 && HW > 1, "whiten_and_color_status: bad shape");
  const WctLayout L = wct_layout(1, C, HW, false);
  double* ws = static_cast<double*>(const_cast<void*>(workspace));
  return matfun_wct_status(ws + L.mf, 1, C, status, as_stream(stream));
}

extern "C" size_t rpst_matrix_power_workspace_size(int n, int batch) {
  if (n <= 0 || batch <= 0) return 0;
  return matfun_power_work_doubles(n, batch) * sizeof(double);
}

extern "C" int rpst_matrix_power_psd_f64(const double* A, double* out, int n, int batch,
                                         int inverse, double* residual, void* workspace,
                                         size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(A && out, "matrix_power: null pointer");
  RPST_REQUIRE(n > 0 && n <= 1024 && batch > 0 && batch <= 65535, "matrix_power: bad shape");
  if (!workspace || workspace_bytes < rpst_matrix_power_workspace_size(n, batch)) {
    set_error("matrix_power: workspace too small");
    return RPST_EWORKSPACE;
  }
  return matfun_power(A, out, n, batch, inverse, residual, static_cast<double*>(workspace),
                      as_stream(stream));
}
