// WCT matrices on gfx950 (network/wct_rp.py:7-40, 82-109): the covariance SYRK of fp32
// features, the closed-form matrix functions as ONE persistent launch, and the reference's
// SVD form for inputs Newton-Schulz cannot take.
//
// 1. cov_syrk_kernel (C <= 128) / cov_syrk16_kernel (C in (128, 256], 16 waves, operand reuse:
//    see its comment): one workgroup per (image matrix, K split) computes EVERY
//    upper-triangular 16x16 block of the C x C product (C <= 256), so the k-run of all C
//    rows is staged once (fp32 -> fp64, centred) and serves as both MFMA operands
//    (v_mfma_f64_16x16x4_f64: A[l&15][k=l>>4] and B[k=l>>4][l&15] are the same lane map of
//    X). The 128x128-tile SYRK of rpst_wct.hip staged the rows of each diagonal tile twice
//    and computed 3/4 of the square; here the executed blocks are (NB+1)/(2 NB) of it and each
//    staged element feeds NB+1 ... 2 NB blocks. K splits are a function of HW only (bitwise
//    batch invariance), partials are combined in fixed order by cov_finish_kernel.
// 2. matfun_kernel: the Newton-Schulz square roots, the products Sc Cs Sc and Ic Mid Ic and the
//    offset mu_s - T mu_c for every image in one launch. A group of P workgroups (one 64x64
//    output tile each) works on one matrix at a time; the phases of a matrix are separated by a
//    group barrier (agent-scope release / acquire, MI355X_MICROARCH.md inter-workgroup
//    visibility) and every reduction (Frobenius norms, the residual ||I - Z Y||_F) is summed by
//    every workgroup from the per-tile partials in the same fixed order, so the convergence
//    decision is uniform over the group and deterministic. No host synchronisation: the
//    iteration count lives on the device (the previous version polled convergence flags from
//    the host every 4 iterations).
//    Convergence (per matrix): r_k = 2 ||T_k - I||_F below max(1e-10, the fp64 rounding floor
//    8 eps n ||Y_k||_F ||Z_k||_F), or stalled (r_k > 0.9 r_{k-1} once r_{k-1} < 1e-6): an
//    ill-conditioned but valid input (Mid's argument with a dead style channel) stops at its
//    rounding floor instead of failing a fixed absolute bar.
// 3. jacobi_power_kernel: torch.svd's form V diag(s^p) V^T (s >= 1e-5 only) by one-sided
//    (Hestenes) Jacobi, for the function-level matrix_sqrt / matrix_inv_sqrt on inputs that are
//    not symmetric, not positive definite or whose smallest eigenvalue may be under the 1e-5
//    truncation (cheap exit for every other matrix; no host decision).
#include "rpst_wct.h"

#include <type_traits>

namespace rpst {

// ======================= 1. covariance of fp32 features ==================================

constexpr int kCovBK = 32;       // staged k depth
constexpr int kCovSplits = 8;    // K splits per matrix (HW >= 8 x 32): 8 x 2n workgroups
#ifndef RPST_COV_UNROLL  // cov_syrk16_kernel: k sub-steps unrolled per stage (1 / 2 / 8:
#define RPST_COV_UNROLL 2  // wct_params 12.35 / 12.08 / 13.03 ms at n 16, C 256, 512^2)
#endif

struct CovArgs {
  const float* X0;     // content (n, C, HW)
  const float* X1;     // style (n, C, HW)
  const float* mu32;   // (2n, C) centring means
  double* part;        // [2n][ksplit * KG][nblk][16][16]
  double* rsum;        // [2n][ksplit][C]
  int n, C, ksplit, kper;
  int64_t HW;
};

__host__ __device__ constexpr int cov_nb(int C) { return C <= 64 ? 4 : (C <= 128 ? 8 : 16); }
__host__ __device__ constexpr int cov_kg(int NB) { return NB == 4 ? 4 : (NB == 8 ? 2 : 1); }

template <int NB, bool VEC>
__global__ __launch_bounds__(512, 1) void cov_syrk_kernel(CovArgs a) {
  constexpr int KG = cov_kg(NB);          // k groups (waves splitting the k4 sub-steps)
  constexpr int R = 16 * NB, LDX = R + 16;  // LDX: k and k+1 rows on opposite bank halves
  constexpr int TPR = 512 / R, EPT = kCovBK / TPR;
  constexpr int NBLK = NB * (NB + 1) / 2, WGR = 8 / KG, MB = (NBLK + WGR - 1) / WGR;
  static_assert(EPT % 4 == 0, "16-B staging runs");
  __shared__ __attribute__((aligned(16))) double Xs[2][kCovBK * LDX];

  const int split = blockIdx.x, z = blockIdx.y;
  const int n = a.n, C = a.C;
  const float* X = z < n ? a.X0 + (int64_t)z * C * a.HW : a.X1 + (int64_t)(z - n) * C * a.HW;
  const int64_t kbeg = (int64_t)split * a.kper;
  const int64_t kend = a.HW < kbeg + a.kper ? a.HW : kbeg + a.kper;
  const int nst = (int)((kend - kbeg + kCovBK - 1) / kCovBK);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kgrp = wave % KG, wgrp = wave / KG;
  const int sr = tid % R, sk = tid / R;  // staged row, k segment
  const bool rok = sr < C;
  const float mu = rok ? a.mu32[(int64_t)z * C + sr] : 0.f;
  const float* xr = X + (int64_t)(rok ? sr : 0) * a.HW;

  float rx[EPT];
  double rs = 0.0;  // row sum of the centred values this thread staged
  auto load = [&](int st) {
    const int64_t k0 = kbeg + (int64_t)st * kCovBK + sk * EPT;
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const int64_t k = k0 + 4 * q;
      if (VEC) {  // HW % 4 == 0: a 16-B run is wholly inside or outside [kbeg, kend)
        float4 v = make_float4(mu, mu, mu, mu);
        if (rok && k < kend) v = *reinterpret_cast<const float4*>(xr + k);
        rx[4 * q] = v.x;
        rx[4 * q + 1] = v.y;
        rx[4 * q + 2] = v.z;
        rx[4 * q + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) rx[4 * q + e] = (rok && k + e < kend) ? xr[k + e] : mu;
      }
    }
  };
  auto store = [&](double* xs) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const double d = (double)rx[e] - (double)mu;  // exact in fp64
      rs += d;
      xs[(sk * EPT + e) * LDX + sr] = d;
    }
  };

  // this wave's blocks: slot q -> block b = wgrp + q * WGR of the row-major upper triangle
  int bi[MB], bj[MB];
#pragma unroll
  for (int q = 0; q < MB; ++q) {
    int b = wgrp + q * WGR, i = 0;
    if (b >= NBLK) b = 0;
    while (b >= NB - i) {
      b -= NB - i;
      ++i;
    }
    bi[q] = 16 * i;
    bj[q] = 16 * (i + b);
  }
  doublex4 acc[MB];
#pragma unroll
  for (int q = 0; q < MB; ++q) acc[q] = doublex4{0.0, 0.0, 0.0, 0.0};

  if (nst > 0) {
    load(0);
    store(Xs[0]);
  }
  for (int st = 0; st < nst; ++st) {
    __syncthreads();  // stage st is in Xs[st & 1]; every wave is done with stage st - 1
    if (st + 1 < nst) load(st + 1);
    const double* xs = Xs[st & 1];
#pragma unroll
    for (int ks = 0; ks < kCovBK / 4; ++ks) {
      if (ks % KG != kgrp) continue;
      const double* xk = xs + (4 * ks + (lane >> 4)) * LDX + (lane & 15);
#pragma unroll
      for (int q = 0; q < MB; ++q) {
        if (wgrp + q * WGR >= NBLK) continue;
        const double av = xk[bi[q]], bv = xk[bj[q]];
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[q], 0, 0, 0);
      }
    }
    if (st + 1 < nst) store(Xs[(st + 1) & 1]);
  }

  // partial blocks: D col = lane & 15, row = (lane >> 4) + 4 r
  const int PS = a.ksplit * KG, ps = split * KG + kgrp;
  double* P = a.part + ((int64_t)z * PS + ps) * NBLK * 256;
#pragma unroll
  for (int q = 0; q < MB; ++q) {
    const int b = wgrp + q * WGR;
    if (b >= NBLK) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) P[(b * 16 + (lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[q][r];
  }
  // row sums over the TPR threads of a row (fixed order)
  __syncthreads();
  double* red = Xs[0];
  red[sk * R + sr] = rs;
  __syncthreads();
  if (tid < R && tid < C) {
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < TPR; ++t) s += red[t * R + tid];
    a.rsum[((int64_t)z * a.ksplit + split) * C + tid] = s;
  }
}

// C in (128, 256] (NB = 16): the same product with 16 waves (four per SIMD) and operand
// reuse. The upper triangle of 16 x 16 blocks is 10 super-blocks of 4 x 4 blocks: waves 0-11
// each own half of an off-diagonal super-block (4 x 2 blocks from 6 operand reads per k
// sub-step: A and B share one lane map, so the registers of block row I serve as A of row I
// and as B of column I), waves 12-15 one diagonal super-block each (10 blocks from 4 reads);
// every SIMD (waves s, s + 4, s + 8, s + 12) carries 3 x 8 + 10 = 34 blocks. The strided map
// of cov_syrk_kernel reads two operands per MFMA. Partials as cov_syrk_kernel<16> (KG = 1).
template <bool VEC>
__global__ __launch_bounds__(1024, 1) void cov_syrk16_kernel(CovArgs a) {
  constexpr int NB = 16, R = 256, LDX = R + 16;
  constexpr int TPR = 1024 / R, EPT = kCovBK / TPR;
  constexpr int NBLK = NB * (NB + 1) / 2;
  static_assert(EPT % 4 == 0, "16-B staging runs");
  __shared__ __attribute__((aligned(16))) double Xs[2][kCovBK * LDX];

  const int split = blockIdx.x, z = blockIdx.y;
  const int n = a.n, C = a.C;
  const float* X = z < n ? a.X0 + (int64_t)z * C * a.HW : a.X1 + (int64_t)(z - n) * C * a.HW;
  const int64_t kbeg = (int64_t)split * a.kper;
  const int64_t kend = a.HW < kbeg + a.kper ? a.HW : kbeg + a.kper;
  const int nst = (int)((kend - kbeg + kCovBK - 1) / kCovBK);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sr = tid % R, sk = tid / R;  // staged row, k segment
  const bool rok = sr < C;
  const float mu = rok ? a.mu32[(int64_t)z * C + sr] : 0.f;
  const float* xr = X + (int64_t)(rok ? sr : 0) * a.HW;

  float rx[EPT];
  double rs = 0.0;
  auto load = [&](int st) {
    const int64_t k0 = kbeg + (int64_t)st * kCovBK + sk * EPT;
#pragma unroll
    for (int q = 0; q < EPT / 4; ++q) {
      const int64_t k = k0 + 4 * q;
      if (VEC) {
        float4 v = make_float4(mu, mu, mu, mu);
        if (rok && k < kend) v = *reinterpret_cast<const float4*>(xr + k);
        rx[4 * q] = v.x;
        rx[4 * q + 1] = v.y;
        rx[4 * q + 2] = v.z;
        rx[4 * q + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) rx[4 * q + e] = (rok && k + e < kend) ? xr[k + e] : mu;
      }
    }
  };
  auto store = [&](double* xs) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const double d = (double)rx[e] - (double)mu;  // exact in fp64
      rs += d;
      xs[(sk * EPT + e) * LDX + sr] = d;
    }
  };

  // roles: off-diagonal super-block pairs (0,1) (0,2) (0,3) (1,2) (1,3) (2,3), two column
  // halves each (waves 0-11); diagonal super-blocks 0-3 (waves 12-15)
  const bool diag = wave >= 12;
  int rI = 0, cJ = 0;  // first block row / column of the wave's region
  if (!diag) {
    const int sb = wave >> 1, h = wave & 1;
    const int si = sb < 3 ? 0 : (sb < 5 ? 1 : 2);
    const int sj = sb < 3 ? sb + 1 : (sb < 5 ? sb - 1 : 3);
    rI = 4 * si;
    cJ = 4 * sj + 2 * h;
  } else {
    rI = cJ = 4 * (wave - 12);
  }
  double* P = a.part + ((int64_t)z * a.ksplit + split) * NBLK * 256;
  auto put = [&](int bi, int bj, const doublex4& v) {
    const int b = bi * NB - bi * (bi - 1) / 2 + (bj - bi);
#pragma unroll
    for (int r = 0; r < 4; ++r) P[(b * 16 + (lane >> 4) + 4 * r) * 16 + (lane & 15)] = v[r];
  };
  // one loop per role (the two accumulator layouts never meet in one loop's registers);
  // both run nst stages with one barrier each, so the workgroup's barriers stay uniform
  auto run = [&](auto DIAGc) __attribute__((always_inline)) {
    constexpr bool D = decltype(DIAGc)::value;
    constexpr int NA = D ? 10 : 8;
    doublex4 acc[NA];
#pragma unroll
    for (int q = 0; q < NA; ++q) acc[q] = doublex4{0.0, 0.0, 0.0, 0.0};
    if (nst > 0) {
      load(0);
      store(Xs[0]);
    }
    for (int st = 0; st < nst; ++st) {
      __syncthreads();  // stage st is in Xs[st & 1]; every wave is done with stage st - 1
      if (st + 1 < nst) load(st + 1);
      const double* xs = Xs[st & 1];
#pragma unroll RPST_COV_UNROLL
      for (int ks = 0; ks < kCovBK / 4; ++ks) {
        const double* xk = xs + (4 * ks + (lane >> 4)) * LDX + (lane & 15);
        double r[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = xk[16 * (rI + i)];
        if constexpr (!D) {
          double c[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) c[j] = xk[16 * (cJ + j)];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[2 * i + j] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[i], c[j], acc[2 * i + j], 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j) {
              const int q = i * 4 - i * (i - 1) / 2 + (j - i);
              acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(r[i], r[j], acc[q], 0, 0, 0);
            }
        }
      }
      if (st + 1 < nst) store(Xs[(st + 1) & 1]);
    }
    // partial blocks (f64 map: D col = lane & 15, row = (lane >> 4) + 4 r)
    if constexpr (!D) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) put(rI + i, cJ + j, acc[2 * i + j]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) put(rI + i, rI + j, acc[i * 4 - i * (i - 1) / 2 + (j - i)]);
    }
  };
  if (diag) run(std::true_type{});
  else run(std::false_type{});
  // row sums over the TPR threads of a row (fixed order)
  __syncthreads();
  double* red = Xs[0];
  red[sk * R + sr] = rs;
  __syncthreads();
  if (tid < R && tid < C) {
    double sum = 0.0;
#pragma unroll
    for (int t = 0; t < TPR; ++t) sum += red[t * R + tid];
    a.rsum[((int64_t)z * a.ksplit + split) * C + tid] = sum;
  }
}

// Cc / Cs / mu64 from the partials: S = sum of the partials of the (r, c) block (upper
// triangle; the lower one mirrors it), delta_r = (row sum of x - mu32) / HW,
// cov = (S - HW delta_r delta_c) / (HW - 1) (+ I for the content matrices, wct_rp.py:89).
__global__ void cov_finish_kernel(const double* __restrict__ part, const double* __restrict__ rsum,
                                  const float* __restrict__ mu32, double* __restrict__ Cc,
                                  double* __restrict__ Cs, double* __restrict__ mu64, int n, int C,
                                  int NB, int PS, int ksplit, int64_t HW) {
  const int64_t cc = (int64_t)C * C;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * n * cc) return;
  const int z = (int)(i / cc);
  const int rem = (int)(i - (int64_t)z * cc);
  const int r = rem / C, c = rem - r * C;
  int rr = r, cl = c;
  if (rr / 16 > cl / 16) {
    rr = c;
    cl = r;
  }
  const int bi = rr / 16, bj = cl / 16, nblk = NB * (NB + 1) / 2;
  const int b = bi * NB - bi * (bi - 1) / 2 + (bj - bi);
  const double* p = part + ((int64_t)z * PS * nblk + b) * 256 + (rr & 15) * 16 + (cl & 15);
  double s = 0.0;
  for (int q = 0; q < PS; ++q) s += p[(int64_t)q * nblk * 256];
  double sr = 0.0, sc = 0.0;
  for (int q = 0; q < ksplit; ++q) {
    sr += rsum[((int64_t)z * ksplit + q) * C + r];
    sc += rsum[((int64_t)z * ksplit + q) * C + c];
  }
  const double dr = sr / (double)HW, dc = sc / (double)HW;
  const double cov = (s - (double)HW * dr * dc) / (double)(HW - 1);
  if (z < n) Cc[(int64_t)z * cc + rem] = cov + (r == c ? 1.0 : 0.0);
  else Cs[(int64_t)(z - n) * cc + rem] = cov;
  if (c == 0) mu64[(int64_t)z * C + r] = (double)mu32[(int64_t)z * C + r] + dr;
}

bool cov_v2_supported(int C) { return C >= 1 && C <= 256; }

// k per split: HW / 8 rounded up to whole 32-deep stages (512^2: 32768), so every shape
// fills 8 x 2n workgroups (C = 128 at 256^2 ran 2 splits, C = 256 at 128^2 one); a function
// of HW only, so an image's bits never depend on its batch
static int64_t cov_kper(int64_t HW) {
  const int64_t k = (HW + kCovSplits - 1) / kCovSplits;
  return (k + kCovBK - 1) / kCovBK * kCovBK;
}
static int cov_ksplit(int64_t HW) { return (int)((HW + cov_kper(HW) - 1) / cov_kper(HW)); }

size_t cov_v2_work_doubles(int n, int C, int64_t HW) {
  const int NB = cov_nb(C), nblk = NB * (NB + 1) / 2, ks = cov_ksplit(HW);
  return (size_t)2 * n * ks * cov_kg(NB) * nblk * 256 + (size_t)2 * n * ks * C;
}

int cov_v2(const float* cF, const float* sF, const float* mu32, int n, int C, int64_t HW,
           double* Cc, double* Cs, double* mu64, double* work, hipStream_t st) {
  if (!cov_v2_supported(C) || HW < 2 || 2 * n > 65535) {
    set_error("cov_v2: unsupported shape n=%d C=%d HW=%lld", n, C, (long long)HW);
    return RPST_EINVAL;
  }
  CovArgs a{};
  a.X0 = cF;
  a.X1 = sF;
  a.mu32 = mu32;
  a.n = n;
  a.C = C;
  a.HW = HW;
  a.ksplit = cov_ksplit(HW);
  a.kper = (int)cov_kper(HW);
  const int NB = cov_nb(C), nblk = NB * (NB + 1) / 2, PS = a.ksplit * cov_kg(NB);
  a.part = work;
  a.rsum = work + (size_t)2 * n * PS * nblk * 256;
  const bool vec = HW % 4 == 0 && (reinterpret_cast<uintptr_t>(cF) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(sF) & 15) == 0;
  const dim3 grid(a.ksplit, 2 * n);
#define RPST_COV_LAUNCH(NBv)                                                   \
  (vec ? (cov_syrk_kernel<NBv, true><<<grid, 512, 0, st>>>(a), 0)              \
       : (cov_syrk_kernel<NBv, false><<<grid, 512, 0, st>>>(a), 0))
  // RPST_COV_COMPACT=0: the strided 8-wave form for C > 128 too (A/B)
  const char* ce = getenv("RPST_COV_COMPACT");
  const bool compact = !(ce && *ce == '0');
  if (NB == 4) RPST_COV_LAUNCH(4);
  else if (NB == 8) RPST_COV_LAUNCH(8);
  else if (compact) {
    if (vec) cov_syrk16_kernel<true><<<grid, 1024, 0, st>>>(a);
    else cov_syrk16_kernel<false><<<grid, 1024, 0, st>>>(a);
  } else RPST_COV_LAUNCH(16);
#undef RPST_COV_LAUNCH
  if (int e = launch_status("cov_syrk_kernel")) return e;
  const int64_t tot = (int64_t)2 * n * C * C;
  cov_finish_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(a.part, a.rsum, mu32, Cc, Cs,
                                                                  mu64, n, C, NB, PS, a.ksplit, HW);
  return launch_status("cov_finish_kernel");
}

// ======================= 2. persistent matrix functions ===================================

constexpr int kMT = 64;              // output tile of a workgroup
constexpr int kMK = 32;              // staged k depth
constexpr int kMLD = kMT + 16;
constexpr int kNSMax = 64;           // Newton-Schulz iteration cap
constexpr double kNSAbsTol = 1e-10;  // on ||I - Z Y||_F
constexpr int kRedSlots = 4;
enum { MF_WCT = 0, MF_POWER = 1 };
enum { FL_NOCONV = 1, FL_EXACT = 2, FL_TIMEOUT = 4 };

struct MfArgs {
  int mode, n, batch, tpd, P, G;
  // MF_WCT
  const double* Cc;
  const double* Cs;
  const double* mu;  // (2 batch, n): mu_c rows then mu_s rows
  double* T;
  double* offset;
  // MF_POWER
  const double* A;
  double* out;
  int inverse;
  double* residual;  // MF_WCT: 2 batch; MF_POWER: batch (may be null)
  int* flags;        // per matrix
  double* scratch;   // per group: kMfBufs n x n
  double* red;       // per group: [2][kRedSlots][P]
  unsigned* bar;     // per group barrier counter, zero at launch
  // debug knob (RPST_MATFUN_DEBUG_SKIP=1, tests only): workgroup P - 1 of group 0 never arrives
  // at its barriers, as if it were not resident; the spin bound shrinks so the test is quick
  int dbg_skip;
};
constexpr int kMfBufs = 11;

struct MfCtx {
  int n, P, p, ti, tj;
  bool skip;         // dbg_skip: this workgroup does not arrive at barriers
  unsigned spin_cap;
  unsigned* bar;
  unsigned* abort;  // launch-wide: set by a timed-out barrier, every later barrier passes
  unsigned phase;
  double* red;
  int* flag;
  double* As;
  double* Bs;
  double* bc;  // LDS broadcast slots
};

// group barrier: every wave's stores drained, workgroup barrier, lane 0 releases (agent) and
// arrives on the monotonic counter, polls until all P workgroups of the group have arrived,
// acquires (agent); bounded spin (a timeout flags the matrix and lets the launch drain)
__device__ __forceinline__ void mf_sync(MfCtx& c) {
  ++c.phase;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (c.P > 1) {
      if (!c.skip) __hip_atomic_fetch_add(c.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = c.phase * (unsigned)c.P;
      unsigned spins = 0;
      while (__hip_atomic_load(c.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        // ~0.25 s: far beyond any phase (a matrix function takes ~1 ms); on a timeout the
        // matrix is flagged and every later barrier of the launch gives up after 1024 spins,
        // flagging the matrix it belongs to, so the launch drains. Every flagged matrix is
        // overwritten with NaN after the launch (mf_poison_kernel): a barrier that did not
        // synchronise never yields a finite result
        if ((++spins & 1023u) == 0 &&
            (spins > c.spin_cap ||
             __hip_atomic_load(c.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
          __hip_atomic_fetch_or(c.flag, FL_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(c.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// block sum of v into thread 0's return (fixed order)
__device__ __forceinline__ double block_sum(double v, double* bc) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) bc[threadIdx.x >> 6] = v;
  __syncthreads();
  return (bc[0] + bc[1]) + (bc[2] + bc[3]);
}

// publish this workgroup's partials (slot s of the current parity) before a barrier ...
__device__ __forceinline__ void mf_put(MfCtx& c, int s, double v) {
  if (threadIdx.x == 0) c.red[((int)((c.phase + 1) & 1) * kRedSlots + s) * c.P + c.p] = v;
}
// ... and after it every workgroup sums the P partials in the same order
__device__ __forceinline__ double mf_get(const MfCtx& c, int s) {
  const double* r = c.red + ((int)(c.phase & 1) * kRedSlots + s) * c.P;
  double t = 0.0;
  for (int q = 0; q < c.P; ++q) t += r[q];
  return t;
}

// D = alpha A B + beta I on this workgroup's tile (n x n row-major fp64); returns
// sum (D - I)^2 (dev) and sum D^2 (sq) over the tile, block-reduced.
__device__ __forceinline__ void tile_gemm(MfCtx& c, const double* A, const double* B, double* D, double alpha,
                          double beta, double* dev_out, double* sq_out) {
  const int n = c.n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, lr = lane & 15, lk = lane >> 4;
  const int m0 = c.ti * kMT, n0 = c.tj * kMT;
  doublex4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
  const int am = m0 + (tid >> 2), ak = (tid & 3) * 8;
  const int bk = tid >> 3, bn = n0 + (tid & 7) * 8;
  // software pipeline: the k-step kt + 1 operands are loaded into registers while kt's
  // MFMAs run from the other LDS buffer (one barrier per k-step; the matrices are L2-resident,
  // so the loads cost latency, not bandwidth)
  double ra[8], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + ak + e;
      ra[e] = (am < n && k < n) ? A[(int64_t)am * n + k] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + bk;
      rb[e] = (k < n && bn + e < n) ? B[(int64_t)k * n + bn + e] : 0.0;
    }
  };
  const int nk = (n + kMK - 1) / kMK;
  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    double* As = c.As + (kt & 1) * kMK * kMLD;
    double* Bs = c.Bs + (kt & 1) * kMK * kMLD;
#pragma unroll
    for (int e = 0; e < 8; ++e) As[(ak + e) * kMLD + (tid >> 2)] = ra[e];
#pragma unroll
    for (int e = 0; e < 8; ++e) Bs[bk * kMLD + (tid & 7) * 8 + e] = rb[e];
    __syncthreads();  // buffer kt & 1 complete; every wave is done with buffer (kt - 1) & 1
    if (kt + 1 < nk) load((kt + 1) * kMK);
#pragma unroll
    for (int ks = 0; ks < kMK / 4; ++ks) {
      double av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[(4 * ks + lk) * kMLD + wm * 32 + i * 16 + lr];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[(4 * ks + lk) * kMLD + wn * 32 + j * 16 + lr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // the next GEMM's first store overwrites buffer 0
  double dev = 0.0, sq = 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * 32 + i * 16 + lk + 4 * r;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = n0 + wn * 32 + j * 16 + lr;
        if (m < n && col < n) {
          const double id = m == col ? 1.0 : 0.0;
          const double v = alpha * acc[i][j][r] + beta * id;
          D[(int64_t)m * n + col] = v;
          dev = fma(v - id, v - id, dev);
          sq = fma(v, v, sq);
        }
      }
    }
  if (dev_out) *dev_out = block_sum(dev, c.bc);
  if (sq_out) *sq_out = block_sum(sq, c.bc);
}

// elementwise over this workgroup's tile: f(m, col, index)
template <typename F>
__device__ __forceinline__ void tile_each(const MfCtx& c, F f) {
  const int n = c.n, m0 = c.ti * kMT, n0 = c.tj * kMT;
  for (int e = threadIdx.x; e < kMT * kMT; e += blockDim.x) {
    const int m = m0 + e / kMT, col = n0 + e % kMT;
    if (m < n && col < n) f(m, col, (int64_t)m * n + col);
  }
}

struct NsBufs {
  double *Y, *Z, *Yn, *Zn, *T;
};

struct NsOut {
  const double* Y;  // (X/s)^(1/2)
  const double* Z;  // (X/s)^(-1/2)
  double s, r, nz;
  bool conv;
};

// Coupled Newton-Schulz on (X + add I) / s, s = ||X + add I||_F, with the buffers bufs[0..4]
// (Y, Z, Y', Z', T); see the file comment for the stopping rule.
__device__ __forceinline__ NsOut ns_run(MfCtx& c, const double* X, double add, NsBufs bufs) {
  double *Y = bufs.Y, *Z = bufs.Z, *Yn = bufs.Yn, *Zn = bufs.Zn, *Tn = bufs.T;
  // ||X + add I||_F
  double ssq = 0.0;
  tile_each(c, [&](int m, int col, int64_t i) {
    const double v = X[i] + (m == col ? add : 0.0);
    ssq = fma(v, v, ssq);
  });
  ssq = block_sum(ssq, c.bc);
  mf_put(c, 0, ssq);
  mf_sync(c);
  const double s = sqrt(mf_get(c, 0));
  const double inv = 1.0 / s;
  tile_each(c, [&](int m, int col, int64_t i) {
    Y[i] = (X[i] + (m == col ? add : 0.0)) * inv;
    Z[i] = m == col ? 1.0 : 0.0;
  });
  mf_sync(c);
  const double n = (double)c.n;
  double ny = 1.0, nz = n;  // ||Y_0||_F^2 = 1, ||Z_0||_F^2 = n
  double r = __builtin_inf(), rprev = __builtin_inf();
  bool conv = false;
  for (int it = 0; it < kNSMax && !conv; ++it) {
    double dev;
    tile_gemm(c, Z, Y, Tn, -0.5, 1.5, &dev, nullptr);  // T = (3 I - Z Y) / 2
    mf_put(c, 0, dev);
    mf_sync(c);
    r = 2.0 * sqrt(mf_get(c, 0));
    const double floor_ = 8.0 * 2.220446049250313e-16 * n * sqrt(ny * nz);
    conv = r < fmax(kNSAbsTol, floor_) || (rprev < 1e-6 && r > 0.9 * rprev);
    double sy, sz;
    tile_gemm(c, Y, Tn, Yn, 1.0, 0.0, nullptr, &sy);  // Y <- Y T, Z <- T Z
    tile_gemm(c, Tn, Z, Zn, 1.0, 0.0, nullptr, &sz);
    mf_put(c, 1, sy);
    mf_put(c, 2, sz);
    mf_sync(c);
    ny = mf_get(c, 1);
    nz = mf_get(c, 2);
    double* t = Y;
    Y = Yn;
    Yn = t;
    t = Z;
    Z = Zn;
    Zn = t;
    rprev = r;
  }
  return NsOut{Y, Z, s, r, nz, conv};
}

__global__ __launch_bounds__(256) void matfun_kernel(MfArgs a) {
  __shared__ double As[2 * kMK * kMLD];
  __shared__ double Bs[2 * kMK * kMLD];
  __shared__ double bc[8];
  // bijective XCD remap (cdna_hip_programming.md 'XCD swizzle must be bijective'): the P
  // workgroups of a group get consecutive ids on one XCD where possible (speed only)
  const int nwg = (int)gridDim.x, orig = (int)blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, x = orig % 8;
  const int wg = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + orig / 8;
  const int g = wg / a.P, p = wg % a.P;
  if (g >= a.G) return;
  MfCtx c{};
  c.n = a.n;
  c.P = a.P;
  c.p = p;
  c.ti = p / a.tpd;
  c.tj = p % a.tpd;
  c.skip = a.dbg_skip && g == 0 && p == a.P - 1;
  c.spin_cap = a.dbg_skip ? (1u << 14) : (1u << 22);
  c.bar = a.bar + g;
  c.abort = a.bar + a.G;
  c.phase = 0;
  c.red = a.red + (size_t)g * 2 * kRedSlots * a.P;
  c.As = As;
  c.Bs = Bs;
  c.bc = bc;
  const int64_t nn = (int64_t)a.n * a.n;
  double* S = a.scratch + (size_t)g * kMfBufs * nn;
  const NsBufs set1{S, S + nn, S + 2 * nn, S + 3 * nn, S + 4 * nn};
  const NsBufs set2{S + 5 * nn, S + 6 * nn, S + 7 * nn, S + 8 * nn, S + 4 * nn};
  double* tmp = S + 9 * nn;
  double* M0 = S + 10 * nn;

  for (int b = g; b < a.batch; b += a.G) {
    c.flag = a.flags + b;
    if (a.mode == MF_POWER) {
      const double* A = a.A + (int64_t)b * nn;
      // symmetry of A: sum (A - A^T)^2 against sum A^2
      double asq = 0.0, nsq = 0.0;
      tile_each(c, [&](int m, int col, int64_t i) {
        const double v = A[i], d = v - A[(int64_t)col * a.n + m];
        asq = fma(d, d, asq);
        nsq = fma(v, v, nsq);
      });
      asq = block_sum(asq, bc);
      nsq = block_sum(nsq, bc);
      mf_put(c, 1, asq);
      mf_put(c, 2, nsq);
      mf_sync(c);
      const double sym_dev = mf_get(c, 1), sym_ref = mf_get(c, 2);
      const NsOut o = ns_run(c, A, 1e-4, set1);
      const double scale = a.inverse ? 1.0 / sqrt(o.s) : sqrt(o.s);
      const double* src = a.inverse ? o.Z : o.Y;
      double* out = a.out + (int64_t)b * nn;
      tile_each(c, [&](int, int, int64_t i) { out[i] = src[i] * scale; });
      if (threadIdx.x == 0 && p == 0) {
        const double lmin_bound = o.s / o.nz;  // lambda_min(A + 1e-4 I) >= s / ||Z||_F^2
        int fl = o.conv ? 0 : FL_NOCONV;
        if (!o.conv || !(lmin_bound >= 1e-5) || !(sym_dev <= 1e-24 * sym_ref)) fl |= FL_EXACT;
        __hip_atomic_fetch_or(c.flag, fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.residual) a.residual[b] = o.r;
      }
      mf_sync(c);  // the next matrix reuses the group's buffers
    } else {
      const double* Cc = a.Cc + (int64_t)b * nn;
      const double* Cs = a.Cs + (int64_t)b * nn;
      const NsOut o1 = ns_run(c, Cc, 1e-4, set1);  // Sc = sqrt(s1) Y1, Ic = Z1 / sqrt(s1)
      tile_gemm(c, o1.Y, Cs, tmp, 1.0, 0.0, nullptr, nullptr);
      mf_sync(c);
      tile_gemm(c, tmp, o1.Y, M0, o1.s, 0.0, nullptr, nullptr);  // Sc Cs Sc
      mf_sync(c);
      const NsOut o2 = ns_run(c, M0, 1e-4, set2);  // Mid = sqrt(s2) Y2
      tile_gemm(c, o1.Z, o2.Y, tmp, 1.0, 0.0, nullptr, nullptr);
      mf_sync(c);
      double* T = a.T + (int64_t)b * nn;
      const bool ok = o1.conv && o2.conv;
      tile_gemm(c, tmp, o1.Z, T, ok ? sqrt(o2.s) / o1.s : __builtin_nan(""), 0.0, nullptr,
                nullptr);  // Ic Mid Ic
      mf_sync(c);
      // offset rows [p n / P, (p + 1) n / P): mu_s - T mu_c (fixed-order fma over k)
      const double* muc = a.mu + (int64_t)b * a.n;
      const double* mus = a.mu + ((int64_t)a.batch + b) * a.n;
      const int r0 = (int)((int64_t)p * a.n / a.P), r1 = (int)((int64_t)(p + 1) * a.n / a.P);
      for (int m = r0 + (int)threadIdx.x; m < r1; m += blockDim.x) {
        const double* t = T + (int64_t)m * a.n;
        double s = 0.0;
        for (int k = 0; k < a.n; ++k) s = fma(t[k], muc[k], s);
        a.offset[(int64_t)b * a.n + m] = ok ? mus[m] - s : __builtin_nan("");
      }
      if (threadIdx.x == 0 && p == 0) {
        if (a.residual) {
          a.residual[b] = o1.r;
          a.residual[a.batch + b] = o2.r;
        }
        if (!ok) __hip_atomic_fetch_or(c.flag, FL_NOCONV, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      mf_sync(c);  // the next matrix reuses the group's buffers
    }
  }
}

// ======================= 3. reference SVD form by one-sided Jacobi ========================
// M = A + 1e-4 I; rotations of column pairs (p, q) (round-robin ordering, n/2 disjoint pairs
// per step) until no pair has |m_p . m_q| > 1e-15 ||m_p|| ||m_q||: M V = U S, so the columns of
// V are torch.svd's right singular vectors and s_p = ||m_p||; out = sum over s_p >= 1e-5 of
// s_p^(+-1/2) v_p v_p^T (wct_rp.py:13-21, 30-39: the truncation keeps exactly those).
constexpr int kJacobiMaxN = 1024;
__global__ __launch_bounds__(1024) void jacobi_power_kernel(const double* __restrict__ A,
                                                            double* __restrict__ out,
                                                            const int* __restrict__ flags, int n,
                                                            int inverse, double* __restrict__ work) {
  const int b = blockIdx.x;
  if (!(flags[b] & (FL_EXACT | FL_NOCONV | FL_TIMEOUT))) return;  // Newton-Schulz result stands
  const int tid = threadIdx.x;
  const int64_t nn = (int64_t)n * n;
  const int np = n + (n & 1);  // a zero column pads an odd n
  double* Mc = work + (int64_t)b * 2 * np * np;  // Mc[p * np + i] = M[i][p]
  double* Vc = Mc + (int64_t)np * np;
  const double* Ab = A + (int64_t)b * nn;
  for (int64_t e = tid; e < (int64_t)np * np; e += 1024) {
    const int p = (int)(e / np), i = (int)(e % np);
    Mc[e] = (p < n && i < n) ? Ab[(int64_t)i * n + p] + (i == p ? 1e-4 : 0.0) : 0.0;
    Vc[e] = p == i ? 1.0 : 0.0;
  }
  __syncthreads();
  const int npairs = np / 2;
  int tpp = 64;
  while (tpp > 1 && tpp * npairs > 1024) tpp >>= 1;
  const int per_pass = 1024 / tpp, sub = tid % tpp;
  __shared__ int rotated;
  for (int sweep = 0; sweep < 40; ++sweep) {
    if (tid == 0) rotated = 0;
    __syncthreads();
    for (int step = 0; step < np - 1; ++step) {
      for (int k = tid / tpp; k < npairs; k += per_pass) {
        const int p = k == 0 ? step % (np - 1) : (step + k) % (np - 1);
        const int q = k == 0 ? np - 1 : (step - k + np - 1) % (np - 1);
        double* mp = Mc + (int64_t)p * np;
        double* mq = Mc + (int64_t)q * np;
        double al = 0.0, be = 0.0, ga = 0.0;
        for (int i = sub; i < np; i += tpp) {
          const double x = mp[i], y = mq[i];
          al = fma(x, x, al);
          be = fma(y, y, be);
          ga = fma(x, y, ga);
        }
        for (int o = tpp >> 1; o > 0; o >>= 1) {
          al += __shfl_xor(al, o, 64);
          be += __shfl_xor(be, o, 64);
          ga += __shfl_xor(ga, o, 64);
        }
        if (ga != 0.0 && fabs(ga) > 1e-15 * sqrt(al * be)) {
          const double zeta = (be - al) / (2.0 * ga);
          const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
          double* vp = Vc + (int64_t)p * np;
          double* vq = Vc + (int64_t)q * np;
          for (int i = sub; i < np; i += tpp) {
            const double x = mp[i], y = mq[i];
            mp[i] = cs * x - sn * y;
            mq[i] = sn * x + cs * y;
            const double u = vp[i], w = vq[i];
            vp[i] = cs * u - sn * w;
            vq[i] = sn * u + cs * w;
          }
          if (sub == 0) rotated = 1;
        }
      }
      __syncthreads();
    }
    if (!rotated) break;
    __syncthreads();
  }
  __shared__ double wgt[kJacobiMaxN];
  for (int p = tid; p < np; p += 1024) {
    double s2 = 0.0;
    for (int i = 0; i < np; ++i) s2 = fma(Mc[(int64_t)p * np + i], Mc[(int64_t)p * np + i], s2);
    const double s = sqrt(s2);
    wgt[p] = (p < n && s >= 1e-5) ? (inverse ? 1.0 / sqrt(s) : sqrt(s)) : 0.0;
  }
  __syncthreads();
  for (int64_t e = tid; e < nn; e += 1024) {
    const int i = (int)(e / n), j = (int)(e % n);
    double acc = 0.0;
    for (int p = 0; p < np; ++p)
      acc = fma(wgt[p] * Vc[(int64_t)p * np + i], Vc[(int64_t)p * np + j], acc);
    out[(int64_t)b * nn + e] = acc;
  }
}

// MF_WCT: T and offset of every matrix whose barriers timed out (FL_TIMEOUT: some barrier of
// its group did not synchronise, so its partials may be stale) become NaN. One block per
// flagged-or-not matrix; unflagged ones exit at once.
__global__ __launch_bounds__(256) void mf_poison_kernel(const int* __restrict__ flags,
                                                        double* __restrict__ T,
                                                        double* __restrict__ offset, int n) {
  const int b = blockIdx.x;
  if (!(flags[b] & FL_TIMEOUT)) return;
  const double nan = __builtin_nan("");
  const int64_t nn = (int64_t)n * n;
  for (int64_t e = threadIdx.x; e < nn; e += 256) T[(int64_t)b * nn + e] = nan;
  for (int e = threadIdx.x; e < n; e += 256) offset[(int64_t)b * n + e] = nan;
}

// ======================= host side =======================================================

// workgroups of matfun_kernel the device holds at once (occupancy x CUs; 256 when unknown,
// e.g. no device in a CPU-only process sizing a workspace)
static int mf_resident_cap() {
  static const int cap = [] {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, matfun_kernel, 256, 0) != hipSuccess ||
        cus <= 0 || per <= 0) {
      (void)hipGetLastError();
      return 256;
    }
    return cus * per;
  }();
  return cap;
}

// layout geometry (the workspace is sized for G = 256 / P groups, whatever the device)
static void mf_geometry(int n, int batch, int& tpd, int& P, int& G) {
  tpd = (n + kMT - 1) / kMT;
  P = tpd * tpd;
  G = 256 / P;
  if (G < 1) G = 1;
  if (G > batch) G = batch;
}

static size_t mf_work_doubles(int n, int batch) {
  int tpd, P, G;
  mf_geometry(n, batch, tpd, P, G);
  // scratch, reduction slots, barrier counters + abort word, flags (ints, rounded up)
  return (size_t)G * kMfBufs * n * n + (size_t)G * 2 * kRedSlots * P + (size_t)(G + 1 + 1) / 2 +
         (size_t)(batch + 1) / 2 + 2;
}

// per-matrix flags of the last launch on this workspace (layout of mf_launch)
static int* mf_flags(double* work, int n, int batch) {
  int tpd, P, G;
  mf_geometry(n, batch, tpd, P, G);
  return reinterpret_cast<int*>(
      reinterpret_cast<unsigned*>(work + (size_t)G * kMfBufs * n * n + (size_t)G * 2 * kRedSlots * P) +
      G + 1);
}

static int mf_launch(MfArgs a, double* work, hipStream_t st) {
  int Gl;
  mf_geometry(a.n, a.batch, a.tpd, a.P, Gl);
  a.scratch = work;
  a.red = a.scratch + (size_t)Gl * kMfBufs * a.n * a.n;
  a.bar = reinterpret_cast<unsigned*>(a.red + (size_t)Gl * 2 * kRedSlots * a.P);
  a.flags = reinterpret_cast<int*>(a.bar + Gl + 1);
  // groups that the device can hold at once: the group barriers need every workgroup of a
  // group resident (a smaller device, or a grid the occupancy does not cover, gets fewer
  // groups looping over more matrices)
  const int cap = mf_resident_cap();
  if (cap < a.P) {
    set_error("matfun: %d workgroups per matrix but only %d resident on this device", a.P, cap);
    return RPST_EINVAL;
  }
  a.G = Gl < cap / a.P ? Gl : cap / a.P;
  {
    const char* e = getenv("RPST_MATFUN_DEBUG_SKIP");
    a.dbg_skip = (e && *e && atoi(e) != 0 && a.P > 1) ? 1 : 0;
  }
  // barrier counters (the layout's Gl of them) + abort word + flags
  if (hipMemsetAsync(a.bar, 0, sizeof(unsigned) * (Gl + 1) + sizeof(int) * a.batch, st) !=
      hipSuccess) {
    set_error("matfun: workspace reset failed");
    return RPST_EHIP;
  }
  matfun_kernel<<<a.G * a.P, 256, 0, st>>>(a);
  if (int e = launch_status("matfun_kernel")) return e;
  if (a.mode == MF_WCT) {
    mf_poison_kernel<<<a.batch, 256, 0, st>>>(a.flags, a.T, a.offset, a.n);
    return launch_status("mf_poison_kernel");
  }
  return RPST_OK;
}

int matfun_wct_status(double* work, int n, int C, int* status, hipStream_t st) {
  if (hipMemcpyAsync(status, mf_flags(work, C, n), sizeof(int) * (size_t)n,
                     hipMemcpyDeviceToDevice, st) != hipSuccess) {
    set_error("wct_status: copy failed");
    return RPST_EHIP;
  }
  return RPST_OK;
}

size_t matfun_wct_work_doubles(int n, int C) { return mf_work_doubles(C, n); }

int matfun_wct_clear_status(double* work, int n, int C, hipStream_t st) {
  if (hipMemsetAsync(mf_flags(work, C, n), 0, sizeof(int) * (size_t)n, st) != hipSuccess) {
    set_error("wct: status reset failed");
    return RPST_EHIP;
  }
  return RPST_OK;
}

int matfun_wct(const double* Cc, const double* Cs, const double* mu64, double* T, double* offset,
               double* residual, int n, int C, double* work, hipStream_t st) {
  if (C > kJacobiMaxN || n < 1) {
    set_error("matfun_wct: unsupported shape n=%d C=%d", n, C);
    return RPST_EINVAL;
  }
  MfArgs a{};
  a.mode = MF_WCT;
  a.n = C;
  a.batch = n;
  a.Cc = Cc;
  a.Cs = Cs;
  a.mu = mu64;
  a.T = T;
  a.offset = offset;
  a.residual = residual;
  return mf_launch(a, work, st);
}

size_t matfun_power_work_doubles(int n, int batch) {
  const size_t np = (size_t)(n + (n & 1));
  return mf_work_doubles(n, batch) + (size_t)batch * 2 * np * np;
}

int matfun_power(const double* A, double* out, int n, int batch, int inverse, double* residual,
                 double* work, hipStream_t st) {
  if (n > kJacobiMaxN || n < 1 || batch < 1) {
    set_error("matrix_power: unsupported shape n=%d batch=%d", n, batch);
    return RPST_EINVAL;
  }
  MfArgs a{};
  a.mode = MF_POWER;
  a.n = n;
  a.batch = batch;
  a.A = A;
  a.out = out;
  a.inverse = inverse;
  a.residual = residual;
  if (int e = mf_launch(a, work, st)) return e;
  double* jw = work + mf_work_doubles(n, batch);
  const int* flags = mf_flags(work, n, batch);
  jacobi_power_kernel<<<batch, 1024, 0, st>>>(A, out, flags, n, inverse, jw);
  return launch_status("jacobi_power_kernel");
}

}  // namespace rpst
