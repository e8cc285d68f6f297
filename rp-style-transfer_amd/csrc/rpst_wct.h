// Internal interface between rpst_wct.hip (the WCT entry points) and rpst_wct_mat.hip
// (covariance SYRK for fp32 features, the persistent matrix-function launch and the
// one-sided Jacobi fallback). Not part of the C ABI.
#pragma once

#include "rpst_common.h"

namespace rpst {

// ---- covariance of fp32 features, C <= 256 (cov_syrk_kernel + cov_finish_kernel) ----------
// For z < n: Cc_z = (cF_z - mu)(cF_z - mu)^T / (HW - 1) + I, for z >= n: Cs = (sF - mu)(..)^T /
// (HW - 1), mu the fp64 row means (wct_rp.py:85-94). The features are centred on the fp32
// means `mu32` (2n x C, content rows then style rows) while staged; the fp64 mean follows from
// the row sums of the centred rows, delta = sum(x - mu32) / HW, and the product is corrected by
// -HW delta delta^T, so mu64 = mu32 + delta and the covariance are those of the exact fp64
// centring. Outputs Cc, Cs (n x C x C, symmetric) and mu64 (2n x C).
bool cov_v2_supported(int C);
size_t cov_v2_work_doubles(int n, int C, int64_t HW);
int cov_v2(const float* cF, const float* sF, const float* mu32, int n, int C, int64_t HW,
           double* Cc, double* Cs, double* mu64, double* work, hipStream_t st);

// ---- persistent matrix functions (one launch; groups of workgroups per matrix) -------------
// WCT: T_b = Ic Mid Ic with Sc, Ic = (Cc_b + 1e-4 I)^(+-1/2), Mid = (Sc Cs_b Sc + 1e-4 I)^(1/2)
// (wct_rp.py:104-109) and offset_b = mu_s - T_b mu_c; residual (2n, may be null): the final
// Newton-Schulz residuals of the two square roots. A matrix whose iteration did not converge
// (non-finite input), or whose group barriers timed out, gets NaN in T and offset; its flags
// word (RPST_WCT_NOCONV / RPST_WCT_TIMEOUT) is copied out by matfun_wct_status.
size_t matfun_wct_work_doubles(int n, int C);
int matfun_wct(const double* Cc, const double* Cs, const double* mu64, double* T, double* offset,
               double* residual, int n, int C, double* work, hipStream_t st);
int matfun_wct_status(double* work, int n, int C, int* status, hipStream_t st);
int matfun_wct_clear_status(double* work, int n, int C, hipStream_t st);

// Power: out = (A + 1e-4 I)^(1/2) (inverse = 0) or ^(-1/2), exactly the reference's SVD form
// V diag(s^p) V^T truncated at s < 1e-5 (wct_rp.py:7-40): Newton-Schulz for symmetric inputs
// whose smallest eigenvalue is provably >= 1e-5, a one-sided Jacobi SVD otherwise.
size_t matfun_power_work_doubles(int n, int batch);
int matfun_power(const double* A, double* out, int n, int batch, int inverse, double* residual,
                 double* work, hipStream_t st);

// out[n] = W T[n] for W (rows x K) fp32 and T (n, K, K) fp64 -> (n, rows, K) fp64 (fp64 MFMA)
int gemm_f32w_f64(const float* W, const double* T, double* out, int n, int rows, int K,
                  hipStream_t st);

}  // namespace rpst
