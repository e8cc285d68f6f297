// SAModel training (network/sanet.py:248-275 + total_loss.backward(), train.py:186-189):
// the backward pieces the AdaIN-RP step (rpst_train.hip) does not have.
//   1-pixel pad        pad1_kernel: ReflectionPad2d(1) or zero pad, as a materialised
//                        tensor (a reflect-padded conv's weight gradient is then the zero-pad
//                        wgrad of the padded input against the zero-extended output grad)
//   upsample backward  upsample2x_backward_kernel: nearest x2 (sanet.py:145,166,179,186)
//   mean_variance_norm backward (sanet.py:20-24): dx = (dy - mean(dy) - y sum(dy y)/(n-1))/s
//                        with y = (x - mean)/s, s = sqrt(var_unbiased + eps); one block per
//                        plane, fp64 sums in a fixed order (optionally added into dx)
//   row softmax        softmax_rows_kernel / softmax_rows_backward_kernel: P = softmax(S)
//                        over a row (sanet.py:92-93) and dS = P (dP - sum(dP P)), one block
//                        per row
// All reductions are fixed-order (no atomics): results are deterministic.
#include "rpst_common.h"

namespace rpst {

__global__ __launch_bounds__(256) void pad1_kernel(const float* __restrict__ x,
                                                   float* __restrict__ out, int64_t planes,
                                                   int H, int W, int reflect) {
  const int Ho = H + 2, Wo = W + 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= planes * Ho * Wo) return;
  const int ox = (int)(i % Wo);
  const int64_t r = i / Wo;
  const int oy = (int)(r % Ho);
  const int64_t p = r / Ho;
  int y = oy - 1, xx = ox - 1;
  float v;
  if (reflect) {
    v = x[(p * H + reflect1(y, H)) * W + reflect1(xx, W)];
  } else {
    v = (y >= 0 && y < H && xx >= 0 && xx < W) ? x[(p * H + y) * W + xx] : 0.f;
  }
  out[i] = v;
}

// dx[p][y][x] = sum of g[p][2y + a][2x + b], a, b in {0, 1} (g is 2H x 2W)
__global__ __launch_bounds__(256) void upsample2x_backward_kernel(const float* __restrict__ g,
                                                                  float* __restrict__ dx,
                                                                  int64_t planes, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= planes * H * W) return;
  const int x = (int)(i % W);
  const int64_t r = i / W;
  const int y = (int)(r % H);
  const int64_t p = r / H;
  const int W2 = 2 * W;
  const float* s = g + (p * 2 * H + 2 * y) * W2 + 2 * x;
  dx[i] = (s[0] + s[1]) + (s[W2] + s[W2 + 1]);
}

// fixed-order block sums of two fp64 values (256 threads = 4 waves)
__device__ __forceinline__ void block_sum2(double& a, double& b, double* sh) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sh[wave] = a;
    sh[4 + wave] = b;
  }
  __syncthreads();
  a = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  b = (sh[4] + sh[5]) + (sh[6] + sh[7]);
  __syncthreads();
}

__global__ __launch_bounds__(256) void mvn_backward_kernel(const float* __restrict__ y,
                                                           const float* __restrict__ dy,
                                                           const float* __restrict__ sd,
                                                           float* __restrict__ dx, int64_t HW,
                                                           int accumulate) {
  __shared__ double sh[8];
  const int64_t p = blockIdx.x;
  const float* yp = y + p * HW;
  const float* gp = dy + p * HW;
  double s_g = 0.0, s_gy = 0.0;
  for (int64_t i = threadIdx.x; i < HW; i += 256) {
    const double g = gp[i];
    s_g += g;
    s_gy += g * (double)yp[i];
  }
  block_sum2(s_g, s_gy, sh);
  const double mg = s_g / (double)HW;
  const double k = HW > 1 ? s_gy / (double)(HW - 1) : 0.0;
  const double inv = 1.0 / (double)sd[p];
  float* dp = dx + p * HW;
  for (int64_t i = threadIdx.x; i < HW; i += 256) {
    const float v = (float)(((double)gp[i] - mg - (double)yp[i] * k) * inv);
    dp[i] = accumulate ? dp[i] + v : v;
  }
}

__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ S,
                                                           float* __restrict__ P, int cols) {
  __shared__ float shm[4];
  __shared__ double shs[8];
  const int64_t row = blockIdx.x;
  const float* s = S + row * cols;
  float m = -__builtin_inff();
  for (int i = threadIdx.x; i < cols; i += 256) m = fmaxf(m, s[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) shm[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(shm[0], shm[1]), fmaxf(shm[2], shm[3]));
  double z = 0.0, unused = 0.0;
  for (int i = threadIdx.x; i < cols; i += 256) z += (double)__expf(s[i] - m);
  block_sum2(z, unused, shs);
  const float inv = (float)(1.0 / z);
  float* p = P + row * cols;
  for (int i = threadIdx.x; i < cols; i += 256) p[i] = __expf(s[i] - m) * inv;
}

// dS may alias dP (each element is read before its own write)
__global__ __launch_bounds__(256) void softmax_rows_backward_kernel(const float* __restrict__ P,
                                                                    const float* dP, float* dS,
                                                                    int cols) {
  __shared__ double sh[8];
  const int64_t row = blockIdx.x;
  const float* p = P + row * cols;
  const float* g = dP + row * cols;
  double s = 0.0, unused = 0.0;
  for (int i = threadIdx.x; i < cols; i += 256) s += (double)g[i] * (double)p[i];
  block_sum2(s, unused, sh);
  const float sf = (float)s;
  float* d = dS + row * cols;
  for (int i = threadIdx.x; i < cols; i += 256) d[i] = p[i] * (g[i] - sf);
}

static unsigned grid256(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace rpst

using namespace rpst;

extern "C" int rpst_pad1(const float* x, float* out, int64_t planes, int H, int W, int reflect,
                         rpst_stream_t stream) {
  RPST_REQUIRE(x && out && planes >= 0 && H >= 1 && W >= 1, "pad1: bad arguments");
  RPST_REQUIRE(!reflect || (H >= 2 && W >= 2), "pad1: reflect padding needs H, W >= 2");
  const int64_t n = planes * (H + 2) * (W + 2);
  if (n == 0) return RPST_OK;
  RPST_REQUIRE(grid256(n) <= 0x7fffffffu, "pad1: tensor too large");
  pad1_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(x, out, planes, H, W, reflect);
  return launch_status("pad1_kernel");
}

extern "C" int rpst_upsample_nearest2x_backward(const float* g, float* dx, int64_t planes, int H,
                                                int W, rpst_stream_t stream) {
  RPST_REQUIRE(g && dx && planes >= 0 && H >= 1 && W >= 1, "upsample backward: bad arguments");
  const int64_t n = planes * H * W;
  if (n == 0) return RPST_OK;
  RPST_REQUIRE(grid256(n) <= 0x7fffffffu, "upsample backward: tensor too large");
  upsample2x_backward_kernel<<<grid256(n), 256, 0, as_stream(stream)>>>(g, dx, planes, H, W);
  return launch_status("upsample2x_backward_kernel");
}

extern "C" int rpst_mean_variance_norm_backward(const float* y, const float* dy, const float* std,
                                                float* dx, int64_t planes, int64_t HW,
                                                int accumulate, rpst_stream_t stream) {
  RPST_REQUIRE(y && dy && std && dx && planes >= 0 && HW >= 1,
               "mean_variance_norm backward: bad arguments");
  RPST_REQUIRE(planes <= 0x7fffffffLL, "mean_variance_norm backward: too many planes");
  if (planes == 0) return RPST_OK;
  mvn_backward_kernel<<<(unsigned)planes, 256, 0, as_stream(stream)>>>(y, dy, std, dx, HW,
                                                                      accumulate);
  return launch_status("mvn_backward_kernel");
}

extern "C" int rpst_softmax_rows(const float* S, float* P, int64_t rows, int cols,
                                 rpst_stream_t stream) {
  RPST_REQUIRE(S && P && rows >= 0 && cols >= 1, "softmax_rows: bad arguments");
  RPST_REQUIRE(rows <= 0x7fffffffLL, "softmax_rows: too many rows");
  if (rows == 0) return RPST_OK;
  softmax_rows_kernel<<<(unsigned)rows, 256, 0, as_stream(stream)>>>(S, P, cols);
  return launch_status("softmax_rows_kernel");
}

extern "C" int rpst_softmax_rows_backward(const float* P, const float* dP, float* dS, int64_t rows,
                                          int cols, rpst_stream_t stream) {
  RPST_REQUIRE(P && dP && dS && rows >= 0 && cols >= 1, "softmax_rows backward: bad arguments");
  RPST_REQUIRE(rows <= 0x7fffffffLL, "softmax_rows backward: too many rows");
  if (rows == 0) return RPST_OK;
  softmax_rows_backward_kernel<<<(unsigned)rows, 256, 0, as_stream(stream)>>>(P, dP, dS, cols);
  return launch_status("softmax_rows_backward_kernel");
}
