// Channel statistics, AdaIN and mean-variance normalisation (HBM-bound).
//
//   calc_mean_std                    network/base.py:399-407
//   adaptive_instance_normalization  network/base.py:410-418
//   mean_variance_norm               network/sanet.py:20-24
//
// Layout: NCHW fp32, one (n,c) plane = HW contiguous floats.
// Stats: one 256-thread workgroup per plane streams it with 16-B loads and keeps a
// shifted sum / sum-of-squares per lane in fp64 (shift = the plane's first element),
// then reduces wave64 -> LDS in a fixed order (deterministic). var is formed in fp64,
// rounded to fp32, then eps is added and sqrt taken in fp32 exactly as torch does
// (`var(dim=2) + eps`, `.sqrt()`), so results sit within 1 ulp of the reference.
// Apply: elementwise, 16-B loads/stores, contraction off to reproduce ATen's separate
// sub / div / mul / add roundings.
#include "rpst_common.h"

namespace rpst {

constexpr int kStatThreads = 256;

// One workgroup per plane; `planes` may span two tensors (content then style).
__global__ __launch_bounds__(kStatThreads) void plane_stats_kernel(
    const float* __restrict__ x0, const float* __restrict__ x1, int planes0,
    int64_t HW, float eps, float* __restrict__ mean0, float* __restrict__ std0,
    float* __restrict__ mean1, float* __restrict__ std1) {
  const int p = blockIdx.x;
  const bool second = p >= planes0;
  const int lp = second ? p - planes0 : p;
  const float* __restrict__ x = (second ? x1 : x0) + (int64_t)lp * HW;
  const float shift = x[0];
  double s1 = 0.0, s2 = 0.0;
  const int tid = threadIdx.x;
  if ((HW & 3) == 0) {
    const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x);
    const int64_t n4 = HW >> 2;
    int64_t i = tid;
    // 4 loads in flight per lane
    for (; i + 3 * kStatThreads < n4; i += 4 * kStatThreads) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = x4[i + u * kStatThreads];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        double a = (double)v[u].x - shift, b = (double)v[u].y - shift;
        double c = (double)v[u].z - shift, d = (double)v[u].w - shift;
        s1 += (a + b) + (c + d);
        s2 += (a * a + b * b) + (c * c + d * d);
      }
    }
    for (; i < n4; i += kStatThreads) {
      float4 v = x4[i];
      double a = (double)v.x - shift, b = (double)v.y - shift;
      double c = (double)v.z - shift, d = (double)v.w - shift;
      s1 += (a + b) + (c + d);
      s2 += (a * a + b * b) + (c * c + d * d);
    }
  } else {
    for (int64_t i = tid; i < HW; i += kStatThreads) {
      double a = (double)x[i] - shift;
      s1 += a;
      s2 += a * a;
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  __shared__ double red[2][kStatThreads / kWave];
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int k = 0; k < kStatThreads / kWave; ++k) {
      t1 += red[0][k];
      t2 += red[1][k];
    }
    const double n = (double)HW;
    const double m = t1 / n;  // mean of shifted data
    const double var = (t2 - t1 * m) / (n - 1.0);  // NaN for n == 1, like torch.var
    float varf = (float)(var < 0.0 ? 0.0 : var);
    if (HW == 1) varf = __int_as_float(0x7fc00000);
    float* mo = second ? mean1 : mean0;
    float* so = second ? std1 : std0;
    mo[lp] = (float)((double)shift + m);
    so[lp] = __fsqrt_rn(__fadd_rn(varf, eps));
  }
}

template <bool kAdain>
__global__ __launch_bounds__(256) void plane_apply_kernel(
    const float* __restrict__ x, float* __restrict__ out, const float* __restrict__ m0,
    const float* __restrict__ s0, const float* __restrict__ m1,
    const float* __restrict__ s1, int64_t HW, int chunks_per_plane) {
#pragma clang fp contract(off)
  const int plane = blockIdx.x / chunks_per_plane;
  const int chunk = blockIdx.x - plane * chunks_per_plane;
  const float mc = m0[plane], sc = s0[plane];
  float ms = 0.f, ss = 1.f;
  if (kAdain) {
    ms = m1[plane];
    ss = s1[plane];
  }
  const float* __restrict__ xp = x + (int64_t)plane * HW;
  float* __restrict__ op = out + (int64_t)plane * HW;
  if ((HW & 3) == 0) {
    const int64_t n4 = HW >> 2;
    const float4* __restrict__ x4 = reinterpret_cast<const float4*>(xp);
    float4* __restrict__ o4 = reinterpret_cast<float4*>(op);
    const int64_t base = (int64_t)chunk * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int64_t i = base + u * 256 + threadIdx.x;
      if (i < n4) {
        float4 v = x4[i];
        float4 r;
        if (kAdain) {
          r.x = (v.x - mc) / sc * ss + ms;
          r.y = (v.y - mc) / sc * ss + ms;
          r.z = (v.z - mc) / sc * ss + ms;
          r.w = (v.w - mc) / sc * ss + ms;
        } else {
          r.x = (v.x - mc) / sc;
          r.y = (v.y - mc) / sc;
          r.z = (v.z - mc) / sc;
          r.w = (v.w - mc) / sc;
        }
        o4[i] = r;
      }
    }
  } else {
    const int64_t base = (int64_t)chunk * 4096;
    for (int u = 0; u < 16; ++u) {
      int64_t i = base + u * 256 + threadIdx.x;
      if (i < HW) {
        float v = xp[i];
        op[i] = kAdain ? (v - mc) / sc * ss + ms : (v - mc) / sc;
      }
    }
  }
}

static int check_nchw(const void* a, int N, int C, int64_t HW) {
  RPST_REQUIRE(a != nullptr, "null tensor pointer");
  RPST_REQUIRE(N > 0 && C > 0 && HW > 0, "bad shape N=%d C=%d HW=%lld", N, C, (long long)HW);
  RPST_REQUIRE((int64_t)N * C <= 0x7fffffff / 2, "too many planes");
  return RPST_OK;
}

static int launch_apply(bool adain, const float* x, float* out, const float* m0,
                        const float* s0, const float* m1, const float* s1, int planes,
                        int64_t HW, hipStream_t st) {
  const int64_t per = ((HW & 3) == 0) ? 4096 : 4096;  // elements per workgroup
  const int64_t chunks = (HW + per - 1) / per;
  RPST_REQUIRE(chunks * planes <= 0x7fffffffLL, "grid too large");
  dim3 grid((unsigned)(chunks * planes));
  if (adain)
    plane_apply_kernel<true><<<grid, 256, 0, st>>>(x, out, m0, s0, m1, s1, HW, (int)chunks);
  else
    plane_apply_kernel<false><<<grid, 256, 0, st>>>(x, out, m0, s0, m1, s1, HW, (int)chunks);
  return launch_status("plane_apply_kernel");
}

}  // namespace rpst

using namespace rpst;

extern "C" int rpst_calc_mean_std(const float* feat, float* mean, float* std_out, int N,
                                  int C, int64_t HW, float eps, rpst_stream_t stream) {
  if (int e = check_nchw(feat, N, C, HW)) return e;
  RPST_REQUIRE(mean && std_out, "null output pointer");
  const int planes = N * C;
  plane_stats_kernel<<<planes, kStatThreads, 0, as_stream(stream)>>>(
      feat, feat, planes, HW, eps, mean, std_out, mean, std_out);
  return launch_status("plane_stats_kernel");
}

extern "C" size_t rpst_adain_workspace_size(int N, int C) {
  return (size_t)4 * sizeof(float) * (size_t)(N > 0 ? N : 0) * (size_t)(C > 0 ? C : 0);
}

extern "C" int rpst_adain(const float* content, const float* style, float* out, int N,
                          int C, int64_t HW, float eps, void* workspace,
                          size_t workspace_bytes, rpst_stream_t stream) {
  if (int e = check_nchw(content, N, C, HW)) return e;
  RPST_REQUIRE(style && out, "null tensor pointer");
  if (workspace_bytes < rpst_adain_workspace_size(N, C) || !workspace) {
    set_error("adain: workspace %zu < %zu bytes", workspace_bytes,
              rpst_adain_workspace_size(N, C));
    return RPST_EWORKSPACE;
  }
  const int planes = N * C;
  float* ws = static_cast<float*>(workspace);
  float *mc = ws, *sc = ws + planes, *ms = ws + 2 * planes, *ss = ws + 3 * planes;
  hipStream_t st = as_stream(stream);
  plane_stats_kernel<<<2 * planes, kStatThreads, 0, st>>>(content, style, planes, HW, eps,
                                                          mc, sc, ms, ss);
  if (int e = launch_status("plane_stats_kernel")) return e;
  return launch_apply(true, content, out, mc, sc, ms, ss, planes, HW, st);
}

extern "C" int rpst_mean_variance_norm(const float* feat, float* out, int N, int C,
                                       int64_t HW, float eps, void* workspace,
                                       size_t workspace_bytes, rpst_stream_t stream) {
  if (int e = check_nchw(feat, N, C, HW)) return e;
  RPST_REQUIRE(out, "null output pointer");
  if (workspace_bytes < rpst_adain_workspace_size(N, C) || !workspace) {
    set_error("mean_variance_norm: workspace too small");
    return RPST_EWORKSPACE;
  }
  const int planes = N * C;
  float* ws = static_cast<float*>(workspace);
  hipStream_t st = as_stream(stream);
  plane_stats_kernel<<<planes, kStatThreads, 0, st>>>(feat, feat, planes, HW, eps, ws,
                                                      ws + planes, ws, ws + planes);
  if (int e = launch_status("plane_stats_kernel")) return e;
  return launch_apply(false, feat, out, ws, ws + planes, nullptr, nullptr, planes, HW, st);
}
