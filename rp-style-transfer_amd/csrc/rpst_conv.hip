// Direct 3x3 / 1x1 convolution as an implicit GEMM on fp32 MFMA (gfx950).
//
// Replaces the ATen conv stacks of the reference hot path:
//   RP encoder / decoder  Conv2d(k3, zero pad 1) + ReLU      network/base.py:363-396
//   VGG encoder           ReflectionPad2d(1) + Conv2d + ReLU network/base.py:57-111
//                         (+ MaxPool2d(2,2,ceil) fused into the next conv's loader)
//   VGG-mirror decoder    ReflectionPad2d(1) + Conv2d [+ReLU] network/base.py:25-55,
//                         sanet.py:162-192 (+ nearest Upsample x2 fused into the loader)
//   SANet 1x1 f/g/h/out   Conv2d(k1) (+ residual add)         network/sanet.py:76-98
//   Transform merge_conv  ReflectionPad2d + Conv2d on a + up2(b) network/sanet.py:146-149
//
// GEMM view per image n:  out[co][p] = sum_k W[co][k] * X[k][p],  k = (ci, kh, kw).
//   M = Cout (block tile BM), N = pixels (block tile TH rows x 32 cols), K = Cin*KS*KS.
// Per K chunk of CK input channels the block stages into LDS
//   Ws[tap][ci][co]  : CK*KS*KS rows of BM weights (pre-packed K-major, 16-B loads)
//   Xs[ci][py][px]   : the (TH+KS-1) x (32+KS-1) input halo patch per channel, built by
//                      the loader with zero/reflect padding and pool/upsample/add applied
// and every wave runs v_mfma_f32_32x32x2_f32 over its MT x NT sub-tiles of 32x32.
// MFMA operand maps (cdna_hip_programming.md §3): lane l holds A[i=l&31][k=l>>5] and
// B[k=l>>5][j=l&31]; C row = (r&3) + 8*(r>>2) + 4*(l>>5), col = l&31. The two K values
// of one MFMA are channels ci, ci+1 at the same tap, so lane half h reads channel 2cp+h.
// Loads of chunk c+1 are issued into registers before the MFMAs of chunk c and written
// to LDS after them (issue-early / write-late), two workgroups per CU.
// Patch loader: thread -> (channel group tid>>5, column tid&31), so each half-wave reads
// a 128-B row segment and all row index math is wave-uniform (scalar).
// Numerics: exact fp32 products, fp32 accumulation (MFMA = k-ordered fmaf chain).
#include "rpst_conv.h"

#include <cstdlib>
#include <cstring>

namespace rpst {

// CKK = input channels per kernel chunk (divides the packing chunk K::CK);
// DB = double-buffered LDS (one barrier per chunk instead of two).
template <int KS, int BM, int TH, int WM, int WN, int INOP, int NTH, int CKK, bool DB>
__global__ __launch_bounds__(NTH, 2) void conv_mfma_kernel(ConvArgs a) {
  using K = ConvK<KS>;
  constexpr int PCK = K::CK, TAPS = K::TAPS;
  constexpr int CK = CKK, KCH = TAPS * CK;
  static_assert(PCK % CK == 0, "kernel chunk must divide the packing chunk");
  constexpr int OFF = (KS == 3) ? 1 : 0;
  constexpr int PH = TH + KS - 1, PW = kTW + KS - 1;
  constexpr int WTM = BM / WM;       // co per wave
  constexpr int MT = WTM / 32;       // 32-row M sub-tiles per wave
  constexpr int NT = TH / WN;        // rows (32-px N sub-tiles) per wave
  static_assert(WM * WN == NTH / kWave, "one wave per sub-tile");
  static_assert(MT >= 1 && NT >= 1 && (CK % 2) == 0, "tile");
  constexpr int NW4 = KCH * BM / 4;  // float4 weight loads per chunk
  constexpr int WLD = (NW4 + NTH - 1) / NTH;
  constexpr bool WFULL = (NW4 % NTH) == 0;
  // patch loader: NTH/32 groups of 32 lanes; a group owns CPT channels and 1/RS of
  // their rows (RS > 1 when there are more groups than channels in a chunk)
  constexpr int GROUPS = NTH / 32;
  constexpr int CPT = CK > GROUPS ? CK / GROUPS : 1;
  constexpr int RS = GROUPS > CK ? GROUPS / CK : 1;
  constexpr int CGS = GROUPS / RS;                 // distinct channel groups
  constexpr int RPT = (PH + RS - 1) / RS;          // rows per thread
  constexpr int HALO = (KS == 3) ? (2 * PH + 32 * RS - 1) / (32 * RS) : 0;  // halo loads per lane
  constexpr int XN = RPT + HALO;
  static_assert(CPT * CGS == CK, "channel split");

  constexpr int NBUF = DB ? 2 : 1;
  __shared__ float Wsb[NBUF][KCH * BM];
  __shared__ float Xsb[NBUF][CK * PH * PW];

  // block -> (co tile, image, tile row, tile col); co tile slowest so resident blocks
  // share one weight slice in L2
  int bid = blockIdx.x;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  bid /= a.tiles_y;
  const int n = bid % a.N;
  const int ct = bid / a.N;
  const int co0 = ct * BM;
  const int y0 = ty * TH, x0 = tx * kTW;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int h = lane >> 5, j = lane & 31;

  // ---- buffer descriptors (wave-uniform) -------------------------------------------
  const bool pooled = (INOP == RPST_IN_MAXPOOL2 || INOP == RPST_IN_UPSAMPLE2);
  const unsigned in_plane = pooled ? (unsigned)(a.Hs * a.Ws) : (unsigned)(a.H * a.W);
  const unsigned aux_plane = aux_plane_of<INOP>(a);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)conv_in_img(a, n, (int64_t)a.Cin * in_plane), (short)0, (int)(a.Cin * in_plane * 4u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t raux = aux_rsrc<INOP>(a, n);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.wpk + co0), (short)0, 0x7fffffff, 0x00020000);

  // weights: thread -> kernel row r = tid/(BM/4) + u*NTH/(BM/4) = (tap, cl), float4
  // column tid%(BM/4). Packed row of (tap, channel c*CK+cl) = pchunk*TAPS*PCK + tap*PCK + ci%PCK.
  // When the per-u row step RU is a multiple of CK the packed row is linear in u.
  constexpr int RU = NTH / (BM / 4);
  constexpr bool WLIN = (RU % CK) == 0;
  unsigned w_voff[WLIN ? 1 : WLD];
  unsigned w_ustride = 0;
  {
    const int r0 = tid / (BM / 4);
    if (WLIN) {
      w_voff[0] = ((unsigned)((r0 / CK) * PCK + r0 % CK) * a.Cout_pad + (tid % (BM / 4)) * 4) * 4u;
      w_ustride = (unsigned)(RU / CK) * PCK * a.Cout_pad * 4u;
    } else {
#pragma unroll
      for (int u = 0; u < (WLIN ? 1 : WLD); ++u) {
        const int r = r0 + u * RU;
        w_voff[u] = ((unsigned)((r / CK) * PCK + r % CK) * a.Cout_pad + (tid % (BM / 4)) * 4) * 4u;
      }
    }
  }

  // patch: thread -> (channel group cg, row slice rs, column jc); row math is uniform
  const int cg = (tid >> 5) % CGS, rs = (tid >> 5) / CGS, jc = tid & 31;
  int bx = x0 + jc;
  const bool bx_ok = resolve(bx, a.W, a.pad, KS == 3);
  int hy[HALO > 0 ? HALO : 1], hx[HALO > 0 ? HALO : 1];  // (HALO == 0: unused)
  bool h_ok[HALO > 0 ? HALO : 1], has_halo[HALO > 0 ? HALO : 1];
#pragma unroll
  for (int e = 0; e < HALO; ++e) {
    const int hi = jc + 32 * (rs + RS * e);
    has_halo[e] = hi < 2 * PH;
    hy[e] = y0 - OFF + (hi >> 1);
    hx[e] = (hi & 1) ? x0 + kTW : x0 - 1;
    const bool ok1 = resolve(hy[e], a.H, a.pad, true);
    const bool ok2 = resolve(hx[e], a.W, a.pad, true);
    h_ok[e] = has_halo[e] && ok1 && ok2;
  }

  floatx16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  constexpr int R = RawN<INOP>::R;
  u32x4 wreg[WLD];
  float xraw[CPT][XN][R];
  AdainP ap[CPT];

#define RPST_CONV_LOAD(c)                                                                   \
  {                                                                                         \
    const unsigned c0 = (unsigned)(c) * CK;                                                 \
    const unsigned wc = ((c0 / PCK) * TAPS * PCK + c0 % PCK) * a.Cout_pad * 4u;            \
    _Pragma("unroll") for (int u = 0; u < WLD; ++u) {                                       \
      const bool wv = WFULL || tid + u * NTH < NW4;                                         \
      wreg[u] = __builtin_amdgcn_raw_buffer_load_b128(                                      \
          rw, (int)(wv ? (WLIN ? w_voff[0] + u * w_ustride : w_voff[WLIN ? 0 : u]) + wc    \
                       : kOOB), 0, 0);                                                      \
    }                                                                                       \
    _Pragma("unroll") for (int q = 0; q < CPT; ++q) {                                       \
      const unsigned ch = (unsigned)((c) * CK + cg + CGS * q);                              \
      const unsigned pb = ch * in_plane * 4u, ab = ch * aux_plane * 4u;                     \
      if (INOP == RPST_IN_ADAIN || INOP == RPST_IN_ADD_ADAIN)                               \
        ap[q] = adain_params(a.aux, n, (int)ch, a);                                         \
      _Pragma("unroll") for (int i = 0; i < RPT; ++i) {                                     \
        const int py = rs * RPT + i;                                                        \
        int y = y0 - OFF + py;                                                              \
        const bool yok = resolve(y, a.H, a.pad, KS == 3) && py < PH;                        \
        fetch_raw<INOP>(xraw[q][i], rin, raux, pb, ab, y, bx, yok && bx_ok, a);             \
      }                                                                                     \
      _Pragma("unroll") for (int e = 0; e < HALO; ++e)                                      \
        fetch_raw<INOP>(xraw[q][RPT + e], rin, raux, pb, ab, hy[e], hx[e], h_ok[e], a);     \
    }                                                                                       \
  }

  const int aoff = h * BM + wm * WTM + j;
  const int boff = h * PH * PW + (wn * NT) * PW + j;

  RPST_CONV_LOAD(0)
  const int nchunks = (a.Cin + CK - 1) / CK;
  for (int c = 0; c < nchunks; ++c) {
    float* Ws = Wsb[DB ? (c & 1) : 0];
    float* Xs = Xsb[DB ? (c & 1) : 0];
#pragma unroll
    for (int u = 0; u < WLD; ++u)
      if (WFULL || tid + u * NTH < NW4)
        *reinterpret_cast<u32x4*>(Ws + 4 * (tid + u * NTH)) = wreg[u];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      float* xs = Xs + (cg + CGS * q) * PH * PW;
      const bool chok = (int)(c * CK + cg + CGS * q) < a.Cin;
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int py = rs * RPT + i;
        bool ok = chok && bx_ok;
        if (INOP == RPST_IN_ADAIN || INOP == RPST_IN_ADD_ADAIN) {
          int y = y0 - OFF + py;
          ok = ok && resolve(y, a.H, a.pad, KS == 3);
        }
        const float v = combine<INOP>(xraw[q][i], ok, ap[q]);
        if ((PH % RS) == 0 || py < PH) xs[py * PW + jc + OFF] = v;
      }
#pragma unroll
      for (int e = 0; e < HALO; ++e) {
        const int hi = jc + 32 * (rs + RS * e);
        const float v = combine<INOP>(xraw[q][RPT + e], chok && h_ok[e], ap[q]);
        if (has_halo[e]) xs[(hi >> 1) * PW + ((hi & 1) ? PW - 1 : 0)] = v;
      }
    }
    __syncthreads();
    if (c + 1 < nchunks) RPST_CONV_LOAD(c + 1)
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const int kh = t / KS, kw = t % KS;
#pragma unroll
      for (int cp = 0; cp < CK / 2; ++cp) {
        float av[MT], bv[NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) av[mt] = Ws[aoff + (t * CK + 2 * cp) * BM + mt * 32];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          bv[nt] = Xs[boff + (2 * cp) * PH * PW + (nt + kh) * PW + kw];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mt], bv[nt], acc[mt][nt],
                                                               0, 0, 0);
      }
    }
    if (!DB) __syncthreads();  // double-buffered: the next chunk's barrier suffices
  }
#undef RPST_CONV_LOAD

  // epilogue: bias, ReLU, residual, predicated coalesced stores (128 B per half-wave)
  const int x = x0 + j;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wm * WTM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co >= a.Cout) continue;
      const float b = a.bias ? a.bias[co] : 0.f;
      const int64_t pbase = ((int64_t)n * a.Cout + co) * a.H * a.W;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int y = y0 + wn * NT + nt;
        float v = acc[mt][nt][r] + b;
        v = activate(v, a.relu);
        if (y < a.H && x < a.W) {
          const int64_t o = pbase + (int64_t)y * a.W + x;
          if (a.res) v += a.res[o];
          if (a.mask && !(a.mask[o] > 0.f)) v = 0.f;
          a.out[o] = v;
        }
        acc[mt][nt][r] = v;
      }
    }
  }

  // optional output statistics (AdaIN / calc_mean_std of this layer's output, fused):
  // each half-wave holds 16 output channels (r) x NT rows x 32 columns of this tile per
  // mt. Two-pass per channel: sums via a half-wave reduce-scatter (16 shuffles for 16
  // values), means broadcast back, centred sums of squares the same way -> (mean, M2)
  // per (channel, wave tile), merged in fp64 by stat_merge_kernel.
  // (compiled only for tiles with >= 4 rows per wave: with NT <= 2 hipcc keeps the
  // accumulators dynamically indexed and spills thousands of VGPRs)
  if constexpr (NT >= 4) if (a.stat_part) {
    const int rows = max(0, min(NT, a.H - (y0 + wn * NT)));
    const int cols = max(0, min(kTW, a.W - x0));
    const int cnt = rows * cols;
    const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
    const bool xv = x < a.W;
    const int pidx = (ty * a.tiles_x + tx) * WN + wn;
    const int e = (j >> 1) & 15;  // channel index r this lane ends up holding
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float t = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) t += (xv && nt < rows) ? acc[mt][nt][r] : 0.f;
        v[r] = t;
      }
      const float mean = halfwave_reduce_scatter16(v, j) * inv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float mr = __shfl(mean, (h << 5) + 2 * r, 64);
        float t = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const float d = acc[mt][nt][r] - mr;
          t += (xv && nt < rows) ? d * d : 0.f;
        }
        v[r] = t;
      }
      const float m2 = halfwave_reduce_scatter16(v, j);
      const int co = co0 + wm * WTM + mt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if ((j & 1) == 0 && co < a.Cout)
        a.stat_part[((int64_t)n * a.Cout + co) * a.stat_P + pidx] = make_float2(mean, m2);
    }
  }
}

// Merge the (mean, M2) partials of one (n, c) plane in fp64 (Chan et al.), fixed order:
// lane l folds partials l, l+64, ...; then a butterfly over lanes. Writes calc_mean_std.
__global__ __launch_bounds__(256) void stat_merge_kernel(const float2* __restrict__ part,
                                                         float* __restrict__ mean,
                                                         float* __restrict__ stdv, int planes,
                                                         int P, int tiles_x, int WN, int NT,
                                                         int TW, int H, int W, float eps) {
  const int plane = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (plane >= planes) return;
  double cn = 0.0, cm = 0.0, c2 = 0.0;
  for (int p = lane; p < P; p += 64) {
    const int tile = p / WN, wn = p - tile * WN;
    const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
    const int rows = max(0, min(NT, H - (ty * NT * WN + wn * NT)));
    const int cols = max(0, min(TW, W - tx * TW));
    const double nb = (double)(rows * cols);
    if (nb == 0.0) continue;
    const float2 v = part[(int64_t)plane * P + p];
    const double n2 = cn + nb, d = (double)v.x - cm;
    cm += d * nb / n2;
    c2 += (double)v.y + d * d * cn * nb / n2;
    cn = n2;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double on = __shfl_xor(cn, o, 64), om = __shfl_xor(cm, o, 64), o2 = __shfl_xor(c2, o, 64);
    const double n2 = cn + on;
    if (n2 > 0.0) {
      const double d = om - cm;
      cm += d * on / n2;
      c2 += o2 + d * d * cn * on / n2;
    }
    cn = n2;
  }
  if (lane == 0) {
    float varf = (float)(cn > 1.0 ? c2 / (cn - 1.0) : __builtin_nan(""));
    mean[plane] = (float)cm;
    stdv[plane] = __fsqrt_rn(__fadd_rn(varf, eps));
  }
}

// The same merge for partials in [n][partial][co] order (ConvGeom::stat_t): a block takes 64
// consecutive channels of one image (coalesced 512-B reads per partial); its 4 waves fold
// the partials in 4 consecutive segments, each lane in order, then the 4 segment states are
// combined in segment order -- a fixed order, as above (the float2 partials are rounded the
// same; the fp64 merge tree differs from stat_merge_kernel's).
__global__ __launch_bounds__(256) void stat_merge_t_kernel(const float2* __restrict__ part,
                                                           float* __restrict__ mean,
                                                           float* __restrict__ stdv, int Cout,
                                                           int P, int tiles_x, int WN, int NT,
                                                           int TW, int H, int W, float eps) {
  const int cgroups = (Cout + 63) / 64;
  const int n = blockIdx.x / cgroups;
  const int co = (blockIdx.x - n * cgroups) * 64 + (threadIdx.x & 63);
  const int seg = threadIdx.x >> 6;
  const int per = (P + 3) / 4, p0 = seg * per, p1 = min(P, p0 + per);
  double cn = 0.0, cm = 0.0, c2 = 0.0;
  if (co < Cout) {
    const float2* pp = part + (int64_t)n * P * Cout + co;
    for (int p = p0; p < p1; ++p) {
      const int tile = p / WN, wn = p - tile * WN;
      const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
      const int rows = max(0, min(NT, H - (ty * NT * WN + wn * NT)));
      const int cols = max(0, min(TW, W - tx * TW));
      const double nb = (double)(rows * cols);
      if (nb == 0.0) continue;
      const float2 v = pp[(int64_t)p * Cout];
      const double n2 = cn + nb, d = (double)v.x - cm;
      cm += d * nb / n2;
      c2 += (double)v.y + d * d * cn * nb / n2;
      cn = n2;
    }
  }
  __shared__ double sh[3][256];
  sh[0][threadIdx.x] = cn;
  sh[1][threadIdx.x] = cm;
  sh[2][threadIdx.x] = c2;
  __syncthreads();
  if (seg != 0 || co >= Cout) return;
  for (int s = 1; s < 4; ++s) {
    const int t = s * 64 + threadIdx.x;
    const double on = sh[0][t], om = sh[1][t], o2 = sh[2][t];
    const double n2 = cn + on;
    if (n2 > 0.0) {
      const double d = om - cm;
      cm += d * on / n2;
      c2 += o2 + d * d * cn * on / n2;
    }
    cn = n2;
  }
  const float varf = (float)(cn > 1.0 ? c2 / (cn - 1.0) : __builtin_nan(""));
  mean[(int64_t)n * Cout + co] = (float)cm;
  stdv[(int64_t)n * Cout + co] = __fsqrt_rn(__fadd_rn(varf, eps));
}

// ---- weight packing: (Cout,Cin,KS,KS) -> [chunk][tap][ci_local][Cout_pad] ------------
__global__ void conv_pack_kernel(const float* __restrict__ w, float* __restrict__ pk,
                                 int Cout, int Cin, int KS, int CK, int Cout_pad,
                                 int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int taps = KS * KS;
  const int co = (int)(i % Cout_pad);
  int64_t r = i / Cout_pad;
  const int cl = (int)(r % CK);
  r /= CK;
  const int t = (int)(r % taps);
  const int c = (int)(r / taps);
  const int ci = c * CK + cl;
  float v = 0.f;
  if (ci < Cin && co < Cout) v = w[(((int64_t)co * Cin + ci) * taps) + t];
  pk[i] = v;
}

struct TileCfg {
  int BM, TH;
};

static TileCfg pick_cfg(int Cout) {
  if (Cout > 64) return {128, 8};
  if (Cout > 32) return {64, 8};
  return {32, 16};
}

static int pad_cout(int Cout) {
  const int bm = pick_cfg(Cout).BM;
  return (Cout + bm - 1) / bm * bm;
}

static int ck_of(int ksize) { return ksize == 3 ? ConvK<3>::CK : ConvK<1>::CK; }

// ---- narrow 3x3 layers on the VALU ------------------------------------------------------
// Cout <= 4 with Cin <= 64, or Cout <= 16 with Cin <= 4 (narrow_shape; the RP stacks'
// 3->16 input and 16->3 output convs, base.py:363-396 encoder / decoder ends, and the
// MultiScale decoder's last block 32->3, whose loader forms stylized + AdaIN(c) per element:
// INOP = RPST_IN_ADD_ADAIN, adain_rp.py:301): an MFMA tile
// pads such a layer to 32 output channels (16->3: 10x the work) or 8 input channels, so
// these run as plain FMAs instead (algorithm RPST_CONV_NARROW). Block = 4 RPT rows x 64
// columns, 256 threads (column, RPT rows); per input channel the (4 RPT+2) x 66 patch is
// staged in LDS with the padding resolved, weights [ci][tap][co] sit in LDS for the
// whole block. Same epilogue as the direct kernel: bias, activation, residual. Images go
// on grid.z: batches above 65535 images (or 65535 row tiles) take the MFMA direct path.
#ifndef RPST_NR_ALL  // 3->16 @512^2 N64 0.453 -> 0.437 (patch loads before the weight
#define RPST_NR_ALL 1  // staging) -> 0.364 ms (every channel up front): profiles/r05/narrow_ab.log
#endif
constexpr int kNrTW = 64, kNrPW = kNrTW + 2;
constexpr int kNrMaxCin = 64, kNrMaxCo = 16, kNrWl = 256 * 9;  // weight floats in LDS

static bool narrow_shape(int Cin, int Cout) {
  return (Cout <= 4 && Cin <= kNrMaxCin) || (Cout <= kNrMaxCo && Cin <= 4);
}
// the largest Cin * CO an instantiation can meet must fit the LDS weight array
static_assert(kNrMaxCin * 9 * 4 <= kNrWl && 4 * 9 * kNrMaxCo <= kNrWl, "narrow weights fit LDS");

template <int CO, int RPT, int INOP = RPST_IN_NONE>  // block = 4 RPT rows x 64 columns
__global__ __launch_bounds__(256) void conv3x3_narrow_kernel(ConvArgs a) {
  static_assert(INOP == RPST_IN_NONE || INOP == RPST_IN_ADD_ADAIN, "narrow loaders");
  constexpr bool kSkip = INOP == RPST_IN_ADD_ADAIN;
  constexpr int CK = ConvK<3>::CK, kNrTH = 4 * RPT, kNrPS = (kNrTH + 2) * kNrPW;
  __shared__ float patch[kNrPS];
  __shared__ __attribute__((aligned(8))) float wl[kNrWl];  // Cin * 9 * CO <= 2304 (narrow_shape)
  const int x0 = blockIdx.x * kNrTW, y0 = blockIdx.y * kNrTH, n = blockIdx.z;
  const int tid = threadIdx.x, col = tid & 63, rg = tid >> 6;  // output rows RPT rg ..
  // accumulators in channel pairs: one v_pk_fma_f32 per two output channels
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 acc2[RPT][CO / 2];
#pragma unroll
  for (int r = 0; r < RPT; ++r)
#pragma unroll
    for (int c2 = 0; c2 < CO / 2; ++c2) acc2[r][c2] = f2{0.f, 0.f};
  const int64_t plane = (int64_t)a.H * a.W;
  const float* in = conv_in_img(a, n, (int64_t)a.Cin * plane);
  // this thread's patch elements (slot s: element tid + 256 s), their in-plane offsets
  // resolved against the padding once (-1: zero padding / outside the patch); channel ci + 1
  // is loaded into registers while channel ci is computed (the load latency hides under
  // the FMAs instead of stalling every channel)
  constexpr int kSl = (kNrPS + 255) / 256;
  int off[kSl];
#pragma unroll
  for (int sl = 0; sl < kSl; ++sl) {
    const int i = tid + 256 * sl;
    const int r = i / kNrPW, c = i - r * kNrPW;
    int y = y0 - 1 + r, x = x0 - 1 + c;
    const bool oky = resolve(y, a.H, a.pad, true), okx = resolve(x, a.W, a.pad, true);
    off[sl] = (i < kNrPS && oky && okx) ? y * a.W + x : -1;
  }
  // ADD_ADAIN: the skip feature c (aux2) of the same shape; the element is
  // stylized + ((c - mean_c) / std_c) * std_s + mean_s (0 at zero padding)
  const float* cin = kSkip ? a.aux2 + (int64_t)n * a.Cin * plane : nullptr;
  float pre[kSl], prc[kSkip ? kSl : 1];
  auto fetch = [&](int ci) {
    const float* src = in + (int64_t)ci * plane;
#pragma unroll
    for (int sl = 0; sl < kSl; ++sl) pre[sl] = off[sl] >= 0 ? src[off[sl]] : 0.f;
    if constexpr (kSkip) {
      const float* cs = cin + (int64_t)ci * plane;
#pragma unroll
      for (int sl = 0; sl < kSl; ++sl) prc[sl] = off[sl] >= 0 ? cs[off[sl]] : 0.f;
    }
  };
  // RPST_NR_ALL: with Cin <= 4 (the 16-channel form) every channel's patch is loaded up
  // front, so no channel waits on its own loads
  constexpr bool kAll = RPST_NR_ALL && CO == 16 && !kSkip;
  float preA[kAll ? 4 : 1][kSl];
  if constexpr (kAll) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int sl = 0; sl < kSl; ++sl)
        preA[c][sl] = (c < a.Cin && off[sl] >= 0) ? in[(int64_t)c * plane + off[sl]] : 0.f;
  } else {
    fetch(0);
  }
  // direct-packed weights [ci / CK][tap][ci % CK][Cout_pad] (zero beyond Cout), staged while
  // the first patch loads are in flight
  for (int i = tid; i < a.Cin * 9 * CO; i += 256) {
    const int co = i % CO, t = (i / CO) % 9, ci = i / (9 * CO);
    wl[i] = a.wpk[((int64_t)(ci / CK) * 9 + t) * CK * a.Cout_pad + (ci % CK) * a.Cout_pad + co];
  }
  for (int ci = 0; ci < a.Cin; ++ci) {
    if constexpr (kAll) {
#pragma unroll
      for (int sl = 0; sl < kSl; ++sl)
        pre[sl] = ci == 0 ? preA[0][sl] : ci == 1 ? preA[1][sl] : ci == 2 ? preA[2][sl] : preA[3][sl];
    }
    __syncthreads();  // the previous channel's patch is consumed (first pass: weights)
    if constexpr (kSkip) {
      const AdainP pa = adain_params(a.aux, n, ci, a);
#pragma unroll
      for (int sl = 0; sl < kSl; ++sl)
        if (tid + 256 * sl < kNrPS)
          patch[tid + 256 * sl] = off[sl] >= 0 ? pre[sl] + fmaf(prc[sl] - pa.mc, pa.scale, pa.ms) : 0.f;
    } else {
#pragma unroll
      for (int sl = 0; sl < kSl; ++sl)
        if (tid + 256 * sl < kNrPS) patch[tid + 256 * sl] = pre[sl];
    }
    __syncthreads();
    if (!kAll && ci + 1 < a.Cin) fetch(ci + 1);
    float win[RPT + 2][3];
#pragma unroll
    for (int r = 0; r < RPT + 2; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) win[r][c] = patch[(RPT * rg + r) * kNrPW + col + c];
    const f2* w = reinterpret_cast<const f2*>(wl + ci * 9 * CO);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int c2 = 0; c2 < CO / 2; ++c2) {
        const f2 wv = w[t * (CO / 2) + c2];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
          const float xv = win[t / 3 + r][t % 3];
          acc2[r][c2] = __builtin_elementwise_fma(f2{xv, xv}, wv, acc2[r][c2]);
        }
      }
  }
  float acc[RPT][CO];
#pragma unroll
  for (int r = 0; r < RPT; ++r)
#pragma unroll
    for (int c2 = 0; c2 < CO / 2; ++c2) {
      acc[r][2 * c2] = acc2[r][c2].x;
      acc[r][2 * c2 + 1] = acc2[r][c2].y;
    }
  const int x = x0 + col;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int y = y0 + RPT * rg + r;
    if (y >= a.H || x >= a.W) continue;
#pragma unroll
    for (int co = 0; co < CO; ++co) {
      if (co >= a.Cout) continue;  // (not break: the loop stays fully unrolled)
      const int64_t o = ((int64_t)n * a.Cout + co) * plane + (int64_t)y * a.W + x;
      float v = activate(acc[r][co] + (a.bias ? a.bias[co] : 0.f), a.relu);
      if (a.res) v += a.res[o];
      if (a.mask && !(a.mask[o] > 0.f)) v = 0.f;
      a.out[o] = v;
    }
  }
}

static bool narrow_enabled() {
  const char* e = getenv("RPST_CONV_NARROW");  // A/B switch
  return !(e && *e && atoi(e) == 0);
}

// Tile variants per BM. RPST_CONV_VARIANT (tools/bench_conv.py) forces one for tuning;
// otherwise pick_variant() chooses from the measured table (profiles/r01_bench_conv.log):
//   BM=128: 3x3 -> v1 (128 co x 8x32 px, 8 accumulators/wave, 134-143 TF/s);
//           max-pool input or 1x1 -> v2 (128 x 4x32, lighter loader, 113-128 TF/s);
//   BM=64 / BM=32 -> v1 (4-channel chunks, double-buffered LDS, 1 barrier per chunk).
// <BM, TH, WM, WN, NTH, CK, DB>: block tile BM x (TH x 32 px), WM x WN waves of NTH/64.
template <int KS, int INOP>
static void launch_conv(const ConvArgs& a, int BM, int variant, hipStream_t st) {
  const int blocks = a.tiles_x * a.tiles_y * a.N * a.co_tiles;
#define RPST_LAUNCH(BM_, TH_, WM_, WN_, NTH_, CK_, DB_) \
  conv_mfma_kernel<KS, BM_, TH_, WM_, WN_, INOP, NTH_, CK_, DB_><<<blocks, NTH_, 0, st>>>(a)
  constexpr int C8 = ConvK<KS>::CK, C4 = ConvK<KS>::CK / 2;
  // loaders with 2-4 raw loads per element only get the short-tile variants (the tall
  // ones run out of registers)
  constexpr bool HEAVY = RawN<INOP>::R > 1;
  if constexpr (HEAVY) {
    if (BM == 128) {
      if (variant == 4) RPST_LAUNCH(128, 4, 2, 2, 256, C4, true);
      else RPST_LAUNCH(128, 4, 2, 2, 256, C8, false);
    } else if (BM == 64) {
      if (variant == 0) RPST_LAUNCH(64, 8, 1, 4, 256, C8, false);
      else RPST_LAUNCH(64, 8, 1, 4, 256, C4, true);
    } else {
      if (variant == 2) RPST_LAUNCH(32, 8, 1, 4, 256, C8, false);
      else RPST_LAUNCH(32, 8, 1, 4, 256, C4, true);
    }
  } else {
  if (BM == 128) {
    switch (variant) {
      case 0: RPST_LAUNCH(128, 8, 2, 4, 512, C8, false); break;
      case 2: RPST_LAUNCH(128, 4, 2, 2, 256, C8, false); break;
      case 3: RPST_LAUNCH(128, 8, 2, 2, 256, C4, true); break;
      case 4: RPST_LAUNCH(128, 4, 2, 2, 256, C4, true); break;
      default: RPST_LAUNCH(128, 8, 2, 2, 256, C8, false);
    }
  } else if (BM == 64) {
    switch (variant) {
      case 0: RPST_LAUNCH(64, 8, 1, 4, 256, C8, false); break;
      case 2: RPST_LAUNCH(64, 8, 1, 8, 512, C8, false); break;
      default: RPST_LAUNCH(64, 8, 1, 4, 256, C4, true);
    }
  } else {
    switch (variant) {
      case 0: RPST_LAUNCH(32, 16, 1, 4, 256, C8, false); break;
      case 2: RPST_LAUNCH(32, 8, 1, 4, 256, C8, false); break;
      default: RPST_LAUNCH(32, 8, 1, 4, 256, C4, true);
    }
  }
  }
#undef RPST_LAUNCH
}

static bool heavy_loader(int in_op) {
  return in_op == RPST_IN_MAXPOOL2 || in_op == RPST_IN_ADD_UPSAMPLE2 ||
         in_op == RPST_IN_ADD_ADAIN;
}

static int pick_variant(int BM, int ksize, int in_op) {
  if (BM == 128 && (heavy_loader(in_op) || ksize == 1)) return 2;
  return 1;
}

// TH of a variant (the host needs it for the grid)
static int variant_th(int BM, int variant) {
  if (BM == 128) return (variant == 2 || variant == 4) ? 4 : 8;
  if (BM == 64) return 8;
  return variant == 0 ? 16 : 8;
}

// threads per workgroup of a variant
static int variant_nth(int BM, int variant) {
  return ((BM == 128 && variant == 0) || (BM == 64 && variant == 2)) ? 512 : 256;
}

// WN (waves along the pixel rows) of a variant: rows per wave = TH / WN
static int variant_wn(int BM, int variant) {
  if (BM == 128) return variant == 0 ? 4 : 2;
  if (BM == 64) return variant == 2 ? 8 : 4;
  return 4;
}

static int conv_variant(int BM, int ksize, int in_op) {
  const char* e = getenv("RPST_CONV_VARIANT");
  int v = (e && *e) ? atoi(e) : pick_variant(BM, ksize, in_op);
  if (heavy_loader(in_op)) {  // the variants launch_conv instantiates for heavy loaders
    if (BM == 128) v = (v == 4) ? 4 : 2;
    else if (BM == 64) v = (v == 0) ? 0 : 1;
    else v = (v == 2) ? 2 : 1;
  }
  return v;
}

// Algorithm for a 3x3 conv: Winograd F(4x4,3x3) (rpst_wino4.hip) for the loader
// operators it implements, F(2x2,3x3) (rpst_wino.hip) for the others, the direct implicit
// GEMM for the 16-wide layers and every 1x1. RPST_CONV_ALGO=direct|winograd|winograd4
// overrides (tests, A/B benches; winograd4 falls back to winograd where unsupported).
// rpst_conv2d_set_precise: at 1 this thread's launches keep to F(2x2) where F(4x4) would
// run; at 2 F(4x4) runs, on its 32-channel form only (wino4q_applies)
static thread_local int t_conv_precise = 0;
// rpst_conv2d_set_quarter: -1 (default) follows RPST_W4Q, read per launch
static thread_local int t_conv_quarter = -1;

bool conv_quarter_allowed() { return t_conv_precise != 2; }

int conv_quarter_mode() {
  if (t_conv_quarter >= 0) return t_conv_quarter;
  const char* e = getenv("RPST_W4Q");
  return (e && *e) ? atoi(e) : 1;
}

static int conv_algo(int Cout, int Cin, int Hs, int Ws, int ksize, int in_op) {
  if (ksize != 3) return RPST_CONV_DIRECT;
  const bool w4 = wino4_supports(in_op) && wino4_fits(1, Cin, Hs, Ws, in_op);
  const bool nr = (in_op == RPST_IN_NONE || (in_op == RPST_IN_ADD_ADAIN && Cout <= 4)) &&
                  narrow_shape(Cin, Cout) && narrow_enabled();
  const char* e = getenv("RPST_CONV_ALGO");
  if (e && *e) {
    if (e[0] == 'd') return nr ? RPST_CONV_NARROW : RPST_CONV_DIRECT;
    if (!strcmp(e, "winograd")) return RPST_CONV_WINOGRAD;
    if (!strcmp(e, "winograd4")) return w4 ? RPST_CONV_WINOGRAD4 : RPST_CONV_WINOGRAD;
  }
  // measured (profiles/r01_bench_conv_wino4.log): F(4x4) wins every layer with >= 16 input
  // channels it supports, the 16-wide 32->16 decoder layer included; the narrow shapes
  // (3->16 / 16->3 of the RP stacks, <= 4-channel outputs) run on the VALU kernel (3->16
  // 0.44 / 16->3 0.16 ms vs 0.57 / 0.64 on MFMA tiles; the VGG decoders' 64->3 reflect at
  // 512^2, N = 32: 0.63 ms vs 1.05 on F(4x4), profiles/r04/narrow64.log); the wider 3-channel first convs
  // (VGG 3->64, MultiScale 3->32) run on F(4x4): 3->64 reflect at 512^2, N = 64: 1.25 ms vs
  // 1.59 direct and 2.49 on the VALU kernel (tools/bench_conv.py); other inputs below 16
  // channels, and precise mode, stay direct
  if (nr) return RPST_CONV_NARROW;
  if (Cin <= 4 && w4 && t_conv_precise != 1) return RPST_CONV_WINOGRAD4;
  if (Cin < 16) return RPST_CONV_DIRECT;
  if (w4 && t_conv_precise != 1) return RPST_CONV_WINOGRAD4;
  if (w4) return RPST_CONV_WINOGRAD;  // precise mode, same shapes as F(4x4)
  return Cout >= 32 ? RPST_CONV_WINOGRAD : RPST_CONV_DIRECT;
}

static void logical_hw(int Hs, int Ws, int in_op, int* H, int* W) {
  *H = Hs;
  *W = Ws;
  if (in_op == RPST_IN_MAXPOOL2) {
    *H = (Hs + 1) / 2;
    *W = (Ws + 1) / 2;
  } else if (in_op == RPST_IN_UPSAMPLE2) {
    *H = 2 * Hs;
    *W = 2 * Ws;
  }
}

// Launch geometry shared by the entry points: blocks, threads per block, statistics
// partials per plane and their (rows per partial, partials per tile row) layout.
struct ConvGeom {
  int algo;
  int64_t blocks;
  int nth, stat_P, stat_nt, stat_wn, stat_tw, tiles_x;
  bool stat_t;  // partials in [n][partial][co] order (the position-quarter F(4x4) kernel)
};

// rows per thread of the narrow kernel: 4 for Cout <= 4 (16->3: 0.307 vs 0.348 ms;
// RPST_CONV_NARROW_RPT=2 overrides), 2 for Cout <= 16 (3->16 at 4 rows spills to scratch:
// 1.47 vs 0.51 ms)
static int narrow_rpt(int Cout) {
  const char* e = getenv("RPST_CONV_NARROW_RPT");
  return Cout <= 4 && !(e && *e && atoi(e) == 2) ? 4 : 2;
}

// the narrow kernel puts the images on grid.z and the row tiles on grid.y (<= 65535 each);
// it has no statistics epilogue
static bool narrow_launchable(int N, int H, int Cout, bool stats) {
  return !stats && N <= 65535 && (H + 4 * narrow_rpt(Cout) - 1) / (4 * narrow_rpt(Cout)) <= 65535;
}

static ConvGeom conv_geom(int N, int Cin, int Hs, int Ws, int Cout, int ksize, int in_op,
                          bool stats = false) {
  int H, W;
  logical_hw(Hs, Ws, in_op, &H, &W);
  ConvGeom g{};
  g.algo = conv_algo(Cout, Cin, Hs, Ws, ksize, in_op);
  if (g.algo == RPST_CONV_NARROW && !narrow_launchable(N, H, Cout, stats))
    g.algo = RPST_CONV_DIRECT;
  if (g.algo == RPST_CONV_NARROW) {
    const int rows = 4 * narrow_rpt(Cout);
    g.tiles_x = (W + kNrTW - 1) / kNrTW;
    g.blocks = (int64_t)g.tiles_x * ((H + rows - 1) / rows) * N;
    g.nth = 256;
    g.stat_tw = kNrTW;
    return g;
  }
  g.tiles_x = (W + kTW - 1) / kTW;
  g.stat_tw = kTW;
  if (g.algo == RPST_CONV_WINOGRAD4) {
    const int nr = wino4_rows(Cin, Cout, in_op);
    g.tiles_x = (W + kW4Cols - 1) / kW4Cols;
    const int ty = (H + 4 * nr - 1) / (4 * nr);
    g.blocks = (int64_t)g.tiles_x * ty * N * (wino4_persist() ? 1 : (Cout + kW4Co - 1) / kW4Co);
    g.stat_t = wino4q_applies(Cin, Cout, in_op);
    g.nth = g.stat_t ? 512 : 128 * nr;
    g.stat_P = g.tiles_x * ty * nr;
    g.stat_nt = 4;
    g.stat_wn = nr;
    g.stat_tw = kW4Cols;
    return g;
  }
  if (g.algo == RPST_CONV_WINOGRAD) {
    const int th = wino_th(), bm = wino_bm();
    const int ty = (H + th - 1) / th;
    g.blocks = (int64_t)g.tiles_x * ty * N * (wino_persist(in_op, (int64_t)g.tiles_x * ty * N) ? 1 : (Cout + bm - 1) / bm);
    g.nth = kWinoNTH;
    g.stat_P = g.tiles_x * ty;
    g.stat_nt = th;
    g.stat_wn = 1;
    return g;
  }
  const TileCfg cfg = pick_cfg(Cout);
  const int variant = conv_variant(cfg.BM, ksize, in_op);
  const int th = variant_th(cfg.BM, variant), wn = variant_wn(cfg.BM, variant);
  const int ty = (H + th - 1) / th;
  g.blocks = (int64_t)g.tiles_x * ty * N * (pad_cout(Cout) / cfg.BM);
  g.nth = variant_nth(cfg.BM, variant);
  g.stat_P = g.tiles_x * ty * wn;
  g.stat_nt = th / wn;
  g.stat_wn = wn;
  return g;
}

static size_t direct_packed_floats(int Cout, int Cin, int ksize) {
  const int ck = ck_of(ksize);
  const size_t nch = (size_t)(Cin + ck - 1) / ck;
  return nch * ksize * ksize * ck * (size_t)pad_cout(Cout);
}

}  // namespace rpst

using namespace rpst;

// 3x3 weights are packed three times: the direct image, the F(2x2) Winograd image and
// the F(4x4) Winograd image (the algorithm is chosen per launch; all are small).
extern "C" size_t rpst_conv2d_packed_size(int Cout, int Cin, int ksize) {
  if (Cout <= 0 || Cin <= 0 || (ksize != 1 && ksize != 3)) return 0;
  size_t f = direct_packed_floats(Cout, Cin, ksize);
  if (ksize == 3)
    f += wino_packed_floats(Cout, Cin) + wino4_packed_floats(Cout, Cin) +
         wino4q_packed_floats(Cout, Cin);
  return f * sizeof(float);
}

extern "C" int64_t rpst_conv2d_grid_threads(int N, int Cin, int Hs, int Ws, int Cout,
                                            int ksize, int in_op) {
  if (N <= 0 || Cin <= 0 || Hs <= 0 || Ws <= 0 || Cout <= 0 || (ksize != 1 && ksize != 3))
    return 0;
  const ConvGeom g = conv_geom(N, Cin, Hs, Ws, Cout, ksize, in_op);
  return g.blocks * g.nth;
}

extern "C" int rpst_conv2d_set_precise(int on) {
  const int old = t_conv_precise;
  t_conv_precise = on == 2 ? 2 : on != 0;
  return old;
}

extern "C" int rpst_conv2d_set_quarter(int mode) {
  const int old = t_conv_quarter;
  t_conv_quarter = mode < 0 ? -1 : (mode > 2 ? 2 : mode);
  return old;
}

extern "C" int rpst_conv2d_algorithm(int Cout, int Cin, int Hs, int Ws, int ksize, int in_op) {
  return conv_algo(Cout, Cin, Hs, Ws, ksize, in_op);
}

extern "C" int rpst_conv2d_quarter(int Cout, int Cin, int Hs, int Ws, int ksize, int in_op) {
  if (conv_algo(Cout, Cin, Hs, Ws, ksize, in_op) != RPST_CONV_WINOGRAD4) return 0;
  return wino4q_applies(Cin, Cout, in_op) ? 1 : 0;
}

extern "C" int rpst_conv2d_pack(const float* weight, float* packed, int Cout, int Cin,
                                int ksize, rpst_stream_t stream) {
  RPST_REQUIRE(weight && packed, "conv2d_pack: null pointer");
  RPST_REQUIRE(Cout > 0 && Cin > 0, "conv2d_pack: bad channels");
  RPST_REQUIRE(ksize == 1 || ksize == 3, "conv2d_pack: ksize must be 1 or 3, got %d", ksize);
  const int64_t total = (int64_t)direct_packed_floats(Cout, Cin, ksize);
  const int threads = 256;
  conv_pack_kernel<<<(unsigned)((total + threads - 1) / threads), threads, 0,
                     as_stream(stream)>>>(weight, packed, Cout, Cin, ksize, ck_of(ksize),
                                          pad_cout(Cout), total);
  if (int e = launch_status("conv_pack_kernel")) return e;
  if (ksize == 3) {
    if (int e = wino_pack(weight, packed + total, Cout, Cin, as_stream(stream))) return e;
    float* w4 = packed + total + wino_packed_floats(Cout, Cin);
    if (int e = wino4_pack(weight, w4, Cout, Cin, as_stream(stream))) return e;
    return wino4q_pack(weight, w4 + wino4_packed_floats(Cout, Cin), Cout, Cin, as_stream(stream));
  }
  return RPST_OK;
}

// out = mask > 0 ? out : 0 in place (threshold_backward after a kernel without the mask
// epilogue)
__global__ __launch_bounds__(256) void mask_apply_kernel(float* __restrict__ out,
                                                         const float* __restrict__ mask,
                                                         int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 3 < n && ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(mask)) & 15) == 0) {
    float4 v = *reinterpret_cast<float4*>(out + i);
    const float4 m = *reinterpret_cast<const float4*>(mask + i);
    if (!(m.x > 0.f)) v.x = 0.f;
    if (!(m.y > 0.f)) v.y = 0.f;
    if (!(m.z > 0.f)) v.z = 0.f;
    if (!(m.w > 0.f)) v.w = 0.f;
    *reinterpret_cast<float4*>(out + i) = v;
  } else {
    for (int64_t j = i; j < n && j < i + 4; ++j)
      if (!(mask[j] > 0.f)) out[j] = 0.f;
  }
}

static int conv_common(const float* input, const float* aux, const float* aux2,
                       const float* packed_weight,
                       const float* bias, const float* residual, float* out, int N, int Cin,
                       int Hs, int Ws, int Cout, int ksize, int pad_mode, int in_op, int relu,
                       float2* stat_part, int* stat_P, ConvArgs* args_out, hipStream_t st,
                       float* fold_ws = nullptr, int skip_from = 0,
                       const float* in2 = nullptr, int in2_from = 0,
                       const float* mask = nullptr, int pool_out = 0) {
  RPST_REQUIRE(input && packed_weight && out, "conv2d: null pointer");
  RPST_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && Hs > 0 && Ws > 0, "conv2d: bad shape");
  RPST_REQUIRE(ksize == 1 || ksize == 3, "conv2d: ksize must be 1 or 3, got %d", ksize);
  RPST_REQUIRE(pad_mode == RPST_PAD_ZERO || pad_mode == RPST_PAD_REFLECT, "conv2d: bad pad");
  RPST_REQUIRE(in_op >= RPST_IN_NONE && in_op <= RPST_IN_ADD_ADAIN, "conv2d: bad in_op");
  RPST_REQUIRE(relu >= RPST_ACT_NONE && relu <= RPST_ACT_LRELU, "conv2d: bad activation %d", relu);
  RPST_REQUIRE(!(mask && stat_part), "conv2d: the mask epilogue has no statistics");
  RPST_REQUIRE(!(pool_out && (stat_part || mask || residual)),
               "conv2d: the pooled output has no statistics / mask / residual epilogue");
  ConvArgs a{};
  a.mask = mask;
  a.pool_out = pool_out;
  a.skip_from = skip_from;
  a.in = input;
  a.in2 = in2;
  a.in2_from = in2 ? in2_from : 0;
  a.aux = aux;
  a.aux2 = aux2;
  a.wpk = packed_weight;
  a.bias = bias;
  a.res = residual;
  a.out = out;
  a.N = N;
  a.Cin = Cin;
  a.Hs = Hs;
  a.Ws = Ws;
  a.Cout = Cout;
  a.pad = pad_mode;
  a.relu = relu;
  switch (in_op) {
    case RPST_IN_MAXPOOL2:
      a.H = (Hs + 1) / 2;
      a.W = (Ws + 1) / 2;
      break;
    case RPST_IN_UPSAMPLE2:
      a.H = 2 * Hs;
      a.W = 2 * Ws;
      break;
    case RPST_IN_ADD_UPSAMPLE2:
      RPST_REQUIRE(aux != nullptr, "conv2d: ADD_UPSAMPLE2 needs aux");
      RPST_REQUIRE((Hs % 2) == 0 && (Ws % 2) == 0, "conv2d: ADD_UPSAMPLE2 needs even H,W");
      a.H = Hs;
      a.W = Ws;
      break;
    case RPST_IN_ADAIN:
      RPST_REQUIRE(aux != nullptr, "conv2d: ADAIN needs aux (AdaIN statistics)");
      a.H = Hs;
      a.W = Ws;
      break;
    case RPST_IN_ADD_ADAIN:
      RPST_REQUIRE(aux != nullptr && aux2 != nullptr,
                   "conv2d: ADD_ADAIN needs the content feature and AdaIN statistics");
      a.H = Hs;
      a.W = Ws;
      break;
    default:
      a.H = Hs;
      a.W = Ws;
  }
  if (ksize == 3 && pad_mode == RPST_PAD_REFLECT)
    RPST_REQUIRE(a.H >= 2 && a.W >= 2, "conv2d: reflect padding needs H,W >= 2");
  RPST_REQUIRE((int64_t)N * (Cout > Cin ? Cout : Cin) * a.H * a.W < (1LL << 40),
               "conv2d: tensor too large");
  // per-image input (plus one chunk of channel padding) must be addressable by a 31-bit
  // buffer offset
  RPST_REQUIRE(((int64_t)Cin + 16) * Hs * Ws * 4 < (1LL << 31),
               "conv2d: one image's input exceeds 2 GiB");
  int algo = conv_algo(Cout, Cin, Hs, Ws, ksize, in_op);
  if (algo == RPST_CONV_NARROW && !narrow_launchable(N, a.H, Cout, stat_part != nullptr))
    algo = RPST_CONV_DIRECT;
  // the residual epilogue (SANet out_conv, sanet.py:97-98) exists on the direct and narrow
  // kernels only
  if (residual && (algo == RPST_CONV_WINOGRAD || algo == RPST_CONV_WINOGRAD4))
    algo = RPST_CONV_DIRECT;
  RPST_REQUIRE(!pool_out || algo == RPST_CONV_WINOGRAD4,
               "conv2d_pool: the pooled-output epilogue exists on the F(4x4) path only "
               "(rpst_conv2d_algorithm == RPST_CONV_WINOGRAD4)");
  if (algo == RPST_CONV_WINOGRAD4) {
    a.wpk = packed_weight + direct_packed_floats(Cout, Cin, ksize) + wino_packed_floats(Cout, Cin);
    a.stat_part = stat_part;
    int op = in_op;
    // AdaIN in the weights (not with the statistics epilogue: that layer keeps the loader)
    const bool fold = in_op == RPST_IN_ADAIN && fold_ws && !stat_part && a.H >= 2 && a.W >= 2;
    if (fold) op = RPST_IN_NONE;
    // the position-quarter kernel's image follows the F(4x4) one
    if (wino4q_applies(Cin, Cout, op)) a.wpk += wino4_packed_floats(Cout, Cin);
    if (fold) {
      if (int e = wino4_fold(a, packed_weight, pad_cout(Cout), fold_ws, st)) return e;
    }
    if (int e = wino4_launch(a, op, st)) return e;
    if (mask) {  // F(4x4)'s epilogue has no mask: threshold the output in a second pass
      const int64_t n = (int64_t)N * Cout * a.H * a.W;
      mask_apply_kernel<<<(unsigned)((n + 1023) / 1024), 256, 0, st>>>(out, mask, n);
      if (int e = launch_status("mask_apply_kernel")) return e;
    }
    if (stat_P) *stat_P = a.stat_P;
    if (args_out) *args_out = a;
    return RPST_OK;
  }
  if (algo == RPST_CONV_WINOGRAD) {
    a.wpk = packed_weight + direct_packed_floats(Cout, Cin, ksize);
    a.stat_part = stat_part;
    if (int e = wino_launch(a, in_op, st)) return e;
    if (stat_P) *stat_P = a.stat_P;
    if (args_out) *args_out = a;
    return RPST_OK;
  }
  const TileCfg cfg = pick_cfg(Cout);
  const int variant = conv_variant(cfg.BM, ksize, in_op);
  const int th = variant_th(cfg.BM, variant);
  const int ck = ck_of(ksize);
  a.Cout_pad = pad_cout(Cout);
  a.nchunks = (Cin + ck - 1) / ck;
  a.tiles_x = (a.W + kTW - 1) / kTW;
  a.tiles_y = (a.H + th - 1) / th;
  a.co_tiles = a.Cout_pad / cfg.BM;
  const int wn = variant_wn(cfg.BM, variant);
  a.stat_P = a.tiles_x * a.tiles_y * wn;
  a.stat_part = stat_part;
  if (stat_P) *stat_P = a.stat_P;
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * N * a.co_tiles;
  RPST_REQUIRE(blocks <= 0x7fffffffLL, "conv2d: grid too large");
  if (args_out) *args_out = a;
  if (algo == RPST_CONV_NARROW) {
    const int rpt = narrow_rpt(Cout);
    const int nco = Cout <= 4 ? 4 : 16;
    RPST_REQUIRE(Cin * 9 * nco <= kNrWl, "conv2d: narrow weights exceed LDS");
    dim3 grid((unsigned)((a.W + kNrTW - 1) / kNrTW), (unsigned)((a.H + 4 * rpt - 1) / (4 * rpt)), N);
    if (in_op == RPST_IN_ADD_ADAIN) {
      RPST_REQUIRE(Cout <= 4, "conv2d: narrow skip-AdaIN conv needs Cout <= 4");
      if (rpt == 4) conv3x3_narrow_kernel<4, 4, RPST_IN_ADD_ADAIN><<<grid, 256, 0, st>>>(a);
      else conv3x3_narrow_kernel<4, 2, RPST_IN_ADD_ADAIN><<<grid, 256, 0, st>>>(a);
    } else if (Cout <= 4) {
      if (rpt == 4) conv3x3_narrow_kernel<4, 4><<<grid, 256, 0, st>>>(a);
      else conv3x3_narrow_kernel<4, 2><<<grid, 256, 0, st>>>(a);
    } else {
      conv3x3_narrow_kernel<16, 2><<<grid, 256, 0, st>>>(a);
    }
    return launch_status("conv3x3_narrow_kernel");
  }
  if (ksize == 1) {
    RPST_REQUIRE(in_op == RPST_IN_NONE, "conv2d: 1x1 conv supports in_op NONE only");
    launch_conv<1, RPST_IN_NONE>(a, cfg.BM, variant, st);
  } else if (in_op == RPST_IN_MAXPOOL2) {
    launch_conv<3, RPST_IN_MAXPOOL2>(a, cfg.BM, variant, st);
  } else if (in_op == RPST_IN_UPSAMPLE2) {
    launch_conv<3, RPST_IN_UPSAMPLE2>(a, cfg.BM, variant, st);
  } else if (in_op == RPST_IN_ADD_UPSAMPLE2) {
    launch_conv<3, RPST_IN_ADD_UPSAMPLE2>(a, cfg.BM, variant, st);
  } else if (in_op == RPST_IN_ADAIN) {
    launch_conv<3, RPST_IN_ADAIN>(a, cfg.BM, variant, st);
  } else if (in_op == RPST_IN_ADD_ADAIN) {
    launch_conv<3, RPST_IN_ADD_ADAIN>(a, cfg.BM, variant, st);
  } else {
    launch_conv<3, RPST_IN_NONE>(a, cfg.BM, variant, st);
  }
  return launch_status("conv_mfma_kernel");
}

extern "C" int rpst_conv2d(const float* input, const float* aux, const float* packed_weight,
                           const float* bias, const float* residual, float* out, int N,
                           int Cin, int Hs, int Ws, int Cout, int ksize, int pad_mode,
                           int in_op, int relu, rpst_stream_t stream) {
  RPST_REQUIRE(in_op != RPST_IN_ADD_ADAIN, "conv2d: ADD_ADAIN goes through rpst_conv2d_skip_adain");
  return conv_common(input, aux, nullptr, packed_weight, bias, residual, out, N, Cin, Hs, Ws,
                     Cout, ksize, pad_mode, in_op, relu, nullptr, nullptr, nullptr,
                     as_stream(stream));
}

extern "C" int rpst_conv2d_pair(const float* input, const float* input2, int n1,
                                const float* packed_weight, const float* bias, float* out, int N,
                                int Cin, int Hs, int Ws, int Cout, int ksize, int pad_mode,
                                int relu, rpst_stream_t stream) {
  RPST_REQUIRE(n1 > 0 && n1 <= N, "conv2d_pair: need 0 < n1 <= N (n1=%d, N=%d)", n1, N);
  RPST_REQUIRE(n1 == N || input2, "conv2d_pair: null second input");
  return conv_common(input, nullptr, nullptr, packed_weight, bias, nullptr, out, N, Cin, Hs, Ws,
                     Cout, ksize, pad_mode, RPST_IN_NONE, relu, nullptr, nullptr, nullptr,
                     as_stream(stream), nullptr, 0, n1 < N ? input2 : nullptr, n1 < N ? n1 : 0);
}

extern "C" int rpst_conv2d_masked(const float* input, const float* packed_weight,
                                  const float* bias, const float* mask, float* out, int N,
                                  int Cin, int Hs, int Ws, int Cout, int ksize, int pad_mode,
                                  rpst_stream_t stream) {
  RPST_REQUIRE(mask, "conv2d_masked: null mask");
  return conv_common(input, nullptr, nullptr, packed_weight, bias, nullptr, out, N, Cin, Hs, Ws,
                     Cout, ksize, pad_mode, RPST_IN_NONE, RPST_ACT_NONE, nullptr, nullptr,
                     nullptr, as_stream(stream), nullptr, 0, nullptr, 0, mask);
}

extern "C" int rpst_conv2d_pool(const float* input, const float* aux, const float* packed_weight,
                                const float* bias, float* out, int N, int Cin, int Hs, int Ws,
                                int Cout, int ksize, int pad_mode, int in_op, int relu,
                                rpst_stream_t stream) {
  RPST_REQUIRE(in_op != RPST_IN_ADD_ADAIN, "conv2d_pool: ADD_ADAIN has no pooled form");
  return conv_common(input, aux, nullptr, packed_weight, bias, nullptr, out, N, Cin, Hs, Ws,
                     Cout, ksize, pad_mode, in_op, relu, nullptr, nullptr, nullptr,
                     as_stream(stream), nullptr, 0, nullptr, 0, nullptr, 1);
}

// workspace of the F(4x4) conv with RPST_IN_ADAIN folded into per-image weights (0 for
// every other layer)
static size_t fold_bytes(int N, int Cin, int Hs, int Ws, int Cout, int ksize, int in_op) {
  if (N <= 0 || Cin <= 0 || Hs < 2 || Ws < 2 || Cout <= 0 || ksize != 3 || in_op != RPST_IN_ADAIN)
    return 0;
  if (conv_algo(Cout, Cin, Hs, Ws, ksize, in_op) != RPST_CONV_WINOGRAD4) return 0;
  return wino4_fold_floats(N, Cin, Cout) * sizeof(float);
}

extern "C" size_t rpst_conv2d_workspace_size(int N, int Cin, int Hs, int Ws, int Cout, int ksize,
                                             int in_op) {
  return fold_bytes(N, Cin, Hs, Ws, Cout, ksize, in_op);
}

extern "C" int rpst_conv2d_ws(const float* input, const float* aux, const float* packed_weight,
                              const float* bias, const float* residual, float* out, int N,
                              int Cin, int Hs, int Ws, int Cout, int ksize, int pad_mode,
                              int in_op, int relu, void* workspace, size_t workspace_bytes,
                              rpst_stream_t stream) {
  RPST_REQUIRE(in_op != RPST_IN_ADD_ADAIN, "conv2d: ADD_ADAIN goes through rpst_conv2d_skip_adain");
  const size_t need = fold_bytes(N, Cin, Hs, Ws, Cout, ksize, in_op);
  if (need && (!workspace || workspace_bytes < need)) {
    set_error("conv2d: workspace %zu < %zu bytes", workspace_bytes, need);
    return RPST_EWORKSPACE;
  }
  return conv_common(input, aux, nullptr, packed_weight, bias, residual, out, N, Cin, Hs, Ws,
                     Cout, ksize, pad_mode, in_op, relu, nullptr, nullptr, nullptr,
                     as_stream(stream), need ? static_cast<float*>(workspace) : nullptr);
}

// conv(pad(T_n x + c_n)): F(4x4) layers fold T_n / c_n into per-image weights and border
// biases (wino4_mix); other layers materialise z = T x + c (fp32 MFMA GEMM) and convolve it
static bool mix_folds(int Cin, int H, int W, int Cout, int ksize) {
  return ksize == 3 && H >= 2 && W >= 2 &&
         conv_algo(Cout, Cin, H, W, ksize, RPST_IN_NONE) == RPST_CONV_WINOGRAD4;
}

extern "C" size_t rpst_conv2d_mix_workspace_size(int N, int Cin, int H, int W, int Cout,
                                                 int ksize) {
  if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0 || Cout <= 0 || (ksize != 1 && ksize != 3)) return 0;
  if (mix_folds(Cin, H, W, Cout, ksize)) return (wino4_mix_floats(N, Cin, Cout) + 64) * sizeof(float);
  return ((size_t)N * Cin * H * W + wct_apply_scratch_floats(N, Cin) + 64) * sizeof(float);
}

extern "C" int rpst_conv2d_mix(const float* input, const double* T, const double* offset,
                               const float* packed_weight, const float* bias, float* out, int N,
                               int Cin, int H, int W, int Cout, int ksize, int pad_mode,
                               int relu, void* workspace, size_t workspace_bytes,
                               rpst_stream_t stream) {
  RPST_REQUIRE(input && T && offset && packed_weight && out, "conv2d_mix: null pointer");
  RPST_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && H > 0 && W > 0, "conv2d_mix: bad shape");
  const size_t need = rpst_conv2d_mix_workspace_size(N, Cin, H, W, Cout, ksize);
  if (!workspace || workspace_bytes < need) {
    set_error("conv2d_mix: workspace %zu < %zu bytes", workspace_bytes, need);
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* ws = static_cast<float*>(workspace);
  if (!mix_folds(Cin, H, W, Cout, ksize)) {
    float* z = ws;
    if (int e = wct_apply_f32(T, offset, input, z, N, Cin, (int64_t)H * W,
                              z + (size_t)N * Cin * H * W, st))
      return e;
    return conv_common(z, nullptr, nullptr, packed_weight, bias, nullptr, out, N, Cin, H, W, Cout,
                       ksize, pad_mode, RPST_IN_NONE, relu, nullptr, nullptr, nullptr, st);
  }
  // the F(4x4) launch of conv_common with the folded weights: set up the arguments the way
  // conv_common does for a NONE loader, then fold and launch
  RPST_REQUIRE(pad_mode == RPST_PAD_ZERO || pad_mode == RPST_PAD_REFLECT, "conv2d_mix: bad pad");
  RPST_REQUIRE(relu >= RPST_ACT_NONE && relu <= RPST_ACT_LRELU, "conv2d_mix: bad activation");
  RPST_REQUIRE(((int64_t)Cin + 16) * H * W * 4 < (1LL << 31), "conv2d_mix: image too large");
  ConvArgs a{};
  a.in = input;
  a.wpk = packed_weight + direct_packed_floats(Cout, Cin, ksize) + wino_packed_floats(Cout, Cin);
  if (wino4q_applies(Cin, Cout, RPST_IN_NONE)) a.wpk += wino4_packed_floats(Cout, Cin);
  a.bias = bias;
  a.out = out;
  a.N = N;
  a.Cin = Cin;
  a.Hs = a.H = H;
  a.Ws = a.W = W;
  a.Cout = Cout;
  a.pad = pad_mode;
  a.relu = relu;
  if (int e = wino4_mix(a, T, offset, packed_weight, pad_cout(Cout), ws, st)) return e;
  return wino4_launch(a, RPST_IN_NONE, st);
}

extern "C" int rpst_conv2d_skip_adain(const float* stylized, const float* content,
                                      const float* params, const float* packed_weight,
                                      const float* bias, float* out, int N, int Cin, int H, int W,
                                      int Cout, int ksize, int pad_mode, int relu,
                                      rpst_stream_t stream) {
  RPST_REQUIRE(ksize == 3, "conv2d_skip_adain: 3x3 convs only");
  return conv_common(stylized, params, content, packed_weight, bias, nullptr, out, N, Cin, H, W,
                     Cout, ksize, pad_mode, RPST_IN_ADD_ADAIN, relu, nullptr, nullptr, nullptr,
                     as_stream(stream));
}

extern "C" size_t rpst_conv2d_stats_workspace_size(int N, int Cin, int Hs, int Ws, int Cout,
                                                   int ksize, int in_op) {
  if (N <= 0 || Cin <= 0 || Hs <= 0 || Ws <= 0 || Cout <= 0 || (ksize != 1 && ksize != 3)) return 0;
  // the partial count depends on the kernel the thread's precise / quarter settings select:
  // sized for the largest of them, so a workspace sized under one setting serves a launch
  // under any other
  int stat_P = 0;
  {
    const int sp = t_conv_precise, sq = t_conv_quarter;
    for (int p = 0; p < 3; ++p)
      for (int q = -1; q < 3; ++q) {
        t_conv_precise = p;
        t_conv_quarter = q;
        const ConvGeom g = conv_geom(N, Cin, Hs, Ws, Cout, ksize, in_op, true);
        stat_P = g.stat_P > stat_P ? g.stat_P : stat_P;
      }
    t_conv_precise = sp;
    t_conv_quarter = sq;
  }
  const size_t stats = ((size_t)N * Cout * stat_P * sizeof(float2) + 255) / 256 * 256;
  return stats + fold_bytes(N, Cin, Hs, Ws, Cout, ksize, in_op);
}

static int conv2d_stats_impl(const float* input, const float* aux, const float* packed_weight,
                             const float* bias, const float* residual, float* out, int N,
                             int Cin, int Hs, int Ws, int Cout, int ksize, int pad_mode,
                             int in_op, int relu, float* mean, float* std_out, float eps,
                             void* workspace, size_t workspace_bytes, int store_n,
                             rpst_stream_t stream) {
  RPST_REQUIRE(mean && std_out, "conv2d_stats: null statistics pointer");
  RPST_REQUIRE(store_n >= 1 && store_n <= N, "conv2d_stats: store_n=%d outside [1, N=%d]",
               store_n, N);
  const size_t need = rpst_conv2d_stats_workspace_size(N, Cin, Hs, Ws, Cout, ksize, in_op);
  if (!workspace || workspace_bytes < need) {
    set_error("conv2d_stats: workspace %zu < %zu bytes", workspace_bytes, need);
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  ConvArgs a{};
  int P = 0;
  const ConvGeom g = conv_geom(N, Cin, Hs, Ws, Cout, ksize, in_op, true);
  const int planes = N * Cout;
  if (g.algo == RPST_CONV_DIRECT && g.stat_nt < 4) {  // tile without the fused statistics epilogue
    if (int e = conv_common(input, aux, nullptr, packed_weight, bias, residual, out, N, Cin, Hs,
                            Ws, Cout, ksize, pad_mode, in_op, relu, nullptr, &P, &a, st))
      return e;
    return rpst_calc_mean_std(out, mean, std_out, N, Cout, (int64_t)a.H * a.W, eps, stream);
  }
  const size_t fb = fold_bytes(N, Cin, Hs, Ws, Cout, ksize, in_op);
  float* fold_ws = fb ? reinterpret_cast<float*>(static_cast<char*>(workspace) + (need - fb))
                      : nullptr;
  if (int e = conv_common(input, aux, nullptr, packed_weight, bias, residual, out, N, Cin, Hs, Ws,
                          Cout, ksize, pad_mode, in_op, relu, static_cast<float2*>(workspace), &P,
                          &a, st, fold_ws, store_n < N ? store_n : 0))
    return e;
  if (g.stat_t) {
    stat_merge_t_kernel<<<N * ((Cout + 63) / 64), 256, 0, st>>>(
        static_cast<const float2*>(workspace), mean, std_out, Cout, P, a.tiles_x, g.stat_wn,
        g.stat_nt, g.stat_tw, a.H, a.W, eps);
    return launch_status("stat_merge_t_kernel");
  }
  stat_merge_kernel<<<(planes + 3) / 4, 256, 0, st>>>(static_cast<const float2*>(workspace), mean,
                                                      std_out, planes, P, a.tiles_x, g.stat_wn,
                                                      g.stat_nt, g.stat_tw, a.H, a.W, eps);
  return launch_status("stat_merge_kernel");
}

extern "C" int rpst_conv2d_stats(const float* input, const float* aux,
                                 const float* packed_weight, const float* bias,
                                 const float* residual, float* out, int N, int Cin, int Hs,
                                 int Ws, int Cout, int ksize, int pad_mode, int in_op, int relu,
                                 float* mean, float* std_out, float eps, void* workspace,
                                 size_t workspace_bytes, rpst_stream_t stream) {
  return conv2d_stats_impl(input, aux, packed_weight, bias, residual, out, N, Cin, Hs, Ws, Cout,
                           ksize, pad_mode, in_op, relu, mean, std_out, eps, workspace,
                           workspace_bytes, N, stream);
}

extern "C" int rpst_conv2d_stats_store(const float* input, const float* aux,
                                       const float* packed_weight, const float* bias,
                                       const float* residual, float* out, int N, int Cin, int Hs,
                                       int Ws, int Cout, int ksize, int pad_mode, int in_op,
                                       int relu, float* mean, float* std_out, float eps,
                                       int store_n, void* workspace, size_t workspace_bytes,
                                       rpst_stream_t stream) {
  return conv2d_stats_impl(input, aux, packed_weight, bias, residual, out, N, Cin, Hs, Ws, Cout,
                           ksize, pad_mode, in_op, relu, mean, std_out, eps, workspace,
                           workspace_bytes, store_n, stream);
}

// ---- stand-alone max-pool / upsample (used where no conv follows directly) ----------
__global__ void maxpool2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                int64_t planes, int H, int W, int Ho, int Wo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= planes * Ho * Wo) return;
  const int x = (int)(i % Wo);
  const int64_t r = i / Wo;
  const int y = (int)(r % Ho);
  const int64_t p = r / Ho;
  const float* s = in + p * H * W;
  const int sy = 2 * y, sx = 2 * x;
  float v = s[(int64_t)sy * W + sx];
  if (sx + 1 < W) v = fmaxf(v, s[(int64_t)sy * W + sx + 1]);
  if (sy + 1 < H) v = fmaxf(v, s[(int64_t)(sy + 1) * W + sx]);
  if (sx + 1 < W && sy + 1 < H) v = fmaxf(v, s[(int64_t)(sy + 1) * W + sx + 1]);
  out[i] = v;
}

__global__ void upsample2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                 int64_t planes, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int Wo = 2 * W, Ho = 2 * H;
  if (i >= planes * Ho * Wo) return;
  const int x = (int)(i % Wo);
  const int64_t r = i / Wo;
  const int y = (int)(r % Ho);
  const int64_t p = r / Ho;
  out[i] = in[p * H * W + (int64_t)(y >> 1) * W + (x >> 1)];
}

// out = a + upsample_nearest2x(b): a (planes, H, W), b (planes, H/2, W/2) read at
// (y >> 1, x >> 1), the RPST_IN_ADD_UPSAMPLE2 loader's operand, materialised
__global__ void add_upsample2_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                     float* __restrict__ out, int64_t planes, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= planes * H * W) return;
  const int x = (int)(i % W);
  const int64_t r = i / W;
  const int y = (int)(r % H);
  const int64_t p = r / H;
  const int Wb = W >> 1, Hb = H >> 1;
  out[i] = a[i] + b[(p * Hb + (y >> 1)) * Wb + (x >> 1)];
}

extern "C" int rpst_add_upsample_nearest2x(const float* a, const float* b, float* out, int N,
                                           int C, int H, int W, rpst_stream_t stream) {
  RPST_REQUIRE(a && b && out && N > 0 && C > 0 && H >= 2 && W >= 2 && H % 2 == 0 && W % 2 == 0,
               "add_upsample2x: bad args");
  const int64_t total = (int64_t)N * C * H * W;
  add_upsample2_kernel<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(
      a, b, out, (int64_t)N * C, H, W);
  return launch_status("add_upsample2_kernel");
}

extern "C" int rpst_maxpool2x2_ceil(const float* in, float* out, int N, int C, int H, int W,
                                    rpst_stream_t stream) {
  RPST_REQUIRE(in && out && N > 0 && C > 0 && H > 0 && W > 0, "maxpool2x2: bad args");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int64_t total = (int64_t)N * C * Ho * Wo;
  maxpool2_kernel<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(
      in, out, (int64_t)N * C, H, W, Ho, Wo);
  return launch_status("maxpool2_kernel");
}

extern "C" int rpst_upsample_nearest2x(const float* in, float* out, int N, int C, int H,
                                       int W, rpst_stream_t stream) {
  RPST_REQUIRE(in && out && N > 0 && C > 0 && H > 0 && W > 0, "upsample2x: bad args");
  const int64_t total = (int64_t)N * C * 4 * H * W;
  upsample2_kernel<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(
      in, out, (int64_t)N * C, H, W);
  return launch_status("upsample2_kernel");
}
