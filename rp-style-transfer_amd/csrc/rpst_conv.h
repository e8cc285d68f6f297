// Shared pieces of the conv kernels (direct implicit GEMM in rpst_conv.hip, Winograd
// F(2x2,3x3) in rpst_wino.hip): launch arguments, padding resolution, buffer loads and
// the fused input operators of the tile loaders.
#pragma once

#include "rpst_common.h"

namespace rpst {

constexpr int kTW = 32;  // pixels per N sub-tile = one row segment

struct ConvArgs {
  const float* in;
  const float* aux;
  const float* aux2;  // RPST_IN_ADD_ADAIN: the content feature c (N,Cin,H,W)
  const float* wpk;
  const float* bias;
  const float* res;
  float* out;
  int N, Cin, Hs, Ws, H, W, Cout, Cout_pad, nchunks;
  int tiles_x, tiles_y, co_tiles;
  int pad, relu;
  int persist;        // Winograd: one block loops over all co tiles of its spatial tile
  int cosplit;        // F(4x4): co tiles split over this many blocks per spatial tile
  float2* stat_part;  // optional: per-(n, co, wave tile) (mean, M2) of the output
  int stat_P;         // partials per (n, co) = tiles_x * tiles_y * WN
  // F(4x4) with AdaIN folded into per-image weights (wino4_fold): image n's packed weights
  // start at wpk + n * wstride (0: shared); btab = per-(n, co) bias by border class
  // [n][co][3 row classes][3 column classes] replacing `bias` (nullptr: use `bias`)
  int64_t wstride;
  const float* btab;
  // > 0: images n >= skip_from are not written, only their statistics are reduced (the
  // AdaIN-RP encoder's style half, whose feature only feeds calc_mean_std). F(4x4) honours
  // it; the other kernels write everything (still correct)
  int skip_from;
  // > 0: images n >= in2_from are read from in2 + (n - in2_from) * Cin * plane instead of in
  // (rpst_conv2d_pair: an encoder's first conv over [content; style] without the concat)
  const float* in2;
  int in2_from;
  // optional ReLU-backward mask: out = mask > 0 ? v : 0 (rpst_conv2d_masked, the dgrad of a
  // conv whose input is a ReLU output: threshold_backward fused into the epilogue)
  const float* mask;
  // F(4x4) only: out holds max_pool2d(., 2, 2, ceil_mode=True) of the result, planes of
  // ((H + 1) / 2, (W + 1) / 2) (rpst_conv2d_pool: a conv whose output only feeds a pool)
  int pool_out;
};

// image n's input planes (block-uniform n)
__device__ __forceinline__ const float* conv_in_img(const ConvArgs& a, int n, int64_t per) {
  return (a.in2_from > 0 && n >= a.in2_from) ? a.in2 + (int64_t)(n - a.in2_from) * per
                                             : a.in + (int64_t)n * per;
}

template <int KS>
struct ConvK {
  static constexpr int CK = (KS == 3) ? 8 : 16;  // input channels per chunk
  static constexpr int TAPS = KS * KS;
  static constexpr int KCH = TAPS * CK;  // K values per chunk
};

// Resolve a logical (post-in_op) coordinate against padding. Returns false for a zero
// pad position. Tile overhang beyond the image is clamped (its results are discarded).
__device__ __forceinline__ bool resolve(int& v, int n, int pad, bool padded) {
  if (padded) {
    if (pad == RPST_PAD_ZERO) {
      if (v < 0 || v >= n) return false;
    } else {
      v = reflect1(v, n);
    }
  }
  v = v < 0 ? 0 : (v >= n ? n - 1 : v);
  return true;
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// Byte offset the buffer unit treats as out of range (returns 0, no fault): every
// descriptor below has num_records < 2^31.
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// Raw global loads per patch element for each input operator; they are combined into
// the element value only when the chunk is written to LDS (after the current chunk's
// MFMAs), so no wait for the loads sits in front of the compute phase.
template <int INOP>
struct RawN {
  static constexpr int R = INOP == RPST_IN_MAXPOOL2
                               ? 4
                               : ((INOP == RPST_IN_ADD_UPSAMPLE2 || INOP == RPST_IN_ADD_ADAIN) ? 2 : 1);
};

// Second-operand tensor of the two-load input operators (per image), read through the
// `raux` descriptor: ADD_UPSAMPLE2 -> aux (N,Cin,H/2,W/2); ADD_ADAIN -> aux2 (N,Cin,H,W).
template <int INOP>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t aux_rsrc(const ConvArgs& a, int n) {
  if constexpr (INOP == RPST_IN_ADD_ADAIN) {
    const unsigned plane = (unsigned)(a.H * a.W);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(a.aux2 + (int64_t)n * a.Cin * plane),
                                             (short)0, (int)(a.Cin * plane * 4u), 0x00020000);
  } else {
    const unsigned plane = (unsigned)((a.H >> 1) * (a.W >> 1));
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(INOP == RPST_IN_ADD_UPSAMPLE2 ? a.aux + (int64_t)n * a.Cin * plane : a.in),
        (short)0, (int)(a.Cin * plane * 4u), 0x00020000);
  }
}

template <int INOP>
__device__ __forceinline__ unsigned aux_plane_of(const ConvArgs& a) {
  return INOP == RPST_IN_ADD_ADAIN ? (unsigned)(a.H * a.W) : (unsigned)((a.H >> 1) * (a.W >> 1));
}

// epilogue activation: 0 none, 1 ReLU, 2 LeakyReLU(0.2) (torch: x > 0 ? x : x * slope)
__device__ __forceinline__ float activate(float v, int act) {
  if (act == RPST_ACT_RELU) return fmaxf(v, 0.f);
  if (act == RPST_ACT_LRELU) return v > 0.f ? v : v * 0.2f;
  return v;
}

// Issue the loads of one element: logical (post-in_op) resolved row yr / column xr of the
// plane at byte offset `pbyte` (image-relative). ok == false -> zero (pad position /
// padded channel): every load goes out of range and returns 0.
template <int INOP>
__device__ __forceinline__ void fetch_raw(float (&r)[RawN<INOP>::R], __amdgpu_buffer_rsrc_t rin,
                                          __amdgpu_buffer_rsrc_t raux, unsigned pbyte,
                                          unsigned abyte, int yr, int xr, bool ok,
                                          const ConvArgs& a) {
  if constexpr (INOP == RPST_IN_MAXPOOL2) {
    // 2x2 window of the source; missing right/bottom neighbours (ceil mode) re-read the
    // top-left element so the max is unaffected
    const int sy = 2 * yr, sx = 2 * xr;
    const unsigned o = pbyte + (unsigned)(sy * a.Ws + sx) * 4u;
    const unsigned dx = sx + 1 < a.Ws ? 4u : 0u, dy = sy + 1 < a.Hs ? 4u * a.Ws : 0u;
    r[0] = bload(rin, ok ? o : kOOB);
    r[1] = bload(rin, ok ? o + dx : kOOB);
    r[2] = bload(rin, ok ? o + dy : kOOB);
    r[3] = bload(rin, ok ? o + dx + dy : kOOB);
  } else if constexpr (INOP == RPST_IN_UPSAMPLE2) {
    r[0] = bload(rin, ok ? pbyte + (unsigned)((yr >> 1) * a.Ws + (xr >> 1)) * 4u : kOOB);
  } else if constexpr (INOP == RPST_IN_ADD_UPSAMPLE2) {
    r[0] = bload(rin, ok ? pbyte + (unsigned)(yr * a.W + xr) * 4u : kOOB);
    r[1] = bload(raux, ok ? abyte + (unsigned)((yr >> 1) * (a.W >> 1) + (xr >> 1)) * 4u : kOOB);
  } else if constexpr (INOP == RPST_IN_ADD_ADAIN) {
    r[0] = bload(rin, ok ? pbyte + (unsigned)(yr * a.W + xr) * 4u : kOOB);
    r[1] = bload(raux, ok ? abyte + (unsigned)(yr * a.W + xr) * 4u : kOOB);
  } else {  // RPST_IN_NONE and RPST_IN_ADAIN
    r[0] = bload(rin, ok ? pbyte + (unsigned)(yr * a.W + xr) * 4u : kOOB);
  }
}

// AdaIN on load (RPST_IN_ADAIN): ((v - mean_c) / std_c) * std_s + mean_s per (n, ci),
// evaluated as fma(v - mean_c, std_s / std_c, mean_s). aux = [mean_c|mean_s|std_c|std_s],
// each N*Cin floats.
struct AdainP {
  float mc, scale, ms;
};
__device__ __forceinline__ AdainP adain_params(const float* __restrict__ aux, int n, int ci,
                                               const ConvArgs& a) {
  const int64_t nc = (int64_t)a.N * a.Cin;
  const int64_t i = (int64_t)n * a.Cin + (ci < a.Cin ? ci : 0);
  return {aux[i], aux[3 * nc + i] / aux[2 * nc + i], aux[nc + i]};
}

template <int INOP>
__device__ __forceinline__ float combine(const float (&r)[RawN<INOP>::R], bool ok,
                                         const AdainP& p) {
  if constexpr (INOP == RPST_IN_MAXPOOL2) return fmaxf(fmaxf(r[0], r[1]), fmaxf(r[2], r[3]));
  else if constexpr (INOP == RPST_IN_ADD_UPSAMPLE2) return r[0] + r[1];
  else if constexpr (INOP == RPST_IN_ADAIN) return ok ? fmaf(r[0] - p.mc, p.scale, p.ms) : 0.f;
  else if constexpr (INOP == RPST_IN_ADD_ADAIN)
    return ok ? r[0] + fmaf(r[1] - p.mc, p.scale, p.ms) : 0.f;
  else return r[0];
}

// Sum each of v[0..15] over the 32 lanes of a half-wave. Returns the total of element
// e = (j >> 1) & 15 (lanes 2e and 2e+1 of the half hold it); 16 shuffles instead of 80.
__device__ __forceinline__ float halfwave_reduce_scatter16(float (&v)[16], int j) {
  float w[8], u[4], t[2];
  bool b = (j & 16) != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = (b ? v[i + 8] : v[i]) + __shfl_xor(b ? v[i] : v[i + 8], 16, 64);
  b = (j & 8) != 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = (b ? w[i + 4] : w[i]) + __shfl_xor(b ? w[i] : w[i + 4], 8, 64);
  b = (j & 4) != 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) t[i] = (b ? u[i + 2] : u[i]) + __shfl_xor(b ? u[i] : u[i + 2], 4, 64);
  b = (j & 2) != 0;
  float s = (b ? t[1] : t[0]) + __shfl_xor(b ? t[0] : t[1], 2, 64);
  return s + __shfl_xor(s, 1, 64);
}

// Bijective XCD-aware remap of a block index (cdna_hip_programming.md T1): blocks
// b, b+8, b+16, ... share an XCD (and its L2) under the observed round-robin dispatch, so
// give each such group a contiguous range of logical ids. Speed only, never correctness.
__device__ __forceinline__ int xcd_swizzle(int b, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// Sum each of v[0..V-1] (V a power of two <= 16) over the 32 lanes of a half-wave.
// Returns the total of element e = (j >> (5 - log2 V)) & (V - 1) (the lanes of one group
// of 32/V hold it).
template <int V>
__device__ __forceinline__ float halfwave_reduce_scatter(float (&v)[V], int j) {
  static_assert(V >= 1 && V <= 16 && (V & (V - 1)) == 0, "power of two <= 16");
  float w[V];
#pragma unroll
  for (int i = 0; i < V; ++i) w[i] = v[i];
  int n = V, bit = 16;
#pragma unroll
  for (; n > 1; n >>= 1, bit >>= 1) {
    const bool b = (j & bit) != 0;
#pragma unroll
    for (int i = 0; i < n / 2; ++i)
      w[i] = (b ? w[i + n / 2] : w[i]) + __shfl_xor(b ? w[i] : w[i + n / 2], bit, 64);
  }
  float s = w[0];
#pragma unroll
  for (; bit > 0; bit >>= 1) s += __shfl_xor(s, bit, 64);
  return s;
}

// Sum each of v[0..7] over the 32 lanes of a half-wave. Returns the total of element
// e = (j >> 2) & 7 (lanes 4e..4e+3 of the half hold it).
__device__ __forceinline__ float halfwave_reduce_scatter8(float (&v)[8], int j) {
  float u[4], t[2];
  bool b = (j & 16) != 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = (b ? v[i + 4] : v[i]) + __shfl_xor(b ? v[i] : v[i + 4], 16, 64);
  b = (j & 8) != 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) t[i] = (b ? u[i + 2] : u[i]) + __shfl_xor(b ? u[i] : u[i + 2], 8, 64);
  b = (j & 4) != 0;
  float s = (b ? t[1] : t[0]) + __shfl_xor(b ? t[0] : t[1], 4, 64);
  s += __shfl_xor(s, 2, 64);
  return s + __shfl_xor(s, 1, 64);
}

// ---- Winograd F(2x2,3x3) path (rpst_wino.hip) ----------------------------------------
constexpr int kWinoNTH = 256;  // threads per block
// tile shape in use: output channels (BM) x rows (TH, x kTW columns) per block
int wino_bm();
int wino_th();
int wino_persist(int in_op, int64_t spatial_blocks);  // 1: grid over spatial tiles only, each block loops over co tiles
// floats of the Winograd weight image (stored after the direct image for 3x3 convs)
size_t wino_packed_floats(int Cout, int Cin);
int wino_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st);
// a: shape/operator fields filled in, a.wpk = the Winograd weight image. Sets the tiling
// fields (Cout_pad, nchunks, tiles_*, co_tiles, stat_P) and launches.
int wino_launch(ConvArgs& a, int in_op, hipStream_t st);

// ---- Winograd F(4x4,3x3) path (rpst_wino4.hip) ----------------------------------------
// 16 x 64 outputs x 32 channels per 512-thread block; statistics partials per tile row
// of 4 rows x 64 columns.
constexpr int kW4Rows = 16, kW4Cols = 64, kW4Co = 32;
bool wino4_supports(int in_op);
bool wino4_fits(int N, int Cin, int Hs, int Ws, int in_op);
int wino4_persist();
// tile rows per F(4x4) block: 4 (16 output rows) or 2 (the position-quarter kernel, or the
// small layers' 2-row block); statistics partials are per tile row either way
int wino4_rows(int Cin, int Cout, int in_op);
size_t wino4_packed_floats(int Cout, int Cin);
int wino4_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st);
int wino4_launch(ConvArgs& a, int in_op, hipStream_t st);
size_t wino4_fold_floats(int N, int Cin, int Cout);
int wino4_fold(ConvArgs& a, const float* direct_packed, int direct_cout_pad, float* ws,
               hipStream_t st);
size_t wino4_mix_floats(int N, int Cin, int Cout);
int wino4_mix(ConvArgs& a, const double* T, const double* cvec, const float* direct_packed,
              int direct_cout_pad, float* ws, hipStream_t st);

// ---- F(4x4,3x3), position-quarter form (rpst_wino4q.hip) ------------------------------
// 8 x 64 outputs x 64 channels per 512-thread block, each wave 9 of the 36 positions. Its
// weight image follows the F(4x4) one in the packed buffer; wino4_launch / wino4_fold /
// wino4_mix dispatch to it for the layers wino4q_applies to.
bool wino4q_applies(int Cin, int Cout, int in_op);
// false while the calling thread is at precise level 2 (rpst_conv.hip)
bool conv_quarter_allowed();
// 0 off / 1 default rule / 2 forced: the calling thread's rpst_conv2d_set_quarter, else the
// RPST_W4Q environment variable, read per call (rpst_conv.hip)
int conv_quarter_mode();
size_t wino4q_packed_floats(int Cout, int Cin);
int wino4q_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st);
int wino4q_pack_mix(const double* wm, float* pk, int N, int Cout, int Cin, hipStream_t st);
int wino4q_fold_w(const float* pk, float* out, const float* aux, int N, int Cout, int Cin,
                  hipStream_t st);
int wino4q_launch(ConvArgs& a, int in_op, hipStream_t st);
// floats of the F(4x4) weight image a layer launches with (per image when folded)
inline size_t wino4_image_floats(int Cout, int Cin, int in_op) {
  return wino4q_applies(Cin, Cout, in_op) ? wino4q_packed_floats(Cout, Cin)
                                          : wino4_packed_floats(Cout, Cin);
}
// the larger of the two images: workspace sizes use it, so a workspace sized under one
// precise / quarter setting stays large enough for a launch under another (with Cout % 64
// in 1..32 the quarter image is the larger one)
inline size_t wino4_image_floats_max(int Cout, int Cin) {
  const size_t q = wino4q_packed_floats(Cout, Cin), p = wino4_packed_floats(Cout, Cin);
  return q > p ? q : p;
}


}  // namespace rpst
