// Winograd F(2x2, 3x3) convolution on fp32 MFMA (gfx950) for the 3x3 conv stacks of
// the reference hot path (network/base.py:25-111,363-396; sanet.py:162-192) — the same
// layers and fused loader operators as conv_mfma_kernel (rpst_conv.hip), with 16 instead
// of 36 multiplies per 2x2 output tile (Lavin & Gray, "Fast Algorithms for
// Convolutional Neural Networks", 2016):
//
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A     g: 3x3 filter, d: 4x4 input tile (stride 2)
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]   G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   A^T = [1 1 1 0; 0 1 -1 -1]
//
// All arithmetic is fp32 (true fp32 MFMA, no reduced-precision inputs); the transforms
// use the coefficients 0, +-1, +-1/2 only, so the result differs from the direct
// convolution by rounding only (tests/test_gpu_kernels.py states the tolerance).
//
// Block = 4 waves; for each of the 16 positions xi = (i, jj) of the transformed domain it
// computes the GEMM  M_xi[co][tile] = sum_ci U_xi[co][ci] V_xi[ci][tile]  over a tile of
// BM = 32*MT output channels x 32*NT Winograd tiles (TH = 4*NT output rows x 32 columns),
// MT * NT = 2. Wave w owns the transform row i = w: 4 positions x MT x NT = 8 accumulators
// of 32x32, so
//   * U = G g G^T is pre-transformed and pre-shuffled at pack time into exactly the
//     per-lane MFMA A-operand order: a lane loads its 16*MT weights of a chunk with
//     contiguous 16-B loads straight into registers (no LDS round trip), refilled pair by
//     pair as the MFMAs consume them;
//   * V = B^T d B is computed by every wave in registers from the LDS input patch, for
//     its own row i only (row i of B^T touches two input rows), in the MFMA B-operand
//     layout: lane (h, j) builds the 4 values of channel 2cp+h for tiles j (+32);
//   * the output transform's column half (M A) is done in registers; the row half (A^T)
//     needs all four rows, exchanged once through LDS at the end.
// Each weight register feeds NT MFMAs and each V value MT: MT = 1 / NT = 2 halves the
// weight traffic (the dominant load stream) at the cost of more patch rows per block.
// One barrier per K chunk of 8 channels protects the double-buffered patch, which is
// prefetched two chunks ahead (its loads come from HBM).
#include "rpst_conv.h"

#include <cstdlib>

namespace rpst {

constexpr int kWCK = 8;  // input channels per chunk (packing and kernel)

// ---- weight transform + packing -------------------------------------------------------
// image MT: packed[(((ct * nch + c) * 4 + i) * 64 + lane) * 16MT + (cp * 4 + jj) * MT + mt]
//   = U_(i,jj)[co = ct*32MT + mt*32 + (lane & 31)][ci = c*8 + 2*cp + (lane >> 5)]
// with U = G g G^T evaluated in fp64 and rounded once to fp32.
template <int MT>
__global__ void wino_pack_kernel(const float* __restrict__ w, float* __restrict__ pk, int Cout,
                                 int Cin, int nch, int64_t total) {
  constexpr int LANEW = 16 * MT;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int idx = (int)(t % LANEW);
  int64_t r = t / LANEW;
  const int lane = (int)(r & 63);
  r >>= 6;
  const int i = (int)(r & 3);
  r >>= 2;
  const int c = (int)(r % nch);
  const int ct = (int)(r / nch);
  const int mt = idx % MT, jj = (idx / MT) & 3, cp = idx / (4 * MT);
  const int co = ct * 32 * MT + mt * 32 + (lane & 31);
  const int ci = c * kWCK + 2 * cp + (lane >> 5);
  float v = 0.f;
  if (co < Cout && ci < Cin) {
    const double G[4][3] = {{1, 0, 0}, {.5, .5, .5}, {.5, -.5, .5}, {0, 0, 1}};
    const float* g = w + ((int64_t)co * Cin + ci) * 9;
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int q = 0; q < 3; ++q) s += G[i][u] * (double)g[u * 3 + q] * G[jj][q];
    v = (float)s;
  }
  pk[t] = v;
}

static size_t wino_image_floats(int MT, int Cout, int Cin) {
  const size_t bm = 32 * (size_t)MT;
  const size_t co_tiles = (Cout + bm - 1) / bm;
  const size_t nch = (size_t)(Cin + kWCK - 1) / kWCK;
  return co_tiles * nch * 4 * 64 * 16 * MT;
}

// Tile shape: MT = 1 (32 co x 64 tiles per block) measured faster than MT = 2 (64 co x 32
// tiles) on every layer of the three models (profiles/r01_bench_conv_wino.log), so only
// its weight image is packed. Persistence over the co tiles pays for the one-load
// loaders; the two- and four-load loaders keep one co tile per block (their extra
// raw registers would spill across the co-tile loop).
constexpr int kWMT = 1;
int wino_bm() { return 32 * kWMT; }
int wino_th() { return 4 * (2 / kWMT); }
// spatial_blocks = tiles_x * tiles_y * N: a persistent grid of fewer than 512 blocks (two
// per CU) leaves CUs idle (the 64x64 relu4_1 / relu5_1 layers of SAModel training at B = 8:
// 128 blocks), so such layers take one co tile per block
int wino_persist(int in_op, int64_t spatial_blocks) {
  const char* e = getenv("RPST_WINO_PERSIST");  // A/B switch for the one-load loaders
  if (in_op == RPST_IN_MAXPOOL2 || in_op == RPST_IN_ADD_UPSAMPLE2 || in_op == RPST_IN_ADD_ADAIN)
    return 0;
  return (e && *e) ? atoi(e) != 0 : spatial_blocks >= 512;
}

size_t wino_packed_floats(int Cout, int Cin) { return wino_image_floats(kWMT, Cout, Cin); }

int wino_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st) {
  const int nch = (Cin + kWCK - 1) / kWCK;
  const int64_t t = (int64_t)wino_image_floats(kWMT, Cout, Cin);
  wino_pack_kernel<kWMT><<<(unsigned)((t + 255) / 256), 256, 0, st>>>(w, pk, Cout, Cin, nch, t);
  return launch_status("wino_pack_kernel");
}

// ---- the kernel -------------------------------------------------------------------------
// DBG (timing experiments only, tools/wino_dbg.sh; results are wrong): bit0 no global
// loads in the loop, bit1 no LDS reads, bit2 no barrier, bit3 no patch stores, bit4 no
// weight loads, bit5 no patch loads; 256 = the production kernel through that switch.
template <int INOP, int MT, bool PERSIST, int DBG = 0>
__global__ __launch_bounds__(kWinoNTH, 2) void wino_mfma_kernel(ConvArgs a) {
  constexpr int NT = 2 / MT;
  constexpr int BM = 32 * MT, TH = 4 * NT;
  constexpr int CK = kWCK, PH = TH + 2, PW = kTW + 2;
  constexpr int LANEW = 16 * MT;            // weights per lane per chunk
  constexpr int R = RawN<INOP>::R;
  constexpr int XN = PH + 1;                // patch rows + 1 halo element per lane
  constexpr int XS = CK * PH * PW;          // one patch buffer
  constexpr int PS = 4 * 2 * 2 * 16 * 64;   // output exchange (i, c, mt*NT+nt, r, lane)
  constexpr int SMEM = 2 * XS > PS ? 2 * XS : PS;
  static_assert(MT * NT == 2, "8 accumulators per wave");
  static_assert(kWinoNTH == 32 * CK, "one 32-lane loader group per channel of a chunk");
  static_assert(2 * PH <= 32, "one halo element per lane");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];

  // block -> (column tile, row tile, image), XCD-swizzled so neighbouring spatial tiles
  // (which share halo rows) run on one XCD; all co tiles of a spatial tile are computed by
  // the same block (a.persist) or by consecutive blocks of one XCD, so the input patch is
  // read from HBM once and the layer's weights (a few MB) stay in every XCD's L2.
  int bid = xcd_swizzle(blockIdx.x, (int)gridDim.x), ct0 = 0;
  if (!PERSIST) {
    ct0 = bid % a.co_tiles;
    bid /= a.co_tiles;
  }
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  bid /= a.tiles_y;
  const int n = bid;
  const int ct_end = PERSIST ? a.co_tiles : ct0 + 1;
  const int y0 = ty * TH, x0 = tx * kTW;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;

  const bool pooled = (INOP == RPST_IN_MAXPOOL2 || INOP == RPST_IN_UPSAMPLE2);
  const unsigned in_plane = pooled ? (unsigned)(a.Hs * a.Ws) : (unsigned)(a.H * a.W);
  const unsigned aux_plane = aux_plane_of<INOP>(a);
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)conv_in_img(a, n, (int64_t)a.Cin * in_plane), (short)0, (int)(a.Cin * in_plane * 4u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t raux = aux_rsrc<INOP>(a, n);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wpk, (short)0, 0x7fffffff, 0x00020000);
  const unsigned w_off = (unsigned)((wave * 64 + lane) * LANEW) * 4u;
  constexpr unsigned w_chunk = 4u * 64 * LANEW * 4;
  // K chunks per co tile, padded to even (the two patch register sets / LDS buffers
  // alternate with the chunk parity; a padding chunk reads zero input)
  const int nch = a.nchunks, ncp = nch + (nch & 1);

  // patch loader: thread -> (channel cg = tid>>5, column jc); one halo element per lane
  const int cg = tid >> 5, jc = tid & 31;
  int bx = x0 + jc;
  const bool bx_ok = resolve(bx, a.W, a.pad, true);
  const bool has_halo = jc < 2 * PH;
  int hy = y0 - 1 + (jc >> 1);
  int hx = (jc & 1) ? x0 + kTW : x0 - 1;
  const bool hy_ok = resolve(hy, a.H, a.pad, true);
  const bool hx_ok = resolve(hx, a.W, a.pad, true);
  const bool h_ok = has_halo && hy_ok && hx_ok;

  floatx16 acc[4][MT][NT];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][mt][nt][r] = 0.f;

  u32x4 wr[LANEW / 4];
  // raw patch loads: prefetch distance PD = 2 chunks (sets xA / xB for even / odd
  // chunks), 1 for the 4-load max-pool loader (two sets of it do not fit in registers)
  constexpr int PD = R <= 2 ? 2 : 1;
  float xA[XN][R], xB[PD == 2 ? XN : 1][R];
  AdainP apA, apB;

  // weights of (co tile ct, chunk c); out of range (zeros) past the end / in padding
#define RPST_WINO_WLOAD(ct, c, q)                                                           \
  wr[q] = __builtin_amdgcn_raw_buffer_load_b128(                                            \
      rw,                                                                                   \
      (int)((ct) < ct_end && (c) < nch                                                      \
                ? w_off + (unsigned)((ct) * nch + (c)) * w_chunk + 16u * (q)                \
                : kOOB),                                                                    \
      0, 0);

// (branch-free: past the last chunk every load goes out of range and returns 0, so the
// waitcnt the compiler derives after the loads does not merge a path without them)
#define RPST_WINO_LOAD(c, live, X, AP)                                                      \
  {                                                                                         \
    const unsigned ch = (unsigned)((c) * CK + cg);                                          \
    const unsigned pb = ch * in_plane * 4u, ab = ch * aux_plane * 4u;                       \
    if (INOP == RPST_IN_ADAIN || INOP == RPST_IN_ADD_ADAIN)                                 \
      AP = adain_params(a.aux, n, (int)ch, a);                                              \
    _Pragma("unroll") for (int py = 0; py < PH; ++py) {                                     \
      int y = y0 - 1 + py;                                                                  \
      const bool yok = resolve(y, a.H, a.pad, true);                                        \
      fetch_raw<INOP>(X[py], rin, raux, pb, ab, y, bx, live && yok && bx_ok, a);            \
    }                                                                                       \
    fetch_raw<INOP>(X[PH], rin, raux, pb, ab, hy, hx, live && h_ok, a);                     \
  }

  // write chunk c's raw patch (loaded PD chunks earlier) into patch buffer c&1
#define RPST_WINO_STORE(c, X, AP)                                                           \
  {                                                                                         \
    float* xs = smem + ((c) & 1) * XS + cg * PH * PW;                                       \
    const bool chok = (int)((c) * CK + cg) < a.Cin;                                         \
    _Pragma("unroll") for (int py = 0; py < PH; ++py) {                                     \
      bool ok = chok && bx_ok;                                                              \
      if (INOP == RPST_IN_ADAIN || INOP == RPST_IN_ADD_ADAIN) {                             \
        int y = y0 - 1 + py;                                                                \
        ok = ok && resolve(y, a.H, a.pad, true);                                            \
      }                                                                                     \
      xs[py * PW + jc + 1] = combine<INOP>(X[py], ok, AP);                                  \
    }                                                                                       \
    const float hv = combine<INOP>(X[PH], chok && h_ok, AP);                                \
    if (has_halo) xs[(jc >> 1) * PW + ((jc & 1) ? PW - 1 : 0)] = hv;                        \
  }

  // the two input rows (ra, rb) of channel pair cp for this lane's NT tiles
#define RPST_WINO_READ(c, cp, D)                                                            \
  if (!(DBG & 2)) {                                                                         \
    const float* xs = smem + ((c) & 1) * XS + xoff + 2 * (cp) * PH * PW;                    \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                     \
      D[nt][0] = *reinterpret_cast<const float2*>(xs + (4 * nt + ra) * PW);                 \
      D[nt][1] = *reinterpret_cast<const float2*>(xs + (4 * nt + ra) * PW + 2);             \
      D[nt][2] = *reinterpret_cast<const float2*>(xs + (4 * nt + rb) * PW);                 \
      D[nt][3] = *reinterpret_cast<const float2*>(xs + (4 * nt + rb) * PW + 2);             \
    }                                                                                       \
  }

  // V (this wave's transform row) of channel pair cp from D; the next pair's LDS reads
  // are issued into DN before the 8 MFMAs of pair cp; then the weight quads of pair cp
  // are refilled with chunk c+1's values
#define RPST_WINO_CP(c, cp, D, DN, wct, wc)                                                 \
  {                                                                                         \
    float v[NT][4];                                                                         \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                     \
      const float t0 = fmaf(sg, D[nt][2].x, D[nt][0].x);                                    \
      const float t1 = fmaf(sg, D[nt][2].y, D[nt][0].y);                                    \
      const float t2 = fmaf(sg, D[nt][3].x, D[nt][1].x);                                    \
      const float t3 = fmaf(sg, D[nt][3].y, D[nt][1].y);                                    \
      v[nt][0] = t0 - t2;                                                                   \
      v[nt][1] = t1 + t2;                                                                   \
      v[nt][2] = t2 - t1;                                                                   \
      v[nt][3] = t1 - t3;                                                                   \
    }                                                                                       \
    if ((cp) + 1 < CK / 2) RPST_WINO_READ(c, (cp) + 1, DN)                                  \
    __builtin_amdgcn_sched_barrier(0); /* issue the next pair's reads before the MFMAs */   \
    _Pragma("unroll") for (int jj = 0; jj < 4; ++jj)                                        \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                   \
        const int idx = ((cp) * 4 + jj) * MT + mt;                                          \
        const float u = __uint_as_float(wr[idx >> 2][idx & 3]);                             \
        _Pragma("unroll") for (int nt = 0; nt < NT; ++nt)                                   \
          acc[jj][mt][nt] =                                                                 \
              __builtin_amdgcn_mfma_f32_32x32x2f32(u, v[nt][jj], acc[jj][mt][nt], 0, 0, 0); \
      }                                                                                     \
    if (!(DBG & 17)) {                                                                      \
      _Pragma("unroll") for (int q = (cp) * MT; q < ((cp) + 1) * MT; ++q)                   \
        RPST_WINO_WLOAD(wct, wc, q)                                                         \
      __builtin_amdgcn_sched_barrier(0);                                                    \
    }                                                                                       \
  }

  // one K chunk (ct, c): patch c to LDS, barrier, patch loads PD chunks ahead (wrapping
  // into the next co tile, whose input is the same), MFMAs of chunk c with the weight
  // refill for the next chunk
#define RPST_WINO_CHUNK(ct, c, X, AP)                                                       \
  {                                                                                         \
    if (!(DBG & 8)) RPST_WINO_STORE(c, X, AP)                                               \
    if (!(DBG & 4)) __syncthreads();                                                        \
    const bool pwrap = (c) + PD >= ncp;                                                     \
    const int pc = pwrap ? (c) + PD - ncp : (c) + PD;                                       \
    if (!(DBG & 33)) RPST_WINO_LOAD(pc, (pwrap ? (ct) + 1 : (ct)) < ct_end, X, AP)           \
    const bool wwrap = (c) + 1 >= ncp;                                                      \
    const int wct = wwrap ? (ct) + 1 : (ct), wc = wwrap ? 0 : (c) + 1;                      \
    float2 d0[NT][4], d1[NT][4];                                                            \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt)                                       \
      _Pragma("unroll") for (int k = 0; k < 4; ++k) d0[nt][k] = d1[nt][k] = make_float2(1.f, 2.f); \
    RPST_WINO_READ(c, 0, d0)                                                                \
    RPST_WINO_CP(c, 0, d0, d1, wct, wc)                                                     \
    RPST_WINO_CP(c, 1, d1, d0, wct, wc)                                                     \
    RPST_WINO_CP(c, 2, d0, d1, wct, wc)                                                     \
    RPST_WINO_CP(c, 3, d1, d0, wct, wc)                                                     \
  }

  // transform row i = wave of B^T: t = d[ra] + sg * d[rb]
  const int ra = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int rb = wave == 0 ? 2 : (wave == 1 ? 2 : (wave == 2 ? 1 : 3));
  const float sg = wave == 1 ? 1.f : -1.f;
  const int xoff = h * PH * PW + 2 * (j >> 4) * PW + 2 * (j & 15);

#pragma unroll
  for (int q = 0; q < LANEW / 4; ++q) RPST_WINO_WLOAD(ct0, 0, q)
  RPST_WINO_LOAD(0, true, xA, apA)
  if constexpr (PD == 2) RPST_WINO_LOAD(1, true, xB, apB)
  // persistent over the co tiles of this spatial tile (a.persist): the input patch is the
  // same for each, so the next co tile's first chunks are prefetched during this one's
  // last, and only the first co tile waits on a cold pipeline
  // (a constant single iteration without PERSIST: nothing stays live across the epilogue)
  for (int it = 0; it < (PERSIST ? a.co_tiles : 1); ++it) {
  const int ct = ct0 + it;
  for (int c = 0; c < ncp; c += 2) {
    RPST_WINO_CHUNK(ct, c, xA, apA)
    if constexpr (PD == 2) {
      RPST_WINO_CHUNK(ct, c + 1, xB, apB)
    } else {
      RPST_WINO_CHUNK(ct, c + 1, xA, apA)
    }
  }
  const int co0 = ct * BM;
#undef RPST_WINO_CHUNK
#undef RPST_WINO_CP
#undef RPST_WINO_READ
#undef RPST_WINO_STORE
#undef RPST_WINO_LOAD
#undef RPST_WINO_WLOAD

  // ---- output transform ---------------------------------------------------------------
  // column half in registers: P[i][0] = M0 + M1 + M2, P[i][1] = M1 - M2 - M3 (i = wave)
  __syncthreads();  // every wave is done with the patch buffers
  float* Ps = smem;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int mt = s / NT, nt = s % NT;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float m0 = acc[0][mt][nt][r], m1 = acc[1][mt][nt][r];
      const float m2 = acc[2][mt][nt][r], m3 = acc[3][mt][nt][r];
      Ps[(((wave * 2 + 0) * 2 + s) * 16 + r) * 64 + lane] = (m0 + m1) + m2;
      Ps[(((wave * 2 + 1) * 2 + s) * 16 + r) * 64 + lane] = (m1 - m2) - m3;
    }
  }
  __syncthreads();

  // row half: wave w finishes accumulator rows r = 4w..4w+3 of both sub-tiles s
  const int gx = x0 + 2 * (j & 15);
  const bool vx0 = gx < a.W, vx1 = gx + 1 < a.W;
  const bool vec = vx1 && (a.W & 1) == 0;
  float yv[2][4][4];  // [s][q][output 2x2], zero outside the image
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int mt = s / NT, nt = s % NT;
    const int gy = y0 + 4 * nt + 2 * (j >> 4);
    const bool vy0 = gy < a.H, vy1 = gy + 1 < a.H;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * wave + q;
      float P[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) P[i][cc] = Ps[(((i * 2 + cc) * 2 + s) * 16 + r) * 64 + lane];
      float y[4] = {(P[0][0] + P[1][0]) + P[2][0], (P[0][1] + P[1][1]) + P[2][1],
                    (P[1][0] - P[2][0]) - P[3][0], (P[1][1] - P[2][1]) - P[3][1]};
      const int co = co0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co < a.Cout) {
        const float b = a.bias ? a.bias[co] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[e] += b;
          y[e] = activate(y[e], a.relu);
        }
        const int64_t off = (((int64_t)n * a.Cout + co) * a.H + gy) * a.W + gx;
        float* o = a.out + off;
        if (a.mask) {
          const float* mk = a.mask + off;
          if (vy0 && vx0 && !(mk[0] > 0.f)) y[0] = 0.f;
          if (vy0 && vx1 && !(mk[1] > 0.f)) y[1] = 0.f;
          if (vy1 && vx0 && !(mk[a.W] > 0.f)) y[2] = 0.f;
          if (vy1 && vx1 && !(mk[a.W + 1] > 0.f)) y[3] = 0.f;
        }
        if (vec) {
          if (vy0) *reinterpret_cast<float2*>(o) = make_float2(y[0], y[1]);
          if (vy1) *reinterpret_cast<float2*>(o + a.W) = make_float2(y[2], y[3]);
        } else {
          if (vy0 && vx0) o[0] = y[0];
          if (vy0 && vx1) o[1] = y[1];
          if (vy1 && vx0) o[a.W] = y[2];
          if (vy1 && vx1) o[a.W + 1] = y[3];
        }
      }
      yv[s][q][0] = (vy0 && vx0) ? y[0] : 0.f;
      yv[s][q][1] = (vy0 && vx1) ? y[1] : 0.f;
      yv[s][q][2] = (vy1 && vx0) ? y[2] : 0.f;
      yv[s][q][3] = (vy1 && vx1) ? y[3] : 0.f;
    }
  }

  // optional output statistics, as conv_mfma_kernel: per (channel, block) (mean, M2) of
  // the written values; one partial per block (stat_P = tiles_x * tiles_y). A lane holds
  // MT*4 channels (mt, q), each over NT tiles x 4 outputs.
  if (a.stat_part) {
    constexpr int V = 4 * MT, SH = MT == 2 ? 2 : 3;  // channels per lane; lane group shift
    const int rows = max(0, min(TH, a.H - y0)), cols = max(0, min(kTW, a.W - x0));
    const int cnt = rows * cols;
    const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
    bool m[NT][4];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int gy = y0 + 4 * nt + 2 * (j >> 4);
      m[nt][0] = gy < a.H && vx0;
      m[nt][1] = gy < a.H && vx1;
      m[nt][2] = gy + 1 < a.H && vx0;
      m[nt][3] = gy + 1 < a.H && vx1;
    }
    float v[V];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float t = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          t += (yv[mt * NT + nt][q][0] + yv[mt * NT + nt][q][1]) +
               (yv[mt * NT + nt][q][2] + yv[mt * NT + nt][q][3]);
        v[mt * 4 + q] = t;
      }
    const float mean = halfwave_reduce_scatter<V>(v, j) * inv;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float me = __shfl(mean, (h << 5) + ((mt * 4 + q) << SH), 64);
        float t = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = yv[mt * NT + nt][q][e] - me;
            t += m[nt][e] ? d * d : 0.f;
          }
        v[mt * 4 + q] = t;
      }
    const float m2 = halfwave_reduce_scatter<V>(v, j);
    const int e = (j >> SH) & (V - 1), mt = e >> 2, r = 4 * wave + (e & 3);
    const int co = co0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if ((j & ((1 << SH) - 1)) == 0 && co < a.Cout)
      a.stat_part[((int64_t)n * a.Cout + co) * a.stat_P + ty * a.tiles_x + tx] =
          make_float2(mean, m2);
  }
  if (ct + 1 < ct_end) {
    __syncthreads();  // the next co tile's first patch store reuses the exchange buffer
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[q][mt][nt][r] = 0.f;
  }
  }  // co tiles
}

int wino_launch(ConvArgs& a, int in_op, hipStream_t st) {
  constexpr int MT = kWMT, BM = 32 * MT, TH = 4 * (2 / MT);
  a.Cout_pad = (a.Cout + BM - 1) / BM * BM;
  a.nchunks = (a.Cin + kWCK - 1) / kWCK;
  a.tiles_x = (a.W + kTW - 1) / kTW;
  a.tiles_y = (a.H + TH - 1) / TH;
  a.co_tiles = a.Cout_pad / BM;
  a.stat_P = a.tiles_x * a.tiles_y;
  a.persist = wino_persist(in_op, (int64_t)a.tiles_x * a.tiles_y * a.N);
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.N * (a.persist ? 1 : a.co_tiles);
  RPST_REQUIRE(blocks <= 0x7fffffffLL, "conv2d: grid too large");
  const unsigned nb = (unsigned)blocks;
  const char* dbg = getenv("RPST_WINO_DBG");
  if (dbg && *dbg && in_op == RPST_IN_NONE && a.persist) {
    switch (atoi(dbg)) {
#define RPST_WINO_DBGCASE(D) \
  case D: wino_mfma_kernel<RPST_IN_NONE, MT, true, D><<<nb, kWinoNTH, 0, st>>>(a); break;
      RPST_WINO_DBGCASE(1) RPST_WINO_DBGCASE(2) RPST_WINO_DBGCASE(4) RPST_WINO_DBGCASE(15)
      RPST_WINO_DBGCASE(16) RPST_WINO_DBGCASE(32) RPST_WINO_DBGCASE(256)
#undef RPST_WINO_DBGCASE
      default: break;
    }
    return launch_status("wino_mfma_kernel(debug)");
  }
#define RPST_WINO_GO(OP)                                                                  \
  (a.persist ? (void)(wino_mfma_kernel<OP, MT, true><<<nb, kWinoNTH, 0, st>>>(a))          \
             : (void)(wino_mfma_kernel<OP, MT, false><<<nb, kWinoNTH, 0, st>>>(a)))
  switch (in_op) {
    case RPST_IN_MAXPOOL2:
      wino_mfma_kernel<RPST_IN_MAXPOOL2, MT, false><<<nb, kWinoNTH, 0, st>>>(a);
      break;
    case RPST_IN_ADD_UPSAMPLE2:
      wino_mfma_kernel<RPST_IN_ADD_UPSAMPLE2, MT, false><<<nb, kWinoNTH, 0, st>>>(a);
      break;
    case RPST_IN_ADD_ADAIN:
      wino_mfma_kernel<RPST_IN_ADD_ADAIN, MT, false><<<nb, kWinoNTH, 0, st>>>(a);
      break;
    case RPST_IN_UPSAMPLE2: RPST_WINO_GO(RPST_IN_UPSAMPLE2); break;
    case RPST_IN_ADAIN: RPST_WINO_GO(RPST_IN_ADAIN); break;
    default: RPST_WINO_GO(RPST_IN_NONE);
  }
#undef RPST_WINO_GO
  return launch_status("wino_mfma_kernel");
}

}  // namespace rpst
