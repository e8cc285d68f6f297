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
// Block = 4 waves, 64 output channels x (4 rows x 32 columns) = 2 x 16 tiles of 2x2.
// For each 16 positions xi = (i, jj) of the transformed domain the block computes the
// GEMM  M_xi[co][tile] = sum_ci U_xi[co][ci] V_xi[ci][tile]  (64 x 32 x Cin).
// Wave w owns the transform row i = w (4 positions x 2 co sub-tiles = 8 accumulators of
// 32x32), so:
//   * U = G g G^T is pre-transformed and pre-shuffled at pack time into exactly the
//     per-lane MFMA A-operand order: each lane loads its 32 weights of a chunk with 8
//     contiguous 16-B loads straight into registers (no LDS round trip for weights);
//   * V = B^T d B is computed by every wave in registers from the LDS input patch, for
//     its own row i only (row i of B^T touches two input rows), in the MFMA B-operand
//     layout: lane (h, j) builds the 4 values of channel 2cp+h, tile j;
//   * the output transform's column half (M A) is done in registers; the row half (A^T)
//     needs all four rows, exchanged once through LDS at the end.
// One barrier per K chunk: chunk c+1's patch is loaded into registers while chunk c's
// MFMAs run (the patch is double-buffered in LDS); each lane's weight registers are
// refilled with chunk c+1's values as soon as chunk c's MFMAs have consumed them.
#include "rpst_conv.h"

#include <cstdlib>

namespace rpst {

constexpr int kWCK = 8;            // input channels per chunk (packing and kernel)
constexpr int kWPH = kWinoTH + 2;  // patch rows
constexpr int kWPW = kTW + 2;      // patch columns
constexpr int kWLane = 4 * kWCK;   // packed weights per lane per chunk (cp, jj, mt)

// ---- weight transform + packing -------------------------------------------------------
// packed[(((ct * nch + c) * 4 + i) * 64 + lane) * 32 + (cp * 4 + jj) * 2 + mt]
//   = U_(i,jj)[co = ct*64 + mt*32 + (lane & 31)][ci = c*8 + 2*cp + (lane >> 5)]
// with U = G g G^T evaluated in fp64 and rounded once to fp32.
__global__ void wino_pack_kernel(const float* __restrict__ w, float* __restrict__ pk, int Cout,
                                 int Cin, int nch, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int idx = (int)(t % kWLane);
  int64_t r = t / kWLane;
  const int lane = (int)(r & 63);
  r >>= 6;
  const int i = (int)(r & 3);
  r >>= 2;
  const int c = (int)(r % nch);
  const int ct = (int)(r / nch);
  const int mt = idx & 1, jj = (idx >> 1) & 3, cp = idx >> 3;
  const int co = ct * kWinoBM + mt * 32 + (lane & 31);
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

size_t wino_packed_floats(int Cout, int Cin) {
  const size_t co_tiles = (size_t)(Cout + kWinoBM - 1) / kWinoBM;
  const size_t nch = (size_t)(Cin + kWCK - 1) / kWCK;
  return co_tiles * nch * 4 * 64 * kWLane;
}

int wino_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st) {
  const int64_t total = (int64_t)wino_packed_floats(Cout, Cin);
  const int nch = (Cin + kWCK - 1) / kWCK;
  wino_pack_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(w, pk, Cout, Cin, nch, total);
  return launch_status("wino_pack_kernel");
}

// ---- the kernel -------------------------------------------------------------------------
// WDB: double-buffered weight registers (next chunk loaded a whole chunk ahead) instead of
// a rolling refill of one set; the input patch is always prefetched two chunks ahead
// (its loads come from HBM, whose latency exceeds one chunk of MFMA work).
template <int INOP, bool WDB>
__global__ __launch_bounds__(kWinoNTH, 2) void wino_mfma_kernel(ConvArgs a) {
  constexpr int CK = kWCK, PH = kWPH, PW = kWPW, TH = kWinoTH;
  constexpr int R = RawN<INOP>::R;
  constexpr int XN = PH + 1;                  // patch rows + 1 halo element per lane
  constexpr int XS = CK * PH * PW;            // one patch buffer
  constexpr int PS = 4 * 2 * 2 * 16 * 64;     // output exchange (i, c, mt, r, lane)
  constexpr int SMEM = 2 * XS > PS ? 2 * XS : PS;
  static_assert(kWinoNTH == 32 * CK, "one 32-lane loader group per channel of a chunk");
  static_assert(2 * PH <= 32, "one halo element per lane");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];

  // block -> (column tile, row tile, image, co tile), co tile slowest (see rpst_conv.hip)
  int bid = blockIdx.x;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  bid /= a.tiles_y;
  const int n = bid % a.N;
  const int ct = bid / a.N;
  const int co0 = ct * kWinoBM;
  const int y0 = ty * TH, x0 = tx * kTW;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, j = lane & 31;

  const bool pooled = (INOP == RPST_IN_MAXPOOL2 || INOP == RPST_IN_UPSAMPLE2);
  const unsigned in_plane = pooled ? (unsigned)(a.Hs * a.Ws) : (unsigned)(a.H * a.W);
  const unsigned aux_plane = (unsigned)((a.H >> 1) * (a.W >> 1));
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (int64_t)n * a.Cin * in_plane), (short)0, (int)(a.Cin * in_plane * 4u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t raux = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(INOP == RPST_IN_ADD_UPSAMPLE2 ? a.aux + (int64_t)n * a.Cin * aux_plane : a.in),
      (short)0, (int)(a.Cin * aux_plane * 4u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.wpk + (int64_t)ct * a.nchunks * 4 * 64 * kWLane), (short)0, 0x7fffffff,
      0x00020000);
  const unsigned w_off = (unsigned)((wave * 64 + lane) * kWLane) * 4u;
  constexpr unsigned w_chunk = 4u * 64 * kWLane * 4;

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

  floatx16 acc[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[q][mt][r] = 0.f;

  u32x4 wA[kWLane / 4], wB[WDB ? kWLane / 4 : 1];
  // raw patch loads: prefetch distance PD = 2 chunks (sets xA / xB for even / odd chunks),
  // 1 for the 4-load max-pool loader (two sets of it do not fit in registers)
  constexpr int PD = R <= 2 ? 2 : 1;
  float xA[XN][R], xB[PD == 2 ? XN : 1][R];
  AdainP apA, apB;

#define RPST_WINO_WLOAD(W, c, q)                                                            \
  W[q] = __builtin_amdgcn_raw_buffer_load_b128(                                             \
      rw, (int)((c) < nchunks ? w_off + (unsigned)(c) * w_chunk + 16u * (q) : kOOB), 0, 0);

#define RPST_WINO_LOAD(c, X, AP)                                                            \
  {                                                                                         \
    const unsigned ch = (unsigned)((c) * CK + cg);                                          \
    const unsigned pb = ch * in_plane * 4u, ab = ch * aux_plane * 4u;                       \
    if (INOP == RPST_IN_ADAIN) AP = adain_params(a.aux, n, (int)ch, a);                     \
    _Pragma("unroll") for (int py = 0; py < PH; ++py) {                                     \
      int y = y0 - 1 + py;                                                                  \
      const bool yok = resolve(y, a.H, a.pad, true);                                        \
      fetch_raw<INOP>(X[py], rin, raux, pb, ab, y, bx, yok && bx_ok, a);                    \
    }                                                                                       \
    fetch_raw<INOP>(X[PH], rin, raux, pb, ab, hy, hx, h_ok, a);                             \
  }

  // write chunk c's raw patch (loaded one chunk earlier) into patch buffer c&1
#define RPST_WINO_STORE(c, X, AP)                                                           \
  {                                                                                         \
    float* xs = smem + ((c) & 1) * XS + cg * PH * PW;                                       \
    const bool chok = (int)((c) * CK + cg) < a.Cin;                                         \
    _Pragma("unroll") for (int py = 0; py < PH; ++py) {                                     \
      bool ok = chok && bx_ok;                                                              \
      if (INOP == RPST_IN_ADAIN) {                                                          \
        int y = y0 - 1 + py;                                                                \
        ok = ok && resolve(y, a.H, a.pad, true);                                            \
      }                                                                                     \
      xs[py * PW + jc + 1] = combine<INOP>(X[py], ok, AP);                                  \
    }                                                                                       \
    const float hv = combine<INOP>(X[PH], chok && h_ok, AP);                                \
    if (has_halo) xs[(jc >> 1) * PW + ((jc & 1) ? PW - 1 : 0)] = hv;                        \
  }

  // V for channel pair cp of chunk c (this wave's transform row), then the 8 MFMAs of
  // that pair with weight registers W; ROLL refills W's two quads with chunk c+1's values
#define RPST_WINO_CP(c, cp, W, ROLL)                                                        \
  {                                                                                         \
    const float* xs = smem + ((c) & 1) * XS + xoff + 2 * (cp) * PH * PW;                    \
    const float2 a0 = *reinterpret_cast<const float2*>(xs + ra * PW);                       \
    const float2 a1 = *reinterpret_cast<const float2*>(xs + ra * PW + 2);                   \
    const float2 b0 = *reinterpret_cast<const float2*>(xs + rb * PW);                       \
    const float2 b1 = *reinterpret_cast<const float2*>(xs + rb * PW + 2);                   \
    const float t0 = fmaf(sg, b0.x, a0.x), t1 = fmaf(sg, b0.y, a0.y);                       \
    const float t2 = fmaf(sg, b1.x, a1.x), t3 = fmaf(sg, b1.y, a1.y);                       \
    const float v[4] = {t0 - t2, t1 + t2, t2 - t1, t1 - t3};                                \
    _Pragma("unroll") for (int jj = 0; jj < 4; ++jj)                                        \
      _Pragma("unroll") for (int mt = 0; mt < 2; ++mt) {                                    \
        const int idx = ((cp) * 4 + jj) * 2 + mt;                                           \
        acc[jj][mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(                                 \
            __uint_as_float(W[idx >> 2][idx & 3]), v[jj], acc[jj][mt], 0, 0, 0);            \
      }                                                                                     \
    if (ROLL) {                                                                             \
      RPST_WINO_WLOAD(W, (c) + 1, 2 * (cp))                                                 \
      RPST_WINO_WLOAD(W, (c) + 1, 2 * (cp) + 1)                                             \
      __builtin_amdgcn_sched_barrier(0);                                                    \
    }                                                                                       \
  }

  // one K chunk: patch c to LDS, barrier, loads for chunk c+1, MFMAs of chunk c.
  // Double-buffered weights (WDB): WN receives chunk c+1's weights a whole chunk ahead.
#define RPST_WINO_CHUNK(c, WC, WN, X, AP)                                                   \
  {                                                                                         \
    RPST_WINO_STORE(c, X, AP)                                                               \
    __syncthreads();                                                                        \
    if ((c) + PD < nchunks) RPST_WINO_LOAD((c) + PD, X, AP)                                 \
    if (WDB) {                                                                              \
      _Pragma("unroll") for (int q = 0; q < kWLane / 4; ++q) RPST_WINO_WLOAD(WN, (c) + 1, q) \
      /* keep the prefetch here: the scheduler would otherwise sink it to the end of the  \
         chunk to save registers, exposing the load latency at the next barrier */        \
      __builtin_amdgcn_sched_barrier(0);                                                    \
    }                                                                                       \
    _Pragma("unroll") for (int cp = 0; cp < CK / 2; ++cp) RPST_WINO_CP(c, cp, WC, !WDB)     \
  }

  // transform row i = wave of B^T: t = d[ra] + sg * d[rb]
  const int ra = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int rb = wave == 0 ? 2 : (wave == 1 ? 2 : (wave == 2 ? 1 : 3));
  const float sg = wave == 1 ? 1.f : -1.f;
  const int tyl = j >> 4, txl = j & 15;
  const int xoff = h * PH * PW + 2 * tyl * PW + 2 * txl;

  const int nchunks = a.nchunks;
#pragma unroll
  for (int q = 0; q < kWLane / 4; ++q) RPST_WINO_WLOAD(wA, 0, q)
  RPST_WINO_LOAD(0, xA, apA)
  if constexpr (PD == 2) {
    if (nchunks > 1) RPST_WINO_LOAD(1, xB, apB)
  }
  for (int c = 0; c < nchunks; c += 2) {
    if constexpr (WDB) {  // (implies PD == 2)
      RPST_WINO_CHUNK(c, wA, wB, xA, apA)
      if (c + 1 < nchunks) RPST_WINO_CHUNK(c + 1, wB, wA, xB, apB)
    } else if constexpr (PD == 2) {
      RPST_WINO_CHUNK(c, wA, wA, xA, apA)
      if (c + 1 < nchunks) RPST_WINO_CHUNK(c + 1, wA, wA, xB, apB)
    } else {
      RPST_WINO_CHUNK(c, wA, wA, xA, apA)
      if (c + 1 < nchunks) RPST_WINO_CHUNK(c + 1, wA, wA, xA, apA)
    }
  }
#undef RPST_WINO_CHUNK
#undef RPST_WINO_CP
#undef RPST_WINO_STORE
#undef RPST_WINO_LOAD
#undef RPST_WINO_WLOAD

  // ---- output transform ---------------------------------------------------------------
  // column half in registers: P[i][0] = M0 + M1 + M2, P[i][1] = M1 - M2 - M3 (i = wave)
  __syncthreads();  // every wave is done with the patch buffers
  float* Ps = smem;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float m0 = acc[0][mt][r], m1 = acc[1][mt][r], m2 = acc[2][mt][r], m3 = acc[3][mt][r];
      Ps[(((wave * 2 + 0) * 2 + mt) * 16 + r) * 64 + lane] = (m0 + m1) + m2;
      Ps[(((wave * 2 + 1) * 2 + mt) * 16 + r) * 64 + lane] = (m1 - m2) - m3;
    }
  __syncthreads();

  // row half: wave w finishes accumulator rows r = 4w..4w+3 of both co sub-tiles
  const int gy = y0 + 2 * tyl, gx = x0 + 2 * txl;
  const bool vy0 = gy < a.H, vy1 = gy + 1 < a.H, vx0 = gx < a.W, vx1 = gx + 1 < a.W;
  const bool vec = vx1 && (a.W & 1) == 0;
  float yv[8][4];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * wave + q;
      float P[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) P[i][cc] = Ps[(((i * 2 + cc) * 2 + mt) * 16 + r) * 64 + lane];
      float y[4] = {(P[0][0] + P[1][0]) + P[2][0], (P[0][1] + P[1][1]) + P[2][1],
                    (P[1][0] - P[2][0]) - P[3][0], (P[1][1] - P[2][1]) - P[3][1]};
      const int co = co0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co < a.Cout) {
        const float b = a.bias ? a.bias[co] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[e] += b;
          if (a.relu) y[e] = fmaxf(y[e], 0.f);
        }
        float* o = a.out + (((int64_t)n * a.Cout + co) * a.H + gy) * a.W + gx;
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
#pragma unroll
      for (int e = 0; e < 4; ++e) yv[mt * 4 + q][e] = y[e];
    }

  // optional output statistics, as conv_mfma_kernel: per (channel, block) (mean, M2) of
  // the written values; one partial per block (stat_P = tiles_x * tiles_y)
  if (a.stat_part) {
    const bool m[4] = {vy0 && vx0, vy0 && vx1, vy1 && vx0, vy1 && vx1};
    const int rows = max(0, min(TH, a.H - y0)), cols = max(0, min(kTW, a.W - x0));
    const int cnt = rows * cols;
    const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = ((m[0] ? yv[e][0] : 0.f) + (m[1] ? yv[e][1] : 0.f)) +
             ((m[2] ? yv[e][2] : 0.f) + (m[3] ? yv[e][3] : 0.f));
    const float mean = halfwave_reduce_scatter8(v, j) * inv;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float me = __shfl(mean, (h << 5) + 4 * e, 64);
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d = yv[e][q] - me;
        s += m[q] ? d * d : 0.f;
      }
      v[e] = s;
    }
    const float m2 = halfwave_reduce_scatter8(v, j);
    const int e = (j >> 2) & 7, mt = e >> 2, r = 4 * wave + (e & 3);
    const int co = co0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if ((j & 3) == 0 && co < a.Cout)
      a.stat_part[((int64_t)n * a.Cout + co) * a.stat_P + ty * a.tiles_x + tx] =
          make_float2(mean, m2);
  }
}

int wino_launch(ConvArgs& a, int in_op, hipStream_t st) {
  a.Cout_pad = (a.Cout + kWinoBM - 1) / kWinoBM * kWinoBM;
  a.nchunks = (a.Cin + kWCK - 1) / kWCK;
  a.tiles_x = (a.W + kTW - 1) / kTW;
  a.tiles_y = (a.H + kWinoTH - 1) / kWinoTH;
  a.co_tiles = a.Cout_pad / kWinoBM;
  a.stat_P = a.tiles_x * a.tiles_y;
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.N * a.co_tiles;
  RPST_REQUIRE(blocks <= 0x7fffffffLL, "conv2d: grid too large");
  const char* e = getenv("RPST_WINO_WDB");
  // measured (tools/bench_conv.py): the rolling single weight set is faster (fewer
  // registers, no false load dependencies at the chunk boundary)
  const bool wdb = (e && *e) ? atoi(e) != 0 : false;
#define RPST_WINO_GO(OP)                                                                   \
  {                                                                                        \
    if (wdb && RawN<OP>::R == 1)                                                           \
      wino_mfma_kernel<OP, RawN<OP>::R == 1><<<(unsigned)blocks, kWinoNTH, 0, st>>>(a);    \
    else                                                                                   \
      wino_mfma_kernel<OP, false><<<(unsigned)blocks, kWinoNTH, 0, st>>>(a);               \
  }
  switch (in_op) {
    case RPST_IN_MAXPOOL2: RPST_WINO_GO(RPST_IN_MAXPOOL2) break;
    case RPST_IN_UPSAMPLE2: RPST_WINO_GO(RPST_IN_UPSAMPLE2) break;
    case RPST_IN_ADD_UPSAMPLE2: RPST_WINO_GO(RPST_IN_ADD_UPSAMPLE2) break;
    case RPST_IN_ADAIN: RPST_WINO_GO(RPST_IN_ADAIN) break;
    default: RPST_WINO_GO(RPST_IN_NONE)
  }
#undef RPST_WINO_GO
  return launch_status("wino_mfma_kernel");
}

}  // namespace rpst
