// Backward kernels of the AdaIN-RP training step:
// AdaINRPNet.forward (network/adain_rp.py:110-138) + total_loss.backward() (train.py:186-189).
//
//   conv dgrad        = the forward conv kernel on flip-transposed weights (conv_flip_kernel
//                       here, packing by rpst_conv2d_pack); reflect-padded convs (the frozen
//                       VGG) add the padded border's gradient folded back onto the rows /
//                       columns it reflects (reflect_ring_kernel + reflect_fold_kernel)
//   conv wgrad        conv_wgrad_kernel: implicit GEMM dW[co][ci][tap] = sum over (n,y,x) of
//                       dY[n][co][y][x] X[n][ci][y+dy][x+dx] on fp32 MFMA, split over K
//                       (pixels) with a fixed-order reduction (wgrad_reduce_kernel)
//   bias grad         reduced by the wgrad kernel's first ci-tile blocks from their dY tiles
//   ReLU / max-pool   relu_backward_kernel, maxpool2_backward_kernel (argmax = first max in
//                       window order, NaN wins, as ATen's max_pool2d)
//   AdaIN             adain_backward_reduce_kernel + adain_backward_apply_kernel
//   losses            loss_seed_kernel (d/dF of calc_style_loss + calc_content_loss) and
//                       sq_diff_sum_kernel (the loss values)
// All reductions are fixed-order (no float atomics): results are deterministic.
#include <cstdlib>

#include "rpst_common.h"

namespace rpst {

// ---- weights for dgrad: wt[ci][co][kh][kw] = w[co][ci][k-1-kh][k-1-kw] ------------------
__global__ __launch_bounds__(256) void conv_flip_kernel(const float* __restrict__ w,
                                                        float* __restrict__ wt, int Cout,
                                                        int Cin, int K) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t kk = (int64_t)K * K;
  if (i >= (int64_t)Cout * Cin * kk) return;
  const int t = (int)(i % kk);
  const int64_t r = i / kk;
  const int ci = (int)(r % Cin), co = (int)(r / Cin);
  wt[((int64_t)ci * Cout + co) * kk + (kk - 1 - t)] = w[i];
}

// ---- ReLU backward: threshold_backward(grad, output, 0) -----------------------------------
// slope = 0: ReLU (threshold_backward: g where y > 0, else 0); slope > 0: LeakyReLU
// (Conv2dBlock base.py:147; leaky_relu_backward on the result: g where y > 0, else slope g)
__global__ __launch_bounds__(256) void relu_backward_kernel(const float* __restrict__ g,
                                                            const float* __restrict__ y,
                                                            float* __restrict__ out, int64_t n,
                                                            float slope) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  auto f = [slope](float gv, float yv) { return yv > 0.f ? gv : (slope == 0.f ? 0.f : gv * slope); };
  if (i + 3 < n) {
    const float4 gv = *reinterpret_cast<const float4*>(g + i);
    const float4 yv = *reinterpret_cast<const float4*>(y + i);
    float4 o;
    o.x = f(gv.x, yv.x);
    o.y = f(gv.y, yv.y);
    o.z = f(gv.z, yv.z);
    o.w = f(gv.w, yv.w);
    *reinterpret_cast<float4*>(out + i) = o;
  } else {
    for (int64_t j = i; j < n; ++j) out[j] = f(g[j], y[j]);
  }
}

// ---- MaxPool2d(2, 2, ceil_mode=True) backward, optionally masked by ReLU(x) > 0 ----------
__global__ __launch_bounds__(256) void maxpool2_backward_kernel(
    const float* __restrict__ x, const float* __restrict__ g, float* __restrict__ dx,
    int64_t planes, int H, int W, int relu_mask) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= planes * Ho * Wo) return;
  const int ox = (int)(i % Wo);
  const int64_t r = i / Wo;
  const int oy = (int)(r % Ho);
  const int64_t p = r / Ho;
  const float* s = x + p * H * W;
  float* d = dx + p * H * W;
  // ATen's CPU max_pool2d: window in row-major order, `val > max || isnan(val)` updates,
  // the index starts at the window's first element
  int best = 0;
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int yy = 2 * oy + (k >> 1), xx = 2 * ox + (k & 1);
    if (yy < H && xx < W) {
      const float v = s[(int64_t)yy * W + xx];
      if (v > m || v != v) {
        m = v;
        best = k;
      }
    }
  }
  const float gv = g[i];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int yy = 2 * oy + (k >> 1), xx = 2 * ox + (k & 1);
    if (yy < H && xx < W) {
      float v = (k == best) ? gv : 0.f;
      if (relu_mask && !(s[(int64_t)yy * W + xx] > 0.f)) v = 0.f;
      d[(int64_t)yy * W + xx] = v;
    }
  }
}

// ---- reflect-pad border gradient ---------------------------------------------------------
// Forward: Y = conv3x3_valid(ReflectionPad2d(1)(X)). The zero-padded dgrad conv gives the
// gradient of the padded input's interior, dXp[1..H][1..W]; the padded border ("ring":
// rows 0 and H+1, columns 0 and W+1) is added to the X element it reflects: row 0 -> 1,
// row H+1 -> H-2, column 0 -> 1, column W+1 -> W-2 (corners both ways).
//   reflect_ring_kernel: dXp on the ring (four 1-D convolutions, tiled below);
//   reflect_fold_kernel: one thread per target element (rows {1, H-2} fully, columns
//     {1, W-2} on the other rows) sums its ring entries in a fixed order and adds them.
// ring layout per plane: [top row q = 0..W+1 | bottom row q = 0..W+1 | left column p = 1..H |
// right column p = 1..H].
__device__ __forceinline__ int refl(int t, int n) { return t < 0 ? -t : (t >= n ? 2 * n - 2 - t : t); }

// The ring is four 1-D convolutions over the image's border lines: for side 0/1 (padded
// row 0 / H+1) the line is dY's row 0 / H-1 and the taps are the weights' row 0 / 2; for side
// 2/3 (padded column 0 / W+1) the line is dY's column 0 / W-1 and the taps the weights'
// column 0 / 2:  ring[ci][u] = sum_co sum_k line[co][u - k] tap[co][ci][k].
// Block = (64 ring positions) x (64 input channels) of one image and side and one of ks
// split-K ranges of co (a latency-bound co loop otherwise: 32 chunks at Cout = 512); co in
// chunks of 16 staged in LDS (line segment with its 2-element halo, taps transposed
// ci-contiguous); each thread accumulates 4 ci x 4 positions. Split s writes ring copy s; the
// fold sums the copies in order (ks is a function of Cout only).
constexpr int kRingKS = 4;  // ring copies in the workspace
static int ring_splits(int Cout) {
  const int ks = Cout / 64;
  return ks < 1 ? 1 : (ks > kRingKS ? kRingKS : ks);
}
__global__ __launch_bounds__(256) void reflect_ring_kernel(
    const float* __restrict__ dy, const float* __restrict__ w, float* __restrict__ ring, int N,
    int Cin, int Cout, int H, int W, int ks) {
  constexpr int CC = 16;
  __shared__ float line[CC][64 + 2];
  __shared__ __attribute__((aligned(16))) float taps[CC][3][64];
  const int split = blockIdx.z % ks, zs = blockIdx.z / ks;
  const int side = zs & 3, n = zs >> 2;
  const int cper = ((Cout + ks - 1) / ks + CC - 1) / CC * CC;
  const int cbeg = split * cper, cend = min(Cout, cbeg + cper);
  const bool row = side < 2;
  const int L = row ? W : H;                  // line length
  const int U = row ? W + 2 : H;              // outputs on this side
  const int u_first = row ? 0 : 1;            // u of output index 0
  const int u0 = blockIdx.x * 64 + u_first;   // first u of the block
  const int ci0 = blockIdx.y * 64;
  const int tid = threadIdx.x, cg = tid >> 4, ug = tid & 15;
  const int64_t HW = (int64_t)H * W;
  const float* dyn = dy + (int64_t)n * Cout * HW;
  float acc[4][4] = {};
  // the next co chunk's line and tap values are loaded into registers while the current
  // chunk computes (the loads are latency-bound: column lines stride W, taps stride 9)
  constexpr int kLn = (CC * 66 + 255) / 256, kTp = CC * 3 * 64 / 256;
  float lv[kLn], tv[kTp];
  auto gload = [&](int c0) {
#pragma unroll
    for (int i = 0; i < kLn; ++i) {
      const int e = tid + 256 * i;
      const int cc = e / 66, tt = e - cc * 66, t = u0 - 2 + tt, co = c0 + cc;
      float v = 0.f;
      if (e < CC * 66 && co < cend && t >= 0 && t < L) {
        const int64_t off = row ? (int64_t)(side == 0 ? 0 : H - 1) * W + t
                                : (int64_t)t * W + (side == 2 ? 0 : W - 1);
        v = dyn[co * HW + off];
      }
      lv[i] = v;
    }
#pragma unroll
    for (int i = 0; i < kTp; ++i) {
      const int e = tid + 256 * i;
      const int cc = e / 192, r = e - cc * 192, k = r / 64, c = r - k * 64;
      const int co = c0 + cc, ci = ci0 + c;
      float v = 0.f;
      if (co < cend && ci < Cin) {
        const int kh = row ? (side == 0 ? 0 : 2) : k, kw = row ? k : (side == 2 ? 0 : 2);
        v = w[((int64_t)co * Cin + ci) * 9 + kh * 3 + kw];
      }
      tv[i] = v;
    }
  };
  gload(cbeg);
  for (int c0 = cbeg; c0 < cend; c0 += CC) {
#pragma unroll
    for (int i = 0; i < kLn; ++i) {
      const int e = tid + 256 * i;
      if (e < CC * 66) line[e / 66][e % 66] = lv[i];
    }
#pragma unroll
    for (int i = 0; i < kTp; ++i) {
      const int e = tid + 256 * i;
      taps[e / 192][(e % 192) / 64][e % 64] = tv[i];
    }
    __syncthreads();
    if (c0 + CC < cend) gload(c0 + CC);
#pragma unroll 4
    for (int cc = 0; cc < CC; ++cc) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float4 wv = *reinterpret_cast<const float4*>(&taps[cc][k][cg * 4]);
        float sv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) sv[e] = line[cc][ug * 4 + e - k + 2];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[0][e] = fmaf(sv[e], wv.x, acc[0][e]);
          acc[1][e] = fmaf(sv[e], wv.y, acc[1][e]);
          acc[2][e] = fmaf(sv[e], wv.z, acc[2][e]);
          acc[3][e] = fmaf(sv[e], wv.w, acc[3][e]);
        }
      }
    }
    __syncthreads();
  }
  const int R = 2 * (W + 2) + 2 * H;
  const int base = side == 0 ? 0 : (side == 1 ? W + 2 : (side == 2 ? 2 * (W + 2) - 1 : 2 * (W + 2) + H - 1));
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int ci = ci0 + cg * 4 + a;
    if (ci >= Cin) continue;
    float* rg = ring + ((int64_t)split * N * Cin + (int64_t)n * Cin + ci) * R;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int u = u0 + ug * 4 + e;
      if (u - u_first < U) rg[base + u] = acc[a][e];
    }
  }
}

__global__ __launch_bounds__(256) void reflect_fold_kernel(
    const float* __restrict__ ring, float* __restrict__ dx, const float* __restrict__ mask,
    int N, int Cin, int H, int W, int nrows, int r0, int r1, int ncols, int c0, int c1, int ks) {
  const int64_t per = (int64_t)nrows * W + (int64_t)ncols * (H - nrows);
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * Cin * per) return;
  const int64_t plane = t / per;
  int64_t k = t - plane * per;
  int i, j;
  if (k < (int64_t)nrows * W) {
    i = (k < W) ? r0 : r1;
    j = (int)(k % W);
  } else {
    k -= (int64_t)nrows * W;
    const int cidx = (int)(k / (H - nrows));
    // the rr-th row that is not one of the full rows
    const int lo = r0 < r1 ? r0 : r1, hi = r0 < r1 ? r1 : r0;
    int rr = (int)(k % (H - nrows));
    if (rr >= lo) ++rr;
    if (nrows == 2 && rr >= hi) ++rr;
    i = rr;
    j = cidx == 0 ? c0 : c1;
  }
  const int R = 2 * (W + 2) + 2 * H;
  const float* rg = ring + plane * R;
  const int64_t copy = (int64_t)N * Cin * R;
  auto rv = [&](int idx) {  // ring entry idx, its ks split-K copies summed in order
    float v = rg[idx];
    for (int s = 1; s < ks; ++s) v += rg[s * copy + idx];
    return v;
  };
  float add = 0.f;
  // padded rows p in {0, H+1}: every column q of the padded row that reflects to j
  for (int pi = 0; pi < 2; ++pi) {
    const int p = pi ? H + 1 : 0;
    if (refl(p - 1, H) != i) continue;
    const int row = pi * (W + 2);
    if (refl(-1, W) == j) add += rv(row);
    add += rv(row + j + 1);
    if (refl(W, W) == j) add += rv(row + W + 1);
  }
  // padded columns q in {0, W+1} on the interior padded row p = i + 1
  if (refl(-1, W) == j) add += rv(2 * (W + 2) + i);
  if (refl(W, W) == j) add += rv(2 * (W + 2) + H + i);
  const int64_t o = plane * H * W + (int64_t)i * W + j;
  if (mask && !(mask[o] > 0.f)) return;  // threshold_backward: dx stays 0 there
  dx[o] = dx[o] + add;
}

// ---- conv weight gradient (3x3, stride 1, zero pad 1) ---------------------------------------
// reflect != 0: ReflectionPad2d(1) instead (the decoders of sanet.py:162-192): rows -1 / H and
// columns -1 / W of X read rows / columns 1 / H - 2 (only column W inside a segment needs a
// fix-up: columns past it multiply a zero dY).
// Block: 256 threads (4 waves), all 9 taps (9 accumulators per wave). TC = 64: tile 64 co x
// 64 ci split 2 x 2 over the waves, K = pixels walked in row segments of PX = 64 columns.
// TC = 32 (Cin, Cout <= 32: the RP stacks' 3..32-channel layers, where a 64-wide tile would
// be 3/4 padding): tile 32 co x 32 ci, segments of PX = 128 columns, and the four waves
// split the segment's pixels (32 each) as four split-K partials of their own (the reduce
// kernel sums 4 x splits partials). LDS holds dY[px][co] (PX x (TC+1)) and X[row][col][ci]
// (3 x (PX+2) x (TC+1), rows y-1..y+1, columns x0-1..x0+PX, zero outside the image);
// v_mfma_f32_32x32x2_f32 with A = dY (co x px) and B = X shifted by the tap (px x ci).
// Staging: thread -> (channel c = tid / (256/TC), 16-column group q of the PX columns); the
// next segment's 16-B buffer loads (dY 4, X 12, X halo 3 per thread) are issued into
// registers before the current segment's MFMAs and written to LDS after them (one load
// latency per segment, hidden behind 288 (TC 64) / 144 (TC 32) MFMAs per wave). Rows /
// channels outside the image read the out-of-range offset (0), columns at or past W are
// masked. Blocks of the first ci tile also reduce the bias gradient (sum of dY over their
// pixels) from the staged dY tile.
constexpr unsigned kWgOOB = 0x80000000u;

typedef unsigned wg_u32x4 __attribute__((ext_vector_type(4)));

template <bool VEC, int TC>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ part,
    float* __restrict__ bpart, int N, int Cin, int H, int W, int Cout, int64_t segs_per_split,
    int reflect) {
  constexpr int PX = 4096 / TC, LD = TC + 1, COLS = PX + 2, QN = PX / 16;
  constexpr int KSPL = TC == 32 ? 4 : 1;  // per-wave pixel split (partials per split)
  __shared__ float Ys[PX * LD];
  __shared__ float Xs[3 * COLS * LD];
  const int tilesCi = (Cin + TC - 1) / TC;
  const int tile = blockIdx.x, split = blockIdx.y;
  const int co0 = (tile / tilesCi) * TC, ci0 = (tile % tilesCi) * TC;
  const bool bias_tile = bpart != nullptr && (tile % tilesCi) == 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = KSPL > 1 ? 0 : wave >> 1, wn = KSPL > 1 ? 0 : wave & 1;
  const int h = lane >> 5, j = lane & 31;
  const int segW = (W + PX - 1) / PX;
  const int64_t segs = (int64_t)N * H * segW;
  const int64_t s0 = (int64_t)split * segs_per_split;
  const int64_t s1 = s0 + segs_per_split < segs ? s0 + segs_per_split : segs;
  const unsigned HW = (unsigned)(H * W);
  const int c = tid / QN, q = tid % QN;
  const bool co_ok = co0 + c < Cout, ci_ok = ci0 + c < Cin;

  floatx16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bacc = 0.f;

  wg_u32x4 ry[4], rx[3][4];
  float rh[3];
  // issue the loads of segment sg into registers (branch-free buffer loads)
  auto load = [&](int64_t sg) {
    const bool live = sg < s1;
    const int64_t sgc = live ? sg : s0;
    const int xs = (int)(sgc % segW);
    const int64_t ry_ = sgc / segW;
    const int y = (int)(ry_ % H), n = (int)(ry_ / H);
    const int x0 = xs * PX;
    const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(dy + (int64_t)n * Cout * HW), (short)0, (int)(Cout * HW * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rxx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + (int64_t)n * Cin * HW), (short)0, (int)(Cin * HW * 4u), 0x00020000);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xx = x0 + q * 16 + 4 * k;
      const bool ok = live && co_ok && (VEC ? xx < W : true);
      const unsigned off = ok ? ((unsigned)(co0 + c) * HW + (unsigned)y * W + xx) * 4u : kWgOOB;
      if (VEC) {
        ry[k] = __builtin_amdgcn_raw_buffer_load_b128(rdy, (int)off, 0, 0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool oe = ok && xx + e < W;
          ry[k][e] = __builtin_amdgcn_raw_buffer_load_b32(rdy, (int)(oe ? off + 4u * e : kWgOOB), 0, 0);
        }
      }
    }
#pragma unroll
    for (int row = 0; row < 3; ++row) {
      int yy = y - 1 + row;
      if (reflect) yy = reflect1(yy, H);
      const bool rok = live && ci_ok && yy >= 0 && yy < H;
      const unsigned rbase = ((unsigned)(ci0 + c) * HW + (unsigned)(rok ? yy : 0) * W) * 4u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int xx = x0 + q * 16 + 4 * k;
        const bool ok = rok && (VEC ? xx < W : true);
        if (VEC) {
          rx[row][k] = __builtin_amdgcn_raw_buffer_load_b128(
              rxx, (int)(ok ? rbase + 4u * xx : kWgOOB), 0, 0);
          // reflect: column W (first element of a group past the image) is column W - 2
          if (reflect && xx == W)
            rx[row][k][0] = __builtin_amdgcn_raw_buffer_load_b32(
                rxx, (int)(rok ? rbase + 4u * (W - 2) : kWgOOB), 0, 0);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int xe = reflect && xx + e == W ? W - 2 : xx + e;
            const bool oe = ok && xe < W;
            rx[row][k][e] = __builtin_amdgcn_raw_buffer_load_b32(
                rxx, (int)(oe ? rbase + 4u * xe : kWgOOB), 0, 0);
          }
        }
      }
      // halo: column x0 - 1 (q == 0) or x0 + PX (q == QN - 1)
      int hx = q == 0 ? x0 - 1 : x0 + PX;
      if (reflect && hx <= W) hx = reflect1(hx, W);
      const bool hok = rok && (q == 0 || q == QN - 1) && hx >= 0 && hx < W;
      rh[row] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(rxx, (int)(hok ? rbase + 4u * hx : kWgOOB), 0, 0));
    }
  };
  // columns at or past W were loaded as 0 (VEC: whole float4 out; scalar: per element)
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) Ys[(q * 16 + 4 * k + e) * LD + c] = __uint_as_float(ry[k][e]);
#pragma unroll
    for (int row = 0; row < 3; ++row) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          Xs[(row * COLS + 1 + q * 16 + 4 * k + e) * LD + c] = __uint_as_float(rx[row][k][e]);
      if (q == 0) Xs[(row * COLS) * LD + c] = rh[row];
      if (q == QN - 1) Xs[(row * COLS + COLS - 1) * LD + c] = rh[row];
    }
  };

  // pixel pairs of this wave: all PX / 2 (TC 64) or its quarter of them (TC 32)
  constexpr int KK = PX / 2 / KSPL;
  const int kk0 = KSPL > 1 ? wave * KK : 0;
  load(s0);
  for (int64_t sg = s0; sg < s1; ++sg) {
    store();
    __syncthreads();
    load(sg + 1);  // in flight during this segment's MFMAs
    if (bias_tile && wave == 0 && lane < TC) {
      float t = 0.f;
      for (int px = 0; px < PX; ++px) t += Ys[px * LD + lane];
      bacc += t;
    }
#pragma unroll 4
    for (int kk = kk0; kk < kk0 + KK; ++kk) {
      const int px = 2 * kk + h;
      const float av = Ys[px * LD + wm * 32 + j];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dyy = t / 3, dxx = t % 3;
        const float bv = Xs[(dyy * COLS + px + dxx) * LD + wn * 32 + j];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (bias_tile && wave == 0 && lane < TC && co0 + lane < Cout)
    bpart[(int64_t)split * Cout + co0 + lane] = bacc;
  // partial[split * KSPL + wave part][co][ci][9]; accumulator element r of lane: row (co) =
  // (r&3) + 8(r>>2) + 4h, column (ci) = j
  const int ci = ci0 + wn * 32 + j;
  if (ci >= Cin || (KSPL == 1 && wn * 32 + j >= TC)) return;
  const int64_t ps = (int64_t)split * KSPL + (KSPL > 1 ? wave : 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = co0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (co >= Cout) continue;
    float* o = part + ((ps * Cout + co) * Cin + ci) * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) o[t] = acc[t][r];
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part,
                                                           float* __restrict__ dw, int64_t n,
                                                           int splits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  // 8 independent loads in flight, summed in split order
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= splits; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(k + u) * n + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < splits; ++k) s += part[(int64_t)k * n + i];
  dw[i] = s;
}

// ---- AdaIN backward ----------------------------------------------------------------------
// out = nc * sigma_s + mu_s, nc = (c - mu_c) / sigma_c, sigma = sqrt(var_unbiased + eps):
//   S1 = sum g, S2 = sum g nc (per plane)
//   dc = (sigma_s / sigma_c) (g - S1 / HW - nc S2 / (HW - 1))
//   ds = S1 / HW + S2 (s - mu_s) / ((HW - 1) sigma_s)
// stats = [mean_c | std_c | mean_s | std_s] (planes each).
__global__ __launch_bounds__(256) void adain_backward_reduce_kernel(
    const float* __restrict__ g, const float* __restrict__ c, const float* __restrict__ stats,
    float* __restrict__ sums, int planes, int64_t HW) {
  const int p = blockIdx.x;
  const float mc = stats[p], sc = stats[planes + p];
  const float* gp = g + (int64_t)p * HW;
  const float* cp = c + (int64_t)p * HW;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t i = threadIdx.x; i < HW; i += 256) {
    const float gv = gp[i];
    const float nc = (cp[i] - mc) / sc;
    s1 += gv;
    s2 += (double)gv * nc;
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  __shared__ double red[2][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sums[p] = (float)(red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    sums[planes + p] = (float)(red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

__global__ __launch_bounds__(256) void adain_backward_apply_kernel(
    const float* __restrict__ g, const float* __restrict__ c, const float* __restrict__ s,
    const float* __restrict__ stats, const float* __restrict__ sums, float* __restrict__ dc,
    float* __restrict__ ds, int planes, int64_t HW) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)planes * HW) return;
  const int p = (int)(i / HW);
  const float mc = stats[p], sc = stats[planes + p];
  const float ms = stats[2 * planes + p], ss = stats[3 * planes + p];
  const float S1 = sums[p], S2 = sums[planes + p];
  const float n = (float)HW, n1 = (float)(HW - 1);
  const float nc = (c[i] - mc) / sc;
  dc[i] = (ss / sc) * (g[i] - S1 / n - nc * S2 / n1);
  ds[i] = S1 / n + S2 * (s[i] - ms) / (n1 * ss);
}

// ---- losses ------------------------------------------------------------------------------
// d/dF of w_s * [mse(mu(F), mu_t) + mse(sigma(F), sigma_t)] (+ w_c * mse(F, Fc)) with
// mse over the (N, C) statistics (mean reduction): per plane
//   a = w_s 2 (mu - mu_t) / (N C HW),  b = w_s 2 (sigma - sigma_t) / (N C (HW - 1) sigma)
//   dF = a + b (F - mu) [+ w_c 2 (F - Fc) / (N C HW)]
// Weights are read from the device (wts[0] = w_s, wts[1] = w_c) so autograd's incoming
// gradient scales them without a host round trip. acc = 1 adds into out.
__global__ __launch_bounds__(256) void loss_seed_kernel(
    const float* __restrict__ F, const float* __restrict__ Fc, const float* __restrict__ st,
    const float* __restrict__ wts, float* __restrict__ out, int planes, int64_t HW, int acc) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)planes * HW) return;
  const int p = (int)(i / HW);
  // st = [mean | std | mean_t | std_t]
  const float mu = st[p], sd = st[planes + p], mut = st[2 * planes + p], sdt = st[3 * planes + p];
  const float ws = wts[0];
  const double nc = (double)planes;
  const float a = (float)(ws * 2.0 * ((double)mu - mut) / (nc * (double)HW));
  const float b = (float)(ws * 2.0 * ((double)sd - sdt) / (nc * (double)(HW - 1) * sd));
  float v = a + b * (F[i] - mu);
  if (Fc) v += (float)(wts[1] * 2.0 / (nc * (double)HW)) * (F[i] - Fc[i]);
  out[i] = acc ? out[i] + v : v;
}

// Deterministic sum of (a - b)^2 over n elements: per-block partials, then one block.
__global__ __launch_bounds__(256) void sq_diff_partial_kernel(const float* __restrict__ a,
                                                              const float* __restrict__ b,
                                                              double* __restrict__ part,
                                                              int64_t n) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double d = (double)a[i] - (double)b[i];
    s += d * d;
  }
  s = wave_sum(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void sq_diff_final_kernel(const double* __restrict__ part,
                                                            int nparts, double scale,
                                                            float* __restrict__ out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = wave_sum(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (float)((red[0] + red[1] + red[2] + red[3]) * scale);
}

}  // namespace rpst

using namespace rpst;

static inline unsigned blocks_for(int64_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

extern "C" int rpst_conv_weight_flip(const float* w, float* wt, int Cout, int Cin, int ksize,
                                     rpst_stream_t stream) {
  RPST_REQUIRE(w && wt && Cout > 0 && Cin > 0 && (ksize == 1 || ksize == 3),
               "conv_weight_flip: bad args");
  const int64_t n = (int64_t)Cout * Cin * ksize * ksize;
  conv_flip_kernel<<<blocks_for(n), 256, 0, as_stream(stream)>>>(w, wt, Cout, Cin, ksize);
  return launch_status("conv_flip_kernel");
}

extern "C" int rpst_relu_backward(const float* g, const float* y, float* out, int64_t n,
                                  rpst_stream_t stream) {
  RPST_REQUIRE(g && y && out && n > 0, "relu_backward: bad args");
  relu_backward_kernel<<<blocks_for((n + 3) / 4), 256, 0, as_stream(stream)>>>(g, y, out, n, 0.f);
  return launch_status("relu_backward_kernel");
}

extern "C" int rpst_leaky_relu_backward(const float* g, const float* y, float* out, int64_t n,
                                        float slope, rpst_stream_t stream) {
  RPST_REQUIRE(g && y && out && n > 0 && slope > 0.f, "leaky_relu_backward: bad args");
  relu_backward_kernel<<<blocks_for((n + 3) / 4), 256, 0, as_stream(stream)>>>(g, y, out, n,
                                                                               slope);
  return launch_status("relu_backward_kernel");
}

extern "C" int rpst_maxpool2x2_ceil_backward(const float* x, const float* g, float* dx, int N,
                                             int C, int H, int W, int relu_mask,
                                             rpst_stream_t stream) {
  RPST_REQUIRE(x && g && dx && N > 0 && C > 0 && H > 0 && W > 0, "maxpool_backward: bad args");
  const int64_t n = (int64_t)N * C * ((H + 1) / 2) * ((W + 1) / 2);
  maxpool2_backward_kernel<<<blocks_for(n), 256, 0, as_stream(stream)>>>(
      x, g, dx, (int64_t)N * C, H, W, relu_mask);
  return launch_status("maxpool2_backward_kernel");
}

extern "C" size_t rpst_reflect_pad_border_grad_workspace_size(int N, int Cin, int H, int W) {
  if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0) return 0;
  return sizeof(float) * kRingKS * (size_t)N * Cin * (2 * (size_t)(W + 2) + 2 * (size_t)H);
}

extern "C" int rpst_reflect_pad_border_grad(const float* dy, const float* w, float* dx, int N,
                                            int Cin, int Cout, int H, int W, void* workspace,
                                            size_t workspace_bytes, rpst_stream_t stream) {
  return rpst_reflect_pad_border_grad_masked(dy, w, nullptr, dx, N, Cin, Cout, H, W, workspace,
                                             workspace_bytes, stream);
}

extern "C" int rpst_reflect_pad_border_grad_masked(const float* dy, const float* w,
                                                   const float* mask, float* dx, int N, int Cin,
                                                   int Cout, int H, int W, void* workspace,
                                                   size_t workspace_bytes, rpst_stream_t stream) {
  RPST_REQUIRE(dy && w && dx && N > 0 && Cin > 0 && Cout > 0, "reflect_border_grad: bad args");
  RPST_REQUIRE(H >= 2 && W >= 2, "reflect_border_grad: ReflectionPad2d(1) needs H, W >= 2");
  if (!workspace || workspace_bytes < rpst_reflect_pad_border_grad_workspace_size(N, Cin, H, W)) {
    set_error("reflect_border_grad: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* ring = static_cast<float*>(workspace);
  const int ks = ring_splits(Cout);
  RPST_REQUIRE((int64_t)N * 4 * ks <= 65535, "reflect_border_grad: batch too large");
  const int umax = (W + 2 > H ? W + 2 : H);
  reflect_ring_kernel<<<dim3((umax + 63) / 64, (Cin + 63) / 64, N * 4 * ks), 256, 0, st>>>(
      dy, w, ring, N, Cin, Cout, H, W, ks);
  if (int e = launch_status("reflect_ring_kernel")) return e;
  const int r0 = 1, r1 = H - 2, c0 = 1, c1 = W - 2;
  const int nrows = (r0 == r1) ? 1 : 2, ncols = (c0 == c1) ? 1 : 2;
  const int64_t per = (int64_t)nrows * W + (int64_t)ncols * (H - nrows);
  reflect_fold_kernel<<<blocks_for((int64_t)N * Cin * per), 256, 0, st>>>(
      ring, dx, mask, N, Cin, H, W, nrows, r0, r1, ncols, c0, c1, ks);
  return launch_status("reflect_fold_kernel");
}

// channel tile of the wgrad kernel: 32 when both channel counts fit one (no padded waves)
static int wgrad_tc(int Cin, int Cout) {
  static const int force = [] {
    const char* e = std::getenv("RPST_WGRAD_TC");  // A/B switch: 64 forces the wide tiles
    return e ? std::atoi(e) : 0;
  }();
  if (force == 64) return 64;
  // both <= 32, or one side <= 8 (a 64-wide tile would run >= 7/8 of its rows or columns
  // on padding: the decoders' 64->3 / 16->3 last convs)
  return (Cin <= 32 && Cout <= 32) || Cin <= 8 || Cout <= 8 ? 32 : 64;
}

static void wgrad_geometry(int N, int Cin, int H, int W, int Cout, int* splits,
                           int64_t* segs_per_split) {
  const int tc = wgrad_tc(Cin, Cout), px = 4096 / tc;
  const int tiles = ((Cout + tc - 1) / tc) * ((Cin + tc - 1) / tc);
  const int64_t segs = (int64_t)N * H * ((W + px - 1) / px);
  // ~1024 workgroups in all, at least 4 segments each
  int64_t s = (1024 + tiles - 1) / tiles;
  if (s > segs / 4) s = segs / 4;
  if (s < 1) s = 1;
  *segs_per_split = (segs + s - 1) / s;
  *splits = (int)((segs + *segs_per_split - 1) / *segs_per_split);
}

extern "C" size_t rpst_conv_wgrad_workspace_size(int N, int Cin, int H, int W, int Cout) {
  if (N <= 0 || Cin <= 0 || H <= 0 || W <= 0 || Cout <= 0) return 0;
  int splits;
  int64_t sps;
  wgrad_geometry(N, Cin, H, W, Cout, &splits, &sps);
  const size_t kspl = wgrad_tc(Cin, Cout) == 32 ? 4 : 1;
  return sizeof(float) * (size_t)splits * Cout * (kspl * Cin * 9 + 1);
}

extern "C" int rpst_conv_wgrad_pad(const float* x, const float* dy, float* dw, float* db,
                                   int N, int Cin, int H, int W, int Cout, int pad,
                                   void* workspace, size_t workspace_bytes,
                                   rpst_stream_t stream) {
  RPST_REQUIRE(x && dy && dw && N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0,
               "conv_wgrad: bad args");
  RPST_REQUIRE(pad == RPST_PAD_ZERO || pad == RPST_PAD_REFLECT, "conv_wgrad: bad pad mode");
  RPST_REQUIRE(pad != RPST_PAD_REFLECT || (H >= 2 && W >= 2),
               "conv_wgrad: reflect padding needs H, W >= 2");
  const int reflect = pad == RPST_PAD_REFLECT;
  if (!workspace || workspace_bytes < rpst_conv_wgrad_workspace_size(N, Cin, H, W, Cout)) {
    set_error("conv_wgrad: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  int splits;
  int64_t sps;
  wgrad_geometry(N, Cin, H, W, Cout, &splits, &sps);
  const int tc = wgrad_tc(Cin, Cout), kspl = tc == 32 ? 4 : 1;
  const int tiles = ((Cout + tc - 1) / tc) * ((Cin + tc - 1) / tc);
  RPST_REQUIRE(tiles <= 65535 * 64 && splits <= 65535, "conv_wgrad: grid too large");
  float* part = static_cast<float*>(workspace);
  float* bpart = part + (size_t)splits * kspl * Cout * Cin * 9;
  RPST_REQUIRE((int64_t)(Cout > Cin ? Cout : Cin) * H * W * 4 < (1LL << 31),
               "conv_wgrad: one image's tensor exceeds 2 GiB");
  const bool vec = (W % 4) == 0;
  const dim3 grid(tiles, splits);
  float* bp = db ? bpart : nullptr;
  if (tc == 32) {
    if (vec) conv_wgrad_kernel<true, 32><<<grid, 256, 0, st>>>(x, dy, part, bp, N, Cin, H, W, Cout, sps, reflect);
    else conv_wgrad_kernel<false, 32><<<grid, 256, 0, st>>>(x, dy, part, bp, N, Cin, H, W, Cout, sps, reflect);
  } else {
    if (vec) conv_wgrad_kernel<true, 64><<<grid, 256, 0, st>>>(x, dy, part, bp, N, Cin, H, W, Cout, sps, reflect);
    else conv_wgrad_kernel<false, 64><<<grid, 256, 0, st>>>(x, dy, part, bp, N, Cin, H, W, Cout, sps, reflect);
  }
  if (int e = launch_status("conv_wgrad_kernel")) return e;
  const int64_t n = (int64_t)Cout * Cin * 9;
  wgrad_reduce_kernel<<<blocks_for(n), 256, 0, st>>>(part, dw, n, splits * kspl);
  if (int e = launch_status("wgrad_reduce_kernel")) return e;
  if (db) {
    wgrad_reduce_kernel<<<blocks_for(Cout), 256, 0, st>>>(bpart, db, Cout, splits);
    return launch_status("wgrad_reduce_kernel(bias)");
  }
  return RPST_OK;
}

extern "C" int rpst_conv_wgrad(const float* x, const float* dy, float* dw, float* db, int N,
                               int Cin, int H, int W, int Cout, void* workspace,
                               size_t workspace_bytes, rpst_stream_t stream) {
  return rpst_conv_wgrad_pad(x, dy, dw, db, N, Cin, H, W, Cout, RPST_PAD_ZERO, workspace,
                             workspace_bytes, stream);
}

extern "C" int rpst_adain_backward(const float* g, const float* c, const float* s,
                                   const float* stats, float* dc, float* ds, int planes,
                                   int64_t HW, void* workspace, size_t workspace_bytes,
                                   rpst_stream_t stream) {
  RPST_REQUIRE(g && c && s && stats && dc && ds && planes > 0 && HW > 1,
               "adain_backward: bad args");
  if (!workspace || workspace_bytes < sizeof(float) * 2 * (size_t)planes) {
    set_error("adain_backward: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* sums = static_cast<float*>(workspace);
  adain_backward_reduce_kernel<<<planes, 256, 0, st>>>(g, c, stats, sums, planes, HW);
  if (int e = launch_status("adain_backward_reduce_kernel")) return e;
  adain_backward_apply_kernel<<<blocks_for((int64_t)planes * HW), 256, 0, st>>>(
      g, c, s, stats, sums, dc, ds, planes, HW);
  return launch_status("adain_backward_apply_kernel");
}

extern "C" int rpst_style_content_loss_grad(const float* F, const float* Fc, const float* stats,
                                            const float* weights, float* out, int planes,
                                            int64_t HW, int accumulate, rpst_stream_t stream) {
  RPST_REQUIRE(F && stats && weights && out && planes > 0 && HW > 1, "loss_grad: bad args");
  loss_seed_kernel<<<blocks_for((int64_t)planes * HW), 256, 0, as_stream(stream)>>>(
      F, Fc, stats, weights, out, planes, HW, accumulate);
  return launch_status("loss_seed_kernel");
}

extern "C" size_t rpst_sq_diff_workspace_size(void) { return sizeof(double) * 1024; }

extern "C" int rpst_sq_diff_sum(const float* a, const float* b, int64_t n, double scale,
                                float* out, void* workspace, size_t workspace_bytes,
                                rpst_stream_t stream) {
  RPST_REQUIRE(a && b && out && n > 0, "sq_diff_sum: bad args");
  if (!workspace || workspace_bytes < rpst_sq_diff_workspace_size()) {
    set_error("sq_diff_sum: workspace too small");
    return RPST_EWORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  int64_t nb = (n + 255) / 256;
  const int parts = (int)(nb < 1024 ? nb : 1024);
  double* part = static_cast<double*>(workspace);
  sq_diff_partial_kernel<<<parts, 256, 0, st>>>(a, b, part, n);
  if (int e = launch_status("sq_diff_partial_kernel")) return e;
  sq_diff_final_kernel<<<1, 256, 0, st>>>(part, parts, scale, out);
  return launch_status("sq_diff_final_kernel");
}
