// Winograd F(4x4, 3x3) convolution on fp32 MFMA (gfx950) for the large 3x3 layers of the
// reference hot path (network/base.py:25-111,363-396; sanet.py:162-192): 36 multiplies per
// 4x4 output tile and (ci, co) instead of the 144 of the direct convolution (F(2x2,3x3) in
// rpst_wino.hip needs 64 per 4x4 outputs). Lavin & Gray 2016 with the points 0, +-1, +-2:
//
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A      g: 3x3 filter, d: 6x6 input tile (stride 4)
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
//
// Everything is fp32 (true fp32 MFMA, U = G g G^T evaluated in fp64 and rounded once); the
// larger transform coefficients cost accuracy against F(2x2): ~2e-6 rel-L2 against an fp64
// convolution at Cin = 128 (direct fp32: 4e-7), inside the 1e-5 bar of a single conv
// (tests/test_gpu_kernels.py, fixture conv_algo).
//
// Block = 8 waves, two per SIMD: an output region of 16 rows x 64 columns = 4 x 16
// Winograd tiles and 32 output channels. Wave w owns tile row w & 3 and the 16 channels of
// half w >> 2: 16 tiles x 16 channels x all 36 transformed positions = 144 accumulator
// registers, so the output transform is lane-local (no exchange). Per K step of 4 channels
// a lane (k = lane >> 4, tile n = lane & 15) reads its 6x6 input window from the LDS patch,
// transforms it to V (144 VALU), and issues 36 v_mfma_f32_16x16x4_f32 (one per position):
// A = U (LDS, one ds_read_b128 per 4 MFMAs), B = V.
// Per chunk of 8 channels: the raw patch of the NEXT chunk is loaded into registers and the
// next weight slice (36 KiB) streams into LDS by LDS-DMA while this chunk computes; one
// barrier per chunk. One block loops over the co tiles of its spatial tile (a.persist).
#include "rpst_conv.h"

namespace rpst {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kW4CK = 8;                   // input channels per chunk
constexpr int kW4BM = 32;                  // output channels per co tile
constexpr int kW4TH = 16, kW4TW = 64;      // output rows x columns per block
constexpr int kW4PH = kW4TH + 2;           // patch rows
constexpr int kW4PS = 68;                  // patch row stride (floats, 16-B aligned rows)
constexpr int kW4CS = 1280;                // patch channel stride (= 0 mod 64 banks)
constexpr int kW4PATCH = kW4CK * kW4CS;    // floats per patch buffer
constexpr int kW4WCH = 36 * kW4BM * kW4CK; // weight floats per (co tile, chunk) = 9216
constexpr int kW4NTH = 512;
static_assert(kW4PH * kW4PS <= kW4CS, "patch channel fits its stride");
static_assert(kW4WCH % (64 * 4) == 0, "weight slice = whole 1-KiB LDS-DMA pieces");

// ---- weight transform + packing -------------------------------------------------------
// packed[(((((ct * nch + c) * 2 + s) * 2 + mt) * 9 + q) * 64 + l) * 4 + e] = U_xi[co][ci]
// with xi = 4q + e (= 6 i + jj), co = ct*32 + mt*16 + (l & 15), ci = c*8 + 4s + (l >> 4):
// lane l's A operands of positions 4q..4q+3 are one 16-B word, and one (co tile, chunk)
// slice is contiguous (the LDS-DMA copies it verbatim).
__global__ void wino4_pack_kernel(const float* __restrict__ w, float* __restrict__ pk, int Cout,
                                  int Cin, int nch, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int e = (int)(t & 3);
  int64_t r = t >> 2;
  const int l = (int)(r & 63);
  r >>= 6;
  const int q = (int)(r % 9);
  r /= 9;
  const int mt = (int)(r & 1);
  r >>= 1;
  const int s = (int)(r & 1);
  r >>= 1;
  const int c = (int)(r % nch);
  const int ct = (int)(r / nch);
  const int xi = 4 * q + e;
  const int i = xi / 6, jj = xi % 6;
  const int co = ct * kW4BM + mt * 16 + (l & 15);
  const int ci = c * kW4CK + 4 * s + (l >> 4);
  float v = 0.f;
  if (co < Cout && ci < Cin) {
    const double G[6][3] = {{0.25, 0, 0},
                            {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                            {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                            {1.0 / 24, 1.0 / 12, 1.0 / 6},
                            {1.0 / 24, -1.0 / 12, 1.0 / 6},
                            {0, 0, 1}};
    const float* g = w + ((int64_t)co * Cin + ci) * 9;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int p = 0; p < 3; ++p) acc += G[i][u] * (double)g[u * 3 + p] * G[jj][p];
    v = (float)acc;
  }
  pk[t] = v;
}

size_t wino4_packed_floats(int Cout, int Cin) {
  const size_t co_tiles = (size_t)(Cout + kW4BM - 1) / kW4BM;
  const size_t nch = (size_t)(Cin + kW4CK - 1) / kW4CK;
  return co_tiles * nch * kW4WCH;
}

int wino4_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st) {
  const int nch = (Cin + kW4CK - 1) / kW4CK;
  const int64_t t = (int64_t)wino4_packed_floats(Cout, Cin);
  wino4_pack_kernel<<<(unsigned)((t + 255) / 256), 256, 0, st>>>(w, pk, Cout, Cin, nch, t);
  return launch_status("wino4_pack_kernel");
}

bool wino4_supports(int in_op) {
  return in_op == RPST_IN_NONE || in_op == RPST_IN_ADAIN || in_op == RPST_IN_UPSAMPLE2;
}
// padding offsets (rpst_wino4 loader): (Cin + 8) planes + 2 x Cin planes < 2^32 bytes
bool wino4_fits(int N, int Cin, int Hs, int Ws, int in_op) {
  (void)N;
  (void)in_op;
  const int64_t plane = (int64_t)Hs * Ws * 4;
  return (int64_t)(3 * Cin + 8) * plane < (1LL << 32) - (1LL << 20);
}
int wino4_persist() {
  const char* e = getenv("RPST_WINO4_PERSIST");  // A/B switch
  return (e && *e) ? atoi(e) != 0 : 1;
}

// B^T row transform of one 6-vector (in place): the shared terms of rows (1,2) and (3,4)
__device__ __forceinline__ void bt6(float& d0, float& d1, float& d2, float& d3, float& d4,
                                    float& d5) {
  const float A = fmaf(-4.f, d2, d4), B = fmaf(-4.f, d1, d3);
  const float C = d4 - d2, E = d3 - d1;
  const float t0 = fmaf(4.f, d0, fmaf(-5.f, d2, d4));
  const float t5 = fmaf(4.f, d1, fmaf(-5.f, d3, d5));
  d0 = t0;
  d1 = A + B;
  d2 = A - B;
  d3 = fmaf(2.f, E, C);
  d4 = fmaf(-2.f, E, C);
  d5 = t5;
}

// A^T applied to one 6-vector -> 4 values
__device__ __forceinline__ void at6(const float (&m)[6], float (&p)[4]) {
  const float s12 = m[1] + m[2], d12 = m[1] - m[2];
  const float s34 = m[3] + m[4], d34 = m[3] - m[4];
  p[0] = (m[0] + s12) + s34;
  p[1] = fmaf(2.f, d34, d12);
  p[2] = fmaf(4.f, s34, s12);
  p[3] = fmaf(8.f, d34, d12) + m[5];
}

// branch-free padding resolution (resolve() in rpst_conv.h, as selects): reflect(1) or
// zero padding; false for a zero-padding position, v clamped into [0, n) either way
__device__ __forceinline__ bool resolve_bf(int& v, int n, bool zero_pad) {
  const bool in = v >= 0 && v < n;
  const int r = reflect1(v, n);
  v = zero_pad ? min(max(v, 0), n - 1) : r;
  return in || !zero_pad;
}

template <int INOP, bool PERSIST>
__global__ __launch_bounds__(kW4NTH, 1) void wino4_mfma_kernel(ConvArgs a) {
  static_assert(RawN<INOP>::R == 1, "one raw load per patch element");
  __shared__ __attribute__((aligned(16))) float smem[2 * kW4PATCH + 2 * kW4WCH];
  float* const wl = smem + 2 * kW4PATCH;

  // block -> (column tile, row tile, image), XCD-swizzled (neighbouring spatial tiles share
  // halo rows and every block of an XCD streams the same weight slices through its L2)
  int bid = xcd_swizzle(blockIdx.x, (int)gridDim.x), ct0 = 0;
  if (!PERSIST) {
    ct0 = bid % a.co_tiles;
    bid /= a.co_tiles;
  }
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int n = bid / a.tiles_y;
  const int nct = PERSIST ? a.co_tiles : 1;
  const int nch = a.nchunks, G = nct * nch;
  const int y0 = ty * kW4TH, x0 = tx * kW4TW;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = lane >> 4, tn = lane & 15;
  const int wr = wave & 3, wm = wave >> 2;  // tile row, channel half

  const bool pooled = INOP == RPST_IN_UPSAMPLE2;
  const unsigned in_plane = pooled ? (unsigned)(a.Hs * a.Ws) : (unsigned)(a.H * a.W);
  // out-of-range offset for a padding position: the image's byte size, added either to
  // the column (VGPR) or the row (SGPR) part; wino4_launch checks that two of them plus the
  // largest channel offset stay below 2^32
  const unsigned oob = a.Cin * in_plane * 4u;
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (int64_t)n * a.Cin * in_plane), (short)0, (int)oob, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wpk, (short)0, (int)((unsigned)(a.co_tiles * nch * kW4WCH) * 4u), 0x00020000);

  // patch loader: wave -> channel cg of the chunk, lane -> column x0 + lane of all 18 patch
  // rows (one 256-B row segment per wave-instruction); lanes < 36 also load one halo
  // element (row lane >> 1, left / right). Row offsets are wave-uniform (soffset), column
  // offsets per lane; a zero-padding position reads out of range (returns 0).
  const int cg = wave;
  const bool zp = a.pad == RPST_PAD_ZERO;
  const int rs = pooled ? a.Ws : a.W;  // source row stride
  int bx = x0 + lane;
  const bool okx = resolve_bf(bx, a.W, zp);
  const unsigned cx = okx ? (unsigned)(pooled ? bx >> 1 : bx) * 4u : oob;
  const bool has_halo = lane < 2 * kW4PH;
  const int hrw = lane >> 1;  // halo patch row
  int hy = y0 - 1 + (has_halo ? hrw : 0), hx = (lane & 1) ? x0 + kW4TW : x0 - 1;
  const bool h_ok = has_halo && resolve_bf(hy, a.H, zp) && resolve_bf(hx, a.W, zp);
  const unsigned hoff =
      h_ok ? ((unsigned)((pooled ? hy >> 1 : hy) * rs) + (unsigned)(pooled ? hx >> 1 : hx)) * 4u
           : oob;
  const int hcol = (lane & 1) ? kW4TW + 1 : 0;

  float X[kW4PH + 1];
  AdainP ap{};

  auto load = [&](int c) {
    const unsigned ch = (unsigned)(c * kW4CK + cg);
    const unsigned pb = ch * in_plane * 4u;  // >= the range for a padding channel
    const unsigned v0 = pb + cx;
    if constexpr (INOP == RPST_IN_ADAIN) ap = adain_params(a.aux, n, (int)ch, a);
#pragma unroll
    for (int py = 0; py < kW4PH; ++py) {
      int y = y0 - 1 + py;
      const bool yok = resolve_bf(y, a.H, zp);
      const int ro = __builtin_amdgcn_readfirstlane(yok ? (int)((pooled ? y >> 1 : y) * rs * 4)
                                                        : (int)oob);
      X[py] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rin, (int)v0, ro, 0));
    }
    X[kW4PH] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rin, (int)(pb + hoff), 0, 0));
  };
  // AdaIN on load: ((v - mean_c) / std_c) * std_s + mean_s, zero at padding positions
  auto comb = [&](float v, bool ok) {
    if constexpr (INOP == RPST_IN_ADAIN) return ok ? fmaf(v - ap.mc, ap.scale, ap.ms) : 0.f;
    else return v;
  };
  auto store = [&](int c, float* pbuf) {
    float* xs = pbuf + cg * kW4CS;
    const bool chok = c * kW4CK + cg < a.Cin;
#pragma unroll
    for (int py = 0; py < kW4PH; ++py) {
      int y = y0 - 1 + py;
      const bool rok = chok && resolve_bf(y, a.H, zp);
      xs[py * kW4PS + 1 + lane] = comb(X[py], rok && okx);
    }
    const float hv = comb(X[kW4PH], chok && h_ok);
    if (has_halo) xs[hrw * kW4PS + hcol] = hv;
  };
  // weight slice of (co tile ct, chunk c) -> LDS by LDS-DMA: 36 pieces of 1 KiB over 8 waves
  auto wdma = [&](int ct, int c, float* wbuf) {
    const unsigned base = (unsigned)((ct * nch + c) * kW4WCH) * 4u + (unsigned)lane * 16u;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int p = wave + 8 * i;
      if (i < 4 || p < 36)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(wbuf + p * 256), 16,
                                                 (int)(base + (unsigned)p * 1024u), 0, 0, 0);
    }
  };

  floatx4 acc[36];
#pragma unroll
  for (int x = 0; x < 36; ++x) acc[x] = floatx4{0.f, 0.f, 0.f, 0.f};

  // one chunk: 2 K steps of 4 channels, each 144 VALU of input transform + 36 MFMAs
  auto compute = [&](const float* pbuf, const float* wbuf) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float* pr = pbuf + (4 * s + k) * kW4CS + 4 * wr * kW4PS + 4 * tn;
      float d[6][6];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const float4 u = *reinterpret_cast<const float4*>(pr + r * kW4PS);
        const float4 v = *reinterpret_cast<const float4*>(pr + r * kW4PS + 4);
        d[r][0] = u.x;
        d[r][1] = u.y;
        d[r][2] = u.z;
        d[r][3] = u.w;
        d[r][4] = v.x;
        d[r][5] = v.y;
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) bt6(d[0][c], d[1][c], d[2][c], d[3][c], d[4][c], d[5][c]);
#pragma unroll
      for (int i = 0; i < 6; ++i) bt6(d[i][0], d[i][1], d[i][2], d[i][3], d[i][4], d[i][5]);
      const float* wq = wbuf + (s * 2 + wm) * 9 * 256 + lane * 4;
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const float4 w4 = *reinterpret_cast<const float4*>(wq + q * 256);
        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int xi = 4 * q + e;
          acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[e], d[xi / 6][xi % 6], acc[xi], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the next K step's reads below these MFMAs
    }
  };

  // output transform, bias, activation, store and the optional per-wave statistics of one
  // co tile; lane (k, tn) holds channels co0 + 16 wm + 4k + r of tile (wr, tn)
  const int gy0 = y0 + 4 * wr, gx0 = x0 + 4 * tn;
  const bool vec = (a.W & 3) == 0 && gx0 + 3 < a.W;
  auto epilogue = [&](int ct) {
    const int rows = max(0, min(4, a.H - gy0)), cols = max(0, min(kW4TW, a.W - x0));
    const int cnt = rows * cols;
    const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float P[6][4];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        float m[6];
#pragma unroll
        for (int jj = 0; jj < 6; ++jj) m[jj] = acc[6 * i + jj][r];
        at6(m, P[i]);
      }
      float Y[4][4];
#pragma unroll
      for (int xx = 0; xx < 4; ++xx) {
        float m[6], p[4];
#pragma unroll
        for (int i = 0; i < 6; ++i) m[i] = P[i][xx];
        at6(m, p);
#pragma unroll
        for (int yy = 0; yy < 4; ++yy) Y[yy][xx] = p[yy];
      }
      const int co = ct * kW4BM + 16 * wm + 4 * k + r;
      const bool cok = co < a.Cout;
      const float b = (a.bias && cok) ? a.bias[co] : 0.f;
      float sum = 0.f;
#pragma unroll
      for (int yy = 0; yy < 4; ++yy)
#pragma unroll
        for (int xx = 0; xx < 4; ++xx) {
          const float v = activate(Y[yy][xx] + b, a.relu);
          Y[yy][xx] = v;
          sum += (yy < rows && gx0 + xx < a.W) ? v : 0.f;
        }
      if (cok) {
        float* o = a.out + (((int64_t)n * a.Cout + co) * a.H + gy0) * a.W + gx0;
#pragma unroll
        for (int yy = 0; yy < 4; ++yy) {
          if (yy < rows) {
            if (vec) {
              *reinterpret_cast<float4*>(o + yy * a.W) =
                  make_float4(Y[yy][0], Y[yy][1], Y[yy][2], Y[yy][3]);
            } else {
#pragma unroll
              for (int xx = 0; xx < 4; ++xx)
                if (gx0 + xx < a.W) o[yy * a.W + xx] = Y[yy][xx];
            }
          }
        }
      }
      if (a.stat_part) {
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) sum += __shfl_xor(sum, m, 64);
        const float mean = sum * inv;
        float m2 = 0.f;
#pragma unroll
        for (int yy = 0; yy < 4; ++yy)
#pragma unroll
          for (int xx = 0; xx < 4; ++xx) {
            const float dv = Y[yy][xx] - mean;
            m2 += (yy < rows && gx0 + xx < a.W) ? dv * dv : 0.f;
          }
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) m2 += __shfl_xor(m2, m, 64);
        if (tn == 0 && cok)
          a.stat_part[((int64_t)n * a.Cout + co) * a.stat_P + (ty * a.tiles_x + tx) * 4 + wr] =
              make_float2(mean, m2);
      }
    }
  };

  // ---- pipeline: chunk g computes from buffers g & 1 while chunk g + 1 is fetched -------
  load(0);
  wdma(ct0, 0, wl);
  store(0, smem);
  for (int g = 0; g < G; ++g) {
    const int b = g & 1;
    __syncthreads();  // chunk g's patch and weights are in LDS; buffers b ^ 1 are free
    const int gn = g + 1;
    const bool more = gn < G;
    const int ctn = ct0 + gn / nch, cn = gn % nch;
    if (more) {
      load(cn);
      wdma(ctn, cn, wl + (b ^ 1) * kW4WCH);
    }
    compute(smem + b * kW4PATCH, wl + b * kW4WCH);
    if (gn % nch == 0) {
      epilogue(ct0 + g / nch);
#pragma unroll
      for (int x = 0; x < 36; ++x) acc[x] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (more) store(cn, smem + (b ^ 1) * kW4PATCH);
  }
}

int wino4_launch(ConvArgs& a, int in_op, hipStream_t st) {
  RPST_REQUIRE(wino4_supports(in_op), "conv2d: winograd4 does not support in_op %d", in_op);
  RPST_REQUIRE(a.res == nullptr, "conv2d: winograd4 has no residual epilogue");
  RPST_REQUIRE(wino4_fits(a.N, a.Cin, a.Hs, a.Ws, in_op), "conv2d: image too large for winograd4");
  a.Cout_pad = (a.Cout + kW4BM - 1) / kW4BM * kW4BM;
  a.nchunks = (a.Cin + kW4CK - 1) / kW4CK;
  a.tiles_x = (a.W + kW4TW - 1) / kW4TW;
  a.tiles_y = (a.H + kW4TH - 1) / kW4TH;
  a.co_tiles = a.Cout_pad / kW4BM;
  a.stat_P = a.tiles_x * a.tiles_y * 4;
  a.persist = wino4_persist();
  RPST_REQUIRE((int64_t)a.co_tiles * a.nchunks * kW4WCH * 4 < (1LL << 31),
               "conv2d: winograd4 weight image exceeds 2 GiB");
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.N * (a.persist ? 1 : a.co_tiles);
  RPST_REQUIRE(blocks <= 0x7fffffffLL, "conv2d: grid too large");
  const unsigned nb = (unsigned)blocks;
#define RPST_W4_GO(OP)                                                                     \
  (a.persist ? (void)(wino4_mfma_kernel<OP, true><<<nb, kW4NTH, 0, st>>>(a))                \
             : (void)(wino4_mfma_kernel<OP, false><<<nb, kW4NTH, 0, st>>>(a)))
  switch (in_op) {
    case RPST_IN_ADAIN: RPST_W4_GO(RPST_IN_ADAIN); break;
    case RPST_IN_UPSAMPLE2: RPST_W4_GO(RPST_IN_UPSAMPLE2); break;
    default: RPST_W4_GO(RPST_IN_NONE);
  }
#undef RPST_W4_GO
  return launch_status("wino4_mfma_kernel");
}

}  // namespace rpst
