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
// Winograd tiles and 32 output channels. Wave w owns tile row w & 3 and the transformed
// rows 3h..3h+2 (h = w >> 2) of all 32 channels: 16 tiles x 32 channels x 18 positions =
// 144 accumulator registers. Per K step of 4 channels a lane (k = lane >> 4, tile
// n = lane & 15) reads 5 rows of its 6x6 input window from the LDS patch, forms its three
// rows of V = B^T d B (72 VALU) and issues 36 v_mfma_f32_16x16x4_f32 (18 positions x 2
// channel halves sharing each V value): A = U (LDS, one ds_read_b128 per 4 MFMAs).
// Per K step the patch (4 channels x 18 rows x 68) and the weight slice (18 KiB) stream
// into a 4-stage LDS ring by LDS-DMA three steps ahead (step g + 3 issued inside step g's
// MFMA stream; per-lane patch offsets resolved against the padding once per block); one
// counted vmcnt wait and one barrier per step. One block loops over the co tiles of its
// spatial tile (split over two same-XCD blocks for Cin >= 128: a.cosplit).
// The output transform splits like the positions: each wave applies A^T . A to its three
// rows (a partial 4x4 tile), the two waves of a tile row swap the partials of the channel
// half the other one finishes through LDS, and each adds, biases, activates and stores 16
// channels. The fp32 MFMA and the VALU do not co-execute on a SIMD (tools/coexec.hip), so
// the design minimises VALU per MFMA; measured alternatives and their timings:
// profiles/r01_wino4_variants.log, profiles/r02_wino4_variants.log.
#include "rpst_conv.h"
#ifndef RPST_W4_CPOL
#define RPST_W4_CPOL 0  // output-store cache policy (aux bits of buffer_store), A/B only
#endif
#include "rpst_wct.h"

#include <type_traits>

namespace rpst {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kW4CK = 8;                   // input channels per chunk
#ifndef RPST_W4DBG
#define RPST_W4DBG 0
#endif
// DMA of step g + 3 issued inside step g's MFMA stream (its address SALU then issues
// beside the matrix pipe): weights after MFMA pair RPST_W4_HW, patch after RPST_W4_HP
// (-1: before the input transform). 0 / 2 measured best (profiles/r02_wino4_variants.log)
#ifndef RPST_W4_HW
#define RPST_W4_HW 0
#endif
#ifndef RPST_W4_HP
#define RPST_W4_HP 2
#endif
#ifndef RPST_W4_AHEAD  // MFMA groups whose A operands are read ahead (NR = 4; NR = 2: 3)
// 2: 64->128 N64 8.17 -> 8.02 ms, 32->64 2.57 -> 2.50, 64->32 1.15 -> 1.11 against 3; NR = 2's
// 16->32 / 32->16 measured 0.005 ms slower at 2 (tools/ab_bench_libs.sh, profiles/r05/ahead_ab.log)
#define RPST_W4_AHEAD 2
#endif
#ifndef RPST_W4_HW2  // the same issue slots for the NR = 2 form
#define RPST_W4_HW2 RPST_W4_HW
#endif
#ifndef RPST_W4_HP2
#define RPST_W4_HP2 RPST_W4_HP
#endif
#ifndef RPST_W4_ORDER  // spatial block order (w4_tile): 3 = row tile fastest (round 5)
#define RPST_W4_ORDER 3
#endif
constexpr int kW4BM = 32;                  // output channels per co tile
constexpr int kW4TH = 16, kW4TW = 64;      // output rows x columns per block
constexpr int kW4PH = kW4TH + 2;           // patch rows
constexpr int kW4PS = 68;                  // patch row stride (floats): 66 columns + 2 spare
// window columns 4-7 read as a second ds_read_b128 (round 6) instead of 4-5 as a b64: the b64
// reads of the four channel groups k of a wave hit the same banks (channel stride 768 floats
// = 0 mod 64 banks): 13-17 % of LDS cycles bank-conflicted on the small-Cin layers
// (profiles/r05_sq_layers.csv), 0 % with the b128 (profiles/r06/sq_rd128.log); layer times
// unchanged within noise (32->64 2.52 / 2.55 ms, 64->128 7.91 / 7.93, profiles/r06/rd128_ab.log)
#ifndef RPST_W4_RD128
#define RPST_W4_RD128 1
#endif
constexpr int kW4CS = 1280;                // channel stride (floats)
constexpr int kW4DMA = 20;                 // 4-B LDS-DMA pieces per patch channel (64 floats)
constexpr int kW4DMA4 = 5;                 // 16-B pieces (256 floats) on interior blocks
constexpr int kW4WCH = 36 * kW4BM * kW4CK; // weight floats per (co tile, 8-channel chunk) = 9216
// LDS ring of 4 stages, one K step (4 input channels) each: patch [4][1280] + weights
// [2 halves][9][64 lanes][4] = 4608; plus a 1 KiB target for the padding DMA pieces
constexpr int kW4SPATCH = 4 * kW4CS;       // 5120
constexpr int kW4SW = kW4WCH / 2;          // 4608
constexpr int kW4STAGE = kW4SPATCH + kW4SW;  // 9728 floats = 38 KiB
constexpr int kW4AffC = 512;               // ADAIN: input channels whose parameters fit LDS
constexpr int kW4NTH = 512;
static_assert(kW4PH * kW4PS <= kW4DMA * 64 && kW4DMA * 64 <= kW4CS, "patch channel pieces");
static_assert(kW4PH * kW4PS <= kW4DMA4 * 256 && kW4DMA4 * 256 <= kW4CS && kW4PS % 4 == 0,
              "16-B pieces never straddle a patch row");
static_assert(kW4WCH % (64 * 4) == 0, "weight slice = whole 1-KiB LDS-DMA pieces");

// Block geometry by tile rows NR: NR = 4 is the block described above (8 waves, 16 output
// rows, 4-stage ring, one block per CU). NR = 2 (layers with few input channels, whose
// 2-16 K steps leave the block prologue and epilogue exposed): 4 waves, 8 output rows, a
// 2-stage ring (DMA one step ahead) in 62 KiB and at most 256 VGPRs, so two blocks share a
// CU and one block's prologue / epilogue runs beside the other's MFMAs. Each wave keeps
// its 16 tiles x 18 positions x 32 channels; per K step the weight slice (18 pieces) is
// split over the 4 waves and each wave streams one whole patch channel.
template <int NR>
struct W4Geo {
  static constexpr int NW = 2 * NR;                 // waves
  static constexpr int NTH = 64 * NW;
  static constexpr int TH = 4 * NR;                 // output rows per block
  static constexpr int PH = TH + 2;                 // patch rows
  static constexpr int NH = NR / 2;                 // waves streaming one patch channel
  static constexpr int CS = NR == 4 ? 1280 : 768;   // patch channel stride (floats)
  static constexpr int DMA = NR == 4 ? 20 : 11;     // 4-B pieces per patch channel
  static constexpr int DMA4 = (PH * 17 + 63) / 64;  // 16-B pieces per patch channel
  static constexpr int SLOW = DMA / NH;             // 4-B pieces per wave
  static constexpr int WIDE = (DMA4 + NH - 1) / NH; // 16-B pieces per wave
  static constexpr int WPI = (18 + NW - 1) / NW;    // weight pieces per wave
  static constexpr int STG = NR == 4 ? 4 : 2;       // ring stages
  static constexpr int SPATCH = 4 * CS;
  static constexpr int STAGE = SPATCH + kW4SW;
  static constexpr int LAUNCH_WPE = NR == 4 ? 1 : 2;  // __launch_bounds__ waves per SIMD
  static_assert(PH * kW4PS <= DMA * 64 && DMA * 64 <= CS && DMA % NH == 0, "4-B pieces");
  static_assert(PH * kW4PS <= DMA4 * 256 && DMA4 * 256 <= CS, "16-B pieces");
  static_assert(NR * 2048 <= STAGE, "epilogue exchange region fits a stage");
};
static_assert(W4Geo<4>::CS == kW4CS && W4Geo<4>::DMA4 == kW4DMA4 && W4Geo<4>::STAGE == kW4STAGE,
              "NR = 4 is the documented block");

// ---- weight transform + packing -------------------------------------------------------
// packed[(((((ct * nch + c) * 2 + s) * 2 + h) * 9 + q) * 64 + l) * 4 + e] = U_xi[co][ci]
// with f = 4q + e, xi = 18 h + (f >> 1) (= 6 i + jj), co = ct*32 + (f & 1)*16 + (l & 15),
// ci = c*8 + 4s + (l >> 4): lane l's A operands of positions 2q, 2q+1 (both channel halves)
// are one 16-B word, and one (co tile, chunk) slice is contiguous (the LDS-DMA copies it
// verbatim).
// TW = float (the layer's weights) or double (per-image folded weights, wino4_mix): image
// b's weights at w + b * Cout * Cin * 9 pack to pk + b * per; element (co, ci, tap) of an
// image at co * sco + ci * sci + tap * stap (PyTorch layout: Cin * 9, 9, 1).
template <typename TW>
__global__ void wino4_pack_kernel(const TW* __restrict__ w, float* __restrict__ pk, int Cout,
                                  int Cin, int nch, int64_t per, int64_t total, int64_t sco,
                                  int64_t sci, int64_t stap) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int64_t img = t / per;
  pk += img * per;
  w += img * (int64_t)Cout * Cin * 9;
  t -= img * per;
  const int e = (int)(t & 3);
  int64_t r = t >> 2;
  const int l = (int)(r & 63);
  r >>= 6;
  const int q = (int)(r % 9);
  r /= 9;
  const int h = (int)(r & 1);
  r >>= 1;
  const int s = (int)(r & 1);
  r >>= 1;
  const int c = (int)(r % nch);
  const int ct = (int)(r / nch);
  const int f = 4 * q + e, xi = 18 * h + (f >> 1), mt = f & 1;
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
    const TW* g = w + co * sco + ci * sci;
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int p = 0; p < 3; ++p) acc += G[i][u] * (double)g[(u * 3 + p) * stap] * G[jj][p];
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
  wino4_pack_kernel<float><<<(unsigned)((t + 255) / 256), 256, 0, st>>>(w, pk, Cout, Cin, nch, t, t,
                                                                    (int64_t)Cin * 9, 9, 1);
  return launch_status("wino4_pack_kernel");
}

bool wino4_supports(int in_op) {
  return in_op == RPST_IN_NONE || in_op == RPST_IN_ADAIN || in_op == RPST_IN_UPSAMPLE2;
}
// padding offsets (rpst_wino4 loader): (Cin + 8) planes + 2 x Cin planes < 2^32 bytes
bool wino4_fits(int N, int Cin, int Hs, int Ws, int in_op) {
  (void)N;
  if (in_op == RPST_IN_ADAIN && Cin > kW4AffC) return false;
  const int64_t plane = (int64_t)Hs * Ws * 4;
  return (int64_t)(3 * Cin + 8) * plane < (1LL << 32) - (1LL << 20);
}
int wino4_persist() { return 1; }  // one block per spatial tile loops over the co tiles
// tile rows per block (W4Geo): 2 for the layers with Cin * Cout <= RPST_WINO4_HALF (512: the
// RP stacks' 16->32 and 32->16), 4 otherwise -- a function of the layer's shape only, so an
// image's bits never depend on its batch. tools/ab_env.sh (bench_conv, ms, NR = 4 / NR = 2,
// two rounds): 16->32 N64 1.018 / 0.974, 32->16 N32 0.665 / 0.627, 32->64 N64 2.506 / 2.585,
// 64->32 N32 1.115 / 1.105, 64->128 N64 8.03 / 8.34 (profiles/r03/wino4_half_ab.log): the
// second block per CU overlaps little, and de-phasing the two (the second-resident blocks
// of the first dispatch round sleeping 16k / 36k cycles first) changed nothing (16->32
// 0.970 / 0.976 / 0.969 ms, profiles/r03/wino4_half_ab.log): the small layers are not bound
// by exposed prologues. Only the two smallest layers switch. Round 5 (A operands read 2
// groups ahead at NR = 4): 64->32 N32 1.10 -> 1.06 ms at NR = 2 (32->64 2.50 either way), so
// layers with <= 32 output channels switch up to Cin * Cout = 2048 (profiles/r05/half_ab.log).
int wino4_rows(int Cin, int Cout, int in_op) {
  static const int lim = [] {  // RPST_WINO4_HALF: the product threshold alone (A/B)
    const char* e = getenv("RPST_WINO4_HALF");
    return (e && *e) ? atoi(e) : -1;
  }();
  if (wino4q_applies(Cin, Cout, in_op)) return 2;  // rpst_wino4q.hip: 8 output rows
  const int64_t cc = (int64_t)Cin * Cout;
  if (lim >= 0) return cc <= lim ? 2 : 4;
  return cc <= 512 || (Cout <= 32 && cc <= 2048) ? 2 : 4;
}

// B^T row transform of one 6-vector (in place): the shared terms of rows (1,2) and (3,4)
// what the F(4x4) epilogue needs besides the tile (wino4_mfma_kernel's epi_ctx)
struct EpiCtx {
  int W, H, Cout, gy0, gx0, rows, n, sidx, statP;
  bool vec, full, bst, edge, store, pool;
  float inv, slope;      // slope: the activation as max(y, slope y): 0 ReLU, 0.2 LReLU, 1 none
  unsigned voff[4];      // bst: byte offset of output row yy inside a channel plane (or OOB)
  float* out;
  float* oimg;           // bst: image n's output planes, obytes bytes
  unsigned obytes;
  const float* btab;
  float2* statp;
};

// kernel arguments loaded at their use (s_load through an opaque copy of the kernarg
// pointer, so the loads are not hoisted out of the loop that contains the use)
typedef const __attribute__((address_space(4))) ConvArgs* KArgs;
__device__ __forceinline__ KArgs late_args() {
  KArgs p = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
#if __HIP_DEVICE_COMPILE__  // the host pass only emits the launch stub (no "s" registers)
  asm volatile("" : "+s"(p));
#endif
  return p;
}
// buffer resource over `bytes` at p, or over zero records (every access reads 0) if !ok
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_or_zero(const float* p, unsigned bytes, bool ok) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, ok ? (int)bytes : 0, 0x00020000);
}
// sum over the 16 lanes of a DPP row, in every lane: four DPP adds (quad xor 1, quad xor 2,
// half-row mirror, row mirror) instead of four ds_bpermute round trips through the LDS
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// a wave-uniform value made opaque at this point (not hoisted out of the enclosing loop)
__device__ __forceinline__ int launder(int v) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+s"(v));
#endif
  return v;
}

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

// Round 5 (tools/ab_bench_libs.sh, profiles/r05/order_ab.log, configs[1], two rounds): row
// tile fastest with the hardware's round-robin XCD assignment 546.5 / 547.6 img/s against
// 543.1 / 544.1 for the round-4 order 0 swizzled (16->32 0.94 -> 0.88 ms, 64->128 8.02 ->
// 7.90); order 0 unswizzled 545.4 / 544.1, order 3 swizzled 543.7 / 543.5.
#ifndef RPST_W4_SWZ  // 1: consecutive logical blocks on one XCD (xcd_swizzle)
#define RPST_W4_SWZ 0
#endif
__device__ __forceinline__ int w4_block_id() {
  return RPST_W4_SWZ ? xcd_swizzle(blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
}

// spatial tile of logical block b (after the co-split digit): order 0 = column tile fastest,
// then row tile, then image; 1 = image fastest, then column, row; 2 = column, image, row;
// 3 = row, column, image
// (RPST_W4_ORDER at build time: which tiles the resident blocks share). tools/ab_variants.sh,
// two rounds (ms, order 0 / 1 / 2): 128->256 N64 28.46 / 28.86 / 28.37, 64->128 8.00 /
// 8.47 / 7.83, 256->128 N32 13.81 / 14.17 / 13.76, 32->64 2.54 / 2.69 / 2.57; in bench.py
// (with the statistics epilogue) order 2 measured 29.30 ms for 128->256 vs 29.09 for order 0
// and the same AdaIN-RP rate within noise (521.5 vs 520.2 img/s): order 0 stays.
__device__ __forceinline__ void w4_tile(int b, int order, int tiles_x, int tiles_y, int N,
                                        int& tx, int& ty, int& n) {
  if (order == 1) {
    n = b % N;
    b /= N;
    tx = b % tiles_x;
    ty = b / tiles_x;
  } else if (order == 2) {
    tx = b % tiles_x;
    b /= tiles_x;
    n = b % N;
    ty = b / N;
  } else if (order == 3) {  // row tile fastest, then column tile, image
    ty = b % tiles_y;
    b /= tiles_y;
    tx = b % tiles_x;
    n = b / tiles_x;
  } else {
    tx = b % tiles_x;
    b /= tiles_x;
    ty = b % tiles_y;
    n = b / tiles_y;
  }
}

// STATS: the calc_mean_std partials epilogue (a.stat_part); BTAB: the folded per-(n, co)
// border-class bias table (a.btab). Both are template arguments so a plain layer's
// epilogue carries none of their VALU; the two transformed-row halves (ph, waves 0-3 and
// 4-7) run epilogues specialised for their half.
template <int NR, int INOP, bool STATS, bool BTAB, bool RELU>
__global__ __launch_bounds__(W4Geo<NR>::NTH, W4Geo<NR>::LAUNCH_WPE) void wino4_mfma_kernel(ConvArgs a) {
  using Geo = W4Geo<NR>;
  constexpr int S = Geo::STG, NW = Geo::NW, NH = Geo::NH;
  // timing-only experiments (results wrong; tools/build_variants.sh -DRPST_W4DBG=n): 1 no
  // patch DMA, 2 no weight DMA, 8 no input transform, 16 no barriers, 32 no epilogue,
  // 64 no weight LDS reads, 128 no DMA waits
  constexpr int DBG = RPST_W4DBG;
  // DMA placement of step g + 3: before the transform (-1) or after MFMA pair q of step g
  constexpr int kHW = NR == 2 ? RPST_W4_HW2 : RPST_W4_HW, kHP = NR == 2 ? RPST_W4_HP2 : RPST_W4_HP;
  static_assert(RawN<INOP>::R == 1, "one raw load per patch element");
  // one __shared__ object per ring stage: the stage a K step reads and the one its DMA
  // fills are then distinct objects, so the compiler's wait insertion does not drain the
  // in-flight DMA before every LDS read (the loop below is unrolled by the ring size)
  __shared__ __attribute__((aligned(16))) float smem0[Geo::STAGE];
  __shared__ __attribute__((aligned(16))) float smem1[Geo::STAGE];
  __shared__ __attribute__((aligned(16))) float smem2[S > 2 ? Geo::STAGE : 4];
  __shared__ __attribute__((aligned(16))) float smem3[S > 3 ? Geo::STAGE : 4];
  __shared__ __attribute__((aligned(16))) float dummy[256];  // target of padding DMA pieces

  // block -> (column tile, row tile, image), XCD-swizzled (neighbouring spatial tiles share
  // halo rows and every block of an XCD streams the same weight slices through its L2);
  // one block loops over every co tile of its spatial tile
  int bid = w4_block_id();
  // a.cosplit blocks per spatial tile (consecutive logical ids: one XCD, dispatched
  // together, so the patch they all stream is served by that XCD's L2), each looping over
  // co_tiles / cosplit co tiles
  const int cog = bid % a.cosplit;
  bid /= a.cosplit;
  const int nct = a.co_tiles / a.cosplit;
  const int ct0 = cog * nct;
  int tx, ty, n;
  w4_tile(bid, RPST_W4_ORDER, a.tiles_x, a.tiles_y, a.N, tx, ty, n);
  const int nch = a.nchunks, K4 = 2 * nch, G = nct * K4;  // K steps per co tile / in total
  const int y0 = ty * Geo::TH, x0 = tx * kW4TW;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = lane >> 4, tn = lane & 15;
  const int wr = wave % NR, ph = wave / NR;  // tile row, transformed-row half
  // optional static priority (a.persist & 2: waves 4-7, & 4: waves 0-3; RPST_WINO4_PRIO=1/2):
  // with the DMA inside the MFMA stream, equal priorities measured fastest (128->256 28.47
  // vs 28.75 ms with waves 4-7 at priority 1; profiles/r02_wino4_variants.log)
  if ((ph && (a.persist & 2)) || (!ph && (a.persist & 4))) __builtin_amdgcn_s_setprio(1);

  const bool pooled = INOP == RPST_IN_UPSAMPLE2;
  const unsigned in_plane = pooled ? (unsigned)(a.Hs * a.Ws) : (unsigned)(a.H * a.W);
  // out-of-range offset for a padding position: the image's byte size, added to the
  // channel offset (wino4_fits keeps two of them plus the largest channel offset < 2^32)
  const unsigned oob = a.Cin * in_plane * 4u;
  const float* in_img = conv_in_img(a, n, (int64_t)a.Cin * in_plane);
  const unsigned wbytes = (unsigned)(a.co_tiles * nch * kW4WCH) * 4u;
  const float* w_img = a.wpk + (int64_t)n * a.wstride;
  // descriptors per issue: a dead piece (past the last step, or a channel >= Cin) goes
  // through a zero-record descriptor, so it reads 0 whatever its offsets (the range check
  // covers only the per-lane offset, not the uniform soffset)
  // (a __device__ helper: a lambda returning a buffer resource silently drops the kernel's
  // host launch stub)
  // LDS targets are re-derived inside each issue from one laundered wave-uniform offset
  // (launder()): precomputed, the ~50 per-stage piece addresses overflow the scalar
  // registers and come back by a VALU readlane each


  // ---- patch of one K step: 4 channels, [18 rows][68] (66 columns + 2 spare) at channel
  // stride 1280; wave w fills half w & 1 of channel w >> 1. One-load operators (NONE,
  // UPSAMPLE2) stream it by LDS-DMA: on interior blocks (every patch column inside the
  // image, no upsampling) piece p < 5 of a channel = 16 B per lane of patch elements
  // 4 (64 p + l)..+3 (68 = 4 x 17: a piece never straddles a row; the source is only 4-B
  // aligned), half 0 taking pieces 0-2, half 1 pieces 3-4 (+ one padding piece); elsewhere
  // 20 pieces of 4 B per lane (element 64 p + l resolved against the padding), 10 per half.
  // Offsets are computed once per block. ADAIN streams the raw feature the same way and
  // each lane applies the affine in place to the elements its own pieces wrote (fix_own).
  const int chl = wave / NH, hf = wave % NH;
  const bool zp = a.pad == RPST_PAD_ZERO;
  const int rs = pooled ? a.Ws : a.W;  // source row stride
  constexpr bool kAff = INOP == RPST_IN_ADAIN;
  constexpr int kSlow = Geo::SLOW, kWide = Geo::WIDE;
  unsigned poff[kSlow];
  unsigned pvalid = 0;  // bit i: slot i of this lane holds image data (ADAIN's affine applies)
  const bool wide = !pooled && x0 >= 1 && x0 + kW4TW < a.W;
  {
    if (wide) {
#pragma unroll
      for (int i = 0; i < kWide; ++i) {
        const int p = kWide * hf + i;
        const int f = 64 * p + lane, row = min(f / 17, Geo::PH - 1), j = f - (f / 17) * 17;
        int y = y0 - 1 + row;
        const bool ok = p < Geo::DMA4 && f < Geo::PH * 17 && resolve_bf(y, a.H, zp);
        poff[i] = ok ? ((unsigned)(y * rs) + (unsigned)(x0 - 1 + 4 * j)) * 4u : oob;
        pvalid |= ok ? (1u << i) : 0u;
      }
    } else {
#pragma unroll
      for (int i = 0; i < kSlow; ++i) {
        const int f = 64 * (kSlow * hf + i) + lane;
        const int row = min(f / kW4PS, Geo::PH - 1), col = f - (f / kW4PS) * kW4PS;
        int y = y0 - 1 + row, x = x0 - 1 + col;
        const bool oky = resolve_bf(y, a.H, zp), okx = resolve_bf(x, a.W, zp);  // both clamp
        const bool ok = col < kW4TW + 2 && oky && okx;
        poff[i] = ok ? ((unsigned)((pooled ? y >> 1 : y) * rs) + (unsigned)(pooled ? x >> 1 : x)) * 4u
                     : oob;
        pvalid |= ok ? (1u << i) : 0u;
      }
    }
  }
  // ADAIN: (mean_c, std_s / std_c, mean_s) of every input channel of image n, in LDS (its
  // global loads happen before any DMA is in flight)
  __shared__ float aparm[kAff ? 3 * kW4AffC : 1];
  if constexpr (kAff) {
    for (int c = tid; c < a.Cin; c += Geo::NTH) {
      const AdainP p = adain_params(a.aux, n, c, a);
      aparm[c] = p.mc;
      aparm[kW4AffC + c] = p.scale;
      aparm[2 * kW4AffC + c] = p.ms;
    }
    __syncthreads();
  }
  floatx4 acc[18][2];
#pragma unroll
  for (int x = 0; x < 18; ++x) acc[x][0] = acc[x][1] = floatx4{0.f, 0.f, 0.f, 0.f};

  // K step g (co tile ct0 + g / K4, channels 4 (g % K4)..+3): weight slice (18 pieces of
  // 1 KiB, pieces w, w + 8, w + 16 of wave w) and patch into its stage by LDS-DMA; every
  // wave issues the same number of pieces per step (the padding ones read out of range
  // into the dummy target), so the ring's waits are counted: kPer per step
  // (weights of global step g are slice g of the block's weight image: no division; ks =
  // g % K4 is tracked by the caller)
  auto issue_w = [&](int g, bool live, float* st) {
    if (!(DBG & 2)) {
      const int wv = launder(wave);
      const int sw = live ? (ct0 * K4 + g) * kW4SW * 4 + wv * 1024 : 0;  // piece wv's bytes
#pragma unroll
      for (int i = 0; i < Geo::WPI; ++i) {
        const bool real = wv + NW * i < 18;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsrc_or_zero(w_img, wbytes, live && real), (lds_ptr_t)(real ? st + Geo::SPATCH + wv * 256 + NW * 256 * i : dummy), 16, lane * 16,
            real ? sw + NW * 1024 * i : 0, 0, 0);
      }
    }
  };
  auto issue_p = [&](int ks, bool live, float* st) {
    {
      if (DBG & 1) return;
      const int wv = launder(wave);
      const int c = 4 * ks + wv / NH;
      const bool ok = live && c < a.Cin;
      const auto r = rsrc_or_zero(in_img, oob, ok);
      const int so = ok ? (int)((unsigned)c * in_plane * 4u) : 0;  // < 2^32 (wino4_fits)
      float* xs = st + (wv / NH) * Geo::CS;
      if (wide) {
#pragma unroll
        for (int i = 0; i < kWide; ++i) {
          const int p = kWide * (wv % NH) + i;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              r, (lds_ptr_t)(p < Geo::DMA4 ? xs + 256 * p : dummy), 16, (int)poff[i], so, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < kSlow; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(xs + 64 * (kSlow * (wv % NH) + i)),
                                                   4, (int)poff[i], so, 0, 0);
      }
    }
  };
  [[maybe_unused]] auto issue = [&](int g, int ks, bool live, float* st) {
    issue_w(g, live, st);
    issue_p(ks, live, st);
  };
  // ADAIN, in place on the elements this lane's own DMA pieces of step g wrote (so a wave
  // needs only its own counted wait, no barrier): ((v - mean_c) / std_c) * std_s + mean_s
  // inside the image, 0 at padding positions (a padding piece lane read 0)
  auto fix_own = [&](int g, float* st) {
    if constexpr (kAff) {
      if (DBG & 4) return;
      const int ks = g % K4, ch = 4 * ks + chl;
      const bool chok = ch < a.Cin;
      const int cc = chok ? ch : 0;
      const float mc = aparm[cc], sc = aparm[kW4AffC + cc], ms = aparm[2 * kW4AffC + cc];
      float* xs = st + chl * Geo::CS;
      if (wide) {
#pragma unroll
        for (int i = 0; i < kWide; ++i) {
          const int p = kWide * hf + i;
          if (p < Geo::DMA4) {
            float4* e = reinterpret_cast<float4*>(xs + 4 * (64 * p + lane));
            const bool ok = chok && ((pvalid >> i) & 1u);
            const float4 v = *e;
            *e = make_float4(ok ? fmaf(v.x - mc, sc, ms) : 0.f, ok ? fmaf(v.y - mc, sc, ms) : 0.f,
                             ok ? fmaf(v.z - mc, sc, ms) : 0.f, ok ? fmaf(v.w - mc, sc, ms) : 0.f);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < kSlow; ++i) {
          float* e = xs + 64 * (kSlow * hf + i) + lane;
          const bool ok = chok && ((pvalid >> i) & 1u);
          *e = ok ? fmaf(*e - mc, sc, ms) : 0.f;
        }
      }
    }
  };


  // one K step of 4 channels from a stage: 72 VALU of input transform + 36 MFMAs
  // hw / hp: called after MFMA pair kHW / kHP (RPST_W4VAR placement experiments)
  // input rows ph .. ph + 4 of this lane's 6x6 window of one step
  auto load_rows = [&](const float* pbuf, float (&d)[5][6]) {
    const float* pr = pbuf + k * Geo::CS + (4 * wr + ph) * kW4PS + 4 * tn;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
#if RPST_W4_RD128
      // columns 4 tn + 4 .. + 7 as a second ds_read_b128 (the empty asm keeps it whole: the
      // compiler narrows it to the b64 of the 2 columns used, whose k-groups share banks)
      floatx4 u = *reinterpret_cast<const floatx4*>(pr + r * kW4PS);
      floatx4 v = *reinterpret_cast<const floatx4*>(pr + r * kW4PS + 4);
      asm("" : "+v"(u), "+v"(v));
      d[r][0] = u[0];
      d[r][1] = u[1];
      d[r][2] = u[2];
      d[r][3] = u[3];
      d[r][4] = v[0];
      d[r][5] = v[1];
#else
      const float4 u = *reinterpret_cast<const float4*>(pr + r * kW4PS);
      const float2 v = *reinterpret_cast<const float2*>(pr + r * kW4PS + 4);
      d[r][0] = u.x;
      d[r][1] = u.y;
      d[r][2] = u.z;
      d[r][3] = u.w;
      d[r][4] = v.x;
      d[r][5] = v.y;
#endif
    }
  };
  // one K step of 4 channels from a stage (its rows already in d): 72 VALU of input
  // transform + 36 MFMAs; hw / hp run after MFMA pair kHW / kHP (the DMA of step g + 3)
  auto compute = [&](const float* pbuf, float (&d)[5][6], auto&& hw, auto&& hp) {
    {
      const float* wq = pbuf + Geo::SPATCH + ph * 9 * 256 + lane * 4;
      float4 w4[9];
      constexpr int kA = NR == 4 ? RPST_W4_AHEAD : 3;  // A-operand groups read ahead
#pragma unroll
      for (int q = 0; q < kA; ++q)
        w4[q] = (DBG & 64) ? make_float4(1.f, 2.f, 3.f, (float)q)
                           : *reinterpret_cast<const float4*>(wq + q * 256);
      // rows 3ph..3ph+2 of B^T d (d[r] = input row ph + r), then B along each row
      float t[3][6];
      if (DBG & 8) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int c = 0; c < 6; ++c) t[i][c] = d[i][c];
      } else if (ph == 0) {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const float A = fmaf(-4.f, d[2][c], d[4][c]), B = fmaf(-4.f, d[1][c], d[3][c]);
          t[0][c] = fmaf(4.f, d[0][c], fmaf(-5.f, d[2][c], d[4][c]));
          t[1][c] = A + B;
          t[2][c] = A - B;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const float C = d[3][c] - d[1][c], E = d[2][c] - d[0][c];
          t[0][c] = fmaf(2.f, E, C);
          t[1][c] = fmaf(-2.f, E, C);
          t[2][c] = fmaf(4.f, d[0][c], fmaf(-5.f, d[2][c], d[4][c]));
        }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (!(DBG & 8)) bt6(t[i][0], t[i][1], t[i][2], t[i][3], t[i][4], t[i][5]);
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        if (q + kA < 9)
          w4[q + kA] = (DBG & 64) ? make_float4(1.f, 2.f, 3.f, (float)q)
                                  : *reinterpret_cast<const float4*>(wq + (q + kA) * 256);
        const int p0 = 2 * q, p1 = 2 * q + 1;
        const float v0 = t[p0 / 6][p0 % 6], v1 = t[p1 / 6][p1 % 6];
        acc[p0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[q].x, v0, acc[p0][0], 0, 0, 0);
        acc[p0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[q].y, v0, acc[p0][1], 0, 0, 0);
        acc[p1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[q].z, v1, acc[p1][0], 0, 0, 0);
        acc[p1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[q].w, v1, acc[p1][1], 0, 0, 0);
        if (q == kHW) hw();
        if (q == kHP) hp();
      }
    }
  };

  // this wave's partial output tile of channel half mt, accumulator element r:
  // sum over its transformed rows i = 3ph + i' of A^T[:, i] (M[i, :] A); PH = ph
  // b (PH = 0 only): the channel's bias, added to transformed row 1 after the column pass:
  // column 1 of A^T is (1, 1, 1, 1), so it reaches all four output rows (4 adds, not 16)
  auto partial = [&](auto PHc, int mt, int r, float (&Y)[16], float b) {
    constexpr int PH = decltype(PHc)::value;
    float P[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      float m[6];
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) m[jj] = acc[6 * i + jj][mt][r];
      at6(m, P[i]);
    }
    if constexpr (PH == 0) {
#pragma unroll
      for (int x = 0; x < 4; ++x) P[1][x] += b;
    }
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      if constexpr (PH == 0) {
        const float s12 = P[1][x] + P[2][x], d12 = P[1][x] - P[2][x];
        Y[0 * 4 + x] = P[0][x] + s12;
        Y[1 * 4 + x] = d12;
        Y[2 * 4 + x] = s12;
        Y[3 * 4 + x] = d12;
      } else {
        const float s34 = P[0][x] + P[1][x], d34 = P[0][x] - P[1][x];
        Y[0 * 4 + x] = s34;
        Y[1 * 4 + x] = 2.f * d34;
        Y[2 * 4 + x] = 4.f * s34;
        Y[3 * 4 + x] = fmaf(8.f, d34, P[2][x]);
      }
    }
  };

  // bias, activation, store and the optional per-wave statistics of one finished tile:
  // channel co of tile (wr, tn). Everything it needs besides the tile is re-derived per
  // epilogue from the kernel arguments (EpiCtx): nothing of it stays live across the main
  // loop, whose scalar registers are full (a spilled SGPR costs a VALU readlane per use)
  auto epi_ctx = [&]() {
    const KArgs L = late_args();
    EpiCtx e;
    e.W = L->W;
    e.H = L->H;
    e.Cout = L->Cout;
    e.slope = L->relu == RPST_ACT_RELU ? 0.f : (L->relu == RPST_ACT_LRELU ? 0.2f : 1.f);
    int btx, bty;
    w4_tile(w4_block_id() / L->cosplit, RPST_W4_ORDER,
            L->tiles_x, L->tiles_y, L->N, btx, bty, e.n);
    const int bx0 = btx * kW4TW;
    e.gy0 = bty * Geo::TH + 4 * wr;
    e.gx0 = bx0 + 4 * tn;
    e.vec = (e.W & 3) == 0 && e.gx0 + 3 < e.W;
    e.rows = max(0, min(4, e.H - e.gy0));
    const int cols = max(0, min(kW4TW, e.W - bx0));
    e.inv = e.rows * cols > 0 ? 1.f / (float)(e.rows * cols) : 0.f;
    e.full = e.rows == 4 && bx0 + kW4TW <= e.W;
    // some output of the wave is on the first / last image row or column (BTAB classes)
    e.edge = e.gy0 == 0 || e.gy0 + 4 >= e.H || bx0 == 0 || bx0 + kW4TW >= e.W;
    e.out = L->out;
    // buffer stores (soffset = channel plane, voffset = row offset; rows past H get an
    // out-of-range offset, so no store needs a mask) when the float4 path applies to every
    // lane of the layer and one image's output fits 2^31 bytes
    const int64_t plane = (int64_t)e.H * e.W;
    e.pool = L->pool_out != 0;
    e.bst = !e.pool && (e.W & 3) == 0 && (int64_t)e.Cout * plane * 4 < (1LL << 31);
    e.oimg = e.out + (int64_t)e.n * e.Cout * plane;
    // images past a.skip_from: statistics only, every store out of range (dropped)
    const bool keep = L->skip_from <= 0 || e.n < L->skip_from;
    e.obytes = keep ? (unsigned)(e.Cout * plane * 4) : 0u;
    e.store = keep;
#pragma unroll
    for (int yy = 0; yy < 4; ++yy)
      e.voff[yy] = (yy < e.rows && e.gx0 < e.W) ? (unsigned)(((e.gy0 + yy) * e.W + e.gx0) * 4)
                                               : 0x80000000u;
    e.btab = L->btab;
    e.statp = L->stat_part;
    e.statP = L->stat_P;
    e.sidx = (bty * L->tiles_x + btx) * NR + wr;
    return e;
  };
  // the bias (interior class for BTAB) is already in Y (partial)
  auto finish = [&](const EpiCtx& e, int co, float (&Y)[16]) {
    const int gy0 = e.gy0, gx0 = e.gx0, rows = e.rows, n = e.n;
    const bool cok = co < e.Cout;
    // folded AdaIN / WCT: the bias depends on which taps of the zero-padded input were
    // inside the image (border class); interior tiles take the interior entry
    const float* bt = BTAB ? e.btab + ((int64_t)n * e.Cout + (cok ? co : 0)) * 9 : nullptr;
    if (BTAB && e.edge) {
      // a wave touching the image border: the nine class biases of co in registers, the
      // row class uniform per output row, the column class per lane
      float b9[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) b9[i] = cok ? bt[i] : 0.f;
      const float b4 = b9[4];
#pragma unroll
      for (int i = 0; i < 9; ++i) b9[i] -= b4;  // the interior class went in with the partials
#pragma unroll
      for (int yy = 0; yy < 4; ++yy) {
        const int gy = gy0 + yy;
        const int rc = gy == 0 ? 0 : (gy >= e.H - 1 ? 2 : 1);
        const float l = rc == 0 ? b9[0] : (rc == 2 ? b9[6] : b9[3]);
        const float m = rc == 0 ? b9[1] : (rc == 2 ? b9[7] : b9[4]);
        const float r = rc == 0 ? b9[2] : (rc == 2 ? b9[8] : b9[5]);
#pragma unroll
        for (int xx = 0; xx < 4; ++xx) {
          const int gx = gx0 + xx;
          Y[yy * 4 + xx] += gx == 0 ? l : (gx >= e.W - 1 ? r : m);
        }
      }
    }
    // activation, branch-free: max(y, slope y) as one v_med3 (fmaxf would add a NaN
    // canonicalisation per element)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      Y[i] = __builtin_amdgcn_fmed3f(Y[i], RELU ? 0.f : e.slope * Y[i], __builtin_inff());
    float sum = 0.f;
    if (STATS) {
      if (e.full) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sum += Y[i];
      } else {
#pragma unroll
        for (int yy = 0; yy < 4; ++yy)
#pragma unroll
          for (int xx = 0; xx < 4; ++xx) sum += (yy < rows && gx0 + xx < e.W) ? Y[yy * 4 + xx] : 0.f;
      }
    }
    if (e.bst) {
      // the channel (per lane: co depends on the lane's k) goes into the per-lane offset;
      // co >= Cout or a row past H lands in [2^31 - 1, 2^32): out of range, dropped
      const auto ro = rsrc_or_zero(e.oimg, e.obytes, true);
      const unsigned cofs = cok ? (unsigned)co * (unsigned)(e.H * e.W) * 4u : 0x7fffffffu;
#pragma unroll
      for (int yy = 0; yy < 4; ++yy) {
        const floatx4 v = {Y[yy * 4], Y[yy * 4 + 1], Y[yy * 4 + 2], Y[yy * 4 + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro,
                                               (int)(e.voff[yy] + cofs), 0, RPST_W4_CPOL);
      }
    } else if (e.pool) {
      // max_pool2d(2, 2, ceil_mode) of the finished tile: tiles start on even rows and
      // columns, so each holds whole windows; fmaxf in the stand-alone kernel's order
      // (maxpool2_kernel), windows cut by the image edge take their in-image elements
      if (cok && e.store) {
        const int Ho = (e.H + 1) >> 1, Wo = (e.W + 1) >> 1;
        float* o = e.out + (((int64_t)n * e.Cout + co) * Ho + (gy0 >> 1)) * Wo + (gx0 >> 1);
#pragma unroll
        for (int py = 0; py < 2; ++py) {
          if (2 * py >= rows) continue;
          const bool y1 = 2 * py + 1 < rows;
          float pv[2];
#pragma unroll
          for (int px = 0; px < 2; ++px) {
            const bool x1 = gx0 + 2 * px + 1 < e.W;
            const float* t = Y + (2 * py) * 4 + 2 * px;
            float v = t[0];
            if (x1) v = fmaxf(v, t[1]);
            if (y1) v = fmaxf(v, t[4]);
            if (x1 && y1) v = fmaxf(v, t[5]);
            pv[px] = v;
          }
          if (gx0 + 3 < e.W && (Wo & 1) == 0) {
            *reinterpret_cast<float2*>(o + py * Wo) = make_float2(pv[0], pv[1]);
          } else {
            if (gx0 < e.W) o[py * Wo] = pv[0];
            if (gx0 + 2 < e.W) o[py * Wo + 1] = pv[1];
          }
        }
      }
    } else if (cok && e.store) {
      float* o = e.out + (((int64_t)n * e.Cout + co) * e.H + gy0) * e.W + gx0;
#pragma unroll
      for (int yy = 0; yy < 4; ++yy) {
        if (yy < rows) {
          if (e.vec) {
            *reinterpret_cast<float4*>(o + yy * e.W) =
                make_float4(Y[yy * 4], Y[yy * 4 + 1], Y[yy * 4 + 2], Y[yy * 4 + 3]);
          } else {
#pragma unroll
            for (int xx = 0; xx < 4; ++xx)
              if (gx0 + xx < e.W) o[yy * e.W + xx] = Y[yy * 4 + xx];
          }
        }
      }
    }
    if constexpr (STATS) {
      sum = row16_sum(sum);
      const float mean = sum * e.inv;
      float m2 = 0.f;
      if (e.full) {
#pragma unroll
        for (int i = 0; i < 16; ++i) m2 = fmaf(Y[i] - mean, Y[i] - mean, m2);
      } else {
#pragma unroll
        for (int yy = 0; yy < 4; ++yy)
#pragma unroll
          for (int xx = 0; xx < 4; ++xx) {
            const float dv = Y[yy * 4 + xx] - mean;
            m2 += (yy < rows && gx0 + xx < e.W) ? dv * dv : 0.f;
          }
      }
      m2 = row16_sum(m2);
      if (tn == 0 && cok)
        e.statp[((int64_t)n * e.Cout + co) * e.statP + e.sidx] = make_float2(mean, m2);
    }
  };

  // epilogue of co tile ct after the K step that used stage xs: the partials travel through
  // that consumed stage, one accumulator element r per pass: 2 KiB-float region per tile
  // row laid out [writer half][float4 group][lane] (conflict-free 16-B accesses). Raw
  // barriers (LDS only): the DMA prefetch of the next steps stays in flight.
  auto lds_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(DBG & 16)) __builtin_amdgcn_s_barrier();
  };
  // PH = ph: the half this wave finishes is channel half PH; it hands the other half's
  // partial tile to its partner wave
  auto epilogue_ph = [&](auto PHc, int ct, float* xs) {
    constexpr int PH = decltype(PHc)::value;
    lds_barrier();  // every wave is done reading the stage
    float* xb = xs + wr * 2048;
    const EpiCtx e = epi_ctx();
    const int co0 = ct * kW4BM + 16 * PH + 4 * k;
    // PH = 0 adds the biases of both channel halves (its own and the partner's partial),
    // loaded once ahead of the passes: [half][r]
    float bias8[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if constexpr (PH == 0) {
      const float* bias = BTAB ? nullptr : late_args()->bias;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = ct * kW4BM + 16 * h + 4 * k + r;
          if (co < e.Cout)
            bias8[h][r] = BTAB ? e.btab[((int64_t)e.n * e.Cout + co) * 9 + 4] : (bias ? bias[co] : 0.f);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float own[16];
      {
        float give[16];
        partial(PHc, PH, r, own, bias8[0][r]);
        partial(PHc, 1 - PH, r, give, bias8[1][r]);
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          *reinterpret_cast<float4*>(xb + ((PH * 4 + g4) * 64 + lane) * 4) =
              make_float4(give[4 * g4], give[4 * g4 + 1], give[4 * g4 + 2], give[4 * g4 + 3]);
      }
      lds_barrier();
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const float4 o4 =
            *reinterpret_cast<const float4*>(xb + (((1 - PH) * 4 + g4) * 64 + lane) * 4);
        own[4 * g4] += o4.x;
        own[4 * g4 + 1] += o4.y;
        own[4 * g4 + 2] += o4.z;
        own[4 * g4 + 3] += o4.w;
      }
      finish(e, co0 + r, own);
      if (r < 3) lds_barrier();  // the next pass overwrites the exchange region
    }
  };
  auto epilogue = [&](int ct, float* xs) {
    if (ph) epilogue_ph(std::integral_constant<int, 1>{}, ct, xs);
    else epilogue_ph(std::integral_constant<int, 0>{}, ct, xs);
  };

  // ---- pipeline: ring of 4 stages, K step g in stage g % 4, issued 3 steps ahead --------
  // Every step issues one group of `per` pieces per wave, also past the last step (those
  // read out of range into a stage no later step reads), so the wait before the barrier
  // that opens step g is one constant: the groups of steps g + 1, g + 2 stay in flight
  // (ADAIN's register loads drain everything at their use, so the count stays conservative).
  // (NR = 2: the 2-stage ring keeps no group in flight past the one being waited for)
  auto wait_ahead2 = [&]() {
    if (DBG & 128) return;
    if constexpr (S == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      static_assert(S == 4 && Geo::WPI == 3 && kWide == 3 && kSlow == 10, "counted waits");
      if (wide) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // 2 x (3 + 3)
      else asm volatile("s_waitcnt vmcnt(26)" ::: "memory");       // 2 x (3 + kSlow)
    }
  };
  issue(0, 0, true, smem0);
  if constexpr (S == 4) {
    issue(1, 1 % K4, G > 1, smem1);
    issue(2, 2 % K4, G > 2, smem2);
  }
  int ks3 = (S - 1) % K4;    // chunk step of g + S - 1
  int ks = 0, ct = ct0;      // chunk step and co tile of g
  if constexpr (kAff) {  // step 0's affine (published by the first step's barrier)
    wait_ahead2();
    fix_own(0, smem0);
  }
  // K step g from stage `cur`; step g + S - 1's DMA into `nx3` (the stage step g - 1 used);
  // ADAIN: step g + 1's affine on this wave's own pieces in `nx1`, after the MFMAs.
  // (Reading the next step's rows one step ahead, under the MFMAs, needs 30 more VGPRs
  // across the step: 650-1800 spills.)
  auto step = [&](int g, float* cur, float* nx1, float* nx3) {
    wait_ahead2();
    lds_barrier();  // step g's stage is complete; nx3 is free
    float d[5][6];
    load_rows(cur, d);
    const bool live3 = g + S - 1 < G;
    if constexpr (kHW < 0) issue_w(g + S - 1, live3, nx3);
    if constexpr (kHP < 0) issue_p(ks3, live3, nx3);
    auto hw = [&]() { if constexpr (kHW >= 0) issue_w(g + S - 1, live3, nx3); };
    auto hp = [&]() { if constexpr (kHP >= 0) issue_p(ks3, live3, nx3); };
    compute(cur, d, hw, hp);
    ks3 = ks3 + 1 == K4 ? 0 : ks3 + 1;
    if (ks == K4 - 1) {
      if (!(DBG & 32)) epilogue(ct, cur);
#pragma unroll
      for (int x = 0; x < 18; ++x) acc[x][0] = acc[x][1] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (kAff) {
      if (g + 1 < G) {
        wait_ahead2();  // this wave's pieces of step g + 1 have landed
        fix_own(g + 1, nx1);
      }
    }
    ct += ks == K4 - 1 ? 1 : 0;
    ks = ks == K4 - 1 ? 0 : ks + 1;
  };
  if constexpr (S == 4) {
    for (int g = 0; g < G; g += 4) {
      step(g, smem0, smem1, smem3);
      if (g + 1 < G) step(g + 1, smem1, smem2, smem0);
      if (g + 2 < G) step(g + 2, smem2, smem3, smem1);
      if (g + 3 < G) step(g + 3, smem3, smem0, smem2);
    }
  } else {
    for (int g = 0; g < G; g += 2) {
      step(g, smem0, smem1, smem1);
      if (g + 1 < G) step(g + 1, smem1, smem0, smem0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the padding DMA has landed too
}

// ---- AdaIN folded into the weights (RPST_IN_ADAIN through the plain NONE loader) -------
// conv(pad0(s * x + b)) = conv_{W s}(pad0(x)) + sum_ci b_ci sum_{taps inside} W[co][ci][tap]
// with s = std_s / std_c and b = mean_s - mean_c * s per (n, ci): image n gets its own
// copy of the packed U scaled by s along ci (U is linear in g), and a bias per (n, co) and
// border class (which rows / columns of the 3x3 window fall on zero padding; with reflect
// padding every tap sees s * x + b, so all nine classes are equal). The conv itself then
// streams the raw feature by plain LDS-DMA: no per-element affine, no extra LDS traffic.
size_t wino4_fold_floats(int N, int Cin, int Cout) {
  // per-image packed U (the layout the folded NONE launch runs) and border biases, then the
  // class sums (fp64)
  return (size_t)N * (wino4_image_floats_max(Cout, Cin) + (size_t)Cout * 9) +
         2 * (size_t)9 * Cout * Cin + 2;
}

__global__ void wino4_fold_w_kernel(const float4* __restrict__ pk, float4* __restrict__ out,
                                    const float* __restrict__ aux, int N, int Cin, int nch,
                                    int64_t per4) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * per4) return;
  const int n = (int)(t / per4);
  const int64_t u = t - (int64_t)n * per4;  // float4 index = element index >> 2
  const int l = (int)(u & 63);
  int64_t r = (u >> 6) / 9;  // ((ct * nch + c) * 2 + s) * 2 + h
  const int s = (int)((r >> 1) & 1);
  const int c = (int)((r >> 2) % nch);
  const int ci = c * kW4CK + 4 * s + (l >> 4);
  const int64_t nc = (int64_t)N * Cin, i = (int64_t)n * Cin + (ci < Cin ? ci : 0);
  const float sc = ci < Cin ? aux[3 * nc + i] / aux[2 * nc + i] : 0.f;
  const float4 v = pk[u];
  out[t] = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
}

// Border-class tap sums of the layer weights, S[cls][co][ci] = sum over the taps of class
// cls = 3 rc + cc that fall inside the image (rc / cc = 0 first row / column: tap 0 on the zero
// padding, 1 interior, 2 last; with reflect padding every tap is inside: all classes equal),
// fp64; direct-packed weights [chunk][tap][ci % 8][cout_pad].
__global__ void class_sums_kernel(const float* __restrict__ dpk, double* __restrict__ S, int Cin,
                                  int Cout, int cout_pad, int reflect) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)9 * Cout * Cin) return;
  const int ci = (int)(t % Cin);
  const int64_t r = t / Cin;
  const int co = (int)(r % Cout), cls = (int)(r / Cout);
  const int rc = cls / 3, cc = cls % 3;
  const float* w = dpk + ((int64_t)(ci >> 3) * 9 * 8 + (ci & 7)) * cout_pad + co;
  double tap = 0.0;
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const bool in = reflect || ((rc != 0 || u != 0) && (rc != 2 || u != 2) &&
                                  (cc != 0 || p != 0) && (cc != 2 || p != 2));
      if (in) tap += (double)w[(int64_t)(u * 3 + p) * 8 * cout_pad];
    }
  S[t] = tap;
}

// btab[(n * Cout + co) * 9 + cls] = bias[co] + sum_ci b_n[ci] S[cls][co][ci] (fp64, fixed order:
// lane-strided partials then a wave sum). b_n = mean_s - mean_c * std_s / std_c (the AdaIN fold,
// aux = [mean_c | mean_s | std_c | std_s]) or c_n (the WCT fold, cvec). One wave per (n, co).
__global__ __launch_bounds__(256) void border_bias_kernel(const double* __restrict__ S,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ aux,
                                                          const double* __restrict__ cvec,
                                                          float* __restrict__ btab, int N, int Cin,
                                                          int Cout) {
  const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wv >= (int64_t)N * Cout) return;
  const int co = (int)(wv % Cout), n = (int)(wv / Cout);
  const int64_t nc = (int64_t)N * Cin;
  double acc[9];
#pragma unroll
  for (int c = 0; c < 9; ++c) acc[c] = 0.0;
  for (int ci = lane; ci < Cin; ci += 64) {
    const int64_t i = (int64_t)n * Cin + ci;
    double b;
    if (cvec) {
      b = cvec[i];
    } else {
      const float sc = aux[3 * nc + i] / aux[2 * nc + i];
      b = (double)aux[nc + i] - (double)aux[i] * (double)sc;
    }
#pragma unroll
    for (int c = 0; c < 9; ++c) acc[c] = fma(b, S[((int64_t)c * Cout + co) * Cin + ci], acc[c]);
  }
  const double b0 = bias ? (double)bias[co] : 0.0;
#pragma unroll
  for (int c = 0; c < 9; ++c) {
    const double v = wave_sum(acc[c]);
    if (lane == 0) btab[((int64_t)n * Cout + co) * 9 + c] = (float)(b0 + v);
  }
}

static int border_biases(const float* dpk, int cout_pad, const float* bias, const float* aux,
                         const double* cvec, float* btab, double* S, int N, int Cin, int Cout,
                         int reflect, hipStream_t st) {
  const int64_t ns = (int64_t)9 * Cout * Cin;
  class_sums_kernel<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(dpk, S, Cin, Cout, cout_pad,
                                                                  reflect);
  if (int e = launch_status("class_sums_kernel")) return e;
  const int64_t waves = (int64_t)N * Cout;
  border_bias_kernel<<<(unsigned)((waves + 3) / 4), 256, 0, st>>>(S, bias, aux, cvec, btab, N, Cin,
                                                                  Cout);
  return launch_status("border_bias_kernel");
}

static double* align8(void* p) {
  return reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
}

int wino4_fold(ConvArgs& a, const float* direct_packed, int direct_cout_pad, float* ws,
               hipStream_t st) {
  RPST_REQUIRE(a.H >= 2 && a.W >= 2, "conv2d: folded AdaIN needs H, W >= 2");
  const int nch = (a.Cin + kW4CK - 1) / kW4CK;
  // a.wpk is the image of the launched (NONE) form: the quarter layout where it applies
  const bool q = wino4q_applies(a.Cin, a.Cout, RPST_IN_NONE);
  const int64_t per = (int64_t)wino4_image_floats(a.Cout, a.Cin, RPST_IN_NONE);
  const int64_t n4 = (int64_t)a.N * (per / 4);
  float* wf = ws;
  float* bt = ws + (int64_t)a.N * per;
  if (q) {
    if (int e = wino4q_fold_w(a.wpk, wf, a.aux, a.N, a.Cout, a.Cin, st)) return e;
  } else {
    wino4_fold_w_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(
        reinterpret_cast<const float4*>(a.wpk), reinterpret_cast<float4*>(wf), a.aux, a.N,
        a.Cin, nch, per / 4);
    if (int e = launch_status("wino4_fold_w_kernel")) return e;
  }
  double* S = align8(bt + (int64_t)a.N * a.Cout * 9);
  if (int e = border_biases(direct_packed, direct_cout_pad, a.bias, a.aux, nullptr, bt, S, a.N,
                            a.Cin, a.Cout, a.pad == RPST_PAD_REFLECT, st))
    return e;
  a.wpk = wf;
  a.wstride = per;
  a.btab = bt;
  return RPST_OK;
}

// ---- a channel-mixing input folded into the weights (WCT feeding the decoder) --------
// conv(pad(T_n x + c_n)) = conv_{W T_n}(pad(x)) + sum_m c_n[m] sum_{taps inside} W[co][m][tap]
// (T_n commutes with the padding: zero padding maps to zero, reflection is spatial). Image
// n gets weights W'_n = W T_n (fp64, from the direct-packed image: W[co][m][tap] =
// dpk[(m / 8 * 9 + tap) * 8 * cout_pad + (m % 8) * cout_pad + co]), packed as U'_n = G W'_n
// G^T with one rounding to fp32, and a bias per (n, co) and border class from c_n. With
// T_n = diag(s), c_n = b this is the AdaIN fold above.
size_t wino4_mix_floats(int N, int Cin, int Cout) {
  // fold (U, biases, class sums) + W T_n (fp64, [n][tap][co][ci]) + W in [tap][co][m] (fp32)
  return wino4_fold_floats(N, Cin, Cout) + 2 * (size_t)N * Cout * Cin * 9 +
         (size_t)9 * Cout * Cin + 4;
}

// Wt[(tap * Cout + co) * Cin + m] = W[co][m][tap] from the direct-packed image (the GEMM A
// operand of W T_n)
__global__ void mix_wt_kernel(const float* __restrict__ dpk, float* __restrict__ wt, int Cin,
                              int Cout, int cout_pad) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)9 * Cout * Cin) return;
  const int m = (int)(t % Cin);
  const int64_t r = t / Cin;
  const int co = (int)(r % Cout), tap = (int)(r / Cout);
  wt[t] = dpk[((int64_t)(m >> 3) * 9 + tap) * 8 * cout_pad + (m & 7) * cout_pad + co];
}

int wino4_mix(ConvArgs& a, const double* T, const double* cvec, const float* direct_packed,
              int direct_cout_pad, float* ws, hipStream_t st) {
  RPST_REQUIRE(a.H >= 2 && a.W >= 2, "conv2d_mix: needs H, W >= 2");
  const int nch = (a.Cin + kW4CK - 1) / kW4CK;
  const bool q = wino4q_applies(a.Cin, a.Cout, RPST_IN_NONE);
  const int64_t per = (int64_t)wino4_image_floats(a.Cout, a.Cin, RPST_IN_NONE);
  float* wf = ws;
  float* bt = ws + (int64_t)a.N * per;
  double* S = align8(bt + (int64_t)a.N * a.Cout * 9);
  double* wm = S + (int64_t)9 * a.Cout * a.Cin;  // W T_n: [n][tap][co][k]
  float* wt = reinterpret_cast<float*>(wm + (int64_t)a.N * a.Cout * 9 * a.Cin);
  const int64_t nt = (int64_t)9 * a.Cout * a.Cin;
  mix_wt_kernel<<<(unsigned)((nt + 255) / 256), 256, 0, st>>>(direct_packed, wt, a.Cin, a.Cout,
                                                              direct_cout_pad);
  if (int e = launch_status("mix_wt_kernel")) return e;
  // W'_n = W T_n on the fp64 MFMA: (9 Cout x Cin) x (Cin x Cin) per image
  if (int e = gemm_f32w_f64(wt, T, wm, a.N, 9 * a.Cout, a.Cin, st)) return e;
  const int64_t tot = (int64_t)a.N * per;
  if (q) {
    if (int e = wino4q_pack_mix(wm, wf, a.N, a.Cout, a.Cin, st)) return e;
  } else {
    wino4_pack_kernel<double><<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(
        wm, wf, a.Cout, a.Cin, nch, per, tot, a.Cin, 1, (int64_t)a.Cout * a.Cin);
    if (int e = launch_status("wino4_pack_kernel(mix)")) return e;
  }
  if (int e = border_biases(direct_packed, direct_cout_pad, a.bias, nullptr, cvec, bt, S, a.N,
                            a.Cin, a.Cout, a.pad == RPST_PAD_REFLECT, st))
    return e;
  a.wpk = wf;
  a.wstride = per;
  a.btab = bt;
  return RPST_OK;
}

int wino4_launch(ConvArgs& a, int in_op, hipStream_t st) {
  RPST_REQUIRE(wino4_supports(in_op), "conv2d: winograd4 does not support in_op %d", in_op);
  RPST_REQUIRE(a.res == nullptr, "conv2d: winograd4 has no residual epilogue");
  RPST_REQUIRE(wino4_fits(a.N, a.Cin, a.Hs, a.Ws, in_op), "conv2d: image too large for winograd4");
  if (wino4q_applies(a.Cin, a.Cout, in_op)) return wino4q_launch(a, in_op, st);
  a.Cout_pad = (a.Cout + kW4BM - 1) / kW4BM * kW4BM;
  a.nchunks = (a.Cin + kW4CK - 1) / kW4CK;
  a.tiles_x = (a.W + kW4TW - 1) / kW4TW;
  const int nr = wino4_rows(a.Cin, a.Cout, in_op);
  a.tiles_y = (a.H + 4 * nr - 1) / (4 * nr);
  a.co_tiles = a.Cout_pad / kW4BM;
  a.stat_P = a.tiles_x * a.tiles_y * nr;
  {
    const char* e = getenv("RPST_WINO4_PRIO");  // A/B switch for a static priority
    const int pr = (e && *e) ? atoi(e) : 0;
    a.persist = 1 | (pr == 1 ? 2 : 0) | (pr == 2 ? 4 : 0);
  }
  RPST_REQUIRE((int64_t)a.co_tiles * a.nchunks * kW4WCH * 4 < (1LL << 31),
               "conv2d: winograd4 weight image exceeds 2 GiB");
  {
    // blocks per spatial tile: 2 once a co tile has >= 32 K steps (Cin >= 128) and there
    // are >= 4 co tiles (the shorter blocks' prologue then costs less than the L2 reuse of
    // the shared patch gains); RPST_WINO4_COSPLIT overrides (A/B)
    const char* e = getenv("RPST_WINO4_COSPLIT");
    int c = (e && *e) ? atoi(e) : (2 * a.nchunks >= 32 && a.co_tiles >= 4 ? 2 : 1);
    c = c < 1 ? 1 : (c > a.co_tiles ? a.co_tiles : c);
    while (a.co_tiles % c) --c;
    a.cosplit = c;
  }
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.N * a.cosplit;
  RPST_REQUIRE(blocks <= 0x7fffffffLL, "conv2d: grid too large");
  const unsigned nb = (unsigned)blocks;
  const bool stats = a.stat_part != nullptr, btab = a.btab != nullptr;
  RPST_REQUIRE(!btab || in_op == RPST_IN_NONE, "conv2d: winograd4 bias table with a loader op");
  // RELU: the activation as one v_med3 per element (the RP stacks and VGG: every large
  // layer); other activations run the general max(y, slope y) form
#define RPST_W4_GO(OP, S, B)                                                          \
  do {                                                                                \
    if (nr == 2) {                                                                    \
      if (a.relu == RPST_ACT_RELU)                                                    \
        wino4_mfma_kernel<2, OP, S, B, true><<<nb, W4Geo<2>::NTH, 0, st>>>(a);        \
      else                                                                            \
        wino4_mfma_kernel<2, OP, S, B, false><<<nb, W4Geo<2>::NTH, 0, st>>>(a);       \
    } else {                                                                          \
      if (a.relu == RPST_ACT_RELU)                                                    \
        wino4_mfma_kernel<4, OP, S, B, true><<<nb, kW4NTH, 0, st>>>(a);               \
      else                                                                            \
        wino4_mfma_kernel<4, OP, S, B, false><<<nb, kW4NTH, 0, st>>>(a);              \
    }                                                                                 \
  } while (0)
  switch (in_op) {
    case RPST_IN_ADAIN:
      if (stats) RPST_W4_GO(RPST_IN_ADAIN, true, false);
      else RPST_W4_GO(RPST_IN_ADAIN, false, false);
      break;
    case RPST_IN_UPSAMPLE2:
      if (stats) RPST_W4_GO(RPST_IN_UPSAMPLE2, true, false);
      else RPST_W4_GO(RPST_IN_UPSAMPLE2, false, false);
      break;
    default:
      RPST_REQUIRE(!(stats && btab), "conv2d: winograd4 folded bias with statistics");
      if (stats) RPST_W4_GO(RPST_IN_NONE, true, false);
      else if (btab) RPST_W4_GO(RPST_IN_NONE, false, true);
      else RPST_W4_GO(RPST_IN_NONE, false, false);
  }
#undef RPST_W4_GO
  return launch_status("wino4_mfma_kernel");
}

}  // namespace rpst
