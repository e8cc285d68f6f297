// Winograd F(4x4, 3x3) on fp32 MFMA, position-quarter form (gfx950): the large 3x3 layers
// with >= 64 output channels of the reference hot path (network/base.py:25-111,363-396;
// sanet.py:162-192). Same arithmetic as rpst_wino4.hip (Y = A^T [U (.) V] A, U = G g G^T in
// fp64 rounded once, everything else fp32 on the true-fp32 MFMA); what changes is how the
// 36 transformed positions are spread over the waves.
//
// rpst_wino4.hip gives a wave 32 output channels x 18 positions x 16 tiles: each transformed
// input value V feeds 2 MFMAs (the two 16-channel halves), and the input transform (72 VALU
// per K step and wave) serialises with the fp32 MFMA on the SIMD (tools/coexec.hip) -- 20 % of
// the launch at 128->256. Here a wave owns 64 output channels x 9 positions x 16 tiles (still
// 144 accumulator registers): positions of one QUARTER of the 6x6 transformed tile (rows
// 3qr..3qr+2, columns 3qc..3qc+2), so each V value feeds 4 MFMAs and the transform is 48 VALU
// per 36 MFMAs (the column pass 3 of 6 outputs per input row, the row pass 3 of 6). The freed
// registers pay for software pipelining: the transform of K step x + 1 (its patch rows read
// and transformed one row per MFMA group) runs inside step x's MFMA stream, so no VALU chain
// and no LDS read latency sits between a step's barrier and its first MFMA.
//
// Block = 8 waves (two per SIMD), output 8 rows x 64 columns x 64 channels: wave w owns tile
// row w >> 2 and quarter w & 3. Per K step (4 input channels) the weight slice (64 co x 36
// positions x 4 ci = 36 KiB) and the patch (4 channels x 10 rows x 68) stream into a 3-stage
// LDS ring by LDS-DMA: W(x + 2) and P(x + 3) are issued inside step x. The four quarters of
// a tile row meet in the epilogue: each wave sends its 9 positions of the other three
// quarters' 16-channel blocks through a weight stage (6 passes of 2 accumulator elements x 3
// positions) and finishes its own block with the full output transform.
#include "rpst_conv.h"
#ifndef RPST_W4_CPOL
#define RPST_W4_CPOL 0  // output-store cache policy (aux bits of buffer_store), A/B only
#endif

#include <type_traits>

namespace rpst {
namespace {

typedef __attribute__((address_space(3))) void* q_lds_t;
typedef const __attribute__((address_space(4))) ConvArgs* QArgs;

// kernel arguments loaded at their use (s_load through an opaque copy of the kernarg
// pointer, so the loads are not hoisted into the main loop's scalar registers)
__device__ __forceinline__ QArgs q_args() {
  QArgs p = (QArgs)__builtin_amdgcn_kernarg_segment_ptr();
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+s"(p));
#endif
  return p;
}
// buffer resource over `bytes` at p, or over zero records (every access reads 0) if !ok;
// the select is a mask, so no branch splits the MFMA stream around it
__device__ __forceinline__ __amdgpu_buffer_rsrc_t q_rsrc(const float* p, unsigned bytes, bool ok) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(bytes & (0u - (unsigned)ok)),
                                           0x00020000);
}
__device__ __forceinline__ int q_mask(int v, bool ok) { return v & -(int)ok; }
// sum over the 16 lanes of a DPP row, in every lane
__device__ __forceinline__ float q_row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// a wave-uniform value made opaque here (not hoisted out of the enclosing loop)
__device__ __forceinline__ int q_launder(int v) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+s"(v));
#endif
  return v;
}
// reflect(1) or zero padding, branch-free; false for a zero-padding position
__device__ __forceinline__ bool q_resolve(int& v, int n, bool zero_pad) {
  const bool in = v >= 0 && v < n;
  const int r = reflect1(v, n);
  v = zero_pad ? min(max(v, 0), n - 1) : r;
  return in || !zero_pad;
}
// A^T applied to one 6-vector -> 4 values
#ifndef RPST_W4Q_DBG
#define RPST_W4Q_DBG 0
#endif
__device__ __forceinline__ void q_at6(const float (&m)[6], float (&p)[4]) {
  if (RPST_W4Q_DBG & 256) {  // timing only: no output transform
    p[0] = m[0]; p[1] = m[1]; p[2] = m[2]; p[3] = m[3] + m[4] + m[5];
    return;
  }
  const float s12 = m[1] + m[2], d12 = m[1] - m[2];
  const float s34 = m[3] + m[4], d34 = m[3] - m[4];
  p[0] = (m[0] + s12) + s34;
  p[1] = fmaf(2.f, d34, d12);
  p[2] = fmaf(4.f, s34, s12);
  p[3] = fmaf(8.f, d34, d12) + m[5];
}
// acc += a * b on v_mfma_f32_16x16x4_f32 with the accumulator tied in place ("+v"). The
// builtin's untied form lets the register allocator rename every accumulator tuple each K
// step (dst != srcC): with 144 accumulator registers that costs 60-100 more and spills.
// hipcc pads no hazard around an asm statement (cdna_hip_programming.md 5.7): an MFMA's
// result taken whole as the next MFMA's C needs no wait states (the chain here); PAD = 1
// opens the statement with s_nop 1 (2 states: an operand a VALU wrote just before); readers
// of the results other than the chain go behind q_mfma_fence.
template <int PAD>
__device__ __forceinline__ void q_mfma(floatx4& acc, float a, float b) {
  if constexpr (PAD)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// LDS-DMA issue (buffer_load ... lds) as inline asm, M0 written in the same statement
// (cdna_hip_programming.md 5.7): the compiler then tracks none of the ring's DMA, so it inserts
// no vmcnt of its own before the ring's LDS reads (its alias analysis cannot separate the
// padding pieces' dummy target from the stages and drained the ring to vmcnt(1) after every
// barrier); the ring's waits are the counted ones of wait_ring. "memory": no LDS access of
// the compiler's moves across an issue.
__device__ __forceinline__ unsigned q_lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
__device__ __forceinline__ void q_dma16(__amdgpu_buffer_rsrc_t r, const float* lds, unsigned voff,
                                        int soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(q_lds_addr(lds)), "v"(voff), "s"(r), "s"(soff) : "memory");
}
__device__ __forceinline__ void q_dma4(__amdgpu_buffer_rsrc_t r, const float* lds, unsigned voff,
                                       int soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %3 offen lds"
               :: "s"(q_lds_addr(lds)), "v"(voff), "s"(r), "s"(soff) : "memory");
}
__device__ __forceinline__ void q_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// B^T half-transform of one 6-vector: H = 0 -> outputs 0, 1, 2 (inputs 0..4); H = 1 ->
// outputs 3, 4, 5 (inputs 1..5). 6 VALU.
template <int H>
__device__ __forceinline__ void q_bt3(float d0, float d1, float d2, float d3, float d4, float d5,
                                      float& u0, float& u1, float& u2) {
  if constexpr (H == 0) {
    const float A = fmaf(-4.f, d2, d4), B = fmaf(-4.f, d1, d3);
    u0 = fmaf(4.f, d0, fmaf(-5.f, d2, d4));
    u1 = A + B;
    u2 = A - B;
  } else {
    const float C = d4 - d2, E = d3 - d1;
    u0 = fmaf(2.f, E, C);
    u1 = fmaf(-2.f, E, C);
    u2 = fmaf(4.f, d1, fmaf(-5.f, d3, d5));
  }
}

}  // namespace

constexpr int kQCo = 64;                     // output channels per co tile
constexpr int kQTH = 8, kQTW = 64;           // output rows x columns per block
#ifndef RPST_W4Q_AL
// 1: patch rows staged from x0 - 4 (16-B aligned sources for the interior blocks' 16-B
// pieces), column x0 - 1 at LDS column 3; 0: from x0 - 1 (4-B aligned sources)
#define RPST_W4Q_AL 1
#endif
#ifndef RPST_W4Q_EDGE
#define RPST_W4Q_EDGE 1
#endif
#ifndef RPST_W4Q_ALRD  // the odd window column: 1 = ds_read_b32, 2 = a whole ds_read_b128
#define RPST_W4Q_ALRD 1
#endif
constexpr int kQXO = RPST_W4Q_AL ? 4 : 1;    // patch columns staged left of the tile
constexpr int kQPS = RPST_W4Q_AL ? 72 : 68;  // patch row stride (floats): 66 used columns
constexpr int kQCS = 768;                    // patch channel stride (floats)
constexpr int kQWS = 9216;                   // weight floats per (co tile, K step)
constexpr int kQPAT = 4 * kQCS;              // patch stage: 4 channels (12 KiB)
constexpr int kQNTH = 512;
constexpr int kQMaxCo = 512;                 // output channels the LDS bias table holds
constexpr int kQWPI = 5;                     // 1-KiB weight pieces per wave and step (36 / 8)
constexpr int kQWide = 2, kQSlow = 6;        // patch pieces per wave and step: 16-B / 4-B
constexpr int kQDMA4 = 3, kQDMA = RPST_W4Q_AL ? 12 : 11;  // patch pieces per channel: 16-B / 4-B
constexpr int kQRP = kQPS / 4;               // 16-B pieces per patch row
constexpr int kQXS = 4 * 3 * 3 * 64 * 2;     // epilogue exchange floats per tile row and pass
// timing-only experiments (results wrong; tools/build_variants.sh -DRPST_W4Q_DBG=n): 1 no patch
// DMA, 2 no weight DMA, 4 no epilogue exchange, 8 no input transform, 16 no step barriers,
// 32 no epilogue at all, 64 no output stores (issued never), 128 no DMA waits, 256 no output
// transform. Round 6 on the final kernel, 128->256 @512^2 N64 (profiles/r06/epilogue_ab.log):
// 26.8 ms; no epilogue 25.3; no output stores 24.8; no exchange 25.7; no transform 26.1
#ifndef RPST_W4Q_WG0
#define RPST_W4Q_WG0 0  // MFMA group of a step whose issue slot takes the first W(x + 1) piece
#endif
#ifndef RPST_W4Q_PG
#define RPST_W4Q_PG 5   // MFMA group after which the P(x + 4) pieces are issued
#endif
#ifndef RPST_W4Q_AHEAD
// MFMA groups whose A operands are read ahead: configs[1] 539.7 / 541.7 img/s at 2, 545.2 /
// 546.6 at 3 (128->256 N64 28.05 -> 27.65 ms), 537 at 4, 522 at 5 (tools/ab_bench_libs.sh,
// profiles/r05/ahead_ab.log)
#define RPST_W4Q_AHEAD 3
#endif
static_assert(10 * kQRP <= kQDMA4 * 64 && kQDMA4 * 256 <= kQCS, "16-B pieces in a channel");
static_assert(10 * kQPS <= kQDMA * 64 && kQDMA * 64 <= kQCS, "4-B pieces in a channel");
static_assert(2 * kQWide >= kQDMA4 && 2 * kQSlow >= kQDMA && 8 * kQWPI >= 36, "coverage");
static_assert(2 * kQXS <= kQWS, "the exchange fits a weight stage");
static_assert((2 * kQWS + 4 * kQPAT) * 4 + 1024 + kQSlow * kQNTH * 4 + 9 * kQMaxCo * 4 <= 163840,
              "LDS");

// ---- weight transform + packing -------------------------------------------------------
// packed[((((ct * K4 + ks) * 4 + q) * 9 + p) * 64 + l) * 4 + cb] = U_xi[co][ci] with
// xi = (3 (q >> 1) + p / 3, 3 (q & 1) + p % 3) (transformed row, column), co = 64 ct + 16 cb +
// (l & 15), ci = 4 ks + (l >> 4): lane l's A operands of position p for the four 16-channel
// blocks are one 16-B word, and one (co tile, K step) slice is contiguous (the LDS-DMA copies
// it verbatim). TW = float (the layer's weights) or double (per-image folded weights).
template <typename TW>
__global__ void wino4q_pack_kernel(const TW* __restrict__ w, float* __restrict__ pk, int Cout,
                                   int Cin, int K4, int64_t per, int64_t total, int64_t sco,
                                   int64_t sci, int64_t stap) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int64_t img = t / per;
  pk += img * per;
  w += img * (int64_t)Cout * Cin * 9;
  t -= img * per;
  const int cb = (int)(t & 3);
  int64_t r = t >> 2;
  const int l = (int)(r & 63);
  r >>= 6;
  const int p = (int)(r % 9);
  r /= 9;
  const int q = (int)(r & 3);
  r >>= 2;
  const int ks = (int)(r % K4);
  const int ct = (int)(r / K4);
  const int i = 3 * (q >> 1) + p / 3, jj = 3 * (q & 1) + p % 3;
  const int co = ct * kQCo + cb * 16 + (l & 15);
  const int ci = ks * 4 + (l >> 4);
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
      for (int s = 0; s < 3; ++s) acc += G[i][u] * (double)g[(u * 3 + s) * stap] * G[jj][s];
    v = (float)acc;
  }
  pk[t] = v;
}

size_t wino4q_packed_floats(int Cout, int Cin) {
  return (size_t)((Cout + kQCo - 1) / kQCo) * ((Cin + 3) / 4) * kQWS;
}

int wino4q_pack(const float* w, float* pk, int Cout, int Cin, hipStream_t st) {
  const int64_t t = (int64_t)wino4q_packed_floats(Cout, Cin);
  wino4q_pack_kernel<float><<<(unsigned)((t + 255) / 256), 256, 0, st>>>(
      w, pk, Cout, Cin, (Cin + 3) / 4, t, t, (int64_t)Cin * 9, 9, 1);
  return launch_status("wino4q_pack_kernel");
}

// per-image folded weights (wino4_mix): W'_n in [n][tap][co][ci] (fp64)
int wino4q_pack_mix(const double* wm, float* pk, int N, int Cout, int Cin, hipStream_t st) {
  const int64_t per = (int64_t)wino4q_packed_floats(Cout, Cin), tot = (int64_t)N * per;
  wino4q_pack_kernel<double><<<(unsigned)((tot + 255) / 256), 256, 0, st>>>(
      wm, pk, Cout, Cin, (Cin + 3) / 4, per, tot, Cin, 1, (int64_t)Cout * Cin);
  return launch_status("wino4q_pack_kernel(mix)");
}

// AdaIN folded into per-image weights: out_n = U scaled by s = std_s / std_c along ci
// (aux = [mean_c | mean_s | std_c | std_s], each N * Cin)
__global__ void wino4q_fold_w_kernel(const float4* __restrict__ pk, float4* __restrict__ out,
                                     const float* __restrict__ aux, int N, int Cin, int K4,
                                     int64_t per4) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N * per4) return;
  const int n = (int)(t / per4);
  const int64_t u = t - (int64_t)n * per4;  // float4 index: ((ct * K4 + ks) * 36 + q * 9 + p) * 64 + l
  const int l = (int)(u & 63);
  const int ks = (int)((u / (kQWS / 4)) % K4);
  const int ci = ks * 4 + (l >> 4);
  const int64_t nc = (int64_t)N * Cin, i = (int64_t)n * Cin + (ci < Cin ? ci : 0);
  const float sc = ci < Cin ? aux[3 * nc + i] / aux[2 * nc + i] : 0.f;
  const float4 v = pk[u];
  out[t] = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
}

int wino4q_fold_w(const float* pk, float* out, const float* aux, int N, int Cout, int Cin,
                  hipStream_t st) {
  const int64_t per4 = (int64_t)wino4q_packed_floats(Cout, Cin) / 4, n4 = (int64_t)N * per4;
  wino4q_fold_w_kernel<<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const float4*>(pk), reinterpret_cast<float4*>(out), aux, N, Cin,
      (Cin + 3) / 4, per4);
  return launch_status("wino4q_fold_w_kernel");
}

// the layers this kernel takes: DMA loaders (NONE, UPSAMPLE2), >= 64 output channels (a
// 64-channel co tile; narrower layers stay on rpst_wino4.hip's 32-channel tile) and >= 128
// input channels in multiples of 16 (a co tile = a whole number of 4-step ring turns).
// Below 128 input channels a block's 8-16 K steps per co tile leave the prologue and the
// 4-way epilogue exposed: 32->64 @512^2 N64 3.12 vs 2.54 ms, 64->128 8.16 vs 8.09 on the
// 32-channel kernel (gpurun_out/w4q_d, profiles/r05). Mode (conv_quarter_mode: the calling
// thread's rpst_conv2d_set_quarter, else RPST_W4Q read per launch like RPST_CONV_ALGO): 0
// off, 1 the rule above, 2 forced on for every shape it supports (Cin >= 16; parity tests,
// A/B). A training step's constant branches (rpst_conv2d_set_precise(2)) keep the 32-channel
// form: same per-conv error (tools/conv_err.py), but the gradient goldens were pinned on its
// rounding pattern.
bool wino4q_applies(int Cin, int Cout, int in_op) {
  const int en = conv_quarter_mode();
  const int min_cin = en == 2 ? 16 : 128;
  return en && conv_quarter_allowed() && (in_op == RPST_IN_NONE || in_op == RPST_IN_UPSAMPLE2) &&
         Cout >= 64 && Cout <= kQMaxCo &&
         Cin >= min_cin && Cin % 16 == 0;
}

// ---- the epilogue of one finished 4x4 tile and channel ---------------------------------
struct QEpi {
  int W, H, Cout, gy0, gx0, rows, n, sidx;
  bool vec, full, bst, edge, store, pool;
  float inv, slope;
  unsigned voff[4];
  float* out;
  float* oimg;
  unsigned obytes;
  const float* btab;
  float2* statp;
  int statP;
};

// Block order (tools/ab_bench_libs.sh, profiles/r05/order_ab.log; configs[1], two rounds):
// row tile fastest with the hardware's round-robin XCD assignment (consecutive blocks on
// consecutive XCDs) 553.3 / 553.1 img/s; column tile fastest with consecutive logical blocks
// on one XCD (xcd_swizzle, the round-4 choice) 548.3 / 547.3; row tile fastest swizzled
// 534.7; column tile fastest unswizzled 536.2; image-fastest orders 503-538.
#ifndef RPST_W4Q_ORDER  // 0 column tile fastest, 1 row tile fastest, 2 / 3 image-fastest forms
#define RPST_W4Q_ORDER 1
#endif
#ifndef RPST_W4Q_SWZ  // 1: consecutive logical blocks on one XCD (xcd_swizzle)
#define RPST_W4Q_SWZ 0
#endif
__device__ __forceinline__ int q_block_id() {
  return RPST_W4Q_SWZ ? xcd_swizzle(blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
}
__device__ __forceinline__ void q_tile(int b, int tiles_x, int tiles_y, int cosplit, int& tx,
                                       int& ty, int& n) {
  if (RPST_W4Q_ORDER == 1) {
    ty = b % tiles_y;
    b /= tiles_y;
    tx = b % tiles_x;
    n = b / tiles_x;
  } else if (RPST_W4Q_ORDER == 2) {  // image fastest, then row tile, column tile
    const int nimg = (int)(gridDim.x / ((unsigned)tiles_x * tiles_y * cosplit));
    n = b % nimg;
    b /= nimg;
    ty = b % tiles_y;
    tx = b / tiles_y;
  } else if (RPST_W4Q_ORDER == 3) {  // row tile, image, column tile
    const int nimg = (int)(gridDim.x / ((unsigned)tiles_x * tiles_y * cosplit));
    ty = b % tiles_y;
    b /= tiles_y;
    n = b % nimg;
    tx = b / nimg;
  } else {
    tx = b % tiles_x;
    b /= tiles_x;
    ty = b % tiles_y;
    n = b / tiles_y;
  }
}

__device__ __forceinline__ QEpi q_epi_ctx(int wr, int tn) {
  const QArgs L = q_args();
  QEpi e;
  e.W = L->W;
  e.H = L->H;
  e.Cout = L->Cout;
  e.slope = L->relu == RPST_ACT_RELU ? 0.f : (L->relu == RPST_ACT_LRELU ? 0.2f : 1.f);
  int btx, bty;
  q_tile(q_block_id() / L->cosplit, L->tiles_x, L->tiles_y, L->cosplit, btx, bty, e.n);
  const int bx0 = btx * kQTW;
  e.gy0 = bty * kQTH + 4 * wr;
  e.gx0 = bx0 + 4 * tn;
  e.vec = (e.W & 3) == 0 && e.gx0 + 3 < e.W;
  e.rows = max(0, min(4, e.H - e.gy0));
  const int cols = max(0, min(kQTW, e.W - bx0));
  // (v_rcp: exact for the 256-pixel full tiles; the IEEE division's ~10-instruction sequence
  // ran per channel)
  e.inv = e.rows * cols > 0 ? __builtin_amdgcn_rcpf((float)(e.rows * cols)) : 0.f;
  e.full = e.rows == 4 && bx0 + kQTW <= e.W;
  e.edge = e.gy0 == 0 || e.gy0 + 4 >= e.H || bx0 == 0 || bx0 + kQTW >= e.W;
  e.out = L->out;
  const int64_t plane = (int64_t)e.H * e.W;
  e.pool = L->pool_out != 0;
  e.bst = !e.pool && (e.W & 3) == 0 && (int64_t)e.Cout * plane * 4 < (1LL << 31);
  e.oimg = e.out + (int64_t)e.n * e.Cout * plane;
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
  e.sidx = (bty * L->tiles_x + btx) * 2 + wr;
  return e;
}

// bias (interior class for BTAB) already in Y; border classes, activation, statistics
// partial, store (or 2x2 ceil-mode max pool) of channel co of this lane's tile
template <bool STATS, bool BTAB, bool RELU>
__device__ __forceinline__ void q_finish(const QEpi& e, int co, float (&Y)[16], int tn) {
  const int gy0 = e.gy0, gx0 = e.gx0, rows = e.rows, n = e.n;
  const bool cok = co < e.Cout;
  if constexpr (BTAB) {
    if (e.edge) {
      const float* bt = e.btab + (cok ? co : 0) * 9;  // this image's table, in LDS
      float b9[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) b9[i] = cok ? bt[i] : 0.f;
      const float b4 = b9[4];
#pragma unroll
      for (int i = 0; i < 9; ++i) b9[i] -= b4;
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
  }
#pragma unroll
  for (int i = 0; i < 16; ++i)
    Y[i] = __builtin_amdgcn_fmed3f(Y[i], RELU ? 0.f : e.slope * Y[i], __builtin_inff());
  float sum = 0.f;
  if constexpr (STATS) {
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
  if ((RPST_W4Q_DBG & 64) && e.statP > -7) {  // timing only: the stores never taken
  } else if (e.bst) {
    const auto ro = q_rsrc(e.oimg, e.obytes, true);
    const unsigned cofs = cok ? (unsigned)co * (unsigned)(e.H * e.W) * 4u : 0x7fffffffu;
#pragma unroll
    for (int yy = 0; yy < 4; ++yy) {
      const floatx4 v = {Y[yy * 4], Y[yy * 4 + 1], Y[yy * 4 + 2], Y[yy * 4 + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro,
                                             (int)(e.voff[yy] + cofs), 0, RPST_W4_CPOL);
    }
  } else if (e.pool) {
    // max_pool2d(2, 2, ceil_mode) of the finished tile, fmaxf in maxpool2_kernel's order
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
#ifndef RPST_W4Q_SDBG
#define RPST_W4Q_SDBG 0
#endif
  if constexpr (STATS) {
    if (!(RPST_W4Q_SDBG & 4)) sum = q_row16_sum(sum);
    const float mean = sum * e.inv;
    float m2 = 0.f;
    if (RPST_W4Q_SDBG & 2) {
    } else if (e.full) {
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
    if (RPST_W4Q_SDBG & 2) m2 = mean;
    if (!(RPST_W4Q_SDBG & 4)) m2 = q_row16_sum(m2);
    // partials in [n][partial][co] order (stat_merge_t_kernel): a wave's 16 channels of one
    // partial fill whole cache lines (in [n][co][partial] order they were 8-B pieces
    // scattered over 16 planes). Statistics cost, 128->256 N64 (tools/ab_stats.py): 1.5 ms
    // of 28.4, of which the store 0.2 (SDBG 8: the store kept but never taken at run time),
    // the centred-square pass 0.33 (SDBG 2); SDBG 1 drops the whole computation (dead code)
    if (!(RPST_W4Q_SDBG & 1) && tn == 0 && cok && (!(RPST_W4Q_SDBG & 8) || e.statP < 0))
      e.statp[((int64_t)n * e.statP + e.sidx) * e.Cout + co] = make_float2(mean, m2);
  }
}

template <int INOP, bool STATS, bool BTAB, bool RELU>
__global__ __launch_bounds__(kQNTH, 1) void wino4q_mfma_kernel(ConvArgs a) {
  // ring: weights in 2 stages (W(x) in wsx % 2), patches in 4 (P(x) in ps x % 4); a co tile
  // has a multiple of 4 K steps (wino4q_applies: Cin % 16 == 0), so its steps run as a
  // 4-unrolled loop whose stage objects are fixed per position, and its last step always
  // reads ws1 -- the epilogue's exchange region. One __shared__ object per stage: the stage a
  // step reads and the ones its DMA fills are distinct objects, so the compiler's wait
  // insertion does not drain the in-flight DMA before the LDS reads.
  __shared__ __attribute__((aligned(16))) float ws0[kQWS];
  __shared__ __attribute__((aligned(16))) float ws1[kQWS];
  __shared__ __attribute__((aligned(16))) float ps0[kQPAT];
  __shared__ __attribute__((aligned(16))) float ps1[kQPAT];
  __shared__ __attribute__((aligned(16))) float ps2[kQPAT];
  __shared__ __attribute__((aligned(16))) float ps3[kQPAT];
  __shared__ __attribute__((aligned(16))) float dummy[256];  // target of padding DMA pieces
  // per-lane patch source offsets (in registers they are spilled, and every reload's vmcnt
  // wait drains the DMA ring): each lane reads only its own column
  __shared__ unsigned poffs[kQSlow][kQNTH];
  // the layer's biases (BTAB: this image's 9 border-class biases per channel), copied once
  // per block before the ring starts: a global load in the epilogue would take a
  // compiler-inserted vmcnt(0) that drains the in-flight DMA ring (wino4q_applies: Cout <= 512)
  __shared__ float btl[BTAB ? 9 * kQMaxCo : kQMaxCo];

  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int k = lane >> 4, tn = lane & 15, wr = wave >> 2;

  // block -> (co-split group, column tile, row tile, image); XCD-swizzled
  int bid = q_block_id();
  const int cog = bid % a.cosplit;
  bid /= a.cosplit;
  const int nct = a.co_tiles / a.cosplit, ct0 = cog * nct;
  int tx, ty, n;
  q_tile(bid, a.tiles_x, a.tiles_y, a.cosplit, tx, ty, n);
  const int K4 = a.nchunks, G = nct * K4;
  const int y0 = ty * kQTH, x0 = tx * kQTW;

  {
    const int nb = BTAB ? 9 * a.Cout : a.Cout;
    const float* src = BTAB ? a.btab + (int64_t)n * nb : a.bias;
    for (int i = threadIdx.x; i < nb; i += kQNTH) btl[i] = src ? src[i] : 0.f;
  }
  constexpr bool up = INOP == RPST_IN_UPSAMPLE2;
  const unsigned in_plane = up ? (unsigned)(a.Hs * a.Ws) : (unsigned)(a.H * a.W);
  const unsigned oob = a.Cin * in_plane * 4u;  // a padding position's (out-of-range) offset
  const float* in_img = conv_in_img(a, n, (int64_t)a.Cin * in_plane);
  const unsigned wbytes = (unsigned)(nct * K4 * kQWS) * 4u;  // this block's co tiles
  const float* w_img = a.wpk + (int64_t)n * a.wstride + (int64_t)ct0 * K4 * kQWS;

  // patch of one K step: 4 channels x [10 rows][68] (66 columns + 2 spare) at channel stride
  // 768; waves 2c, 2c + 1 fill channel c. Interior blocks (every patch column inside the
  // image, no upsampling): 16-B pieces (a 72-float row from x0 - 4 = 18 pieces, 16-B aligned
  // sources, 180 per channel, 3 wave-instructions: half 0 takes 0-1, half 1 takes 2 + a
  // padding piece; columns x0 - 4 .. x0 - 2 and past x0 + 64 are staged but never read);
  // elsewhere 4-B pieces (element 64 p + lane resolved against the padding, 12 per channel,
  // 6 per half). RPST_W4Q_AL 0 stages from x0 - 1 (68-float rows, 4-B aligned sources):
  // 128->256 N64 26.69-26.94 -> 26.55-26.61 ms, folded 256->128 13.01-13.12 -> 12.75-12.96
  // (profiles/r06/aligned_patch_ab.log).
  // Per-lane source offsets are resolved once per block.
  const int hf = wave & 1;
  const bool zp = a.pad == RPST_PAD_ZERO;
  const int rs = up ? a.Ws : a.W;
  // RPST_W4Q_EDGE (with the aligned rows): in a row of W % 4 == 0 floats a 16-B piece is
  // wholly inside or outside the image, so the full-width x-edge tiles take the 16-B pieces
  // too: outside pieces read zero (zero padding), and reflect padding's one halo column is
  // copied in after the stage lands (fix_halo)
  const bool w4a = RPST_W4Q_AL && RPST_W4Q_EDGE && (a.W & 3) == 0;
  const bool wide = !up && ((x0 >= 1 && x0 + kQTW < a.W) || (w4a && x0 + kQTW <= a.W));
  const bool fixL = wide && w4a && !zp && x0 == 0;
  const bool fixR = wide && w4a && !zp && x0 + kQTW == a.W;
  unsigned poff[kQSlow];
  const int tid = threadIdx.x;
  if (wide) {
#pragma unroll
    for (int i = 0; i < kQWide; ++i) {
      const int p = kQWide * hf + i;
      const int f = 64 * p + lane, row = min(f / kQRP, 9), j = f - (f / kQRP) * kQRP;
      int y = y0 - 1 + row;
      const int xs = x0 - kQXO + 4 * j;
      const bool okx = !w4a || (xs >= 0 && xs + 3 < a.W);
      const bool ok = p < kQDMA4 && f < 10 * kQRP && q_resolve(y, a.H, zp) && okx;
      poff[i] = ok ? ((unsigned)(y * rs) + (unsigned)xs) * 4u : oob;
    }
#pragma unroll
    for (int i = kQWide; i < kQSlow; ++i) poff[i] = oob;
  } else {
#pragma unroll
    for (int i = 0; i < kQSlow; ++i) {
      const int p = kQSlow * hf + i;
      const int f = 64 * p + lane;
      const int row = min(f / kQPS, 9), col = f - (f / kQPS) * kQPS;
      int y = y0 - 1 + row, x = x0 - kQXO + col;
      const bool oky = q_resolve(y, a.H, zp), okx = q_resolve(x, a.W, zp);
      const bool ok = p < kQDMA && col >= kQXO - 1 && col < kQXO + 1 + kQTW &&
                      f < 10 * kQPS && oky && okx;
      poff[i] = ok ? ((unsigned)((up ? y >> 1 : y) * rs) + (unsigned)(up ? x >> 1 : x)) * 4u : oob;
    }
  }
#pragma unroll
  for (int i = 0; i < kQSlow; ++i) poffs[i][tid] = poff[i];

  // weight slice of step g (the block's co tiles' slices are consecutive) into stage stg:
  // pieces w + 8 i of its 36 1-KiB pieces; pieces 32-35 come from waves 0-3, waves 4-7 issue
  // a padding piece into the dummy. Dead steps (g >= G) read zero records.
  constexpr int DBG = RPST_W4Q_DBG;
  auto issue_w = [&](int g, float* stg, int i) {
    if (DBG & 2) return;
    const int wv = q_launder(wave);
    const int pc = wv + 8 * i;
    const bool live = g < G;
    const int so = q_mask((g * kQWS + pc * 256) * 4, live);
    if (i < 4) {
      q_dma16(q_rsrc(w_img, wbytes, live), stg + pc * 256, lane * 16, so);
    } else {
      const bool real = pc < 36;
      q_dma16(q_rsrc(w_img, wbytes, live && real), real ? stg + pc * 256 : dummy, lane * 16,
              q_mask(so, real));
    }
  };
  // every patch piece of this wave for step g (K step ks) into stage stg
  auto issue_p = [&](auto WIDEc, int g, int ks, float* stg) {
    constexpr bool WIDE = decltype(WIDEc)::value;
    if (DBG & 1) return;
    const int wv = q_launder(wave);
    const int c = 4 * ks + (wv >> 1);
    const bool ok = g < G && c < a.Cin;
    const auto r = q_rsrc(in_img, oob, ok);
    const int so = q_mask((int)((unsigned)c * in_plane * 4u), ok);
    float* xs = stg + (wv >> 1) * kQCS;
    const bool h1 = (wv & 1) != 0;
    if constexpr (WIDE) {
      q_dma16(r, xs + (h1 ? 512 : 0), poffs[0][tid], so);
      q_dma16(r, h1 ? dummy : xs + 256, poffs[1][tid], so);
    } else {
#pragma unroll
      for (int i = 0; i < kQSlow - 1; ++i)
        q_dma4(r, xs + 64 * (h1 ? kQSlow + i : i), poffs[i][tid], so);
      q_dma4(r, h1 && !RPST_W4Q_AL ? dummy : xs + 64 * (h1 ? 2 * kQSlow - 1 : kQSlow - 1),
             poffs[kQSlow - 1][tid], so);
    }
  };
  // before step x's barrier: W(x) (issued in step x - 1 ahead of its patch group) and
  // everything older have landed; that youngest patch group (2 / 6 pieces) stays in flight
  // The first wait after an epilogue leaves its output stores in flight too: on the buffer-
  // store path (q_epi_ctx's bst, kernel-uniform) every wave issues exactly 16 (4 channels x 4
  // rows; the statistics partial stores come after them, so counting only these 16 is
  // conservative). Waiting them out (vmcnt(2)) stalled every co tile's first step on the
  // stores' write acknowledgements.
  const bool bst_all = !a.pool_out && (a.W & 3) == 0 &&
                       (int64_t)a.Cout * a.H * a.W * 4 < (1LL << 31);
  bool post_epi = false;
  auto wait_ring = [&](bool first) {
    if (DBG & 128) return;
    if (first && post_epi && bst_all) {
      if (wide) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
    } else if (wide) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    if (first) post_epi = false;
  };

  // reflect halo of an x-edge tile staged from 16-B pieces: wave 0 copies column x0 + 1 (LDS
  // column kQXO + 1) into x0 - 1 (kQXO - 1), wave 1 column x0 + 62 into x0 + 64; lanes 0-39
  // take channel l / 10, row l % 10 of the stage
  auto fix_halo = [&](float* stg) {
    if ((wave == 0 && fixL) || (wave == 1 && fixR)) {
      int l = lane;
      asm volatile("" : "+v"(l));
      if (l < 40) {
        const int ch = l / 10, row = l - 10 * ch;
        float* rp = stg + ch * kQCS + row * kQPS;
        if (wave == 0) rp[kQXO - 1] = rp[kQXO + 1];
        else rp[kQXO + kQTW] = rp[kQXO + kQTW - 2];
      }
    }
  };
  // ---- prologue: P(0), P(1), W(0), P(2), P(3) -------------------------------------------
  auto prologue = [&](auto WIDEc) {
    issue_p(WIDEc, 0, 0, ps0);
    issue_p(WIDEc, 1, 1, ps1);
#pragma unroll
    for (int i = 0; i < kQWPI; ++i) issue_w(0, ws0, i);
    issue_p(WIDEc, 2, 2, ps2);
    issue_p(WIDEc, 3, 3, ps3);
  };
  if (wide) prologue(std::true_type{});
  else prologue(std::false_type{});
  wait_ring(false);  // P(3) may stay in flight; conservative for P(2)
  q_lds_barrier();
  if (fixL || fixR) {  // P(0), P(1) (P(x + 2) is fixed in step x)
    fix_halo(ps0);
    fix_halo(ps1);
    q_lds_barrier();
  }

  auto body = [&](auto Qc) {
    constexpr int Q = decltype(Qc)::value, QR = Q >> 1, QC = Q & 1;
    floatx4 acc[9][4];
#pragma unroll
    for (int p = 0; p < 9; ++p)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[p][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
    // lane (k, tn) reads rows 4 wr + QR .. + 4 of channel k of a patch, columns 4 tn .. + 7
    // (two conflict-free ds_read_b128; the empty asm keeps them whole, the compiler would
    // otherwise narrow them to the 5 floats a quarter uses, as bank-conflicted b32 reads)
    const int roff = k * kQCS + (4 * wr + QR) * kQPS + 4 * tn;
    auto read_row = [&](const float* stg, int rr, float (&d)[8]) {
      if (RPST_W4Q_AL) {
        // window columns 4 tn .. + 5 sit at LDS columns 4 tn + 3 .. + 8: the quarter's five
        // (QC = 0: 0-4, QC = 1: 1-5) as two aligned ds_read_b128 (a ds_read_b32 for the odd
        // one: all 64 lanes in one pass, and the four channel groups k share its banks)
        const float* rp = stg + roff + rr * kQPS;
        if (RPST_W4Q_ALRD == 2) {
          floatx4 e = *reinterpret_cast<const floatx4*>(rp + (QC ? 8 : 0));
          floatx4 u = *reinterpret_cast<const floatx4*>(rp + 4);
          asm("" : "+v"(e), "+v"(u));
          d[0] = QC ? 0.f : e[3]; d[1] = u[0]; d[2] = u[1]; d[3] = u[2]; d[4] = u[3];
          d[5] = QC ? e[0] : 0.f; d[6] = 0.f; d[7] = 0.f;
        } else {
          floatx4 u = *reinterpret_cast<const floatx4*>(rp + 4);
          const float e = QC ? rp[8] : rp[3];
          asm("" : "+v"(u));
          d[0] = QC ? 0.f : e; d[1] = u[0]; d[2] = u[1]; d[3] = u[2]; d[4] = u[3];
          d[5] = QC ? e : 0.f; d[6] = 0.f; d[7] = 0.f;
        }
        return;
      }
      floatx4 u = *reinterpret_cast<const floatx4*>(stg + roff + rr * kQPS);
      floatx4 v = *reinterpret_cast<const floatx4*>(stg + roff + rr * kQPS + 4);
      asm("" : "+v"(u), "+v"(v));
      d[0] = u[0]; d[1] = u[1]; d[2] = u[2]; d[3] = u[3];
      d[4] = v[0]; d[5] = v[1]; d[6] = v[2]; d[7] = v[3];
    };
    // column pass of one row (this quarter's 3 transformed columns)
    auto col_pass = [&](const float (&d)[8], float (&u)[3]) {
      if (DBG & 8) {
        u[0] = d[0]; u[1] = d[1]; u[2] = d[2];
        return;
      }
      q_bt3<QC>(d[0], d[1], d[2], d[3], d[4], d[5], u[0], u[1], u[2]);
    };
    // row pass of column j: u[rr] holds input row QR + rr, so QR = 1's half (inputs 1..5)
    // takes u[0..4] as its inputs 1..5. V[p], p = 3 i + j: transformed row 3 QR + i,
    // column 3 QC + j
    auto row_pass = [&](const float (&u)[5][3], int j, float (&v)[9]) {
      if (DBG & 8) {
        v[j] = u[0][j]; v[3 + j] = u[2][j]; v[6 + j] = u[4][j];
        return;
      }
      if constexpr (QR == 0)
        q_bt3<0>(u[0][j], u[1][j], u[2][j], u[3][j], u[4][j], 0.f, v[j], v[3 + j], v[6 + j]);
      else
        q_bt3<1>(0.f, u[0][j], u[1][j], u[2][j], u[3][j], u[4][j], v[j], v[3 + j], v[6 + j]);
    };
    float V[9];
    {  // V(0), not pipelined
      float u[5][3];
#pragma unroll
      for (int rr = 0; rr < 5; ++rr) {
        float d[8];
        read_row(ps0, rr, d);
        col_pass(d, u[rr]);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) row_pass(u, j, V);
    }

    const int woff = Q * 9 * 256 + lane * 4;  // this wave's A operands in a weight stage
    int x = 0;                                // global K step
    // one K step: W(x) from wsx, P(x + 1) from psn (-> V(x + 1)), DMA W(x + 1) into wsn and
    // P(x + 4) into psx. MFMA groups in column-major position order, so the row pass of
    // column j overwrites V[j], V[3 + j], V[6 + j] after their last use.
    // (first: the step that may follow an epilogue, the first of an iteration)
    auto step = [&](float* wsx, float* psn, float* wsn, float* psx, float* pfx, int ks,
                    bool first) {
      wait_ring(first);
      if (DBG & 16) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else q_lds_barrier();  // W(x), P(x + 1) complete; every wave is done with step x - 1
      constexpr int ord[9] = {0, 3, 6, 1, 4, 7, 2, 5, 8};
      constexpr int kA = RPST_W4Q_AHEAD;  // A-operand groups read ahead
      float4 w4[9];
#pragma unroll
      for (int q = 0; q < kA; ++q)
        w4[ord[q]] = *reinterpret_cast<const float4*>(wsx + woff + ord[q] * 256);
      float d[8];
      read_row(psn, 0, d);
      float u[5][3];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int p = ord[q];
        if (q + kA < 9)
          w4[ord[q + kA]] = *reinterpret_cast<const float4*>(wsx + woff + ord[q + kA] * 256);
        q_mfma<1>(acc[p][0], w4[p].x, V[p]);  // V[p] / a zeroed accumulator may be fresh
        q_mfma<0>(acc[p][1], w4[p].y, V[p]);
        q_mfma<0>(acc[p][2], w4[p].z, V[p]);
        q_mfma<0>(acc[p][3], w4[p].w, V[p]);
        if (q >= RPST_W4Q_WG0 && q < RPST_W4Q_WG0 + kQWPI) issue_w(x + 1, wsn, q - RPST_W4Q_WG0);
        // P(x + 4): K step ks + 4 of this co tile, or of the next one
        if (q == RPST_W4Q_PG) {
          const int k4 = ks + 4 < K4 ? ks + 4 : ks + 4 - K4;
          if (wide) issue_p(std::true_type{}, x + 4, k4, psx);
          else issue_p(std::false_type{}, x + 4, k4, psx);
        }
        // pipelined transform of P(x + 1): rows at groups 0-4, column j's row pass at
        // groups 5, 6 and (after its MFMAs) 8
        if (q < 5) {  // row q (read one group ahead) -> u[q], then read row q + 1
          col_pass(d, u[q]);
          if (q + 1 < 5) read_row(psn, q + 1, d);
        }
        if (q == 5 || q == 6 || q == 8) row_pass(u, q == 8 ? 2 : q - 5, V);
        // P(x + 2) landed for every wave at this step's barrier and is read from step x + 1
        if (q == 7) fix_halo(pfx);
      }
      ++x;
    };

    // epilogue of co tile ctile (its last step read ws1): the quarters of a tile row exchange
    // their blocks through ws1 and each wave finishes its own 16 channels (co = 64 ctile +
    // 16 Q + 4 k + r) of tile (wr, tn)
    auto epilogue = [&](int ctile) {
#ifdef RPST_W4Q_NOEPI  // register-pressure experiment: keep the accumulators live only
      {
        float t = 0.f;
#pragma unroll
        for (int p = 0; p < 9; ++p)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) t += acc[p][cb][0] + acc[p][cb][1] + acc[p][cb][2] + acc[p][cb][3];
        q_args()->out[threadIdx.x + ctile] = t;
#pragma unroll
        for (int p = 0; p < 9; ++p)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) acc[p][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
        return;
      }
#endif
      if (DBG & 32) {  // keep the accumulators live, skip the epilogue
        float t = 0.f;
#pragma unroll
        for (int p = 0; p < 9; ++p)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) t += acc[p][cb][0];
        if (t == 1.2345f) q_args()->out[threadIdx.x] = t;
#pragma unroll
        for (int p = 0; p < 9; ++p)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) acc[p][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
        return;
      }
      q_lds_barrier();  // every wave is done reading ws1
      // 12 wait states between the last MFMAs and the first reader of their results (8-pass
      // XDL), with every accumulator passed through the statements so no read moves above them
      asm volatile("s_nop 7\n\ts_nop 4" : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[0][2]),
                   "+v"(acc[0][3]), "+v"(acc[1][0]), "+v"(acc[1][1]), "+v"(acc[1][2]),
                   "+v"(acc[1][3]), "+v"(acc[2][0]), "+v"(acc[2][1]), "+v"(acc[2][2]),
                   "+v"(acc[2][3]), "+v"(acc[3][0]), "+v"(acc[3][1]), "+v"(acc[3][2]),
                   "+v"(acc[3][3]), "+v"(acc[4][0]), "+v"(acc[4][1]));
      asm volatile("" : "+v"(acc[4][2]), "+v"(acc[4][3]), "+v"(acc[5][0]), "+v"(acc[5][1]),
                   "+v"(acc[5][2]), "+v"(acc[5][3]), "+v"(acc[6][0]), "+v"(acc[6][1]),
                   "+v"(acc[6][2]), "+v"(acc[6][3]), "+v"(acc[7][0]), "+v"(acc[7][1]),
                   "+v"(acc[7][2]), "+v"(acc[7][3]), "+v"(acc[8][0]), "+v"(acc[8][1]),
                   "+v"(acc[8][2]), "+v"(acc[8][3]));
      const int co0 = ctile * kQCo + 16 * Q + 4 * k;
      // 6 passes (accumulator element pair rp, position row pt): each wave writes its 3
      // positions of row pt of the other quarters' blocks (elements 2 rp, 2 rp + 1) into ws1
      // and, after a barrier, reads the other quarters' positions of its own block. After pass pt it holds transformed rows
      // pt and 3 + pt of M for channels co0 + 2 rp + {0, 1}: their column transform (A^T along
      // the row) runs at once, so only P = M A (6 x 4 per channel) stays live, never M.
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        float P[2][6][4];
#pragma unroll
        for (int pt = 0; pt < 3; ++pt) {
          float* xb = ws1 + wr * kQXS;
#pragma unroll
          for (int dq = 0; dq < 4; ++dq) {
            if (dq == Q || (DBG & 4)) continue;
            const int slot = (Q - dq - 1) & 3;
#pragma unroll
            for (int j = 0; j < 3; ++j)
              *reinterpret_cast<float2*>(xb + (((dq * 3 + slot) * 3 + j) * 64 + lane) * 2) =
                  make_float2(acc[3 * pt + j][dq][2 * rp], acc[3 * pt + j][dq][2 * rp + 1]);
          }
          if (!(DBG & 4)) q_lds_barrier();
          float m[2][2][6];  // [element][row pt / 3 + pt][six columns]
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              float2 v;
              if (s == Q || (DBG & 4)) {
                const int src = (DBG & 4) ? s : Q;
                v = make_float2(acc[3 * pt + j][src][2 * rp], acc[3 * pt + j][src][2 * rp + 1]);
              } else {
                v = *reinterpret_cast<const float2*>(
                    xb + (((Q * 3 + ((s - Q - 1) & 3)) * 3 + j) * 64 + lane) * 2);
              }
              m[0][s >> 1][3 * (s & 1) + j] = v.x;
              m[1][s >> 1][3 * (s & 1) + j] = v.y;
            }
          }
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            q_at6(m[e2][0], P[e2][pt]);
            q_at6(m[e2][1], P[e2][3 + pt]);
          }
          if (!(DBG & 4) && (rp == 0 || pt < 2)) q_lds_barrier();  // the next pass rewrites ws1
        }
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          const int r = 2 * rp + e2;
          // the epilogue context is re-derived per channel from the kernel arguments: kept
          // across the exchange passes it overflows the scalar registers
          QEpi e = q_epi_ctx(wr, tn);
          e.btab = btl;
          float bias = 0.f;
          {
            const int co = co0 + r;
            if (co < e.Cout) bias = BTAB ? btl[co * 9 + 4] : btl[co];
          }
#pragma unroll
          for (int x = 0; x < 4; ++x) P[e2][1][x] += bias;
          float Y[16];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            float c6[6], y[4];
#pragma unroll
            for (int I = 0; I < 6; ++I) c6[I] = P[e2][I][x];
            q_at6(c6, y);
#pragma unroll
            for (int yy = 0; yy < 4; ++yy) Y[yy * 4 + x] = y[yy];
          }
          q_finish<STATS, BTAB, RELU>(e, co0 + r, Y, tn);
        }
      }
#pragma unroll
      for (int p = 0; p < 9; ++p)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[p][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
    };

    // one flat loop over the block's K steps, 4 per iteration (a co tile is a whole number
    // of iterations); the epilogue closes the iteration that ends a co tile (a loop over the
    // co tiles around a loop over their K steps makes the last step's accumulators two-use
    // values, and the compiler then renames every such MFMA's destination)
    int ks = 0, ct = ct0;
    for (int g = 0; g < G; g += 4) {
      step(ws0, ps1, ws1, ps0, ps2, ks, true);
      step(ws1, ps2, ws0, ps1, ps3, ks + 1, false);
      step(ws0, ps3, ws1, ps2, ps0, ks + 2, false);
      step(ws1, ps0, ws0, ps3, ps1, ks + 3, false);
      ks += 4;
      if (ks == K4) {
        epilogue(ct);
        post_epi = true;
        ks = 0;
        ++ct;
      }
    }
  };
#ifdef RPST_W4Q_ONEQ
  body(std::integral_constant<int, 0>{});
  if (0)
#endif
  switch (wave & 3) {
    case 0: body(std::integral_constant<int, 0>{}); break;
    case 1: body(std::integral_constant<int, 1>{}); break;
    case 2: body(std::integral_constant<int, 2>{}); break;
    default: body(std::integral_constant<int, 3>{}); break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the padding DMA has landed too
}

int wino4q_launch(ConvArgs& a, int in_op, hipStream_t st) {
  RPST_REQUIRE(in_op == RPST_IN_NONE || in_op == RPST_IN_UPSAMPLE2,
               "conv2d: winograd4 (quarter) does not support in_op %d", in_op);
  a.Cout_pad = (a.Cout + kQCo - 1) / kQCo * kQCo;
  a.nchunks = (a.Cin + 3) / 4;  // K steps of 4 channels
  a.tiles_x = (a.W + kQTW - 1) / kQTW;
  a.tiles_y = (a.H + kQTH - 1) / kQTH;
  a.co_tiles = a.Cout_pad / kQCo;
  a.stat_P = a.tiles_x * a.tiles_y * 2;
  RPST_REQUIRE((int64_t)a.co_tiles * a.nchunks * kQWS * 4 < (1LL << 31),
               "conv2d: winograd4 weight image exceeds 2 GiB");
  {
    // blocks per spatial tile: the co tiles split over RPST_W4Q_COSPLIT same-XCD blocks
    // (default 1: 128->256 @512^2 N64 27.08 / 27.70 / 29.04 ms at 1 / 2 / 4 blocks, the longer
    // blocks amortise the ring's prologue; gpurun_out/w4q_cs)
    const char* e = getenv("RPST_W4Q_COSPLIT");
    int c = (e && *e) ? atoi(e) : 1;
    c = c < 1 ? 1 : (c > a.co_tiles ? a.co_tiles : c);
    while (a.co_tiles % c) --c;
    a.cosplit = c;
  }
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * a.N * a.cosplit;
  RPST_REQUIRE(blocks <= 0x7fffffffLL, "conv2d: grid too large");
  const unsigned nb = (unsigned)blocks;
  const bool stats = a.stat_part != nullptr, btab = a.btab != nullptr;
  RPST_REQUIRE(!btab || in_op == RPST_IN_NONE, "conv2d: winograd4 bias table with a loader op");
  RPST_REQUIRE(!(stats && btab), "conv2d: winograd4 folded bias with statistics");
#define RPST_W4Q_GO(OP, S, B)                                                  \
  do {                                                                         \
    if (a.relu == RPST_ACT_RELU)                                               \
      wino4q_mfma_kernel<OP, S, B, true><<<nb, kQNTH, 0, st>>>(a);             \
    else                                                                       \
      wino4q_mfma_kernel<OP, S, B, false><<<nb, kQNTH, 0, st>>>(a);            \
  } while (0)
#ifdef RPST_W4Q_DEV
  wino4q_mfma_kernel<RPST_IN_NONE, true, false, true><<<nb, kQNTH, 0, st>>>(a);
  (void)stats; (void)btab;
  if (0)
#endif
  if (in_op == RPST_IN_UPSAMPLE2) {
    if (stats) RPST_W4Q_GO(RPST_IN_UPSAMPLE2, true, false);
    else RPST_W4Q_GO(RPST_IN_UPSAMPLE2, false, false);
  } else {
    if (stats) RPST_W4Q_GO(RPST_IN_NONE, true, false);
    else if (btab) RPST_W4Q_GO(RPST_IN_NONE, false, true);
    else RPST_W4Q_GO(RPST_IN_NONE, false, false);
  }
#undef RPST_W4Q_GO
  return launch_status("wino4q_mfma_kernel");
}

}  // namespace rpst
