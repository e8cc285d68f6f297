// Flash-style SANet attention (network/sanet.py:82-99): O = H softmax(F^T G)^T per image
// without S in memory. Its own translation unit so the MFMA accumulators can live in arch
// VGPRs (-mllvm -amdgpu-mfma-vgpr-form=1, Makefile): the online softmax rescales the O
// accumulator, which the VALU can only do on VGPRs (in AGPRs every rescale became 256
// accvgpr moves and pinned the whole VGPR file, so the LDS operand reads could not be
// issued ahead of the MFMAs that use them).
#include <cstdlib>

#include "rpst_common.h"

namespace rpst {

// ---- flash-style SANet attention (sanet.py:82-99 forward) ------------------------------
// O[c][i] = sum_j H[c][j] softmax_j(S[i][j]), S = F^T G, without S in memory: one workgroup
// per (image, 64 queries), 4 waves (one per SIMD), wave w owning queries 16 w .. 16 w + 15.
// A wave keeps its 16 queries' F column block in registers (Q, C / 4 per lane: the B operand
// of v_mfma_f32_16x16x4_f32 with k = channel 4 s + lane / 16) and their O accumulator (C x 16,
// C / 4 per lane), and walks the keys 16 at a time:
//   S^T (16 keys x 16 queries) = G_tile^T Q        (K = C; A = G[c][key] from LDS)
//   online softmax: running max m and lane-partial sum l per query, O *= exp(m_old - m_new)
//     only when some query's max moved (lazy rescale; rare after the first key blocks)
//   O += H_tile P^T                                (K = 16 keys; A = H[c][4 keys] from LDS)
// The S^T accumulator of lane l holds keys 4 (l / 16) + r, query l % 16 -- exactly the B
// operand of the second product for k-step r when k-step r covers keys 4 (l / 16) + r, so P
// never leaves the registers. G and H tiles (C x 16 fp32 each) stream into a double-buffered
// LDS ring by LDS-DMA one key block ahead (one barrier per key block); the H tile is stored
// with its 16-B segments XOR-swizzled by (c / 4) % 4 so that the ds_read_b128 of 16 lanes
// reading 16 channel rows is conflict-free. No 1/sqrt(d) (sanet.py:90-91). Keys past HW are
// masked to -inf; queries past HW are not stored. HW % 4 == 0 (16-B rows) and C in
// {64, 128, 256, 512}; other shapes take the two-GEMM path below.
constexpr int kFBM = 64, kFBN = 16;
// timing-only builds (results wrong; tools/build_variants.sh rpst_flash.hip "x:-DRPST_FLDBG=n"):
// 1 no softmax (P = S), 2 no DMA waits / barriers, 4 no DMA, 8 no O update
#ifndef RPST_FLDBG
#define RPST_FLDBG 0
#endif

__device__ __forceinline__ int attn_xcd_swizzle(int b, int nwg) {
  // bijective: consecutive logical ids land on one XCD (b % 8 = hardware XCD of block b)
  const int q = nwg >> 3, r = nwg & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

typedef __attribute__((address_space(3))) void* attn_lds_ptr_t;

// max over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (one query's four key groups): the gfx950
// row-swap permutes (VALU, no LDS round trip as ds_bpermute). A swap of a register with a
// copy of itself leaves (lo, lo) in one and (hi, hi) in the other. The two results are made
// opaque: this compiler folds a combination of them into the first one (max(a, b) -> a)
__device__ __forceinline__ void swap_halves(float v, int rows, float& a, float& b) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  unsigned x, y;
  if (rows == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    x = r[0];
    y = r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    x = r[0];
    y = r[1];
  }
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(x), "+v"(y));
#endif
  a = __builtin_bit_cast(float, x);
  b = __builtin_bit_cast(float, y);
}
__device__ __forceinline__ float rows4_max(float v) {
  float a, b;
  swap_halves(v, 32, a, b);
  swap_halves(fmaxf(a, b), 16, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float rows4_sum(float v) {
  float a, b;
  swap_halves(v, 32, a, b);
  swap_halves(a + b, 16, a, b);
  return a + b;
}
constexpr float kLog2e = 1.4426950408889634f;

// What the kernel forms from a block of scores S (AdaptiveSANet, sanet.py:100-124, runs two
// passes, since its clamp sigmoid(scale (P - c)) / relu-softmax needs each query's final
// softmax statistics before any key's weight is known):
//   AM_SOFTMAX  SANet: online softmax, O = H softmax(S)^T
//   AM_STATS    pass 1: m = max_j S_ij, inv = 1 / sum_j exp(S_ij - m) only (no H, no O)
//   AM_AEA      pass 2, AEAModule (sanet.py:42-47): O = H Q^T, Q = sigmoid(scale (P - c))
//   AM_AEAR     pass 2, AEALReluModule (sanet.py:63-69): Q = softmax_j(relu(P - c)), whose
//               max is known from pass 1 (max_j P_ij = inv_i: m2 = relu(inv - c)), so pass 2
//               accumulates O and sum_j exp(relu(P - c) - m2) with no rescaling
// with P_ij = exp(S_ij - m_i) inv_i. Neither pass writes S: no B x HW x HW workspace.
enum { AM_SOFTMAX = 0, AM_STATS = 1, AM_AEA = 2, AM_AEAR = 3 };
struct AttnRows {
  const float* m;    // AM_AEA / AM_AEAR: pass 1's row max ...
  const float* inv;  // ... and inverse row sum
  const float* c;    // clamp value per query row
  float scale;       // AM_AEA: sigmoid slope (scale_value)
  float* out_m;      // AM_STATS outputs
  float* out_inv;
};

template <int C, bool PIPE, int AM = AM_SOFTMAX>
__global__ __launch_bounds__(256, 1) void sanet_flash_kernel(const float* __restrict__ F,
                                                             const float* __restrict__ G,
                                                             const float* __restrict__ H,
                                                             float* __restrict__ O, int HW,
                                                             int qblocks, AttnRows rows) {
  constexpr int NQ = C / 4;            // Q registers per lane
  constexpr int NMB = C / 16;          // O accumulators (16 channel rows each)
  constexpr int TILE = C * kFBN;       // floats per G / H tile
  constexpr int PPW = TILE / 256 / 4;  // 1-KiB DMA pieces per wave per tile
  static_assert(PPW >= 1 && TILE % 1024 == 0, "C in {64, 128, 256, 512}");
  __shared__ __attribute__((aligned(16))) float Gs0[TILE];
  __shared__ __attribute__((aligned(16))) float Gs1[TILE];
  __shared__ __attribute__((aligned(16))) float Hs0[TILE];
  __shared__ __attribute__((aligned(16))) float Hs1[TILE];

  const int bid = attn_xcd_swizzle(blockIdx.x, (int)gridDim.x);
  const int b = bid / qblocks, qb = bid - b * qblocks;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, lq = lane & 15;
  const int q = qb * kFBM + wave * 16 + lq;  // this lane's query
  const int64_t plane = (int64_t)C * HW;
  const float* Fb = F + b * plane;
  const unsigned bytes = (unsigned)(plane * 4);
  const auto rG = __builtin_amdgcn_make_buffer_rsrc((void*)(G + b * plane), (short)0, (int)bytes, 0x00020000);
  const auto rH = __builtin_amdgcn_make_buffer_rsrc((void*)(H + b * plane), (short)0, (int)bytes, 0x00020000);
  // DMA piece j of a tile: lane -> (channel row 16 j + lane / 4, 16-B segment lane % 4). The
  // whole offset goes in voffset (not the piece's uniform row offset in soffset): the buffer
  // range check covers voffset only, and with HW % 16 != 0 the last key block of the last
  // channel row runs past the image plane -- those keys must read as 0, not as whatever
  // follows the tensor (a non-finite H there would turn 0 * H into NaN in O)
  const int prow = lane >> 2, pseg = lane & 3;
  const unsigned voffG = (unsigned)(prow * HW + 4 * pseg) * 4u;
  const unsigned voffH = (unsigned)(prow * HW + 4 * (pseg ^ ((lane >> 4) & 3))) * 4u;
  // one DMA piece (jj < PPW: G piece jj, else H piece jj - PPW) of key block k0 / 16; a
  // step's 2 PPW pieces are spread one per MFMA group (scores: NQ / SG = 2 PPW groups) so each
  // issue hides in an MFMA gap instead of stalling a clustered run of them
  auto piece = [&](int jj, int k0g, float* gs, int k0h, float* hs) {
    if (RPST_FLDBG & 4) return;
    const bool isg = jj < PPW;
    const int j = wave * PPW + (isg ? jj : jj - PPW);
    if (isg) {
      if (k0g >= 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rG, (attn_lds_ptr_t)(gs + 256 * j), 16, (int)(voffG + (unsigned)(16 * j * HW + k0g) * 4u), 0,
                                                 0, 0);
    } else if (k0h >= 0) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rH, (attn_lds_ptr_t)(hs + 256 * j), 16, (int)(voffH + (unsigned)(16 * j * HW + k0h) * 4u), 0,
                                               0, 0);
    }
  };
  static_assert(NQ / 8 == 2 * PPW, "one DMA piece per MFMA group of scores()");
  auto issue_g = [&](int k0, float* gs) {
#pragma unroll
    for (int jj = 0; jj < PPW; ++jj) {
      const int j = wave * PPW + jj;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rG, (attn_lds_ptr_t)(gs + 256 * j), 16, (int)(voffG + (unsigned)(16 * j * HW + k0) * 4u), 0,
                                               0, 0);
    }
  };
  auto issue_h = [&](int k0, float* hs) {
#pragma unroll
    for (int jj = 0; jj < PPW; ++jj) {
      const int j = wave * PPW + jj;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rH, (attn_lds_ptr_t)(hs + 256 * j), 16, (int)(voffH + (unsigned)(16 * j * HW + k0) * 4u), 0,
                                               0, 0);
    }
  };
  const int nk = (HW + kFBN - 1) / kFBN;
  issue_g(0, Gs0);

  float qv[NQ];
#pragma unroll
  for (int s = 0; s < NQ; ++s) qv[s] = q < HW ? Fb[(int64_t)(4 * s + g) * HW + q] : 0.f;
  // Q lives in AGPRs (the MFMA reads its B operand from there): the arch VGPRs hold the O
  // accumulator (rescaled by the VALU) and the LDS operands read ahead of their MFMAs
#pragma unroll
  for (int s = 0; s < NQ; ++s) asm volatile("" : "+a"(qv[s]));
  floatx4 acc[NMB];
#pragma unroll
  for (int mb = 0; mb < NMB; ++mb) acc[mb] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  // pass 2: this lane's query's row statistics and clamp, exp2 arguments pre-scaled
  float a_mL = 0.f, a_inv = 0.f, a_c = 0.f, a_m2L = 0.f;
  if constexpr (AM >= AM_AEA) {
    if (q < HW) {
      const int64_t r = (int64_t)b * HW + q;
      a_mL = rows.m[r] * kLog2e;
      a_inv = rows.inv[r];
      a_c = rows.c[r];
    }
    a_m2L = fmaxf(a_inv - a_c, 0.f) * kLog2e;
  }
  const int hsw = 4 * (g ^ ((lq >> 2) & 3));  // swizzled segment of keys 4 g .. 4 g + 3

  float p[4] = {0.f, 0.f, 0.f, 0.f};  // P of the key block whose O update is pending
  // LDS operands are read one group ahead of the MFMAs that use them (explicit register
  // double buffering: a wave is alone on its SIMD, so an LDS read the next MFMA waits on
  // leaves the matrix pipe idle for its whole latency)
  constexpr int SG = 8;  // S k-steps per group
  auto scores = [&](int kb, const float* gs, auto&& group_dma) {
    (void)kb;
    // S^T = G_tile^T Q: two accumulation chains (the 16x16x4 dependent latency is 40 cycles)
    floatx4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
    float ga[2][SG];
    auto ld = [&](float (&a)[SG], int t) {
#pragma unroll
      for (int e = 0; e < SG; ++e) a[e] = gs[(4 * (SG * t + e) + g) * kFBN + lq];
    };
    ld(ga[0], 0);
#pragma unroll
    for (int t = 0; t < NQ / SG; ++t) {
      group_dma(t);  // DMA piece t of the next key blocks
      if (t + 1 < NQ / SG) ld(ga[(t + 1) & 1], t + 1);
      __builtin_amdgcn_sched_barrier(0);  // the reads issue before this group's MFMAs
#pragma unroll
      for (int e = 0; e < SG; e += 2) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[t & 1][e], qv[SG * t + e], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[t & 1][e + 1], qv[SG * t + e + 1], s1, 0, 0, 0);
      }
    }
    return s0 + s1;
  };
  // online softmax over this lane's keys kb * 16 + 4 g + r for query lq: O rescaled to the
  // new running max (lazily), p = exp(S - m)
  auto softmax = [&](int kb, const floatx4& sc) {
    if (RPST_FLDBG & 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = sc[r];
      return;
    }
    const int kbase = kb * kFBN + 4 * g;
    if constexpr (AM >= AM_AEA) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float P = __builtin_amdgcn_exp2f(fmaf(sc[r], kLog2e, -a_mL)) * a_inv;
        float v;
        if constexpr (AM == AM_AEA) {
          // sigmoid(scale (P - c)); exp2 overflows to +inf far below the clamp: weight 0
          const float e = __builtin_amdgcn_exp2f(-rows.scale * kLog2e * (P - a_c));
          v = __builtin_amdgcn_rcpf(1.f + e);
        } else {
          v = __builtin_amdgcn_exp2f(fmaf(fmaxf(P - a_c, 0.f), kLog2e, -a_m2L));
        }
        p[r] = kbase + r < HW ? v : 0.f;  // keys past HW weigh nothing
        if constexpr (AM == AM_AEAR) l_run += p[r];
      }
      return;
    }
    float sv[4], mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sv[r] = kbase + r < HW ? sc[r] : -INFINITY;
      mx = fmaxf(mx, sv[r]);
    }
    const float m_new = fmaxf(m_run, rows4_max(mx));
    // exp(x - m) as v_exp_f32 (base 2) of fma(x, log2 e, -m log2 e): one rounding before
    // the hardware exp instead of expf's range-reduced software sequence; masked keys
    // (-inf) give 0
    const float mL = m_new * kLog2e;
    // (exactly 1 while the max stands: fma(m, log2 e, -m log2 e) is the product's rounding
    // residual, not 0)
    const float alpha = m_run == m_new ? 1.f
                        : (m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(fmaf(m_run, kLog2e, -mL)));
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = __builtin_amdgcn_exp2f(fmaf(sv[r], kLog2e, -mL));
      ps += p[r];
    }
    l_run = fmaf(l_run, alpha, ps);
    m_run = m_new;
    if (AM == AM_SOFTMAX && __builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
      for (int mb = 0; mb < NMB; ++mb) acc[mb] *= alpha;
    }
  };
  // O += H_tile P^T: k-step r = keys 4 g + r, A = H[16 mb + lq][4 g + r]; channel blocks in
  // groups of UG, the H reads of group u + 1 issued before group u's MFMAs
  constexpr int UG = NMB >= 4 ? 4 : NMB;
  auto update = [&](const float* hs) {
    if ((RPST_FLDBG & 8) || AM == AM_STATS) return;
    float4 hb[2][UG];
    auto ld = [&](float4 (&h)[UG], int u) {
#pragma unroll
      for (int e = 0; e < UG; ++e)
        h[e] = *reinterpret_cast<const float4*>(hs + (16 * (UG * u + e) + lq) * kFBN + hsw);
    };
    ld(hb[0], 0);
#pragma unroll
    for (int u = 0; u < NMB / UG; ++u) {
      if (u + 1 < NMB / UG) ld(hb[(u + 1) & 1], u + 1);
      __builtin_amdgcn_sched_barrier(0);  // the reads issue before this group's MFMAs
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int e = 0; e < UG; ++e) {
          const int mb = UG * u + e;
          const float4 h4 = hb[u & 1][e];
          const float hv = r == 0 ? h4.x : (r == 1 ? h4.y : (r == 2 ? h4.z : h4.w));
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv, p[r], acc[mb], 0, 0, 0);
        }
    }
  };
  constexpr bool useH = AM != AM_STATS;
  if constexpr (!PIPE) {
    if (useH) issue_h(0, Hs0);
    auto step = [&](int kb, const float* gs, const float* hs, float* gn, float* hn) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's key tile kb has landed
      __builtin_amdgcn_s_barrier();                     // ... for every wave; the other
      // (the other buffers are free: step kb - 1 is done everywhere)
      const int k1 = kb + 1 < nk ? (kb + 1) * kFBN : -1;
      softmax(kb, scores(kb, gs, [&](int t) { piece(t, k1, gn, useH ? k1 : -1, hn); }));
      update(hs);
    };
    for (int kb = 0; kb < nk; kb += 2) {
      step(kb, Gs0, Hs0, Gs1, Hs1);
      if (kb + 1 < nk) step(kb + 1, Gs1, Hs1, Gs0, Hs0);
    }
  } else {
    // software pipeline over key blocks: iteration kb computes S(kb), then the O update of
    // block kb - 1 (whose P is in registers), then the softmax of kb, so the softmax's
    // shuffle / exp latency sits behind the update's MFMAs. H lags G by one block: H(kb) is
    // loaded in iteration kb into the buffer of H(kb - 2) and consumed in iteration kb + 1.
    auto step = [&](int kb, const float* gs, const float* hprev, float* gn, float* hcur) {
      if (!(RPST_FLDBG & 2)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // G(kb), H(kb - 1) have landed
        __builtin_amdgcn_s_barrier();
      }
      const int kg = kb + 1 < nk ? (kb + 1) * kFBN : -1,
                kh = useH && kb < nk ? kb * kFBN : -1;
      floatx4 sc = {0.f, 0.f, 0.f, 0.f};
      if (kb < nk) sc = scores(kb, gs, [&](int t) { piece(t, kg, gn, kh, hcur); });
      // (the last iteration has no scores and no DMA left: kg, kh < 0)
      if (kb >= 1) update(hprev);
      if (kb < nk) softmax(kb, sc);
    };
    for (int kb = 0; kb <= nk; kb += 2) {
      step(kb, Gs0, Hs1, Gs1, Hs0);
      if (kb + 1 <= nk) step(kb + 1, Gs1, Hs0, Gs0, Hs1);
    }
  }
  // the row sum over the four lane groups holding a query's keys; O / l
  if constexpr (AM != AM_AEA) l_run = rows4_sum(l_run);
  if constexpr (AM == AM_STATS) {
    if (q < HW && g == 0) {
      rows.out_m[(int64_t)b * HW + q] = m_run;
      rows.out_inv[(int64_t)b * HW + q] = 1.f / l_run;
    }
    return;
  }
  if (q < HW) {
    const float inv = AM == AM_AEA ? 1.f : 1.f / l_run;
    float* Ob = O + b * plane + q;
#pragma unroll
    for (int mb = 0; mb < NMB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ob[(int64_t)(16 * mb + 4 * g + r) * HW] = acc[mb][r] * inv;
  }
}

// 8-wave form (two waves per SIMD): waves w and w + 4 own the same 16 queries and split the
// channels, wave w + 4 c in [C/2, C): each computes the partial S^T over its channel half (its Q
// half in registers, C / 8 per lane), the halves are exchanged through LDS (one barrier) and
// summed in the same order by both, so both run the identical online softmax; then each
// accumulates O for its own channel half (C / 8 accumulator registers per lane). Twice the
// waves of sanet_flash_kernel at half the registers: a SIMD's two waves hide each other's LDS
// and softmax latency. RPST_SANET_FLASH=2 selects it.
template <int C>
__global__ __launch_bounds__(512, 1) void sanet_flash8_kernel(const float* __restrict__ F,
                                                              const float* __restrict__ G,
                                                              const float* __restrict__ H,
                                                              float* __restrict__ O, int HW,
                                                              int qblocks) {
  constexpr int CH = C / 2;            // channels per wave
  constexpr int NQ = CH / 4;           // Q registers per lane
  constexpr int NMB = CH / 16;         // O accumulators
  constexpr int TILE = C * kFBN;
  constexpr int PPW = TILE / 256 / 8;  // DMA pieces per wave per tile
  static_assert(PPW >= 1 && TILE % 2048 == 0, "C in {128, 256, 512}");
  __shared__ __attribute__((aligned(16))) float Gs0[TILE];
  __shared__ __attribute__((aligned(16))) float Gs1[TILE];
  __shared__ __attribute__((aligned(16))) float Hs0[TILE];
  __shared__ __attribute__((aligned(16))) float Hs1[TILE];
  __shared__ __attribute__((aligned(16))) float xs[8 * 64 * 4];  // partial S^T exchange

  const int bid = attn_xcd_swizzle(blockIdx.x, (int)gridDim.x);
  const int b = bid / qblocks, qb = bid - b * qblocks;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qw = wave & 3, half = wave >> 2;
  const int g = lane >> 4, lq = lane & 15;
  const int q = qb * kFBM + qw * 16 + lq;
  const int c0 = half * CH;
  const int64_t plane = (int64_t)C * HW;
  const float* Fb = F + b * plane;
  const unsigned bytes = (unsigned)(plane * 4);
  const auto rG = __builtin_amdgcn_make_buffer_rsrc((void*)(G + b * plane), (short)0, (int)bytes, 0x00020000);
  const auto rH = __builtin_amdgcn_make_buffer_rsrc((void*)(H + b * plane), (short)0, (int)bytes, 0x00020000);
  const int prow = lane >> 2, pseg = lane & 3;
  const unsigned voffG = (unsigned)(prow * HW + 4 * pseg) * 4u;
  const unsigned voffH = (unsigned)(prow * HW + 4 * (pseg ^ ((lane >> 4) & 3))) * 4u;
  auto issue = [&](int k0, float* gs, float* hs) {
#pragma unroll
    for (int jj = 0; jj < PPW; ++jj) {
      const int j = wave * PPW + jj;
      const unsigned so = (unsigned)(16 * j * HW + k0) * 4u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rG, (attn_lds_ptr_t)(gs + 256 * j), 16, (int)(voffG + so), 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rH, (attn_lds_ptr_t)(hs + 256 * j), 16, (int)(voffH + so), 0, 0, 0);
    }
  };
  const int nk = (HW + kFBN - 1) / kFBN;
  issue(0, Gs0, Hs0);

  float qv[NQ];
#pragma unroll
  for (int s = 0; s < NQ; ++s) qv[s] = q < HW ? Fb[(int64_t)(c0 + 4 * s + g) * HW + q] : 0.f;
  floatx4 acc[NMB];
#pragma unroll
  for (int mb = 0; mb < NMB; ++mb) acc[mb] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  const int hsw = 4 * (g ^ ((lq >> 2) & 3));
  float* xmine = xs + (wave * 64 + lane) * 4;
  const float* xpart = xs + ((wave ^ 4) * 64 + lane) * 4;

  auto step = [&](int kb, const float* gs, const float* hs, float* gn, float* hn) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kb + 1 < nk) issue((kb + 1) * kFBN, gn, hn);
    floatx4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NQ; s += 2) {
      const float a0 = gs[(c0 + 4 * s + g) * kFBN + lq];
      const float a1 = gs[(c0 + 4 * s + 4 + g) * kFBN + lq];
      s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, qv[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, qv[s + 1], s1, 0, 0, 0);
    }
    const floatx4 mine = s0 + s1;
    *reinterpret_cast<floatx4*>(xmine) = mine;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const floatx4 other = *reinterpret_cast<const floatx4*>(xpart);
    // the same sum in both waves: channel half 0's partial first
    const floatx4 sf = half == 0 ? mine + other : other + mine;
    const int kbase = kb * kFBN + 4 * g;
    float sv[4], mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sv[r] = kbase + r < HW ? sf[r] : -INFINITY;
      mx = fmaxf(mx, sv[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = m_run == -INFINITY ? 0.f : expf(m_run - m_new);
    float p[4], ps = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p[r] = expf(sv[r] - m_new);
      ps += p[r];
    }
    l_run = fmaf(l_run, alpha, ps);
    m_run = m_new;
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
      for (int mb = 0; mb < NMB; ++mb) acc[mb] *= alpha;
    }
#pragma unroll
    for (int mb = 0; mb < NMB; ++mb) {
      const float4 h4 = *reinterpret_cast<const float4*>(hs + (c0 + 16 * mb + lq) * kFBN + hsw);
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(h4.x, p[0], acc[mb], 0, 0, 0);
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(h4.y, p[1], acc[mb], 0, 0, 0);
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(h4.z, p[2], acc[mb], 0, 0, 0);
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(h4.w, p[3], acc[mb], 0, 0, 0);
    }
  };
  for (int kb = 0; kb < nk; kb += 2) {
    step(kb, Gs0, Hs0, Gs1, Hs1);
    if (kb + 1 < nk) step(kb + 1, Gs1, Hs1, Gs0, Hs0);
  }
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  if (q < HW) {
    const float inv = 1.f / l_run;
    float* Ob = O + b * plane + q;
#pragma unroll
    for (int mb = 0; mb < NMB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ob[(int64_t)(c0 + 16 * mb + 4 * g + r) * HW] = acc[mb][r] * inv;
  }
}

// flash path (RPST_SANET_FLASH=0: the two-GEMM path with S in the workspace, A/B)
static int sanet_flash_mode() {
  static const int on = [] {
    const char* e = std::getenv("RPST_SANET_FLASH");
    return (e && *e) ? std::atoi(e) : 1;
  }();
  return on;
}
bool sanet_flash_ok(int C, int HW) {
  return sanet_flash_mode() != 0 && (C == 64 || C == 128 || C == 256 || C == 512) &&
         HW % 4 == 0 && (int64_t)C * HW * 4 < (1LL << 31);
}

int sanet_flash(const float* F, const float* G, const float* H, float* O, int B, int C,
                       int HW, hipStream_t st) {
  const int qblocks = (HW + kFBM - 1) / kFBM;
  const int64_t nb = (int64_t)B * qblocks;
  RPST_REQUIRE(nb <= 0x7fffffffLL, "sanet_attention: grid too large");
  if (sanet_flash_mode() == 2 && C >= 128) {
    switch (C) {
      case 128: sanet_flash8_kernel<128><<<(unsigned)nb, 512, 0, st>>>(F, G, H, O, HW, qblocks); break;
      case 256: sanet_flash8_kernel<256><<<(unsigned)nb, 512, 0, st>>>(F, G, H, O, HW, qblocks); break;
      default: sanet_flash8_kernel<512><<<(unsigned)nb, 512, 0, st>>>(F, G, H, O, HW, qblocks); break;
    }
    return launch_status("sanet_flash8_kernel");
  }
#define RPST_FLASH_GO(P)                                                                      \
  switch (C) {                                                                                \
    case 64: sanet_flash_kernel<64, P><<<(unsigned)nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, {}); break;   \
    case 128: sanet_flash_kernel<128, P><<<(unsigned)nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, {}); break; \
    case 256: sanet_flash_kernel<256, P><<<(unsigned)nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, {}); break; \
    default: sanet_flash_kernel<512, P><<<(unsigned)nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, {}); break;  \
  }
  if (sanet_flash_mode() == 3) RPST_FLASH_GO(false)
  else RPST_FLASH_GO(true)
#undef RPST_FLASH_GO
  return launch_status("sanet_flash_kernel");
}

// AdaptiveSANet attention without S (sanet.py:100-124): pass 1 writes each query's softmax
// statistics (rm, rinv: B x HW each), pass 2 recomputes S per key block and accumulates
// O = H Q^T with the clamp applied in registers. mode 0 = AEAModule, 1 = AEALReluModule.
template <int AM>
static void adaptive_flash_launch(int C, unsigned nb, hipStream_t st, const float* F,
                                  const float* G, const float* H, float* O, int HW, int qblocks,
                                  const AttnRows& rows) {
  switch (C) {
    case 64: sanet_flash_kernel<64, true, AM><<<nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, rows); break;
    case 128: sanet_flash_kernel<128, true, AM><<<nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, rows); break;
    case 256: sanet_flash_kernel<256, true, AM><<<nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, rows); break;
    default: sanet_flash_kernel<512, true, AM><<<nb, 256, 0, st>>>(F, G, H, O, HW, qblocks, rows); break;
  }
}

int adaptive_flash_stats(const float* F, const float* G, int B, int C, int HW, float* rm,
                         float* rinv, hipStream_t st) {
  const int qblocks = (HW + kFBM - 1) / kFBM;
  const int64_t nb = (int64_t)B * qblocks;
  RPST_REQUIRE(nb <= 0x7fffffffLL, "adaptive_attention: grid too large");
  AttnRows rows{};
  rows.out_m = rm;
  rows.out_inv = rinv;
  adaptive_flash_launch<AM_STATS>(C, (unsigned)nb, st, F, G, nullptr, nullptr, HW, qblocks, rows);
  return launch_status("sanet_flash_kernel(stats)");
}

int adaptive_flash_apply(const float* F, const float* G, const float* H, float* O, int B, int C,
                         int HW, const float* rm, const float* rinv, const float* clamp, int mode,
                         float scale, hipStream_t st) {
  const int qblocks = (HW + kFBM - 1) / kFBM;
  const int64_t nb = (int64_t)B * qblocks;
  RPST_REQUIRE(nb <= 0x7fffffffLL, "adaptive_attention: grid too large");
  const AttnRows rows{rm, rinv, clamp, scale, nullptr, nullptr};
  if (mode == 0)
    adaptive_flash_launch<AM_AEA>(C, (unsigned)nb, st, F, G, H, O, HW, qblocks, rows);
  else
    adaptive_flash_launch<AM_AEAR>(C, (unsigned)nb, st, F, G, H, O, HW, qblocks, rows);
  return launch_status("sanet_flash_kernel(adaptive)");
}

}  // namespace rpst
