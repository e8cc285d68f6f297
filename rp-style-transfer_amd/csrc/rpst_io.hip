// Host I/O around the path: the pixel conversions of the reference's
// test driver, on the GPU so only uint8 pixels cross PCIe (3 B instead of 12 B per pixel).
//
//   load:  transforms.ToTensor (test.py:49-54 -> torchvision): uint8 HWC -> fp32 CHW / 255
//   store: torchvision.utils.save_image (test.py:145-149): make_grid(padding=2, pad_value=0)
//          then x.mul(255).add_(0.5).clamp_(0, 255) -> uint8 HWC
//
// Both are byte/elementwise and bound by HBM (and by PCIe around them). Arithmetic follows
// the reference op by op in fp32 with contraction off (mul, then add, then clamp, then the
// truncating cast), so the pixels are bit-identical to the torchvision path.
#include "rpst_common.h"

namespace rpst {

// One thread per pixel: 3 bytes in (HWC), 3 floats out (one per channel plane).
__global__ __launch_bounds__(256) void u8hwc_to_f32_kernel(const uint8_t* __restrict__ in,
                                                           float* __restrict__ out, int64_t N,
                                                           int64_t HW) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N * HW) return;
  const int64_t n = i / HW, p = i - n * HW;
  const uint8_t* px = in + i * 3;
  float* o = out + n * 3 * HW + p;
  o[0] = (float)px[0] / 255.f;
  o[HW] = (float)px[1] / 255.f;
  o[2 * HW] = (float)px[2] / 255.f;
}

// One thread per pixel of the tile: image n of `in` (3,H,W) goes to canvas n at (y0, x0).
__global__ __launch_bounds__(256) void f32_to_u8_tile_kernel(const float* __restrict__ in,
                                                             uint8_t* __restrict__ canvas,
                                                             int64_t N, int H, int W, int CH,
                                                             int CW, int y0, int x0) {
#pragma clang fp contract(off)
  const int64_t HW = (int64_t)H * W;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N * HW) return;
  const int64_t n = i / HW, p = i - n * HW;
  const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
  const float* src = in + n * 3 * HW + p;
  uint8_t* dst = canvas + ((n * CH + y0 + y) * (int64_t)CW + x0 + x) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float v = src[c * HW] * 255.f;
    v = v + 0.5f;
    v = fminf(fmaxf(v, 0.f), 255.f);  // clamp_ (NaN -> 0 like the uint8 cast of torch)
    dst[c] = (uint8_t)(v == v ? v : 0.f);
  }
}

// PNG "Up" filter (PNG spec 9.2, filter type 2) of N images of H rows x rowbytes bytes:
// out row y = [2, (row y - row y-1) mod 256 ...] (row -1 = 0), so the host only runs zlib over
// the filtered scanlines (rpst.imageio.write_png). One thread per 4 output bytes of a row.
__global__ __launch_bounds__(256) void png_filter_up_kernel(const uint8_t* __restrict__ in,
                                                            uint8_t* __restrict__ out, int64_t rows,
                                                            int H, int rowbytes) {
  const int ob = rowbytes + 1;
  const int per_row = (ob + 3) >> 2;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * per_row) return;
  const int64_t r = t / per_row;
  const int j0 = (int)(t - r * per_row) * 4;
  const bool first = (r % H) == 0;
  const uint8_t* cur = in + r * rowbytes;
  const uint8_t* prev = cur - rowbytes;
  uint8_t* o = out + r * ob;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int j = j0 + e;
    if (j >= ob) break;
    o[j] = j == 0 ? (uint8_t)2 : (uint8_t)(cur[j - 1] - (first ? 0 : prev[j - 1]));
  }
}

// PNG reconstruction (PNG spec 9.2-9.4: filter types 0 None, 1 Sub, 2 Up, 3 Average, 4 Paeth;
// 8-bit RGB, 3 bytes per pixel) of N images of H scanlines [type, 3 W bytes] into H x 3 W
// bytes: the host only inflates (rpst.imageio.read_png_filtered). Each byte depends on its
// left, upper and upper-left neighbours, so a row is a serial chain and the rows follow one
// another. One wave per image works a band of R <= 64 scanlines at a time as a diagonal
// wavefront: lane l reconstructs row r0 + l one pixel behind lane l - 1, taking the pixel
// above and above-left from lane l - 1's last two outputs by a lane shuffle (lane 0: from the
// previous band's last row, kept in LDS as it is produced). The band's filtered rows are
// staged in LDS by dword loads, reconstructed in place and written out by dword stores.
// HBM / latency bound: 2 (1 + 3 W) H bytes per image; ~W + R serial steps per band.
__device__ __forceinline__ uint32_t png_pred(uint32_t a, uint32_t b, uint32_t c, int ft) {
  switch (ft) {
    case 1: return a;
    case 2: return b;
    case 3: return (a + b) >> 1;
    case 4: {
      const int p = (int)a + (int)b - (int)c;
      const int pa = abs(p - (int)a), pb = abs(p - (int)b), pc = abs(p - (int)c);
      return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
    }
    default: return 0u;
  }
}

__global__ __launch_bounds__(64) void png_unfilter_kernel(const uint8_t* __restrict__ in,
                                                          uint8_t* __restrict__ out, int H,
                                                          int W, int R) {
  extern __shared__ __attribute__((aligned(16))) uint8_t png_lds[];
  const int rb = 1 + 3 * W, ob = 3 * W;
  uint8_t* up_row = png_lds;              // reconstructed row above the band (3 W bytes)
  uint8_t* band = png_lds + ((ob + 15) & ~15);  // staged rows, from the dword below the band
  const int n = blockIdx.x, lane = threadIdx.x;
  const uint8_t* img = in + (int64_t)n * H * rb;
  uint8_t* oimg = out + (int64_t)n * H * ob;
  for (int r0 = 0; r0 < H; r0 += R) {
    const int rows = min(R, H - r0);
    // stage rows r0 .. r0 + rows - 1 (contiguous in `in`) from the aligned dword at or below
    const uint8_t* src = img + (int64_t)r0 * rb;
    const uintptr_t a0 = (uintptr_t)src & ~(uintptr_t)3;
    const int shift = (int)((uintptr_t)src - a0), len = shift + rows * rb;
    const int ndw = len >> 2;  // whole dwords (the bytes before `src` belong to the buffer)
    for (int i = lane; i < ndw; i += 64)
      reinterpret_cast<uint32_t*>(band)[i] = reinterpret_cast<const uint32_t*>(a0)[i];
    for (int i = (ndw << 2) + lane; i < len; i += 64) band[i] = *(const uint8_t*)(a0 + i);
    __syncthreads();
    // wavefront: lane l = row r0 + l; L / LL = its last two reconstructed pixels (RGB packed)
    const bool rowok = lane < rows;
    uint8_t* row = band + shift + lane * rb;
    const int ft = rowok ? row[0] : 0;
    uint32_t L = 0u, LL = 0u;
    for (int t = 0; t < W + rows - 1; ++t) {
      const int x = t - lane;
      const bool act = rowok && x >= 0 && x < W;
      uint32_t upv = __shfl_up(L, 1, 64), ulv = __shfl_up(LL, 1, 64);
      if (lane == 0) {
        const bool have = r0 > 0 && x >= 0 && x < W;
        upv = have ? (uint32_t)up_row[3 * x] | ((uint32_t)up_row[3 * x + 1] << 8) |
                         ((uint32_t)up_row[3 * x + 2] << 16)
                   : 0u;
        ulv = have && x > 0 ? (uint32_t)up_row[3 * x - 3] | ((uint32_t)up_row[3 * x - 2] << 8) |
                                  ((uint32_t)up_row[3 * x - 1] << 16)
                            : 0u;
      }
      if (x == 0) ulv = 0u;
      uint32_t rec = 0u;
      if (act) {
        const uint32_t lv = x > 0 ? L : 0u;
        uint8_t* px = row + 1 + 3 * x;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const uint32_t a = (lv >> (8 * c)) & 255u, b = (upv >> (8 * c)) & 255u,
                         cc = (ulv >> (8 * c)) & 255u;
          const uint32_t v = (px[c] + png_pred(a, b, cc, ft)) & 255u;
          px[c] = (uint8_t)v;
          rec |= v << (8 * c);
        }
        // (reads of up_row above come before this write in every lane: lane 0 has consumed
        // positions x and x - 1 of the old row by the time the band's last lane writes x)
        if (lane == rows - 1) {
          up_row[3 * x] = (uint8_t)rec;
          up_row[3 * x + 1] = (uint8_t)(rec >> 8);
          up_row[3 * x + 2] = (uint8_t)(rec >> 16);
        }
        LL = L;
        L = rec;
      }
    }
    __syncthreads();
    // out rows r0 .. r0 + rows - 1: 3 W bytes each, the filter byte skipped
    uint8_t* dst = oimg + (int64_t)r0 * ob;
    const int total = rows * ob;
    if ((((uintptr_t)dst) & 3) == 0 && (ob & 3) == 0) {
      for (int i = 4 * lane; i < total; i += 256) {
        const int r = i / ob, j = i - r * ob;
        const uint8_t* sp = band + shift + r * rb + 1 + j;
        reinterpret_cast<uint32_t*>(dst)[i >> 2] =
            (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16) | ((uint32_t)sp[3] << 24);
      }
    } else {
      for (int i = lane; i < total; i += 64) {
        const int r = i / ob, j = i - r * ob;
        dst[i] = band[shift + r * rb + 1 + j];
      }
    }
    __syncthreads();  // the next band's staging overwrites `band`
  }
}

// rows per band: as many of the 64 lanes as the LDS holds (up row + staged rows + 4 B slack)
static int png_band_rows(int W) {
  const int rb = 1 + 3 * W, ob = 3 * W;
  const int avail = 150 * 1024 - ((ob + 15) & ~15) - 4;
  return avail / rb < 64 ? avail / rb : 64;
}
static size_t png_lds_bytes(int W, int R) {
  return (size_t)((3 * W + 15) & ~15) + (size_t)R * (1 + 3 * W) + 4;
}

}  // namespace rpst

using namespace rpst;

extern "C" int rpst_png_unfilter(const uint8_t* in, uint8_t* out, int N, int H, int W,
                                 rpst_stream_t stream) {
  RPST_REQUIRE(in && out, "png_unfilter: null pointer");
  RPST_REQUIRE(((uintptr_t)in & 3) == 0, "png_unfilter: input not 4-byte aligned");
  RPST_REQUIRE(N > 0 && H > 0 && W > 0, "png_unfilter: bad shape");
  const int R = png_band_rows(W);
  RPST_REQUIRE(R >= 1, "png_unfilter: row of %d pixels does not fit the LDS", W);
  const size_t lds = png_lds_bytes(W, R);
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)png_unfilter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024 + 64);
  RPST_REQUIRE(attr == hipSuccess, "png_unfilter: dynamic LDS attribute: %s", hipGetErrorString(attr));
  png_unfilter_kernel<<<(unsigned)N, 64, lds, as_stream(stream)>>>(in, out, H, W, R);
  return launch_status("png_unfilter_kernel");
}

extern "C" int rpst_png_filter_up(const uint8_t* in, uint8_t* out, int N, int H, int rowbytes,
                                  rpst_stream_t stream) {
  RPST_REQUIRE(in && out, "png_filter_up: null pointer");
  RPST_REQUIRE(N > 0 && H > 0 && rowbytes > 0, "png_filter_up: bad shape");
  const int64_t rows = (int64_t)N * H, threads = rows * ((rowbytes + 1 + 3) / 4);
  RPST_REQUIRE((threads + 255) / 256 <= 0x7fffffffLL, "png_filter_up: too large");
  png_filter_up_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, as_stream(stream)>>>(
      in, out, rows, H, rowbytes);
  return launch_status("png_filter_up_kernel");
}

extern "C" int rpst_u8hwc_to_f32nchw(const uint8_t* in, float* out, int N, int H, int W,
                                     rpst_stream_t stream) {
  RPST_REQUIRE(in && out, "u8hwc_to_f32nchw: null pointer");
  RPST_REQUIRE(N > 0 && H > 0 && W > 0, "u8hwc_to_f32nchw: bad shape");
  const int64_t total = (int64_t)N * H * W;
  RPST_REQUIRE((total + 255) / 256 <= 0x7fffffffLL, "u8hwc_to_f32nchw: too large");
  u8hwc_to_f32_kernel<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(
      in, out, N, (int64_t)H * W);
  return launch_status("u8hwc_to_f32_kernel");
}

extern "C" int rpst_f32nchw_to_u8_tile(const float* in, uint8_t* canvas, int N, int H, int W,
                                       int canvas_h, int canvas_w, int y0, int x0,
                                       rpst_stream_t stream) {
  RPST_REQUIRE(in && canvas, "f32nchw_to_u8_tile: null pointer");
  RPST_REQUIRE(N > 0 && H > 0 && W > 0, "f32nchw_to_u8_tile: bad shape");
  RPST_REQUIRE(y0 >= 0 && x0 >= 0 && y0 + H <= canvas_h && x0 + W <= canvas_w,
               "f32nchw_to_u8_tile: tile (%d,%d)+(%d,%d) outside canvas %dx%d", y0, x0, H, W,
               canvas_h, canvas_w);
  const int64_t total = (int64_t)N * H * W;
  RPST_REQUIRE((total + 255) / 256 <= 0x7fffffffLL, "f32nchw_to_u8_tile: too large");
  f32_to_u8_tile_kernel<<<(unsigned)((total + 255) / 256), 256, 0, as_stream(stream)>>>(
      in, canvas, N, H, W, canvas_h, canvas_w, y0, x0);
  return launch_status("f32_to_u8_tile_kernel");
}
