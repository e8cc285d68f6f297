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

}  // namespace rpst

using namespace rpst;

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
