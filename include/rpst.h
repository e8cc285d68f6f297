/*
 * rpst.h — C ABI of the MI355X (gfx950) style-transfer forward path.
 *
 * Drop-in boundary: the reference (LuletterSoul/RP-Style-Transfer) has no FFI; its
 * boundary is the Python API of the `network` package (network/__init__.py:1-6).
 * Each entry point below replaces the ATen work behind one reference function, cited
 * as path:line relative to the reference root. The Python mirror in
 * rp-style-transfer_amd/network/ binds these symbols with ctypes.
 *
 * Conventions
 *  - All tensor pointers are DEVICE pointers to contiguous row-major (NCHW) data.
 *  - The library never allocates: ops that need scratch take (workspace, bytes) and
 *    expose a *_workspace_size() query; the caller allocates (e.g. torch caching
 *    allocator).
 *  - Every call is ordered on `stream` (a hipStream_t passed as void*; NULL = default
 *    stream) and never synchronises the device.
 *  - Return value: RPST_OK (0) or a negative RPST_E* code; rpst_last_error() returns a
 *    thread-local message describing the last failure.
 *  - fp32 in / fp32 out unless the name says f64. Results are deterministic (no float
 *    atomics; fixed-order reductions).
 */
#ifndef RPST_H_
#define RPST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rpst_stream_t;

#define RPST_OK 0
#define RPST_EINVAL (-1)  /* bad argument / unsupported shape            */
#define RPST_EHIP (-2)    /* HIP launch or runtime error                  */
#define RPST_EWORKSPACE (-3) /* workspace smaller than *_workspace_size() */

/* conv2d padding mode */
#define RPST_PAD_ZERO 0    /* nn.Conv2d(padding=1)            base.py:366-395            */
#define RPST_PAD_REFLECT 1 /* nn.ReflectionPad2d((1,1,1,1))   base.py:26-54, base.py:59-110 */
/* conv2d input operator applied on the fly while loading the input tile */
#define RPST_IN_NONE 0
#define RPST_IN_MAXPOOL2 1 /* nn.MaxPool2d((2,2),(2,2),(0,0),ceil_mode=True) base.py:65,72,85,98 */
#define RPST_IN_UPSAMPLE2 2 /* nn.Upsample(scale_factor=2, mode='nearest') base.py:29,42,49     */
#define RPST_IN_ADD_UPSAMPLE2 3 /* x + Upsample2(y)   sanet.py:149 (Transform merge input)   */
#define RPST_IN_ADAIN 4 /* ((x-mean_c)/std_c)*std_s+mean_s per (n,ci): AdaIN base.py:416-418 fused
                           into the consumer conv; aux = [mean_c|mean_s|std_c|std_s], N*Cin each */
#define RPST_IN_ADD_ADAIN 5 /* x + AdaIN(c): the skip fusion of MultiScaleAdaINRPNet.decode,
                           adain_rp.py:301 (rp_decoder[i+1](stylized + AdaIN(c_i, s_i)))  */

/* conv2d epilogue activation (the `relu` argument) */
#define RPST_ACT_NONE 0
#define RPST_ACT_RELU 1  /* nn.ReLU                                     */
#define RPST_ACT_LRELU 2 /* nn.LeakyReLU(0.2): Conv2dBlock base.py:147 */

/* Library version (major*10000 + minor*100 + patch). */
int rpst_version(void);
/* Message of the last failing call on this host thread ("" if none). */
const char* rpst_last_error(void);

/* ---- a1: calc_mean_std(feat, eps)  network/base.py:399-407 ----------------------
 * mean[n,c] = mean over HW; std[n,c] = sqrt(var_unbiased + eps) (eps on the variance).
 * feat (N,C,HW) -> mean, std (N,C). HW == 1 yields NaN std like torch.var. */
int rpst_calc_mean_std(const float* feat, float* mean, float* std_out, int N, int C,
                       int64_t HW, float eps, rpst_stream_t stream);

/* ---- a2: adaptive_instance_normalization(c, s)  network/base.py:410-418 ----------
 * out = (c - mean_c) / std_c * std_s + mean_s, statistics per (n,c) as in a1.
 * content/style/out (N,C,HW). Workspace: rpst_adain_workspace_size(N, C). */
size_t rpst_adain_workspace_size(int N, int C);
int rpst_adain(const float* content, const float* style, float* out, int N, int C,
               int64_t HW, float eps, void* workspace, size_t workspace_bytes,
               rpst_stream_t stream);

/* ---- a10: mean_variance_norm(feat)  network/sanet.py:20-24 -----------------------
 * out = (x - mean) / std with a1 statistics. Workspace: rpst_adain_workspace_size(N,C). */
int rpst_mean_variance_norm(const float* feat, float* out, int N, int C, int64_t HW,
                            float eps, void* workspace, size_t workspace_bytes,
                            rpst_stream_t stream);

/* ---- a3/a5/a6/a12: Conv2d (3x3 or 1x1, stride 1) + bias [+ReLU] [+residual] -------
 * nn.Conv2d(k=3, padding=1) + ReLU         base.py:363-396 (RP encoder / decoder)
 * ReflectionPad2d(1) + Conv2d(k=3) [+ReLU] base.py:25-111, sanet.py:146-147,162-192
 * Conv2d(k=1)                              base.py:58, sanet.py:76-80
 * Weights are first repacked once into the kernel's K-major layout:
 *   rpst_conv2d_pack(weight (Cout,Cin,k,k), packed) with
 *   packed bytes = rpst_conv2d_packed_size(Cout, Cin, ksize).
 * in_op is applied to the input while it is loaded (pool / upsample / add), so
 *   RPST_IN_MAXPOOL2:     input (N,Cin,Hs,Ws), conv runs at H=ceil(Hs/2), W=ceil(Ws/2)
 *   RPST_IN_UPSAMPLE2:    input (N,Cin,Hs,Ws), conv runs at H=2Hs, W=2Ws
 *   RPST_IN_ADD_UPSAMPLE2: input (N,Cin,H,W) + aux (N,Cin,H/2,W/2) upsampled
 *   RPST_IN_ADAIN:        input (N,Cin,H,W) normalised on load with aux statistics
 *   RPST_IN_NONE:         input (N,Cin,H,W)
 * (Hs, Ws) are the dims of `input`. out (N,Cout,H,W):
 *   out = act(conv(in_op(input)) + bias) [+ residual]   (residual (N,Cout,H,W) or NULL),
 *   act = `relu`: RPST_ACT_NONE / RPST_ACT_RELU / RPST_ACT_LRELU
 * ksize 1 ignores pad_mode. Reflect padding needs H,W >= 2. */
size_t rpst_conv2d_packed_size(int Cout, int Cin, int ksize);
int rpst_conv2d_pack(const float* weight, float* packed, int Cout, int Cin, int ksize,
                     rpst_stream_t stream);
int rpst_conv2d(const float* input, const float* aux, const float* packed_weight,
                const float* bias, const float* residual, float* out, int N, int Cin,
                int Hs, int Ws, int Cout, int ksize, int pad_mode, int in_op, int relu,
                rpst_stream_t stream);

/* rpst_conv2d (in_op RPST_IN_NONE, no residual) over the batch [input; input2]: images
 * 0..n1-1 are input's, n1..N-1 are input2's (N - n1 images), read in place -- an encoder's
 * first conv over content and style without materialising torch.cat (adain_rp.py:94-95,
 * wct_rp.py:141-144, sanet.py:240-242 encode both in one pass). 0 < n1 <= N. */
int rpst_conv2d_pair(const float* input, const float* input2, int n1, const float* packed_weight,
                     const float* bias, float* out, int N, int Cin, int Hs, int Ws, int Cout,
                     int ksize, int pad_mode, int relu, rpst_stream_t stream);

/* Conv whose output only feeds a 2x2 max pool (VGG relu1_2 / relu2_2 / relu3_4 -> MaxPool2d
 * (2, 2, ceil_mode=True) -> next conv, network/base.py vgg, sanet.py:195-199 enc_2..enc_5):
 * out (N, Cout, (H+1)/2, (W+1)/2) = max_pool2d(act(conv(in_op(input)) + bias)), the pool
 * taken on the finished output tiles in the F(4x4) epilogue, so the full-resolution map is
 * never written. Bit-identical to rpst_conv2d followed by rpst_maxpool2x2_ceil. Only for
 * layers whose rpst_conv2d_algorithm is RPST_CONV_WINOGRAD4 (RPST_EINVAL otherwise: run
 * the two calls). */
int rpst_conv2d_pool(const float* input, const float* aux, const float* packed_weight,
                     const float* bias, float* out, int N, int Cin, int Hs, int Ws, int Cout,
                     int ksize, int pad_mode, int in_op, int relu, rpst_stream_t stream);

/* Conv (in_op NONE, no activation) whose output is zeroed where mask <= 0 (mask has the
 * output's shape): the input gradient of a conv whose input is a ReLU output y, dgrad and
 * threshold_backward(., y) in one pass (torch.autograd's ConvolutionBackward + ReluBackward
 * under total_loss.backward(), train.py:186-189). Bit-identical to rpst_conv2d followed by
 * rpst_relu_backward; the F(4x4) path thresholds in a second pass. */
int rpst_conv2d_masked(const float* input, const float* packed_weight, const float* bias,
                       const float* mask, float* out, int N, int Cin, int Hs, int Ws, int Cout,
                       int ksize, int pad_mode, rpst_stream_t stream);

/* Same conv with a caller-provided workspace (rpst_conv2d_workspace_size bytes, 0 when the
 * layer needs none). With RPST_IN_ADAIN on the F(4x4) path the workspace holds per-image
 * weights with the AdaIN scale std_s/std_c folded in along Cin and a per-(n, co) bias by
 * border class carrying mean_s - mean_c*std_s/std_c, so the conv streams the raw feature
 * (conv(pad0(s*x + b)) = conv_{W*s}(pad0(x)) + sum over in-image taps of W*b). Same result
 * as rpst_conv2d within fp32 rounding; rpst_conv2d applies the affine in its tile loader. */
size_t rpst_conv2d_workspace_size(int N, int Cin, int Hs, int Ws, int Cout, int ksize,
                                  int in_op);
int rpst_conv2d_ws(const float* input, const float* aux, const float* packed_weight,
                   const float* bias, const float* residual, float* out, int N, int Cin,
                   int Hs, int Ws, int Cout, int ksize, int pad_mode, int in_op, int relu,
                   void* workspace, size_t workspace_bytes, rpst_stream_t stream);

/* Same conv, additionally returning calc_mean_std (base.py:399-407) of its OUTPUT per
 * (n, co): the statistics are reduced in the conv epilogue from registers and merged in
 * fp64, so an AdaIN consumer never re-reads the feature. mean/std_out: N*Cout floats.
 * Workspace: rpst_conv2d_stats_workspace_size(N, Cin, Hs, Ws, Cout, ksize, in_op). */
size_t rpst_conv2d_stats_workspace_size(int N, int Cin, int Hs, int Ws, int Cout, int ksize,
                                        int in_op);
int rpst_conv2d_stats(const float* input, const float* aux, const float* packed_weight,
                      const float* bias, const float* residual, float* out, int N, int Cin,
                      int Hs, int Ws, int Cout, int ksize, int pad_mode, int in_op, int relu,
                      float* mean, float* std_out, float eps, void* workspace,
                      size_t workspace_bytes, rpst_stream_t stream);
/* Same, writing `out` for images n < store_n only (1 <= store_n <= N); the statistics cover
 * all N images. For a batch whose tail images are needed only through their statistics
 * (AdaINRPNet.test, adain_rp.py:94-101: the style half of the encoder output feeds
 * calc_mean_std alone). Images >= store_n of `out` are left unspecified. Same workspace. */
int rpst_conv2d_stats_store(const float* input, const float* aux, const float* packed_weight,
                            const float* bias, const float* residual, float* out, int N,
                            int Cin, int Hs, int Ws, int Cout, int ksize, int pad_mode,
                            int in_op, int relu, float* mean, float* std_out, float eps,
                            int store_n, void* workspace, size_t workspace_bytes,
                            rpst_stream_t stream);

/* MultiScaleAdaINRPNet skip fusion (adain_rp.py:301): out = act(conv(pad(x + AdaIN(c))) +
 * bias), x = `stylized` and c = `content` both (N,Cin,H,W), AdaIN with the calc_mean_std
 * statistics `params` = [mean_c | mean_s | std_c | std_s] (4*N*Cin floats, as
 * RPST_IN_ADAIN). The sum is formed while the conv stages its input tile. */
int rpst_conv2d_skip_adain(const float* stylized, const float* content, const float* params,
                           const float* packed_weight, const float* bias, float* out, int N,
                           int Cin, int H, int W, int Cout, int ksize, int pad_mode, int relu,
                           rpst_stream_t stream);

/* Launch geometry (total threads) rpst_conv2d would use for this shape — host-only; lets
 * profilers match rocprofv3 per-dispatch records (Grid_Size) to a layer. */
int64_t rpst_conv2d_grid_threads(int N, int Cin, int Hs, int Ws, int Cout, int ksize,
                                 int in_op);

/* Algorithm rpst_conv2d uses for this layer — host-only: RPST_CONV_NARROW (VALU kernel for
 * 3x3 layers with loader NONE and Cout <= 4, Cin <= 16 or Cout <= 16, Cin <= 4: the RP
 * stacks' 3->16 / 16->3 convs; batches above 65535 images and the statistics entry point
 * take the direct path instead), RPST_CONV_DIRECT (implicit GEMM: every 1x1 layer and the
 * other 3x3 layers with < 16 input channels), RPST_CONV_WINOGRAD4 (F(4x4,3x3) in fp32: 3x3
 * layers with >= 16 input channels whose loader operator is NONE / ADAIN / UPSAMPLE2) or
 * RPST_CONV_WINOGRAD (F(2x2,3x3) in fp32: the other 3x3 layers with >= 16 input and >= 32
 * output channels). The environment variable RPST_CONV_ALGO=direct|winograd|winograd4
 * overrides ("direct" keeps the narrow kernel for narrow shapes; RPST_CONV_NARROW=0 turns
 * it off). */
#define RPST_CONV_DIRECT 0
#define RPST_CONV_WINOGRAD 1
#define RPST_CONV_WINOGRAD4 2
#define RPST_CONV_NARROW 3
int rpst_conv2d_algorithm(int Cout, int Cin, int Hs, int Ws, int ksize, int in_op);

/* Precise mode for the CALLING THREAD (host-only): while on, the default choice never picks
 * F(4x4,3x3) (its fp32 rounding, ~1e-6 per conv, compounds through the ~30 convolutions of
 * a training step's backward chain); F(2x2) runs instead. Returns the previous setting.
 * on = 2: F(4x4) allowed, on its 32-channel form only (not the position-quarter kernel):
 * a training step's constant branches. The training autograd path (rpst/autograd.py)
 * sets it; an explicit RPST_CONV_ALGO still wins. */
int rpst_conv2d_set_precise(int on);

/* Position-quarter F(4x4) kernel (rpst_wino4q.hip) for the CALLING THREAD (host-only): mode
 * 0 off (every F(4x4) layer on the 32-channel kernel), 1 the default rule (Cin >= 128, Cin %
 * 16 == 0, 64 <= Cout <= 512, loader NONE / UPSAMPLE2 or the folded AdaIN), 2 forced on for
 * every shape it supports (Cin >= 16), -1 back to the RPST_W4Q environment variable (read
 * per launch; unset = 1). Same arithmetic as the 32-channel kernel within fp32 rounding.
 * Returns the previous setting. Workspace-size queries cover every setting.
 * rpst_conv2d_quarter reports whether a layer runs on it under the current settings. */
int rpst_conv2d_set_quarter(int mode);
int rpst_conv2d_quarter(int Cout, int Cin, int Hs, int Ws, int ksize, int in_op);

/* ---- stand-alone pool / upsample (same semantics as the conv input operators) ----- */
int rpst_maxpool2x2_ceil(const float* in, float* out, int N, int C, int H, int W,
                         rpst_stream_t stream);
int rpst_upsample_nearest2x(const float* in, float* out, int N, int C, int H, int W,
                            rpst_stream_t stream);
/* out (N,C,H,W) = a + upsample_nearest2x(b), b (N,C,H/2,W/2), H and W even: the merge
 * conv's input of Transform.forward (sanet.py:140-149) when that conv runs on F(4x4). */
int rpst_add_upsample_nearest2x(const float* a, const float* b, float* out, int N, int C, int H,
                                int W, rpst_stream_t stream);

/* ---- a11: SANet attention core  network/sanet.py:86-94 ------------------------------
 * O[b] = H[b] softmax_rows(F[b]^T G[b])^T  for F, G, H, O of shape (B, C, HW):
 *   S = F^T G (HW x HW, no 1/sqrt(C) scale), row softmax over keys, O = H S^T.
 * The 1x1 convs f/g/h/out_conv and mean_variance_norm run through rpst_conv2d /
 * rpst_mean_variance_norm. C in {64, 128, 256, 512} with HW % 4 == 0 runs flash-style (S
 * is never written: the keys stream through a double-buffered LDS ring with an online
 * softmax; no workspace); other shapes materialise S (B*HW*HW floats).
 * Workspace: rpst_sanet_attention_workspace_size_c(B, C, HW) (0 on the flash path);
 * rpst_sanet_attention_workspace_size(B, HW) is the materialised-S size (always enough). */
size_t rpst_sanet_attention_workspace_size(int B, int HW);
size_t rpst_sanet_attention_workspace_size_c(int B, int C, int HW);
int rpst_sanet_attention(const float* F, const float* G, const float* H, float* O, int B,
                         int C, int HW, void* workspace, size_t workspace_bytes,
                         rpst_stream_t stream);

/* ---- f3: AdaptiveSANet  network/sanet.py:12-18, 26-71, 100-138 ----
 * cal_affinity_matrix(c, s) (sanet.py:12-18): out[b] = normalize(c[b])^T normalize(s[b]),
 * normalize = x / max(||x||_2 over channels, 1e-12). c, s (B, C, HW) -> out (B, HW, HW).
 * Workspace: rpst_cosine_affinity_workspace_size(B, C, HW). */
size_t rpst_cosine_affinity_workspace_size(int B, int C, int HW);
int rpst_cosine_affinity(const float* content, const float* style, float* out, int B, int C,
                         int HW, void* workspace, size_t workspace_bytes, rpst_stream_t stream);

/* AEAModule.forward (mode 0, sanet.py:42-47) / AEALReluModule.forward (mode 1, :63-69):
 * clamp[b,i] = head(w2 . LeakyReLU_0.2(W1 x[b,i,:] + b1) + b2), head = sigmoid(t)*interval
 * + from (mode 0) or (tanh(t)+1)/2 (mode 1); out_fx = sigmoid(scale (fx - clamp)) (mode 0)
 * or softmax_rows(relu(fx - clamp)) (mode 1). x, fx, out_fx (B, HW, HW); W1 (hidden, HW),
 * b1 (hidden), w2 (hidden), b2 (1) device pointers; out_clamp (B, HW).
 * Workspace: rpst_aea_clamp_workspace_size(B, HW, hidden). */
size_t rpst_aea_clamp_workspace_size(int B, int HW, int hidden);
int rpst_aea_clamp(const float* x, const float* fx, const float* w1, const float* b1,
                   const float* w2, const float* b2, int hidden, int mode, float scale,
                   float from, float interval, float* out_fx, float* out_clamp, int B, int HW,
                   void* workspace, size_t workspace_bytes, rpst_stream_t stream);

/* AdaptiveSANet attention core (sanet.py:106-124): with S = F^T G and P = softmax_rows(S),
 * O[b] = H[b] Q^T with Q = AEA(cal_affinity_matrix(content, style), P) as rpst_aea_clamp
 * (mode/scale/from/interval). For C in {64, 128, 256, 512} and HW % 4 == 0 S is never
 * stored: a flash pass forms each query's softmax statistics, a second recomputes S per key
 * block and applies P and Q in registers (no B x HW x HW workspace); other shapes form S in
 * the workspace and apply P and Q while staging it into the second GEMM. claim_before /
 * claim_after (B, HW, HW) are written only when non-null; claim_value (B, HW) receives the
 * clamp values when non-null.
 * Workspace: rpst_adaptive_attention_workspace_size(B, C, HW, hidden). */
size_t rpst_adaptive_attention_workspace_size(int B, int C, int HW, int hidden);
int rpst_adaptive_attention(const float* F, const float* G, const float* H,
                            const float* content, const float* style, const float* w1,
                            const float* b1, const float* w2, const float* b2, int hidden,
                            int mode, float scale, float from, float interval, float* O,
                            float* claim_value, float* claim_before, float* claim_after, int B,
                            int C, int HW, void* workspace, size_t workspace_bytes,
                            rpst_stream_t stream);

/* ---- f4: host I/O pixel conversions  test.py:49-54, 139-149 ------
 * transforms.ToTensor: in (N, H, W, 3) uint8 -> out (N, 3, H, W) fp32 = u8 / 255. */
int rpst_u8hwc_to_f32nchw(const uint8_t* in, float* out, int N, int H, int W,
                          rpst_stream_t stream);
/* torchvision.utils.save_image's pixel path: in (N, 3, H, W) fp32 -> uint8 of
 * clamp(x * 255 + 0.5, 0, 255) written as the tile at (y0, x0) of each of N canvases
 * (canvas_h, canvas_w, 3) HWC. make_grid's padding is the caller's memset of the canvas. */
int rpst_f32nchw_to_u8_tile(const float* in, uint8_t* canvas, int N, int H, int W,
                            int canvas_h, int canvas_w, int y0, int x0, rpst_stream_t stream);

/* PNG "Up" filter of N 8-bit images of H rows x rowbytes bytes (e.g. rpst_f32nchw_to_u8_tile's
 * canvases, rowbytes = 3 W): out (N, H, rowbytes + 1) = per row the filter-type byte 2 then
 * (row y - row y-1) mod 256 (row -1 = 0), i.e. the PNG IDAT scanlines before zlib, so the host
 * side of save_image (test.py:139-149) is only the deflate (rpst.imageio.write_png). */
int rpst_png_filter_up(const uint8_t* in, uint8_t* out, int N, int H, int rowbytes,
                       rpst_stream_t stream);

/* ---- f2: training backward  AdaINRPNet.forward adain_rp.py:110-138 +
 * total_loss.backward() train.py:186-189. Conv dgrad runs on rpst_conv2d with weights from
 * rpst_conv_weight_flip (packed by rpst_conv2d_pack); reflect-padded convs then add
 * rpst_reflect_pad_border_grad.
 * w (Cout, Cin, k, k) -> wt (Cin, Cout, k, k), wt[ci][co][a][b] = w[co][ci][k-1-a][k-1-b]. */
int rpst_conv_weight_flip(const float* w, float* wt, int Cout, int Cin, int ksize,
                          rpst_stream_t stream);
/* ReLU backward: out = y > 0 ? g : 0 (y = the ReLU output), n elements. */
int rpst_relu_backward(const float* g, const float* y, float* out, int64_t n,
                       rpst_stream_t stream);
/* LeakyReLU(slope) backward (Conv2dBlock's activation, base.py:147; slope > 0):
 * out = y > 0 ? g : slope * g (y = the activation output, same sign as its input). */
int rpst_leaky_relu_backward(const float* g, const float* y, float* out, int64_t n, float slope,
                             rpst_stream_t stream);
/* MaxPool2d(2, 2, ceil_mode=True) backward: x (N,C,H,W) the pool input, g the gradient at
 * its output -> dx (N,C,H,W) (argmax as ATen: first max in window order, NaN wins);
 * relu_mask = 1 also applies ReLU backward with y = x (x is a ReLU output). */
int rpst_maxpool2x2_ceil_backward(const float* x, const float* g, float* dx, int N, int C,
                                  int H, int W, int relu_mask, rpst_stream_t stream);
/* ReflectionPad2d(1) + conv3x3 backward, border part: dy (N,Cout,H,W), w (Cout,Cin,3,3);
 * dx (N,Cin,H,W) holds the zero-padded dgrad and receives the padded border's gradient
 * folded onto the rows / columns it reflects. H, W >= 2.
 * Workspace: rpst_reflect_pad_border_grad_workspace_size(N, Cin, H, W). */
size_t rpst_reflect_pad_border_grad_workspace_size(int N, int Cin, int H, int W);
int rpst_reflect_pad_border_grad(const float* dy, const float* w, float* dx, int N, int Cin,
                                 int Cout, int H, int W, void* workspace, size_t workspace_bytes,
                                 rpst_stream_t stream);
/* The same, for a conv whose input is a ReLU output y (mask = y, N x Cin x H x W): the border
 * gradient is added only where y > 0, so with dx from rpst_conv2d_masked the result equals
 * rpst_relu_backward(dgrad + border, y) bit for bit (threshold_backward fused, train.py:186-189
 * backward through the decoders' Conv2d -> ReLU chains). mask may be NULL. */
int rpst_reflect_pad_border_grad_masked(const float* dy, const float* w, const float* mask,
                                        float* dx, int N, int Cin, int Cout, int H, int W,
                                        void* workspace, size_t workspace_bytes,
                                        rpst_stream_t stream);
/* conv3x3 (stride 1, zero pad 1) weight / bias gradient: x (N,Cin,H,W) the conv input, dy
 * (N,Cout,H,W) the gradient at its output -> dw (Cout,Cin,3,3), db (Cout) (db may be NULL).
 * Workspace: rpst_conv_wgrad_workspace_size(N, Cin, H, W, Cout). */
size_t rpst_conv_wgrad_workspace_size(int N, int Cin, int H, int W, int Cout);
int rpst_conv_wgrad(const float* x, const float* dy, float* dw, float* db, int N, int Cin,
                    int H, int W, int Cout, void* workspace, size_t workspace_bytes,
                    rpst_stream_t stream);
/* the same with the conv's padding: RPST_PAD_ZERO, or RPST_PAD_REFLECT (ReflectionPad2d(1) +
 * conv3x3 pad 0, the decoders of sanet.py:162-192 / base.py Conv2dBlock 'reflect'; H, W >= 2),
 * read in the loader (no padded copy). Same workspace. */
int rpst_conv_wgrad_pad(const float* x, const float* dy, float* dw, float* db, int N, int Cin,
                        int H, int W, int Cout, int pad, void* workspace,
                        size_t workspace_bytes, rpst_stream_t stream);
/* adaptive_instance_normalization backward (base.py:410-418): g the gradient at the AdaIN
 * output, c / s the content / style features (planes x HW), stats = [mean_c | std_c |
 * mean_s | std_s] (planes each) -> dc, ds. Workspace: 2*planes floats. */
int rpst_adain_backward(const float* g, const float* c, const float* s, const float* stats,
                        float* dc, float* ds, int planes, int64_t HW, void* workspace,
                        size_t workspace_bytes, rpst_stream_t stream);
/* Gradient of weights[0] * calc_style_loss(F, target) (+ weights[1] * mse(F, Fc) when Fc is
 * non-NULL) w.r.t. F (planes x HW), adain_rp.py:84-88 / 131-136 with MSELoss (mean);
 * stats = [mean | std | mean_t | std_t] (planes each); weights is a DEVICE pointer;
 * accumulate = 1 adds into out. */
int rpst_style_content_loss_grad(const float* F, const float* Fc, const float* stats,
                                 const float* weights, float* out, int planes, int64_t HW,
                                 int accumulate, rpst_stream_t stream);
/* ---- SAModel training (network/sanet.py:248-275): the extra backward pieces --------
 * 1-pixel pad of `planes` H x W planes to (H+2) x (W+2): reflect = 1 ReflectionPad2d(1)
 * (H, W >= 2), 0 zeros. A reflect-padded conv's weight gradient is rpst_conv_wgrad of the
 * padded input against the zero-padded output gradient. */
int rpst_pad1(const float* x, float* out, int64_t planes, int H, int W, int reflect,
              rpst_stream_t stream);
/* nn.Upsample(scale_factor=2, mode='nearest') backward: g (planes, 2H, 2W) -> dx (planes,
 * H, W), each dx the sum of its 2x2 block of g (sanet.py:145,166,179,186). */
int rpst_upsample_nearest2x_backward(const float* g, float* dx, int64_t planes, int H, int W,
                                     rpst_stream_t stream);
/* mean_variance_norm backward (sanet.py:20-24): y the normalised output, dy its gradient,
 * std (planes) = sqrt(var_unbiased + eps) -> dx = (dy - mean(dy) - y sum(dy y)/(HW-1))/std
 * (accumulate = 1 adds into dx). */
int rpst_mean_variance_norm_backward(const float* y, const float* dy, const float* std,
                                     float* dx, int64_t planes, int64_t HW, int accumulate,
                                     rpst_stream_t stream);
/* Row softmax (sanet.py:92-93, dim=-1) and its backward dS = P (dP - rowsum(dP P)), for
 * `rows` rows of `cols` contiguous floats (dS may alias dP). */
int rpst_softmax_rows(const float* S, float* P, int64_t rows, int cols, rpst_stream_t stream);
int rpst_softmax_rows_backward(const float* P, const float* dP, float* dS, int64_t rows,
                               int cols, rpst_stream_t stream);
/* SANet attention backward (sanet.py:86-94 under autograd; the rocBLAS batched GEMMs of
 * round 2 replaced): for F (B,C,HWc), G, H (B,C,HWs) and dO (B,C,HWc), with S = F^T G and
 * P = softmax_rows(S): dH = dO P, dP = dO^T H, dS = P (dP - rowsum(dP P)), dF = G dS^T,
 * dG = F dS. P is formed from S while staged, never stored. Workspace:
 * rpst_sanet_attention_backward_workspace_size(B, HWc, HWs) (S and dP). */
size_t rpst_sanet_attention_backward_workspace_size(int B, int HWc, int HWs);
int rpst_sanet_attention_backward(const float* F, const float* G, const float* H,
                                  const float* dO, float* dF, float* dG, float* dH, int B, int C,
                                  int HWc, int HWs, void* workspace, size_t workspace_bytes,
                                  rpst_stream_t stream);
/* The same gradients without the B x HWc x HWs terms (the training path): S and dP exist for
 * 2048 queries (whole rows) at a time; dF is written per query chunk, dH and dG are summed
 * over the chunks in order. S, its row statistics and dS are the single pass's bit for bit.
 * Workspace: rpst_sanet_attention_backward_chunked_workspace_size(B, C, HWc, HWs) =
 * 4 (2 B q HWs + 2 B q) bytes, q = min(HWc, 2048). */
size_t rpst_sanet_attention_backward_chunked_workspace_size(int B, int C, int HWc, int HWs);
int rpst_sanet_attention_backward_chunked(const float* F, const float* G, const float* H,
                                          const float* dO, float* dF, float* dG, float* dH,
                                          int B, int C, int HWc, int HWs, void* workspace,
                                          size_t workspace_bytes, rpst_stream_t stream);
/* AdaptiveSANet attention backward (sanet.py:100-138 under autograd; AdaptiveSAModel trains
 * through it, train.py:118-119): with A the cosine affinity of content / style, c the f_psi
 * clamp, S = F^T G, P = softmax_rows(S) and Q = AEA(P) (mode 0 aea: sigmoid(scale (P - c)),
 * mode 1 relu: softmax_rows(relu(P - c))), O = H Q^T: from dO (B,C,HW) -> dF, dG, dH (B,C,HW)
 * and the f_psi gradients dw1 (hidden,HW), db1 (hidden), dw2 (hidden), db2 (1). Q and P are
 * formed from S where staged, never stored; S and dQ exist for 2048 queries (whole rows) at
 * a time (no B x HW x HW term; dH, dG summed over the query chunks in order). Workspace:
 * rpst_adaptive_attention_backward_workspace_size(B, C, HW, hidden). */
size_t rpst_adaptive_attention_backward_workspace_size(int B, int C, int HW, int hidden);
int rpst_adaptive_attention_backward(const float* F, const float* G, const float* H,
                                     const float* content, const float* style, const float* w1,
                                     const float* b1, const float* w2, const float* b2,
                                     int hidden, int mode, float scale, float from,
                                     float interval, const float* dO, float* dF, float* dG,
                                     float* dH, float* dw1, float* db1, float* dw2, float* db2,
                                     int B, int C, int HW, void* workspace,
                                     size_t workspace_bytes, rpst_stream_t stream);
/* 1x1 conv weight / bias gradient over a batch (sanet.py:76-80, 97 f / g / h / out_conv):
 * dw (Cout,Cin) = sum_n dy_n x_n^T, db (Cout, may be NULL) = sum over n and pixels of dy.
 * Per-image products then a fixed-order batch sum. Workspace:
 * rpst_conv1x1_wgrad_workspace_size(N, Cin, Cout). */
size_t rpst_conv1x1_wgrad_workspace_size(int N, int Cin, int Cout);
int rpst_conv1x1_wgrad(const float* x, const float* dy, float* dw, float* db, int N, int Cin,
                       int64_t HW, int Cout, void* workspace, size_t workspace_bytes,
                       rpst_stream_t stream);
/* *out = scale * sum (a - b)^2 over n elements (fp64 accumulation, fixed order).
 * Workspace: rpst_sq_diff_workspace_size(). */
size_t rpst_sq_diff_workspace_size(void);
int rpst_sq_diff_sum(const float* a, const float* b, int64_t n, double scale, float* out,
                     void* workspace, size_t workspace_bytes, rpst_stream_t stream);

/* ---- a7: matrix_sqrt / matrix_inv_sqrt  network/wct_rp.py:7-40 ----------------------
 * out[b] = (A[b] + 1e-4 I)^(+1/2) (inverse = 0) or ^(-1/2) (inverse = 1), fp64 n x n,
 * batch of `batch`: the reference's SVD form V diag(s^p) V^T with singular values < 1e-5
 * dropped, for any input. One persistent launch runs coupled Newton-Schulz per matrix
 * (stop at the product's rounding floor, max(1e-10, 8 eps n ||Y||_F ||Z||_F), or on
 * stagnation; at most 64 steps) -- equal to the SVD form on symmetric inputs whose smallest
 * eigenvalue is provably >= 1e-5; a matrix that is not symmetric, may be truncated or did
 * not converge is recomputed by a one-sided Jacobi SVD (n <= 1024). residual (batch doubles,
 * may be NULL) receives each matrix's last Newton-Schulz residual (informational). Fully
 * asynchronous on `stream` (no host synchronisation).
 * Workspace: rpst_matrix_power_workspace_size(n, batch). */
size_t rpst_matrix_power_workspace_size(int n, int batch);
int rpst_matrix_power_psd_f64(const double* A, double* out, int n, int batch, int inverse,
                              double* residual, void* workspace, size_t workspace_bytes,
                              rpst_stream_t stream);

/* ---- a8: WCTRPNet.whiten_and_color(cF, sF, 'closed-form')  network/wct_rp.py:82-114 ---
 * cF, sF, out: (C, HW) fp64. out = T (cF - mu_c) + mu_s with the closed-form T.
 * residual (2 doubles or NULL): Newton-Schulz residuals of Cc + 1e-4 I and of Mid's argument
 * (informational; a non-finite input gives NaN in out).
 * Workspace: rpst_wct_workspace_size(1, C, HW). */
size_t rpst_wct_workspace_size(int n, int C, int64_t HW);
int rpst_whiten_and_color_f64(const double* cF, const double* sF, double* out, int C,
                              int64_t HW, double* residual, void* workspace,
                              size_t workspace_bytes, rpst_stream_t stream);

/* whiten_and_color(cF, sF, 'original') (Li et al., wct_rp.py:96-101): out =
 * matrix_sqrt(Cs) matrix_inv_sqrt(Cc + I) (cF - mu_c) + mu_s, both matrix functions in the
 * reference's SVD form (as rpst_matrix_power_psd_f64, including the 1e-5 truncation), with
 * Cc, Cs the covariances of wct_rp.py:89-94 (the content one + I). Same shapes and workspace
 * as rpst_whiten_and_color_f64. */
int rpst_whiten_and_color_original_f64(const double* cF, const double* sF, double* out, int C,
                                       int64_t HW, void* workspace, size_t workspace_bytes,
                                       rpst_stream_t stream);

/* ---- a9: WCTRPNet.fuse(content_feats, style_feats)  network/wct_rp.py:157-166 --------
 * content, style, out: (n, C, HW) fp32. Per image: widen to fp64, whiten_and_color, round
 * to fp32 — all n images in one set of launches. residual: 2n doubles or NULL (as a8, per
 * image). Workspace: rpst_wct_workspace_size(n, C, HW). */
int rpst_wct_fuse(const float* content, const float* style, float* out, int n, int C,
                  int64_t HW, double* residual, void* workspace, size_t workspace_bytes,
                  rpst_stream_t stream);

/* ---- a9 split for the fused WCTRPNet.test: the closed-form matrices without the product
 * T: (n, C, C) fp64 and offset c = mu_s - T mu_c: (n, C) fp64, so that the fused feature
 * T (cF - mu_c) + mu_s = T cF + c (wct_rp.py:109-113) is formed inside the decoder's first
 * conv (rpst_conv2d_mix) instead of being written. means: optional fp32 row means (2n x C,
 * content rows then style rows, e.g. the encoder's statistics epilogue); NULL computes them.
 * Workspace: rpst_wct_workspace_size(n, C, HW). */
int rpst_wct_params(const float* content, const float* style, const float* means, double* T,
                    double* offset, int n, int C, int64_t HW, double* residual, void* workspace,
                    size_t workspace_bytes, rpst_stream_t stream);

/* Per-image status of the last rpst_wct_fuse / rpst_wct_params call on `workspace` (same n,
 * C, HW), copied asynchronously on `stream` into status (n ints, device memory): 0 = valid,
 * otherwise a bit mask of RPST_WCT_NOCONV (a Newton-Schulz iteration did not converge:
 * non-finite features) and RPST_WCT_TIMEOUT (a group barrier of the persistent matrix-function
 * launch timed out, e.g. its workgroups were not all resident beside other work). Any non-zero
 * status comes with NaN in that image's T / offset / output — never a silently wrong finite
 * value. Read it at the caller's next natural synchronisation.
 * rpst_whiten_and_color_status: the same for the last rpst_whiten_and_color_f64 call. */
#define RPST_WCT_NOCONV 1
#define RPST_WCT_TIMEOUT 4
int rpst_wct_status(const void* workspace, int n, int C, int64_t HW, int* status,
                    rpst_stream_t stream);
int rpst_whiten_and_color_status(const void* workspace, int C, int64_t HW, int* status,
                                 rpst_stream_t stream);

/* Measurement (bench.py): while armed (rpst_wct_phase_timing(1); returns the previous
 * setting), rpst_wct_params / rpst_wct_fuse record HIP events around their covariance phase
 * (means + SYRK + reduce) and their matrix-function launch; rpst_wct_phase_ms waits for the
 * last armed call and returns the two durations in milliseconds. */
int rpst_wct_phase_timing(int on);
int rpst_wct_phase_ms(float* cov_ms, float* matfun_ms);

/* out = act(conv(pad(T_n x + c_n)) + bias) per image n: the WCT colour transform fused into
 * the consumer conv. F(4x4) layers fold T_n into per-image weights W T_n (fp64, rounded
 * once) and c_n into per-(n, co) border-class biases; other layers materialise T x + c.
 * x: (N, Cin, H, W) fp32; T: (N, Cin, Cin) fp64; offset: (N, Cin) fp64.
 * Workspace: rpst_conv2d_mix_workspace_size(N, Cin, H, W, Cout, ksize). */
size_t rpst_conv2d_mix_workspace_size(int N, int Cin, int H, int W, int Cout, int ksize);
int rpst_conv2d_mix(const float* input, const double* T, const double* offset,
                    const float* packed_weight, const float* bias, float* out, int N, int Cin,
                    int H, int W, int Cout, int ksize, int pad_mode, int relu, void* workspace,
                    size_t workspace_bytes, rpst_stream_t stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* RPST_H_ */
