/*
 * dp_mi355x.h -- C ABI of the MI355X-native Depth Pro hot path (libdp_mi355x.so).
 *
 * The reference (tdj28/ml-depth-pro-video) has no native code: its hot path
 * `DepthPro.infer` (src/depth_pro/depth_pro.py:243-298) dispatches PyTorch and
 * timm ops.  Each entry point below replaces a group of those ops; the comment
 * on each one cites the reference code it stands in for.  The binding the
 * reference-side would add (ctypes) is shown in INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - plain device pointers (HBM), sizes and a HIP stream (hipStream_t passed as
 *     an opaque pointer; NULL = legacy default stream);
 *   - no allocation, no host<->device copies, no synchronisation, so every call
 *     is hipGraph-capturable; the caller owns all buffers;
 *   - return 0 on success, a hipError_t value (< 1000) if a launch failed, or a
 *     DP_ERR_* code (>= 1000) for an argument/shape error detected on the host
 *     before anything was launched;
 *   - 16-bit tensors are raw bits (uint16) whose kind is given by a DP_BF16 /
 *     DP_F16 dtype argument; fp32 tensors are `float`.
 *   - safe for concurrent calls from several host threads on distinct streams: the
 *     library's only process-wide state is a per-device CU-count cache (written once,
 *     same value from every writer) and the debug/fault-injection word of the
 *     tools-only `dp_gemm_debug_flags` (not declared here), which must not change
 *     while other threads launch.
 */
#ifndef DP_MI355X_H
#define DP_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* dp_stream_t;

enum { DP_BF16 = 0, DP_F16 = 1, DP_F32 = 2 };
enum { DP_OK = 0, DP_ERR_ARG = 1000, DP_ERR_SHAPE = 1001, DP_ERR_ALIGN = 1002, DP_ERR_DTYPE = 1003 };
enum { DP_ACT_NONE = 0, DP_ACT_RELU = 1, DP_ACT_GELU = 2 };
enum { DP_A_DENSE = 0, DP_A_CONV = 1 };
enum { DP_STORE_ROWS = 0, DP_STORE_DECONV2X2 = 1, DP_STORE_HEAD_PS = 2 };

/* ABI version of this header; the Python loader refuses a mismatching .so. */
#define DP_ABI_VERSION 14
int dp_abi_version(void);

/*
 * dp_gemm: C = epilogue(A . B^T), bf16/f16 MFMA (v_mfma_f32_16x16x32_*), fp32 accumulate.
 *
 * Replaces every Linear / Conv2d / ConvTranspose2d(k2 s2) of the hot path:
 *   timm ViT qkv / proj / fc1 / fc2 Linears and the k16 s16 patch-embed conv
 *     (vit_factory.py:97-99; DINOv2 Block), fov.encoder.1 Linear (fov.py:45-47);
 *   encoder 1x1 projections + k2s2 deconvs + fuse_lowres (encoder.py:60-130, 314-324);
 *   decoder 3x3 convs, residual blocks, deconv+out_conv (decoder.py:54-206);
 *   depth head (depth_pro.py:182-207) and FOV convs (fov.py:28-54, 75-82).
 *
 * A operand: DP_A_DENSE  -> A[m][k] row-major, leading dim lda (elements);
 *            DP_A_CONV   -> implicit im2col of an NHWC tensor [batch][in_h][in_w][in_c]
 *                           for a k_h x k_w conv (stride, pad) with output out_h x out_w;
 *                           M = batch*out_h*out_w, K = k_h*k_w*in_c,
 *                           k = ((ci/64 * k_h + ky) * k_w + kx) * 64 + ci%64 (the taps of one
 *                           64-channel block are consecutive: shifted input re-reads hit L2).
 * B operand: packed weights B[n][k] row-major (ldb), i.e. W for a Linear,
 *            [Cout][Cin/64][ky][kx][64] for a conv, [(dy,dx,Cout)][Cin] for a k2s2 deconv.
 * Requirements: K % 64 == 0, N % 4 == 0, lda/ldb % 8 == 0, in_c % 64 == 0 (conv).
 *
 * Epilogue, per element, in this order:
 *   v = acc (+ bias[n]) ; act(v) ; (* gamma[n]) ; (+ pos[(m % pos_group) + pos_off][n])
 *   (+ R1[m][n]) (+ R2[m][n]) ; (+ C[m][n] when accumulate) ; store
 * Store:   DP_STORE_ROWS      -> C[row(m)][n], row(m) = m, or grouped remap
 *                                (m / row_group) * row_group_out + row_off + m % row_group;
 *          DP_STORE_DECONV2X2 -> pixel shuffle: m = (b, y, x) on a dc_h x dc_w grid,
 *                                n = (dy*2+dx)*dc_cout + co  ->  out pixel (b, 2y+dy, 2x+dx),
 *                                address C + pixel*ldc + co.
 * Fused 1x1 head (head_w != NULL; requires N <= 32): out[m] = relu(sum_n v[n]*head_w[n] + head_b)
 *   written as fp32 to C[m] (the depth head tail, depth_pro.py:200-204).
 * DP_STORE_HEAD_PS (depth head deconv + conv3x3 + ReLU + 1x1 + ReLU, depth_pro.py:182-207, composed
 *   at pack time into ONE 3x3 implicit conv over the pre-upsampling map): A_CONV over [out_h][out_w]
 *   pixels, N = 128 columns = (parity q = 2*dy+dx, channel o < 32); per output pixel
 *   (2y+dy, 2x+dx) of the 2*out_h x 2*out_w fp32 map C:
 *   relu(sum_o head_w[o] * relu(v[q*32+o] - border(q, y, x, o)) + head_b), where border() sums
 *   head_corr[(a*3+c)*32 + o] over the taps (a, c) of the 3x3 kernel that fall outside the
 *   upsampled image (the deconv bias those zero-padded taps must not carry).
 */
typedef struct dp_gemm_args {
  int32_t M, N, K;
  int32_t dtype;            /* DP_BF16 | DP_F16 : element kind of A, B, R1, R2 */
  const void* A;
  int64_t lda;
  const void* B;
  int64_t ldb;
  int32_t a_mode;           /* DP_A_DENSE | DP_A_CONV */
  int32_t relu_a;           /* apply ReLU to A elements as they are loaded */
  int32_t in_h, in_w, in_c, k_h, k_w, stride, pad, out_h, out_w;  /* conv geometry */
  const float* bias;        /* [N] or NULL */
  int32_t act;              /* DP_ACT_* */
  const float* gamma;       /* [N] or NULL (LayerScale) */
  const float* pos;         /* fp32 [*][ldpos] or NULL */
  int64_t ldpos;
  int32_t pos_group, pos_off;
  const void* R1;           /* residuals, same element kind, or NULL */
  int64_t ldr1;
  const void* R2;
  int64_t ldr2;
  void* C;
  int64_t ldc;
  int32_t c_dtype;          /* DP_BF16 | DP_F16 | DP_F32 */
  int32_t accumulate;       /* C += v (fp32 C only) */
  int32_t store_mode;       /* DP_STORE_* */
  int32_t dc_h, dc_w, dc_cout;
  int32_t row_group, row_group_out, row_off;
  const float* head_w;      /* [N] or NULL */
  float head_b;
  const float* head_corr;   /* DP_STORE_HEAD_PS: [9][32] border corrections; DP_STORE_ROWS with a
                               stride-1 pad-1 3x3 implicit conv on the 512x128 or the patch-conv
                               engine (N = 128 at M >= 512*256, or those tile hints): [9][N]
                               per-tap values subtracted where the tap falls in the zero padding
                               (a composed 1x1-then-3x3 conv's bias); else NULL */
  int32_t tile;             /* 0 = auto, else a DP_TILE_* hint */
  void* workspace;          /* NULL, or >= dp_gemm_workspace_size() bytes of device memory owned by
                               the caller for THIS stream (never shared by concurrent launches);
                               enables the persistent stream-K engine for large 256x256-tiled GEMMs */
  int64_t workspace_bytes;
  /* LayerNorm folded across the GEMM boundary (timm Block norm1 / norm2, eps ln_eps), dense A,
   * the 8-phase 320 x 256 engine (DP_TILE_8PH_320x256; NULL fields: off):
   *  producer -- the residual GEMM (accumulate into fp32 C, act none) also writes
   *    ln_xb_out:   the new rows of C in 16 bits (dtype), [M][ldc];
   *    ln_part_out: fp32 [M][N/128][2]: (mean, M2) of each 128-column chunk of the new rows;
   *  consumer -- A = a producer's ln_xb_out (un-normalised rows), B = W o ln.weight (per k)
   *    [o gamma (per n)], bias = (b + W . ln.bias) [* gamma], gamma = NULL,
   *    ln_part_in = the producer's ln_part_out ([M][K/128][2]), ln_colsum[N] = sum_k B[n][k]
   *    (the 16-bit values, summed exactly); the epilogue's value before act is
   *      v = rstd * acc - rstd * mean * ln_colsum[n] + bias[n]
   *    with (mean, rstd) of the row merged from its K/128 chunks: LN(x) . W^T + b exactly, up
   *    to where the 16-bit rounding falls (x instead of LN(x)).
   *  producer on a SPLIT residual (ABI 12, ln_xl != NULL): the residual stream is held as a 16-bit
   *    high part (ln_xb_out, dtype, [M][ldc]) and an int8 low part (ln_xl, [M][ldc] bytes), read and
   *    updated in place:  x = hi + q * 2^(e - S)  with e the frexp exponent of hi (hi = m 2^e,
   *    m in [0.5, 1)), S = 16 (bf16) / 19 (f16), i.e. q counts steps of ulp(hi) / 256;
   *    x' = v + x;  hi' = x' rounded to 16 bits;  q' = clamp(rint((x' - hi') 2^(S - e')), -128, 127)
   *    (~16 significant bits: the patch encoder's error vs fp32 moves 2.3788e-3 -> 2.3809e-3,
   *    tools/hilo_emul.py); ln_part_out as above or NULL; C (fp32, [M][ldc]) is not read: NULL, or
   *    written with x' (for a reader of the fp32 rows); accumulate = 1, act none, N % 128 == 0,
   *    M * ldc * 4 < 2^32 - 256.  6 instead of 10 bytes of HBM traffic per element in a residual
   *    GEMM's epilogue. */
  float* ln_part_out;
  void* ln_xb_out;
  const float* ln_part_in;
  const float* ln_colsum;
  float ln_eps;
  void* ln_xl;
  /* ABI 13: the row statistics merged by the producer (the persistent consumer's merge pre-pass
   * folded into the split-residual producer): with ln_rs_out set (split producer, N == 1024,
   * ln_part_out set, a workspace), the last workgroup to finish each row tile merges the tile's
   * rows' 8 chunk statistics into ln_rs_out[m] = (rstd, -rstd * mean) (eps ln_eps; the arithmetic
   * of the pre-pass, bit for bit); a consumer on the persistent 8-phase engine takes ln_rs_in =
   * that array instead of ln_part_in (no pre-pass launch, no workspace needed).  ln_rs_in holds
   * M rounded up to an even number of rows (its reads go in row pairs). */
  float* ln_rs_out;
  const float* ln_rs_in;
} dp_gemm_args;

enum { DP_TILE_AUTO = 0, DP_TILE_128x128 = 1, DP_TILE_256x64 = 2, DP_TILE_256x32 = 3,
       DP_TILE_BIG_256x256 = 4, DP_TILE_BIG_256x128 = 5, DP_TILE_BIG_256x256_K32 = 6,
       DP_TILE_BIG_256x128_K32 = 7, DP_TILE_8PH_256x256 = 8, DP_TILE_DEEP4_256x256 = 9,
       DP_TILE_DEEP5_256x256 = 10, DP_TILE_DEEP_256x128 = 11, DP_TILE_STREAMK_256x256 = 12,
       DP_TILE_BIG_320x256 = 13, DP_TILE_BIG_512x128 = 14, DP_TILE_PBIG_320x256 = 15,
       DP_TILE_PBIG_256x256 = 16, DP_TILE_DUAL_256x128 = 17,
       DP_TILE_P8PH_256x256 = 18, DP_TILE_8PH_320x256 = 19, DP_TILE_CV3_256x256 = 20,
       DP_TILE_SPLITK_256x256 = 21, DP_TILE_CV3_192x256 = 22, DP_TILE_CV3_384x128 = 23 };
/* DP_TILE_P8PH_256x256: persistent 8-phase engine (min(tiles, CUs) workgroups, each a stream of
   K steps over its tiles; dense A, N % 256 == 0, K >= 128, 16-bit C without per-row operands);
   the auto choice for the ViT fc1.  DP_TILE_8PH_320x256: 8-phase 320 x 256 engine (dense A, no
   ReLU prologue, N % 256 == 0; 16-bit C without per-row operands, or an fp32 C accumulated into
   without activation); the auto choice for the ViT qkv / proj / fc2.  A hint an engine cannot
   serve returns DP_ERR_ARG.  DP_TILE_CV3_256x256: stride-1 pad-1 3x3 implicit conv on 16 x 16 pixel
   tiles with the input patch in LDS (square maps, side % 16 == 0, in_c % 64 == 0; N % 256 == 0 with
   ReLU / residual epilogues, or N % 128 == 0 with head_corr, or DP_STORE_HEAD_PS); the auto choice
   for the many-round ResidualBlock convs and the border-corrected composed conv at 768^2.
   DP_TILE_CV3_192x256: the same engine on 12 x 16-pixel tiles (side % 48 == 0, N % 256 == 0, the
   ReLU / residual epilogues): the auto choice where those tiles make whole rounds of workgroups and
   16 x 16 ones do not (the 384^2 ResidualBlock convs and projection: 768 tiles = 3 rounds).
   DP_TILE_CV3_384x128 (ABI 14): the same engine on 24 x 16-pixel tiles of 128 output channels
   (side % 48 == 0, N == 128, with head_corr: the border-corrected composed conv, or
   DP_STORE_HEAD_PS): the auto choice for the former (out_conv∘head.0 at 768^2: 1536 tiles =
   6 rounds); a hint for the composed depth head, whose auto choice stays the 512 x 128 engine.
   DP_TILE_SPLITK_256x256 (ABI 11, a hint only, needs a workspace): split-K for small grids -- the
   256 x 256 tiles' K steps split over up to (CUs / tiles) workgroups that write fp32 partials into
   the workspace, then a reduce launch sums them in split order and runs the epilogue
   (DP_STORE_ROWS, no row groups / head); DP_ERR_SHAPE when no split of >= 2 fits.
   Sizes: the 8-phase 320 x 256 engine, the persistent engines (P8PH, PBIG) and the patch-conv
   engine keep 32-bit element offsets from the A / B bases, so they serve M * lda and N * ldb
   below 2^31 only; past that the planner takes the 64-bit-pointer engines and a hint for one
   of those returns DP_ERR_ARG. */

int dp_gemm(const dp_gemm_args* args, dp_stream_t stream);

/*
 * dp_gemm_grouped: `groups` (1..4) dp_gemm problems in ONE launch.  args[0..groups-1] must agree
 * in every field but the operand pointers A, B, bias, gamma, pos, R1, R2 and C (dense A, row
 * stores, no fused head); each problem gives exactly the result its own dp_gemm call would
 * (the 256 x 128 big engine; the tile hint is ignored).  Replaces the image encoder's and the FOV
 * encoder's ViT Linears / patch embeds -- two ViT-L with their own weights over the same x2 input
 * (encoder.py:308-311, fov.py:66-72) -- run side by side as one workgroup range per problem.
 */
int dp_gemm_grouped(const dp_gemm_args* args, int32_t groups, dp_stream_t stream);

/*
 * Bytes of workspace the stream-K engine needs (flags + one fp32 256x256 partial
 * tile per persistent workgroup).  The caller zeroes it once after allocation; every
 * hand-off flag a stream-K launch sets is reset by the workgroup that consumes it, so
 * the flags are zero again whenever a launch ends (no per-launch clearing, nothing but
 * kernels touches it -- graph-replay safe), the rest is scratch -- except the ERROR WORD: the
 * uint32 at byte offset DP_GEMM_WS_ERROR_OFFSET becomes non-zero when a stream-K
 * launch on this workspace gave up waiting for another workgroup's partial tile
 * (bounded spin; the output of that launch is then wrong).  It is sticky: nothing
 * but the caller clears it, so one read after a whole forward / graph replay covers
 * every launch in it.  After a timeout the flags may be left set: zero the first 1 KiB
 * (or the whole workspace) before reusing it.
 */
#define DP_GEMM_WS_ERROR_OFFSET 4092
int64_t dp_gemm_workspace_size(void);

/*
 * dp_gemm_workspace_check: for the end of a forward (after every launch on `workspace`):
 * *status (device int32) = the sticky error word; if it is set, the error word and every
 * hand-off flag are zeroed, so the next forward starts clean and its own status reflects only
 * its own launches.  One tiny kernel, graph-capturable.  (Reference: none -- the per-frame
 * failure detection of SURVEY.md section 5 replacing the reference's per-frame try/except,
 * generate_depth_maps.py:147-151.)
 */
int dp_gemm_workspace_check(void* workspace, int32_t* status, dp_stream_t stream);

/*
 * Which engine / tile and how many workgroups dp_gemm would launch for `args`
 * (no launch): *tile receives a DP_TILE_* value (DP_TILE_STREAMK_256x256 for the
 * persistent engine), *grid the workgroup count.  For tests and the bench.
 */
int dp_gemm_plan(const dp_gemm_args* args, int32_t* tile, int32_t* grid);

/*
 * dp_layernorm: y[r] = LN(x[r]) * w + b over `cols`, fp32 in, 16-bit out.
 * Replaces timm Block norm1/norm2 and the final `norm` (eps 1e-6).
 */
int dp_layernorm(const float* x, int64_t ldx, const float* w, const float* b, void* y, int64_t ldy,
                 int32_t rows, int32_t cols, float eps, int32_t dtype, dp_stream_t stream);

/*
 * dp_layernorm_stats: the input side of a folded LayerNorm (dp_gemm_args.ln_*): for the rows of
 * fp32 x [rows][cols] (cols % 128 == 0, <= 2048) write x in 16 bits (xb [rows][ldxb], dtype) and
 * part fp32 [rows][cols/128][2] = (mean, M2) of each 128-column chunk -- what the residual GEMMs'
 * producer epilogue writes, for the rows no GEMM produced (the patch embed + cls rows that enter
 * ViT block 0).  xl (ABI 12; NULL: none): the int8 low part of the split residual ([rows][ldxb]
 * bytes, the encoding of dp_gemm_args.ln_xl), so that (xb, xl) is the stream a split-residual
 * producer reads.
 */
int dp_layernorm_stats(const float* x, int64_t ldx, int32_t rows, int32_t cols, void* xb, int64_t ldxb,
                       void* xl, float* part, int32_t dtype, dp_stream_t stream);

/*
 * dp_layernorm_grouped: dp_layernorm over groups * rows_per_group rows, rows of group g taking
 * w[g] / b[g] (w, b: HOST arrays of `groups` (1..4) device pointers) -- the image and FOV
 * encoders' norm1 / norm2 / final norm in one launch.
 */
int dp_layernorm_grouped(const float* x, int64_t ldx, const float* const* w, const float* const* b,
                         int32_t groups, void* y, int64_t ldy, int32_t rows_per_group, int32_t cols,
                         float eps, int32_t dtype, dp_stream_t stream);

/*
 * dp_attention: multi-head softmax attention, flash-style (no S x S in HBM).
 * qkv: [batch*seq][3*heads*head_dim] (timm's qkv Linear output, (3, heads, hd) column order);
 * out: [batch*seq][heads*head_dim] (timm's transpose(1,2).reshape). head_dim must be 64.
 * Replaces timm Attention's F.scaled_dot_product_attention (scale = head_dim^-0.5).
 */
int dp_attention(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads,
                 int32_t head_dim, float scale, int32_t dtype, dp_stream_t stream);

/*
 * dp_attention_log2q: dp_attention for a qkv whose Q columns already hold
 * Q * scale * log2(e) -- folded into the qkv Linear's epilogue as a per-column gamma --
 * so the scores leave the MFMA in log2 units and the softmax needs one exp2 per score.
 * Same result as dp_attention up to where the scale is rounded (before the 16-bit Q).
 */
int dp_attention_log2q(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads,
                       int32_t head_dim, int32_t dtype, dp_stream_t stream);

/*
 * dp_normalize_u8: uint8 HWC image -> (x/255 - 0.5)/0.5 planar CHW (fp32 or 16-bit).
 * Replaces the transform Compose (depth_pro.py:125-132) with the u8 upload + GPU normalize.
 */
int dp_normalize_u8(const uint8_t* img_hwc, int32_t H, int32_t W, void* out_chw, int32_t out_dtype,
                    dp_stream_t stream);

/*
 * dp_resize_bilinear: planar C x H x W (fp32 or 16-bit) -> C x OH x OW fp32,
 * bilinear, align_corners=False, no antialias, optional scalar pre-multiply
 * (F.interpolate as used by DepthPro.infer, depth_pro.py:271-279 and 288-291).
 */
int dp_resize_bilinear(const void* src, int32_t src_dtype, int32_t C, int32_t H, int32_t W,
                       float* dst, int32_t OH, int32_t OW, dp_stream_t stream);

/*
 * dp_resize: dp_resize_bilinear with the F.interpolate mode DepthPro.infer passes through
 * (`interpolation_mode`, depth_pro.py:243-279): DP_INTERP_BILINEAR, or DP_INTERP_BICUBIC
 * (upsample_bicubic2d, align_corners=False, A = -0.75, border taps clamped).
 */
enum { DP_INTERP_BILINEAR = 0, DP_INTERP_BICUBIC = 1 };
int dp_resize(const void* src, int32_t src_dtype, int32_t C, int32_t H, int32_t W, float* dst,
              int32_t OH, int32_t OW, int32_t mode, dp_stream_t stream);

/*
 * dp_patchify_pyramid: 1536^2 planar fp32 image -> im2col rows of the 35 sliding
 * windows [35*576][768] (k = c*256 + ky*16 + kx), building the 768^2 and 384^2
 * pyramid levels on the fly (the bilinear 0.5 / 0.25 resizes are exact 2x2 box
 * averages).  Replaces _create_pyramid + split + cat (encoder.py:151-188, 245-263)
 * and the patch-embed unfold.  Window 34 (384^2 level) is also the image-encoder
 * and FOV-encoder input (encoder.py:308-311, fov.py:66-72).
 */
int dp_patchify_pyramid(const float* x0, void* cols, int32_t dtype, dp_stream_t stream);

/*
 * dp_vit_cls_rows: x[w*577] = cls + pos[0] for w < n_images (timm _pos_embed cls row),
 * x fp32 [n_images*577][1024].
 */
int dp_vit_cls_rows(float* x, const float* cls, const float* pos, int32_t n_images, dp_stream_t stream);

/*
 * dp_merge_windows: stitch steps x steps token windows into an NHWC map, dropping the
 * cls token and cropping `padding` tokens at inner edges (encoder.py:190-231).
 * src rows: window w token t at row (w*577 + t), ld_src elements, fp32 or 16-bit;
 * dst: [S][S][1024] 16-bit with S = steps*24 - 2*padding*(steps-1).
 */
int dp_merge_windows(const void* src, int32_t src_dtype, int64_t ld_src, int32_t first_window,
                     int32_t steps, int32_t padding, void* dst, int32_t dtype, dp_stream_t stream);

/*
 * dp_merge_windows_range: dp_merge_windows restricted to the windows w_lo <= w < w_hi of the
 * steps x steps grid (w = row * steps + column); the other pixels of dst are not written.
 * For a patch encoder run as several independent window groups (each merges its own share
 * of a hooked block's output before it moves on).
 */
int dp_merge_windows_range(const void* src, int32_t src_dtype, int64_t ld_src, int32_t first_window,
                           int32_t steps, int32_t padding, int32_t w_lo, int32_t w_hi, void* dst,
                           int32_t dtype, dp_stream_t stream);

/*
 * dp_fov_tail: final FOV conv 6x6 (32 -> 1) + bias on the 6x6x32 NHWC map
 * (fov.py:46, head[4]).  w is the PyTorch weight [1][32][6][6] fp32.
 */
int dp_fov_tail(const void* x6, int32_t dtype, const float* w, float bias, float* fov_deg,
                dp_stream_t stream);

/*
 * dp_infer_epilogue (depth_pro.py:282-298):
 *   f_px = use_given ? f_given : 0.5*W / tan(0.5*deg2rad(fov_deg))   (fp32)
 *   inv  = canonical * scale, scale = use_given ? (float)(W / f_given) : W / f_px
 *   inv  = bilinear(inv, (H, W)) when (H, W) != (1536, 1536)
 *   depth = 1 / clamp(inv, 1e-4, 1e4)   (a NaN stays NaN, as torch.clamp)  -> depth [H][W] fp32
 * f_px_out (device float) receives f_px.  nonfinite (optional device int32): incremented by the
 * number of NaN / inf values written (depth and f_px) -- a per-frame health word the frame loops
 * read back before writing a frame's files.
 */
int dp_infer_epilogue(const float* canonical, int32_t src_h, int32_t src_w, const float* fov_deg,
                      int32_t use_given, double f_given, int32_t H, int32_t W, float* depth,
                      float* f_px_out, int32_t* nonfinite, dp_stream_t stream);

/* dp_infer_epilogue_mode: the same with the resize back to (H, W) in `mode` (DP_INTERP_*,
 * depth_pro.py:288-291 passes interpolation_mode). */
int dp_infer_epilogue_mode(const float* canonical, int32_t src_h, int32_t src_w, const float* fov_deg,
                           int32_t use_given, double f_given, int32_t H, int32_t W, float* depth,
                           float* f_px_out, int32_t* nonfinite, int32_t mode, dp_stream_t stream);

/*
 * dp_resize_u8_cv: cv2.resize of an 8-bit HWC 3-channel frame to OH x OW -- the reference's
 * --downscale_factor (generate_depth_maps.py:95-110: INTER_AREA for factor < 1, INTER_LINEAR
 * otherwise, new size int(H * factor) x int(W * factor)).  OpenCV 4.x's published fixed-point
 * bilinear (11-bit coefficients) and area-averaging rules, restated in oracle/cv_resize_oracle.py
 * (parity unpinned vs a cv2 binary: none is available).
 */
enum { DP_CV_INTER_LINEAR = 1, DP_CV_INTER_AREA = 3 };   /* cv2's constants */
int dp_resize_u8_cv(const uint8_t* src, int32_t H, int32_t W, uint8_t* dst, int32_t OH, int32_t OW,
                    int32_t interpolation, dp_stream_t stream);

/*
 * dp_depth_to_points: camera-space point cloud of a depth map -- the reference's
 * depth_to_3d (img_to_normalized_pointcloud.py:819-856), used before its PLY write-out
 * (:1318).  valid = !isnan(depth) && depth > 0, points in row-major pixel order (numpy
 * boolean indexing), fp64 as numpy computes them:
 *   x = -1*(u - W/2)*z/f, y = -1*(v - H/2)*z/f, z = depth      (f = f_px if use_given,
 *   else (double)*f_px_dev, e.g. dp_infer_epilogue's f_px_out).
 * row_offsets: int32 [H+1] scratch; receives the exclusive prefix of valid counts per row
 * and the total in row_offsets[H].  xyz: fp64 [H*W][3] (capacity); rgb_out (optional):
 * uint8 [H*W][3] colours gathered from rgb_hwc (uint8 [H][W][3]) at the same pixels.
 */
int dp_depth_to_points(const float* depth, int32_t H, int32_t W, const float* f_px_dev, double f_px,
                       int32_t use_given, const uint8_t* rgb_hwc, int32_t* row_offsets, double* xyz,
                       uint8_t* rgb_out, dp_stream_t stream);

/*
 * dp_depth_to_image: the frame loop's depth writers on the GPU (generate_depth_maps.py:15-44
 * colorize_depth, :135-143 --raw): nanmin / nanmax of depth[n] into minmax (2 x uint32 scratch,
 * order-preserving keys), then per pixel v = (d - min) / (max - min) in fp32 and
 *   DP_DEPTH_IMG_COLOR: out uint8 [n][3] = lut[trunc(clip(v, 0, 1) * N)] (N -> N - 1; NaN -> entry
 *     N + 2, matplotlib's "bad"); lut uint8 [(N + 3)][3] = (colormap lut * 255).astype(uint8);
 *   DP_DEPTH_IMG_RAW16: out uint16 [n] = (uint16)(v * 65535) (NaN -> 0).
 * Byte-identical to the reference's numpy / matplotlib arithmetic.
 */
enum { DP_DEPTH_IMG_COLOR = 0, DP_DEPTH_IMG_RAW16 = 1 };
int dp_depth_to_image(const float* depth, int64_t n, uint32_t* minmax, const uint8_t* lut, int32_t lut_n,
                      int32_t mode, void* out, dp_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DP_MI355X_H */
