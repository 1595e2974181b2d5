// dp_gemm.hip -- host side of dp_gemm: argument checks, the engine chooser (gemm_plan), the
// C ABI entry points.  The engines live in dp_gemm_impl.h, instantiated by dp_gemm_*.hip.
#include "dp_gemm_impl.h"

namespace dpg {
// Process-wide ablation / fault-injection bits, set only by dp_gemm_debug_flags (tools and
// tests; not in the ABI header).  Read once per dp_gemm call.
std::atomic<int> g_dbg_flags{0};

// persistent workgroups of the stream-K engine: one per CU, at most one per tile.
// CU count per device, cached (benign race: every writer stores the same value).
constexpr int DP_MAX_DEV = 64;
std::atomic<int> g_num_cu[DP_MAX_DEV];
int num_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  std::atomic<int>& slot = g_num_cu[dev < DP_MAX_DEV ? dev : 0];
  int n = slot.load(std::memory_order_relaxed);
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev < DP_MAX_DEV) slot.store(n, std::memory_order_relaxed);
  }
  return n;
}
}  // namespace dpg

namespace {
// the engine family that owns `tile`
int launch_tile(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s) {
  switch (tile) {
    case DP_TILE_PBIG_320x256: case DP_TILE_PBIG_256x256: return launch_part_pbig(p, tile, conv, bf16, s);
    case DP_TILE_256x64: case DP_TILE_256x32: case DP_TILE_128x128: case DP_TILE_DUAL_256x128:
      return launch_part_small(p, tile, conv, bf16, s);
    case DP_TILE_8PH_256x256: case DP_TILE_P8PH_256x256: return launch_part_8ph(p, tile, conv, bf16, s);
    case DP_TILE_8PH_320x256: return launch_part_8ph320(p, conv, bf16, s);
    case DP_TILE_CV3_256x256: return launch_part_cv3(p, conv, bf16, s);
    case DP_TILE_CV3_192x256: return launch_part_cv3(p, conv, bf16, s, 12);
    case DP_TILE_CV3_384x128: return launch_part_cv3(p, conv, bf16, s, 24);
    case DP_TILE_BIG_320x256: case DP_TILE_BIG_512x128: return launch_part_big320(p, tile, conv, bf16, s);
    default: return launch_part_big(p, tile, conv, bf16, s);
  }
}
}  // namespace


// Not part of the ABI header: ablation switches for the GEMM microbenchmark only.
extern "C" int dp_gemm_debug_flags(int flags) {
  g_dbg_flags.store(flags, std::memory_order_relaxed);
  return 0;
}

extern "C" int64_t dp_gemm_workspace_size(void) { return SK_FLAG_BYTES + (int64_t)SK_MAX_WG * SK_TILE_F * 4; }

namespace {
// After a forward (every launch that used `ws` has ended): report the sticky error word and,
// if it is set, clear it and every hand-off flag (a producer that published after its consumer
// gave up leaves its flag set; the next launch would read it as a fresh hand-off).
__global__ void ws_check_kernel(uint32_t* __restrict__ ws, int32_t* __restrict__ status) {
  const uint32_t err = ws[DP_GEMM_WS_ERROR_OFFSET / 4];
  if (threadIdx.x == 0) status[0] = (int32_t)err;
  if (err == 0) return;
  __syncthreads();
  for (int i = threadIdx.x; i < (int)(SK_FLAG_BYTES / 4); i += blockDim.x) ws[i] = 0u;
}
}  // namespace

extern "C" int dp_gemm_workspace_check(void* workspace, int32_t* status, dp_stream_t stream) {
  if (!workspace || !status) return DP_ERR_ARG;
  hipLaunchKernelGGL(ws_check_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, (uint32_t*)workspace, status);
  DP_CHECK_LAUNCH();
  return 0;
}

namespace {
// Validate the arguments, fill the kernel parameters and pick the engine.
int gemm_plan(const dp_gemm_args* a, GemmP& p, int& tile) {
  if (!a) return DP_ERR_ARG;
  if (a->M <= 0 || a->N <= 0 || a->K <= 0) return DP_ERR_SHAPE;
  if (a->K % BK != 0 || a->N % 4 != 0) return DP_ERR_SHAPE;
  if (a->ldb % 8 != 0 || (a->a_mode == DP_A_DENSE && a->lda % 8 != 0)) return DP_ERR_ALIGN;
  if (!a->A || !a->B || (!a->C && !a->ln_xl)) return DP_ERR_ARG;   // split-residual producer: C optional
  if (a->dtype != DP_BF16 && a->dtype != DP_F16) return DP_ERR_DTYPE;
  if (a->c_dtype != DP_BF16 && a->c_dtype != DP_F16 && a->c_dtype != DP_F32) return DP_ERR_DTYPE;
  if (a->c_dtype != DP_F32 && a->c_dtype != a->dtype) return DP_ERR_DTYPE;
  if (a->accumulate && a->c_dtype != DP_F32) return DP_ERR_DTYPE;
  if (a->pos && (a->pos_group <= 0)) return DP_ERR_ARG;
  if (a->a_mode == DP_A_CONV) {
    if (a->in_c % BK != 0 || a->k_h * a->k_w * a->in_c != a->K) return DP_ERR_SHAPE;
    if (a->out_h <= 0 || a->out_w <= 0 || a->stride <= 0 || a->M % (a->out_h * a->out_w) != 0)
      return DP_ERR_SHAPE;
  }
  if (a->store_mode == DP_STORE_HEAD_PS) {
    if (a->a_mode != DP_A_CONV || a->N != 128 || !a->head_w || !a->head_corr || a->c_dtype != DP_F32 ||
        a->accumulate || a->R1 || a->R2 || a->pos || a->gamma || a->act != DP_ACT_NONE)
      return DP_ERR_ARG;
  }
  if (a->store_mode == DP_STORE_ROWS && a->head_corr) {
    // composed conv with border correction: a stride-1, pad-1 3x3 implicit conv, rows = pixels
    // (no ReLU prologue: the correction is compiled into the non-ReLU conv instantiation only)
    if (a->a_mode != DP_A_CONV || a->k_h != 3 || a->k_w != 3 || a->pad != 1 || a->stride != 1 || a->head_w ||
        a->relu_a ||
        a->row_group || a->out_h != a->in_h || a->out_w != a->in_w || a->N % 8 != 0 || a->N < 128 ||
        (a->tile != DP_TILE_AUTO && a->tile <= DP_TILE_256x32))   // the small engines have no correction
      return DP_ERR_ARG;
  }
  if (a->store_mode == DP_STORE_DECONV2X2) {
    if (a->dc_cout % 4 != 0 || a->N != 4 * a->dc_cout || a->dc_h <= 0 || a->dc_w <= 0 ||
        a->M % (a->dc_h * a->dc_w) != 0)
      return DP_ERR_SHAPE;
  }
  // folded LayerNorm (ln_*): the 8-phase 320 x 256 engine only, producer = the fp32 residual
  // accumulate without activation (N % 128 == 0), consumer = 16-bit C over K = 1024 rows whose
  // gamma is folded into B / bias
  const bool lnp = a->ln_part_out || a->ln_xb_out || a->ln_xl || a->ln_rs_out,
             lnc = a->ln_part_in || a->ln_colsum || a->ln_rs_in;
  if (lnp && lnc) return DP_ERR_ARG;
  if (lnp && !a->ln_xl && (!a->ln_part_out || !a->ln_xb_out || !a->accumulate || !a->C || a->c_dtype != DP_F32 ||
                           a->act != DP_ACT_NONE || a->N % 128 != 0))
    return DP_ERR_ARG;
  // the split residual (ABI 12): x = ln_xb_out + ln_xl, both 16-bit [M][ldc], updated in place; part and
  // an fp32 copy in C optional; every byte extent below the buffer-store bound
  if (a->ln_xl && (!a->ln_xb_out || !a->accumulate || a->c_dtype != DP_F32 || a->act != DP_ACT_NONE ||
                   a->N % 128 != 0 || a->ldc % 8 != 0 || (long long)a->M * a->ldc * 4 >= 0xFFFFFF00LL))
    return DP_ERR_ARG;
  if (lnc && (!(a->ln_part_in || a->ln_rs_in) || (a->ln_part_in && a->ln_rs_in) || !a->ln_colsum || a->K != 1024 ||
              a->accumulate || a->c_dtype == DP_F32 || a->gamma || (a->act != DP_ACT_NONE && a->act != DP_ACT_GELU) ||
              !(a->ln_eps > 0.f)))
    return DP_ERR_ARG;
  // ABI 13: the producer-merged row statistics -- the split producer (8 chunks per row) with a
  // workspace for its row-tile counters; the consumer only on the persistent engine (the 320 x 256
  // consumer merges the chunks itself)
  if (a->ln_rs_out && (!a->ln_xl || !a->ln_part_out || a->N != 1024 || !(a->ln_eps > 0.f) ||
                       !(a->workspace && a->workspace_bytes >= dp_gemm_workspace_size()) ||
                       (a->M + 319) / 320 > 1023 - LN_CNT_WORD))
    return DP_ERR_ARG;
  if (a->ln_rs_in && a->tile != DP_TILE_AUTO && a->tile != DP_TILE_P8PH_256x256) return DP_ERR_ARG;
  if ((lnp || lnc) && a->tile != DP_TILE_AUTO && a->tile != DP_TILE_8PH_320x256 &&
      !(lnc && a->tile == DP_TILE_P8PH_256x256))   // (a consumer may ask for the persistent engine)
    return DP_ERR_ARG;
  const bool ws_ok = a->workspace && a->workspace_bytes >= dp_gemm_workspace_size();
  const int dbg = g_dbg_flags.load(std::memory_order_relaxed);
  tile = a->tile;
  if (a->store_mode == DP_STORE_HEAD_PS) {
    // 32-column parity groups must not straddle a wave's columns (TN = 32 or 64); the patch-conv
    // engine (one parity per wave) only when asked for: at 768^2 it runs 347 - 355 us in-frame vs
    // 249 - 255 on the 512 x 128 engine (profiles/r03w/)
    if (tile != DP_TILE_CV3_256x256 && tile != DP_TILE_CV3_384x128 && tile != DP_TILE_BIG_256x128)
      tile = a->M >= 512 * 256 ? DP_TILE_BIG_512x128 : DP_TILE_BIG_256x128;
  } else if (a->head_w) {
    if (a->N > 32 || a->store_mode != DP_STORE_ROWS) return DP_ERR_SHAPE;
    tile = DP_TILE_256x32;
  }
  const long long tiles256 = (long long)((a->M + 255) / 256) * (a->N / 256);
  if (tile == DP_TILE_STREAMK_256x256 && (!ws_ok || a->N % 256 != 0)) return DP_ERR_ARG;
  if (tile == DP_TILE_AUTO) {
    if (a->N <= 32) tile = DP_TILE_256x32;
    else if (a->N <= 64) tile = DP_TILE_256x64;
    else if (a->N % 8 != 0) tile = DP_TILE_128x128;
    else if (a->N == 128 && a->M >= 512 * 256) {   // N = 128 convs at 768^2: the head.0 conv
      // the patch-conv engine for the stride-1 square ones (the composed out_conv∘head.0), on
      // 24 x 16-pixel tiles where the side allows (48 MFMAs per wave and K step instead of 32: 381 ->
      // 369 us alone, profiles/r05am_cv3_24row/); debug 4096: the 512 x 128 engine
      const bool cv3 = a->a_mode == DP_A_CONV && a->k_h == 3 && a->k_w == 3 && a->stride == 1 && a->pad == 1 &&
                       a->in_h == a->in_w && a->out_h == a->in_h && a->out_w == a->in_w && a->in_w % 16 == 0 &&
                       a->in_c % 64 == 0 && a->head_corr && a->store_mode == DP_STORE_ROWS && a->c_dtype != DP_F32 &&
                       !a->R1 && !a->R2 && !a->gamma && !a->pos && !a->accumulate && !a->row_group && !(dbg & 4096);
      tile = !cv3 ? DP_TILE_BIG_512x128
             : a->in_w % 48 == 0 ? DP_TILE_CV3_384x128 : DP_TILE_CV3_256x256;
    }
    else if (a->N % 256 != 0) tile = DP_TILE_BIG_256x128;
    else if (ws_ok && a->a_mode == DP_A_CONV && !(dbg & 32) && tiles256 < num_cus() &&
             a->K >= 4608) {
      // Implicit convs with fewer 256 x 256 tiles than CUs and K >= 4608 (the decoder's
      // 512/1024-channel projections at 48^2 - 192^2) on the stream-K engine, each
      // tile's K range split (sk_grid): 153 -> 108, 152 -> 112, 152 -> 126 us in-frame
      // (tools/frame_shapes.py; debug flag 32 = off).  Measured and rejected: the split
      // at K = 2304 (48^2: 50 -> 80 us), and stream-K for the 384^2 / 768^2 ResidualBlock
      // convs (ReLU prologue + residual epilogue): 199 -> 265 and 744 -> 970 us in-frame,
      // although a bias-only conv of the same shape gains 8 % (tools/gemm_bench.py).
      tile = DP_TILE_STREAMK_256x256;
    } else if (ws_ok && a->K <= 256 && tiles256 >= 1024) {
      // short-K, many tiles (the 384^2 -> 768^2 deconvs: 4 K steps per tile): the
      // persistent stream-K engine keeps the next tile's loads in flight under each
      // epilogue, which otherwise dominates (tools/gemm_bench.py: 162 vs 198 us)
      tile = DP_TILE_STREAMK_256x256;
    } else {
      // Wide-N GEMMs: 256 x 256 tiles (8-phase engine once there are >= 600 of
      // them: tools/gemm_bench.py), or 320 x 256 when that needs fewer rounds of
      // workgroups over the CUs per unit of tile work -- e.g. the ViT's M = 20195
      // is exactly 64 tiles of 320 rows, so proj/fc2 (N = 1024) run as ONE round
      // of 256 tiles instead of 2 rounds of 316.
      const long long ncu = num_cus();
      const long long tiles320 = (long long)((a->M + 319) / 320) * (a->N / 256);
      const long long tiles128 = (long long)((a->M + 255) / 256) * (a->N / 128);
      // rounds x rows-of-work per tile; the 256x128 engine's loop runs ~15 % slower per FLOP
      const long long cost256 = (tiles256 + ncu - 1) / ncu * 256 * 20, cost320 = (tiles320 + ncu - 1) / ncu * 320 * 20;
      const long long cost128 = (tiles128 + ncu - 1) / ncu * 128 * 23;
      if (cost128 < cost256 && cost128 < cost320) tile = DP_TILE_BIG_256x128;
      // Measured and rejected (round 2): the 320 x 256 engine for the 768^2 ResidualBlock convs
      // (bias-only conv in isolation 648 vs 740 us, but the ReLU-prologue + residual variants
      // in-frame: eager conv total 5.61-5.71 -> 5.83-5.88 ms); fc1 on 320 x 256 (ties, below):
      // frame 24.50-24.54 vs 24.62-24.67 ms, within the box's noise.
      // ties (fc1: 4 rounds of 320 rows = 5 of 256) stay on the 8-phase engine: the
      // 320 x 256 engine is 6 % faster on fc1 in isolation (205 vs 217 us) but equal
      // in-frame (199-203 us both, profiles/r01s_fc1_engine_ab/)
      else if (cost320 < cost256) tile = DP_TILE_BIG_320x256;
      else tile = (tiles256 >= 600 && a->a_mode != DP_A_CONV) ? DP_TILE_8PH_256x256 : DP_TILE_BIG_256x256;
      // A/B switches for the fc1 shape (8-phase by default): debug 8192 -> 320 x 256,
      // 16384 -> 256 x 256 (both persistent below when eligible)
      if (tile == DP_TILE_8PH_256x256 && (dbg & 8192)) tile = DP_TILE_BIG_320x256;
      else if (tile == DP_TILE_8PH_256x256 && (dbg & 16384)) tile = DP_TILE_BIG_256x256;
    }
  }
  // split-K for small grids of long-K GEMMs (DP_TILE_SPLITK_256x256, an explicit hint; needs a
  // workspace): each 256 x 256 tile's K steps go to S = min(CUs / tiles, K steps / 2, workspace
  // slabs, 32) workgroups, then one reduce launch.  Not the auto choice: alone it takes the
  // decoder's 48^2 / 96^2 convs and projections from 49 - 115 to 34 - 74 us, but in the frame
  // their few-workgroup launches already share the chip with the decoder's other streams, and
  // taking every CU made the frame slower (47.64 vs 48.05 fps; K >= 4608 only: 47.80; at most
  // half the CUs: 48.04 -- profiles/r04o_splitk_ab/, r04n_splitk_ab/, r04m_splitk/)
  int ksplit = 1;
  if (tile == DP_TILE_SPLITK_256x256) {
    if (!ws_ok || a->N % 256 != 0 || a->store_mode != DP_STORE_ROWS || a->row_group || a->head_w || a->head_corr ||
        lnp || lnc)
      return DP_ERR_ARG;
    const long long ncu = num_cus(), kt = a->K / BK;
    const long long slab = (long long)a->M * a->N * 4;
    long long sp = ncu / tiles256;
    if (sp > kt / 2) sp = kt / 2;
    if (sp > (a->workspace_bytes - SK_FLAG_BYTES) / slab) sp = (a->workspace_bytes - SK_FLAG_BYTES) / slab;
    if (sp > 32) sp = 32;
    if (sp < 2) return DP_ERR_SHAPE;
    ksplit = (int)sp;
  }
  // byte extent of C for the persistent engine's bounded buffer stores (0: not eligible)
  unsigned c_bytes = 0;
  if (a->store_mode == DP_STORE_ROWS && !a->head_w && !a->head_corr) {
    long long last = a->M - 1;
    if (a->row_group) last = (last / a->row_group) * a->row_group_out + a->row_off + last % a->row_group;
    const long long ext = (last * a->ldc + a->N) * (a->c_dtype == DP_F32 ? 4 : 2);
    if (ext < 0xFFFFFF00LL) c_bytes = (unsigned)ext;
  }
  // the same for the deconv store of the persistent 8-phase engine (4 M output pixels; no other
  // engine takes c_bytes with that store mode)
  unsigned dcv_bytes = 0;
  if (a->store_mode == DP_STORE_DECONV2X2 && a->c_dtype != DP_F32) {
    const long long ext = ((4LL * a->M - 1) * a->ldc + a->dc_cout) * 2;
    if (ext < 0xFFFFFF00LL) dcv_bytes = (unsigned)ext;
  }
  // the persistent engines and the 8-phase 320 x 256 one keep 32-bit operand offsets (element
  // offsets from the A / B bases): beyond 2^31 elements only the 64-bit-pointer engines run
  const bool off32 = (a->a_mode != DP_A_DENSE || (long long)a->M * a->lda < (1LL << 31)) &&
                     (long long)a->N * a->ldb < (1LL << 31);
  if (!off32) c_bytes = dcv_bytes = 0;
  if ((tile == DP_TILE_PBIG_320x256 || tile == DP_TILE_PBIG_256x256) && (!c_bytes || a->N % 256)) return DP_ERR_ARG;
  // Multi-round GEMMs on the 320 x 256 / 256 x 256 engines (the ViT qkv: 768 tiles, the
  // 768^2 decoder convs: 2304) run persistent: the next tile's first K step loads under
  // each epilogue and the stores drain under the next K loop.  Debug flag 1024: off.
  if (a->tile == DP_TILE_AUTO && c_bytes && !(dbg & 1024)) {
    const long long ncu = num_cus();
    // dense (ViT) GEMMs only with debug 2048: they run beside the side encoders, and a
    // persistent grid whose workgroups cannot all start at once ends on a tail (qkv: 146 ->
    // 140 us alone, frame 23.74 -> 23.89 ms in-frame)
    const bool dense_ok = a->a_mode == DP_A_CONV || (dbg & 2048);
    if (dense_ok && tile == DP_TILE_BIG_320x256 && (long long)((a->M + 319) / 320) * (a->N / 256) >= 2 * ncu)
      tile = DP_TILE_PBIG_320x256;
    else if (dense_ok && tile == DP_TILE_BIG_256x256 && tiles256 >= 2 * ncu)
      tile = DP_TILE_PBIG_256x256;
  }
  // the persistent 8-phase engine: dense, N % 256 == 0, K >= 128, the load-free epilogue with a
  // 16-bit C and bounded buffer stores -- the planner's 8-phase launches (ViT fc1) run on it
  // (in-frame A/B, profiles/r03c_p8ph, r03d: 46.67 -> 46.79 / 46.95 fps; debug 1 << 22: off)
  // (measured and rejected: an implicit-conv A loader for the 768^2 ResidualBlock convs, 675 vs
  // 666 us on the persistent big engine, profiles/r03g_conv768_p8ph.txt)
  // the 2x2 stride-2 deconvs with >= 128 tiles on it too: short K (4 steps per tile at K = 256),
  // so the epilogue stores bound them, and here they drain under the next tile's K loop (or go
  // out as buffer stores from the MFMA layout): 384^2 -> 768^2 162 - 166 -> 136 - 137, 192^2 ->
  // 384^2 62 -> 47 us in-frame, 47.93 / 48.09 -> 48.28 / 48.37 fps (profiles/r03ab_deconv_p8ph/);
  // 96^2 -> 192^2 29.6 -> 22, 48^2 -> 96^2 (K = 1024) 42.7 -> 36, 96^2 (N = 2048) 47.5 -> 44.6 us;
  // 48 and 36 tiles were slower (26.9 -> 34, 17.1 -> 18.3 us; profiles/r03ad_deconv_small/).
  // Debug 1 << 23: off.
  const bool dcv = a->store_mode == DP_STORE_DECONV2X2 && !a->relu_a && !a->gamma && a->act == DP_ACT_NONE &&
                   a->dc_w >= 8;   // (the persistent engine's deconv store steps its rows 8 pixels at a time)
  if (a->tile == DP_TILE_AUTO && dcv && !(dbg & (1 << 23)) && tiles256 >= 128) tile = DP_TILE_P8PH_256x256;
  if (tile == DP_TILE_P8PH_256x256 || (a->tile == DP_TILE_AUTO && tile == DP_TILE_8PH_256x256 && !(dbg & (1 << 22)))) {
    const bool ok = a->a_mode == DP_A_DENSE && a->N % 256 == 0 && a->K >= 128 && a->c_dtype != DP_F32 &&
                    ((a->store_mode == DP_STORE_ROWS && c_bytes) || (dcv && dcv_bytes)) && !a->R1 && !a->R2 && !a->pos && !a->accumulate &&
                    !a->row_group && !a->head_w && !a->head_corr && !(dbg & (1 << 20));
    if (tile == DP_TILE_P8PH_256x256 && !ok) return DP_ERR_ARG;
    if (ok) tile = DP_TILE_P8PH_256x256;
    if (ok && dcv) c_bytes = dcv_bytes;
  }
  // the 8-phase 320 x 256 engine: dense, no ReLU prologue, N % 256 == 0, and an epilogue it has
  // (load-free with a 16-bit C, or the fp32 residual accumulate without activation) -- the
  // planner's dense 320 x 256 launches (ViT qkv / proj / fc2) run on it (qkv 130.6 -> 115.8,
  // fc2 149.6 -> 142.0 us, profiles/r03d_8ph320; debug 1 << 15: off)
  // the engines with the folded-LN epilogues: the 8-phase 320 x 256 one (producer and consumer),
  // and for a consumer the planner put on the persistent 8-phase engine (the ViT fc1) that one,
  // given a workspace for its merged row statistics (debug 1 << 25: the 320 x 256 engine)
  const bool lnc_p8 = lnc && tile == DP_TILE_P8PH_256x256 && (ws_ok || a->ln_rs_in) && !(dbg & (1 << 25)) &&
                      (a->ln_rs_in || (long long)(a->M + 255) / 256 * 256 * 8 <= (long long)SK_TILE_F * 4);
  if (a->ln_rs_in && !lnc_p8) return DP_ERR_ARG;
  if ((lnp || lnc) && !lnc_p8) tile = DP_TILE_8PH_320x256;
  if (tile == DP_TILE_8PH_320x256 || (a->tile == DP_TILE_AUTO && tile == DP_TILE_BIG_320x256 && !(dbg & (1 << 15)))) {
    const bool plain = a->a_mode == DP_A_DENSE && !a->relu_a && a->N % 256 == 0 && a->store_mode == DP_STORE_ROWS &&
                       !a->R1 && !a->R2 && !a->pos && !a->row_group && !a->head_w && !a->head_corr &&
                       !(dbg & (1 << 20)) && off32;
    const bool epi_ok = (!a->accumulate && a->c_dtype != DP_F32) ||
                        (a->accumulate && a->c_dtype == DP_F32 && a->act == DP_ACT_NONE);
    if (tile == DP_TILE_8PH_320x256 && !(plain && epi_ok)) return DP_ERR_ARG;
    if (plain && epi_ok) tile = DP_TILE_8PH_320x256;
  }
  // the 3x3 patch-conv engine for the many-round stride-1 3x3 convs (the decoder's 768^2
  // ResidualBlock convs: 722 -> 641 - 652 us in-frame, 45.30 / 45.41 -> 46.17 / 46.04 fps,
  // profiles/r03s_cv3/, r03u_cv3_8ph/; debug 1 << 16: off)
  if (a->tile == DP_TILE_AUTO && !(dbg & (1 << 16)) && a->a_mode == DP_A_CONV && a->k_h == 3 && a->k_w == 3 &&
      a->stride == 1 && a->pad == 1 && a->in_h == a->in_w && a->out_h == a->in_h && a->out_w == a->in_w &&
      a->in_w % 16 == 0 && a->in_c % 64 == 0 && a->N % 256 == 0 && a->store_mode == DP_STORE_ROWS &&
      !a->row_group && !a->head_w && !a->head_corr && (long long)a->M * a->in_c < (1LL << 30) && off32 &&
      a->c_dtype != DP_F32 && !a->gamma && !a->pos && !a->accumulate && a->act != DP_ACT_GELU &&
      (long long)(a->M / 256) * (a->N / 256) >= 4LL * num_cus())   // many rounds (the 768^2 maps; 384^2: 201 vs 185 us)
    tile = DP_TILE_CV3_256x256;
  // ... and on 12 x 16-pixel tiles where those make whole rounds of workgroups and 16 x 16 ones do not
  // (the 384^2 maps: 768 tiles = 3 rounds instead of 576 = 2.25: 218 -> 187 us, 49.53 / 49.77 ->
  // 50.00 / 49.99 fps same box, profiles/r05y_cv3_12row/)
  else if (a->tile == DP_TILE_AUTO && !(dbg & (1 << 16)) && a->a_mode == DP_A_CONV &&
           a->k_h == 3 && a->k_w == 3 && a->stride == 1 && a->pad == 1 && a->in_h == a->in_w &&
           a->out_h == a->in_h && a->out_w == a->in_w && a->in_w % 16 == 0 && a->in_w % 12 == 0 &&
           a->in_c % 64 == 0 && a->N % 256 == 0 && a->store_mode == DP_STORE_ROWS && !a->row_group && !a->head_w &&
           !a->head_corr && (long long)a->M * a->in_c < (1LL << 30) && off32 && a->c_dtype != DP_F32 && !a->gamma &&
           !a->pos && !a->accumulate && a->act != DP_ACT_GELU) {
    const long long t12 = (long long)(a->M / ((long long)a->in_w * a->in_w)) * (a->in_w / 12) * (a->in_w / 16) * (a->N / 256);
    const long long ncu = num_cus();
    if (t12 >= 2 * ncu && t12 % ncu == 0 && ((long long)(a->M / 256) * (a->N / 256)) % ncu != 0) tile = DP_TILE_CV3_192x256;
    // ... and single-round grids of at least half the CUs (the 192^2 convs: 192 workgroups of
    // 192 x 256 instead of 144 of 256 x 256: 81.8 -> 62.7 us alone, 49.02 / 49.09 -> 49.39 / 49.25 fps
    // same box, profiles/r05z_cv3_192/)
    else if (t12 <= ncu && 2 * t12 >= ncu) tile = DP_TILE_CV3_192x256;
  }
  if (tile >= DP_TILE_BIG_256x256 && a->N % 8 != 0) return DP_ERR_SHAPE;  // 8-column epilogue chunks
  // the border-corrected composed conv exists in the 512 x 128 conv engine only
  if (a->store_mode == DP_STORE_ROWS && a->head_corr && tile != DP_TILE_BIG_512x128 && tile != DP_TILE_CV3_256x256 &&
      tile != DP_TILE_CV3_384x128)
    return DP_ERR_ARG;
  if (tile == DP_TILE_CV3_384x128 && (!a->head_corr || a->N != 128)) return DP_ERR_ARG;

  p.M = a->M; p.N = a->N; p.K = a->K;
  p.A = (const u16*)a->A; p.lda = a->lda;
  p.B = (const u16*)a->B; p.ldb = a->ldb;
  p.relu_a = a->relu_a;
  p.in_h = a->in_h; p.in_w = a->in_w; p.in_c = a->in_c; p.k_h = a->k_h; p.k_w = a->k_w;
  p.stride = a->stride; p.pad = a->pad; p.out_h = a->out_h; p.out_w = a->out_w;
  p.bias = a->bias; p.act = a->act; p.gamma = a->gamma;
  p.pos = a->pos; p.ldpos = a->ldpos; p.pos_group = a->pos_group; p.pos_off = a->pos_off;
  p.R1 = (const u16*)a->R1; p.ldr1 = a->ldr1; p.R2 = (const u16*)a->R2; p.ldr2 = a->ldr2;
  p.C = a->C; p.ldc = a->ldc; p.c_dtype = a->c_dtype; p.accumulate = a->accumulate;
  p.store_mode = a->store_mode; p.dc_h = a->dc_h; p.dc_w = a->dc_w; p.dc_cout = a->dc_cout;
  p.row_group = a->row_group; p.row_group_out = a->row_group_out; p.row_off = a->row_off;
  p.head_w = a->head_w; p.head_b = a->head_b; p.head_corr = a->head_corr;
  p.ln_part_out = a->ln_part_out; p.ln_xb_out = (u16*)a->ln_xb_out; p.ln_xl = (u16*)a->ln_xl;
  p.ln_part_in = a->ln_part_in; p.ln_colsum = a->ln_colsum; p.ln_eps = a->ln_eps;
  p.ln_rs = a->ln_rs_in;
  p.ln_rs_out = a->ln_rs_out;
  p.ln_cnt = a->ln_rs_out ? (unsigned*)a->workspace + LN_CNT_WORD : nullptr;
  p.tiles_n = 1;
  p.tiles_m = 1;
  if (tile == DP_TILE_STREAMK_256x256) {
    p.tiles_n = a->N / 256;
    p.tiles_m = (a->M + 255) / 256;
  }
  p.dbg = dbg;
  p.c_bytes = c_bytes;
  p.ksplit = ksplit;
  p.kpart = ksplit > 1 ? (float*)((char*)a->workspace + SK_FLAG_BYTES) : nullptr;
  p.groups = 1;
  return 0;
}
}  // namespace

extern "C" int dp_gemm_plan(const dp_gemm_args* a, int32_t* tile_out, int32_t* grid_out) {
  GemmP p;
  int tile = 0;
  const int rc = gemm_plan(a, p, tile);
  if (rc) return rc;
  const int N = a->N, M = a->M;
  int bm = 256, bn = 128;
  switch (tile) {
    case DP_TILE_256x64: bn = 64; break;
    case DP_TILE_256x32: bn = 32; break;
    case DP_TILE_128x128: bm = 128; bn = 128; break;
    case DP_TILE_BIG_256x128: case DP_TILE_BIG_256x128_K32: case DP_TILE_DEEP_256x128: bn = 128; break;
    case DP_TILE_BIG_320x256: bm = 320; bn = 256; break;
    case DP_TILE_BIG_512x128: bm = 512; bn = 128; break;
    case DP_TILE_DUAL_256x128: bn = 128; break;
    case DP_TILE_PBIG_320x256: case DP_TILE_8PH_320x256: bm = 320; bn = 256; break;
    case DP_TILE_CV3_192x256: bm = 192; bn = 256; break;
    case DP_TILE_CV3_384x128: bm = 384; bn = 128; break;
    default: bn = 256;
  }
  if (tile_out) *tile_out = tile;
  int grid = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  if (tile == DP_TILE_PBIG_320x256 || tile == DP_TILE_PBIG_256x256 || tile == DP_TILE_P8PH_256x256)
    grid = grid < num_cus() ? grid : num_cus();
  if (tile == DP_TILE_SPLITK_256x256) grid *= p.ksplit;
  if (grid_out) *grid_out = tile == DP_TILE_STREAMK_256x256 ? sk_grid(p) : grid;
  return 0;
}

extern "C" int dp_gemm(const dp_gemm_args* a, dp_stream_t stream) {
  GemmP p;
  int tile = 0;
  const int rc = gemm_plan(a, p, tile);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const bool conv = a->a_mode == DP_A_CONV;
  if (tile == DP_TILE_STREAMK_256x256) return launch_part_sk(p, conv, a->workspace, a->dtype == DP_BF16, s);
  if (tile == DP_TILE_SPLITK_256x256) return launch_part_splitk(p, conv, a->dtype == DP_BF16, s);
  if (tile == DP_TILE_P8PH_256x256 && a->ln_part_in && !a->ln_rs_in) {
    // folded-LN consumer on the persistent engine: merge each row's chunk statistics into
    // (rstd, -rstd * mean) in the workspace's first partial-tile slot (no stream-K launch uses
    // it meanwhile: the workspace belongs to this stream), read by the epilogue via LDS
    float* rs = (float*)((char*)a->workspace + SK_FLAG_BYTES);
    hipLaunchKernelGGL(ln_merge_kernel, dim3((a->M + 255) / 256), dim3(256), 0, s, a->ln_part_in, a->M, a->ln_eps, rs);
    DP_CHECK_LAUNCH();
    p.ln_rs = rs;
  }
  return launch_tile(p, tile, conv, a->dtype == DP_BF16, s);
}

// Same-shape problems that differ only in their operand pointers, one launch (the image and FOV
// encoders' ViT GEMMs: encoder.py:308-311 and fov.py:66-72 run two ViT-L on the same x2 input).
// Always the 256 x 128 big engine (the tile hint is ignored): the side encoders' M = 577 plans
// onto it anyway.
extern "C" int dp_gemm_grouped(const dp_gemm_args* a, int32_t groups, dp_stream_t stream) {
  if (!a || groups < 1 || groups > DP_MAX_GROUPS) return DP_ERR_ARG;
  if (groups == 1) return dp_gemm(a, stream);
  GemmP p;
  for (int g = 0; g < groups; ++g) {
    GemmP q;
    int t = 0;
    const int rc = gemm_plan(&a[g], q, t);
    if (rc) return rc;
    const dp_gemm_args &x = a[0], &y = a[g];
    // everything but the operand pointers must agree
    if (y.M != x.M || y.N != x.N || y.K != x.K || y.dtype != x.dtype || y.lda != x.lda || y.ldb != x.ldb ||
        y.a_mode != DP_A_DENSE || x.a_mode != DP_A_DENSE || y.relu_a || y.act != x.act ||
        !y.bias != !x.bias || !y.gamma != !x.gamma || !y.pos != !x.pos || y.ldpos != x.ldpos ||
        y.pos_group != x.pos_group || y.pos_off != x.pos_off || !y.R1 != !x.R1 || y.ldr1 != x.ldr1 ||
        !y.R2 != !x.R2 || y.ldr2 != x.ldr2 || y.ldc != x.ldc || y.c_dtype != x.c_dtype ||
        y.accumulate != x.accumulate || y.store_mode != DP_STORE_ROWS || x.store_mode != DP_STORE_ROWS ||
        y.row_group != x.row_group || y.row_group_out != x.row_group_out || y.row_off != x.row_off ||
        y.head_w || y.head_corr || y.N % 8 != 0 || y.ln_part_out || y.ln_xb_out || y.ln_xl || y.ln_part_in ||
        y.ln_rs_out || y.ln_rs_in ||
        y.ln_colsum)
      return DP_ERR_ARG;
    if (g == 0) p = q;
    p.grp[g] = GemmP::Group{q.A, q.B, q.bias, q.gamma, q.pos, q.R1, q.R2, q.C};
  }
  p.groups = groups;
  hipStream_t s = (hipStream_t)stream;
  // 128 x 128 tiles: 2 x 577 rows in 10 row tiles, each workgroup a quarter of a 256 x 256 tile's
  // work, so the side workgroups that hold CUs when a one-round patch-encoder launch starts free
  // them sooner (in-frame: 48.39 -> 48.91 fps, fc1 172 -> 165 us, profiles/r04h_side_tiles/; 64 x
  // 128: 48.47, profiles/r04i_side_tiles/; final round-5 tree: 49.81 / 50.38 / 50.23 / 49.98 vs
  // 48.83 / 48.84 / 48.85 / 48.74 fps on 256 x 128, profiles/r05ay_side_tiles/).
  return launch_part_big(p, TILE_GRP_128x128, false, a->dtype == DP_BF16, s);
}

