// dp_gemm_impl.h -- the dp_gemm engines (device code + launchers), shared by the
// translation units that instantiate them (dp_gemm_*.hip, one engine family each, so the
// build compiles them in parallel) and the host API (dp_gemm.hip).
//
// dp_gemm: bf16/f16 MFMA GEMM with an implicit-conv A loader and a fused
// epilogue, for gfx950 (CDNA4).  Two tile engines share one epilogue:
//
// * "big" (256 x BN x 64, BN in {256, 128}; 512 threads = 8 wave64s as 2 x 4,
//   each wave 128 x BN/4): operands stream global -> LDS directly with
//   global_load_lds_dwordx4 (no VGPR staging) into a 2-stage LDS ring; the
//   loads for K-tile t+2 are issued as soon as tile t has been consumed, so a
//   whole tile of MFMA work covers their latency, and the waits are counted
//   (`s_waitcnt vmcnt(N)` + raw `s_barrier`, never a full drain in the loop).
//   1 workgroup per CU; the 256-row A panel halves L2->LDS traffic per FLOP
//   compared with a 128^2 tile.  Block ids are remapped so that the blocks one
//   XCD runs are a contiguous range of tiles (shared A panels stay in that
//   XCD's L2).
// * "small" (BM x BN x 64, 256 threads, register-staged, 2 workgroups/CU):
//   N <= 64 outputs (depth-head tail, FOV head) and the fused 1x1 head.
//
// Both: LDS rows are 128 B (64 x 16-bit) with the 16-B chunk index XOR-swizzled
// by (row & 7) -> conflict-free ds_read_b128 fragment reads.  The MFMA
// v_mfma_f32_16x16x32_{bf16,f16} is issued with the weight fragment as its
// A-operand and the activation fragment as B, so D = C^T: each lane ends up
// with 4 consecutive output channels of one output row, and bias / gamma /
// residual loads and the stores are 8-16 B per lane.

#include "dp_common.h"

#pragma once
#include <atomic>
#include <type_traits>

namespace dpg {

constexpr int BK = 64;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

constexpr int DP_MAX_GROUPS = 4;   // dp_gemm_grouped

struct GemmP {
  int M, N, K;
  const u16* A;
  long long lda;
  const u16* B;
  long long ldb;
  int relu_a;
  int in_h, in_w, in_c, k_h, k_w, stride, pad, out_h, out_w;
  const float* bias;
  int act;
  const float* gamma;
  const float* pos;
  long long ldpos;
  int pos_group, pos_off;
  const u16* R1;
  long long ldr1;
  const u16* R2;
  long long ldr2;
  void* C;
  long long ldc;
  int c_dtype;
  int accumulate;
  int store_mode;
  int dc_h, dc_w, dc_cout;
  int row_group, row_group_out, row_off;
  const float* head_w;
  float head_b;
  const float* head_corr;
  int tiles_n, tiles_m;
  int dbg;  // ablation bits for tools/gemm_bench.py: 1 no stores, 2 no loads in loop, 4 no MFMA
  unsigned c_bytes;  // persistent engine: byte extent of C from p.C (buffer-store bound)
  // LayerNorm folded across the GEMM boundary (dp_gemm_args.ln_*; the 8-phase 320 x 256 engine)
  float* ln_part_out;      // producer: (mean, M2) per 128-column chunk of the new C rows
  u16* ln_xb_out;          // producer: the new C rows in 16 bits ([M][ldc])
  u16* ln_xl;              // producer on a split residual (hi = ln_xb_out, lo = ln_xl; read + written)
  const float* ln_part_in; // consumer: the A rows' chunk statistics ([M][K/128][2])
  const float* ln_colsum;  // consumer: sum_k B[n][k]
  float ln_eps;
  const float* ln_rs;      // consumer on the persistent 8-phase engine: per row (rstd, -rstd * mean),
                           // merged from ln_part_in by ln_merge_kernel into the GEMM workspace, or
                           // the producer's ln_rs_out (ABI 13)
  float* ln_rs_out;        // split producer: the last workgroup of each row tile merges its rows
  unsigned* ln_cnt;        // ... counting the tile's arrivals here (workspace words LN_CNT_WORD ..)
  // dp_gemm_grouped: `groups` problems of one shape in one launch (workgroup range g * tiles_m *
  // tiles_n ... covers problem g, whose operand pointers are grp[g]); 1 otherwise
  int groups;
  // split-K (DP_TILE_SPLITK_256x256): workgroup range s * tiles ... covers K-steps [s KT / ksplit,
  // (s+1) KT / ksplit) of every tile and stores raw fp32 partials into kpart + s M N; a reduce
  // launch adds them and runs the epilogue; 1 otherwise
  int ksplit;
  float* kpart;
  struct Group {
    const u16* A;
    const u16* B;
    const float* bias;
    const float* gamma;
    const float* pos;
    const u16* R1;
    const u16* R2;
    void* C;
  } grp[DP_MAX_GROUPS];
};


// Process-wide ablation / fault-injection bits (dp_gemm.hip), set only by dp_gemm_debug_flags
// (tools and tests; not in the ABI header).  Read once per dp_gemm call.
extern std::atomic<int> g_dbg_flags;
// CU count of the current device (cached, dp_gemm.hip)
int num_cus();

// Engine families, one translation unit each: launch `p` (planned by dp_gemm.hip) on `tile`.
int launch_part_big(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s);      // dp_gemm_big.hip
constexpr int TILE_GRP_128x128 = -1;   // internal: the grouped (side-encoder) launches' 128 x 128 big tile
int launch_part_big320(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s);   // dp_gemm_big320.hip
int launch_part_8ph(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s);      // dp_gemm_8ph.hip
int launch_part_8ph320(const GemmP& p, bool conv, bool bf16, hipStream_t s);             // dp_gemm_8ph320.hip
int launch_part_cv3(const GemmP& p, bool conv, bool bf16, hipStream_t s, int th = 16);                // dp_gemm_cv3.hip
int launch_part_pbig(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s);     // dp_gemm_pbig.hip
int launch_part_small(const GemmP& p, int tile, bool conv, bool bf16, hipStream_t s);    // dp_gemm_small.hip
int launch_part_sk(const GemmP& p, bool conv, void* ws, bool bf16, hipStream_t s);       // dp_gemm_sk.hip
int launch_part_splitk(const GemmP& p, bool conv, bool bf16, hipStream_t s);             // dp_gemm_splitk.hip
}  // namespace dpg

namespace {
using namespace dpg;

// Fewer tiles than CUs (the decoder's 48^2 - 192^2 convs: 9 - 144 tiles of 256 x 256,
// 36 - 144 k-steps): the K range of every tile is split over up to SK_MAX_SPLIT
// workgroups of >= SK_MIN_STEPS k-steps each (the owner adds the others' fp32
// partials, 256 KiB apiece), or, at more than half a chip of tiles, spread over
// every CU.  debug flag 32 restores one workgroup per tile.
constexpr int SK_MIN_STEPS = 8, SK_MAX_SPLIT = 6;
int sk_grid(const GemmP& p) {
  const int tiles = p.tiles_m * p.tiles_n;
  int g = num_cus();
  if (g > 256) g = 256;   // == SK_MAX_WG (workspace slots)
  if (tiles >= g) return g;
  if (p.dbg & 32) return tiles;
  const int kt = p.K / 64;
  int s = g / tiles;
  if (s < 2) return kt >= 2 * SK_MIN_STEPS ? g : tiles;
  if (s > SK_MAX_SPLIT) s = SK_MAX_SPLIT;
  if (s > kt / SK_MIN_STEPS) s = kt / SK_MIN_STEPS;
  return tiles * (s < 1 ? 1 : s);
}

#ifdef DP_STAMPS
// Timing-only builds (make stamps): per-workgroup s_memrealtime (100 MHz) stamps
// [start, first tile visible, main loop done, end, hw_id | xcc_id << 32].
__device__ unsigned long long g_stamps[5 * 65536];
#define DP_STAMP(v)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");    \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#define DP_STAMPS_DECL unsigned long long st0_ = 0, st1_ = 0, st2_ = 0, st3_ = 0
// the persistent 8-phase engine: per workgroup and tile (up to P8_STAMP_TILES) [K loop start, K loop
// done (boundary issue + epilogue begin), epilogue done (its stores issued)], + hw_id | xcc_id << 32
constexpr int P8_STAMP_TILES = 8, P8_STAMP_W = 3 * P8_STAMP_TILES + 1;
__device__ unsigned long long g_p8_stamps[P8_STAMP_W * 1024];
#define DP_STAMP_SAVE(wg)                                                             \
  do {                                                                                \
    if (threadIdx.x == 0 && (wg) < 65536) {                                           \
      unsigned hw_, xcc_;                                                             \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));              \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));            \
      unsigned long long* d_ = g_stamps + 5 * (wg);                                   \
      d_[0] = st0_; d_[1] = st1_; d_[2] = st2_; d_[3] = st3_;                         \
      d_[4] = hw_ | ((unsigned long long)xcc_ << 32);                                 \
    }                                                                                 \
  } while (0)
#else
#define DP_STAMP(v) do { } while (0)
#define DP_STAMPS_DECL
#define DP_STAMP_SAVE(wg) do { } while (0)
#endif

// 256 zero bytes: source of the implicit-conv zero padding for LDS-DMA loads and of the
// persistent engine's absent column constants
__device__ __attribute__((aligned(16))) uint32_t g_zero_page[64];

__device__ __forceinline__ int lds_off(int row, int chunk) {  // element offset, 64-wide rows
  return row * BK + ((chunk ^ (row & 7)) << 3);
}

// ---------------------------------------------------------------- epilogue
// v[0..3] = accumulators of output (m, n..n+3).  Order: bias, act, gamma, pos,
// R1, R2, (+C), store; with head_w the values are folded into hsum instead.
template <typename K_>
__device__ __forceinline__ void epilogue4(const GemmP& p, int m, int n, float (&v)[4], float& hsum) {
  if (p.bias) {
    float4 b = *(const float4*)(p.bias + n);
    v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
  }
  if (p.act == DP_ACT_RELU) {
    #pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
  } else if (p.act == DP_ACT_GELU) {
    #pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
  }
  if (p.gamma) {
    float4 g = *(const float4*)(p.gamma + n);
    v[0] *= g.x; v[1] *= g.y; v[2] *= g.z; v[3] *= g.w;
  }
  if (p.pos) {
    const float* pp = p.pos + (long long)(m % p.pos_group + p.pos_off) * p.ldpos + n;
    float4 q = *(const float4*)pp;
    v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
  }
  if (p.R1) {
    uint2 r = *(const uint2*)(p.R1 + (long long)m * p.ldr1 + n);
    v[0] += K_::to_f(r.x & 0xffff); v[1] += K_::to_f(r.x >> 16);
    v[2] += K_::to_f(r.y & 0xffff); v[3] += K_::to_f(r.y >> 16);
  }
  if (p.R2) {
    uint2 r = *(const uint2*)(p.R2 + (long long)m * p.ldr2 + n);
    v[0] += K_::to_f(r.x & 0xffff); v[1] += K_::to_f(r.x >> 16);
    v[2] += K_::to_f(r.y & 0xffff); v[3] += K_::to_f(r.y >> 16);
  }
  if (p.head_w) {
    float4 w = *(const float4*)(p.head_w + n);
    hsum += v[0] * w.x + v[1] * w.y + v[2] * w.z + v[3] * w.w;
    return;
  }
  long long off;
  if (p.store_mode == DP_STORE_DECONV2X2) {
    const int hw = p.dc_h * p.dc_w;
    const int b = m / hw, rr = m - b * hw;
    const int y = rr / p.dc_w, x = rr - y * p.dc_w;
    const int q = n / p.dc_cout, co = n - q * p.dc_cout;
    const long long pix = ((long long)b * 2 * p.dc_h + 2 * y + (q >> 1)) * (2 * p.dc_w) + 2 * x + (q & 1);
    off = pix * p.ldc + co;
  } else {
    long long row = m;
    if (p.row_group) row = (long long)(m / p.row_group) * p.row_group_out + p.row_off + m % p.row_group;
    off = row * p.ldc + n;
  }
  if (p.c_dtype == DP_F32) {
    float* c = (float*)p.C + off;
    if (p.accumulate) {
      float4 o = *(const float4*)c;
      v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
    }
    *(float4*)c = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 o;
    o.x = (uint32_t)K_::from_f(v[0]) | ((uint32_t)K_::from_f(v[1]) << 16);
    o.y = (uint32_t)K_::from_f(v[2]) | ((uint32_t)K_::from_f(v[3]) << 16);
    *(uint2*)((u16*)p.C + off) = o;
  }
}

// Same epilogue for 8 consecutive columns n..n+7 (N % 8 == 0 on this path):
// 16-32 B loads and stores per lane.
template <typename K_>
__device__ __forceinline__ void add8_16(float (&v)[8], const u16* p) {
  const uint4 r = *(const uint4*)p;
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  #pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] += K_::to_f(w[k] & 0xffff);
    v[2 * k + 1] += K_::to_f(w[k] >> 16);
  }
}
__device__ __forceinline__ void add8_f32(float (&v)[8], const float* p) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
  v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
}
template <typename K_>
__device__ __forceinline__ void epilogue8(const GemmP& p, int m, int n, float (&v)[8]) {
  if (p.bias) add8_f32(v, p.bias + n);
  if (p.act == DP_ACT_RELU) {
    #pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
  } else if (p.act == DP_ACT_GELU) {
    #pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = gelu_erf(v[r]);
  }
  if (p.gamma) {
    const float4 a = *(const float4*)(p.gamma + n), b = *(const float4*)(p.gamma + n + 4);
    v[0] *= a.x; v[1] *= a.y; v[2] *= a.z; v[3] *= a.w;
    v[4] *= b.x; v[5] *= b.y; v[6] *= b.z; v[7] *= b.w;
  }
  if (p.pos) add8_f32(v, p.pos + (long long)(m % p.pos_group + p.pos_off) * p.ldpos + n);
  if (p.R1) add8_16<K_>(v, p.R1 + (long long)m * p.ldr1 + n);
  if (p.R2) add8_16<K_>(v, p.R2 + (long long)m * p.ldr2 + n);
  long long off;
  if (p.store_mode == DP_STORE_DECONV2X2) {
    const int hw = p.dc_h * p.dc_w;
    const int b = m / hw, rr = m - b * hw;
    const int y = rr / p.dc_w, x = rr - y * p.dc_w;
    const int q = n / p.dc_cout, co = n - q * p.dc_cout;
    const long long pix = ((long long)b * 2 * p.dc_h + 2 * y + (q >> 1)) * (2 * p.dc_w) + 2 * x + (q & 1);
    off = pix * p.ldc + co;
  } else {
    long long row = m;
    if (p.row_group) row = (long long)(m / p.row_group) * p.row_group_out + p.row_off + m % p.row_group;
    off = row * p.ldc + n;
  }
  if (p.c_dtype == DP_F32) {
    float* c = (float*)p.C + off;
    if (p.accumulate) add8_f32(v, c);
    *(float4*)c = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    uint4 o;
    o.x = (uint32_t)K_::from_f(v[0]) | ((uint32_t)K_::from_f(v[1]) << 16);
    o.y = (uint32_t)K_::from_f(v[2]) | ((uint32_t)K_::from_f(v[3]) << 16);
    o.z = (uint32_t)K_::from_f(v[4]) | ((uint32_t)K_::from_f(v[5]) << 16);
    o.w = (uint32_t)K_::from_f(v[6]) | ((uint32_t)K_::from_f(v[7]) << 16);
    *(uint4*)((u16*)p.C + off) = o;
  }
}

// Row-staged epilogue for the big engines.  Per-column operands (bias, LayerScale
// gamma) are loaded once per lane -- a lane keeps the same 8 columns for the whole
// tile -- and each batch of NIT rows issues ALL of its row-dependent loads
// (residuals, the fp32 C being accumulated into) before any arithmetic or store, so
// their latencies overlap instead of serialising behind the stores.
struct ColConst {
  float b[8], g[8];
};
__device__ __forceinline__ void load_colconst(const GemmP& p, int n, ColConst& c) {
  const bool ok = n < p.N;
  if (p.bias && ok) {
    const float4 x = *(const float4*)(p.bias + n), y = *(const float4*)(p.bias + n + 4);
    c.b[0] = x.x; c.b[1] = x.y; c.b[2] = x.z; c.b[3] = x.w; c.b[4] = y.x; c.b[5] = y.y; c.b[6] = y.z; c.b[7] = y.w;
  } else {
    #pragma unroll
    for (int r = 0; r < 8; ++r) c.b[r] = 0.f;
  }
  if (p.gamma && ok) {
    const float4 x = *(const float4*)(p.gamma + n), y = *(const float4*)(p.gamma + n + 4);
    c.g[0] = x.x; c.g[1] = x.y; c.g[2] = x.z; c.g[3] = x.w; c.g[4] = y.x; c.g[5] = y.y; c.g[6] = y.z; c.g[7] = y.w;
  } else {
    #pragma unroll
    for (int r = 0; r < 8; ++r) c.g[r] = 1.f;
  }
}
__device__ __forceinline__ long long out_offset(const GemmP& p, int m, int n) {
  if (p.store_mode == DP_STORE_DECONV2X2) {
    const int hw = p.dc_h * p.dc_w;
    const int b = m / hw, rr = m - b * hw;
    const int y = rr / p.dc_w, x = rr - y * p.dc_w;
    const int q = n / p.dc_cout, co = n - q * p.dc_cout;
    const long long pix = ((long long)b * 2 * p.dc_h + 2 * y + (q >> 1)) * (2 * p.dc_w) + 2 * x + (q & 1);
    return pix * p.ldc + co;
  }
  long long row = m;
  if (p.row_group) row = (long long)(m / p.row_group) * p.row_group_out + p.row_off + m % p.row_group;
  return row * p.ldc + n;
}
template <typename K_>
__device__ __forceinline__ void add8_u4(float (&v)[8], uint4 r) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  #pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] += K_::to_f(w[k] & 0xffff);
    v[2 * k + 1] += K_::to_f(w[k] >> 16);
  }
}
// Composed 3x3-after-1x1 conv (DP_STORE_ROWS with head_corr, engine.compose_head0): the 1x1's
// bias rides in the composed bias for all 9 taps; at the image border the taps that fall in
// the 3x3's zero padding must not contribute it: subtract corr[(ky*3+kx)*N + n] for each.
__device__ __forceinline__ void border_correct(const GemmP& p, int m, int nc, float (&z)[8]) {
  const int hw = p.out_h * p.out_w;
  const int rr = m % hw;
  const int yy = rr / p.out_w, xx = rr - yy * p.out_w;
  const bool top = yy == 0, bot = yy == p.out_h - 1, lft = xx == 0, rgt = xx == p.out_w - 1;
  if (!(top || bot || lft || rgt)) return;
  // a rolled loop with two 16-B loads per tap: few live registers in an epilogue that is
  // already at the 256-VGPR limit (the unrolled 9 x 8 form cost 71 spills)
  #pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    const int a = t / 3, c = t - 3 * (t / 3);
    const bool oob = (a == 0 && top) || (a == 2 && bot) || (c == 0 && lft) || (c == 2 && rgt);
    if (oob) {
      const float4 lo = *(const float4*)(p.head_corr + t * p.N + nc);
      const float4 hi = *(const float4*)(p.head_corr + t * p.N + nc + 4);
      z[0] -= lo.x; z[1] -= lo.y; z[2] -= lo.z; z[3] -= lo.w;
      z[4] -= hi.x; z[5] -= hi.y; z[6] -= hi.z; z[7] -= hi.w;
    }
  }
}
// v[it][0..7] = accumulators of row ms[it], columns n..n+7.  Loads go to clamped
// (always valid) rows with no predicate, so the compiler issues the whole batch
// back to back instead of sinking each load into its own branch; only the
// stores are predicated.
// BC: this instantiation applies the composed-conv border correction (only the 512 x 128 conv
// engine has it: compiled into every engine's epilogue it costs the 320 x 256 one ~170 spills)
template <typename K_, int NIT, bool BC = false>
__device__ __forceinline__ void epilogue_rows(const GemmP& p, const ColConst& cc, const int (&ms)[NIT], int n,
                                              float (&v)[NIT][8]) {
  const int nc = n < p.N ? n : p.N - 8;
  int mc[NIT];
  long long off[NIT];
  #pragma unroll
  for (int it = 0; it < NIT; ++it) {
    mc[it] = ms[it] < p.M ? ms[it] : p.M - 1;
    off[it] = out_offset(p, mc[it], nc);
  }
  uint4 r1[NIT], r2[NIT];
  float4 c0[NIT], c1[NIT];
  if (p.R1) {
    #pragma unroll
    for (int it = 0; it < NIT; ++it) r1[it] = *(const uint4*)(p.R1 + (long long)mc[it] * p.ldr1 + nc);
  }
  if (p.R2) {
    #pragma unroll
    for (int it = 0; it < NIT; ++it) r2[it] = *(const uint4*)(p.R2 + (long long)mc[it] * p.ldr2 + nc);
  }
  const bool acc32 = p.accumulate && p.c_dtype == DP_F32;
  if (acc32) {
    #pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float* c = (const float*)p.C + off[it];
      c0[it] = *(const float4*)c;
      c1[it] = *(const float4*)(c + 4);
    }
  }
  #pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float (&x)[8] = v[it];
    #pragma unroll
    for (int r = 0; r < 8; ++r) x[r] += cc.b[r];
    if constexpr (BC) {
      if (p.head_corr) border_correct(p, mc[it], nc, x);
    }
    if (p.act == DP_ACT_RELU) {
      #pragma unroll
      for (int r = 0; r < 8; ++r) x[r] = fmaxf(x[r], 0.f);
    } else if (p.act == DP_ACT_GELU) {
      #pragma unroll
      for (int r = 0; r < 8; ++r) x[r] = gelu_erf(x[r]);
    }
    if (p.gamma) {
      #pragma unroll
      for (int r = 0; r < 8; ++r) x[r] *= cc.g[r];
    }
    if (p.pos) add8_f32(x, p.pos + (long long)(mc[it] % p.pos_group + p.pos_off) * p.ldpos + nc);
    if (p.R1) add8_u4<K_>(x, r1[it]);
    if (p.R2) add8_u4<K_>(x, r2[it]);
    if (acc32) {
      x[0] += c0[it].x; x[1] += c0[it].y; x[2] += c0[it].z; x[3] += c0[it].w;
      x[4] += c1[it].x; x[5] += c1[it].y; x[6] += c1[it].z; x[7] += c1[it].w;
    }
  }
  const bool nok = n < p.N;
  #pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const float (&x)[8] = v[it];
    if (!(nok && ms[it] < p.M)) continue;
    if (p.c_dtype == DP_F32) {
      float* c = (float*)p.C + off[it];
      *(float4*)c = make_float4(x[0], x[1], x[2], x[3]);
      *(float4*)(c + 4) = make_float4(x[4], x[5], x[6], x[7]);
    } else {
      uint4 o;
      o.x = (uint32_t)K_::from_f(x[0]) | ((uint32_t)K_::from_f(x[1]) << 16);
      o.y = (uint32_t)K_::from_f(x[2]) | ((uint32_t)K_::from_f(x[3]) << 16);
      o.z = (uint32_t)K_::from_f(x[4]) | ((uint32_t)K_::from_f(x[5]) << 16);
      o.w = (uint32_t)K_::from_f(x[6]) | ((uint32_t)K_::from_f(x[7]) << 16);
      *(uint4*)((u16*)p.C + off[it]) = o;
    }
  }
}

// epilogue_rows for the persistent engine: the same arithmetic, C written with buffer stores
// that EVERY lane issues -- rows past M (or columns past N) get the out-of-range offset
// c_bytes and are dropped -- so the number of stores per tile is a compile-time constant
// the engine's counted vmcnt relies on.  DP_STORE_ROWS only.
template <typename K_, int NIT>
__device__ __forceinline__ void epilogue_rows_buf(const GemmP& p, const ColConst& cc, const int (&ms)[NIT], int n,
                                                  float (&v)[NIT][8], __amdgpu_buffer_rsrc_t crs, int esz) {
  const int nc = n < p.N ? n : p.N - 8;
  int mc[NIT];
  long long off[NIT];
  #pragma unroll
  for (int it = 0; it < NIT; ++it) {
    mc[it] = ms[it] < p.M ? ms[it] : p.M - 1;
    off[it] = out_offset(p, mc[it], nc);
  }
  uint4 r1[NIT], r2[NIT];
  float4 c0[NIT], c1[NIT];
  if (p.R1) {
    #pragma unroll
    for (int it = 0; it < NIT; ++it) r1[it] = *(const uint4*)(p.R1 + (long long)mc[it] * p.ldr1 + nc);
  }
  if (p.R2) {
    #pragma unroll
    for (int it = 0; it < NIT; ++it) r2[it] = *(const uint4*)(p.R2 + (long long)mc[it] * p.ldr2 + nc);
  }
  const bool acc32 = p.accumulate && p.c_dtype == DP_F32;
  if (acc32) {
    #pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float* c = (const float*)p.C + off[it];
      c0[it] = *(const float4*)c;
      c1[it] = *(const float4*)(c + 4);
    }
  }
  const bool nok = n < p.N;
  #pragma unroll
  for (int it = 0; it < NIT; ++it) {
    float (&x)[8] = v[it];
    #pragma unroll
    for (int r = 0; r < 8; ++r) x[r] += cc.b[r];
    if (p.act == DP_ACT_RELU) {
      #pragma unroll
      for (int r = 0; r < 8; ++r) x[r] = fmaxf(x[r], 0.f);
    } else if (p.act == DP_ACT_GELU) {
      #pragma unroll
      for (int r = 0; r < 8; ++r) x[r] = gelu_erf(x[r]);
    }
    if (p.gamma) {
      #pragma unroll
      for (int r = 0; r < 8; ++r) x[r] *= cc.g[r];
    }
    if (p.pos) add8_f32(x, p.pos + (long long)(mc[it] % p.pos_group + p.pos_off) * p.ldpos + nc);
    if (p.R1) add8_u4<K_>(x, r1[it]);
    if (p.R2) add8_u4<K_>(x, r2[it]);
    if (acc32) {
      x[0] += c0[it].x; x[1] += c0[it].y; x[2] += c0[it].z; x[3] += c0[it].w;
      x[4] += c1[it].x; x[5] += c1[it].y; x[6] += c1[it].z; x[7] += c1[it].w;
    }
    const unsigned bo = (nok && ms[it] < p.M) ? (unsigned)(off[it] * esz) : p.c_bytes;
    if (p.c_dtype == DP_F32) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, f32x4_t{x[0], x[1], x[2], x[3]}), crs, bo, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, f32x4_t{x[4], x[5], x[6], x[7]}), crs,
                                             bo == p.c_bytes ? bo : bo + 16, 0, 0);
    } else {
      u32x4_t o;
      o[0] = (uint32_t)K_::from_f(x[0]) | ((uint32_t)K_::from_f(x[1]) << 16);
      o[1] = (uint32_t)K_::from_f(x[2]) | ((uint32_t)K_::from_f(x[3]) << 16);
      o[2] = (uint32_t)K_::from_f(x[4]) | ((uint32_t)K_::from_f(x[5]) << 16);
      o[3] = (uint32_t)K_::from_f(x[6]) | ((uint32_t)K_::from_f(x[7]) << 16);
      __builtin_amdgcn_raw_buffer_store_b128(o, crs, bo, 0, 0);
    }
  }
}

// epilogue_acc32_wide + the producer side of a folded LayerNorm: besides C (fp32, accumulated),
// the new rows go out in 16 bits (p.ln_xb_out, staged through the wave's LDS region so each row
// leaves as one 256-B segment) and, per row, (mean, M2) of the wave's 128 columns
// (p.ln_part_out[m][n_base / 128]) -- shifted single-pass sums (shift = the row's first value,
// so no cancellation) reduced over the row's 4 lanes.  C is bit-identical to epilogue_acc32_wide.
// `slab`: the wave's LDS region, >= 5 KiB.
template <typename K_, int FM, int FN>
__device__ __forceinline__ void epilogue_acc32_wide_ln(const GemmP& p, f32x4_t (&acc)[FM][FN], char* slab, int lane,
                                                       int m_base, int n_base) {
  #pragma clang fp contract(off)
  static_assert(FN == 8, "wide epilogue");
  constexpr int H = FN / 2;
  const int t = lane & 15, g = lane >> 4;
  {
    const int c = 4 * (lane & 31), n = n_base + c;
    f32x4_t v;
    if (lane < 32) v = (p.bias && n < p.N) ? *(const f32x4_t*)(p.bias + n) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    else v = (p.gamma && n < p.N) ? *(const f32x4_t*)(p.gamma + n) : f32x4_t{1.f, 1.f, 1.f, 1.f};
    *(f32x4_t*)(slab + (lane < 32 ? 0 : 512) + c * 4) = v;
  }
  char* const xst = slab + 1024;          // 16 rows x 128 columns x 16 bit, chunk ^ row swizzle
  float* const C = (float*)p.C;
  const int nch = p.N / 128;
  f32x4_t cur[H], nxt[H];
  auto load = [&](int ch, f32x4_t (&c)[H]) __attribute__((always_inline)) {
    const int fm = ch >> 1, h = ch & 1;
    const int m = min(m_base + fm * 16 + t, p.M - 1);
    #pragma unroll
    for (int f = 0; f < H; ++f)
      c[f] = *(const f32x4_t*)(C + (long long)m * p.ldc + n_base + (h * H + f) * 16 + 4 * g);
  };
  load(0, cur);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float sh = 0.f, s1 = 0.f, s2 = 0.f;
  #pragma unroll
  for (int ch = 0; ch < 2 * FM; ++ch) {
    if (ch + 1 < 2 * FM) load(ch + 1, nxt);
    const int fm = ch >> 1, h = ch & 1;
    const int m = m_base + fm * 16 + t;
    #pragma unroll
    for (int f = 0; f < H; ++f) {
      const int fn = h * H + f;
      const f32x4_t b = *(const f32x4_t*)(slab + (fn * 16 + 4 * g) * 4);
      const f32x4_t q = *(const f32x4_t*)(slab + 512 + (fn * 16 + 4 * g) * 4);
      f32x4_t x;
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[fm][fn][r] + b[r];
        x[r] = v * q[r] + cur[f][r];
      }
      if (m < p.M) *(f32x4_t*)(C + (long long)m * p.ldc + n_base + fn * 16 + 4 * g) = x;
      if (h == 0 && f == 0) {
        sh = __shfl(x[0], t);             // the row's value at column n_base (lane t, g = 0)
        s1 = 0.f;
        s2 = 0.f;
      }
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = x[r] - sh;
        s1 += d;
        s2 += d * d;
      }
      uint2 w;
      w.x = K_::pack2(x[0], x[1]);
      w.y = K_::pack2(x[2], x[3]);
      *(uint2*)(xst + t * 256 + (((fn * 2 + (g >> 1)) ^ t) << 4) + (g & 1) * 8) = w;
    }
    #pragma unroll
    for (int f = 0; f < H; ++f) cur[f] = nxt[f];
    if (h == 1) {
      // the row's 128 columns: 4 lanes (g) of 32 values each
      s1 += __shfl_xor(s1, 16);
      s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      if (g == 0 && m < p.M) {
        const float mc = sh + s1 * (1.f / 128);
        const float m2 = s2 - s1 * (s1 * (1.f / 128));
        *(float2*)(p.ln_part_out + ((long long)m * nch + n_base / 128) * 2) = make_float2(mc, m2);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's staging writes
      #pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = k * 4 + (lane >> 4), chunk = lane & 15;
        const uint4 d = *(const uint4*)(xst + row * 256 + ((chunk ^ row) << 4));
        const int mm = m_base + fm * 16 + row;
        if (mm < p.M) *(uint4*)(p.ln_xb_out + (long long)mm * p.ldc + n_base + chunk * 8) = d;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read back before the next row's writes
    }
  }
}


// Epilogue variants.  needs_rowld: the launch reads per-row operands (R1 / R2, pos, the fp32 C
// it accumulates into) or stores through a remap (deconv pixel shuffle, row groups, the fused /
// composed heads).  Without any of those (and with a 16-bit C) the engines take the load-free
// epilogue_mfma below: no loads at all, so the compiler needs no `s_waitcnt vmcnt(0)` between
// row batches (in the general epilogue a runtime-conditional load in a batch makes it wait for
// every older VMEM op, i.e. for the previous batches' stores: the epilogue serialised on store
// latency, fc1 221.6 -> 211.2 us and qkv 146.3 -> 135.1 us without it).
__host__ __device__ inline bool needs_rowld(const GemmP& p) {
  return p.R1 || p.R2 || p.pos || p.accumulate || p.store_mode != DP_STORE_ROWS || p.row_group || p.head_corr ||
         p.head_w;
}
// Load-free epilogue in the MFMA register layout (no per-row operands, 16-bit C): lane
// (t = lane & 15, g = lane >> 4) of accumulator fragment (fm, fn) holds token row fm * 16 + t,
// channels fn * 16 + 4 g .. + 3.  bias / ACT / gamma are applied right there, on all FM x FN x 4
// values of the lane at once (no per-row batches: the compiler interleaves 128 independent GELU
// chains), packed to 16 bits and staged through the wave's LDS slab as [rows][TN] 16-bit rows
// (16-B chunks XOR-swizzled by row), which are read back row-major and stored as whole row
// segments (TN * 2 bytes per row, 16 B per lane).  PF fragment rows per pass (slab: PF * 16 *
// TN * 2 bytes per wave).  LDS operations of one wave complete in order, so the write -> read
// -> next pass's write sequence needs no barrier (the slab is the wave's own).
template <typename K_, int ACT, int FM, int FN, int TN, int PF>
__device__ __forceinline__ void epilogue_mfma(const GemmP& p, f32x4_t (&acc)[FM][FN], char* slab, int lane,
                                              int m_base, int n_base) {
  constexpr int CH = TN / 8;            // 16-B chunks per staged row
  constexpr int RPI = 64 / CH;          // rows per read-back instruction
  static_assert(FM % PF == 0 && (CH == 16 || CH == 8 || CH == 4), "tile");
  const int t = lane & 15, g = lane >> 4;
  float bias[FN][4], gam[FN][4];
  #pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int n = n_base + fn * 16 + 4 * g;
    const bool ok = n < p.N;
    const float4 b = (p.bias && ok) ? *(const float4*)(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 q = (p.gamma && ok) ? *(const float4*)(p.gamma + n) : make_float4(1.f, 1.f, 1.f, 1.f);
    bias[fn][0] = b.x; bias[fn][1] = b.y; bias[fn][2] = b.z; bias[fn][3] = b.w;
    gam[fn][0] = q.x; gam[fn][1] = q.y; gam[fn][2] = q.z; gam[fn][3] = q.w;
  }
  #pragma unroll
  for (int f0 = 0; f0 < FM; f0 += PF) {
    #pragma unroll
    for (int fm = 0; fm < PF; ++fm)
      #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        // packed-f32 arithmetic on the lane's 4 columns (gelu_erf4): same values as per element
        f32x4_t x = acc[f0 + fm][fn] + f32x4_t{bias[fn][0], bias[fn][1], bias[fn][2], bias[fn][3]};
        if constexpr (ACT == DP_ACT_RELU) {
          #pragma unroll
          for (int r = 0; r < 4; ++r) x[r] = fmaxf(x[r], 0.f);
        } else if constexpr (ACT == DP_ACT_GELU) {
          x = gelu_erf4(x);
        }
        x = x * f32x4_t{gam[fn][0], gam[fn][1], gam[fn][2], gam[fn][3]};
        const int row = fm * 16 + t;
        const int chunk = fn * 2 + (g >> 1);
        uint2 w;
        w.x = K_::pack2(x[0], x[1]);
        w.y = K_::pack2(x[2], x[3]);
        *(uint2*)(slab + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4) + (g & 1) * 8) = w;
      }
    #pragma unroll
    for (int k = 0; k < PF * 16 / RPI; ++k) {
      const int row = k * RPI + lane / CH, chunk = lane % CH;
      const uint4 d = *(const uint4*)(slab + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4));
      const int m = m_base + f0 * 16 + row, n = n_base + chunk * 8;
      if (m < p.M && n < p.N) *(uint4*)((u16*)p.C + (long long)m * p.ldc + n) = d;
    }
  }
}

// epilogue_mfma for the consumer of a folded LayerNorm (the ViT qkv / fc1 over un-normalised
// 16-bit rows, dp_gemm_args.ln_part_in): per value v = rstd * acc - rstd * mean * colsum[n] +
// bias[n], then ACT, packed to 16 bits and stored as epilogue_mfma does (PF = 1).  The wave's
// bias / colsum live in its LDS region (first KiB; staging after it), and each fragment row's
// 8 chunk statistics are loaded one row ahead and merged (Chan) -- no per-column or per-row
// register arrays beside the 160 accumulators.  `slab` >= 1 KiB + 16 * TN * 2 bytes.
template <typename K_, int ACT, int FM, int FN, int TN>
__device__ __forceinline__ void epilogue_mfma_lnc(const GemmP& p, f32x4_t (&acc)[FM][FN], char* slab, int lane,
                                                  int m_base, int n_base) {
  constexpr int CH = TN / 8, RPI = 64 / CH;
  static_assert(TN == 128 && FN == 8, "wide consumer epilogue");
  const int t = lane & 15, g = lane >> 4;
  {
    // lanes 0-31: bias of columns 4 lane .. +3; lanes 32-63: colsum
    const int c = 4 * (lane & 31), n = n_base + c;
    f32x4_t v;
    if (lane < 32) v = (p.bias && n < p.N) ? *(const f32x4_t*)(p.bias + n) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    else v = n < p.N ? *(const f32x4_t*)(p.ln_colsum + n) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    *(f32x4_t*)(slab + (lane < 32 ? 0 : 512) + c * 4) = v;
  }
  char* const stg = slab + 1024;
  f32x4_t cur[4], nxt[4];
  auto load = [&](int fm, f32x4_t (&c)[4]) __attribute__((always_inline)) {
    const int m = min(m_base + fm * 16 + t, p.M - 1);
    const f32x4_t* pp = (const f32x4_t*)(p.ln_part_in + (long long)m * 16);
    #pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = pp[i];
  };
  load(0, cur);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the constants, before any read of them
  #pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    if (fm + 1 < FM) load(fm + 1, nxt);
    // the row's mean / rstd from its 8 chunks of 128 columns
    const float mean = (((cur[0][0] + cur[0][2]) + (cur[1][0] + cur[1][2])) +
                        ((cur[2][0] + cur[2][2]) + (cur[3][0] + cur[3][2]))) * (1.f / 8);
    float m2 = 0.f;
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d0 = cur[i][0] - mean, d1 = cur[i][2] - mean;
      m2 += (cur[i][1] + 128.f * d0 * d0) + (cur[i][3] + 128.f * d1 * d1);
    }
    const float rs = rsqrtf(m2 * (1.f / 1024) + p.ln_eps), nm = -rs * mean;
    #pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const f32x4_t b = *(const f32x4_t*)(slab + (fn * 16 + 4 * g) * 4);
      const f32x4_t q = *(const f32x4_t*)(slab + 512 + (fn * 16 + 4 * g) * 4);
      f32x4_t x = __builtin_elementwise_fma(acc[fm][fn], (f32x4_t)(rs), __builtin_elementwise_fma(q, (f32x4_t)(nm), b));
      if constexpr (ACT == DP_ACT_RELU) {
        #pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = fmaxf(x[r], 0.f);
      } else if constexpr (ACT == DP_ACT_GELU) {
        x = gelu_erf4(x);
      }
      const int row = t;
      const int chunk = fn * 2 + (g >> 1);
      uint2 w;
      w.x = K_::pack2(x[0], x[1]);
      w.y = K_::pack2(x[2], x[3]);
      *(uint2*)(stg + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4) + (g & 1) * 8) = w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    #pragma unroll
    for (int k = 0; k < 16 / RPI; ++k) {
      const int row = k * RPI + lane / CH, chunk = lane % CH;
      const uint4 d = *(const uint4*)(stg + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4));
      const int m = m_base + fm * 16 + row, n = n_base + chunk * 8;
      if (m < p.M && n < p.N) *(uint4*)((u16*)p.C + (long long)m * p.ldc + n) = d;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    #pragma unroll
    for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
  }
}
// Residual-accumulate epilogue in the MFMA register layout (fp32 C += (acc + bias) act * gamma,
// no other per-row operand: the ViT proj / fc2 with LayerScale, timm Block's x + ls(...)).  Each
// lane reads and writes its 4 consecutive fp32 columns of one row (16 B; a fragment pair covers a
// whole 128-B line of 16 rows), no LDS round trip, and the C loads of fragment row fm + 1 are in
// flight while row fm is computed and stored (straight-line code: the compiler counts the waits
// instead of draining every earlier store).  Same arithmetic, in the same order, as
// epilogue_rows -- no contraction of the gamma product into the residual add, which the general
// path's separate (runtime-conditional) steps do not get either: bit-identical results.
template <int ACT, int FM, int FN>
__device__ __forceinline__ void epilogue_acc32(const GemmP& p, f32x4_t (&acc)[FM][FN], int lane, int m_base,
                                               int n_base) {
  #pragma clang fp contract(off)
  const int t = lane & 15, g = lane >> 4;
  float bias[FN][4], gam[FN][4];
  #pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int n = n_base + fn * 16 + 4 * g;
    const bool ok = n < p.N;
    const float4 b = (p.bias && ok) ? *(const float4*)(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 q = (p.gamma && ok) ? *(const float4*)(p.gamma + n) : make_float4(1.f, 1.f, 1.f, 1.f);
    bias[fn][0] = b.x; bias[fn][1] = b.y; bias[fn][2] = b.z; bias[fn][3] = b.w;
    gam[fn][0] = q.x; gam[fn][1] = q.y; gam[fn][2] = q.z; gam[fn][3] = q.w;
  }
  float* const C = (float*)p.C;
  f32x4_t cur[FN], nxt[FN];
  auto load_row = [&](int fm, f32x4_t (&c)[FN]) __attribute__((always_inline)) {
    const int m = min(m_base + fm * 16 + t, p.M - 1);
    #pragma unroll
    for (int fn = 0; fn < FN; ++fn) c[fn] = *(const f32x4_t*)(C + (long long)m * p.ldc + n_base + fn * 16 + 4 * g);
  };
  load_row(0, cur);
  #pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    if (fm + 1 < FM) load_row(fm + 1, nxt);
    const int m = m_base + fm * 16 + t;
    #pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      f32x4_t x;
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[fm][fn][r] + bias[fn][r];
        if constexpr (ACT == DP_ACT_RELU) v = fmaxf(v, 0.f);
        else if constexpr (ACT == DP_ACT_GELU) v = gelu_erf(v);
        x[r] = v * gam[fn][r] + cur[fn][r];
      }
      if (m < p.M) *(f32x4_t*)(C + (long long)m * p.ldc + n_base + fn * 16 + 4 * g) = x;
    }
    #pragma unroll
    for (int fn = 0; fn < FN; ++fn) cur[fn] = nxt[fn];
  }
}

// epilogue_acc32 for wide wave tiles (FN = 8: the 8-phase 320 x 256 engine), where 8 columns'
// bias / gamma and two rows of C in flight would not fit beside the 160 accumulators: the
// wave's bias / gamma go through its LDS slab (ds_read per half row), and C is read and
// written in half rows (4 fragments = 64 columns), the next half row's loads in flight while
// one is computed.  Same arithmetic in the same order as epilogue_acc32: bit-identical.
template <int ACT, int FM, int FN>
__device__ __forceinline__ void epilogue_acc32_wide(const GemmP& p, f32x4_t (&acc)[FM][FN], char* slab, int lane,
                                                    int m_base, int n_base) {
  #pragma clang fp contract(off)
  static_assert(FN == 8, "wide epilogue");
  constexpr int H = FN / 2;
  const int t = lane & 15, g = lane >> 4;
  {
    // lanes 0-31: bias of columns 4 lane .. +3; lanes 32-63: gamma (1 and 0 when absent)
    const int c = 4 * (lane & 31), n = n_base + c;
    f32x4_t v;
    if (lane < 32) v = (p.bias && n < p.N) ? *(const f32x4_t*)(p.bias + n) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    else v = (p.gamma && n < p.N) ? *(const f32x4_t*)(p.gamma + n) : f32x4_t{1.f, 1.f, 1.f, 1.f};
    *(f32x4_t*)(slab + (lane < 32 ? 0 : 512) + c * 4) = v;
  }
  float* const C = (float*)p.C;
  f32x4_t cur[H], nxt[H];
  auto load = [&](int ch, f32x4_t (&c)[H]) __attribute__((always_inline)) {
    const int fm = ch >> 1, h = ch & 1;
    const int m = min(m_base + fm * 16 + t, p.M - 1);
    #pragma unroll
    for (int f = 0; f < H; ++f)
      c[f] = *(const f32x4_t*)(C + (long long)m * p.ldc + n_base + (h * H + f) * 16 + 4 * g);
  };
  load(0, cur);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slab writes, before any read of them
  #pragma unroll
  for (int ch = 0; ch < 2 * FM; ++ch) {
    if (ch + 1 < 2 * FM) load(ch + 1, nxt);
    const int fm = ch >> 1, h = ch & 1;
    const int m = m_base + fm * 16 + t;
    #pragma unroll
    for (int f = 0; f < H; ++f) {
      const int fn = h * H + f;
      const f32x4_t b = *(const f32x4_t*)(slab + (fn * 16 + 4 * g) * 4);
      const f32x4_t q = *(const f32x4_t*)(slab + 512 + (fn * 16 + 4 * g) * 4);
      f32x4_t x;
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[fm][fn][r] + b[r];
        if constexpr (ACT == DP_ACT_RELU) v = fmaxf(v, 0.f);
        else if constexpr (ACT == DP_ACT_GELU) v = gelu_erf(v);
        x[r] = v * q[r] + cur[f][r];
      }
      if (m < p.M) *(f32x4_t*)(C + (long long)m * p.ldc + n_base + fn * 16 + 4 * g) = x;
    }
    #pragma unroll
    for (int f = 0; f < H; ++f) cur[f] = nxt[f];
  }
}

// EACT of the engine variants: the compile-time epilogue.  -1: the general, runtime one;
// DP_ACT_*: epilogue_mfma (no per-row operand, 16-bit C); EPI_ACC + DP_ACT_*: epilogue_acc32
// (fp32 C accumulated into, no other per-row operand).
constexpr int EPI_ACC = 16;
__host__ inline int fast_epi_act(const GemmP& p) {
  if (p.dbg & (1 << 20)) return -1;
  if (!needs_rowld(p)) return p.c_dtype == DP_F32 ? -1 : p.act;
  const bool acc_only = p.accumulate && p.c_dtype == DP_F32 && !p.R1 && !p.R2 && !p.pos &&
                        p.store_mode == DP_STORE_ROWS && !p.row_group && !p.head_corr && !p.head_w;
  return acc_only ? EPI_ACC + p.act : -1;
}

// DP_STORE_HEAD_PS epilogue (depth head tail, depth_pro.py:182-207, composed at
// pack time): the GEMM ran the 3x3 conv of head.2 over the 2x-upsampled map as a
// 3x3 conv of the pre-upsampling map h0 whose N = 128 columns are (parity q =
// 2*dy + dx, channel o < 32).  Per output pixel (2y+dy, 2x+dx): z = acc + bias,
// minus the deconv-bias share of the taps that fall in head.2's zero padding
// (image border only), ReLU, dot with head.4's 32 weights, + bias, ReLU -> fp32.
// The 8 columns of a lane lie in one parity group; the 4 lanes of a row finish
// the 32-channel dot with two xor-shuffles.  Requires TN == 32 (one parity per wave).
template <int NIT>
__device__ __forceinline__ void head_ps_rows(const GemmP& p, const ColConst& cc, const int (&ms)[NIT], int n,
                                             float (&v)[NIT][8], int lane) {
  const int q = n >> 5, o0 = n & 31, dy = q >> 1, dx = q & 1;
  const int hw = p.out_h * p.out_w;
  float hw8[8];
  #pragma unroll
  for (int r = 0; r < 8; ++r) hw8[r] = p.head_w[o0 + r];
  #pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int m = ms[it] < p.M ? ms[it] : p.M - 1;
    const int b = m / hw, rr = m - b * hw;
    const int y = rr / p.out_w, x = rr - y * p.out_w;
    float z[8];
    #pragma unroll
    for (int r = 0; r < 8; ++r) z[r] = v[it][r] + cc.b[r];
    const bool top = y == 0 && dy == 0, bot = y == p.out_h - 1 && dy == 1;
    const bool lft = x == 0 && dx == 0, rgt = x == p.out_w - 1 && dx == 1;
    if (top || bot || lft || rgt) {
      #pragma unroll
      for (int a = 0; a < 3; ++a)
        #pragma unroll
        for (int c = 0; c < 3; ++c) {
          const bool oob = (a == 0 && top) || (a == 2 && bot) || (c == 0 && lft) || (c == 2 && rgt);
          if (oob) {
            #pragma unroll
            for (int r = 0; r < 8; ++r) z[r] -= p.head_corr[(a * 3 + c) * 32 + o0 + r];
          }
        }
    }
    float hs = 0.f;
    #pragma unroll
    for (int r = 0; r < 8; ++r) hs += fmaxf(z[r], 0.f) * hw8[r];
    hs += __shfl_xor(hs, 1);
    hs += __shfl_xor(hs, 2);
    if ((lane & 3) == 0 && ms[it] < p.M) {
      const long long W2 = 2LL * p.out_w;
      ((float*)p.C)[((long long)b * 2 * p.out_h + 2 * y + dy) * W2 + 2 * x + dx] = fmaxf(hs + p.head_b, 0.f);
    }
  }
}


// Tile order within the XCD-contiguous workgroup ranges.  Row-major (tile_n fastest)
// puts the 32 workgroups an XCD runs at once on ~2 rows of tiles x all columns;
// with BAND > 1 they sweep bands of BAND tile rows column by column instead, so the
// tiles in flight on one XCD form a squarer block (e.g. 4 x 8) that shares fewer
// distinct A / B panels in its 4 MiB L2: qkv 155 -> 150 us, fc1 197 -> 190 us
// (tools/gemm_bench.py --dbg 16 restores row-major, for A/B).
__device__ __forceinline__ void tile_coords(const GemmP& p, int wgid, int& tile_m, int& tile_n) {
  // debug 16: row-major; 1 << 18: bands of 8 rows; 1 << 19: bands of 2 rows (A/B)
  const int band = (p.dbg & 16) ? 1 : (p.dbg & (1 << 18)) ? 8 : (p.dbg & (1 << 19)) ? 2 : 4;
  const int tm_full = p.tiles_m / band * band;       // rows covered by whole bands
  const int per_band = band * p.tiles_n;
  if (band > 1 && wgid < tm_full * p.tiles_n) {
    const int b = wgid / per_band, r = wgid - b * per_band;
    tile_n = r / band;
    tile_m = b * band + (r - tile_n * band);
  } else {
    tile_n = wgid % p.tiles_n;
    tile_m = wgid / p.tiles_n;
  }
}

// implicit-conv row descriptor: output pixel m -> top-left input tap
struct ConvRow {
  int iy, ix, pix;
};
__device__ __forceinline__ ConvRow conv_row(const GemmP& p, int m) {
  ConvRow r;
  const bool ok = m < p.M;
  const int mc = ok ? m : p.M - 1;
  const int hw = p.out_h * p.out_w;
  const int b = mc / hw, rr = mc - b * hw;
  const int oy = rr / p.out_w, ox = rr - oy * p.out_w;
  r.iy = ok ? oy * p.stride - p.pad : -(1 << 28);
  r.ix = ox * p.stride - p.pad;
  r.pix = b * p.in_h * p.in_w;
  return r;
}
__device__ __forceinline__ const u16* conv_src(const GemmP& p, const ConvRow& r, int ky, int kx, int ci, bool& inb) {
  const int iy = r.iy + ky, ix = r.ix + kx;
  inb = (unsigned)iy < (unsigned)p.in_h && (unsigned)ix < (unsigned)p.in_w;
  const long long pix = (long long)r.pix + (long long)iy * p.in_w + ix;
  return p.A + pix * p.in_c + ci;
}

// Implicit-conv K order: k = ((cb * k_h + ky) * k_w + kx) * 64 + c -- the taps of one
// 64-channel block are consecutive K steps, so the shifted re-reads of the same input
// lines by neighbouring taps are one K step apart and hit in L2 (with the channel block
// innermost, the re-read came 4-36 steps later, after the XCD's 32 workgroups had
// streamed several MiB through the 4 MiB L2).  Weights are packed to match
// ([Cout][Cin/64][ky][kx][64], ops.conv_weight).  k0 % 32 == 0.
__device__ __forceinline__ void conv_tap(const GemmP& p, int k0, int& ky, int& kx, int& ci) {
  const int chunk = k0 >> 6, c = k0 & 63;
  const int taps = p.k_h * p.k_w;
  const int cb = chunk / taps, tap = chunk - cb * taps;
  ky = tap / p.k_w;
  kx = tap - ky * p.k_w;
  ci = cb * 64 + c;
}

// ============================================================ big-tile engine
constexpr int NT_BIG = 512;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// One 16-B-per-lane LDS-DMA piece (1 KiB per wave) written at the wave-uniform
// LDS byte address `lds_dst`.  Issued from inline asm so the compiler does not
// add its conservative `s_waitcnt vmcnt(0)` in front of every later ds_read:
// completion is tracked by hand with the counted waits below.
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_dst)
      : "memory");
}

// The same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset (saddr form):
// a K step's addresses are one scalar add away from the last step's, no per-lane 64-bit arithmetic.
__device__ __forceinline__ void glds16s(uint32_t voff, const void* sbase, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_dst)
      : "memory");
}

// The same through a buffer resource (4 SGPRs: base, num_records = bytes, raw): a lane whose byte
// offset is past the buffer's end reads zeros -- the implicit conv's zero padding without a second
// (zero page) address per lane.
__device__ __forceinline__ void glds16b(uint32_t voff, u32x4_t rsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds_dst)
      : "memory");
}
// Raw buffer resource of `bytes` bytes at p (stride 0): the SGPR words of glds16b's rsrc.
__device__ __forceinline__ u32x4_t raw_rsrc(const void* p, uint32_t bytes) {
  const unsigned long long a = (unsigned long long)(uintptr_t)p;
  u32x4_t r;
  r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000u;
  return r;
}

// LDS image of one operand tile: rows of BKT 16-bit elements (64 or 128 B), the
// 16-B chunk index XOR-swizzled so that the 16 rows one ds_read_b128 lane group
// reads hit 16 distinct bank slots (conflict-free, checked with SQ_LDS_BANK_CONFLICT).
template <int BKT>
__device__ __forceinline__ int lds_off_t(int row, int chunk) {
  if constexpr (BKT == 64) return row * 64 + ((chunk ^ (row & 7)) << 3);
  else return row * 32 + ((chunk ^ ((row >> 1) & 3)) << 3);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt_le(int n) {  // s_waitcnt vmcnt(n), n <= N, n a multiple of step
  if constexpr (N == 0) {
    wait_vmcnt<0>();
  } else {
    if (n >= N) wait_vmcnt<N>();
    else wait_vmcnt_le<N - 1>(n);
  }
}

// Folded-LN producer on a SPLIT residual stream (dp_gemm_args.ln_xl, LNM = 3 of the 8-phase
// 320 x 256 engine): the ViT residual x is held as hi (16 bits, = ln_xb_out, the next GEMM's A
// operand anyway) and an 8-bit low part (ln_xl: x - hi in steps of ulp(hi) / 256, lo8_encode):
// about 16 significant bits against fp32's 24 -- the patch encoder's rel-L1 vs the fp32 reference
// 2.3809e-3 against 2.3788e-3 with an fp32 stream (a 16-bit low part 2.3789e-3, bf16 hi alone
// 1.06e-2; tools/hilo_emul.py).  Per element: x' = (acc + b) * gamma + (hi + lo) (the fp32
// epilogue's operation order), hi' = r16(x'), lo' = lo8(x', hi'); (mean, M2) of each row's 128
// columns as epilogue_acc32_wide_ln (when ln_part_out); C (fp32) = x' when given (never read).
// 6 B of HBM per element instead of 10 (fp32 read + write, 16-bit hi write): the epilogue of a
// one-round launch (proj / fc2) is HBM-bound (10 -> 8 B with a 16-bit low part: proj 85 -> 75,
// fc2 172 -> 161 us, profiles/r05a_split_residual).
// The wave's 80 x 128 outputs go in NI = 10 chunks of 16 rows x 64 columns (fragment row fm,
// column half h), whose hi rows (2 KiB) and lo rows (1 KiB) arrive by LDS-DMA AHEAD chunks ahead
// into a 4-deep per-wave ring (the 16-B chunks XOR-swizzled by row on the source address: the
// MFMA-layout reads are conflict-free), are read in the MFMA layout, updated in place, read back as
// rows and leave as 128-B (hi) / 64-B (lo) row segments.  Every store is a buffer store whose masked
// lanes (rows past M, an absent output) carry an out-of-range offset, so each chunk issues a fixed
// number of VMEM instructions and the counted wait for a chunk's DMA is a compile-time constant.
// AHEAD = 3 and 1 measured the same in the frame (profiles/r05b_epilogue_dma_depth; 1 = debug 1 << 27).
// `slab`: the wave's LDS region, >= 13 KiB.
template <typename K_, int FM, int FN, int AHEAD = 3>
__device__ __forceinline__ void epilogue_hilo_ln(const GemmP& p, f32x4_t (&acc)[FM][FN], char* slab, int lane,
                                                 int m_base, int n_base) {
  #pragma clang fp contract(off)
  static_assert(FN == 8 && AHEAD >= 1 && AHEAD <= 3, "128 columns per wave, <= 4 ring slots");
  constexpr int NI = 2 * FM, CB = 3072, LO = 2048;   // chunks, ring slot bytes (hi | lo), lo offset
  constexpr int PCS = 3;                              // DMA pieces per chunk: hi 2, lo 1
  // the counted wait for chunk i's DMA: younger are the DMAs of chunks i+1 .. i+AHEAD and the
  // stores of the chunks processed since chunk i's DMA was issued (C 4, part (second half), hi 2, lo 1)
  constexpr auto younger = [](int i) constexpr {
    int n = PCS * ((i + AHEAD < NI - 1 ? i + AHEAD : NI - 1) - i);
    for (int j = (i - AHEAD > 0 ? i - AHEAD : 0); j < i; ++j) n += 4 + (j & 1) + 3;
    return n;
  };
  const int t = lane & 15, g = lane >> 4;
  {
    const int c = 4 * (lane & 31), n = n_base + c;
    f32x4_t v;
    if (lane < 32) v = (p.bias && n < p.N) ? *(const f32x4_t*)(p.bias + n) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    else v = (p.gamma && n < p.N) ? *(const f32x4_t*)(p.gamma + n) : f32x4_t{1.f, 1.f, 1.f, 1.f};
    *(f32x4_t*)(slab + (lane < 32 ? 0 : 512) + c * 4) = v;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // the constants, before any DMA is counted
  constexpr unsigned OOB = 0xFFFFFFF0u;   // a masked store's offset: past every extent (host: < 0xFFFFFF00)
  const u16* const hi_in = p.ln_xb_out;
  const unsigned char* const lo_in = (const unsigned char*)p.ln_xl;
  const unsigned row_b = (unsigned)(p.M * p.ldc * 2);              // bytes of hi (lo: half)
  const __amdgpu_buffer_rsrc_t rs_hi = __builtin_amdgcn_make_buffer_rsrc((void*)p.ln_xb_out, (short)0, (int)row_b, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_lo = __builtin_amdgcn_make_buffer_rsrc((void*)p.ln_xl, (short)0, (int)(row_b / 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_c = __builtin_amdgcn_make_buffer_rsrc(p.C ? p.C : (void*)p.ln_xl, (short)0,
                                                                        p.C ? (int)(2 * row_b) : 0, 0x00020000);
  const int nch = p.N / 128;
  const __amdgpu_buffer_rsrc_t rs_pt = __builtin_amdgcn_make_buffer_rsrc(
      p.ln_part_out ? (void*)p.ln_part_out : (void*)p.ln_xl, (short)0, p.ln_part_out ? (int)(p.M * nch * 8) : 0,
      0x00020000);
  const uint32_t slab_lds = __builtin_amdgcn_readfirstlane(lds_addr(slab)) + 1024;
  // chunk i = (fm, h): rows fm * 16 .. + 15, columns h * 64 .. + 63 of the wave's range; ring slot
  // i & 3.  hi: [16][128 B], piece pc = rows pc * 8 + lane / 8, 8 lanes x 16 B per row, physical 16-B
  // chunk lane & 7 = logical (lane & 7) ^ ((row >> 1) & 7).  lo: [16][64 B], one piece, 4 lanes x
  // 16 B per row (row lane / 4), physical chunk lane & 3 = logical (lane & 3) ^ ((row >> 2) & 3).
  auto dma = [&](int i) __attribute__((always_inline)) {
    const int fm = i >> 1, h = i & 1;
    #pragma unroll
    for (int pc = 0; pc < 2; ++pc) {
      const int r = pc * 8 + (lane >> 3);
      const int m = min(m_base + fm * 16 + r, p.M - 1);
      const long long o = (long long)m * p.ldc + n_base + h * 64 + (((lane & 7) ^ ((r >> 1) & 7)) << 3);
      glds16(hi_in + o, slab_lds + (i & 3) * CB + pc * 1024);
    }
    const int r = lane >> 2;
    const int m = min(m_base + fm * 16 + r, p.M - 1);
    glds16(lo_in + (long long)m * p.ldc + n_base + h * 64 + (((lane & 3) ^ ((r >> 2) & 3)) << 4),
           slab_lds + (i & 3) * CB + LO);
  };
  #pragma unroll
  for (int i = 0; i < AHEAD && i < NI; ++i) dma(i);
  float sh = 0.f, s1 = 0.f, s2 = 0.f;
  #pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int fm = i >> 1, h = i & 1;
    char* const buf = slab + 1024 + (i & 3) * CB;
    if (i + AHEAD < NI) dma(i + AHEAD);
    wait_vmcnt_le<48>(younger(i));   // a constant once the loop is unrolled
    const int m = m_base + fm * 16 + t;
    const bool mok = m < p.M;
    #pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int fn = h * 4 + f;
      const int off = t * 128 + (((f * 2 + (g >> 1)) ^ ((t >> 1) & 7)) << 4) + (g & 1) * 8;
      const int loff = LO + t * 64 + ((f ^ ((t >> 2) & 3)) << 4) + g * 4;
      const uint2 hv = *(const uint2*)(buf + off);
      const uint32_t lv = *(const uint32_t*)(buf + loff);
      const float hf[4] = {K_::to_f(hv.x & 0xffff), K_::to_f(hv.x >> 16), K_::to_f(hv.y & 0xffff), K_::to_f(hv.y >> 16)};
      const f32x4_t b = *(const f32x4_t*)(slab + (fn * 16 + 4 * g) * 4);
      const f32x4_t q = *(const f32x4_t*)(slab + 512 + (fn * 16 + 4 * g) * 4);
      f32x4_t x;
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[fm][fn][r] + b[r];
        x[r] = v * q[r] + lo8_decode<K_>(hf[r], unpack_i8(lv, r));
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, x), rs_c,
                                             mok ? (unsigned)(((long long)m * p.ldc + n_base + fn * 16 + 4 * g) * 4)
                                                 : OOB, 0, 0);
      if (fn == 0) {
        sh = __shfl(x[0], t);             // the row's value at column n_base (lane t, g = 0)
        s1 = 0.f;
        s2 = 0.f;
      }
      #pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = x[r] - sh;
        s1 += d;
        s2 += d * d;
      }
      uint2 wh;
      wh.x = K_::pack2(x[0], x[1]);
      wh.y = K_::pack2(x[2], x[3]);
      const uint32_t wl = pack_i8x4(lo8_encode<K_>(x[0], K_::to_f(wh.x & 0xffff)), lo8_encode<K_>(x[1], K_::to_f(wh.x >> 16)),
                                    lo8_encode<K_>(x[2], K_::to_f(wh.y & 0xffff)), lo8_encode<K_>(x[3], K_::to_f(wh.y >> 16)));
      *(uint2*)(buf + off) = wh;
      *(uint32_t*)(buf + loff) = wl;
    }
    if (h == 1) {
      // the row's 128 columns: 4 lanes (g) of 32 values each
      s1 += __shfl_xor(s1, 16);
      s2 += __shfl_xor(s2, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      const float mc = sh + s1 * (1.f / 128);
      const float m2 = s2 - s1 * (s1 * (1.f / 128));
      const unsigned po = (g == 0 && mok) ? (unsigned)(((long long)m * nch + n_base / 128) * 8) : OOB;
      // sc1 (write-through): another workgroup of the row tile may merge it (ln_merge_last)
      __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{__float_as_uint(mc), __float_as_uint(m2)}, rs_pt, po, 0, 16);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's staging writes
    #pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = k * 8 + (lane >> 3), chunk = lane & 7;
      const int o = row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
      const uint4 dh = *(const uint4*)(buf + o);
      const int mm = m_base + fm * 16 + row;
      const unsigned bo = mm < p.M ? (unsigned)(((long long)mm * p.ldc + n_base + h * 64 + chunk * 8) * 2) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{dh.x, dh.y, dh.z, dh.w}, rs_hi, bo, 0, 0);
    }
    {
      const int row = lane >> 2, chunk = lane & 3;
      const uint4 dl = *(const uint4*)(buf + LO + row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4));
      const int mm = m_base + fm * 16 + row;
      const unsigned bo = mm < p.M ? (unsigned)((long long)mm * p.ldc + n_base + h * 64 + chunk * 16) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{dl.x, dl.y, dl.z, dl.w}, rs_lo, bo, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // read back before this slot's next DMA
  }
}


// NW = waves per workgroup: 8 (one workgroup per CU), or 4 (two workgroups per CU, each
// wave one per SIMD: one workgroup's epilogue runs beside the other's K loop).
// EACT: -1 = the general epilogue (runtime operand set); DP_ACT_* = the load-free MFMA-layout
// epilogue with that activation (epilogue_mfma; fast_epi_act decides on the host).
// GRP: a dp_gemm_grouped launch -- the workgroup's problem (wgid / tiles per problem) supplies the
// operand pointers.
template <typename K_, int BM, int BN, int BKT, int NS, bool PIPE, bool CONV, bool RELU, int NW = 8, int EACT = -1,
          bool GRP = false, bool SPLIT = false>
__global__ void __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) gemm_big_kernel(const GemmP p_arg) {
  // 8 waves as WM x WN; the 512 x 128 tile (N = 128 layers) uses 4 x 2 so that every
  // wave still owns a 128 x 64 sub-tile (same fragment reuse as the 256 x 256 tile);
  // 4 waves as 2 x 2 (256 x 128: 128 x 64 per wave)
  constexpr int WN = NW == 4 ? 2 : (BM == 512 ? 2 : 4), WM = NW / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int RB = BKT * 2;                 // LDS row bytes
  constexpr int CR = BKT / 8;                 // 16-B chunks per row
  constexpr int ROWS_PER_WAVE_PIECE = 1024 / RB;
  constexpr int ROWS_PER_ROUND = NW * ROWS_PER_WAVE_PIECE;  // rows covered by one piece of every wave
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int LA = BM / ROWS_PER_ROUND;     // LDS-DMA pieces per thread per A tile
  constexpr int LB = BN / ROWS_PER_ROUND;
  constexpr int LT = LA + LB;
  constexpr int EPI_BYTES = NW * 32 * (TN + 4) * 4;  // epilogue staging (NW waves x 32 fp32 rows)
  constexpr int SMEM = NS * STAGE > EPI_BYTES ? NS * STAGE : EPI_BYTES;
  static_assert(NS >= 2 && SMEM <= 160 * 1024 && LB >= 1, "LDS ring");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap (blocks b and b+8 share an XCD under round-robin dispatch)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  GemmP p_grp;
  if constexpr (GRP) {
    const int per = p_arg.tiles_m * p_arg.tiles_n;
    const int g = wgid / per;
    wgid -= g * per;
    p_grp = p_arg;
    const GemmP::Group& q = p_arg.grp[g];
    p_grp.A = q.A; p_grp.B = q.B; p_grp.bias = q.bias; p_grp.gamma = q.gamma; p_grp.pos = q.pos;
    p_grp.R1 = q.R1; p_grp.R2 = q.R2; p_grp.C = q.C;
  }
  // split-K: this workgroup's K-step range and its fp32 partial slab as a plain C (no epilogue
  // operands: the reduce launch applies them to the sum)
  int kbeg = 0, kcnt = p_arg.K / BKT;
  if constexpr (SPLIT) {
    const int per = p_arg.tiles_m * p_arg.tiles_n;
    const int sp = wgid / per;
    wgid -= sp * per;
    const int kt_all = p_arg.K / BKT;
    kbeg = sp * kt_all / p_arg.ksplit;
    kcnt = (sp + 1) * kt_all / p_arg.ksplit - kbeg;
    p_grp = p_arg;
    p_grp.C = p_arg.kpart + (long long)sp * p_arg.M * p_arg.N;
    p_grp.ldc = p_arg.N; p_grp.c_dtype = DP_F32; p_grp.accumulate = 0; p_grp.store_mode = DP_STORE_ROWS;
    p_grp.bias = nullptr; p_grp.gamma = nullptr; p_grp.pos = nullptr; p_grp.R1 = nullptr; p_grp.R2 = nullptr;
    p_grp.act = DP_ACT_NONE; p_grp.row_group = 0; p_grp.head_w = nullptr; p_grp.head_corr = nullptr;
  }
  const GemmP& p = (GRP || SPLIT) ? p_grp : p_arg;
  int tile_m, tile_n;
  tile_coords(p, wgid, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  DP_STAMPS_DECL;
  DP_STAMP(st0_);

  // LDS-DMA piece i of this thread covers tile row i*ROWS_PER_ROUND + wave*ROWS_PER_WAVE_PIECE + lane/CR;
  // LDS slot lane%CR of that row holds logical chunk (lane%CR) ^ swz(row): the swizzle is
  // applied on the SOURCE address, the LDS image stays lane-linear.
  const int prow = wave * ROWS_PER_WAVE_PIECE + lane / CR;
  const int pchunk = BKT == 64 ? ((lane & 7) ^ ((lane >> 3) & 7)) : ((lane & 3) ^ ((lane >> 3) & 3));
  const u16* a_src[LA];
  ConvRow a_cr[LA];
  #pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int m = m0 + i * ROWS_PER_ROUND + prow;
    if constexpr (CONV) {
      a_cr[i] = conv_row(p, m);
    } else {
      a_src[i] = p.A + (long long)(m < p.M ? m : p.M - 1) * p.lda + pchunk * 8;
    }
  }
  const u16* b_src[LB];
  #pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int n = n0 + i * ROWS_PER_ROUND + prow;
    b_src[i] = p.B + (long long)(n < p.N ? n : p.N - 1) * p.ldb + pchunk * 8;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem)) + wave_u * 1024;
  auto issue = [&](int kt, int stage) {
    const uint32_t sa = lds_base + stage * STAGE;
    const uint32_t sb = sa + A_BYTES;
    const int k0 = (kt + kbeg) * BKT;
    int t_ky = 0, t_kx = 0, t_ci = 0;
    if constexpr (CONV) conv_tap(p, k0, t_ky, t_kx, t_ci);
    #pragma unroll
    for (int i = 0; i < LA; ++i) {
      const void* src;
      if constexpr (CONV) {
        bool inb;
        const u16* s = conv_src(p, a_cr[i], t_ky, t_kx, t_ci + pchunk * 8, inb);
        src = inb ? (const void*)s : (const void*)g_zero_page;
      } else {
        src = a_src[i] + k0;
      }
      glds16(src, sa + i * NW * 1024);
    }
    #pragma unroll
    for (int i = 0; i < LB; ++i) glds16(b_src[i] + k0, sb + i * NW * 1024);
  };

  f32x4_t acc[FM][FN];
  #pragma unroll
  for (int i = 0; i < FM; ++i)
    #pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // (measured and rejected, round 2: static priority 1 for waves 4-7 instead of the raise / drop
  // around every MFMA group, profiles/r02q_prio_band/)

  const int frow = lane & 15, fchunk = lane >> 4;
  constexpr int KS = BKT / 32;
  auto compute = [&](int stage) {
    const u16* sa = (const u16*)(smem + stage * STAGE);
    const u16* sb = (const u16*)(smem + stage * STAGE + A_BYTES);
    #pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 bf[FN];
      #pragma unroll
      for (int j = 0; j < FN; ++j)
        bf[j] = *(const uint4*)(sb + lds_off_t<BKT>(wn * TN + j * 16 + frow, ks * 4 + fchunk));
      // all FM A fragments of the sub-step are read up front: the MFMAs then wait
      // on lgkmcnt(FM-1 .. 0) instead of one read at a time (fc1 191 -> 182 us,
      // 768^2 conv 675 -> 650 us on the 320x256 / 256x256 engines, same VGPR count)
      uint4 afs[FM];
      #pragma unroll
      for (int i = 0; i < FM; ++i) afs[i] = *(const uint4*)(sa + lds_off_t<BKT>(wm * TM + i * 16 + frow, ks * 4 + fchunk));
      __builtin_amdgcn_s_setprio(1);
      #pragma unroll
      for (int i = 0; i < FM; ++i) {
        uint4 af = afs[i];
        if constexpr (RELU) af = relu_pk16(af);
        #pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = K_::mfma16(bf[j], af, acc[i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
    }
  };

  const int KT = kcnt;
  auto nxt = [&](int st) { return st + 1 == NS ? 0 : st + 1; };
  // wait until tile t has landed: tiles issued so far are 0 .. min(KT-1, t+NS-2)
  auto wait_tile = [&](int t) { wait_vmcnt_le<(NS - 2) * LT>(min(NS - 2, KT - 1 - t) * LT); };
  if constexpr (!PIPE) {
    // NS-stage ring, one barrier per K step.  Top of iteration kt: tiles kt ..
    // kt+NS-2 are in flight; wait for tile kt only (counted vmcnt), then the
    // barrier makes it visible to every wave AND certifies that every wave
    // finished compute(kt-1), whose stage is refilled with tile kt+NS-1 right
    // away -- NS-1 steps of MFMA work cover each load.
    #pragma unroll
    for (int t = 0; t < NS - 1; ++t)
      if (t < KT) issue(t, t);
    int stage = 0;
    for (int kt = 0; kt < KT; ++kt) {
      wait_tile(kt);
      lds_barrier();
#ifdef DP_STAMPS
      if (kt == 0) DP_STAMP(st1_);
#endif
      if (kt + NS - 1 < KT && !(p.dbg & 2)) {
        const int st = stage + NS - 1;
        issue(kt + NS - 1, st >= NS ? st - NS : st);
      }
      if (p.dbg & 4) {
        const u16* sa = (const u16*)(smem + stage * STAGE);
        uint4 t = *(const uint4*)(sa + lds_off_t<BKT>(wm * TM + frow, fchunk));
        asm volatile("" ::"v"(t.x));
      } else {
        compute(stage);
      }
      stage = nxt(stage);
    }
  } else {
    // NS >= 3: software-pipelined.  The fragments of the next k sub-step (or of
    // the next K step's first sub-step, once its tile is visible) are read from
    // LDS while the MFMAs of the current sub-step run, alternating between two
    // register sets; one barrier per K step, NS-2 steps of loads in flight.
    uint4 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
    auto rd = [&](uint4 (&fa)[FM], uint4 (&fb)[FN], int stg, int ks) {
      const u16* sa = (const u16*)(smem + stg * STAGE);
      const u16* sb = (const u16*)(smem + stg * STAGE + A_BYTES);
      #pragma unroll
      for (int j = 0; j < FN; ++j)
        fb[j] = *(const uint4*)(sb + lds_off_t<BKT>(wn * TN + j * 16 + frow, ks * 4 + fchunk));
      #pragma unroll
      for (int i = 0; i < FM; ++i)
        fa[i] = *(const uint4*)(sa + lds_off_t<BKT>(wm * TM + i * 16 + frow, ks * 4 + fchunk));
    };
    auto mma = [&](const uint4 (&fa)[FM], const uint4 (&fb)[FN]) {
      __builtin_amdgcn_s_setprio(1);
      #pragma unroll
      for (int i = 0; i < FM; ++i) {
        uint4 a = fa[i];
        if constexpr (RELU) a = relu_pk16(a);
        #pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = K_::mfma16(fb[j], a, acc[i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
    };
    #pragma unroll
    for (int t = 0; t < NS - 1; ++t)
      if (t < KT) issue(t, t);
    wait_tile(0);
    lds_barrier();
    DP_STAMP(st1_);
    rd(fa0, fb0, 0, 0);
    int stage = 0;
    if constexpr (KS == 2) {
      for (int kt = 0; kt < KT; ++kt) {
        if (kt + NS - 1 < KT) {
          int st = stage + NS - 1;
          issue(kt + NS - 1, st >= NS ? st - NS : st);
        }
        rd(fa1, fb1, stage, 1);
        mma(fa0, fb0);
        const int nst = nxt(stage);
        if (kt + 1 < KT) {
          wait_tile(kt + 1);
          lds_barrier();
          rd(fa0, fb0, nst, 0);
        }
        mma(fa1, fb1);
        stage = nst;
      }
    } else {
      for (int kt = 0; kt < KT; kt += 2) {
        if (kt + NS - 1 < KT) {
          int st = stage + NS - 1;
          issue(kt + NS - 1, st >= NS ? st - NS : st);
        }
        int nst = nxt(stage);
        if (kt + 1 < KT) {
          wait_tile(kt + 1);
          lds_barrier();
          rd(fa1, fb1, nst, 0);
        }
        mma(fa0, fb0);
        stage = nst;
        if (kt + 1 >= KT) break;
        if (kt + NS < KT) {
          int st = stage + NS - 1;
          issue(kt + NS, st >= NS ? st - NS : st);
        }
        nst = nxt(stage);
        if (kt + 2 < KT) {
          wait_tile(kt + 2);
          lds_barrier();
          rd(fa0, fb0, nst, 0);
        }
        mma(fa1, fb1);
        stage = nst;
      }
    }
  }

  DP_STAMP(st2_);
  if (p.dbg & 1) {
    #pragma unroll
    for (int i = 0; i < FM; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j][0]), "v"(acc[i][j][1]), "v"(acc[i][j][2]), "v"(acc[i][j][3]));
    return;
  }
  if constexpr (EACT >= EPI_ACC) {
    epilogue_acc32<EACT - EPI_ACC, FM, FN>(p, acc, lane, m0 + wm * TM, n0 + wn * TN);
    return;
  } else if constexpr (EACT >= 0) {
    lds_barrier();  // the ring is free once every wave has left the K loop
    constexpr int PF = (FM * 16 * TN * 2 * NW <= SMEM) ? FM : FM / 2;
    epilogue_mfma<K_, EACT, FM, FN, TN, PF>(p, acc, smem + wave * (PF * 16 * TN * 2), lane, m0 + wm * TM,
                                            n0 + wn * TN);
    return;
  }
  // Epilogue through LDS: the MFMA layout gives each lane 4 columns of one row
  // (16 rows x 32-64 B per store instruction -- partial cache lines, measured at
  // ~half of the kernel's time on the ViT shapes).  Each wave instead parks 32
  // rows of its fp32 tile in a private LDS slab and reads them back row-major,
  // so every lane owns 8 consecutive columns and a store instruction writes
  // whole 128-256 B row segments.
  lds_barrier();  // the ring is free once every wave has left the K loop
  constexpr int SROW = TN + 4;                // fp32 row stride (bank-conflict-free writes)
  constexpr int CPR = TN / 8;                 // 8-column chunks per row
  constexpr int RPI = 64 / CPR;               // rows per read instruction
  float* stg = (float*)smem + wave * (32 * SROW);
  constexpr int NIT = 32 / RPI;
  const int c8 = (lane % CPR) * 8, n_l = n0 + wn * TN + c8;
  ColConst cc;
  load_colconst(p, n_l, cc);
  #pragma unroll
  for (int q = 0; q < FM / 2; ++q) {          // 32 rows (two 16-row fragments) per pass
    #pragma unroll
    for (int i = 0; i < 2; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j)
        *(f32x4_t*)(stg + (i * 16 + (lane & 15)) * SROW + j * 16 + 4 * (lane >> 4)) = acc[2 * q + i][j];
    // rows of per-row operands batched per epilogue call: all of a pass's rows, except
    // for the 128-160-row wave tiles whose accumulators leave room for only 2 at a time
    constexpr int NITC = FM >= 8 && NIT > 2 ? 2 : NIT;
    #pragma unroll
    for (int c0 = 0; c0 < NIT; c0 += NITC) {
      float v[NITC][8];
      int ms[NITC];
      #pragma unroll
      for (int it = 0; it < NITC; ++it) {
        const int row = (c0 + it) * RPI + lane / CPR;
        const f32x4_t lo = *(const f32x4_t*)(stg + row * SROW + c8);
        const f32x4_t hi = *(const f32x4_t*)(stg + row * SROW + c8 + 4);
        #pragma unroll
        for (int r = 0; r < 4; ++r) { v[it][r] = lo[r]; v[it][4 + r] = hi[r]; }
        ms[it] = m0 + wm * TM + q * 32 + row;
      }
      if constexpr (TN % 32 == 0) {
        if (p.store_mode == DP_STORE_HEAD_PS) {
          head_ps_rows<NITC>(p, cc, ms, n_l, v, lane);
          continue;
        }
      }
      epilogue_rows<K_, NITC, CONV && BM == 512 && !RELU>(p, cc, ms, n_l, v);
    }
  }
  DP_STAMP(st3_);
  DP_STAMP_SAVE(wgid);
}


// ============================================== persistent data-parallel big engine
// gemm_big_kernel's K loop (2-stage ring, one barrier per K step, all A fragments of a
// sub-step read up front) inside a tile loop: min(tiles, CUs) workgroups walk tiles
// wgid, wgid + G, ...  At the last K step of a tile the FIRST K step of the next tile is
// issued into the stage just freed, so its LDS-DMA runs under the epilogue; the epilogue
// stages through the stage it just computed from and writes C with buffer stores that
// every lane issues (rows past M get an out-of-range offset: dropped by the hardware),
// so the next tile's first wait can be a COUNTED vmcnt that lets this tile's stores
// drain under its K loop instead of a per-round dispatch + prologue + store drain.
// Store modes: rows (incl. row-group remap), no fused head.
// ROWLD: the epilogue reads per-row operands (residuals, pos, the fp32 C being accumulated
// into); without them it needs fewer VGPRs (the 320 x 256 tile is at the 256 limit).
//
template <typename K_, int BM, int BN, bool CONV, bool RELU, bool ROWLD>
__global__ void __launch_bounds__(NT_BIG, 1) gemm_pbig_kernel(const GemmP p) {
  constexpr int BKT = 64, WN = 4, WM = 2;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int LA = BM / 64, LB = BN / 64;
  constexpr int SROW = TN + 4;                                   // fp32 staging row stride
  constexpr int PR = 8 * 32 * SROW * 4 <= STAGE ? 32 : 16;       // staged rows per pass per wave
  constexpr int CPR = TN / 8, RPI = 64 / CPR, NIT = PR / RPI;
  constexpr int STORES = (FM * 16 / PR) * NIT;                   // 16-B stores per lane per tile (16-bit C)
  static_assert(8 * PR * SROW * 4 <= STAGE && FM % (PR / 16) == 0 && NIT % 2 == 0, "staging");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave / WN, wn = wave % WN;
  const int G = gridDim.x, bid = blockIdx.x;
  const int T = p.tiles_m * p.tiles_n;
  // static walk: this workgroup's tiles are wgid, wgid + G, ...: at any moment the
  // workgroups of one XCD (consecutive wgids) work on consecutive tiles of the band
  // raster, as the rounds of the data-parallel launch do (shared A / B panels in that
  // XCD's L2)
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  if (wgid >= T) return;
  const int t_begin = wgid;

  const int prow = wave * 8 + (lane >> 3);
  const int pchunk = (lane & 7) ^ ((lane >> 3) & 7);
  // 32-bit element offsets from the (uniform) A / B bases instead of 64-bit pointers: they
  // stay live through the epilogue (the next tile's loads are in flight), so they are kept
  // small (the host guarantees M * lda and N * ldb < 2^31)
  int a_off[LA];
  ConvRow a_cr[LA];
  int b_off[LB];
  auto setup = [&](int m0, int n0) {
    #pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int m = m0 + i * 64 + prow;
      if constexpr (CONV) a_cr[i] = conv_row(p, m);
      else a_off[i] = (m < p.M ? m : p.M - 1) * (int)p.lda + pchunk * 8;
    }
    #pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int n = n0 + i * 64 + prow;
      b_off[i] = (n < p.N ? n : p.N - 1) * (int)p.ldb + pchunk * 8;
    }
  };
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem)) + wave_u * 1024;
  auto issue = [&](int kt, int stage) {
    const uint32_t sa = lds_base + stage * STAGE;
    const uint32_t sb = sa + A_BYTES;
    const int k0 = kt * BKT;
    int t_ky = 0, t_kx = 0, t_ci = 0;
    if constexpr (CONV) conv_tap(p, k0, t_ky, t_kx, t_ci);
    #pragma unroll
    for (int i = 0; i < LA; ++i) {
      const void* src;
      if constexpr (CONV) {
        bool inb;
        const u16* s = conv_src(p, a_cr[i], t_ky, t_kx, t_ci + pchunk * 8, inb);
        src = inb ? (const void*)s : (const void*)g_zero_page;
      } else {
        src = p.A + (a_off[i] + k0);
      }
      glds16(src, sa + i * 8192);
    }
    #pragma unroll
    for (int i = 0; i < LB; ++i) glds16(p.B + (b_off[i] + k0), sb + i * 8192);
  };

  f32x4_t acc[FM][FN];
  const int frow = lane & 15, fchunk = lane >> 4;
  auto compute = [&](int stage) {
    const u16* sa = (const u16*)(smem + stage * STAGE);
    const u16* sb = (const u16*)(smem + stage * STAGE + A_BYTES);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 bf[FN];
      #pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = *(const uint4*)(sb + lds_off_t<BKT>(wn * TN + j * 16 + frow, ks * 4 + fchunk));
      // A fragments read up front in groups of FA (all FM for the 256-row tile; two halves
      // for the 320-row tile, whose persistent state leaves no room for ten)
      constexpr int FA = FM > 8 ? FM / 2 : FM;
      #pragma unroll
      for (int i0 = 0; i0 < FM; i0 += FA) {
        uint4 afs[FA];
        #pragma unroll
        for (int i = 0; i < FA; ++i)
          afs[i] = *(const uint4*)(sa + lds_off_t<BKT>(wm * TM + (i0 + i) * 16 + frow, ks * 4 + fchunk));
        __builtin_amdgcn_s_setprio(1);
        #pragma unroll
        for (int i = 0; i < FA; ++i) {
          uint4 af = afs[i];
          if constexpr (RELU) af = relu_pk16(af);
          #pragma unroll
          for (int j = 0; j < FN; ++j) acc[i0 + i][j] = K_::mfma16(bf[j], af, acc[i0 + i][j]);
        }
        __builtin_amdgcn_s_setprio(0);
      }
    }
  };

  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, (int)p.c_bytes, 0x00020000);
  const int esz = p.c_dtype == DP_F32 ? 4 : 2;
  const int KT = p.K / BKT;
  int tm, tn;
  tile_coords(p, t_begin, tm, tn);
  int m0 = tm * BM, n0 = tn * BN;
  setup(m0, n0);
  issue(0, 0);
  int stage = 0;
  for (int t = t_begin, first = 1;; first = 0) {
    #pragma unroll
    for (int i = 0; i < FM; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    int t_next = t + G < T ? t + G : -1;
    int m0n = 0, n0n = 0;
    for (int kt = 0; kt < KT; ++kt) {
      // step 0 of a later tile: only its own DMA (issued before the previous epilogue's
      // STORES stores) has to have landed; the stores may still be draining
      if (kt == 0 && !first) wait_vmcnt<STORES>();
      else wait_vmcnt<0>();
      lds_barrier();
      if (kt + 1 < KT) {
        issue(kt + 1, stage ^ 1);
      } else {
        if (t_next >= 0) {
          tile_coords(p, t_next, tm, tn);
          m0n = tm * BM;
          n0n = tn * BN;
          setup(m0n, n0n);
          issue(0, stage ^ 1);
        }
      }
      compute(stage);
      stage ^= 1;
    }
    // epilogue of tile t, staged through the stage just computed from (stage ^ 1)
    lds_barrier();
    float* stg = (float*)(smem + (stage ^ 1) * STAGE) + wave * (PR * SROW);
    const int c8 = (lane % CPR) * 8, n_l = n0 + wn * TN + c8;
    ColConst cc;
    load_colconst(p, n_l, cc);
    #pragma unroll
    for (int q = 0; q < FM * 16 / PR; ++q) {
      #pragma unroll
      for (int i = 0; i < PR / 16; ++i)
        #pragma unroll
        for (int j = 0; j < FN; ++j)
          *(f32x4_t*)(stg + (i * 16 + (lane & 15)) * SROW + j * 16 + 4 * (lane >> 4)) = acc[q * (PR / 16) + i][j];
      #pragma unroll
      for (int c0 = 0; c0 < NIT; c0 += 2) {
        float v[2][8];
        int ms[2];
        #pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int row = (c0 + it) * RPI + lane / CPR;
          const f32x4_t lo = *(const f32x4_t*)(stg + row * SROW + c8);
          const f32x4_t hi = *(const f32x4_t*)(stg + row * SROW + c8 + 4);
          #pragma unroll
          for (int r = 0; r < 4; ++r) { v[it][r] = lo[r]; v[it][4 + r] = hi[r]; }
          ms[it] = m0 + wm * TM + q * PR + row;
        }
        if constexpr (ROWLD) {
          epilogue_rows_buf<K_, 2>(p, cc, ms, n_l, v, crs, esz);
        } else {
          GemmP q = p;
          q.R1 = nullptr; q.R2 = nullptr; q.pos = nullptr; q.accumulate = 0;
          epilogue_rows_buf<K_, 2>(q, cc, ms, n_l, v, crs, esz);
        }
      }
      // the next pass rewrites this wave's slab: its reads of this pass are done first
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (t_next < 0) break;
    t = t_next;
    m0 = m0n;
    n0 = n0n;
  }
}

// ======================================================= 8-phase 256x256 engine
// 256 x 256 x 64 tile, 8 waves (2 x 4, wave tile 128 x 64), K loop cut into 4
// phases per K tile -- one 64 x 32 C quadrant x K 64 = 16 MFMAs per wave per
// phase -- each phase {fragment ds_reads, ONE half-tile LDS-DMA prefetch,
// s_barrier, lgkmcnt(0), 16 MFMAs at raised priority, s_barrier}.  The LDS
// holds 2 K tiles as 4 half-tiles each (A rows 0-127 / 128-255, B cols
// 0-127 / 128-255, 16 KiB each); a half is refilled one phase after its last
// read, so global loads stream continuously with up to 3 half-tiles in flight
// and the only vmcnt wait is once per K tile (counted, never a drain while
// tiles remain).  Quadrant order (qm,qn): (0,0) (0,1) (1,0) (1,1); reads:
// p0 A(qm0)+B(qn0), p1 B(qn1), p2 A(qm1), p3 none.  Issue order of tile
// t+1 / t+2 halves: p0 A0(t+1), p1 A1(t+1), p2 B0(t+2), p3 B1(t+2).
template <typename K_, bool CONV, bool RELU, int EACT = -1>
__global__ void __launch_bounds__(512, 1) gemm_8ph_kernel(const GemmP p) {
  constexpr int HALF = 128 * 128;   // bytes: 128 rows x 64 16-bit
  constexpr int TILEB = 4 * HALF;   // A0 A1 B0 B1
  constexpr int TN = 64, TM = 128;
  constexpr int EPI_BYTES = 8 * 32 * (TN + 4) * 4;
  constexpr int SMEM = 2 * TILEB > EPI_BYTES ? 2 * TILEB : EPI_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tile_m, tile_n;
  tile_coords(p, wgid, tile_m, tile_n);
  const int m0 = tile_m * 256, n0 = tile_n * 256;

  // LDS-DMA pieces: half-tile row r = i*64 + wave*8 + lane/8 (i = 0,1), swizzle on the source
  const int prow = wave * 8 + (lane >> 3);
  const int pchunk = (lane & 7) ^ ((lane >> 3) & 7);
  const u16* a_src[2][2];
  ConvRow a_cr[2][2];
  const u16* b_src[2][2];
  #pragma unroll
  for (int h = 0; h < 2; ++h)
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + 128 * h + i * 64 + prow;
      if constexpr (CONV) a_cr[h][i] = conv_row(p, m);
      else a_src[h][i] = p.A + (long long)(m < p.M ? m : p.M - 1) * p.lda + pchunk * 8;
      const int n = n0 + 128 * h + i * 64 + prow;
      b_src[h][i] = p.B + (long long)(n < p.N ? n : p.N - 1) * p.ldb + pchunk * 8;
    }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem)) + wave_u * 1024;
  auto issueA = [&](int h, int t) {  // A half h of K tile t -> buffer t&1
    const uint32_t dst = lds_base + (t & 1) * TILEB + h * HALF;
    int ci = 0, ky = 0, kx = 0;
    if constexpr (CONV) {
      conv_tap(p, t * 64, ky, kx, ci);
    }
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
      const void* src;
      if constexpr (CONV) {
        bool inb;
        const u16* s = conv_src(p, a_cr[h][i], ky, kx, ci + pchunk * 8, inb);
        src = inb ? (const void*)s : (const void*)g_zero_page;
      } else {
        src = a_src[h][i] + t * 64;
      }
      glds16(src, dst + i * 8192);
    }
  };
  auto issueB = [&](int h, int t) {
    const uint32_t dst = lds_base + (t & 1) * TILEB + (2 + h) * HALF;
    #pragma unroll
    for (int i = 0; i < 2; ++i) glds16(b_src[h][i] + t * 64, dst + i * 8192);
  };

  f32x4_t acc[8][4];
  #pragma unroll
  for (int i = 0; i < 8; ++i)
    #pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15, fchunk = lane >> 4;
  uint4 af[2][4], bf[2][2][2];
  auto readA = [&](int qm, int buf) {
    const u16* sa = (const u16*)(smem + buf * TILEB + wm * HALF);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fm = 0; fm < 4; ++fm)
        af[ks][fm] = *(const uint4*)(sa + lds_off(qm * 64 + fm * 16 + frow, ks * 4 + fchunk));
  };
  auto readB = [&](int qn, int buf) {
    const u16* sb = (const u16*)(smem + buf * TILEB + (2 + (wn >> 1)) * HALF);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fn = 0; fn < 2; ++fn)
        bf[qn][ks][fn] = *(const uint4*)(sb + lds_off((wn & 1) * 64 + qn * 32 + fn * 16 + frow, ks * 4 + fchunk));
  };
  auto mma = [&](int qm, int qn) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fm = 0; fm < 4; ++fm) {
        uint4 a = af[ks][fm];
        if constexpr (RELU) a = relu_pk16(a);
        #pragma unroll
        for (int fn = 0; fn < 2; ++fn)
          acc[qm * 4 + fm][qn * 2 + fn] = K_::mfma16(bf[qn][ks][fn], a, acc[qm * 4 + fm][qn * 2 + fn]);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() { asm volatile("s_barrier" ::: "memory"); };

  const int KT = p.K / 64;
  issueA(0, 0); issueA(1, 0); issueB(0, 0); issueB(1, 0);
  if (KT > 1) {
    issueB(0, 1); issueB(1, 1);
    wait_vmcnt<4>();
  } else {
    wait_vmcnt<0>();
  }
  lds_barrier();
  // Wave rows run staggered by one barrier: while one wave of a SIMD waits on
  // its fragment reads the other issues MFMAs.  Every LDS-DMA wait therefore
  // sits one phase before the first read of what it retires (phase 3 for the
  // next K tile, read from phase 0 on), so both wave groups have passed their
  // wait before either reads.
  if (wm == 1) bar();
  for (int t = 0; t < KT; ++t) {
    const int buf = t & 1;
    const bool n1 = t + 1 < KT, n2 = t + 2 < KT;
    // phase 0: quadrant (0,0)
    readA(0, buf); readB(0, buf);
    if (n1) issueA(0, t + 1);
    bar(); mma(0, 0); bar();
    // phase 1: quadrant (0,1)
    readB(1, buf);
    if (n1) issueA(1, t + 1);
    bar(); mma(0, 1); bar();
    // phase 2: quadrant (1,0)
    readA(1, buf);
    if (n2) issueB(0, t + 2);
    bar(); mma(1, 0); bar();
    // phase 3: quadrant (1,1); tile t+1 must have landed before this phase's first barrier
    if (n2) wait_vmcnt<2>(); else wait_vmcnt<0>();
    if (n2) issueB(1, t + 2);
    bar(); mma(1, 1);
    bar();
  }
  if (wm == 0) bar();
  if (p.dbg & 1) {   // ablation (tools/gemm_bench.py --ablate): no epilogue
    #pragma unroll
    for (int i = 0; i < 8; ++i)
      #pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j][0]), "v"(acc[i][j][1]), "v"(acc[i][j][2]), "v"(acc[i][j][3]));
    return;
  }

  if constexpr (EACT >= 0) {
    lds_barrier();   // the ring (128 KiB) is free: a 16 KiB slab per wave holds its whole 128 x 64 tile
    epilogue_mfma<K_, EACT, 8, 4, 64, 8>(p, acc, smem + wave * 16384, lane, m0 + wm * TM, n0 + wn * TN);
    return;
  }
  // epilogue: identical to the big engine (LDS-staged, row-coalesced)
  lds_barrier();
  constexpr int SROW = TN + 4, CPR = TN / 8, RPI = 64 / CPR, NIT = 32 / RPI;
  float* stg = (float*)smem + wave * (32 * SROW);
  const int c8 = (lane % CPR) * 8, n_l = n0 + wn * TN + c8;
  ColConst cc;
  load_colconst(p, n_l, cc);
  #pragma unroll
  for (int q = 0; q < 4; ++q) {
    #pragma unroll
    for (int i = 0; i < 2; ++i)
      #pragma unroll
      for (int j = 0; j < 4; ++j)
        *(f32x4_t*)(stg + (i * 16 + (lane & 15)) * SROW + j * 16 + 4 * (lane >> 4)) = acc[2 * q + i][j];
    #pragma unroll
    for (int c0 = 0; c0 < NIT; c0 += 2) {     // 2 rows per call: 128 accumulators still live
      float v[2][8];
      int ms[2];
      #pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int row = (c0 + it) * RPI + lane / CPR;
        const f32x4_t lo = *(const f32x4_t*)(stg + row * SROW + c8);
        const f32x4_t hi = *(const f32x4_t*)(stg + row * SROW + c8 + 4);
        #pragma unroll
        for (int r = 0; r < 4; ++r) { v[it][r] = lo[r]; v[it][4 + r] = hi[r]; }
        ms[it] = m0 + wm * TM + q * 32 + row;
      }
      epilogue_rows<K_, 2>(p, cc, ms, n_l, v);
    }
  }
}

template <typename K_>
int launch_8ph(const GemmP& p0, bool conv, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = (p.N + 255) / 256;
  p.tiles_m = (p.M + 255) / 256;
  dim3 grid(p.tiles_n * p.tiles_m);
  const int ea = fast_epi_act(p);   // debug 1 << 20: the general epilogue (A/B)
#define DP_8PH(C_, R_) do { \
    if (ea == DP_ACT_NONE) hipLaunchKernelGGL((gemm_8ph_kernel<K_, C_, R_, DP_ACT_NONE>), grid, dim3(512), 0, s, p); \
    else if (ea == DP_ACT_RELU) hipLaunchKernelGGL((gemm_8ph_kernel<K_, C_, R_, DP_ACT_RELU>), grid, dim3(512), 0, s, p); \
    else if (ea == DP_ACT_GELU) hipLaunchKernelGGL((gemm_8ph_kernel<K_, C_, R_, DP_ACT_GELU>), grid, dim3(512), 0, s, p); \
    else hipLaunchKernelGGL((gemm_8ph_kernel<K_, C_, R_, -1>), grid, dim3(512), 0, s, p); } while (0)   /* (acc: general) */
  if (conv && p.relu_a) DP_8PH(true, true);
  else if (conv) DP_8PH(true, false);
  else if (p.relu_a) DP_8PH(false, true);
  else DP_8PH(false, false);
#undef DP_8PH
  DP_CHECK_LAUNCH();
  return 0;
}

// ============================================ persistent 8-phase 256x256 engine
// gemm_8ph_kernel's K loop run over the workgroup's whole tile list (tiles wgid, wgid + G,
// ... of the band raster, G = min(tiles, CUs)) as ONE stream of K steps: the LDS-DMA of the
// next tile's first K steps is issued by the same per-phase schedule as any other step, so
// it is in flight (or landed) while this tile's epilogue runs, and there is no per-tile
// dispatch, prologue or store drain.  At a tile boundary the next tile's second A tile is
// issued BEFORE the epilogue's stores, so the counted wait that retires it (phase 3 of the
// next tile's first step) can leave the stores draining: vmcnt counts loads, stores and
// LDS-DMA together in issue order (MI355X_MICROARCH.md), and the epilogue issues exactly
// ESTORES buffer stores per lane (every lane stores; rows past M / columns past N get an
// out-of-range offset, dropped by the hardware), so the count is a compile-time constant.
// The epilogue is the load-free MFMA-layout one (bias, activation, gamma; 16-bit C) staged
// through a 2 KiB slab per wave beside the 128 KiB ring (+ 2 x 1 KiB column-constant slots
// per wave: 160 KiB of LDS in all), so no LDS the ring uses is touched.  Dense A only (the ViT's fc1 / qkv).  Requires K >= 128.
// The wave's column constants (bias / gamma of its 64 columns) come from its LDS const slot
// (filled by LDS-DMA with the tile's loads), so the epilogue issues no global load: hipcc
// would put a vmcnt(0) in front of one -- a wait for every LDS-DMA in flight, i.e. the next
// tile's first K steps.
template <typename K_, int ACT, bool HG, bool DCV, bool LNC = false>
__device__ __forceinline__ void epilogue_mfma_buf(const GemmP& p, f32x4_t (&acc)[8][4], char* slab,
                                                  const float* cst, int lane, int m_base, int n_base,
                                                  __amdgpu_buffer_rsrc_t crs, const char* rstat = nullptr) {
  constexpr int FM = 8, FN = 4, TN = 64, PF = 1, CH = TN / 8, RPI = 64 / CH;
  const int t = lane & 15, g = lane >> 4;
  f32x4_t bias[FN], gam[FN];
  #pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    bias[fn] = *(const f32x4_t*)(cst + fn * 16 + 4 * g);
    if constexpr (HG || LNC) gam[fn] = *(const f32x4_t*)(cst + 64 + fn * 16 + 4 * g);   // LNC: colsum
  }
  // folded LayerNorm: row r = fm * 16 + t of the wave group's 128 lives in the const slot of its
  // wave wn' = r / 32 (each wave DMAs 32 rows' (rstd, -rstd * mean), issue_cst); all 8 read up front
  float2 rst[LNC ? FM : 1];
  if constexpr (LNC) {
    #pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int r = fm * 16 + t;
      rst[fm] = *(const float2*)(rstat + (r >> 5) * 2048 + (r & 31) * 8);
    }
  }
  // DP_STORE_DECONV2X2: a lane's 8 columns are one sub-pixel q and channels co..co+7 for the whole
  // tile, and its rows advance by RPI = 8 pixels per store: (b, y, x) of its first row once per
  // tile, then stepped (the per-store integer divisions cost the 384^2 -> 768^2 deconv 32 us of
  // 158: the same GEMM with a row store ran 126 us, tools/gemm_bench.py)
  int dq = 0, dco = 0, db = 0, dy = 0, dx = 0;
  if constexpr (DCV) {
    const int n = n_base + (lane % CH) * 8;
    dq = n / p.dc_cout;
    dco = n - dq * p.dc_cout;
    const int m = m_base + lane / CH, hw = p.dc_h * p.dc_w;
    db = m / hw;
    const int rr = m - db * hw;
    dy = rr / p.dc_w;
    dx = rr - dy * p.dc_w;
  }
  #pragma unroll
  for (int f0 = 0; f0 < FM; f0 += PF) {
    #pragma unroll
    for (int fm = 0; fm < PF; ++fm)
      #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        // packed-f32 arithmetic (the 4 columns of a lane as one vector): same values as the
        // scalar epilogue_mfma, half the VALU issue slots
        f32x4_t x;
        if constexpr (LNC) {
          x = __builtin_elementwise_fma(acc[f0 + fm][fn], (f32x4_t)(rst[f0 + fm].x),
                                        __builtin_elementwise_fma(gam[fn], (f32x4_t)(rst[f0 + fm].y), bias[fn]));
        } else {
          x = acc[f0 + fm][fn] + bias[fn];
        }
        if constexpr (ACT == DP_ACT_RELU) {
          #pragma unroll
          for (int r = 0; r < 4; ++r) x[r] = fmaxf(x[r], 0.f);
        } else if constexpr (ACT == DP_ACT_GELU) {
          x = gelu_erf4(x);
        }
        if constexpr (HG) x = x * gam[fn];
        const int row = fm * 16 + t;
        const int chunk = fn * 2 + (g >> 1);
        uint2 w;
        w.x = K_::pack2(x[0], x[1]);
        w.y = K_::pack2(x[2], x[3]);
        *(uint2*)(slab + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4) + (g & 1) * 8) = w;
      }
    #pragma unroll
    for (int k = 0; k < PF * 16 / RPI; ++k) {
      const int row = k * RPI + lane / CH, chunk = lane % CH;
      const uint4 d = *(const uint4*)(slab + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4));
      const int m = m_base + f0 * 16 + row, n = n_base + chunk * 8;
      unsigned bo = p.c_bytes;
      if (m < p.M && n < p.N) {
        if constexpr (DCV) {
          // DP_STORE_DECONV2X2 (epilogue4): row m = input pixel (b, y, x), column n = sub-pixel q,
          // channel co -> output pixel (b, 2y + q / 2, 2x + q % 2)
          const long long pix = ((long long)db * 2 * p.dc_h + 2 * dy + (dq >> 1)) * (2 * p.dc_w) + 2 * dx + (dq & 1);
          bo = (unsigned)((pix * p.ldc + dco) * 2);
        } else {
          bo = (unsigned)(((long long)m * p.ldc + n) * 2);
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{d.x, d.y, d.z, d.w}, crs, bo, 0, 0);
      if constexpr (DCV) {   // the lane's next row: RPI = 8 pixels on (host: dc_w >= 8)
        dx += RPI;
        if (dx >= p.dc_w) {
          dx -= p.dc_w;
          if (++dy == p.dc_h) { dy = 0; ++db; }
        }
      }
    }
  }
}

template <typename K_, bool RELU, int ACT, bool HG, bool DCV = false, bool LNC = false>
__global__ void __launch_bounds__(512, 1) gemm_p8ph_kernel(const GemmP p) {
  constexpr int HALF = 128 * 128;   // bytes: 128 rows x 64 16-bit
  constexpr int TILEB = 4 * HALF;   // A0 A1 B0 B1
  constexpr int RING = 2 * TILEB;   // 128 KiB
  constexpr int TN = 64, TM = 128;
  constexpr int SLAB = 16 * TN * 2;              // epilogue slab per wave (1 fragment row)
  constexpr int CST = 1024;                      // column-constant slot per wave and tile parity
  constexpr int ESTORES = 8 * 16 * TN * 2 / 1024; // 16-B stores per lane per tile
  // ring | 8 slabs | 8 x 2 const slots = 128 + 16 + 16 KiB
  __shared__ __attribute__((aligned(1024))) char smem[RING + 8 * SLAB + 16 * CST];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x, bid = blockIdx.x;
  const int T = p.tiles_m * p.tiles_n;
  const int KT = p.K / 64;
  // tile order: the static walk wgid, wgid + G, ... (XCD-contiguous, as the data-parallel
  // launch's rounds).  Measured and rejected: per-XCD tile-ticket queues (a workgroup that
  // starts late takes fewer tiles), 44.63 / 44.56 vs 44.98 / 44.96 fps (profiles/r03c_p8ph/).
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  if (wgid >= T) return;
  auto next_tile = [&](int t) { return t + G < T ? t + G : -1; };
  int t_cur = wgid, t_nxt = next_tile(t_cur);

  const int prow = wave * 8 + (lane >> 3);
  const int pchunk = (lane & 7) ^ ((lane >> 3) & 7);
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem)) + wave_u * 1024;

  // issue cursors: the next A K tile to stream is global step sa (tile ta, k ka), the next B
  // K tile step sb (tile tb, k kb); a cursor whose tile is -1 is done (it wraps to its tile's
  // successor in the walk: up to two tiles ahead of the one computed at KT = 2).  32-bit
  // element offsets of this lane's rows (host: M * lda, N * ldb < 2^31).
  int sa = 0, ta = t_cur, ka = 0, sb = 0, tb = t_cur, kb = 0;
  // byte offsets of this lane's rows from the K step's scalar base (p.A + 64 ka, p.B + 64 kb): the
  // DMA is issued in the saddr form, no per-lane 64-bit address arithmetic per K step (host: M * lda,
  // N * ldb < 2^31 elements)
  uint32_t aoff[2][2], boff[2][2];
  auto a_tile = [&](int t) {
    int tm, tn;
    tile_coords(p, t, tm, tn);
    #pragma unroll
    for (int h = 0; h < 2; ++h)
      #pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = tm * 256 + 128 * h + j * 64 + prow;
        aoff[h][j] = 2u * (uint32_t)((m < p.M ? m : p.M - 1) * (int)p.lda + pchunk * 8);
      }
  };
  auto b_tile = [&](int t) {
    int tm, tn;
    tile_coords(p, t, tm, tn);
    #pragma unroll
    for (int h = 0; h < 2; ++h)
      #pragma unroll
      for (int j = 0; j < 2; ++j) boff[h][j] = 2u * (uint32_t)((tn * 256 + 128 * h + j * 64 + prow) * (int)p.ldb + pchunk * 8);
  };
  auto issueA = [&](int h) {   // A half h of step sa -> buffer sa & 1
    const uint32_t dst = lds_base + (sa & 1) * TILEB + h * HALF;
    #pragma unroll
    for (int j = 0; j < 2; ++j) glds16s(aoff[h][j], p.A + ka * 64, dst + j * 8192);
  };
  auto nextA = [&]() {
    ++sa;
    if (++ka == KT) {
      ka = 0;
      ta = next_tile(ta);
      if (ta >= 0) a_tile(ta);
    }
  };
  auto issueB = [&](int h) {
    const uint32_t dst = lds_base + (sb & 1) * TILEB + (2 + h) * HALF;
    #pragma unroll
    for (int j = 0; j < 2; ++j) glds16s(boff[h][j], p.B + kb * 64, dst + j * 8192);
  };
  auto nextB = [&]() {
    ++sb;
    if (++kb == KT) {
      kb = 0;
      tb = next_tile(tb);
      if (tb >= 0) b_tile(tb);
    }
  };
  f32x4_t acc[8][4];
  const int frow = lane & 15, fchunk = lane >> 4;
  uint4 af[2][4], bf[2][2][2];
  // fragment addresses: per-lane bases per (buffer, ks) + compile-time ds_read immediates -- a
  // fragment row r = q 64 / 32 + f 16 + frow has r & 7 = frow & 7, so its swizzled chunk is lane-fixed;
  // the K loop below is unrolled by the two buffers (KT even), so the base is a constant choice
  typedef __attribute__((address_space(3))) const char lds_c;
  typedef __attribute__((address_space(3))) const u32x4_t lds_u4;
  uint32_t abase[2], bbase[2];   // buffer 0; buffer 1 sits TILEB above (64 KB: past the ds_read immediate)
  {
    const uint32_t l0 = lds_addr(smem);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t sw = (uint32_t)(((ks * 4 + fchunk) ^ (frow & 7)) << 4);
      abase[ks] = l0 + wm * HALF + frow * 128 + sw;
      bbase[ks] = l0 + (2 + (wn >> 1)) * HALF + ((wn & 1) * 64 + frow) * 128 + sw;
    }
  }
  // the buffer as a std::integral_constant (unrolled loop) or a runtime int (odd KT); buffer 1's
  // address is one add on a laundered base, so the compiler does not keep both in registers
  auto pick = [](const uint32_t (&b)[2], auto buf, int ks) __attribute__((always_inline)) -> uint32_t {
    uint32_t x = b[ks];
    if constexpr (std::is_integral_v<decltype(buf)>) return x + (buf ? (uint32_t)TILEB : 0u);
    else if constexpr (decltype(buf)::value == 0) return x;
    else {
      asm volatile("" : "+v"(x));
      return x + (uint32_t)TILEB;
    }
  };
  auto readA = [&](int qm, auto buf) __attribute__((always_inline)) {
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      lds_c* base = (lds_c*)(uintptr_t)pick(abase, buf, ks);
      #pragma unroll
      for (int fm = 0; fm < 4; ++fm)
        af[ks][fm] = __builtin_bit_cast(uint4, *(lds_u4*)(base + (qm * 64 + fm * 16) * 128));
    }
  };
  auto readB = [&](int qn, auto buf) __attribute__((always_inline)) {
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      lds_c* base = (lds_c*)(uintptr_t)pick(bbase, buf, ks);
      #pragma unroll
      for (int fn = 0; fn < 2; ++fn)
        bf[qn][ks][fn] = __builtin_bit_cast(uint4, *(lds_u4*)(base + (qn * 32 + fn * 16) * 128));
    }
  };
  // FIRST: a tile's first K step -- its ks = 0 MFMAs start from a zero accumulator (no
  // per-tile clearing of the 128 accumulator registers)
  auto mma = [&](int qm, int qn, auto first) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fm = 0; fm < 4; ++fm) {
        uint4 a = af[ks][fm];
        if constexpr (RELU) a = relu_pk16(a);
        #pragma unroll
        for (int fn = 0; fn < 2; ++fn) {
          f32x4_t& c = acc[qm * 4 + fm][qn * 2 + fn];
          if constexpr (decltype(first)::value) c = K_::mfma16(bf[qn][ks][fn], a, ks == 0 ? f32x4_t{0.f, 0.f, 0.f, 0.f} : c);
          else c = K_::mfma16(bf[qn][ks][fn], a, c);
        }
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() { asm volatile("s_barrier" ::: "memory"); };
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, (int)p.c_bytes, 0x00020000);
  char* slab = smem + RING + wave * SLAB;
  // column constants of tile t -> this wave's const slot `par`: ONE LDS-DMA piece per wave
  // (lanes 0-15: bias of the wave's 64 columns, 16-31: gamma, 32-63 repeat 0-31), issued
  // with the tile's loads and retired by the same counted waits (only this wave reads it)
  // LNC (folded-LayerNorm consumer): lanes 16-31 bring the column sums instead of gamma and
  // lanes 32-47 the (rstd, -rstd * mean) of 32 of the wave group's 128 rows (2 rows per lane,
  // rows wn * 32 ..), so the 4 waves of a group hold its rows between them (read across waves
  // in the epilogue: that tile's whole K loop, with its barriers, lies between)
  auto issue_cst = [&](int t, int par) {
    int tm, tn;
    tile_coords(p, t, tm, tn);
    const int l = lane & 15, n = tn * 256 + wn * TN + 4 * l;
    const float* src;
    if ((lane & 16) == 0 && lane < 32) src = p.bias ? p.bias + n : (const float*)g_zero_page + 4 * l;
    else if (lane < 32) src = HG ? p.gamma + n : LNC ? p.ln_colsum + n : (const float*)g_zero_page + 4 * l;
    else if (LNC && lane < 48) {
      // rows past M (the last row tile) re-read the pair holding row M - 1, whose values they
      // never store: the caller's buffer holds M rounded up to even rows
      const int row = tm * 256 + wm * TM + wn * 32 + 2 * (lane - 32);
      src = p.ln_rs + 2 * (row < p.M ? row : ((p.M - 1) & ~1));
    }
    else src = (const float*)g_zero_page + 4 * l;
    glds16(src, __builtin_amdgcn_readfirstlane(lds_addr(smem)) + RING + 8 * SLAB + (wave_u * 2 + par) * CST);
  };

  // prologue: tile 0's column constants, step 0 (A and B) and step 1's B (KT >= 2)
  issue_cst(t_cur, 0);
  a_tile(t_cur);
  b_tile(t_cur);
  issueA(0); issueA(1); nextA();
  issueB(0); issueB(1); nextB();
  issueB(0); issueB(1); nextB();
  wait_vmcnt<4>();
  lds_barrier();
  // wave rows staggered by one barrier (gemm_8ph_kernel); kept across tiles
  if (wm == 1) bar();
  int s = 0;
  // one K step s (k-th of the i-th tile): the 8-phase schedule of gemm_8ph_kernel with the
  // issue cursors deciding what streams in
  auto step = [&](int i, int k, auto first, auto buf) __attribute__((always_inline)) {
    const bool a1 = sa == s + 1 && ta >= 0;   // step s+1's A not issued yet (it was at a boundary)
    const bool b2 = tb >= 0;                  // sb == s + 2
    // phase 0: quadrant (0,0)
    readA(0, buf); readB(0, buf);
    if (a1) issueA(0);
    bar(); mma(0, 0, first); bar();
    // phase 1: quadrant (0,1)
    readB(1, buf);
    if (a1) { issueA(1); nextA(); }
    bar(); mma(0, 1, first); bar();
    // phase 2: quadrant (1,0)
    readA(1, buf);
    if (b2) issueB(0);
    bar(); mma(1, 0, first); bar();
    // phase 3: step s+1 must have landed before this phase's first barrier; younger than
    // it: B0 of step s+2 (this step's phase 2) and, in a tile's first step, the previous
    // tile's epilogue stores (issued after step s+1's loads)
    if (k == 0 && i > 0) {
      if (b2) wait_vmcnt<ESTORES + 2>(); else wait_vmcnt<ESTORES>();
    } else {
      if (b2) wait_vmcnt<2>(); else wait_vmcnt<0>();
    }
    if (b2) { issueB(1); nextB(); }
    bar(); mma(1, 1, first);
    bar();
    ++s;
  };
#ifdef DP_STAMPS
  unsigned long long p8st_[3 * P8_STAMP_TILES] = {};
#endif
  for (int i = 0;; ++i) {
#ifdef DP_STAMPS
    if (i < P8_STAMP_TILES) DP_STAMP(p8st_[3 * i]);
#endif
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    if ((KT & 1) == 0) {   // step s = i KT + k is in buffer k & 1
      step(i, 0, std::true_type{}, B0{});
      int k = 1;
      for (; k + 1 < KT; k += 2) {
        step(i, k, std::false_type{}, B1{});
        step(i, k + 1, std::false_type{}, B0{});
      }
      step(i, k, std::false_type{}, B1{});
    } else {
      step(i, 0, std::true_type{}, s & 1);
      for (int k = 1; k < KT; ++k) step(i, k, std::false_type{}, s & 1);
    }
#ifdef DP_STAMPS
    if (i < P8_STAMP_TILES) DP_STAMP(p8st_[3 * i + 1]);
#endif
    // tile boundary: the next tile's second A K tile goes out before the epilogue's stores
    // (its buffer's last reads were this step's phases 0 / 2, two barriers back)
    if (t_nxt >= 0) {
      if (ta >= 0) { issueA(0); issueA(1); nextA(); }
      issue_cst(t_nxt, (i + 1) & 1);
    }
    int tm, tn;
    tile_coords(p, t_cur, tm, tn);
    const float* cst = (const float*)(smem + RING + 8 * SLAB + (wave * 2 + (i & 1)) * CST);
    const char* rstat = smem + RING + 8 * SLAB + (wm * 8 + (i & 1)) * CST + 512;   // wave group's row stats
    epilogue_mfma_buf<K_, ACT, HG, DCV, LNC>(p, acc, slab, cst, lane, tm * 256 + wm * TM, tn * 256 + wn * TN, crs,
                                             rstat);
#ifdef DP_STAMPS
    if (i < P8_STAMP_TILES) DP_STAMP(p8st_[3 * i + 2]);
#endif
    if (t_nxt < 0) break;
    t_cur = t_nxt;
    t_nxt = next_tile(t_cur);
  }
  if (wm == 0) bar();
#ifdef DP_STAMPS
  if (threadIdx.x == 0 && wgid < 1024) {
    unsigned hw_, xcc_;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));
    unsigned long long* d_ = g_p8_stamps + P8_STAMP_W * wgid;
    for (int j = 0; j < 3 * P8_STAMP_TILES; ++j) d_[j] = p8st_[j];
    d_[3 * P8_STAMP_TILES] = hw_ | ((unsigned long long)xcc_ << 32);
  }
#endif
}

// (rstd, -rstd * mean) of a row from its 8 chunk statistics (K = 1024; Chan's merge, as
// epilogue_mfma_lnc): ln_merge_kernel and ln_merge_last, the same arithmetic
__device__ __forceinline__ float2 ln_merge_row(const f32x4_t (&c)[4], float eps) {
  const float mean = (((c[0][0] + c[0][2]) + (c[1][0] + c[1][2])) + ((c[2][0] + c[2][2]) + (c[3][0] + c[3][2]))) *
                     (1.f / 8);
  float m2 = 0.f;
  #pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float d0 = c[i][0] - mean, d1 = c[i][2] - mean;
    m2 += (c[i][1] + 128.f * d0 * d0) + (c[i][3] + 128.f * d1 * d1);
  }
  const float rs = rsqrtf(m2 * (1.f / 1024) + eps);
  return make_float2(rs, -rs * mean);
}

// The split producer's row merge (ABI 13, p.ln_rs_out): after its epilogue every workgroup of a
// row tile adds one to the tile's counter; the last of the tiles_n arrivals merges the tile's rows
// from ln_part_out (stored write-through, sc1, and drained before the add; read back with sc1
// loads) into ln_rs_out and resets the counter for the next launch.  Replaces the persistent
// consumer's pre-pass launch (ln_merge_kernel).  Guideline 16's sc1 hand-off, no fences: the
// measured-valid form of MI355X_MICROARCH.md's hand-off table, row 1 (every byte stored sc1 and
// drained by each storing wave before the barrier, ONE lane's agent-scope add to one counter, the
// last adder's workgroup loading only with sc1 buffer loads after a barrier) -- an agent-scope
// acq_rel add would also write back the XCD L2's dirty lines of the whole epilogue (~2-6 us per
// workgroup at the end of every proj / fc2).  The signal fences keep the compiler from moving the
// loads above the add (the barrier orders them too).
__device__ __forceinline__ void ln_merge_last(const GemmP& p, int tile_m, int rows, char* smem, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's part stores (sc1) have landed
  __syncthreads();
  int* last = (int*)smem;
  if (tid == 0) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const unsigned old = __hip_atomic_fetch_add(p.ln_cnt + tile_m, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    *last = old == (unsigned)(p.tiles_n - 1);
  }
  __syncthreads();
  if (!*last) return;
  if (tid == 0) __hip_atomic_store(p.ln_cnt + tile_m, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const __amdgpu_buffer_rsrc_t rs_pt = __builtin_amdgcn_make_buffer_rsrc((void*)p.ln_part_out, (short)0,
                                                                         (int)(p.M * 64), 0x00020000);
  for (int r = tid; r < rows; r += blockDim.x) {
    const int m = tile_m * rows + r;
    if (m >= p.M) break;
    f32x4_t c[4];
    #pragma unroll
    for (int i = 0; i < 4; ++i)
      c[i] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs_pt, (unsigned)(m * 64 + i * 16), 0, 16));
    *(float2*)(p.ln_rs_out + 2LL * m) = ln_merge_row(c, p.ln_eps);
  }
}

// Folded LayerNorm, consumer on the persistent 8-phase engine: per row (rstd, -rstd * mean) from
// its 8 chunk statistics (K = 1024; Chan's merge, as epilogue_mfma_lnc), one thread per row.
__global__ void __launch_bounds__(256) ln_merge_kernel(const float* __restrict__ part, int M, float eps,
                                                       float* __restrict__ out) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const f32x4_t* pp = (const f32x4_t*)(part + (long long)m * 16);
  f32x4_t c[4];
  #pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = pp[i];
  *(float2*)(out + 2LL * m) = ln_merge_row(c, eps);
}

template <typename K_>
int launch_p8ph(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = p.N / 256;
  p.tiles_m = (p.M + 255) / 256;
  const int T = p.tiles_n * p.tiles_m;
  const bool dcv = p.store_mode == DP_STORE_DECONV2X2;
  const int ea = dcv ? p.act : fast_epi_act(p);
  if (p.N % 256 || p.K < 128 || !p.c_bytes || p.c_dtype == DP_F32 || ea < 0 || ea >= EPI_ACC) return DP_ERR_ARG;
  int G = num_cus();
  if (G > T) G = T;
  dim3 grid(G);
  if (dcv) {   // the 2x2 stride-2 deconvs: bias only (no per-row operands, no activation)
    if (p.relu_a || p.gamma || p.pos || p.R1 || p.R2 || p.accumulate || p.row_group || p.head_w || p.head_corr ||
        ea != DP_ACT_NONE || p.dc_cout % 8 || p.dbg & (1 << 20))
      return DP_ERR_ARG;
    hipLaunchKernelGGL((gemm_p8ph_kernel<K_, false, DP_ACT_NONE, false, true>), grid, dim3(512), 0, s, p);
    DP_CHECK_LAUNCH();
    return 0;
  }
  if (p.store_mode != DP_STORE_ROWS) return DP_ERR_ARG;
  if (p.ln_rs) {   // folded-LayerNorm consumer (the ViT fc1): dense, no ReLU prologue, no gamma
    if (p.relu_a || p.gamma) return DP_ERR_ARG;
    if (ea == DP_ACT_NONE) hipLaunchKernelGGL((gemm_p8ph_kernel<K_, false, DP_ACT_NONE, false, false, true>), grid, dim3(512), 0, s, p);
    else if (ea == DP_ACT_GELU) hipLaunchKernelGGL((gemm_p8ph_kernel<K_, false, DP_ACT_GELU, false, false, true>), grid, dim3(512), 0, s, p);
    else return DP_ERR_ARG;
    DP_CHECK_LAUNCH();
    return 0;
  }
#define DP_P8(R_, G_) do { \
    if (ea == DP_ACT_NONE) hipLaunchKernelGGL((gemm_p8ph_kernel<K_, R_, DP_ACT_NONE, G_>), grid, dim3(512), 0, s, p); \
    else if (ea == DP_ACT_RELU) hipLaunchKernelGGL((gemm_p8ph_kernel<K_, R_, DP_ACT_RELU, G_>), grid, dim3(512), 0, s, p); \
    else hipLaunchKernelGGL((gemm_p8ph_kernel<K_, R_, DP_ACT_GELU, G_>), grid, dim3(512), 0, s, p); } while (0)
  // (a gamma-free launch -- fc1 -- skips the multiply by 1 per output)
  if (p.relu_a) { if (p.gamma) DP_P8(true, true); else DP_P8(true, false); }
  else { if (p.gamma) DP_P8(false, true); else DP_P8(false, false); }
#undef DP_P8
  DP_CHECK_LAUNCH();
  return 0;
}


// ======================================================= 8-phase 320x256 engine
// The 8-phase schedule (gemm_8ph_kernel) on the 320 x 256 tile that gives the ViT's M = 20195
// exactly 64 row tiles (proj / fc2: ONE round of 256 workgroups; qkv: 3).  8 waves as 4 (M) x
// 2 (N), wave tile 80 x 128 (acc 5 x 8 fragments = 160 VGPRs).  A K step (BK 64) is 4 phases,
// one per 32-column quarter of the wave's 128 columns: {ds_reads, LDS-DMA pieces, counted
// vmcnt, s_barrier, 20 MFMAs at raised priority, s_barrier}; phase 0 also reads the wave's 10
// A fragments (kept for the step).  The two wave groups (waves 0-3 / 4-7: one of each per
// SIMD) run staggered by one barrier, so one wave of a SIMD issues MFMAs while the other reads.
// LDS: 2 K-tile buffers of A (320 x 128 B) + B (256 x 128 B) = 144 KiB.
// Streaming, per step s (9 pieces of 1 KiB per wave): B quarter q of step s+1 in phase q (its
// buffer's quarter was last read 4 phases earlier), A of step s+2 in phases 2 / 3 (3 + 2
// pieces; the buffer's A was read in phase 0, two barriers back).  Every phase waits (counted)
// for what the NEXT phase reads -- B quarter q+1 of this step, or A and B quarter 0 of step
// s+1 in phase 3 -- so each piece has 4+ phases to land and the count is 8 in steady state.
// Dense A only; epilogues: the load-free MFMA-layout one (EACT = DP_ACT_*; 16-bit C) or the
// fp32 residual-accumulate one (EACT = EPI_ACC + act).
// (Measured and rejected, round 5: the K loop's first steps also streaming the wave's epilogue rows
// of the residual into a dummy LDS slot, so the epilogue's reads would hit the caches: proj 71.1 ->
// 76.9 us cold, fc2 155.9 -> 162.5, in-frame -0.8 fps, profiles/r05av_residual_touch/.)
template <typename K_, int EACT, int LNM = 0>   // LNM: 1 folded-LN producer, 2 consumer, 3 (4) producer on hi + lo
__global__ void __launch_bounds__(512, 1) gemm_8ph320_kernel(const GemmP p) {
  constexpr int BM = 320;
  constexpr int A_BYTES = BM * 128, B_BYTES = 256 * 128, BUF = A_BYTES + B_BYTES;
  constexpr int FM = 5, FN = 8, TM = 80, TN = 128;
  constexpr int RING = 2 * BUF;                                   // 144 KiB
  constexpr int PF = 1, SLAB = PF * 16 * TN * 2;                  // epilogue_mfma slab per wave
  constexpr int SMEM = RING > 8 * SLAB ? RING : 8 * SLAB;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave & 3, wn = wave >> 2;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tile_m, tile_n;
  tile_coords(p, wgid, tile_m, tile_n);
  const int m0 = tile_m * BM, n0 = tile_n * 256;

  // LDS-DMA pieces: 8 rows x 128 B per wave, the 16-B chunk swizzled on the source address
  const int pchunk = (lane & 7) ^ ((lane >> 3) & 7);
  // byte offsets of this lane's rows from the step's scalar base (saddr DMA; the planner's off32:
  // M * lda, N * ldb < 2^31 elements)
  uint32_t aoff[5];
  #pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int m = m0 + j * 64 + wave * 8 + (lane >> 3);
    aoff[j] = 2u * (uint32_t)((m < p.M ? m : p.M - 1) * (int)p.lda + pchunk * 8);
  }
  // B quarter q = output columns {q*32 .. +31} u {128 + q*32 .. +31}: waves 0-3 / 4-7 take 8 rows each
  const int brow0 = wave_u < 4 ? wave_u * 8 : 128 + (wave_u - 4) * 8;   // + q * 32
  const uint32_t boff = 2u * (uint32_t)((n0 + brow0 + (lane >> 3)) * (int)p.ldb + pchunk * 8);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  auto issueA = [&](int j, int t) {
    glds16s(aoff[j], p.A + t * 64, lds0 + (t & 1) * BUF + j * 8192 + wave_u * 1024);
  };
  auto issueB = [&](int q, int t) {
    glds16s(boff, p.B + (q * 32 * (int)p.ldb + t * 64), lds0 + (t & 1) * BUF + A_BYTES + (brow0 + q * 32) * 128);
  };

  f32x4_t acc[FM][FN];
  #pragma unroll
  for (int i = 0; i < FM; ++i)
    #pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15, fchunk = lane >> 4;
  uint4 af[2][FM], bf[2][2];
  // fragment addresses: per-lane bases (buffer 0) per ks + ds_read immediates -- fragment row r =
  // 16 f + frow (+ 80 wm / 32 q) has r & 7 = frow & 7, so its swizzled chunk is lane-fixed.  Buffer 1
  // sits BUF (72 KiB) above, past the 16-bit immediate: one add on a laundered base (the compiler
  // would otherwise keep all four bases live across the loop)
  typedef __attribute__((address_space(3))) const char lds_c;
  typedef __attribute__((address_space(3))) const u32x4_t lds_u4;
  uint32_t abase[2], bbase[2];
  #pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t sw = (uint32_t)(((ks * 4 + fchunk) ^ (frow & 7)) << 4);
    abase[ks] = lds0 + (wm * TM + frow) * 128 + sw;
    bbase[ks] = lds0 + A_BYTES + (wn * TN + frow) * 128 + sw;
  }
  auto pick = [](const uint32_t (&b)[2], auto buf, int ks) __attribute__((always_inline)) -> uint32_t {
    uint32_t x = b[ks];
    if constexpr (std::is_integral_v<decltype(buf)>) return x + (buf ? (uint32_t)BUF : 0u);
    else if constexpr (decltype(buf)::value == 0) return x;
    else {
      asm volatile("" : "+v"(x));
      return x + (uint32_t)BUF;
    }
  };
  auto readA = [&](auto buf) __attribute__((always_inline)) {
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      lds_c* base = (lds_c*)(uintptr_t)pick(abase, buf, ks);
      #pragma unroll
      for (int fm = 0; fm < FM; ++fm) af[ks][fm] = __builtin_bit_cast(uint4, *(lds_u4*)(base + fm * 16 * 128));
    }
  };
  auto readB = [&](int q, auto buf) __attribute__((always_inline)) {
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      lds_c* base = (lds_c*)(uintptr_t)pick(bbase, buf, ks);
      #pragma unroll
      for (int f = 0; f < 2; ++f) bf[ks][f] = __builtin_bit_cast(uint4, *(lds_u4*)(base + (q * 32 + f * 16) * 128));
    }
  };
  auto mma = [&](int q) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fm = 0; fm < FM; ++fm)
        #pragma unroll
        for (int f = 0; f < 2; ++f) acc[fm][2 * q + f] = K_::mfma16(bf[ks][f], af[ks][fm], acc[fm][2 * q + f]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() { asm volatile("s_barrier" ::: "memory"); };

  const int KT = p.K / 64;
  // prologue = "step -1" in the steady-state issue order: A(0); Bq0..3(0) with A(1) after Bq2 / Bq3
  #pragma unroll
  for (int j = 0; j < 5; ++j) issueA(j, 0);
  issueB(0, 0);
  issueB(1, 0);
  issueB(2, 0);
  if (KT > 1) { issueA(0, 1); issueA(1, 1); issueA(2, 1); }
  issueB(3, 0);
  if (KT > 1) { issueA(3, 1); issueA(4, 1); }
  // A(0) and Bq0(0) landed: younger are Bq1..3(0) and A(1)
  if (KT > 1) wait_vmcnt<8>(); else wait_vmcnt<3>();
  lds_barrier();
  if (wave >= 4) bar();
  // one K step s in buffer buf (a std::integral_constant when the loop below is unrolled by the
  // two buffers -- KT even -- else s & 1)
  auto step = [&](int s, auto buf) __attribute__((always_inline)) {
    const bool a1 = s + 1 < KT, a2 = s + 2 < KT;
    // phase 0: A fragments + B quarter 0; retire Bq1(s) (younger: 2 + 6 a1)
    readA(buf); readB(0, buf);
    if (a1) issueB(0, s + 1);
    if (a1) wait_vmcnt<8>(); else wait_vmcnt<2>();
    bar(); mma(0); bar();
    // phase 1: retire Bq2(s) (younger: 1 + 7 a1)
    readB(1, buf);
    if (a1) issueB(1, s + 1);
    if (a1) wait_vmcnt<8>(); else wait_vmcnt<1>();
    bar(); mma(1); bar();
    // phase 2: A(s+2) pieces 0-2 into this step's buffer; retire Bq3(s) (younger: 5 a1 + 3 a2)
    readB(2, buf);
    if (a1) issueB(2, s + 1);
    if (a2) { issueA(0, s + 2); issueA(1, s + 2); issueA(2, s + 2); }
    if (a2) wait_vmcnt<8>(); else if (a1) wait_vmcnt<5>(); else wait_vmcnt<0>();
    bar(); mma(2); bar();
    // phase 3: retire A(s+1) and Bq0(s+1) (younger: 3 + 5 a2)
    readB(3, buf);
    if (a1) issueB(3, s + 1);
    if (a2) { issueA(3, s + 2); issueA(4, s + 2); }
    if (a2) wait_vmcnt<8>(); else if (a1) wait_vmcnt<3>();
    bar(); mma(3); bar();
  };
  if ((KT & 1) == 0) {
    for (int s = 0; s < KT; s += 2) {
      step(s, std::integral_constant<int, 0>{});
      step(s + 1, std::integral_constant<int, 1>{});
    }
  } else {
    for (int s = 0; s < KT; ++s) step(s, s & 1);
  }
  if (wave < 4) bar();
  if (p.dbg & 1) {   // ablation (tools/gemm_bench.py --ablate): no epilogue
    #pragma unroll
    for (int i = 0; i < FM; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j][0]), "v"(acc[i][j][1]), "v"(acc[i][j][2]), "v"(acc[i][j][3]));
    return;
  }
  lds_barrier();   // the ring is free once every wave has left the K loop
  if constexpr (LNM == 3 || LNM == 4) {
    epilogue_hilo_ln<K_, FM, FN, LNM == 3 ? 3 : 1>(p, acc, smem + wave * 13312, lane, m0 + wm * TM, n0 + wn * TN);
    if (p.ln_rs_out) ln_merge_last(p, tile_m, BM, smem, tid);
  }
  else if constexpr (LNM == 1)
    epilogue_acc32_wide_ln<K_, FM, FN>(p, acc, smem + wave * 8192, lane, m0 + wm * TM, n0 + wn * TN);
  else if constexpr (EACT >= EPI_ACC)
    epilogue_acc32_wide<EACT - EPI_ACC, FM, FN>(p, acc, smem + wave * SLAB, lane, m0 + wm * TM, n0 + wn * TN);
  else if constexpr (LNM == 2)
    epilogue_mfma_lnc<K_, EACT, FM, FN, TN>(p, acc, smem + wave * 8192, lane, m0 + wm * TM, n0 + wn * TN);
  else
    epilogue_mfma<K_, EACT, FM, FN, TN, PF>(p, acc, smem + wave * SLAB, lane, m0 + wm * TM, n0 + wn * TN);
}

template <typename K_>
int launch_8ph320(const GemmP& p0, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = p.N / 256;
  p.tiles_m = (p.M + 319) / 320;
  const int ea = fast_epi_act(p);
  if (p.N % 256 || ea < 0 || p.relu_a) return DP_ERR_ARG;
  dim3 grid(p.tiles_n * p.tiles_m);
  if (p.ln_xl) {         // folded-LN producer on the split (hi + lo) residual stream
    if (!p.ln_xb_out || p.act != DP_ACT_NONE) return DP_ERR_ARG;
    static_assert(8 * 13312 <= 2 * (320 * 128 + 256 * 128), "hi/lo staging fits the ring");
    if (p.dbg & (1 << 27)) hipLaunchKernelGGL((gemm_8ph320_kernel<K_, EPI_ACC + DP_ACT_NONE, 4>), grid, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((gemm_8ph320_kernel<K_, EPI_ACC + DP_ACT_NONE, 3>), grid, dim3(512), 0, s, p);
    DP_CHECK_LAUNCH();
    return 0;
  }
  if (p.ln_part_out) {   // folded-LN producer: the residual accumulate
    if (ea != EPI_ACC + DP_ACT_NONE || !p.ln_xb_out) return DP_ERR_ARG;
    hipLaunchKernelGGL((gemm_8ph320_kernel<K_, EPI_ACC + DP_ACT_NONE, 1>), grid, dim3(512), 0, s, p);
    DP_CHECK_LAUNCH();
    return 0;
  }
  if (p.ln_part_in) {    // folded-LN consumer (qkv / fc1): 16-bit C, K = 1024
    switch (ea) {
      case DP_ACT_NONE: hipLaunchKernelGGL((gemm_8ph320_kernel<K_, DP_ACT_NONE, 2>), grid, dim3(512), 0, s, p); break;
      case DP_ACT_GELU: hipLaunchKernelGGL((gemm_8ph320_kernel<K_, DP_ACT_GELU, 2>), grid, dim3(512), 0, s, p); break;
      default: return DP_ERR_ARG;
    }
    DP_CHECK_LAUNCH();
    return 0;
  }
  switch (ea) {
    case DP_ACT_NONE: hipLaunchKernelGGL((gemm_8ph320_kernel<K_, DP_ACT_NONE>), grid, dim3(512), 0, s, p); break;
    case DP_ACT_RELU: hipLaunchKernelGGL((gemm_8ph320_kernel<K_, DP_ACT_RELU>), grid, dim3(512), 0, s, p); break;
    case DP_ACT_GELU: hipLaunchKernelGGL((gemm_8ph320_kernel<K_, DP_ACT_GELU>), grid, dim3(512), 0, s, p); break;
    case EPI_ACC + DP_ACT_NONE: hipLaunchKernelGGL((gemm_8ph320_kernel<K_, EPI_ACC + DP_ACT_NONE>), grid, dim3(512), 0, s, p); break;
    default: return DP_ERR_ARG;
  }
  DP_CHECK_LAUNCH();
  return 0;
}


// ================================================= stream-K persistent engine
// 256 x 256 x 64 tiles, 8 waves (2 x 4, wave tile 128 x 64), one persistent
// workgroup per CU.  The T tiles x KT k-steps of the GEMM form one list of
// "units" (tile-major, k inner) that is cut into G equal contiguous ranges,
// one per workgroup (stream-K), so that
//  * every CU gets the same work (no 3.7-round quantisation tail),
//  * the LDS-DMA ring runs on across tile boundaries: the next tile's first
//    k-step is in flight while the previous tile's epilogue runs (no prologue
//    per tile), and
//  * tile boundaries -- hence the epilogue store bursts -- fall at different
//    times on different CUs instead of all 256 CUs storing at once.
// A range that starts inside a tile computes that tile's last k-steps and
// publishes them as an fp32 partial (write-through stores + flag); the
// workgroup whose range covers the tile's k-step 0 (it reaches it at the END
// of its range) owns the tile: it adds every partial of the tile, then runs the
// normal epilogue.  A workgroup only ever waits for a higher-numbered one,
// which published at the START of its range: no cycle, no deadlock, and the
// spin is bounded (a timeout sets an error word instead of hanging the GPU).
// The epilogue stages 16-row slices through its own 32 KiB of LDS so that the
// 128 KiB ring stays live underneath it.
constexpr int SK_A_BYTES = 256 * 128;            // 256 rows x 64 16-bit
constexpr int SK_STAGE = 2 * SK_A_BYTES;         // A + B
constexpr int SK_RING = 2 * SK_STAGE;            // 2 stages: 128 KiB
constexpr int SK_EPI = 8 * 16 * 64 * 4;          // 8 waves x 16 rows x 64 fp32
constexpr int SK_TILE_F = 256 * 256;             // floats per partial slot
constexpr long long SK_FLAG_BYTES = 4096;        // flags [0, G) (each reset by its consumer), error word at [1023] (sticky)
constexpr int LN_CNT_WORD = 512;                 // the split producer's row-tile counters: words [512, 1023)
static_assert(DP_GEMM_WS_ERROR_OFFSET == 4 * 1023, "error word offset (dp_mi355x.h)");
constexpr int SK_MAX_WG = 256;

struct SkP {
  uint32_t* flags;
  float* part;
  int kt, tiles, units;
};

// ROWLD: the epilogue reads per-row operands (residuals R1/R2, the fp32 C being
// accumulated into, pos-embed); without them it needs ~40 fewer VGPRs.
template <typename K_, bool CONV, bool RELU, bool ROWLD>
__global__ void __launch_bounds__(512, 1) gemm_sk_kernel(const GemmP p, const SkP s) {
  constexpr int TM = 128, TN = 64, FM = 8, FN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[SK_RING + SK_EPI];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int KT = s.kt, U = s.units;
  const int u0 = (int)((long long)w * U / G), u1 = (int)((long long)(w + 1) * U / G);
  auto wg_of_unit = [&](int u) { return (int)(((long long)(u + 1) * G - 1) / U); };
  // Tile positions are walked column-major over an R x G grid of tile ids
  // (id = row * G + column): range w then covers ~column w, i.e. tiles w, w+G,
  // w+2G, ... as in a data-parallel launch, so the tiles in flight at any
  // moment are ~consecutive ids (shared A/B panels in L2), while the fractional
  // range length staggers the tile boundaries across workgroups.
  const int T = s.tiles, R = (T + G - 1) / G, r0 = T - (R - 1) * G;
  auto tile_of = [&](int pos) {
    int c, r;
    if (pos < r0 * R) {
      c = pos / R;
      r = pos - c * R;
    } else {
      const int q = pos - r0 * R;
      c = r0 + q / (R - 1);
      r = q - (c - r0) * (R - 1);
    }
    return r * G + c;
  };

  // ---- LDS-DMA issue side (runs one unit ahead of the MFMAs).  Only the
  // tile's scalar origin is kept: per-lane source addresses are recomputed per
  // issue (a few VALU ops under 64 MFMAs) so the 128 accumulators, the
  // fragments and the epilogue fit in 256 VGPRs without spilling.
  const int prow = wave * 8 + (lane >> 3);
  const int pchunk = (lane & 7) ^ ((lane >> 3) & 7);
  int is_tile = -1, is_m0 = 0, is_n0 = 0;
  ConvRow a_cr[CONV ? 4 : 1];
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(smem)) + wave_u * 1024;
  auto issue = [&](int u, int stage) {
    const int t = u / KT, ks = u - t * KT;
    if (t != is_tile) {
      is_tile = t;
      const int id = tile_of(t);
      is_m0 = (id / p.tiles_n) * 256;
      is_n0 = (id % p.tiles_n) * 256;
      if constexpr (CONV) {
        #pragma unroll
        for (int i = 0; i < 4; ++i) a_cr[i] = conv_row(p, is_m0 + i * 64 + prow);
      }
    }
    const uint32_t sa = lds_base + stage * SK_STAGE, sb = sa + SK_A_BYTES;
    const int k0 = ks * 64;
    int ky = 0, kx = 0, ci = 0;
    if constexpr (CONV) {
      conv_tap(p, k0, ky, kx, ci);
    }
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const void* src;
      if constexpr (CONV) {
        bool inb;
        const u16* q = conv_src(p, a_cr[i], ky, kx, ci + pchunk * 8, inb);
        src = inb ? (const void*)q : (const void*)g_zero_page;
      } else {
        const int m = is_m0 + i * 64 + prow;
        src = p.A + (long long)(m < p.M ? m : p.M - 1) * p.lda + k0 + pchunk * 8;
      }
      glds16(src, sa + i * 8192);
    }
    #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = is_n0 + i * 64 + prow;
      glds16(p.B + (long long)(n < p.N ? n : p.N - 1) * p.ldb + k0 + pchunk * 8, sb + i * 8192);
    }
  };

  f32x4_t acc[FM][FN];
  auto zero_acc = [&]() {
    #pragma unroll
    for (int i = 0; i < FM; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  };
  const int frow = lane & 15, fchunk = lane >> 4;
  auto compute = [&](int stage) {
    const u16* sa = (const u16*)(smem + stage * SK_STAGE);
    const u16* sb = (const u16*)(smem + stage * SK_STAGE + SK_A_BYTES);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 bf[FN];
      #pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = *(const uint4*)(sb + lds_off(wn * TN + j * 16 + frow, ks * 4 + fchunk));
      __builtin_amdgcn_s_setprio(1);
      #pragma unroll
      for (int i = 0; i < FM; ++i) {
        uint4 af = *(const uint4*)(sa + lds_off(wm * TM + i * 16 + frow, ks * 4 + fchunk));
        if constexpr (RELU) af = relu_pk16(af);
        #pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = K_::mfma16(bf[j], af, acc[i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
    }
  };

  // ---- epilogue of one finished tile: 16-row slices through this wave's LDS slab,
  // read back row-major (8 rows x 8 columns per lane instruction pair)
  float* stg = (float*)(smem + SK_RING) + wave * (16 * 64);
  auto epilogue = [&](int t) {
    const int id = tile_of(t);
    const int m0 = (id / p.tiles_n) * 256, n0 = (id % p.tiles_n) * 256;
    const int c8 = (lane & 7) * 8, n_l = n0 + wn * TN + c8;
    ColConst cc;                     // bias / LayerScale of this lane's 8 columns, loaded once
    load_colconst(p, n_l, cc);
    #pragma unroll
    for (int i = 0; i < FM; ++i) {
      // lane holds row (lane & 15), 16-B chunks j*4 + (lane >> 4); chunk index XOR row
      #pragma unroll
      for (int j = 0; j < FN; ++j)
        *(f32x4_t*)(stg + frow * 64 + (((j * 4 + fchunk) ^ frow) << 2)) = acc[i][j];
      float v[2][8];
      int ms[2];
      #pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int row = it * 8 + (lane >> 3);
        const f32x4_t lo = *(const f32x4_t*)(stg + row * 64 + (((2 * (lane & 7)) ^ row) << 2));
        const f32x4_t hi = *(const f32x4_t*)(stg + row * 64 + (((2 * (lane & 7) + 1) ^ row) << 2));
        #pragma unroll
        for (int r = 0; r < 4; ++r) { v[it][r] = lo[r]; v[it][4 + r] = hi[r]; }
        ms[it] = m0 + wm * TM + i * 16 + row;
      }
      if constexpr (ROWLD) {
        epilogue_rows<K_, 2>(p, cc, ms, n_l, v);   // both rows' loads issued before any math
      } else {
        GemmP q = p;
        q.R1 = nullptr; q.R2 = nullptr; q.pos = nullptr; q.accumulate = 0;
        epilogue_rows<K_, 2>(q, cc, ms, n_l, v);
      }
    }
  };

  // partial slot layout: [wave][i][j][lane] x f32x4 -> 1 KiB contiguous per wave instruction
  auto slot_ptr = [&](int q, int i, int j) {
    return s.part + (long long)q * SK_TILE_F + ((((wave * FM + i) * FN + j) * 64 + lane) << 2);
  };
  auto publish = [&]() {
    // write-through (sc1) 16-B buffer stores of this wave's accumulators into slot w:
    // visible to the owner after its agent-scope acquire (Guideline 16, R1)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(s.part + (long long)w * SK_TILE_F, (short)0, SK_TILE_F * 4, 0x00020000);
    const int vo = (wave * FM * FN * 64 + lane) * 16;
    #pragma unroll
    for (int i = 0; i < FM; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[i][j]), rs, vo + (i * FN + j) * 1024, 0,
                                               16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its stores
    __syncthreads();
    if (tid == 0) __hip_atomic_store(s.flags + w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto absorb = [&](int q) {   // add workgroup q's published partial of the tile
    if (tid == 0) {
      unsigned spins = 0;
      // debug bit 64 (tests only): give up at once, as a starved wait would
      const unsigned limit = (p.dbg & 64) ? 0u : (1u << 24);
      while (__hip_atomic_load(s.flags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u || (p.dbg & 64)) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > limit) {  // ~seconds: never hang the GPU; report in the sticky error word instead
          __hip_atomic_store(s.flags + 1023, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      // consumed: back to 0, so every flag is 0 again when the launch ends (no per-launch
      // clearing; a memset node of a replayed HIP graph raced the next launch's polls and let
      // an owner add the previous replay's partials -- found by tools/parity_probe.py)
      __hip_atomic_store(s.flags + q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    #pragma unroll
    for (int i = 0; i < FM; ++i) {   // one fragment row at a time (bounded live registers)
      #pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] += *(const f32x4_t*)slot_ptr(q, i, j);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (u0 >= u1) return;
  zero_acc();
  issue(u0, 0);
  int stage = 0, seg0 = u0;
  int t = u0 / KT, ks = u0 - t * KT;
  for (int u = u0; u < u1; ++u) {
    wait_vmcnt<0>();
    lds_barrier();
    if (u + 1 < u1) issue(u + 1, stage ^ 1);
    compute(stage);
    stage ^= 1;
    if (ks == KT - 1 || u + 1 == u1) {
      const bool head = seg0 == t * KT;
      if (!head) {
        publish();                       // only ever this range's first segment
      } else {
        if (ks != KT - 1) {              // split tile, owned here: the range's last segment
          const int last = wg_of_unit(t * KT + KT - 1);
          for (int q = w + 1; q <= last; ++q) absorb(q);
        }
        epilogue(t);
      }
      zero_acc();
      seg0 = u + 1;
      ++t;
      ks = 0;
    } else {
      ++ks;
    }
  }
}

template <typename K_>
int launch_sk(const GemmP& p0, bool conv, void* ws, hipStream_t st) {
  GemmP p = p0;
  SkP s;
  s.kt = p.K / 64;
  s.tiles = p.tiles_m * p.tiles_n;
  s.units = s.tiles * s.kt;
  const int G = sk_grid(p);
  s.flags = (uint32_t*)ws;
  s.part = (float*)((char*)ws + SK_FLAG_BYTES);
  dim3 grid(G);
  const bool rowld = p.R1 || p.R2 || p.pos || p.accumulate;
#define DP_SK(C_, R_, L_) hipLaunchKernelGGL((gemm_sk_kernel<K_, C_, R_, L_>), grid, dim3(512), 0, st, p, s)
  if (rowld) {
    if (conv && p.relu_a) DP_SK(true, true, true);
    else if (conv) DP_SK(true, false, true);
    else if (p.relu_a) DP_SK(false, true, true);
    else DP_SK(false, false, true);
  } else {
    if (conv && p.relu_a) DP_SK(true, true, false);
    else if (conv) DP_SK(true, false, false);
    else if (p.relu_a) DP_SK(false, true, false);
    else DP_SK(false, false, false);
  }
#undef DP_SK
  DP_CHECK_LAUNCH();
  return 0;
}

// ========================================================== split-K (small grids, long K)
// Launch 1: the 256 x 256 big engine over tiles x ksplit workgroups, each a K-step range of one
// tile, raw fp32 partials into the workspace ([ksplit][M][N]); launch 2 (this kernel): every
// thread sums the ksplit partials of 2 rows x 8 columns in split order (deterministic) and runs
// the same row epilogue the engines use (bias, activation, gamma, pos, residuals, store mode).
// No workgroup ever waits for another (unlike the stream-K hand-off), so a split-K launch can
// run beside any other launch.
template <typename K_>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const GemmP p) {
  const int cpr = p.N / 8;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long pairs = (p.M + 1) / 2;
  if (idx >= pairs * cpr) return;
  const int rp = (int)(idx / cpr), n = (int)(idx - (long long)rp * cpr) * 8;
  int ms[2] = {2 * rp, 2 * rp + 1};
  float v[2][8];
  #pragma unroll
  for (int it = 0; it < 2; ++it)
    #pragma unroll
    for (int r = 0; r < 8; ++r) v[it][r] = 0.f;
  const long long slab = (long long)p.M * p.N;
  const bool two = ms[1] < p.M;
  const float* base = p.kpart + (long long)ms[0] * p.N + n;
  #pragma unroll 4
  for (int sp = 0; sp < p.ksplit; ++sp) {
    const float* q = base + sp * slab;
    const float4 a0 = *(const float4*)q, a1 = *(const float4*)(q + 4);
    float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
    if (two) { b0 = *(const float4*)(q + p.N); b1 = *(const float4*)(q + p.N + 4); }
    v[0][0] += a0.x; v[0][1] += a0.y; v[0][2] += a0.z; v[0][3] += a0.w;
    v[0][4] += a1.x; v[0][5] += a1.y; v[0][6] += a1.z; v[0][7] += a1.w;
    v[1][0] += b0.x; v[1][1] += b0.y; v[1][2] += b0.z; v[1][3] += b0.w;
    v[1][4] += b1.x; v[1][5] += b1.y; v[1][6] += b1.z; v[1][7] += b1.w;
  }
  ColConst cc;
  load_colconst(p, n, cc);
  epilogue_rows<K_, 2>(p, cc, ms, n, v);
}

template <typename K_>
int launch_splitk(const GemmP& p0, bool conv, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = p.N / 256;
  p.tiles_m = (p.M + 255) / 256;
  if (p.ksplit < 2 || !p.kpart || p.N % 256 != 0) return DP_ERR_ARG;
  dim3 g1(p.tiles_n * p.tiles_m * p.ksplit);
#define DP_SPK(C_, R_) hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 256, 64, 2, false, C_, R_, 8, -1, false, true>), g1, dim3(NT_BIG), 0, s, p)
  if (conv && p.relu_a) DP_SPK(true, true);
  else if (conv) DP_SPK(true, false);
  else if (p.relu_a) DP_SPK(false, true);
  else DP_SPK(false, false);
#undef DP_SPK
  DP_CHECK_LAUNCH();
  const long long threads = (long long)((p.M + 1) / 2) * (p.N / 8);
  hipLaunchKernelGGL(splitk_reduce_kernel<K_>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, p);
  DP_CHECK_LAUNCH();
  return 0;
}

// ========================================================== small-tile engine
constexpr int NT = 256;

template <typename K_, int BM, int BN, int WM, int WN, bool CONV>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(const GemmP p) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int CA = BM * 8 / NT;  // 16-B chunks per thread per A tile
  constexpr int CB = BN * 8 / NT;
  static_assert(CA >= 1 && CB >= 1 && WM * WN == 4, "tile config");
  __shared__ __attribute__((aligned(16))) u16 smem[2][(BM + BN) * BK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tile_n = blockIdx.x % p.tiles_n;
  const int tile_m = blockIdx.x / p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kc = tid & 7;      // 16-B chunk within a 64-wide K row
  const int rbase = tid >> 3;  // first row of this thread's chunks (step 32)

  const u16* a_ptr[CA];
  ConvRow a_cr[CA];
  #pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int m = m0 + rbase + 32 * i;
    if constexpr (!CONV) a_ptr[i] = p.A + (long long)(m < p.M ? m : p.M - 1) * p.lda + kc * 8;
    else a_cr[i] = conv_row(p, m);
  }
  const u16* b_ptr[CB];
  #pragma unroll
  for (int i = 0; i < CB; ++i) {
    int n = n0 + rbase + 32 * i;
    n = n < p.N ? n : p.N - 1;
    b_ptr[i] = p.B + (long long)n * p.ldb + kc * 8;
  }

  uint4 ra[CA], rb[CB];

  auto load_tile = [&](int k0) {
    if constexpr (!CONV) {
      #pragma unroll
      for (int i = 0; i < CA; ++i) ra[i] = *(const uint4*)(a_ptr[i] + k0);
    } else {
      int t_ky, t_kx, t_ci;
      conv_tap(p, k0, t_ky, t_kx, t_ci);
      #pragma unroll
      for (int i = 0; i < CA; ++i) {
        bool inb;
        const u16* s = conv_src(p, a_cr[i], t_ky, t_kx, t_ci + kc * 8, inb);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (inb) v = *(const uint4*)s;
        ra[i] = v;
      }
    }
    #pragma unroll
    for (int i = 0; i < CB; ++i) rb[i] = *(const uint4*)(b_ptr[i] + k0);
  };
  auto store_tile = [&](int buf) {
    u16* sa = smem[buf];
    u16* sb = smem[buf] + BM * BK;
    #pragma unroll
    for (int i = 0; i < CA; ++i) {
      uint4 v = ra[i];
      if (p.relu_a) v = relu_pk16(v);
      *(uint4*)(sa + lds_off(rbase + 32 * i, kc)) = v;
    }
    #pragma unroll
    for (int i = 0; i < CB; ++i) *(uint4*)(sb + lds_off(rbase + 32 * i, kc)) = rb[i];
  };

  f32x4_t acc[FM][FN];
  #pragma unroll
  for (int i = 0; i < FM; ++i)
    #pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int KT = p.K / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fchunk = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_tile((kt + 1) * BK);
    const u16* sa = smem[cur];
    const u16* sb = smem[cur] + BM * BK;
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 af[FM], bf[FN];
      #pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *(const uint4*)(sa + lds_off(wm * TM + i * 16 + frow, ks * 4 + fchunk));
      #pragma unroll
      for (int j = 0; j < FN; ++j)
        bf[j] = *(const uint4*)(sb + lds_off(wn * TN + j * 16 + frow, ks * 4 + fchunk));
      #pragma unroll
      for (int i = 0; i < FM; ++i)
        #pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = K_::mfma16(bf[j], af[i], acc[i][j]);
    }
    if (kt + 1 < KT) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds rows m = .. + (lane & 15), cols n = .. + 4*(lane >> 4) + r
  const int em = lane & 15;
  const int en = 4 * (lane >> 4);
  float hsum[FM];
  #pragma unroll
  for (int i = 0; i < FM; ++i) hsum[i] = 0.f;
  #pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm * TM + i * 16 + em;
    #pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + en;
      if (m >= p.M || n >= p.N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      epilogue4<K_>(p, m, n, v, hsum[i]);
    }
  }
  if (p.head_w) {
    // a row's channels live in lanes (lane&15) + 16*{0..3} of the wave (WN == 1)
    #pragma unroll
    for (int i = 0; i < FM; ++i) {
      float s = hsum[i];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      const int m = m0 + wm * TM + i * 16 + em;
      if ((lane >> 4) == 0 && m < p.M) ((float*)p.C)[m] = fmaxf(s + p.head_b, 0.f);
    }
  }
}

template <typename K_, int BM, int BN, int WM, int WN>
int launch_small(const GemmP& p0, bool conv, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  dim3 grid(p.tiles_n * tiles_m);
  if (conv)
    hipLaunchKernelGGL((gemm_kernel<K_, BM, BN, WM, WN, true>), grid, dim3(NT), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_kernel<K_, BM, BN, WM, WN, false>), grid, dim3(NT), 0, s, p);
  DP_CHECK_LAUNCH();
  return 0;
}

// NS = ring depth; PIPE = software-pipelined fragment reads (two register sets:
// only affordable for BN = 128, the 256x256 accumulators leave no room).
template <typename K_, int BM, int BN, int BKT, int NS, bool PIPE>
int launch_big(const GemmP& p0, bool conv, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_m = (p.M + BM - 1) / BM;
  dim3 grid(p.tiles_n * p.tiles_m);
  // the load-free epilogue for launches without per-row operands (needs_rowld), on the BK = 64
  // engines the planner picks; debug 1 << 20: always the general one (A/B)
  const int ea = BKT == 64 ? fast_epi_act(p) : -1;
  if (p.groups > 1) {
    // grouped launches (the side encoders' dense GEMMs) exist for the 256 x 128 / 128 x 128 dense engines
    if constexpr ((BM == 256 || BM == 128) && BN == 128 && BKT == 64 && NS == 3 && PIPE) {
      if (conv || p.relu_a) return DP_ERR_ARG;
      dim3 g(p.tiles_n * p.tiles_m * p.groups);
#define DP_GRP(E_) hipLaunchKernelGGL((gemm_big_kernel<K_, BM, BN, 64, 3, true, false, false, 8, E_, true>), g, dim3(NT_BIG), 0, s, p)
      if (ea == DP_ACT_NONE) DP_GRP(DP_ACT_NONE);
      else if (ea == DP_ACT_GELU) DP_GRP(DP_ACT_GELU);
      else if (ea == EPI_ACC) DP_GRP(EPI_ACC);
      else DP_GRP(-1);
#undef DP_GRP
      DP_CHECK_LAUNCH();
      return 0;
    } else {
      return DP_ERR_ARG;
    }
  }
#define DP_BIGE(C_, R_, E_) hipLaunchKernelGGL((gemm_big_kernel<K_, BM, BN, BKT, NS, PIPE, C_, R_, 8, E_>), grid, dim3(NT_BIG), 0, s, p)
#define DP_BIG(C_, R_) do { \
    if (ea < 0) DP_BIGE(C_, R_, -1); \
    else if constexpr (BKT == 64) { \
      if (ea == DP_ACT_NONE) DP_BIGE(C_, R_, DP_ACT_NONE); \
      else if (ea == DP_ACT_RELU) DP_BIGE(C_, R_, DP_ACT_RELU); \
      else if (ea == DP_ACT_GELU) DP_BIGE(C_, R_, DP_ACT_GELU); \
      else if constexpr (!C_ && !R_) { if (ea == EPI_ACC) DP_BIGE(C_, R_, EPI_ACC); else DP_BIGE(C_, R_, -1); } \
      else DP_BIGE(C_, R_, -1); } \
  } while (0)
  if (conv && p.relu_a) DP_BIG(true, true);
  else if (conv) DP_BIG(true, false);
  else if (p.relu_a) DP_BIG(false, true);
  else DP_BIG(false, false);
#undef DP_BIG
#undef DP_BIGE
  DP_CHECK_LAUNCH();
  return 0;
}

// two 4-wave workgroups per CU (tile 256 x 128, BK 32, 3-stage ring)
template <typename K_>
int launch_dual(const GemmP& p0, bool conv, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = (p.N + 127) / 128;
  p.tiles_m = (p.M + 255) / 256;
  dim3 grid(p.tiles_n * p.tiles_m);
  if (conv && p.relu_a)
    hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, true, true, 4>), grid, dim3(256), 0, s, p);
  else if (conv)
    hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, true, false, 4>), grid, dim3(256), 0, s, p);
  else {
    const int ea = fast_epi_act(p);
    if (p.relu_a)
      hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, false, true, 4>), grid, dim3(256), 0, s, p);
    else if (ea == DP_ACT_NONE)
      hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, false, false, 4, DP_ACT_NONE>), grid, dim3(256), 0, s, p);
    else if (ea == DP_ACT_GELU)
      hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, false, false, 4, DP_ACT_GELU>), grid, dim3(256), 0, s, p);
    else if (ea == EPI_ACC)
      hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, false, false, 4, EPI_ACC>), grid, dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_big_kernel<K_, 256, 128, 32, 3, false, false, false, 4>), grid, dim3(256), 0, s, p);
  }
  DP_CHECK_LAUNCH();
  return 0;
}

template <typename K_, int BM, int BN>
int launch_pbig(const GemmP& p0, bool conv, hipStream_t s) {
  GemmP p = p0;
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_m = (p.M + BM - 1) / BM;
  const int T = p.tiles_n * p.tiles_m;
  int G = num_cus();
  if (G > T) G = T;
  dim3 grid(G);
  const bool rowld = p.R1 || p.R2 || p.pos || p.accumulate;
#define DP_PB(C_, R_, L_) hipLaunchKernelGGL((gemm_pbig_kernel<K_, BM, BN, C_, R_, L_>), grid, dim3(NT_BIG), 0, s, p)
  if (rowld) {
    if (conv && p.relu_a) DP_PB(true, true, true);
    else if (conv) DP_PB(true, false, true);
    else if (p.relu_a) DP_PB(false, true, true);
    else DP_PB(false, false, true);
  } else {
    if (conv && p.relu_a) DP_PB(true, true, false);
    else if (conv) DP_PB(true, false, false);
    else if (p.relu_a) DP_PB(false, true, false);
    else DP_PB(false, false, false);
  }
#undef DP_PB
  DP_CHECK_LAUNCH();
  return 0;
}

}  // namespace
