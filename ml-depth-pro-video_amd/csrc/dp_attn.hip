// dp_attention: flash-style multi-head attention for the DINOv2 ViT-L blocks
// (seq 577, head_dim 64, 16 heads) on gfx950.
//
// One workgroup = 4 wave64s = 128 queries of one (image, head); each wave owns
// 32 queries.  Per 64-key tile the wave computes S^T = K . Q^T with
// v_mfma_f32_32x32x16 (keys on the accumulator rows, its query on the lane), so
// the online-softmax statistics are lane-local up to one permlane32 swap, and
// the S^T accumulator registers, packed to 16 bits, are directly the B operand
// of O^T = V^T . P^T (in a permuted key order that the V^T fragment matches).
// K is staged row-major (padded rows, ds_read_b128); V is staged row-major too
// and read transposed with ds_read_b64_tr_b16 (64-B halves XOR-swizzled on odd
// row pairs: conflict-free).  Registers stage the next tile's K/V from HBM while
// the current tile computes (one barrier per tile); Q stays in registers.
// Softmax: scale folded into one FMA per score, exp2, a deferred running-max
// rescale, and row sums taken by the matrix core (an all-ones V^T block).
// The last, partial key tile is masked and skips its empty 32-key half.
#include <type_traits>

#include "dp_common.h"

namespace {

constexpr int QB = 128;      // queries per workgroup
constexpr int KT = 64;       // keys per tile
constexpr int HD = 64;       // head dim
constexpr int KS = 72;       // K tile row stride (elements): conflict-free b128 reads
constexpr int VRB = 128;     // V tile row bytes (64 d x 16 bit), swizzled

typedef short v4s_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int v_off(int row, int byte) {  // byte offset of (key row, byte in row)
  return row * VRB + (byte ^ (((row >> 1) & 1) << 6));
}

template <typename K_>
__global__ void __launch_bounds__(256, 3)
attn_kernel(const u16* __restrict__ qkv, u16* __restrict__ out, int seq, int heads, int nq, float sl2) {
  __shared__ __attribute__((aligned(16))) u16 sk[2][KT * KS];
  __shared__ __attribute__((aligned(16))) char sv[2][KT * VRB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware remap: workgroup i is dispatched to XCD i % 8, so consecutive work
  // items are handed to the SAME XCD; the nq query blocks of one (image, head),
  // consecutive here, then share that head's K/V panel in one L2 instead of
  // fetching it nq times from the fabric (measured: 455 -> ~130 MB per launch).
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int qblk = wid % nq, bh = wid / nq;
  const int h = bh % heads, b = bh / heads;
  const long long ldq = 3LL * heads * HD;
  const long long ldo = (long long)heads * HD;
  const u16* base = qkv + (long long)b * seq * ldq;
  const int qcol = h * HD, kcol = heads * HD + h * HD, vcol = 2 * heads * HD + h * HD;

  const int l32 = lane & 31, hi = lane >> 5;
  const int q = qblk * QB + wave * 32 + l32;
  // a wave whose 32 queries are all past seq (tail block) only helps stage K/V
  const bool active = __builtin_amdgcn_readfirstlane(qblk * QB + wave * 32) < seq;

  // Q fragments (B operand of S^T = K Q^T): Q[q][16*ks + 8*hi + 0..7]
  uint4 qf[4];
  #pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = make_uint4(0, 0, 0, 0);
    if (q < seq) qf[ks] = *(const uint4*)(base + (long long)q * ldq + qcol + 16 * ks + 8 * hi);
  }

  // staging: thread -> (key row, 16-B d chunk) x 2.  Full tiles load without a
  // predicate from row pointers that advance by one tile per step.
  const int srow = tid >> 3, sch = tid & 7;
  uint4 rk[2], rv[2];
  const u16* kp = base + (long long)srow * ldq + kcol + 8 * sch;
  const long long vk = vcol - kcol, row32 = 32 * ldq, tile_step = KT * ldq;
  auto load = [&](int k0, bool full) {
    const u16* r = kp + (long long)k0 * ldq;
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (full || k0 + srow + 32 * i < seq) {
        rk[i] = *(const uint4*)(r + i * row32);
        rv[i] = *(const uint4*)(r + i * row32 + vk);
      } else {
        rk[i] = make_uint4(0, 0, 0, 0);
        rv[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  (void)tile_step;
  auto store = [&](int buf) {
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = srow + 32 * i;
      *(uint4*)(&sk[buf][key * KS + 8 * sch]) = rk[i];
      *(uint4*)(&sv[buf][v_off(key, 16 * sch)]) = rv[i];
    }
  };
  // transposed V read address (bytes, within a stage) for the A operand of
  // O^T = V^T P^T: d block db, key step (kb, st), first/second 4-key group g2
  const int grp = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  auto vt_addr = [&](int db, int k0, int g2) {
    const int row = k0 + 4 * hi + 8 * g2 + tq;
    const int byte = 2 * (db * 32 + 16 * (grp & 1) + 4 * tp);
    return v_off(row, byte);
  };

  f32x16_t o[2], osum;   // osum: row sums of P, from an all-ones A operand (every row equal)
  #pragma unroll
  for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; osum[i] = 0.f; }
  const uint32_t one2 = K_::pack2(1.f, 1.f);
  const uint4 ones = make_uint4(one2, one2, one2, one2);
  float m_run = -1e30f;

  // One 64-key tile.  PARTIAL (the last tile when seq % 64 != 0): keys past seq
  // are masked, and the second 32-key half is skipped when it holds none.
  auto do_tile = [&](int t, auto partial_tag) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    if (!active) return;
    const int cur = t & 1;
    const int kbase = t * KT;
    const u16* K = sk[cur];
    const char* V = sv[cur];
    const bool two = !PARTIAL || kbase + 32 < seq;
    // ---- S^T for the two 32-key blocks
    f32x16_t s[2];
    #pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (PARTIAL && kb == 1 && !two) {
        #pragma unroll
        for (int i = 0; i < 16; ++i) s[1][i] = -INFINITY;
        break;
      }
      #pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const uint4 kf = *(const uint4*)(K + (kb * 32 + l32) * KS + 16 * ks + 8 * hi);
        s[kb] = K_::mfma32(kf, qf[ks], ks == 0 ? f32x16_t{} : s[kb]);
      }
    }
    if constexpr (PARTIAL) {
      #pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        #pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kbase + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          if (key >= seq) s[kb][r] = -INFINITY;
        }
    }
    // ---- online softmax (this lane's query; rows = keys)
    float mx = fmaxf(s[0][0], s[0][1]);
    #pragma unroll
    for (int r = 2; r < 16; ++r) mx = fmaxf(mx, s[0][r]);
    #pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[1][r]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    // Deferred rescale: the reference max m_run moves only when a row's max
    // exceeds it by more than 8 (log2 units), so P = 2^(s - m_run) <= 256 and
    // the O / row-sum rescale (and its exp) is skipped on most tiles.  P is
    // rounded to 16 bits relative to its own magnitude either way.
    const float m_new = mx * sl2;
    if (__builtin_amdgcn_ballot_w64(m_new > m_run + 8.f)) {
      const float m_upd = fmaxf(m_run, m_new);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_upd);
      #pragma unroll
      for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; osum[i] *= alpha; }
      m_run = m_upd;
    }
    uint4 pf[2][2];
    #pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      #pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint32_t w[4];
        #pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(s[kb][8 * st + 2 * jj], sl2, -m_run));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(s[kb][8 * st + 2 * jj + 1], sl2, -m_run));
          w[jj] = K_::pack2(p0, p1);
        }
        pf[kb][st] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    // ---- O^T += V^T P^T
    #pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (PARTIAL && kb == 1 && !two) break;
      #pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int k0 = kb * 32 + 16 * st;
        #pragma unroll
        for (int db = 0; db < 2; ++db) {
          const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s_t*)(V + vt_addr(db, k0, 0)));
          const v4s_t up = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s_t*)(V + vt_addr(db, k0, 1)));
          const uint2 a = __builtin_bit_cast(uint2, lo), c = __builtin_bit_cast(uint2, up);
          o[db] = K_::mfma32(make_uint4(a.x, a.y, c.x, c.y), pf[kb][st], o[db]);
        }
        osum = K_::mfma32(ones, pf[kb][st], osum);
      }
    }
  };

  const int ntiles = (seq + KT - 1) / KT, nfull = seq / KT;
  load(0, nfull > 0);
  store(0);
  __syncthreads();
  for (int t = 0; t < nfull; ++t) {
    if (t + 1 < ntiles) load((t + 1) * KT, t + 1 < nfull);
    do_tile(t, std::false_type{});
    if (t + 1 < ntiles) store((t & 1) ^ 1);
    __syncthreads();
  }
  if (nfull < ntiles) {
    do_tile(nfull, std::true_type{});
    __syncthreads();
  }
  // ---- normalise and store: stage the wave's 32 x 64 output through LDS so each
  // query row leaves as whole 128-B lines
  const float inv = 1.f / osum[0];
  u16* stg = (u16*)&sk[0][0] + wave * 32 * KS;   // 32 rows x KS (padded) per wave
  #pragma unroll
  for (int db = 0; db < 2; ++db)
    #pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = db * 32 + 8 * g + 4 * hi;
      uint2 w;
      w.x = K_::pack2(o[db][4 * g] * inv, o[db][4 * g + 1] * inv);
      w.y = K_::pack2(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
      *(uint2*)(stg + l32 * KS + d) = w;
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave reads back only its own rows
  #pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = i * 8 + (lane >> 3), ch = lane & 7;
    const int qq = qblk * QB + wave * 32 + row;
    const uint4 v = *(const uint4*)(stg + row * KS + 8 * ch);
    if (qq < seq) *(uint4*)(out + ((long long)b * seq + qq) * ldo + h * HD + 8 * ch) = v;
  }
}

}  // namespace

extern "C" int dp_attention(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads,
                            int32_t head_dim, float scale, int32_t dtype, dp_stream_t stream) {
  if (!qkv || !out) return DP_ERR_ARG;
  if (batch <= 0 || seq <= 0 || heads <= 0 || head_dim != HD) return DP_ERR_SHAPE;
  const int nq = (seq + QB - 1) / QB;
  if ((long long)nq * heads * batch > 0x7fffffffLL) return DP_ERR_SHAPE;
  dim3 grid(nq * heads * batch);
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(attn_kernel<KBF16>, grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, nq, sl2);
  else if (dtype == DP_F16)
    hipLaunchKernelGGL(attn_kernel<KF16>, grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, nq, sl2);
  else
    return DP_ERR_DTYPE;
  DP_CHECK_LAUNCH();
  return 0;
}
