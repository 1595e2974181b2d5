// dp_attention: flash-style multi-head attention for the DINOv2 ViT-L blocks
// (seq 577, head_dim 64, 16 heads) on gfx950.
//
// One workgroup = 4 wave64s = 128 queries of one (image, head); each wave owns
// 32 queries.  Per 64-key tile the wave computes S^T = K . Q^T with
// v_mfma_f32_32x32x16 (keys on the accumulator rows, its query on the lane),
// so the online-softmax row statistics are lane-local (one cross-half
// exchange), and the S^T accumulator registers are directly the B operand of
// O^T = V^T . P^T (the register k-order permutation is matched by the order in
// which the V^T fragment is read).  K is staged row-major and V transposed in
// LDS (double-buffered, one barrier per tile); Q stays in registers.
#include "dp_common.h"

namespace {

constexpr int QB = 128;      // queries per workgroup
constexpr int KT = 64;       // keys per tile
constexpr int HD = 64;       // head dim
constexpr int KS = 72;       // K tile row stride (elements): conflict-free b128 reads
constexpr int VS = 68;       // V^T tile row stride (elements): conflict-free b64 reads

template <typename K_>
__global__ void __launch_bounds__(256, 2)
attn_kernel(const u16* __restrict__ qkv, u16* __restrict__ out, int seq, int heads, float sl2) {
  __shared__ __attribute__((aligned(16))) u16 sk[2][KT * KS];
  __shared__ __attribute__((aligned(16))) u16 sv[2][HD * VS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const long long ldq = 3LL * heads * HD;
  const long long ldo = (long long)heads * HD;
  const u16* base = qkv + (long long)b * seq * ldq;
  const int qcol = h * HD, kcol = heads * HD + h * HD, vcol = 2 * heads * HD + h * HD;

  const int l32 = lane & 31, hi = lane >> 5;
  const int q = blockIdx.x * QB + wave * 32 + l32;

  // Q fragments (B operand of S^T = K Q^T): Q[q][16*ks + 8*hi + 0..7]
  uint4 qf[4];
  #pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = make_uint4(0, 0, 0, 0);
    if (q < seq) qf[ks] = *(const uint4*)(base + (long long)q * ldq + qcol + 16 * ks + 8 * hi);
  }

  // staging: thread -> (key row, 16-B d chunk) x 2
  const int srow = tid >> 3, sch = tid & 7;
  uint4 rk[2], rv[2];
  auto load = [&](int k0) {
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
      int key = k0 + srow + 32 * i;
      rk[i] = make_uint4(0, 0, 0, 0);
      rv[i] = make_uint4(0, 0, 0, 0);
      if (key < seq) {
        const u16* r = base + (long long)key * ldq;
        rk[i] = *(const uint4*)(r + kcol + 8 * sch);
        rv[i] = *(const uint4*)(r + vcol + 8 * sch);
      }
    }
  };
  auto store = [&](int buf) {
    #pragma unroll
    for (int i = 0; i < 2; ++i) {
      int key = srow + 32 * i;
      *(uint4*)(&sk[buf][key * KS + 8 * sch]) = rk[i];
      const uint32_t w4[4] = {rv[i].x, rv[i].y, rv[i].z, rv[i].w};
      #pragma unroll
      for (int j = 0; j < 8; ++j)
        sv[buf][(8 * sch + j) * VS + key] = (u16)(w4[j >> 1] >> (16 * (j & 1)));
    }
  };

  f32x16_t o[2];
  #pragma unroll
  for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
  float m_run = -1e30f, l_run = 0.f;

  const int ntiles = (seq + KT - 1) / KT;
  load(0);
  store(0);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load((t + 1) * KT);
    const u16* K = sk[cur];
    const u16* V = sv[cur];
    // ---- S^T for the two 32-key blocks
    f32x16_t s[2];
    #pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      #pragma unroll
      for (int i = 0; i < 16; ++i) s[kb][i] = 0.f;
      #pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        uint4 kf = *(const uint4*)(K + (kb * 32 + l32) * KS + 16 * ks + 8 * hi);
        s[kb] = K_::mfma32(kf, qf[ks], s[kb]);
      }
    }
    // ---- online softmax (this lane's query; rows = keys)
    const int kbase = t * KT;
    float mx = -INFINITY;
    #pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      #pragma unroll
      for (int r = 0; r < 16; ++r) {
        int key = kbase + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        float v = key < seq ? s[kb][r] * sl2 : -INFINITY;
        s[kb][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    float ls = 0.f;
    uint4 pf[2][2];
    #pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      #pragma unroll
      for (int st = 0; st < 2; ++st) {
        uint32_t w[4];
        #pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float p0 = __builtin_amdgcn_exp2f(s[kb][8 * st + 2 * jj] - m_new);
          float p1 = __builtin_amdgcn_exp2f(s[kb][8 * st + 2 * jj + 1] - m_new);
          u16 b0 = K_::from_f(p0), b1 = K_::from_f(p1);
          ls += K_::to_f(b0) + K_::to_f(b1);
          w[jj] = (uint32_t)b0 | ((uint32_t)b1 << 16);
        }
        pf[kb][st] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    ls += __shfl_xor(ls, 32);
    l_run = l_run * alpha + ls;
    m_run = m_new;
    #pragma unroll
    for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
    // ---- O^T += V^T P^T
    #pragma unroll
    for (int db = 0; db < 2; ++db) {
      const u16* vrow = V + (db * 32 + l32) * VS + 4 * hi;
      #pragma unroll
      for (int kb = 0; kb < 2; ++kb)
        #pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int k0 = kb * 32 + 16 * st;
          uint2 lo = *(const uint2*)(vrow + k0);
          uint2 hi2 = *(const uint2*)(vrow + k0 + 8);
          o[db] = K_::mfma32(make_uint4(lo.x, lo.y, hi2.x, hi2.y), pf[kb][st], o[db]);
        }
    }
    if (t + 1 < ntiles) store(cur ^ 1);
    __syncthreads();
  }
  if (q >= seq) return;
  const float inv = 1.f / l_run;
  u16* orow = out + ((long long)b * seq + q) * ldo + h * HD;
  #pragma unroll
  for (int db = 0; db < 2; ++db)
    #pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = db * 32 + 8 * g + 4 * hi;
      uint2 w;
      w.x = (uint32_t)K_::from_f(o[db][4 * g] * inv) | ((uint32_t)K_::from_f(o[db][4 * g + 1] * inv) << 16);
      w.y = (uint32_t)K_::from_f(o[db][4 * g + 2] * inv) | ((uint32_t)K_::from_f(o[db][4 * g + 3] * inv) << 16);
      *(uint2*)(orow + d) = w;
    }
}

}  // namespace

extern "C" int dp_attention(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads,
                            int32_t head_dim, float scale, int32_t dtype, dp_stream_t stream) {
  if (!qkv || !out) return DP_ERR_ARG;
  if (batch <= 0 || seq <= 0 || heads <= 0 || head_dim != HD) return DP_ERR_SHAPE;
  if (batch > 65535 || heads > 65535) return DP_ERR_SHAPE;
  dim3 grid((seq + QB - 1) / QB, heads, batch);
  const float sl2 = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(attn_kernel<KBF16>, grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, sl2);
  else if (dtype == DP_F16)
    hipLaunchKernelGGL(attn_kernel<KF16>, grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, sl2);
  else
    return DP_ERR_DTYPE;
  DP_CHECK_LAUNCH();
  return 0;
}
