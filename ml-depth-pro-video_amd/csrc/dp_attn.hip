// dp_attention: flash-style multi-head attention for the DINOv2 ViT-L blocks
// (seq 577, head_dim 64, 16 heads) on gfx950.
//
// One workgroup = 4 wave64s = 128 queries of one (image, head); each wave owns
// 32 queries.  Per 64-key tile the wave computes S^T = K . Q^T with
// v_mfma_f32_32x32x16 (keys on the accumulator rows, its query on the lane), so
// the online-softmax statistics are lane-local up to one permlane32 swap, and
// the S^T accumulator registers, packed to 16 bits, are directly the B operand
// of O^T = V^T . P^T (in a permuted key order that the V^T fragment matches).
// K and V tiles travel HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction, no staging registers): the next tile's DMA is in flight while
// the current tile computes, one counted wait + barrier per tile.  Both are stored
// as 128-B key rows with the 16-B chunk XOR-swizzled on the SOURCE address: K by
// (row >> 1) & 7 (conflict-free ds_read_b128 of 16 rows), V by 64-B halves on odd
// row pairs, read transposed with ds_read_b64_tr_b16 (conflict-free).  Q stays in
// registers; 3 workgroups (12 waves) per CU, 152 VGPRs: in the steady state both halves' S^T
// MFMAs go first (K fragments read up front), so the second half's run on the matrix core while
// the first half's softmax runs on the VALU (4 workgroups at 128 VGPRs left the compiler no room
// to overlap them: 66.2 -> 64.2 us, profiles/r04q_attn_3wg/).
// Softmax in log2 units: one FMA + exp2 per score against a running max that only the
// first half key tile sets (an overflow, checked once at the end, sends the workgroup
// through an exact per-tile-max pass), VALU row sums.
// A last, partial key tile is masked and skips its empty 32-key half; one or two
// leftover keys (the ViT's 577 = 9 x 64 + 1) go through the VALU instead (tail_key).
#include <type_traits>

#include "dp_common.h"

namespace {

constexpr int QB = 128;      // queries per workgroup
constexpr int KT = 64;       // keys per tile
constexpr int HD = 64;       // head dim
constexpr int KS = 72;       // output staging row stride (elements): conflict-free b128 reads
constexpr int VRB = 128;     // K / V tile row bytes (64 d x 16 bit), swizzled
constexpr int TILE_B = KT * VRB;   // 8 KiB per operand tile
constexpr int TAIL_VALU = 2;       // leftover keys handled on the VALU instead of a partial tile

typedef short v4s_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int v_off(int row, int byte) {  // byte offset of (key row, byte in row)
  return row * VRB + (byte ^ (((row >> 1) & 1) << 6));
}
__device__ __forceinline__ int k_off(int row, int chunk) {  // byte offset of (key row, 16-B chunk)
  return row * VRB + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// one 16-B-per-lane LDS-DMA piece at the wave-uniform LDS byte address `dst`
// (inline asm: completion is tracked by the counted vmcnt wait in the tile loop)
__device__ __forceinline__ void glds16(const void* src, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}
// the same with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset
// (saddr form): a full tile's addresses are one scalar add away from the last tile's
__device__ __forceinline__ void glds16s(uint32_t voff, const void* sbase, uint32_t dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(dst)
      : "memory");
}

// Running max (m_run, log2 units), set exactly by the first 32-key half tile only; every
// later score is taken as P = 2^(s sl2 - m_run) with no max pass, no compare and no rescale.
// P only has to stay representable (16-bit B operand, fp32 sums), and a later key beyond that
// range (> ~127 log2 units above the first half tile's max for bf16, > ~16 for f16) makes the
// row sum or O non-finite: the workgroup then runs its keys again on the exact path (the
// per-half-tile max and deferred rescale: m_run moves when exceeded by > 8, so P <= 256) --
// rare on real inputs, checked once.
// Row sums of P: f32 VALU adds as ONE serial v_add_f32 chain (nothing independent and
// isomorphic for the compiler to SLP-pack into v_pk_add_f32, which costs more issue beside
// MFMAs).  Not inline asm: an asm add that reads a v_exp_f32 result right away misses the
// transcendental-use wait state the compiler inserts for its own instructions.
// PRE: the Q columns of qkv already hold Q * scale * log2(e) (dp_attention_log2q: the qkv
// GEMM's per-column gamma), so scores come out of the MFMA in log2 units; once the running
// max is set, the S^T accumulator starts at -m_run instead of 0 and P = 2^S^T is ONE v_exp_f32
// per score.
// Measured and rejected (round 2): software-prefetched fragments (3 workgroups per CU), a
// 3-deep K/V ring, packed row-sum adds, row sums on the matrix core (profiles/r02l_attn_pf/,
// r02z6_attn_nst3/, r02p_attn_sadd/).
// Ablation build only (make attnexp: -DDP_ATTN_ABLATE, tools/attn_bench.py --ablate): `dbg` bits
// drop one stage each (outputs invalid) -- 1 the exp2, 2 the P.V MFMAs, 4 the per-tile wait +
// barrier, 8 the K/V LDS-DMA (and the wait), 16 the row-sum adds.  The product build ignores it.
#ifdef DP_ATTN_ABLATE
#define ABL(b) (dbg & (b))
#else
#define ABL(b) false
#endif

template <typename K_, bool PRE>
__global__ void __launch_bounds__(256, 3)
attn_kernel(const u16* __restrict__ qkv, u16* __restrict__ out, int seq, int heads, int nq, float sl2, int dbg) {
  __shared__ __attribute__((aligned(1024))) char smem[2][2 * TILE_B];   // [stage][K tile | V tile]
  auto stage_of = [](int t) { return t & 1; };
  __shared__ int redo;

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
  if (tid == 0) redo = 0;

  // Q fragments (B operand of S^T = K Q^T): Q[q][16*ks + 8*hi + 0..7]
  uint4 qf[4];
  #pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = make_uint4(0, 0, 0, 0);
    if (q < seq) qf[ks] = *(const uint4*)(base + (long long)q * ldq + qcol + 16 * ks + 8 * hi);
  }
  // Q has landed (a wait the compiler sees): otherwise its own vmcnt(0) for Q's
  // first use lands inside the tile loop, where it also waits for the next tile's
  // LDS-DMA (inline asm, invisible to it) and serialises that latency every tile.
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)

  // LDS-DMA staging: piece i of wave w fills key rows 32 i + 8 w + lane / 8, slot
  // lane % 8 of each 128-B row; the slot holds logical chunk slot ^ swizzle(row), so
  // the swizzle lives in the source address.  Rows past seq re-read row seq-1
  // (finite, masked to -inf / weight 0 in the partial tile).
  const int prow = wave * 8 + (lane >> 3), pslot = lane & 7;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_u32(&smem[0][0]) + wave * 1024);
  // full tiles: per-lane byte offsets of the K / V pieces from the tile's first key row (rows
  // prow and prow + 32 share the swizzle) off a wave-uniform tile base; the partial tile clamps
  // its rows past seq to row seq-1 (64-bit per-lane addresses)
  const uint32_t voff_k = (uint32_t)(2 * (prow * ldq + kcol + 8 * (pslot ^ ((prow >> 1) & 7))));
  const uint32_t voff_v = (uint32_t)(2 * (prow * ldq + vcol + 8 * (pslot ^ (((prow >> 1) & 1) << 2))));
  auto issue = [&](int k0, int buf, auto full_tag) __attribute__((always_inline)) {
    if (ABL(8)) return;
    const uint32_t dk = __builtin_amdgcn_readfirstlane(lds0 + buf * 2 * TILE_B), dv = dk + TILE_B;
    if constexpr (decltype(full_tag)::value) {
      const u16* r0 = base + (long long)k0 * ldq;
      const u16* r1 = r0 + 32 * ldq;
      glds16s(voff_k, r0, dk);
      glds16s(voff_v, r0, dv);
      glds16s(voff_k, r1, dk + 4096);
      glds16s(voff_v, r1, dv + 4096);
    } else {
      #pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = prow + 32 * i;
        const int key = min(k0 + row, seq - 1);
        const u16* r = base + (long long)key * ldq;
        glds16(r + kcol + 8 * (pslot ^ ((row >> 1) & 7)), dk + i * 4096);
        glds16(r + vcol + 8 * (pslot ^ (((row >> 1) & 1) << 2)), dv + i * 4096);
      }
    }
  };
  // transposed V read address (bytes, within a stage) for the A operand of
  // O^T = V^T P^T: d block db, key step (kb, st), first/second 4-key group g2
  const int grp = lane >> 4, gi = lane & 15;
  const int tq = gi >> 2, tp = gi & 3;
  auto vt_addr = [&](int db, int k0, int g2) __attribute__((always_inline)) {
    const int row = k0 + 4 * hi + 8 * g2 + tq;
    const int byte = 2 * (db * 32 + 16 * (grp & 1) + 4 * tp);
    return v_off(row, byte);
  };

  f32x16_t o[2];
  float ls4[4];                // this lane's share of its query's row sum (its 32 of 64 keys)
  float m_run;

  auto rescale = [&](float m_upd) __attribute__((always_inline)) {   // m_run -> m_upd (>= m_run)
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_upd);
    #pragma unroll
    for (int i = 0; i < 16; ++i) {
      o[0][i] *= alpha; o[1][i] *= alpha;
    }
    #pragma unroll
    for (int i = 0; i < 4; ++i) ls4[i] *= alpha;
    m_run = m_upd;
  };

  // One 32-key half (kb) of a 64-key tile: S^T = K Q^T, softmax, O^T += V^T P^T; halves go
  // one after the other so only 16 score registers are live.  PARTIAL (the last tile when
  // seq % 64 != 0): keys past seq are masked.  setmax: take this half tile's max (exact:
  // every half tile, with the deferred rescale; lazy: the first one, which sets m_run).
  // `exact` is a workgroup-uniform runtime flag, so the redo pass reuses this code.
  // S^T of one 32-key half: 4 chained MFMAs (accumulator started at -m_run when `off`)
  auto score = [&](int t, int kb, bool off) __attribute__((always_inline)) {
    const char* K = smem[stage_of(t)];
    f32x16_t s;
    uint4 kf[4];     // the half's K fragments read up front: one LDS latency, not four
    #pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[ks] = *(const uint4*)(K + k_off(kb * 32 + l32, 2 * ks + hi));
    #pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      f32x16_t c0 = f32x16_t{};
      if (off) {
        #pragma unroll
        for (int r = 0; r < 16; ++r) c0[r] = -m_run;
      }
      s = K_::mfma32(kf[ks], qf[ks], ks == 0 ? c0 : s);
    }
    return s;
  };
  // the rest of a half: mask, max, P = 2^S, row sums, O^T += V^T P^T
  auto finish = [&](int t, int kb, f32x16_t s, auto partial_tag, bool setmax, bool exact)
                    __attribute__((always_inline)) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    const int cur = stage_of(t);
    const int kbase = t * KT;
    const char* V = smem[cur] + TILE_B;
    const bool off = PRE && !setmax && !exact;
    if constexpr (PARTIAL) {
      #pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (key >= seq) s[r] = -INFINITY;
      }
    }
    if (setmax) {
      // this lane's query; its other 16 keys of the half tile are in lane ^ 32
      float mx = fmaxf(s[0], s[1]);
      #pragma unroll
      for (int r = 2; r < 16; ++r) mx = fmaxf(mx, s[r]);
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      const float m_new = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * sl2;
      if (exact) {
        if (__builtin_amdgcn_ballot_w64(m_new > m_run + 8.f)) rescale(fmaxf(m_run, m_new));
      } else {
        m_run = m_new;   // the first half tile holds a valid key for every lane: finite
      }
    }
    uint4 pf[2];
    #pragma unroll
    for (int st = 0; st < 2; ++st) {
      uint32_t w[4];
      #pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        float p0, p1;
        if (ABL(1)) {
          p0 = s[8 * st + 2 * jj];
          p1 = s[8 * st + 2 * jj + 1];
        } else if (off) {
          p0 = __builtin_amdgcn_exp2f(s[8 * st + 2 * jj]);
          p1 = __builtin_amdgcn_exp2f(s[8 * st + 2 * jj + 1]);
        } else {
          p0 = __builtin_amdgcn_exp2f(fmaf(s[8 * st + 2 * jj], sl2, -m_run));
          p1 = __builtin_amdgcn_exp2f(fmaf(s[8 * st + 2 * jj + 1], sl2, -m_run));
        }
        w[jj] = K_::pack2(p0, p1);
        if (!ABL(16)) ls4[0] = (ls4[0] + p0) + p1;
      }
      pf[st] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (ABL(2)) {   // keep P live without the P.V stage
      asm volatile("" ::"v"(pf[0].x), "v"(pf[0].y), "v"(pf[0].z), "v"(pf[0].w), "v"(pf[1].x), "v"(pf[1].y),
                   "v"(pf[1].z), "v"(pf[1].w));
      return;
    }
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
        o[db] = K_::mfma32(make_uint4(a.x, a.y, c.x, c.y), pf[st], o[db]);
      }
    }
  };
  auto do_half = [&](int t, int kb, auto partial_tag, bool setmax, bool exact) __attribute__((always_inline)) {
    finish(t, kb, score(t, kb, PRE && !setmax && !exact), partial_tag, setmax, exact);
  };
  // a 64-key tile = two halves; the second half of a partial tile is skipped when it holds no key
  auto do_tile = [&](int t, auto partial_tag, bool first, bool exact) __attribute__((always_inline)) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    if (!active) return;
    const bool two = !PARTIAL || t * KT + 32 < seq;
    if (!PARTIAL && PRE && !first && !exact) {
      // steady state (running max fixed): both halves' S^T MFMAs first, so the second half's
      // run on the matrix core while the first half's softmax runs on the VALU
      const f32x16_t s0 = score(t, 0, true);
      const f32x16_t s1 = score(t, 1, true);
      finish(t, 0, s0, partial_tag, false, false);
      finish(t, 1, s1, partial_tag, false, false);
      return;
    }
    do_half(t, 0, partial_tag, exact || first, exact);
    if (two) do_half(t, 1, partial_tag, exact, exact);
  };

  // One leftover key (seq = 64 n + r, r <= TAIL_VALU: the ViT's 577 = 9 x 64 + 1) costs a
  // whole masked MFMA tile on the partial path; on the VALU it is a 64-d dot product per
  // query (each lane holds half of its query's dims: FMAs + one permlane32 swap), the same
  // online-softmax update, and a rank-1 update of O (p rounded to 16 bits like the MFMA path's P).
  auto tail_key = [&](int key) __attribute__((always_inline)) {
    const u16* kr = base + (long long)key * ldq + kcol;
    const u16* vr = base + (long long)key * ldq + vcol;
    float dot = 0.f;
    #pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 kv = *(const uint4*)(kr + 16 * ks + 8 * hi);
      const uint32_t kw[4] = {kv.x, kv.y, kv.z, kv.w};
      const uint32_t qw[4] = {qf[ks].x, qf[ks].y, qf[ks].z, qf[ks].w};
      #pragma unroll
      for (int j = 0; j < 4; ++j) {
        dot = fmaf(K_::to_f(qw[j] & 0xffff), K_::to_f(kw[j] & 0xffff), dot);
        dot = fmaf(K_::to_f(qw[j] >> 16), K_::to_f(kw[j] >> 16), dot);
      }
    }
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dot), __float_as_uint(dot), false, false);
      dot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    const float sc = dot * sl2;
    // m_run = -inf before any key (no MFMA tile ran): the first key always sets it
    if (__builtin_amdgcn_ballot_w64(sc > m_run + 8.f)) rescale(fmaxf(m_run, sc));
    const float pr = __builtin_amdgcn_exp2f(sc - m_run);
    const float p = K_::to_f(K_::from_f(pr));
    ls4[0] += 0.5f * p;   // both half-waves add it: the swap in row_sum doubles it
    #pragma unroll
    for (int db = 0; db < 2; ++db)
      #pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint2 vv = *(const uint2*)(vr + db * 32 + 8 * g + 4 * hi);
        o[db][4 * g + 0] = fmaf(p, K_::to_f(vv.x & 0xffff), o[db][4 * g + 0]);
        o[db][4 * g + 1] = fmaf(p, K_::to_f(vv.x >> 16), o[db][4 * g + 1]);
        o[db][4 * g + 2] = fmaf(p, K_::to_f(vv.y & 0xffff), o[db][4 * g + 2]);
        o[db][4 * g + 3] = fmaf(p, K_::to_f(vv.y >> 16), o[db][4 * g + 3]);
      }
  };

  // All keys for this workgroup's queries.  Tile t lives in stage t & 1.  Top of step t:
  // tile t's DMA was issued one step earlier (own pieces: vmcnt(0); everyone's: the
  // barrier, which also certifies that every wave finished tile t-1, whose stage now
  // receives tile t+1).
  const int ntiles = (seq + KT - 1) / KT, nfull = seq / KT, rem = seq - nfull * KT;
  const bool valu_tail = rem > 0 && rem <= TAIL_VALU;
  const int nmma = valu_tail ? nfull : ntiles;     // tiles that go through the MFMAs
  auto run = [&](bool exact) __attribute__((always_inline)) {
    #pragma unroll
    for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
    #pragma unroll
    for (int i = 0; i < 4; ++i) ls4[i] = 0.f;
    m_run = -INFINITY;
    if (nfull > 0) issue(0, 0, std::true_type{});
    else if (nmma > 0) issue(0, 0, std::false_type{});
    // top of tile t: tile t landed (own pieces: vmcnt(0); everyone's: the barrier, which also
    // frees the stage of tile t-1 for the next issue)
    auto top = [&](int t) __attribute__((always_inline)) {
      if (!ABL(4) && !ABL(8)) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (t + 1 < nfull) issue((t + 1) * KT, stage_of(t + 1), std::true_type{});
      else if (t + 1 < nmma) issue((t + 1) * KT, stage_of(t + 1), std::false_type{});
    };
    if (nfull > 0) {
      top(0);
      do_tile(0, std::false_type{}, true, exact);
    }
    // the steady loop: the next tile is a full one (scalar tile base + lane offsets)
    int t = 1;
    for (; t + 1 < nfull; ++t) {
      if (!ABL(4) && !ABL(8)) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      issue((t + 1) * KT, stage_of(t + 1), std::true_type{});
      do_tile(t, std::false_type{}, false, exact);
    }
    if (t < nfull) {
      top(t);
      do_tile(t, std::false_type{}, false, exact);
    }
    if (nfull < nmma) {
      top(nfull);
      do_tile(nfull, std::true_type{}, nfull == 0, exact);
    }
    if (valu_tail && active) {
      for (int kk = 0; kk < rem; ++kk) tail_key(nfull * KT + kk);
    }
  };
  auto row_sum = [&]() __attribute__((always_inline)) {
    const float l = (ls4[0] + ls4[1]) + (ls4[2] + ls4[3]);
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l), __float_as_uint(l), false, false);
    return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  };
  run(false);
  {
    // a key far above the first half tile's max overflowed P, O or the row sum: all waves
    // of the workgroup take the exact path over their keys again (K/V restaged; rare)
    float chk = row_sum();
    #pragma unroll
    for (int i = 0; i < 16; ++i) chk += o[0][i] + o[1][i];
    if (__builtin_amdgcn_ballot_w64(active && !__builtin_isfinite(chk))) redo = 1;
    __syncthreads();
    if (redo) run(true);
  }
  const float rowsum = row_sum();
  __syncthreads();
  // ---- normalise and store: stage the wave's 32 x 64 output through LDS so each
  // query row leaves as whole 128-B lines
  const float inv = 1.f / rowsum;
  u16* stg = (u16*)&smem[0][0] + wave * 32 * KS;   // 32 rows x KS (padded) per wave (18 KiB of 32)
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

namespace {
int g_attn_dbg = 0;   // ablation build: dp_attn_debug_flags

int attention_launch(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads, int32_t head_dim,
                     float scale, bool pre, int32_t dtype, dp_stream_t stream) {
  if (!qkv || !out) return DP_ERR_ARG;
  if (batch <= 0 || seq <= 0 || heads <= 0 || head_dim != HD) return DP_ERR_SHAPE;
  // Measured and rejected (35 x 577): two independent 32-query sub-blocks per wave (K / V
  // fragments shared, 210 VGPRs, 2 workgroups per CU) 98-101 us vs 75-76 us here -- the
  // occupancy (4 workgroups / 16 waves per CU) hides more than the in-wave ILP adds.
  const int nq = (seq + QB - 1) / QB;
  if ((long long)nq * heads * batch > 0x7fffffffLL) return DP_ERR_SHAPE;
  dim3 grid(nq * heads * batch);
  // softmax(s * scale) = 2^(s * scale * log2 e) / sum: sl2 is the scale in log2 units
  const float sl2 = pre ? 1.0f : (float)((double)scale * 1.4426950408889634);
  hipStream_t s = (hipStream_t)stream;
  if (dtype != DP_BF16 && dtype != DP_F16) return DP_ERR_DTYPE;
  if (pre) {
    if (dtype == DP_BF16) hipLaunchKernelGGL((attn_kernel<KBF16, true>), grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, nq, sl2, g_attn_dbg);
    else hipLaunchKernelGGL((attn_kernel<KF16, true>), grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, nq, sl2, g_attn_dbg);
  } else {
    if (dtype == DP_BF16) hipLaunchKernelGGL((attn_kernel<KBF16, false>), grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, nq, sl2, g_attn_dbg);
    else hipLaunchKernelGGL((attn_kernel<KF16, false>), grid, dim3(256), 0, s, (const u16*)qkv, (u16*)out, seq, heads, nq, sl2, g_attn_dbg);
  }
  DP_CHECK_LAUNCH();
  return 0;
}
}  // namespace

#ifdef DP_ATTN_ABLATE
extern "C" int dp_attn_debug_flags(int flags) {
  g_attn_dbg = flags;
  return 0;
}
#endif

extern "C" int dp_attention(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads,
                            int32_t head_dim, float scale, int32_t dtype, dp_stream_t stream) {
  return attention_launch(qkv, out, batch, seq, heads, head_dim, scale, false, dtype, stream);
}

extern "C" int dp_attention_log2q(const void* qkv, void* out, int32_t batch, int32_t seq, int32_t heads,
                                  int32_t head_dim, int32_t dtype, dp_stream_t stream) {
  return attention_launch(qkv, out, batch, seq, heads, head_dim, 1.0f, true, dtype, stream);
}
