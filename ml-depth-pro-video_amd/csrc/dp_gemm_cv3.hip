// dp_gemm_cv3.hip: the 3x3 patch-conv engine -- a stride-1, pad-1 3x3 implicit-GEMM conv on
// output tiles of 16 x 16 pixels x 256 channels whose input patch (18 x 18 pixels, one 64-channel
// block) sits in LDS, so the 9 taps of a channel block read their A fragments from the patch
// instead of streaming 9 shifted 256-pixel slices from L2.
//
// Why: the row-raster implicit conv (the big / persistent engines) moves 64 KiB per K step
// (256 shifted pixel rows + 256 weight rows); on the decoder's 768^2 convs that load stream
// alone takes as long as the MFMAs (tools/gemm_bench.py --ablate: 364 vs 393 us) and the two
// overlap poorly.  Here a K step moves the 32 KiB weight tile plus 1/9 of a 48 KiB patch.
//
// Layout: 8 waves as 2 (M) x 4 (N), wave tile 128 x 64 = 8 output pixel rows of the tile x 16
// pixels; K order (channel block, tap, 64 channels) = the packed conv weights
// ([Cout][Cin/64][ky][kx][64], ops.conv_weight).  LDS: 2 patch buffers (48 LDS-DMA pieces of
// 1 KiB each: 324 pixels x 128 B, the 16-B chunk XOR-swizzled by pixel index, 7 dummy pieces
// so every wave issues 6) + a 2-stage ring of weight K steps = 160 KiB.  The K loop: two
// half-step phases per K step (two wave groups staggered by one barrier, LDS-DMA issued in the
// phase after its buffer's last read, one counted wait per step) with the A fragments read from
// the patch.  The
// epilogue (bias, ReLU, residuals R1 / R2, 16-bit C) works in the MFMA register layout, one
// 16-pixel output row segment per fragment row.
#include "dp_gemm_impl.h"

namespace {

// Output tiles of TH x 16 pixels: TH = 16 (the 768^2 maps: 2304 tiles = 9 rounds of 256 CUs) or
// TH = 12 (DP_TILE_CV3_192x256, the 384^2 maps: 768 tiles = 3 rounds exactly, where 16 x 16 tiles
// make 2.25 rounds), or TH = 24 (DP_TILE_CV3_384x128, the 128-channel head conv at 768^2: 1536 tiles =
// 6 rounds; 48 MFMAs per wave and K step instead of 32); the patch is (TH + 2) x 18 pixels.
constexpr int CV_TW = 16;                     // output tile width (pixels)
constexpr int CV_PW = CV_TW + 2;              // patch width
template <int TH> struct CvGeo {
  static constexpr int PIX = (TH + 2) * CV_PW;              // patch pixels (324 / 252 / 468)
  static constexpr int PPW = (PIX * 8 + 511) / 512;          // LDS-DMA pieces per wave (6 / 4 / 8)
  static constexpr int PATCH_B = 8 * PPW * 1024;             // bytes the DMA writes per patch buffer
  static constexpr int FM = TH / 2, HQ = FM / 2;             // fragment rows per wave / per phase
  // TIGHT (TH 16 / 12): the two patch buffers PSTRIDE apart = the patch rounded up to whole 1-KiB
  // pieces (41 / 32 KiB), the dummy pieces past it written to a 1-KiB trash slot, so that every
  // fragment read of the second buffer is still base register + a 16-bit immediate (< 64 KiB);
  // TH 24 (59 KiB patches) moves its address registers by +- PATCH_B per channel block instead
  static constexpr int NREAL = (PIX + 7) / 8;                  // pieces holding patch pixels
  static constexpr bool TIGHT = NREAL * 1024 + ((FM + 1) * CV_PW + 2) * 128 < 65536;
  static constexpr int PSTRIDE = TIGHT ? NREAL * 1024 : PATCH_B;
  static constexpr int TRASH = 2 * PSTRIDE;                    // (TIGHT) dummy pieces
  static constexpr int WOFF = TIGHT ? 2 * PSTRIDE + 1024 : 2 * PATCH_B;   // weight ring
};

// BN: output channels per tile (256: the ResidualBlock convs; 128: the head convs).  EPI:
// CV_EPI_RES (bias, ReLU, residuals; BN 256), CV_EPI_BC (bias + the composed conv's border-tap
// correction, DP_STORE_ROWS with head_corr), CV_EPI_HPS (the composed depth head's pixel-shuffle
// + 1x1 epilogue, DP_STORE_HEAD_PS; BN 128: one output parity per wave).
constexpr int CV_EPI_RES = 0, CV_EPI_BC = 1, CV_EPI_HPS = 2;
// ABL (tools/gemm_bench.py --ablate, debug bits 1 / 2 / 4 on the ReLU residual conv only): 1 no
// epilogue, 2 no LDS-DMA in the K loop, 4 no MFMAs -- timing ablations, results garbage; 8: the
// normal kernel plus per-workgroup clock stamps into g_cv3_stamp (tools/cv3_stamps.py); 16: no
// barriers in the K loop; 32: the A fragments' ReLU applied by the reading wave; 64: no weight
// LDS-DMA in the K loop; 128: no patch LDS-DMA in the K loop; 256 (with 8): wave 0's K-loop cycles by
// kind into stamps 6..9; 512: static priority (waves 4-7 at
// priority 1 through the K loop) instead of a raise / drop around every MFMA run; 1024: no priority
// changes at all
constexpr int CV_STAMPS = 10, CV_STAMP_WGS = 4096;   // [6..9] (ABL 256): K-loop cycles in vmcnt waits,
                                                       // barriers, lgkmcnt waits, MFMA issue (wave 0)
__device__ unsigned long long g_cv3_stamp[CV_STAMP_WGS * CV_STAMPS];
template <typename K_, bool RELU, int BN, int EPI, int ABL = 0, int TH = 16>
__global__ void __launch_bounds__(512, 1) gemm_cv3_kernel(const GemmP p) {
  using G = CvGeo<TH>;
  constexpr int FM = G::FM, HQ = G::HQ, PPW = G::PPW, CV_PATCH_B = G::PATCH_B, CV_PIX = G::PIX;
  constexpr bool TIGHT = G::TIGHT;
  constexpr int PSTRIDE = G::PSTRIDE, WOFF = G::WOFF;
  constexpr int TN = BN / 4, FN = TN / 16, QF = FN / 2;          // wave tile 16 FM x TN
  static_assert(TH == 16 || TH == 12 || (TH == 24 && BN == 128), "tile rows");
  constexpr int NBH = BN / 128;                                  // weight halves per K step
  constexpr int B_B = BN * 128;                                  // bytes per weight K step
  static_assert(EPI != CV_EPI_RES || BN == 256, "residual epilogue: BN 256");
  static_assert(EPI != CV_EPI_HPS || BN == 128, "head epilogue: one parity (32 columns) per wave");
  __shared__ __attribute__((aligned(1024))) char smem[WOFF + 2 * B_B];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  unsigned long long st_[CV_STAMPS] = {};
  if constexpr ((ABL & 8) != 0) { st_[0] = __builtin_amdgcn_s_memtime(); st_[4] = __builtin_amdgcn_s_memrealtime(); }
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  // XCD-contiguous: an XCD's workgroups are consecutive tiles of a tile row (shared halos)
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int S = p.out_w, tpr = S / CV_TW, tpi = (S / TH) * tpr;
  const int tn = wgid % p.tiles_n, sp = wgid / p.tiles_n;
  const int img = sp / tpi, r_ = sp - img * tpi;
  const int y0 = (r_ / tpr) * TH, x0 = (r_ % tpr) * CV_TW, n0 = tn * BN;
  const int cin = p.in_c, CB = cin / 64;
  const int KT = CB * 9;

  // patch pieces of this lane: byte offset of its 16-B chunk (channel block 0) in the input map, or
  // CV_PAD when the pixel is in the zero padding or past the patch (read as zeros: past the end of
  // the buffer resource, glds16b; host: the map is < 2 GiB)
  // Computed where the pieces are issued (once per channel block) from a laundered lane index, so
  // that the compiler does not hoist the PPW offsets out of the K loop (they would hold PPW VGPRs
  // through it, where the unrolled loop's address bases need them).
  constexpr uint32_t CV_PAD = 0x80000000u;
  auto patch_off = [&](int i, int c0) __attribute__((always_inline)) {
    const int c = c0 + i * 64;                    // chunk index in the patch image
    const int P = c >> 3, slot = c & 7;
    uint32_t off = CV_PAD;
    if (P < CV_PIX) {
      const int pr = P / CV_PW, pc = P - pr * CV_PW;
      const int iy = y0 - 1 + pr, ix = x0 - 1 + pc;
      if ((unsigned)iy < (unsigned)S && (unsigned)ix < (unsigned)S)
        off = 2u * (uint32_t)(((img * S + iy) * S + ix) * cin + ((slot ^ (P & 7)) << 3));
    }
    return off;
  };
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const u32x4_t a_rs = raw_rsrc(p.A, (uint32_t)((long long)p.M * cin * 2));

  // weight K step t in the 8-phase layout (gemm_8ph_kernel): NBH halves of 128 rows (output
  // channels), 16 KiB each; half h rows h*128 + i*64 + wave*8 + lane/8, chunk swizzled on the source
  constexpr int HALF = 128 * 128;
  const int prow = wave * 8 + (lane >> 3);
  const int pchunk = (lane & 7) ^ ((lane >> 3) & 7);
  // byte offset of this lane's weight row (prow) from the piece's scalar base p.B + (h 128 + i 64)
  // ldb + 64 t (host: N * ldb < 2^31): one VGPR, the rest wave-uniform
  const uint32_t boff = 2u * (uint32_t)((n0 + prow) * (int)p.ldb + pchunk * 8);
  auto issue_b = [&](int h, int t) {   // half h of weight step t -> stage t & 1
    const uint32_t dst = lds0 + WOFF + (t & 1) * B_B + h * HALF + wave_u * 1024;
    #pragma unroll
    for (int i = 0; i < 2; ++i) glds16s(boff, p.B + (long long)(h * 128 + i * 64) * p.ldb + 64 * t, dst + i * 8192);
  };
  auto issue_patch3 = [&](int cb, int buf, int i0) {   // half of the wave's PPW patch pieces
    int c0 = wave * PPW * 64 + lane;              // the lane's chunk of piece 0
    asm volatile("" : "+v"(c0));
    #pragma unroll
    for (int i = i0; i < i0 + PPW / 2; ++i) {
      const int j = wave_u * PPW + i;                   // piece index in the patch image
      const uint32_t dst = lds0 + ((!TIGHT || j < G::NREAL) ? buf * PSTRIDE + j * 1024 : G::TRASH);
      glds16b(patch_off(i, c0) + cb * 128, a_rs, dst);
    }
  };

  f32x4_t acc[FM][FN];
  #pragma unroll
  for (int i = 0; i < FM; ++i)
    #pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15, fchunk = lane >> 4;
  uint4 af[2][HQ], bf[2][2][QF];
  // Fragment addresses as per-lane bases + compile-time offsets (the K loop below is unrolled over
  // the 9 taps and the 2 weight stages): patch pixel P = PB + c with PB = wm FM 18 + frow (this lane)
  // and c = (qm HQ + fm + ky) 18 + kx (constant), whose 16-B chunk is stored at slot chunk ^ (P & 7)
  // = chunk ^ ((PB + (c & 7)) & 7) -- so 8 x 2 bases (c & 7, ks), each + c * 128 as the ds_read
  // immediate (+ PSTRIDE for the second patch buffer when TIGHT; else the bases move by
  // +- CV_PATCH_B per channel block).
  // B: row r = wn TN + qn TN / 2 + fn 16 + frow, r & 7 = frow & 7 (TN / 2 a multiple of 16), so one
  // base per ks + a constant.  (Was: ~80 VALU of address arithmetic per K step.)
  typedef __attribute__((address_space(3))) const char lds_c;
  typedef __attribute__((address_space(3))) const u32x4_t lds_u4;   // (16-B alignment known: one ds_read_b128)
  uint32_t abase[8][2], bbase[2];
  {
    const int PB = wm * FM * CV_PW + frow;
    #pragma unroll
    for (int v = 0; v < 8; ++v)
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks) abase[v][ks] = lds0 + PB * 128 + (((ks * 4 + fchunk) ^ ((PB + v) & 7)) << 4);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      bbase[ks] = lds0 + WOFF + (wn * TN + frow) * 128 + (((ks * 4 + fchunk) ^ (frow & 7)) << 4);
  }
  // half qm of the wave tile = output pixel rows wm*FM + qm*HQ .. +HQ-1; tap (ky, kx) of the current
  // patch buffer (all four compile-time constants in the K loop)
  auto readA = [&](int qm, int ky, int kx, int pb) __attribute__((always_inline)) {
    const int boff_ = TIGHT ? pb * PSTRIDE : 0;
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fm = 0; fm < HQ; ++fm) {
        const int c = (qm * HQ + fm + ky) * CV_PW + kx;
        af[ks][fm] = __builtin_bit_cast(uint4, *(lds_u4*)((lds_c*)(uintptr_t)abase[c & 7][ks] + boff_ + c * 128));
      }
    if constexpr (RELU && (ABL & 32)) {   // the ReLU prologue by the reading wave, before the barrier
      #pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        #pragma unroll
        for (int fm = 0; fm < HQ; ++fm) af[ks][fm] = relu_pk16(af[ks][fm]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto readB = [&](int qn, int st) __attribute__((always_inline)) {   // columns wn*TN + qn*TN/2 .. of the tile
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fn = 0; fn < QF; ++fn)
        bf[qn][ks][fn] = __builtin_bit_cast(uint4, *(lds_u4*)((lds_c*)(uintptr_t)bbase[ks] + st * B_B + (qn * (TN / 2) + fn * 16) * 128));
  };
  auto tick = [&]() -> unsigned long long {
    if constexpr ((ABL & 256) != 0) return __builtin_amdgcn_s_memtime();
    return 0ull;
  };
  auto mma = [&](int qm, int qn) {
    const unsigned long long m0_ = tick();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long m1_ = tick();
    if constexpr ((ABL & 256) != 0) st_[8] += m1_ - m0_;
    if constexpr (ABL & 4) return;
    // the ReLU prologue in place, once per fragment (its first use, qn = 0): no relu'd copies held
    // beside the fragments, half the v_pk_max of a per-use ReLU
    if constexpr (RELU && !(ABL & 32)) {
      if (qn == 0) {
        #pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          #pragma unroll
          for (int fm = 0; fm < HQ; ++fm) af[ks][fm] = relu_pk16(af[ks][fm]);
      }
    }
    if constexpr ((ABL & 1536) == 0) __builtin_amdgcn_s_setprio(1);
    #pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      #pragma unroll
      for (int fm = 0; fm < HQ; ++fm) {
        #pragma unroll
        for (int fn = 0; fn < QF; ++fn)
          acc[qm * HQ + fm][qn * QF + fn] = K_::mfma16(bf[qn][ks][fn], af[ks][fm], acc[qm * HQ + fm][qn * QF + fn]);
      }
    if constexpr ((ABL & 1536) == 0) __builtin_amdgcn_s_setprio(0);
    if constexpr ((ABL & 256) != 0) { __builtin_amdgcn_sched_barrier(0); st_[9] += tick() - m1_; }
  };
  auto bar = [&]() {
    const unsigned long long b0_ = tick();
    if constexpr ((ABL & 16) == 0) asm volatile("s_barrier" ::: "memory");
    if constexpr ((ABL & 256) != 0) st_[7] += tick() - b0_;
  };

  // K loop: per K step (channel block cb, tap) two half-step phases {fragment reads, LDS-DMA,
  // s_barrier, MFMAs, s_barrier}; wave rows staggered by a barrier; weight step t+2 streamed in
  // phase 1 (its stage's reads ended in phase 0), the next block's patch in phase 0 of a block's
  // first step; one counted wait per step (phase 1) for step t+1.
  // prologue: patch of block 0 and weight steps 0 and 1
  issue_patch3(0, 0, 0); issue_patch3(0, 0, PPW / 2);
  #pragma unroll
  for (int h = 0; h < NBH; ++h) issue_b(h, 0);
  if (KT > 1) {
    #pragma unroll
    for (int h = 0; h < NBH; ++h) issue_b(h, 1);
    wait_vmcnt<2 * NBH>();
  } else {
    wait_vmcnt<0>();
  }
  lds_barrier();
  if constexpr ((ABL & 8) != 0) st_[1] = __builtin_amdgcn_s_memtime();
  if constexpr ((ABL & 512) != 0) { if (wave_u >= 4) __builtin_amdgcn_s_setprio(1); }
  if (wm == 1) bar();
  // one channel block cb: its 9 taps unrolled (ky, kx and the weight stage of each step constant:
  // step t = 9 cb + tap is in stage t & 1 = (cb + tap) & 1, ST0 = cb & 1)
  int cb = 0;
  auto block = [&](auto st0_tag) __attribute__((always_inline)) {
    constexpr int ST0 = decltype(st0_tag)::value;
    constexpr int pb = ST0;                       // (cb & 1 = cb * 9 & 1)
    const bool nb = cb + 1 < CB;
    #pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - ky * 3, st = (ST0 + tap) & 1;
      const int t = cb * 9 + tap;
      const bool np = tap == 0 && nb;             // this step streams the next block's patch
      const bool n2 = t + 2 < KT;
      // two half-step phases (A rows qm, both column halves: 16 MFMAs per wave at BN 128, 32 at
      // BN 256) instead of four quadrant phases -- half the barriers per step (head.0c 449 / 453
      // -> 433 / 421 us, the 768^2 ResidualBlock convs 676 / 684 -> 642 / 629 us in-frame,
      // profiles/r03af_cv3_bn128_2phase/, r03ag_cv3_2phase/).  Phase 0 reads the step's weights
      // and streams the next block's patch (its buffer was last read one phase earlier by the
      // wave row behind); phase 1 streams weight step t+2 into this step's stage (read in
      // phase 0), waits for step t+1, then issues the second weight half.
      readA(0, ky, kx, pb); readB(0, st); readB(1, st);
      if (np && !(ABL & 2) && !(ABL & 128)) { issue_patch3(cb + 1, pb ^ 1, 0); issue_patch3(cb + 1, pb ^ 1, PPW / 2); }
      bar(); mma(0, 0); mma(0, 1); bar();
      readA(1, ky, kx, pb);
      if (n2 && !(ABL & 2) && !(ABL & 64)) issue_b(0, t + 2);
      const unsigned long long v0_ = tick();
      if (np) { if (n2) wait_vmcnt<PPW + 2>(); else wait_vmcnt<PPW>(); }
      else { if (n2) wait_vmcnt<2>(); else wait_vmcnt<0>(); }
      if constexpr ((ABL & 256) != 0) st_[6] += tick() - v0_;
      if (NBH == 2 && n2 && !(ABL & 2) && !(ABL & 64)) issue_b(1, t + 2);
      bar(); mma(1, 0); mma(1, 1); bar();
    }
    // the next block reads the other patch buffer
    if constexpr (!TIGHT) {
      const uint32_t d = pb ? (uint32_t)-CV_PATCH_B : (uint32_t)CV_PATCH_B;
      #pragma unroll
      for (int v = 0; v < 8; ++v)
        #pragma unroll
        for (int ks = 0; ks < 2; ++ks) abase[v][ks] += d;
    }
    ++cb;
  };
  for (int pair = 0; pair < CB / 2; ++pair) {
    block(std::integral_constant<int, 0>{});
    block(std::integral_constant<int, 1>{});
  }
  if (CB & 1) block(std::integral_constant<int, 0>{});
  if (wm == 0) bar();
  if constexpr ((ABL & 512) != 0) __builtin_amdgcn_s_setprio(0);

  // epilogues in the MFMA register layout: fragment row fm of the wave is output pixel row
  // wm * FM + fm of the tile (16 consecutive pixels, lane & 15), each lane 4 consecutive
  // channels per fragment column (fn * 16 + 4 (lane >> 4)).  Same operations in the same order as
  // epilogue_rows / head_ps_rows: bit-identical to the row-raster engines.
  lds_barrier();   // the ring is free once every wave has left the K loop
  if constexpr ((ABL & 8) != 0) st_[2] = __builtin_amdgcn_s_memtime();
  if constexpr ((ABL & 1) != 0) {   // keep the accumulators live
    float z = 0.f;
    #pragma unroll
    for (int i = 0; i < FM; ++i)
      #pragma unroll
      for (int j = 0; j < FN; ++j) z += acc[i][j][0];
    if (z == 1234.5f) ((float*)p.C)[tid] = z;
    return;
  }
  const int t = lane & 15, g = lane >> 4;
  const int nw = n0 + wn * TN;
  f32x4_t bias[FN];
  #pragma unroll
  for (int fn = 0; fn < FN; ++fn)
    bias[fn] = p.bias ? *(const f32x4_t*)(p.bias + nw + fn * 16 + 4 * g) : f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto mrow = [&](int fm) { return (long long)((img * S + y0 + wm * FM + fm) * S + x0); };
  if constexpr (EPI == CV_EPI_HPS) {
    // composed depth head (head_ps_rows): this wave's 32 columns are parity q = wn of output
    // channels o = fn * 16 + 4 g + r; z = acc + bias - border taps of head.2's zero padding,
    // ReLU, dot with head.4 (32), + b, ReLU -> the fp32 depth map at (2y + dy, 2x + dx)
    const int q = nw >> 5, dy = q >> 1, dx = q & 1;
    float hw[FN][4];
    #pragma unroll
    for (int fn = 0; fn < FN; ++fn)
      #pragma unroll
      for (int r = 0; r < 4; ++r) hw[fn][r] = p.head_w[(nw & 31) + fn * 16 + 4 * g + r];
    const long long W2 = 2LL * S;
    #pragma unroll 1
    for (int fm = 0; fm < FM; ++fm) {
      const int y = y0 + wm * FM + fm, x = x0 + t;
      float z[FN][4];
      #pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        #pragma unroll
        for (int r = 0; r < 4; ++r) z[fn][r] = acc[fm][fn][r] + bias[fn][r];
      const bool top = y == 0 && dy == 0, bot = y == S - 1 && dy == 1;
      const bool lft = x == 0 && dx == 0, rgt = x == S - 1 && dx == 1;
      if (top || bot || lft || rgt) {
        #pragma unroll
        for (int a = 0; a < 3; ++a)
          #pragma unroll
          for (int c = 0; c < 3; ++c) {
            const bool oob = (a == 0 && top) || (a == 2 && bot) || (c == 0 && lft) || (c == 2 && rgt);
            if (oob) {
              #pragma unroll
              for (int fn = 0; fn < FN; ++fn)
                #pragma unroll
                for (int r = 0; r < 4; ++r) z[fn][r] -= p.head_corr[(a * 3 + c) * 32 + (nw & 31) + fn * 16 + 4 * g + r];
            }
          }
      }
      // the same per-lane sum order as head_ps_rows over a lane's 8 channels: its 4 (fn = 0) then
      // its 4 (fn = 1), then the cross-lane sum -- different lanes than the row-raster engine
      float hs = 0.f;
      #pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        #pragma unroll
        for (int r = 0; r < 4; ++r) hs += fmaxf(z[fn][r], 0.f) * hw[fn][r];
      hs += __shfl_xor(hs, 16);
      hs += __shfl_xor(hs, 32);
      if (g == 0) ((float*)p.C)[((long long)img * 2 * S + 2 * y + dy) * W2 + 2 * x + dx] = fmaxf(hs + p.head_b, 0.f);
    }
  } else {
    // 16-bit rows through the wave's LDS slab (16 rows x TN), stored as whole TN * 2-byte segments
    constexpr int CH = TN / 8, RPI = 64 / CH;
    char* slab = smem + wave * (16 * TN * 2);
    // residual rows PD fragment rows ahead (the K loop's fragment registers are free here): the
    // tile's residual reads were latency-bound one row ahead (epilogue 10.3 vs 4.1 us per tile
    // without residuals, profiles/r05j_cv3_loop/)
    constexpr int PD = 4;
    uint2 rb1[PD][FN], rb2[PD][FN];
    auto loadr = [&](int fm, uint2 (&r1)[FN], uint2 (&r2)[FN]) __attribute__((always_inline)) {
      if constexpr (EPI == CV_EPI_RES) {
        const long long m = mrow(fm) + t;
        #pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int col = nw + fn * 16 + 4 * g;
          if (p.R1) r1[fn] = *(const uint2*)(p.R1 + m * p.ldr1 + col);
          if (p.R2) r2[fn] = *(const uint2*)(p.R2 + m * p.ldr2 + col);
        }
      }
    };
    auto addr = [&](f32x4_t& x, uint2 r) __attribute__((always_inline)) {
      x[0] += K_::to_f(r.x & 0xffff); x[1] += K_::to_f(r.x >> 16);
      x[2] += K_::to_f(r.y & 0xffff); x[3] += K_::to_f(r.y >> 16);
    };
    #pragma unroll
    for (int i = 0; i < PD; ++i) loadr(i, rb1[i], rb2[i]);
    #pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      uint2 (&r1c)[FN] = rb1[fm % PD];
      uint2 (&r2c)[FN] = rb2[fm % PD];
      const int y = y0 + wm * FM + fm, x = x0 + t;
      const bool border = y == 0 || y == S - 1 || x == 0 || x == S - 1;
      #pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        f32x4_t xv = acc[fm][fn] + bias[fn];
        if constexpr (EPI == CV_EPI_BC) {
          // border_correct: the composed conv's bias share of the taps in the next conv's padding
          if (border) {
            #pragma unroll 1
            for (int tp = 0; tp < 9; ++tp) {
              const int a = tp / 3, c = tp - 3 * (tp / 3);
              const bool oob = (a == 0 && y == 0) || (a == 2 && y == S - 1) || (c == 0 && x == 0) || (c == 2 && x == S - 1);
              if (oob) xv -= *(const f32x4_t*)(p.head_corr + tp * p.N + nw + fn * 16 + 4 * g);
            }
          }
        }
        if (p.act == DP_ACT_RELU) {
          #pragma unroll
          for (int r = 0; r < 4; ++r) xv[r] = fmaxf(xv[r], 0.f);
        }
        if constexpr (EPI == CV_EPI_RES) {
          if (p.R1) addr(xv, r1c[fn]);
          if (p.R2) addr(xv, r2c[fn]);
        }
        const int chunk = fn * 2 + (g >> 1);
        uint2 w;
        w.x = K_::pack2(xv[0], xv[1]);
        w.y = K_::pack2(xv[2], xv[3]);
        *(uint2*)(slab + t * (TN * 2) + ((chunk ^ (t & (CH - 1))) << 4) + (g & 1) * 8) = w;
      }
      #pragma unroll
      for (int k = 0; k < 16 / RPI; ++k) {
        const int row = k * RPI + lane / CH, chunk = lane % CH;
        const uint4 d = *(const uint4*)(slab + row * (TN * 2) + ((chunk ^ (row & (CH - 1))) << 4));
        *(uint4*)((u16*)p.C + (mrow(fm) + row) * p.ldc + nw + chunk * 8) = d;
      }
      if (fm + PD < FM) loadr(fm + PD, r1c, r2c);
    }
  }
  if constexpr ((ABL & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_[3] = __builtin_amdgcn_s_memtime();
    st_[5] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && blockIdx.x < CV_STAMP_WGS) {
      #pragma unroll
      for (int k = 0; k < CV_STAMPS; ++k) g_cv3_stamp[blockIdx.x * CV_STAMPS + k] = st_[k];
    }
  }
}

template <typename K_>
int launch_cv3(const GemmP& p0, hipStream_t s, int th) {
  GemmP p = p0;
  const int S = p.out_w;
  if (p.k_h != 3 || p.k_w != 3 || p.stride != 1 || p.pad != 1 || p.in_h != S || p.in_w != S || p.out_h != S ||
      S % CV_TW || S % th || p.in_c % 64 || p.M % (S * S) || p.row_group || (p.head_w && p.store_mode != DP_STORE_HEAD_PS) ||
      p.gamma || p.pos || p.accumulate || (p.act != DP_ACT_NONE && p.act != DP_ACT_RELU))
    return DP_ERR_ARG;
  // (the input map < 2 GiB: the patch DMA's padding offset lies past it; weight byte offsets < 2^32)
  if ((long long)p.M * p.in_c >= (1LL << 30) || (long long)p.N * p.ldb >= (1LL << 31)) return DP_ERR_ARG;
  int epi, bn;
  if (p.store_mode == DP_STORE_HEAD_PS) {
    if (p.N != 128 || !p.head_w || !p.head_corr || p.c_dtype != DP_F32 || p.R1 || p.R2 || p.act) return DP_ERR_ARG;
    epi = CV_EPI_HPS; bn = 128;
  } else if (p.store_mode == DP_STORE_ROWS && p.head_corr) {
    if (p.c_dtype == DP_F32 || p.R1 || p.R2 || p.N % 128) return DP_ERR_ARG;
    epi = CV_EPI_BC; bn = p.N % 256 ? 128 : 256;
  } else if (p.store_mode == DP_STORE_ROWS) {
    if (p.c_dtype == DP_F32 || p.N % 256) return DP_ERR_ARG;
    epi = CV_EPI_RES; bn = 256;
  } else {
    return DP_ERR_ARG;
  }
  if (th == 12 && epi != CV_EPI_RES) return DP_ERR_ARG;   // (12-row tiles: the ResidualBlock-type convs only)
  if (th == 24 && ((epi != CV_EPI_BC && epi != CV_EPI_HPS) || bn != 128)) return DP_ERR_ARG;   // (the 128-channel head convs)
  p.tiles_n = p.N / bn;
  p.tiles_m = (p.M / (S * S)) * (S / th) * (S / CV_TW);
  dim3 grid(p.tiles_m * p.tiles_n);
  // K-loop ablation / stamp variants (tools/cv3_stamps.py): only with debug bit 1 << 24 set, so that
  // the planner's own debug bits (16, 32, 64, 1024, ...) never select one; an ablation
  // value without a variant runs the normal kernel
  const int abl = (p.dbg & (1 << 24)) ? p.dbg & 2047 : 0;
  if (th == 24) {   // 24 x 16-pixel tiles, 128 channels: 2 x 64 KiB patches + 2 x 16 KiB weight steps
    if (epi == CV_EPI_HPS) hipLaunchKernelGGL((gemm_cv3_kernel<K_, false, 128, CV_EPI_HPS, 0, 24>), grid, dim3(512), 0, s, p);
    else if (p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 128, CV_EPI_BC, 0, 24>), grid, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((gemm_cv3_kernel<K_, false, 128, CV_EPI_BC, 0, 24>), grid, dim3(512), 0, s, p);
    DP_CHECK_LAUNCH();
    return 0;
  }
  if (th == 12) {
    if (abl == 8 && p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 256, CV_EPI_RES, 8, 12>), grid, dim3(512), 0, s, p);
    else if (abl == 1032 && p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 256, CV_EPI_RES, 1032, 12>), grid, dim3(512), 0, s, p);
    else if (abl == 520 && p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 256, CV_EPI_RES, 520, 12>), grid, dim3(512), 0, s, p);
    else if (abl == 264 && p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 256, CV_EPI_RES, 264, 12>), grid, dim3(512), 0, s, p);
    else if (p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 256, CV_EPI_RES, 0, 12>), grid, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((gemm_cv3_kernel<K_, false, 256, CV_EPI_RES, 0, 12>), grid, dim3(512), 0, s, p);
    DP_CHECK_LAUNCH();
    return 0;
  }
#define DP_CV3(B_, E_) do { \
    if (p.relu_a) hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, B_, E_>), grid, dim3(512), 0, s, p); \
    else hipLaunchKernelGGL((gemm_cv3_kernel<K_, false, B_, E_>), grid, dim3(512), 0, s, p); } while (0)
  if (epi == CV_EPI_RES && abl && p.relu_a) {
    switch (abl) {
#define DP_CV3A(A_) case A_: hipLaunchKernelGGL((gemm_cv3_kernel<K_, true, 256, CV_EPI_RES, A_>), grid, dim3(512), 0, s, p); break;
      DP_CV3A(1) DP_CV3A(2) DP_CV3A(3) DP_CV3A(4) DP_CV3A(5) DP_CV3A(6) DP_CV3A(7) DP_CV3A(8)
      DP_CV3A(10) DP_CV3A(12) DP_CV3A(14) DP_CV3A(24) DP_CV3A(26) DP_CV3A(28) DP_CV3A(30) DP_CV3A(40) DP_CV3A(72)
      DP_CV3A(136) DP_CV3A(264) DP_CV3A(520) DP_CV3A(1032)
#undef DP_CV3A
      default: DP_CV3(256, CV_EPI_RES);
    }
  } else if (epi == CV_EPI_RES) DP_CV3(256, CV_EPI_RES);
  else if (epi == CV_EPI_HPS) DP_CV3(128, CV_EPI_HPS);
  else if (bn == 256) DP_CV3(256, CV_EPI_BC);
  else DP_CV3(128, CV_EPI_BC);
#undef DP_CV3
  DP_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// debug: copy the clock stamps of the last ABL-8 launch (CV_STAMPS per workgroup) to host memory
extern "C" int dp_cv3_stamps(unsigned long long* dst, int n_wg) {
  if (n_wg > CV_STAMP_WGS) n_wg = CV_STAMP_WGS;
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_cv3_stamp), (size_t)n_wg * CV_STAMPS * 8, 0, hipMemcpyDeviceToHost);
}

namespace dpg {
int launch_part_cv3(const GemmP& p, bool conv, bool bf16, hipStream_t s, int th) {
  if (!conv) return DP_ERR_ARG;
  return bf16 ? launch_cv3<KBF16>(p, s, th) : launch_cv3<KF16>(p, s, th);
}
}  // namespace dpg
