// HBM-bound helper kernels of the Depth Pro hot path (gfx950): LayerNorm,
// input normalisation, bilinear resize, fused pyramid + window im2col, cls
// rows, window merge, FOV tail, infer epilogue.  All loads/stores are 16 B per
// lane where the layout allows (coalesced), one pass over HBM each.
#include "dp_common.h"

namespace {

// ------------------------------------------------------------------ LayerNorm
// One wave64 per row, the row held in registers, two-pass mean / variance in
// fp32 (timm nn.LayerNorm(eps=1e-6)), 16-bit output.  Lane l owns the 8
// consecutive columns 8 l + 512 j (j < VEC / 2): two 16-B loads per group and ONE
// 16-B store (a full 1 KiB line set per wave-instruction; 8-B stores wrote half).
// Affine parameters per row group (dp_layernorm_grouped: rows [g * rpg, (g + 1) * rpg) take
// w[g] / b[g]; dp_layernorm: one group).
constexpr int LN_MAX_GROUPS = 4;
struct LnW {
  const float* w[LN_MAX_GROUPS];
  const float* b[LN_MAX_GROUPS];
  int rpg;
};

template <typename K_, int VEC>
__global__ void __launch_bounds__(256) ln_kernel(const float* __restrict__ x, long long ldx, const LnW lw,
                                                 u16* __restrict__ y, long long ldy, int rows, float eps) {
  static_assert(VEC % 2 == 0, "8 columns per lane");
  constexpr int G = VEC / 2;
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= rows) return;
  const int grp = row / lw.rpg;
  const float* __restrict__ w = lw.w[grp];
  const float* __restrict__ b = lw.b[grp];
  constexpr int COLS = VEC * 256;
  const float* xr = x + (long long)row * ldx;
  float4 v[VEC];
  float s = 0.f;
  #pragma unroll
  for (int j = 0; j < G; ++j) {
    v[2 * j] = *(const float4*)(xr + j * 512 + lane * 8);
    v[2 * j + 1] = *(const float4*)(xr + j * 512 + lane * 8 + 4);
  }
  #pragma unroll
  for (int i = 0; i < VEC; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  #pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s * (1.f / COLS);
  float q = 0.f;
  #pragma unroll
  for (int i = 0; i < VEC; ++i) {
    float a = v[i].x - mean, bb = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
    q += (a * a + bb * bb) + (c * c + d * d);
  }
  #pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = rsqrtf(q * (1.f / COLS) + eps);
  u16* yr = y + (long long)row * ldy;
  #pragma unroll
  for (int j = 0; j < G; ++j) {
    const int c0 = j * 512 + lane * 8;
    uint32_t pk[4];
    #pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 g = *(const float4*)(w + c0 + 4 * h);
      const float4 bb = *(const float4*)(b + c0 + 4 * h);
      const float4 t = v[2 * j + h];
      const float o0 = (t.x - mean) * rstd * g.x + bb.x;
      const float o1 = (t.y - mean) * rstd * g.y + bb.y;
      const float o2 = (t.z - mean) * rstd * g.z + bb.z;
      const float o3 = (t.w - mean) * rstd * g.w + bb.w;
      pk[2 * h] = (uint32_t)K_::from_f(o0) | ((uint32_t)K_::from_f(o1) << 16);
      pk[2 * h + 1] = (uint32_t)K_::from_f(o2) | ((uint32_t)K_::from_f(o3) << 16);
    }
    *(uint4*)(yr + c0) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
}

// 256 columns: one float4 per lane, 8-B stores
template <typename K_>
__global__ void __launch_bounds__(256) ln256_kernel(const float* __restrict__ x, long long ldx, const LnW lw,
                                                    u16* __restrict__ y, long long ldy, int rows, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= rows) return;
  const int grp = row / lw.rpg;
  const float* __restrict__ w = lw.w[grp];
  const float* __restrict__ b = lw.b[grp];
  const float4 v = *(const float4*)(x + (long long)row * ldx + lane * 4);
  float s = (v.x + v.y) + (v.z + v.w);
  #pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s * (1.f / 256);
  const float a = v.x - mean, bb = v.y - mean, c = v.z - mean, d = v.w - mean;
  float q = (a * a + bb * bb) + (c * c + d * d);
  #pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = rsqrtf(q * (1.f / 256) + eps);
  const float4 g = *(const float4*)(w + lane * 4);
  const float4 bv = *(const float4*)(b + lane * 4);
  uint2 pk;
  pk.x = (uint32_t)K_::from_f(a * rstd * g.x + bv.x) | ((uint32_t)K_::from_f(bb * rstd * g.y + bv.y) << 16);
  pk.y = (uint32_t)K_::from_f(c * rstd * g.z + bv.z) | ((uint32_t)K_::from_f(d * rstd * g.w + bv.w) << 16);
  *(uint2*)(y + (long long)row * ldy + lane * 4) = pk;
}

template <typename K_>
int ln_launch(const float* x, long long ldx, const LnW& lw, u16* y, long long ldy,
              int rows, int cols, float eps, hipStream_t s) {
  dim3 grid((rows + 3) / 4);
  switch (cols) {
    case 256: hipLaunchKernelGGL((ln256_kernel<K_>), grid, dim3(256), 0, s, x, ldx, lw, y, ldy, rows, eps); break;
    case 512: hipLaunchKernelGGL((ln_kernel<K_, 2>), grid, dim3(256), 0, s, x, ldx, lw, y, ldy, rows, eps); break;
    case 1024: hipLaunchKernelGGL((ln_kernel<K_, 4>), grid, dim3(256), 0, s, x, ldx, lw, y, ldy, rows, eps); break;
    case 2048: hipLaunchKernelGGL((ln_kernel<K_, 8>), grid, dim3(256), 0, s, x, ldx, lw, y, ldy, rows, eps); break;
    default: return DP_ERR_SHAPE;
  }
  DP_CHECK_LAUNCH();
  return 0;
}

// The input side of a folded LayerNorm (dp_layernorm_stats): one wave per row, lane l owns the 8
// columns 8 l + 512 j (as ln_kernel); each 128-column chunk is 16 lanes.  Writes the row in 16
// bits and the chunk's (mean, M2), two-pass within the chunk (fp32), the same statistics the
// residual GEMMs' producer epilogue writes for the rows it makes (dp_gemm_args.ln_part_out).
template <typename K_, int VEC>
__global__ void __launch_bounds__(256) ln_stats_kernel(const float* __restrict__ x, long long ldx, int rows,
                                                       u16* __restrict__ xb, long long ldxb, int8_t* __restrict__ xl,
                                                       float* __restrict__ part) {
  constexpr int G = VEC / 2, COLS = VEC * 256, NCH = COLS / 128;
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= rows) return;
  const float* xr = x + (long long)row * ldx;
  #pragma unroll
  for (int j = 0; j < G; ++j) {
    const float4 a = *(const float4*)(xr + j * 512 + lane * 8);
    const float4 b = *(const float4*)(xr + j * 512 + lane * 8 + 4);
    float s = (a.x + a.y) + (a.z + a.w) + ((b.x + b.y) + (b.z + b.w));
    #pragma unroll
    for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o);
    const float mean = s * (1.f / 128);
    const float d0 = a.x - mean, d1 = a.y - mean, d2 = a.z - mean, d3 = a.w - mean;
    const float d4 = b.x - mean, d5 = b.y - mean, d6 = b.z - mean, d7 = b.w - mean;
    float q = (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3) + ((d4 * d4 + d5 * d5) + (d6 * d6 + d7 * d7));
    #pragma unroll
    for (int o = 1; o < 16; o <<= 1) q += __shfl_xor(q, o);
    uint4 w;
    w.x = K_::pack2(a.x, a.y); w.y = K_::pack2(a.z, a.w);
    w.z = K_::pack2(b.x, b.y); w.w = K_::pack2(b.z, b.w);
    *(uint4*)(xb + (long long)row * ldxb + j * 512 + lane * 8) = w;
    if (xl) {   // the split residual's 8-bit low part: what the 16-bit rounding dropped (lo8_encode)
      auto lo = [](float v, uint32_t hw, int half) {
        return lo8_encode<K_>(v, K_::to_f((u16)(half ? hw >> 16 : hw & 0xffff)));
      };
      uint2 l;
      l.x = pack_i8x4(lo(a.x, w.x, 0), lo(a.y, w.x, 1), lo(a.z, w.y, 0), lo(a.w, w.y, 1));
      l.y = pack_i8x4(lo(b.x, w.z, 0), lo(b.y, w.z, 1), lo(b.z, w.w, 0), lo(b.w, w.w, 1));
      *(uint2*)(xl + (long long)row * ldxb + j * 512 + lane * 8) = l;
    }
    if ((lane & 15) == 0) {
      const int ch = j * 4 + (lane >> 4);
      *(float2*)(part + ((long long)row * NCH + ch) * 2) = make_float2(mean, q);
    }
  }
}

// --------------------------------------------------------- u8 HWC -> CHW norm
template <int OUT>
__global__ void normalize_kernel(const uint8_t* __restrict__ img, int HW, void* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= HW) return;
  #pragma unroll
  for (int c = 0; c < 3; ++c) {
    // ToTensor: u8 / 255 (fp32), Normalize: (x - 0.5) / 0.5
    float v = ((float)img[3 * i + c] / 255.0f - 0.5f) / 0.5f;
    if constexpr (OUT == DP_F32) ((float*)out)[(long long)c * HW + i] = v;
    else if constexpr (OUT == DP_BF16) ((u16*)out)[(long long)c * HW + i] = KBF16::from_f(v);
    else ((u16*)out)[(long long)c * HW + i] = KF16::from_f(v);
  }
}

// ------------------------------------------------------------ bilinear resize
// PyTorch upsample_bilinear2d, align_corners=False, explicit output size:
// scale = in/out, src = max(scale*(dst+0.5)-0.5, 0), h1 = h0 + (h0 < in-1).
__device__ __forceinline__ void src_index(int d, float scale, int in, int& i0, int& i1, float& l0, float& l1) {
  float s = scale * ((float)d + 0.5f) - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
  l0 = 1.f - l1;
}

template <int SRC>
__device__ __forceinline__ float ld_any(const void* p, long long i) {
  if constexpr (SRC == DP_F32) return ((const float*)p)[i];
  else if constexpr (SRC == DP_BF16) return KBF16::to_f(((const u16*)p)[i]);
  else return KF16::to_f(((const u16*)p)[i]);
}

// PyTorch upsample_bicubic2d, align_corners=False (A = -0.75): src = scale*(dst+0.5)-0.5 NOT
// clamped, i0 = floor(src), t = src - i0, taps i0-1 .. i0+2 clamped to [0, in-1] (bounded access).
__device__ __forceinline__ void cubic_coeffs(float t, float (&c)[4]) {
  constexpr float A = -0.75f;
  auto cc1 = [](float x) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; };          // |x| <= 1
  auto cc2 = [](float x) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; };    // 1 < |x| < 2
  c[0] = cc2(t + 1.f);
  c[1] = cc1(t);
  c[2] = cc1(1.f - t);
  c[3] = cc2(2.f - t);
}
__device__ __forceinline__ void cubic_index(int d, float scale, int in, int (&i)[4], float (&c)[4]) {
  const float s = scale * ((float)d + 0.5f) - 0.5f;
  const float f = floorf(s);
  const int i0 = (int)f;
  cubic_coeffs(s - f, c);
  #pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = i0 - 1 + k;
    i[k] = v < 0 ? 0 : (v > in - 1 ? in - 1 : v);
  }
}

// One output pixel of plane `p` (H x W, element loader ld(i)) at (oy, ox): MODE 0 bilinear, 1 bicubic,
// each value pre-multiplied by `mul` (the infer epilogue's scale, applied before the resize as there).
template <int MODE, typename LD>
__device__ __forceinline__ float resample(LD ld, int H, int W, int oy, int ox, float sh, float sw, float mul) {
  if constexpr (MODE == DP_INTERP_BILINEAR) {
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    src_index(oy, sh, H, y0, y1, ly0, ly1);
    src_index(ox, sw, W, x0, x1, lx0, lx1);
    const float v00 = ld((long long)y0 * W + x0) * mul, v01 = ld((long long)y0 * W + x1) * mul;
    const float v10 = ld((long long)y1 * W + x0) * mul, v11 = ld((long long)y1 * W + x1) * mul;
    return ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
  } else {
    int yi[4], xi[4];
    float cy[4], cx[4];
    cubic_index(oy, sh, H, yi, cy);
    cubic_index(ox, sw, W, xi, cx);
    float r[4];
    #pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long long row = (long long)yi[k] * W;
      r[k] = ld(row + xi[0]) * mul * cx[0] + ld(row + xi[1]) * mul * cx[1] + ld(row + xi[2]) * mul * cx[2] +
             ld(row + xi[3]) * mul * cx[3];
    }
    return r[0] * cy[0] + r[1] * cy[1] + r[2] * cy[2] + r[3] * cy[3];
  }
}

template <int SRC, int MODE>
__global__ void resize_kernel(const void* __restrict__ src, int C, int H, int W, float* __restrict__ dst,
                              int OH, int OW, float sh, float sw) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)C * OH * OW;
  if (i >= total) return;
  const int ox = i % OW;
  const int oy = (i / OW) % OH;
  const int c = i / ((long long)OW * OH);
  const long long pb = (long long)c * H * W;
  dst[i] = resample<MODE>([&](long long j) { return ld_any<SRC>(src, pb + j); }, H, W, oy, ox, sh, sw, 1.f);
}

// Same size in and out: F.interpolate's upsample kernels copy the input then (PyTorch's
// input == output size fast path), so this one does too -- 16 B per lane for fp32 planes
template <int SRC>
__global__ void resize_copy_kernel(const void* __restrict__ src, float* __restrict__ dst, long long total) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= total) return;
  if (SRC == DP_F32 && i + 4 <= total) {
    *(float4*)(dst + i) = *(const float4*)((const float*)src + i);
    return;
  }
  for (long long j = i; j < i + 4 && j < total; ++j) dst[j] = ld_any<SRC>(src, j);
}

// ------------------------------------------- pyramid + sliding windows + im2col
// Row m = w*576 + py*24 + px (window w, token), col k = c*256 + ky*16 + kx.
// Windows 0..24: 1536^2 level, stride 288; 25..33: 768^2 level, stride 192;
// 34: 384^2 level (encoder.py:170-188, 253-263).  The 0.5 / 0.25 bilinear
// resizes (encoder.py:151-168) are exactly 2-tap averages per axis (taps
// {2d, 2d+1} and {4d+1, 4d+2}); they are evaluated in PyTorch's order
// 0.5*(0.5*a + 0.5*b) + 0.5*(0.5*c + 0.5*d).
template <typename K_>
__global__ void patchify_kernel(const float* __restrict__ x0, u16* __restrict__ cols) {
  const int S = 1536;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (m, c, ky)
  const int total = 35 * 576 * 48;
  if (i >= total) return;
  const int ky = i % 16;
  const int c = (i / 16) % 3;
  const int m = i / 48;
  const int w = m / 576, t = m % 576;
  const int py = t / 24, px = t % 24;
  const float* plane = x0 + (long long)c * S * S;
  float v[16];
  if (w < 25) {
    const int oy = (w / 5) * 288, ox = (w % 5) * 288;
    const float* r = plane + (long long)(oy + py * 16 + ky) * S + ox + px * 16;
    #pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 f = *(const float4*)(r + 4 * q);
      v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
    }
  } else if (w < 34) {
    const int ww = w - 25;
    const int Y = (ww / 3) * 192 + py * 16 + ky, X0 = (ww % 3) * 192 + px * 16;
    const float* r0 = plane + (long long)(2 * Y) * S + 2 * X0;
    const float* r1 = r0 + S;
    #pragma unroll
    for (int q = 0; q < 8; ++q) {
      float4 a = *(const float4*)(r0 + 4 * q);
      float4 b = *(const float4*)(r1 + 4 * q);
      v[2 * q] = 0.5f * (0.5f * a.x + 0.5f * a.y) + 0.5f * (0.5f * b.x + 0.5f * b.y);
      v[2 * q + 1] = 0.5f * (0.5f * a.z + 0.5f * a.w) + 0.5f * (0.5f * b.z + 0.5f * b.w);
    }
  } else {
    const int Y = py * 16 + ky, X0 = px * 16;
    const float* r0 = plane + (long long)(4 * Y + 1) * S + 4 * X0;
    const float* r1 = r0 + S;
    #pragma unroll
    for (int q = 0; q < 16; ++q) {
      float4 a = *(const float4*)(r0 + 4 * q);
      float4 b = *(const float4*)(r1 + 4 * q);
      // taps 4X+1, 4X+2 of rows 4Y+1, 4Y+2
      v[q] = 0.5f * (0.5f * a.y + 0.5f * a.z) + 0.5f * (0.5f * b.y + 0.5f * b.z);
    }
  }
  uint32_t pk[8];
  #pragma unroll
  for (int q = 0; q < 8; ++q) pk[q] = (uint32_t)K_::from_f(v[2 * q]) | ((uint32_t)K_::from_f(v[2 * q + 1]) << 16);
  u16* dst = cols + (long long)m * 768 + c * 256 + ky * 16;
  *(uint4*)dst = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  *(uint4*)(dst + 8) = make_uint4(pk[4], pk[5], pk[6], pk[7]);
}

__global__ void cls_kernel(float* __restrict__ x, const float* __restrict__ cls, const float* __restrict__ pos, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 1024) return;
  const int w = i / 1024, c = i % 1024;
  x[(long long)w * 577 * 1024 + c] = cls[c] + pos[c];
}

// ------------------------------------------------------------- window merge
__device__ __forceinline__ void merge_axis(int Y, int steps, int pad, int& j, int& yy) {
  if (steps == 1) { j = 0; yy = Y; return; }
  const int first = 24 - pad, mid = 24 - 2 * pad;
  if (Y < first) { j = 0; yy = Y; return; }
  const int y2 = Y - first;
  j = 1 + y2 / mid;
  if (j > steps - 1) j = steps - 1;
  yy = pad + (y2 - (j - 1) * mid);
}

// Pixels whose source window (j * steps + ii) lies outside [wlo, whi) are left untouched:
// a caller that runs the windows in several independent row groups merges each group's
// share as soon as that group reaches the hooked block.
template <typename K_, int SRC>
__global__ void merge_kernel(const void* __restrict__ src, long long ld, int w0, int steps, int pad, int S,
                             u16* __restrict__ dst, int wlo, int whi) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (pixel, 8-channel group)
  if (i >= (long long)S * S * 128) return;
  const int g = i % 128;
  const int pix = i / 128;
  const int Y = pix / S, X = pix % S;
  int j, yy, ii, xx;
  merge_axis(Y, steps, pad, j, yy);
  merge_axis(X, steps, pad, ii, xx);
  const int win = j * steps + ii;
  if (win < wlo || win >= whi) return;
  const long long row = (long long)(w0 + win) * 577 + 1 + yy * 24 + xx;
  uint32_t pk[4];
  if constexpr (SRC == DP_F32) {
    const float* s = (const float*)src + row * ld + g * 8;
    float4 a = *(const float4*)s, b = *(const float4*)(s + 4);
    pk[0] = (uint32_t)K_::from_f(a.x) | ((uint32_t)K_::from_f(a.y) << 16);
    pk[1] = (uint32_t)K_::from_f(a.z) | ((uint32_t)K_::from_f(a.w) << 16);
    pk[2] = (uint32_t)K_::from_f(b.x) | ((uint32_t)K_::from_f(b.y) << 16);
    pk[3] = (uint32_t)K_::from_f(b.z) | ((uint32_t)K_::from_f(b.w) << 16);
  } else {
    uint4 a = *(const uint4*)((const u16*)src + row * ld + g * 8);
    pk[0] = a.x; pk[1] = a.y; pk[2] = a.z; pk[3] = a.w;
  }
  *(uint4*)(dst + (long long)pix * 1024 + g * 8) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
}

// ------------------------------------------------------------------ FOV tail
template <typename K_>
__global__ void fov_tail_kernel(const u16* __restrict__ x6, const float* __restrict__ w, float bias,
                                float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < 1152; i += 256) {
    const int ci = i % 32, tap = i / 32;  // x6 NHWC: (ky*6+kx)*32 + ci
    s += K_::to_f(x6[i]) * w[ci * 36 + tap];
  }
  #pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]) + bias;
}

// ------------------------------------------------------------ infer epilogue
template <int MODE>
__global__ void infer_epi_kernel(const float* __restrict__ canon, int SH, int SW, const float* __restrict__ fov,
                                 int use_given, float given_scale, float given_fpx, int H, int W,
                                 float* __restrict__ depth, float* __restrict__ fpx_out, int* __restrict__ nonfinite) {
  float fpx, scale;
  if (use_given) {
    fpx = given_fpx;
    scale = given_scale;
  } else {
    const float deg = fov[0];
    const float rad = deg * 0.017453292519943295f;  // torch.deg2rad
    fpx = (0.5f * (float)W) / tanf(0.5f * rad);
    scale = (float)W / fpx;
  }
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    if (fpx_out) fpx_out[0] = fpx;
    if (nonfinite && !__builtin_isfinite(fpx)) atomicAdd(nonfinite, 1);
  }
  if (i >= (long long)H * W) return;
  float v;
  if (H == SH && W == SW) {
    v = canon[i] * scale;
  } else {
    const int ox = i % W, oy = i / W;
    v = resample<MODE>([&](long long j) { return canon[j]; }, SH, SW, oy, ox, (float)SH / (float)H,
                       (float)SW / (float)W, scale);
  }
  // torch.clamp keeps a NaN a NaN (fminf / fmaxf alone would turn it into a bound)
  v = v != v ? v : fminf(fmaxf(v, 1e-4f), 1e4f);
  const float d = 1.0f / v;
  depth[i] = d;
  if (nonfinite) {
    // one add per wave that saw a NaN / inf (a healthy frame issues none)
    const unsigned long long bad = __ballot(!__builtin_isfinite(d));
    if (bad && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(bad)) atomicAdd(nonfinite, (int)__builtin_popcountll(bad));
  }
}

// ------------------------------------------------- cv2.resize for 8-bit RGB frames
// The reference's --downscale_factor (generate_depth_maps.py:95-110): cv2.resize, INTER_AREA for
// factor < 1 and INTER_LINEAR otherwise, on the uint8 HWC frame.  OpenCV 4.x's published
// algorithms (imgproc resize.cpp; restated in oracle/cv_resize_oracle.py): fixed-point bilinear
// with 11-bit coefficients (SIMD vertical form, scalar form in the row tail), and area
// averaging (integer-scale cells; fractional cell weights otherwise, float sums in table order,
// no FMA contraction -- `fp contract(off)` on plain expressions: the __fmul_rn / __fadd_rn helpers
// are plain operators that fuse after inlining -- so that every rounding is OpenCV's).  One
// thread per output pixel.
__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

__device__ __forceinline__ void cv_lin_tap(int d, double scale, int n, bool clamp_index, int& i0, int& w0, int& w1) {
#pragma clang fp contract(off)
  float f = (float)((d + 0.5) * scale - 0.5);
  int sidx = (int)floorf(f);
  f = f - (float)sidx;
  if (clamp_index) {
    if (sidx < 0) { f = 0.f; sidx = 0; }
    if (sidx >= n - 1) { f = 0.f; sidx = n - 1; }
  }
  i0 = sidx;
  w0 = cv_round((1.f - f) * 2048.f);
  w1 = cv_round(f * 2048.f);
}

// one axis of computeResizeAreaTab for output index d: visits (source index, alpha) in table order
template <typename F>
__device__ __forceinline__ void cv_area_taps(int d, double scale, int ssize, F&& f) {
#pragma clang fp contract(off)
  const double fs1 = d * scale, fs2 = fs1 + scale;
  const double cell = fmin(scale, ssize - fs1);
  int s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  if (s1 - fs1 > 1e-3) f(s1 - 1, (float)((s1 - fs1) / cell));
  for (int sx = s1; sx < s2; ++sx) f(sx, (float)(1.0 / cell));
  if (fs2 - s2 > 1e-3) f(s2, (float)(fmin(fmin(fs2 - s2, 1.0), cell) / cell));
}

// mode 0: INTER_LINEAR; 1: INTER_AREA integer cells; 2: INTER_AREA fractional cells
__global__ void __launch_bounds__(256) cv_resize_kernel(const uint8_t* __restrict__ src, int H, int W,
                                                        uint8_t* __restrict__ dst, int OH, int OW, int mode,
                                                        double scale_y, double scale_x, int isy, int isx,
                                                        int tail0) {
#pragma clang fp contract(off)   // every product and sum rounded on its own, as OpenCV's SSE code does
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)OH * OW) return;
  const int dy = (int)(i / OW), dx = (int)(i - (long long)dy * OW);
  uint8_t* o = dst + i * 3;
  if (mode == 0) {
    int x0, ax0, ax1, y0, by0, by1;
    cv_lin_tap(dx, scale_x, W, true, x0, ax0, ax1);
    cv_lin_tap(dy, scale_y, H, false, y0, by0, by1);
    const int x1 = min(x0 + 1, W - 1);
    const int r0 = min(max(y0, 0), H - 1), r1 = min(max(y0 + 1, 0), H - 1);
    const uint8_t* s0 = src + (long long)r0 * W * 3;
    const uint8_t* s1 = src + (long long)r1 * W * 3;
    #pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int h0 = s0[x0 * 3 + c] * ax0 + s0[x1 * 3 + c] * ax1;
      const int h1 = s1[x0 * 3 + c] * ax0 + s1[x1 * 3 + c] * ax1;
      int v;
      if (dx * 3 + c >= tail0) v = (h0 * by0 + h1 * by1 + (1 << 21)) >> 22;          // scalar row tail
      else v = ((((h0 >> 4) * by0) >> 16) + (((h1 >> 4) * by1) >> 16) + 2) >> 2;   // SIMD form
      o[c] = sat_u8(v);
    }
  } else if (mode == 1) {
    int sum[3] = {0, 0, 0};
    for (int a = 0; a < isy; ++a) {
      const uint8_t* r = src + ((long long)(dy * isy + a) * W + (long long)dx * isx) * 3;
      for (int b = 0; b < isx; ++b) {
        sum[0] += r[3 * b]; sum[1] += r[3 * b + 1]; sum[2] += r[3 * b + 2];
      }
    }
    const float sc = 1.f / (float)(isx * isy);
    #pragma unroll
    for (int c = 0; c < 3; ++c) {
      int v;
      if (isx == 2 && isy == 2 && dx < tail0) v = (sum[c] + 2) >> 2;     // SIMD form of the 2 x 2 cells
      else v = cv_round((float)sum[c] * sc);
      o[c] = sat_u8(v);
    }
  } else {
    float acc[3] = {0.f, 0.f, 0.f};
    cv_area_taps(dy, scale_y, H, [&](int sy, float beta) {
      float buf[3] = {0.f, 0.f, 0.f};
      const uint8_t* r = src + (long long)sy * W * 3;
      cv_area_taps(dx, scale_x, W, [&](int sx, float alpha) {
        #pragma unroll
        for (int c = 0; c < 3; ++c) buf[c] = buf[c] + (float)r[sx * 3 + c] * alpha;
      });
      #pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] = acc[c] + beta * buf[c];
    });
    #pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = sat_u8(cv_round(acc[c]));
  }
}

inline int blocks_for(long long n, int bs) { return (int)((n + bs - 1) / bs); }

}  // namespace

extern "C" int dp_abi_version(void) { return DP_ABI_VERSION; }

extern "C" int dp_layernorm_stats(const float* x, int64_t ldx, int32_t rows, int32_t cols, void* xb, int64_t ldxb,
                                  void* xl, float* part, int32_t dtype, dp_stream_t stream) {
  if (!x || !xb || !part) return DP_ERR_ARG;
  if (rows <= 0) return DP_ERR_SHAPE;
  if (ldx % 4 || ldxb % 8) return DP_ERR_ALIGN;
  dim3 grid((rows + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
#define DP_LS(V_) do { \
    if (dtype == DP_BF16) hipLaunchKernelGGL((ln_stats_kernel<KBF16, V_>), grid, dim3(256), 0, s, x, (long long)ldx, rows, (u16*)xb, (long long)ldxb, (int8_t*)xl, part); \
    else if (dtype == DP_F16) hipLaunchKernelGGL((ln_stats_kernel<KF16, V_>), grid, dim3(256), 0, s, x, (long long)ldx, rows, (u16*)xb, (long long)ldxb, (int8_t*)xl, part); \
    else return DP_ERR_DTYPE; } while (0)
  switch (cols) {
    case 512: DP_LS(2); break;
    case 1024: DP_LS(4); break;
    case 2048: DP_LS(8); break;
    default: return DP_ERR_SHAPE;
  }
#undef DP_LS
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_layernorm(const float* x, int64_t ldx, const float* w, const float* b, void* y, int64_t ldy,
                            int32_t rows, int32_t cols, float eps, int32_t dtype, dp_stream_t stream) {
  if (!x || !w || !b || !y) return DP_ERR_ARG;
  if (rows <= 0 || ldx % 4 || ldy % 4) return DP_ERR_SHAPE;
  if (cols > 256 && (ldy % 8 || (uintptr_t)y % 16)) return DP_ERR_ALIGN;   // 16-B row stores
  hipStream_t s = (hipStream_t)stream;
  LnW lw{};
  lw.w[0] = w;
  lw.b[0] = b;
  lw.rpg = rows;
  if (dtype == DP_BF16) return ln_launch<KBF16>(x, ldx, lw, (u16*)y, ldy, rows, cols, eps, s);
  if (dtype == DP_F16) return ln_launch<KF16>(x, ldx, lw, (u16*)y, ldy, rows, cols, eps, s);
  return DP_ERR_DTYPE;
}

extern "C" int dp_layernorm_grouped(const float* x, int64_t ldx, const float* const* w, const float* const* b,
                                    int32_t groups, void* y, int64_t ldy, int32_t rows_per_group, int32_t cols,
                                    float eps, int32_t dtype, dp_stream_t stream) {
  if (!x || !w || !b || !y || groups < 1 || groups > LN_MAX_GROUPS) return DP_ERR_ARG;
  if (rows_per_group <= 0 || ldx % 4 || ldy % 4) return DP_ERR_SHAPE;
  if (cols > 256 && (ldy % 8 || (uintptr_t)y % 16)) return DP_ERR_ALIGN;
  LnW lw{};
  for (int g = 0; g < groups; ++g) {
    if (!w[g] || !b[g]) return DP_ERR_ARG;
    lw.w[g] = w[g];
    lw.b[g] = b[g];
  }
  lw.rpg = rows_per_group;
  const int rows = groups * rows_per_group;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DP_BF16) return ln_launch<KBF16>(x, ldx, lw, (u16*)y, ldy, rows, cols, eps, s);
  if (dtype == DP_F16) return ln_launch<KF16>(x, ldx, lw, (u16*)y, ldy, rows, cols, eps, s);
  return DP_ERR_DTYPE;
}

extern "C" int dp_normalize_u8(const uint8_t* img, int32_t H, int32_t W, void* out, int32_t out_dtype,
                               dp_stream_t stream) {
  if (!img || !out) return DP_ERR_ARG;
  if (H <= 0 || W <= 0) return DP_ERR_SHAPE;
  const int HW = H * W;
  hipStream_t s = (hipStream_t)stream;
  dim3 g(blocks_for(HW, 256));
  if (out_dtype == DP_F32) hipLaunchKernelGGL(normalize_kernel<DP_F32>, g, dim3(256), 0, s, img, HW, out);
  else if (out_dtype == DP_BF16) hipLaunchKernelGGL(normalize_kernel<DP_BF16>, g, dim3(256), 0, s, img, HW, out);
  else if (out_dtype == DP_F16) hipLaunchKernelGGL(normalize_kernel<DP_F16>, g, dim3(256), 0, s, img, HW, out);
  else return DP_ERR_DTYPE;
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_resize(const void* src, int32_t src_dtype, int32_t C, int32_t H, int32_t W, float* dst,
                         int32_t OH, int32_t OW, int32_t mode, dp_stream_t stream) {
  if (!src || !dst) return DP_ERR_ARG;
  if (C <= 0 || H <= 0 || W <= 0 || OH <= 0 || OW <= 0) return DP_ERR_SHAPE;
  if (mode != DP_INTERP_BILINEAR && mode != DP_INTERP_BICUBIC) return DP_ERR_ARG;
  const long long total = (long long)C * OH * OW;
  const float sh = (float)H / (float)OH, sw = (float)W / (float)OW;
  hipStream_t s = (hipStream_t)stream;
  if (H == OH && W == OW && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0) {   // (the 1536^2 infer prologue)
    dim3 gc(blocks_for((total + 3) / 4, 256));
    if (src_dtype == DP_F32) hipLaunchKernelGGL(resize_copy_kernel<DP_F32>, gc, dim3(256), 0, s, src, dst, total);
    else if (src_dtype == DP_BF16) hipLaunchKernelGGL(resize_copy_kernel<DP_BF16>, gc, dim3(256), 0, s, src, dst, total);
    else if (src_dtype == DP_F16) hipLaunchKernelGGL(resize_copy_kernel<DP_F16>, gc, dim3(256), 0, s, src, dst, total);
    else return DP_ERR_DTYPE;
    DP_CHECK_LAUNCH();
    return 0;
  }
  dim3 g(blocks_for(total, 256));
#define DP_RS(M_) do { \
    if (src_dtype == DP_F32) hipLaunchKernelGGL((resize_kernel<DP_F32, M_>), g, dim3(256), 0, s, src, C, H, W, dst, OH, OW, sh, sw); \
    else if (src_dtype == DP_BF16) hipLaunchKernelGGL((resize_kernel<DP_BF16, M_>), g, dim3(256), 0, s, src, C, H, W, dst, OH, OW, sh, sw); \
    else if (src_dtype == DP_F16) hipLaunchKernelGGL((resize_kernel<DP_F16, M_>), g, dim3(256), 0, s, src, C, H, W, dst, OH, OW, sh, sw); \
    else return DP_ERR_DTYPE; } while (0)
  if (mode == DP_INTERP_BILINEAR) DP_RS(DP_INTERP_BILINEAR);
  else DP_RS(DP_INTERP_BICUBIC);
#undef DP_RS
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_resize_bilinear(const void* src, int32_t src_dtype, int32_t C, int32_t H, int32_t W, float* dst,
                                  int32_t OH, int32_t OW, dp_stream_t stream) {
  return dp_resize(src, src_dtype, C, H, W, dst, OH, OW, DP_INTERP_BILINEAR, stream);
}

extern "C" int dp_patchify_pyramid(const float* x0, void* cols, int32_t dtype, dp_stream_t stream) {
  if (!x0 || !cols) return DP_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  dim3 g(blocks_for(35 * 576 * 48, 256));
  if (dtype == DP_BF16) hipLaunchKernelGGL(patchify_kernel<KBF16>, g, dim3(256), 0, s, x0, (u16*)cols);
  else if (dtype == DP_F16) hipLaunchKernelGGL(patchify_kernel<KF16>, g, dim3(256), 0, s, x0, (u16*)cols);
  else return DP_ERR_DTYPE;
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_vit_cls_rows(float* x, const float* cls, const float* pos, int32_t n, dp_stream_t stream) {
  if (!x || !cls || !pos) return DP_ERR_ARG;
  if (n <= 0) return DP_ERR_SHAPE;
  hipLaunchKernelGGL(cls_kernel, dim3(blocks_for(n * 1024, 256)), dim3(256), 0, (hipStream_t)stream, x, cls, pos, n);
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_merge_windows(const void* src, int32_t src_dtype, int64_t ld, int32_t w0, int32_t steps,
                                int32_t pad, void* dst, int32_t dtype, dp_stream_t stream) {
  return dp_merge_windows_range(src, src_dtype, ld, w0, steps, pad, 0, steps * steps, dst, dtype, stream);
}

extern "C" int dp_merge_windows_range(const void* src, int32_t src_dtype, int64_t ld, int32_t w0, int32_t steps,
                                      int32_t pad, int32_t wlo, int32_t whi, void* dst, int32_t dtype,
                                      dp_stream_t stream) {
  if (!src || !dst) return DP_ERR_ARG;
  if (steps <= 0 || pad < 0 || (steps > 1 && 24 - 2 * pad <= 0) || ld % 8) return DP_ERR_SHAPE;
  if (wlo < 0 || whi > steps * steps || wlo >= whi) return DP_ERR_SHAPE;
  const int S = steps == 1 ? 24 : 2 * (24 - pad) + (steps - 2) * (24 - 2 * pad);
  const long long total = (long long)S * S * 128;
  hipStream_t s = (hipStream_t)stream;
  dim3 g(blocks_for(total, 256));
  if (src_dtype != DP_F32 && src_dtype != dtype) return DP_ERR_DTYPE;
  if (dtype == DP_BF16) {
    if (src_dtype == DP_F32) hipLaunchKernelGGL((merge_kernel<KBF16, DP_F32>), g, dim3(256), 0, s, src, ld, w0, steps, pad, S, (u16*)dst, wlo, whi);
    else hipLaunchKernelGGL((merge_kernel<KBF16, DP_BF16>), g, dim3(256), 0, s, src, ld, w0, steps, pad, S, (u16*)dst, wlo, whi);
  } else if (dtype == DP_F16) {
    if (src_dtype == DP_F32) hipLaunchKernelGGL((merge_kernel<KF16, DP_F32>), g, dim3(256), 0, s, src, ld, w0, steps, pad, S, (u16*)dst, wlo, whi);
    else hipLaunchKernelGGL((merge_kernel<KF16, DP_F16>), g, dim3(256), 0, s, src, ld, w0, steps, pad, S, (u16*)dst, wlo, whi);
  } else {
    return DP_ERR_DTYPE;
  }
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_fov_tail(const void* x6, int32_t dtype, const float* w, float bias, float* fov_deg,
                           dp_stream_t stream) {
  if (!x6 || !w || !fov_deg) return DP_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DP_BF16) hipLaunchKernelGGL(fov_tail_kernel<KBF16>, dim3(1), dim3(256), 0, s, (const u16*)x6, w, bias, fov_deg);
  else if (dtype == DP_F16) hipLaunchKernelGGL(fov_tail_kernel<KF16>, dim3(1), dim3(256), 0, s, (const u16*)x6, w, bias, fov_deg);
  else return DP_ERR_DTYPE;
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_infer_epilogue_mode(const float* canonical, int32_t SH, int32_t SW, const float* fov_deg,
                                      int32_t use_given, double f_given, int32_t H, int32_t W, float* depth,
                                      float* f_px_out, int32_t* nonfinite, int32_t mode, dp_stream_t stream) {
  if (!canonical || !depth || (!use_given && !fov_deg)) return DP_ERR_ARG;
  if (H <= 0 || W <= 0 || SH <= 0 || SW <= 0) return DP_ERR_SHAPE;
  if (mode != DP_INTERP_BILINEAR && mode != DP_INTERP_BICUBIC) return DP_ERR_ARG;
  // reference: inverse_depth = canonical * (W / f_px) with W / f_px a Python (double) scalar
  const float given_scale = use_given ? (float)((double)W / f_given) : 0.f;
  dim3 g(blocks_for((long long)H * W, 256));
  if (mode == DP_INTERP_BILINEAR)
    hipLaunchKernelGGL(infer_epi_kernel<DP_INTERP_BILINEAR>, g, dim3(256), 0, (hipStream_t)stream, canonical, SH, SW,
                       fov_deg, use_given, given_scale, (float)f_given, H, W, depth, f_px_out, (int*)nonfinite);
  else
    hipLaunchKernelGGL(infer_epi_kernel<DP_INTERP_BICUBIC>, g, dim3(256), 0, (hipStream_t)stream, canonical, SH, SW,
                       fov_deg, use_given, given_scale, (float)f_given, H, W, depth, f_px_out, (int*)nonfinite);
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_infer_epilogue(const float* canonical, int32_t SH, int32_t SW, const float* fov_deg,
                                 int32_t use_given, double f_given, int32_t H, int32_t W, float* depth,
                                 float* f_px_out, int32_t* nonfinite, dp_stream_t stream) {
  return dp_infer_epilogue_mode(canonical, SH, SW, fov_deg, use_given, f_given, H, W, depth, f_px_out, nonfinite,
                                DP_INTERP_BILINEAR, stream);
}

extern "C" int dp_resize_u8_cv(const uint8_t* src, int32_t H, int32_t W, uint8_t* dst, int32_t OH, int32_t OW,
                               int32_t interpolation, dp_stream_t stream) {
  if (!src || !dst) return DP_ERR_ARG;
  if (H <= 0 || W <= 0 || OH <= 0 || OW <= 0) return DP_ERR_SHAPE;
  if (interpolation != DP_CV_INTER_LINEAR && interpolation != DP_CV_INTER_AREA) return DP_ERR_ARG;
  // cv::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale (doubles)
  const double sx = 1.0 / ((double)OW / W), sy = 1.0 / ((double)OH / H);
  int mode = 0, isx = 0, isy = 0, tail0 = 0;
  if (interpolation == DP_CV_INTER_AREA && sx >= 1.0 && sy >= 1.0) {
    isx = (int)lrint(sx);
    isy = (int)lrint(sy);
    const double eps = 2.220446049250313e-16;
    if (fabs(sx - isx) < eps && fabs(sy - isy) < eps) {
      mode = 1;
      // the 2 x 2 SIMD loop takes whole groups of 16 pixels (48 bytes) of each row
      tail0 = OW * 3 >= 48 ? (OW / 16) * 16 : 0;
    } else {
      mode = 2;
    }
  } else {
    // (INTER_AREA on an upscale is INTER_LINEAR in OpenCV as well)
    const int width = OW * 3;
    int x = width >= 16 ? (width / 16) * 16 : 0;
    while (x < width - 8) x += 8;
    tail0 = x;     // first byte of each row that the scalar tail of the SIMD vertical pass writes
  }
  const long long n = (long long)OH * OW;
  hipLaunchKernelGGL(cv_resize_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, src, H, W, dst,
                     OH, OW, mode, sy, sx, isy, isx, tail0);
  DP_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- point cloud
// depth_to_3d (reference img_to_normalized_pointcloud.py:819-856) with the row-major
// compaction of numpy boolean indexing: valid = !isnan(d) && d > 0;
//   x = -1 * (u - W/2) * z / f,  y = -1 * (v - H/2) * z / f,  z = d      (fp64, numpy's order)
// Three launches: per-row valid counts, one exclusive scan over rows, per-row scatter
// (a block-level prefix over each 256-pixel chunk keeps the reference point order).
namespace {

__device__ __forceinline__ bool depth_valid(float d) { return !(d != d) && d > 0.f; }

template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {
    const int a = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  total = sh[NT - 1];
  const int ex = sh[t] - v;
  __syncthreads();
  return ex;
}

__global__ void __launch_bounds__(256) pts_count_kernel(const float* __restrict__ depth, int W, int* __restrict__ rows) {
  __shared__ int sh[256];
  const int y = blockIdx.x;
  int c = 0;
  for (int x = threadIdx.x; x < W; x += 256) c += depth_valid(depth[(long long)y * W + x]);
  int total;
  block_excl_scan<256>(c, sh, total);
  if (threadIdx.x == 0) rows[y] = total;
}

__global__ void __launch_bounds__(1024) pts_scan_kernel(int* __restrict__ rows, int H) {
  __shared__ int sh[1024];
  int carry = 0;
  for (int base = 0; base < H; base += 1024) {
    const int i = base + threadIdx.x;
    const int v = i < H ? rows[i] : 0;
    int total;
    const int ex = block_excl_scan<1024>(v, sh, total);
    if (i < H) rows[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) rows[H] = carry;
}

__global__ void __launch_bounds__(256) pts_scatter_kernel(const float* __restrict__ depth, int H, int W,
                                                          const float* __restrict__ f_dev, double f_host, int use_host,
                                                          const uint8_t* __restrict__ rgb, const int* __restrict__ rows,
                                                          double* __restrict__ xyz, uint8_t* __restrict__ rgb_out) {
  __shared__ int sh[256];
  const int y = blockIdx.x;
  const double f = use_host ? f_host : (double)*f_dev;
  const double cx = W / 2.0, cy = H / 2.0;
  int off = rows[y];
  for (int x0 = 0; x0 < W; x0 += 256) {
    const int x = x0 + threadIdx.x;
    const float d = x < W ? depth[(long long)y * W + x] : 0.f;
    const int ok = x < W && depth_valid(d);
    int total;
    const int ex = block_excl_scan<256>(ok, sh, total);
    if (ok) {
      const long long i = off + ex;
      const double z = (double)d;
      double px = -1.0 * ((double)x - cx);
      px = px * z;
      px = px / f;
      double py = -1.0 * ((double)y - cy);
      py = py * z;
      py = py / f;
      xyz[3 * i] = px;
      xyz[3 * i + 1] = py;
      xyz[3 * i + 2] = z;
      if (rgb_out) {
        const uint8_t* s = rgb + ((long long)y * W + x) * 3;
        rgb_out[3 * i] = s[0];
        rgb_out[3 * i + 1] = s[1];
        rgb_out[3 * i + 2] = s[2];
      }
    }
    off += total;
  }
}


// ------------------------------------------------- depth map -> 8-bit colour / 16-bit grey
// The frame loop's writers (reference generate_depth_maps.py:15-44 colorize_depth, :135-143 --raw)
// on the GPU: nanmin / nanmax of the depth map (order-preserving integer keys, NaN skipped), then
// per pixel n = (d - min) / (max - min) in fp32 (IEEE division, as numpy's float32 arithmetic),
// colour: np.clip(n, 0, 1), matplotlib Colormap.__call__'s index trunc(n * N) (N -> N - 1, NaN ->
// the "bad" entry) into the colormap's byte table (host-built: (lut * 255).astype(uint8));
// raw: (uint16)(n * 65535) (NaN -> 0, numpy's cast on x86).
__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {   // inverse of order_key; 0xffffffff / 0 -> NaN
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void minmax_init_kernel(uint32_t* __restrict__ mm) {
  if (threadIdx.x < 2) mm[threadIdx.x] = threadIdx.x == 0 ? 0xffffffffu : 0u;
}

__global__ void __launch_bounds__(256) minmax_kernel(const float* __restrict__ d, long long n, uint32_t* __restrict__ mm) {
  __shared__ uint32_t red[2][4];
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  const long long stride = (long long)gridDim.x * 256 * 4;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    float v[4];
    if (i + 3 < n && ((uintptr_t)(d + i) & 15) == 0) {
      const float4 q = *(const float4*)(d + i);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      #pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = i + r < n ? d[i + r] : __builtin_nanf("");
    }
    #pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (v[r] == v[r]) {
        const uint32_t k = order_key(v[r]);
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
      }
    }
  }
  #pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t a = __shfl_xor(kmin, o), b = __shfl_xor(kmax, o);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = kmin; red[1][threadIdx.x >> 6] = kmax; }
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t a = red[0][threadIdx.x & 3], b = red[1][threadIdx.x & 3];
    #pragma unroll
    for (int o = 2; o > 0; o >>= 1) {
      const uint32_t a2 = __shfl_xor(a, o), b2 = __shfl_xor(b, o);
      a = a2 < a ? a2 : a;
      b = b2 > b ? b2 : b;
    }
    if (threadIdx.x == 0) {
      atomicMin(mm, a);
      atomicMax(mm + 1, b);
    }
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) depth_color_kernel(const float* __restrict__ d, long long n,
                                                          const uint32_t* __restrict__ mm, const uint8_t* __restrict__ lut,
                                                          int N, void* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float mn = key_float(mm[0]), mx = key_float(mm[1]);
  const float v = (d[i] - mn) / (mx - mn);
  if constexpr (MODE == 0) {
    int idx;
    if (v != v) {
      idx = N + 2;                                   // matplotlib's _i_bad
    } else {
      float x = fminf(fmaxf(v, 0.f), 1.f) * (float)N;
      if (x == (float)N) x = (float)(N - 1);
      idx = (int)x;
    }
    uint8_t* o = (uint8_t*)out + 3 * i;
    o[0] = lut[3 * idx];
    o[1] = lut[3 * idx + 1];
    o[2] = lut[3 * idx + 2];
  } else {
    const float r = v * 65535.f;
    ((uint16_t*)out)[i] = r == r ? (uint16_t)(int)r : (uint16_t)0;
  }
}
}  // namespace

extern "C" int dp_depth_to_image(const float* depth, int64_t n, uint32_t* minmax, const uint8_t* lut, int32_t lut_n,
                                 int32_t mode, void* out, dp_stream_t stream) {
  if (!depth || !minmax || !out || (mode == DP_DEPTH_IMG_COLOR && (!lut || lut_n <= 0))) return DP_ERR_ARG;
  if (mode != DP_DEPTH_IMG_COLOR && mode != DP_DEPTH_IMG_RAW16) return DP_ERR_ARG;
  if (n <= 0) return DP_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(minmax_init_kernel, dim3(1), dim3(64), 0, s, minmax);
  const int g = (int)(n / 1024 + 1 < 1024 ? n / 1024 + 1 : 1024);
  hipLaunchKernelGGL(minmax_kernel, dim3(g), dim3(256), 0, s, depth, (long long)n, minmax);
  if (mode == DP_DEPTH_IMG_COLOR)
    hipLaunchKernelGGL(depth_color_kernel<0>, dim3(blocks_for(n, 256)), dim3(256), 0, s, depth, (long long)n, minmax,
                       lut, lut_n, out);
  else
    hipLaunchKernelGGL(depth_color_kernel<1>, dim3(blocks_for(n, 256)), dim3(256), 0, s, depth, (long long)n, minmax,
                       lut, lut_n, out);
  DP_CHECK_LAUNCH();
  return 0;
}

extern "C" int dp_depth_to_points(const float* depth, int32_t H, int32_t W, const float* f_px_dev, double f_px,
                                  int32_t use_given, const uint8_t* rgb_hwc, int32_t* row_offsets, double* xyz,
                                  uint8_t* rgb_out, dp_stream_t stream) {
  if (!depth || !row_offsets || !xyz || (!use_given && !f_px_dev) || (rgb_out && !rgb_hwc)) return DP_ERR_ARG;
  if (H <= 0 || W <= 0) return DP_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pts_count_kernel, dim3(H), dim3(256), 0, s, depth, W, row_offsets);
  hipLaunchKernelGGL(pts_scan_kernel, dim3(1), dim3(1024), 0, s, row_offsets, H);
  hipLaunchKernelGGL(pts_scatter_kernel, dim3(H), dim3(256), 0, s, depth, H, W, f_px_dev, f_px, use_given, rgb_hwc,
                     row_offsets, xyz, rgb_out);
  DP_CHECK_LAUNCH();
  return 0;
}
