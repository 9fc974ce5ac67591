// HBM-bound kernels of the DVC forward: layout conversion, pyramids, warp (grid_sample),
// bilinear 2x upsampling, GDN, recon/loss finalisation and the bpp-estimate reductions.
//
// Float expressions that the reference computes as separate ATen ops are written with
// contraction off (no FMA fusion) and in the reference's operand order, so results track the
// CPU path to ~1 ulp.
#include "fvc_common.h"
#include <stdlib.h>
#include "fvc_dist.h"
#include <string.h>

#pragma clang fp contract(off)

namespace {

constexpr int kBlk = 256;
constexpr int kRedBlocks = 1024;  // fixed grid for deterministic reductions

__device__ __forceinline__ int grid_stride_start() { return blockIdx.x * blockDim.x + threadIdx.x; }

// ------------------------------------------------------------------ layout
__global__ void k_nchw_to_nhwc(const float* __restrict__ src, float* __restrict__ dst, int B, int C,
                               int H, int W, int cp) {
  const size_t npix = (size_t)B * H * W;
  for (size_t p = grid_stride_start(); p < npix; p += (size_t)gridDim.x * blockDim.x) {
    const size_t b = p / ((size_t)H * W);
    const size_t hw = p - b * H * W;
    for (int c = 0; c < cp; ++c) {
      dst[p * cp + c] = c < C ? src[(b * C + c) * H * W + hw] : 0.f;
    }
  }
}

__global__ void k_nhwc_to_nchw(const float* __restrict__ src, float* __restrict__ dst, int B, int C,
                               int H, int W, int cp, int clamp01) {
  const size_t n = (size_t)B * C * H * W;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t hw = e % ((size_t)H * W);
    const size_t bc = e / ((size_t)H * W);
    const size_t c = bc % C, b = bc / C;
    const float v = src[(b * H * W + hw) * cp + c];
    dst[e] = clamp01 ? fminf(fmaxf(v, 0.f), 1.f) : v;
  }
}

// avg_pool2d(k=2,s=2): ((x00 + x01) + x10) + x11, then / 4 (ATen CPU order)
// Second half of a cout <= 4 conv / transposed conv computed as a tap-partial GEMM (the x3
// kernel's 1x1 pass writes P[b][iy][ix][t * cout + co] = sum_ci x[b][iy][ix][ci] w_t[ci][co] for
// every input pixel and tap t = ky * ks + kx): y[b][Y][X][co] = bias[co] + sum over the taps that
// reach (Y, X) of P at the source pixel, then activation, residual, exp; pad channel 3 (and any
// co >= cout) = 0. Conv (stride 1): source = (Y + ky - pad, X + kx - pad); transposed (stride s,
// output padding s - 1): source = ((Y + pad - ky) / s, (X + pad - kx) / s) where divisible.
// Fixed tap order: deterministic. HBM-bound (P is re-read from L1/L2 by neighbouring outputs).
template <int KS, int COUT, int TR>
__global__ __launch_bounds__(256) void k_tap_gather(const float* __restrict__ P, int pcp,
                                                    const float* __restrict__ bias,
                                                    const float* __restrict__ res, float* __restrict__ y,
                                                    int B, int H, int W, int Ho, int Wo, float act_slope,
                                                    int post_op) {
  constexpr int pad = KS / 2;
  const size_t n = (size_t)B * Ho * Wo;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const int X = e % Wo;
    const int Y = (e / Wo) % Ho;
    const size_t b = e / ((size_t)Wo * Ho);
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = bias[co];
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      // transposed (stride 2): only taps with ky = Y + pad (mod 2) reach row Y
      if (TR && ((Y + pad - ky) & 1)) continue;
      const int iy = TR ? (Y + pad - ky) >> 1 : Y + ky - pad;  // >> 1: floor for negatives
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        if (TR && ((X + pad - kx) & 1)) continue;
        const int ix = TR ? (X + pad - kx) >> 1 : X + kx - pad;
        if (ix < 0 || ix >= W) continue;
        const float* src = P + ((b * H + iy) * W + ix) * pcp + (ky * KS + kx) * COUT;
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[co] += src[co];
      }
    }
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    float* ov = &o.x;
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float v = acc[co];
      v = fmaxf(v, v * act_slope);
      if (res) v += res[e * 4 + co];
      if (post_op == FVC_POST_EXP) v = expf(v);
      ov[co] = v;
    }
    reinterpret_cast<float4*>(y)[e] = o;
  }
}

// Stage an IR x IC pixel window of P (c4n float4 per pixel, origin (r0, c0), zeros outside the
// image) into LDS at pixel stride ps: eight loads per thread in flight per batch, every address
// clamped into the image and out-of-image values selected to zero after the load (a per-element
// branch made each load wait for the previous one's LDS write: one HBM round trip per element)
__device__ __forceinline__ void stage_p_window(const float* __restrict__ Pb, int pcp, int H, int W, int r0, int c0,
                                               int IR, int IC, int ps, float* sp) {
  constexpr int NB = 8;
  const int c4n = pcp >> 2;
  const int total = IR * IC * c4n;
  for (int e0 = threadIdx.x; e0 < total; e0 += NB * blockDim.x) {
    float4 v[NB];
    int dst[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int e = e0 + k * blockDim.x;
      const int ee = e < total ? e : total - 1;
      const int c4 = ee % c4n, p = ee / c4n;
      const int iy = r0 + p / IC, ix = c0 + p % IC;
      const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
      const float4 t = *reinterpret_cast<const float4*>(Pb + ((size_t)cy * W + cx) * pcp + 4 * c4);
      v[k] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      dst[k] = e < total ? p * ps + 4 * c4 : -1;
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (dst[k] >= 0) {
        float* d = sp + dst[k];
        d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
      }
    }
  }
}

// Stride-1 3x3 tap gather through LDS (the second half of the fused producer + tap path): a block
// stages the P tile of its 16 x 32 outputs plus a 1-pixel halo with coalesced 16-B loads (zeros
// outside the image), pixel stride pcp + 1 words so the per-tap reads of consecutive outputs hit
// distinct banks, then sums bias + taps in k_tap_gather's order (an out-of-image tap adds +0).
template <int COUT, int TH>
__global__ __launch_bounds__(256) void k_tap_gather3_lds(const float* __restrict__ P, int pcp,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ res, float* __restrict__ y,
                                                         int H, int W, float act_slope, int post_op) {
  constexpr int TW = 32, IR = TH + 2, IC = TW + 2;
  extern __shared__ float sp[];
  const int ps = pcp + 1;
  const size_t b = blockIdx.z;
  const int y0 = blockIdx.y * TH, x0 = blockIdx.x * TW;
  const float* Pb = P + b * H * W * pcp;
  stage_p_window(Pb, pcp, H, W, y0 - 1, x0 - 1, IR, IC, ps, sp);
  __syncthreads();
  for (int q = threadIdx.x; q < TH * TW; q += blockDim.x) {
    const int r = q / TW, c = q % TW;
    const int Y = y0 + r, X = x0 + c;
    if (Y >= H || X >= W) continue;
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = bias[co];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float* src = sp + ((r + ky) * IC + c + kx) * ps + (ky * 3 + kx) * COUT;
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[co] += src[co];
      }
    const size_t e = (b * H + Y) * W + X;
    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (res) rv = reinterpret_cast<const float4*>(res)[e];
    const float rr[4] = {rv.x, rv.y, rv.z, rv.w};
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    float* ov = &o.x;
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float v = acc[co];
      v = fmaxf(v, v * act_slope);
      if (res) v += rr[co];
      if (post_op == FVC_POST_EXP) v = expf(v);
      ov[co] = v;
    }
    reinterpret_cast<float4*>(y)[e] = o;
  }
}

// Transposed (stride 2, output padding 1) tap gather through LDS: a block's 16 x 32 outputs read
// input rows Y0/2 - 1 .. Y0/2 + 8 and columns X0/2 - 1 .. X0/2 + 17 of P (k = 3 or 5), staged
// once with coalesced 16-B loads; per output the same tap order as k_tap_gather.
template <int KS, int COUT, int TH>
__global__ __launch_bounds__(256) void k_tap_gather_t2_lds(const float* __restrict__ P, int pcp,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ res, float* __restrict__ y,
                                                           int H, int W, float act_slope, int post_op) {
  // output rows Y0 .. Y0 + TH - 1 read input rows Y0/2 - 1 .. Y0/2 + TH/2 (k <= 5)
  constexpr int TW = 32, IR = TH / 2 + 2, IC = 19, pad = KS / 2;
  extern __shared__ float sp[];
  const int ps = pcp + 1;
  const int Ho = 2 * H, Wo = 2 * W;
  const size_t b = blockIdx.z;
  const int Y0 = blockIdx.y * TH, X0 = blockIdx.x * TW;
  const int r0 = Y0 / 2 - 1, c0 = X0 / 2 - 1;
  const float* Pb = P + b * H * W * pcp;
  stage_p_window(Pb, pcp, H, W, r0, c0, IR, IC, ps, sp);
  __syncthreads();
  for (int q = threadIdx.x; q < TH * TW; q += blockDim.x) {
    const int Y = Y0 + q / TW, X = X0 + q % TW;
    if (Y >= Ho || X >= Wo) continue;
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = bias[co];
#pragma unroll
    for (int ky = 0; ky < KS; ++ky) {
      if ((Y + pad - ky) & 1) continue;
      const int lr = ((Y + pad - ky) >> 1) - r0;  // in [0, IR): out-of-image rows hold zeros
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        if ((X + pad - kx) & 1) continue;
        const int lc = ((X + pad - kx) >> 1) - c0;
        const float* src = sp + (lr * IC + lc) * ps + (ky * KS + kx) * COUT;
#pragma unroll
        for (int co = 0; co < COUT; ++co) acc[co] += src[co];
      }
    }
    const size_t e = (b * Ho + Y) * Wo + X;
    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (res) rv = reinterpret_cast<const float4*>(res)[e];
    const float rr[4] = {rv.x, rv.y, rv.z, rv.w};
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    float* ov = &o.x;
#pragma unroll
    for (int co = 0; co < COUT; ++co) {
      float v = acc[co];
      v = fmaxf(v, v * act_slope);
      if (res) v += rr[co];
      if (post_op == FVC_POST_EXP) v = expf(v);
      ov[co] = v;
    }
    reinterpret_cast<float4*>(y)[e] = o;
  }
}

__global__ void k_avgpool2(const float* __restrict__ src, float* __restrict__ dst, int B, int H, int W,
                           int cp) {
  const int Ho = H / 2, Wo = W / 2, c4n = cp / 4;
  const size_t n = (size_t)B * Ho * Wo * c4n;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const int c4 = e % c4n;
    size_t p = e / c4n;
    const int ox = p % Wo; p /= Wo;
    const int oy = p % Ho;
    const size_t b = p / Ho;
    const float4* s = reinterpret_cast<const float4*>(src);
    const size_t r0 = ((b * H + 2 * oy) * W + 2 * ox) * c4n + c4;
    const size_t r1 = r0 + (size_t)W * c4n;
    const float4 a = s[r0], bb = s[r0 + c4n], c = s[r1], d = s[r1 + c4n];
    float4 o;
    o.x = (((a.x + bb.x) + c.x) + d.x) / 4.f;
    o.y = (((a.y + bb.y) + c.y) + d.y) / 4.f;
    o.z = (((a.z + bb.z) + c.z) + d.z) / 4.f;
    o.w = (((a.w + bb.w) + c.w) + d.w) / 4.f;
    reinterpret_cast<float4*>(dst)[e] = o;
  }
}

// ------------------------------------------------------------------ warp (torch_warp)
// torch.linspace(-1, 1, n)[i] as ATen computes it (symmetric two-sided formula)
__device__ __forceinline__ float linspace_m1p1(int i, int n) {
  if (n == 1) return -1.f;
  const float step = 2.f / (float)(n - 1);
  const int half = n / 2;
  return (i < half) ? (-1.f + step * (float)i) : (1.f - step * (float)(n - 1 - i));
}

struct WarpTap {
  int x0, y0;
  float nw, ne, sw, se;
  bool vx1, vy1;
};

// grid = linspace grid + flow/((n-1)/2); grid_sample(bilinear, border, align_corners=False)
// (endecoder.py:52-67; ATen CPU GridSamplerKernel unnormalize/clip/interp order)
__device__ __forceinline__ WarpTap warp_tap(int y, int x, float fx, float fy, int H, int W) {
  const float gx = linspace_m1p1(x, W) + fx / ((float)(W - 1) / 2.f);
  const float gy = linspace_m1p1(y, H) + fy / ((float)(H - 1) / 2.f);
  float ix = (gx + 1.f) * ((float)W / 2.f) - 0.5f;
  float iy = (gy + 1.f) * ((float)H / 2.f) - 0.5f;
  ix = fminf(fmaxf(ix, 0.f), (float)(W - 1));
  iy = fminf(fmaxf(iy, 0.f), (float)(H - 1));
  const float xw = floorf(ix), yn = floorf(iy);
  const float w = ix - xw, e = 1.f - w;
  const float n = iy - yn, s = 1.f - n;
  WarpTap t;
  t.x0 = (int)xw;
  t.y0 = (int)yn;
  t.nw = s * e; t.ne = s * w; t.sw = n * e; t.se = n * w;
  t.vx1 = t.x0 + 1 < W;
  t.vy1 = t.y0 + 1 < H;
  return t;
}

__device__ __forceinline__ float4 warp_sample4(const float* im, size_t bbase, int W, int c4n, int c4,
                                               const WarpTap& t) {
  const float4* s = reinterpret_cast<const float4*>(im);
  const size_t r0 = (bbase + (size_t)t.y0 * W + t.x0) * c4n + c4;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 vnw = s[r0];
  const float4 vne = t.vx1 ? s[r0 + c4n] : z;
  const float4 vsw = t.vy1 ? s[r0 + (size_t)W * c4n] : z;
  const float4 vse = (t.vx1 && t.vy1) ? s[r0 + (size_t)W * c4n + c4n] : z;
  float4 o;
  o.x = ((vnw.x * t.nw + vne.x * t.ne) + vsw.x * t.sw) + vse.x * t.se;
  o.y = ((vnw.y * t.nw + vne.y * t.ne) + vsw.y * t.sw) + vse.y * t.se;
  o.z = ((vnw.z * t.nw + vne.z * t.ne) + vsw.z * t.sw) + vse.z * t.se;
  o.w = ((vnw.w * t.nw + vne.w * t.ne) + vsw.w * t.sw) + vse.w * t.se;
  return o;
}

// warp_sample4 with every tap loaded unconditionally (an out-of-image tap reads the clamped edge
// pixel): when x0 + 1 == W the border clamp made ix == W - 1 exactly, so the east weights are 0 and
// the tap adds 0 * v where warp_sample4 adds 0 * 0: the same values for finite images (a zero can
// only differ in sign, and only in an exactly-zero sum); no branches, so the compiler can count the
// loads in flight exactly
__device__ __forceinline__ float4 warp_sample4_nb(const float4* __restrict__ s, unsigned bbase, int W, int H,
                                                  const WarpTap& t) {
  const unsigned r0 = bbase + (unsigned)t.y0 * W + t.x0;
  const unsigned dx = t.vx1 ? 1u : 0u, dy = t.vy1 ? (unsigned)W : 0u;
  const float4 vnw = s[r0], vne = s[r0 + dx], vsw = s[r0 + dy], vse = s[r0 + dy + dx];
  float4 o;
  o.x = ((vnw.x * t.nw + vne.x * t.ne) + vsw.x * t.sw) + vse.x * t.se;
  o.y = ((vnw.y * t.nw + vne.y * t.ne) + vsw.y * t.sw) + vse.y * t.se;
  o.z = ((vnw.z * t.nw + vne.z * t.ne) + vsw.z * t.sw) + vse.z * t.se;
  o.w = ((vnw.w * t.nw + vne.w * t.ne) + vsw.w * t.sw) + vse.w * t.se;
  return o;
}

__global__ void k_warp(const float* __restrict__ im, const float* __restrict__ flow, float* __restrict__ out,
                       int B, int H, int W, int cp) {
  const int c4n = cp / 4;
  const size_t npix = (size_t)B * H * W;
  for (size_t p = grid_stride_start(); p < npix; p += (size_t)gridDim.x * blockDim.x) {
    const int x = p % W;
    const int y = (p / W) % H;
    const size_t b = p / ((size_t)H * W);
    const float4 f = reinterpret_cast<const float4*>(flow)[p];
    const WarpTap t = warp_tap(y, x, f.x, f.y, H, W);
    for (int c4 = 0; c4 < c4n; ++c4)
      reinterpret_cast<float4*>(out)[p * c4n + c4] = warp_sample4(im, b * H * W, W, c4n, c4, t);
  }
}

// ------------------------------------------------------------------ bilinear upsampling
struct UpIdx {
  int i0, i1;
  float l0, l1;
};

// ATen compute_indices_weights_linear: src = ac ? scale*d : max(scale*(d+0.5)-0.5, 0)
__device__ __forceinline__ UpIdx up_index(int d, int in, int out, int ac) {
  float src;
  if (ac) {  // = fvc_up_index_scaled (fvc_common.h), which the Winograd kernel's fused staging uses
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    const FvcUpIdx f = fvc_up_index_scaled(d, in, scale);
    return UpIdx{f.i0, f.i1, f.l0, f.l1};
  } else {
    const float scale = (float)in / (float)out;
    src = fmaxf(scale * ((float)d + 0.5f) - 0.5f, 0.f);
  }
  int i0 = (int)floorf(src);
  float lam = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  if (i0 > in - 1) i0 = in - 1;
  UpIdx u;
  u.i0 = i0;
  u.i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  u.l1 = lam;
  u.l0 = 1.f - lam;
  return u;
}

// the 2x upsample kernels' index: align_corners=True with the scale (in - 1) / (out - 1) computed once on
// the host (the float division ATen performs on the CPU; the Winograd kernel's fused upsample-add
// staging takes the same host value), else the half-pixel form of up_index
__device__ __forceinline__ UpIdx up2_index(int d, int in, int out, int ac, float s) {
  if (ac) {
    const FvcUpIdx f = fvc_up_index_scaled(d, in, s);
    return UpIdx{f.i0, f.i1, f.l0, f.l1};
  }
  return up_index(d, in, out, 0);
}

__device__ __forceinline__ float4 up_sample4(const float* src, size_t bbase, int w, int c4n, int c4,
                                             const UpIdx& uy, const UpIdx& ux) {
  const float4* s = reinterpret_cast<const float4*>(src);
  const float4 a = s[(bbase + (size_t)uy.i0 * w + ux.i0) * c4n + c4];
  const float4 b = s[(bbase + (size_t)uy.i0 * w + ux.i1) * c4n + c4];
  const float4 c = s[(bbase + (size_t)uy.i1 * w + ux.i0) * c4n + c4];
  const float4 d = s[(bbase + (size_t)uy.i1 * w + ux.i1) * c4n + c4];
  float4 o;
  o.x = fvc_lerp2d(a.x, b.x, c.x, d.x, ux.l0, ux.l1, uy.l0, uy.l1);
  o.y = fvc_lerp2d(a.y, b.y, c.y, d.y, ux.l0, ux.l1, uy.l0, uy.l1);
  o.z = fvc_lerp2d(a.z, b.z, c.z, d.z, ux.l0, ux.l1, uy.l0, uy.l1);
  o.w = fvc_lerp2d(a.w, b.w, c.w, d.w, ux.l0, ux.l1, uy.l0, uy.l1);
  return o;
}

// 64-channel form (Warp_net's c3_u / c4_u, endecoder.py:288-293): 32-bit indexes with the pixel
// and row divisions as multiply-high by a host-computed ceil(2^32 / d) plus one correction (exact for
// any 32-bit numerator: the estimate is floor(n / d) or one above it), instead of the generic
// kernel's 64-bit divisions per float4. Same arithmetic per element as k_up2_add.
__device__ __forceinline__ unsigned udiv_magic(unsigned n, unsigned d, unsigned m) {
  unsigned q = __umulhi(n, m);
  return q * d > n ? q - 1 : q;
}

__global__ void k_up2_add_q16(const float* __restrict__ src, const float* __restrict__ skip, float* __restrict__ out,
                              int B, int h, int w, int ac, float scale, unsigned mW, unsigned mH, float usy, float usx) {
  const unsigned H = 2u * h, W = 2u * w;
  const unsigned n = (unsigned)B * H * W * 16u;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const unsigned c4 = e & 15u;
    const unsigned p = e >> 4;
    const unsigned row = udiv_magic(p, W, mW);
    const int x = (int)(p - row * W);
    const unsigned b = udiv_magic(row, H, mH);
    const int y = (int)(row - b * H);
    const UpIdx uy = up2_index(y, h, (int)H, ac, usy), ux = up2_index(x, w, (int)W, ac, usx);
    const unsigned bb = b * (unsigned)h * (unsigned)w;
    const float4 a = s4[(bb + (unsigned)uy.i0 * w + ux.i0) * 16u + c4];
    const float4 bq = s4[(bb + (unsigned)uy.i0 * w + ux.i1) * 16u + c4];
    const float4 c = s4[(bb + (unsigned)uy.i1 * w + ux.i0) * 16u + c4];
    const float4 d = s4[(bb + (unsigned)uy.i1 * w + ux.i1) * 16u + c4];
    float4 v;
    v.x = fvc_lerp2d(a.x, bq.x, c.x, d.x, ux.l0, ux.l1, uy.l0, uy.l1);
    v.y = fvc_lerp2d(a.y, bq.y, c.y, d.y, ux.l0, ux.l1, uy.l0, uy.l1);
    v.z = fvc_lerp2d(a.z, bq.z, c.z, d.z, ux.l0, ux.l1, uy.l0, uy.l1);
    v.w = fvc_lerp2d(a.w, bq.w, c.w, d.w, ux.l0, ux.l1, uy.l0, uy.l1);
    if (scale != 1.f) { v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale; }
    if (skip) {
      const float4 sk = reinterpret_cast<const float4*>(skip)[e];
      v.x = sk.x + v.x; v.y = sk.y + v.y; v.z = sk.z + v.z; v.w = sk.w + v.w;
    }
    reinterpret_cast<float4*>(out)[e] = v;
  }
}

// NE elements per thread per iteration (e, e + stride, ...), all loads issued before the stores:
// more independent loads in flight per wave than the one-element loop (as k_mc_assemble_q); NT:
// the skip tensor by non-temporal loads (it is read once)
template <bool NT>
__device__ __forceinline__ float4 up2_q16_elem(const float4* __restrict__ s4, const float* __restrict__ skip,
                                               unsigned e, unsigned H, unsigned W, int h, int w, int ac, float scale,
                                               unsigned mW, unsigned mH, float usy, float usx) {
  const unsigned c4 = e & 15u;
  const unsigned p = e >> 4;
  const unsigned row = udiv_magic(p, W, mW);
  const int x = (int)(p - row * W);
  const unsigned b = udiv_magic(row, H, mH);
  const int y = (int)(row - b * H);
  const UpIdx uy = up2_index(y, h, (int)H, ac, usy), ux = up2_index(x, w, (int)W, ac, usx);
  const unsigned bb = b * (unsigned)h * (unsigned)w;
  const float4 a = s4[(bb + (unsigned)uy.i0 * w + ux.i0) * 16u + c4];
  const float4 bq = s4[(bb + (unsigned)uy.i0 * w + ux.i1) * 16u + c4];
  const float4 c = s4[(bb + (unsigned)uy.i1 * w + ux.i0) * 16u + c4];
  const float4 d = s4[(bb + (unsigned)uy.i1 * w + ux.i1) * 16u + c4];
  float4 v;
  v.x = fvc_lerp2d(a.x, bq.x, c.x, d.x, ux.l0, ux.l1, uy.l0, uy.l1);
  v.y = fvc_lerp2d(a.y, bq.y, c.y, d.y, ux.l0, ux.l1, uy.l0, uy.l1);
  v.z = fvc_lerp2d(a.z, bq.z, c.z, d.z, ux.l0, ux.l1, uy.l0, uy.l1);
  v.w = fvc_lerp2d(a.w, bq.w, c.w, d.w, ux.l0, ux.l1, uy.l0, uy.l1);
  if (scale != 1.f) { v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale; }
  if (skip) {
    float4 sk;
    if constexpr (NT) {
      const float* q = skip + 4 * (size_t)e;
      sk = make_float4(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1), __builtin_nontemporal_load(q + 2),
                       __builtin_nontemporal_load(q + 3));
    } else {
      sk = reinterpret_cast<const float4*>(skip)[e];
    }
    v.x = sk.x + v.x; v.y = sk.y + v.y; v.z = sk.z + v.z; v.w = sk.w + v.w;
  }
  return v;
}

template <int NE, bool NT>
__global__ void k_up2_add_q16p(const float* __restrict__ src, const float* __restrict__ skip, float* __restrict__ out,
                               int B, int h, int w, int ac, float scale, unsigned mW, unsigned mH, float usy,
                               float usx) {
  const unsigned H = 2u * h, W = 2u * w;
  const unsigned n = (unsigned)B * H * W * 16u;
  const unsigned st = gridDim.x * blockDim.x;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += NE * st) {
    unsigned ei[NE];
    float4 v[NE];
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      ei[k] = e + k * st < n ? e + k * st : e;
      v[k] = up2_q16_elem<NT>(s4, skip, ei[k], H, W, h, w, ac, scale, mW, mH, usy, usx);
    }
#pragma unroll
    for (int k = 0; k < NE; ++k) reinterpret_cast<float4*>(out)[ei[k]] = v[k];
  }
}

__global__ void k_up2_add(const float* __restrict__ src, const float* __restrict__ skip, float* __restrict__ out,
                          int B, int h, int w, int cp, int ac, float scale, float usy, float usx) {
  const int H = 2 * h, W = 2 * w, c4n = cp / 4;
  const size_t n = (size_t)B * H * W * c4n;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const int c4 = e % c4n;
    size_t p = e / c4n;
    const int x = p % W; p /= W;
    const int y = p % H;
    const size_t b = p / H;
    const UpIdx uy = up2_index(y, h, H, ac, usy), ux = up2_index(x, w, W, ac, usx);
    float4 v = up_sample4(src, b * h * w, w, c4n, c4, uy, ux);
    if (scale != 1.f) { v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale; }
    if (skip) {
      const float4 s = reinterpret_cast<const float4*>(skip)[e];
      v.x = s.x + v.x; v.y = s.y + v.y; v.z = s.z + v.z; v.w = s.w + v.w;
    }
    reinterpret_cast<float4*>(out)[e] = v;
  }
}

// 4-channel form of k_nchw_to_nhwc (frames and flows: C <= 4 into a 4-channel pixel): one 16-B
// store per pixel instead of four 4-B ones, the image split by a multiply-high division
__global__ void k_nchw_to_nhwc4(const float* __restrict__ src, float* __restrict__ dst, int B, int C,
                                unsigned HW, unsigned mHW) {
  const unsigned npix = (unsigned)B * HW;
  for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += gridDim.x * blockDim.x) {
    const unsigned b = udiv_magic(p, HW, mHW);
    const float* const sp = src + (size_t)b * C * HW + (p - b * HW);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (C > 0) v.x = sp[0];
    if (C > 1) v.y = sp[HW];
    if (C > 2) v.z = sp[2 * (size_t)HW];
    if (C > 3) v.w = sp[3 * (size_t)HW];
    reinterpret_cast<float4*>(dst)[p] = v;
  }
}

// ------------------------------------------------------------------ SpyNet level assembly
__device__ __forceinline__ void spynet_assemble_px(const float* __restrict__ im1, const float* __restrict__ im2,
                                                   const float* __restrict__ flow_prev, float* __restrict__ flow_up,
                                                   float* __restrict__ x8, size_t p, int x, int y, size_t b, int H,
                                                   int W) {
  const int h = H / 2, w = W / 2;
  float4 fu = make_float4(0.f, 0.f, 0.f, 0.f);
  if (flow_prev) {
    const UpIdx uy = up_index(y, h, H, 0), ux = up_index(x, w, W, 0);
    fu = up_sample4(flow_prev, b * h * w, w, 1, 0, uy, ux);
    fu.x = fu.x * 2.f; fu.y = fu.y * 2.f; fu.z = 0.f; fu.w = 0.f;
  }
  reinterpret_cast<float4*>(flow_up)[p] = fu;
  const WarpTap t = warp_tap(y, x, fu.x, fu.y, H, W);
  const float4 wv = warp_sample4(im2, b * H * W, W, 1, 0, t);
  const float4 a = reinterpret_cast<const float4*>(im1)[p];
  float4* o = reinterpret_cast<float4*>(x8) + p * 2;
  o[0] = make_float4(a.x, a.y, a.z, wv.x);
  o[1] = make_float4(wv.y, wv.z, fu.x, fu.y);
}

__global__ void k_spynet_assemble(const float* __restrict__ im1, const float* __restrict__ im2,
                                  const float* __restrict__ flow_prev, float* __restrict__ flow_up,
                                  float* __restrict__ x8, int B, int H, int W) {
  const size_t npix = (size_t)B * H * W;
  for (size_t p = grid_stride_start(); p < npix; p += (size_t)gridDim.x * blockDim.x)
    spynet_assemble_px(im1, im2, flow_prev, flow_up, x8, p, p % W, (p / W) % H, p / ((size_t)H * W), H, W);
}

// 32-bit forms of the pixel-walking kernels (B*H*W*2 < 2^32): the pixel -> (b, y, x) split as two
// multiply-high divisions by host-computed magic numbers (udiv_magic) instead of three 64-bit
// divisions per pixel; the per-pixel arithmetic is the 64-bit kernels' (same device functions)
__global__ void k_spynet_assemble_q(const float* __restrict__ im1, const float* __restrict__ im2,
                                    const float* __restrict__ flow_prev, float* __restrict__ flow_up,
                                    float* __restrict__ x8, int B, int H, int W, unsigned mW, unsigned mH) {
  const unsigned npix = (unsigned)B * H * W;
  const unsigned st = gridDim.x * blockDim.x;
  const int h = H / 2, w = W / 2;
  const float4* const f4 = reinterpret_cast<const float4*>(flow_prev);
  const float4* const i2 = reinterpret_cast<const float4*>(im2);
  const float4* const i1 = reinterpret_cast<const float4*>(im1);
  // two pixels per iteration with every load issued ahead of the stores (see k_mc_assemble_q);
  // the flow upsample is up_sample4's arithmetic with unconditional (clamped: i1 == i0 at the
  // edge, same address) loads
  auto up = [&](unsigned b, int y, int x) -> float4 {
    if (!flow_prev) return make_float4(0.f, 0.f, 0.f, 0.f);
    const UpIdx uy = up_index(y, h, H, 0), ux = up_index(x, w, W, 0);
    const unsigned bb = b * (unsigned)h * (unsigned)w;
    const float4 a = f4[bb + (unsigned)uy.i0 * w + ux.i0], bq = f4[bb + (unsigned)uy.i0 * w + ux.i1];
    const float4 c = f4[bb + (unsigned)uy.i1 * w + ux.i0], d = f4[bb + (unsigned)uy.i1 * w + ux.i1];
    float4 o;
    o.x = fvc_lerp2d(a.x, bq.x, c.x, d.x, ux.l0, ux.l1, uy.l0, uy.l1);
    o.y = fvc_lerp2d(a.y, bq.y, c.y, d.y, ux.l0, ux.l1, uy.l0, uy.l1);
    o.x = o.x * 2.f;
    o.y = o.y * 2.f;
    o.z = 0.f;
    o.w = 0.f;
    return o;
  };
  for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += 2 * st) {
    const unsigned p2 = p + st < npix ? p + st : p;
    const unsigned row1 = udiv_magic(p, W, mW), b1 = udiv_magic(row1, H, mH);
    const unsigned row2 = udiv_magic(p2, W, mW), b2 = udiv_magic(row2, H, mH);
    const int y1 = (int)(row1 - b1 * H), x1 = (int)(p - row1 * W);
    const int y2 = (int)(row2 - b2 * H), x2 = (int)(p2 - row2 * W);
    const float4 a1 = i1[p], a2 = i1[p2];
    const float4 fu1 = up(b1, y1, x1), fu2 = up(b2, y2, x2);
    const WarpTap t1 = warp_tap(y1, x1, fu1.x, fu1.y, H, W);
    const WarpTap t2 = warp_tap(y2, x2, fu2.x, fu2.y, H, W);
    const float4 wv1 = warp_sample4_nb(i2, b1 * H * W, W, H, t1);
    const float4 wv2 = warp_sample4_nb(i2, b2 * H * W, W, H, t2);
    float4* const fo = reinterpret_cast<float4*>(flow_up);
    float4* const o = reinterpret_cast<float4*>(x8);
    fo[p] = fu1;
    o[2 * p] = make_float4(a1.x, a1.y, a1.z, wv1.x);
    o[2 * p + 1] = make_float4(wv1.y, wv1.z, fu1.x, fu1.y);
    fo[p2] = fu2;
    o[2 * p2] = make_float4(a2.x, a2.y, a2.z, wv2.x);
    o[2 * p2 + 1] = make_float4(wv2.y, wv2.z, fu2.x, fu2.y);
  }
}

// motion compensation input: warpframe = warp(ref, mv); x8 = [warpframe, ref, 0, 0]
__device__ __forceinline__ void mc_assemble_px(const float* __restrict__ ref, const float* __restrict__ mv,
                                               float* __restrict__ warpframe, float* __restrict__ x8, size_t p,
                                               int x, int y, size_t b, int H, int W) {
  const float4 f = reinterpret_cast<const float4*>(mv)[p];
  const WarpTap t = warp_tap(y, x, f.x, f.y, H, W);
  float4 wv = warp_sample4(ref, b * H * W, W, 1, 0, t);
  wv.w = 0.f;
  reinterpret_cast<float4*>(warpframe)[p] = wv;
  const float4 r = reinterpret_cast<const float4*>(ref)[p];
  float4* o = reinterpret_cast<float4*>(x8) + p * 2;
  o[0] = make_float4(wv.x, wv.y, wv.z, r.x);
  o[1] = make_float4(r.y, r.z, 0.f, 0.f);
}

__global__ void k_mc_assemble(const float* __restrict__ ref, const float* __restrict__ mv,
                              float* __restrict__ warpframe, float* __restrict__ x8, int B, int H, int W) {
  const size_t npix = (size_t)B * H * W;
  for (size_t p = grid_stride_start(); p < npix; p += (size_t)gridDim.x * blockDim.x)
    mc_assemble_px(ref, mv, warpframe, x8, p, p % W, (p / W) % H, p / ((size_t)H * W), H, W);
}

__global__ void k_mc_assemble_q(const float* __restrict__ ref, const float* __restrict__ mv,
                                float* __restrict__ warpframe, float* __restrict__ x8, int B, int H, int W,
                                unsigned mW, unsigned mH) {
  const unsigned npix = (unsigned)B * H * W;
  const unsigned st = gridDim.x * blockDim.x;
  const float4* const r4 = reinterpret_cast<const float4*>(ref);
#if defined(FVC_MC_ACQ)
  // experiment (r6 race probe): an agent-scope acquire (this CU's L1 invalidated) before any load
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
#if defined(FVC_MC_SC1) || defined(FVC_MC_BUF)
  // experiment (r6 race probe): every load of the kernel as a buffer load; FVC_MC_SC1 sets sc1
  // (bypasses the CU's L1, served by the XCD's L2), FVC_MC_BUF is the plain-policy control
#if defined(FVC_MC_SC1)
  constexpr int kAux = 16;
#else
  constexpr int kAux = 0;
#endif
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)ref, (short)0, (int)(npix * 16u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)mv, (short)0, (int)(npix * 16u), 0x00020000);
  auto ld = [&](const __amdgpu_buffer_rsrc_t& r, unsigned px) -> float4 {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, px * 16u, 0, kAux));
  };
  auto sample = [&](unsigned bbase, const WarpTap& t) -> float4 {
    const unsigned r0 = bbase + (unsigned)t.y0 * W + t.x0;
    const unsigned dx = t.vx1 ? 1u : 0u, dy = t.vy1 ? (unsigned)W : 0u;
#if defined(FVC_MC_NEFIRST)
    // the east taps' loads issued before the west taps' (each pair shares its lines)
    const float4 vne = ld(rr, r0 + dx), vse = ld(rr, r0 + dy + dx);
    __builtin_amdgcn_sched_barrier(0);
    const float4 vnw = ld(rr, r0), vsw = ld(rr, r0 + dy);
#else
    const float4 vnw = ld(rr, r0), vne = ld(rr, r0 + dx), vsw = ld(rr, r0 + dy), vse = ld(rr, r0 + dy + dx);
#endif
    float4 o;
    o.x = ((vnw.x * t.nw + vne.x * t.ne) + vsw.x * t.sw) + vse.x * t.se;
    o.y = ((vnw.y * t.nw + vne.y * t.ne) + vsw.y * t.sw) + vse.y * t.se;
    o.z = ((vnw.z * t.nw + vne.z * t.ne) + vsw.z * t.sw) + vse.z * t.se;
    o.w = ((vnw.w * t.nw + vne.w * t.ne) + vsw.w * t.sw) + vse.w * t.se;
    return o;
  };
#endif
  // two pixels per iteration, all loads of both issued before either's stores: the gathers depend
  // on the flow load (two dependent HBM round trips per pixel), so latency, not bytes, bounds a
  // one-pixel loop
  for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += 2 * st) {
    const unsigned p2 = p + st < npix ? p + st : p;
#if defined(FVC_MC_SC1) || defined(FVC_MC_BUF)
    const float4 f1 = ld(rm, p), f2 = ld(rm, p2);
    const float4 r1 = ld(rr, p), r2 = ld(rr, p2);
#else
    const float4 f1 = reinterpret_cast<const float4*>(mv)[p];
    const float4 f2 = reinterpret_cast<const float4*>(mv)[p2];
    const float4 r1 = r4[p], r2 = r4[p2];
#endif
    const unsigned row1 = udiv_magic(p, W, mW), b1 = udiv_magic(row1, H, mH);
    const unsigned row2 = udiv_magic(p2, W, mW), b2 = udiv_magic(row2, H, mH);
    const WarpTap t1 = warp_tap((int)(row1 - b1 * H), (int)(p - row1 * W), f1.x, f1.y, H, W);
    const WarpTap t2 = warp_tap((int)(row2 - b2 * H), (int)(p2 - row2 * W), f2.x, f2.y, H, W);
#if defined(FVC_MC_SC1) || defined(FVC_MC_BUF)
    float4 w1 = sample(b1 * H * W, t1);
    float4 w2 = sample(b2 * H * W, t2);
#else
    float4 w1 = warp_sample4_nb(r4, b1 * H * W, W, H, t1);
    float4 w2 = warp_sample4_nb(r4, b2 * H * W, W, H, t2);
#endif
    w1.w = 0.f;
    w2.w = 0.f;
    float4* const wf = reinterpret_cast<float4*>(warpframe);
    float4* const o = reinterpret_cast<float4*>(x8);
    wf[p] = w1;
    o[2 * p] = make_float4(w1.x, w1.y, w1.z, r1.x);
    o[2 * p + 1] = make_float4(r1.y, r1.z, 0.f, 0.f);
    wf[p2] = w2;
    o[2 * p2] = make_float4(w2.x, w2.y, w2.z, r2.x);
    o[2 * p2 + 1] = make_float4(r2.y, r2.z, 0.f, 0.f);
  }
}

__global__ void k_sub(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ o, size_t n) {
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) o[e] = a[e] - b[e];
}

// ------------------------------------------------------------------ GDN / IGDN (C = 64)
// norm_i = beta_i + sum_j gamma[i][j] x_j^2 ; y = x / sqrt(norm) (or x * sqrt(norm))
// GDN / IGDN on the fp32 matrix cores. norm = conv1x1(x^2, gamma) + beta is a [32 px x 64] x
// [64 x 64] product per 32-pixel group: 2 N-tiles x 32 v_mfma_f32_32x32x2_f32 (an exact fp32 FMA
// chain per output). gamma^T fragments stay in 64 VGPRs for the whole kernel. Lane (p, h) loads
// channels [32h, 32h+32) of pixel p (its A operand for all 32 MFMAs: MFMA s pairs channel s with
// s+32), parks them in a per-wave LDS tile, and reads x back in the accumulator layout (lane =
// channel, register = pixel) for the normalisation, so HBM sees x once and y once.
constexpr int kGdnWaves = 4;
constexpr int kGdnRow = 68;  // LDS row stride in floats (272 B = 16 x odd: conflict-free b128 writes)

__global__ __launch_bounds__(64 * kGdnWaves) void k_gdn_mfma(const float* __restrict__ x, float* __restrict__ y,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ gamma, size_t npix,
                                                          int inverse) {
  __shared__ float xt[kGdnWaves * 32 * kGdnRow];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  float g0[32], g1[32];  // gamma^T[k = s + 32 lh][n = li (+32)] = gamma[n][k]
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    g0[s] = gamma[li * 64 + s + 32 * lh];
    g1[s] = gamma[(32 + li) * 64 + s + 32 * lh];
  }
  const float b0 = beta[li], b1 = beta[32 + li];
  float* xw = xt + wave * 32 * kGdnRow;
  const size_t ngroups = (npix + 31) / 32;
  // the next group's x is loaded while the current group's MFMAs run
  float4 nx[8];
  auto fetch = [&](size_t gi) {
    const size_t p = gi * 32 + li;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      nx[k] = p < npix ? reinterpret_cast<const float4*>(x + p * 64 + 32 * lh)[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const size_t gstep = (size_t)gridDim.x * kGdnWaves;
  size_t gi = (size_t)blockIdx.x * kGdnWaves + wave;
  if (gi < ngroups) fetch(gi);
  for (; gi < ngroups; gi += gstep) {
    const size_t p0 = gi * 32;
    float a[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float4 v = nx[k];
      a[4 * k] = v.x; a[4 * k + 1] = v.y; a[4 * k + 2] = v.z; a[4 * k + 3] = v.w;
      *reinterpret_cast<float4*>(xw + li * kGdnRow + 32 * lh + 4 * k) = v;
    }
    if (gi + gstep < ngroups) fetch(gi + gstep);
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[r] = 0.f;
      acc1[r] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      const float sq = a[s] * a[s];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(sq, g0[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(sq, g1[s], acc1, 0, 0, 0);
    }
    // accumulator layout: lane (li, lh), register r -> pixel q = (r&3) + 8(r>>2) + 4lh, channel li (+32)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (p0 + q < npix) {
        const float x0 = xw[q * kGdnRow + li], x1 = xw[q * kGdnRow + 32 + li];
        const float n0 = sqrtf(acc0[r] + b0), n1 = sqrtf(acc1[r] + b1);
        float* yo = y + (p0 + q) * 64;
        yo[li] = inverse ? x0 * n0 : x0 / n0;
        yo[32 + li] = inverse ? x1 * n1 : x1 / n1;
      }
    }
  }
}

// GDN / IGDN followed by the next layer's 1x1 tap-partial GEMM (resDecoder igdn3 -> deconv4,
// synthesis.py:26,57: 64 -> 3, 5x5 s2, 75 partials): per 32-pixel group the normalised y goes back
// into the wave's LDS tile (pixel-major), each lane then reads its pixel's channels as split-
// precision B fragments (channel order of fvc_x3_tap_pack_weight) and NPT P tiles of 32 partials
// come out of three fp16 MFMAs per k16 block, P = main * 2^-kt + corr * 2^-kt-11. y itself never
// reaches HBM; fvc_tap_gather_nhwc sums the partials into the deconv's output.
typedef _Float16 gh8 __attribute__((ext_vector_type(8)));
template <int NPT>
__global__ __launch_bounds__(64 * kGdnWaves) void k_gdn_tap_mfma(const float* __restrict__ x, float* __restrict__ P,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ gamma,
                                                             const uint4* __restrict__ tw, float4 tosc,
                                                             size_t npix, int inverse, int pcp, int* ovf) {
  __shared__ float xt[kGdnWaves * 32 * kGdnRow];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  float g0[32], g1[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    g0[s] = gamma[li * 64 + s + 32 * lh];
    g1[s] = gamma[(32 + li) * 64 + s + 32 * lh];
  }
  const float b0 = beta[li], b1 = beta[32 + li];
  const float ts[4] = {tosc.x, tosc.y, tosc.z, tosc.w};
  float* xw = xt + wave * 32 * kGdnRow;
  const size_t ngroups = (npix + 31) / 32;
  float4 nx[8];
  auto fetch = [&](size_t gi) {
    const size_t p = gi * 32 + li;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      nx[k] = p < npix ? reinterpret_cast<const float4*>(x + p * 64 + 32 * lh)[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const size_t gstep = (size_t)gridDim.x * kGdnWaves;
  size_t gi = (size_t)blockIdx.x * kGdnWaves + wave;
  float mx = 0.f;
  if (gi < ngroups) fetch(gi);
  for (; gi < ngroups; gi += gstep) {
    const size_t p0 = gi * 32;
    float a[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float4 v = nx[k];
      a[4 * k] = v.x; a[4 * k + 1] = v.y; a[4 * k + 2] = v.z; a[4 * k + 3] = v.w;
      *reinterpret_cast<float4*>(xw + li * kGdnRow + 32 * lh + 4 * k) = v;
    }
    if (gi + gstep < ngroups) fetch(gi + gstep);
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[r] = 0.f;
      acc1[r] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      const float sq = a[s] * a[s];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(sq, g0[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(sq, g1[s], acc1, 0, 0, 0);
    }
    // y (the same expression as k_gdn_mfma) back into the tile; pixels past npix hold 0
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int q = (r & 3) + 8 * (r >> 2) + 4 * lh;
      const bool ok = p0 + q < npix;
      const float x0 = xw[q * kGdnRow + li], x1 = xw[q * kGdnRow + 32 + li];
      const float n0 = sqrtf(acc0[r] + b0), n1 = sqrtf(acc1[r] + b1);
      const float y0 = inverse ? x0 * n0 : x0 / n0, y1 = inverse ? x1 * n1 : x1 / n1;
      xw[q * kGdnRow + li] = ok ? y0 : 0.f;
      xw[q * kGdnRow + 32 + li] = ok ? y1 : 0.f;
    }
    // lane (li, lh): pixel li's channels 16 kb + 4 lh + {0-3, 8-11} as hi / lo*2^11 halves
    gh8 yh[4], yl[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const float* row = xw + li * kGdnRow + 16 * kb + 4 * lh;
      const float4 u = *reinterpret_cast<const float4*>(row), v = *reinterpret_cast<const float4*>(row + 8);
      const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const _Float16 h = (_Float16)f[t];
        yh[kb][t] = h;
        yl[kb][t] = (_Float16)((f[t] - (float)h) * 2048.f);
        mx = fmaxf(mx, fabsf(f[t]));
      }
    }
    const bool px_ok = p0 + li < npix;
#pragma unroll
    for (int pt = 0; pt < NPT; ++pt) {
      f32x16 pa, pc;
#pragma unroll
      for (int r = 0; r < 16; ++r) pa[r] = pc[r] = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const uint4* f = tw + (size_t)((pt * 4 + kb) * 2) * 64 + lane;
        const gh8 wh = __builtin_bit_cast(gh8, f[0]), wl = __builtin_bit_cast(gh8, f[64]);
        pa = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yh[kb], pa, 0, 0, 0);
        pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, yh[kb], pc, 0, 0, 0);
        pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yl[kb], pc, 0, 0, 0);
      }
      const float sc = ts[pt], scc = ts[pt] * (1.0f / 2048.f);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int pp = pt * 32 + 8 * g + 4 * lh;
        if (px_ok && pp < pcp) {
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = fmaf(pc[4 * g + i], scc, pa[4 * g + i] * sc);
          *reinterpret_cast<float4*>(P + (p0 + li) * pcp + pp) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  }
  if (!(mx < 65000.f) && ovf) atomicOr(ovf, 1);
}

// GDN / IGDN with the norm on the split-precision fp16 matrix cores (the conv kernels' scheme):
// norm = beta + gamma . x^2 is a [64 out ch] x [64 in ch] x [32 px] GEMM per 32-pixel group with
// gamma as the row operand (one launch-wide scale 2^kw: max |gamma| * 2^kw in [2^13, 2^14)) and
// x^2 * 2^-8 as the column operand, both split exactly into fp16 hi + lo * 2^-11:
// 2 N-tiles x 4 k-blocks x 3 v_mfma_f32_32x32x16_f16 (24 MFMAs of 8 passes) instead of 64
// v_mfma_f32_32x32x2_f32 of 16 passes -- the fp32 form's matrix time is as long as its HBM time.
// Lane (li, lh) owns pixel li and channels 32t + 8g + 4lh + {0..3} (t = 0..1, g = 0..3) from load
// to store: k-block kb = 2t + gp orders its channels {16gp + 4lh + 0-3 | 16gp + 8 + 4lh + 0-3}
// (+32t), so a lane's column operand is its own x / accumulator registers 8gp .. 8gp + 7 and no
// LDS tile is needed (the same order as fvc_x3_tap_pack_weight: in the tap form (NPT > 0) the
// normalised y already is the B fragment of the tap GEMM). The omitted lo * lo term and the lo
// roundings are ~2^-22 relative per product; every term of the norm is >= 0, so the norm carries
// that relative error (fp32 chain: ~2^-24 per add). The column operand carries a power-of-two
// scale per pixel, x^2 * 2^e with the pixel's max x^2 * 2^e in [2^14, 2^15) (e clamped to
// [-60, 60]), undone per lane in the epilogue (the accumulator column of a lane is its own pixel):
// small activations stay in the fp16 normal range, so the ~2^-22 relative bound holds for every
// pixel whose max |x| is above ~1e-11, whatever beta is. A group with an inf or NaN x^2 runs the
// fp32 MFMA chain instead (wave-uniform branch, gamma read from L2).
template <int NPT, bool INV>
__global__ __launch_bounds__(256, 2) void k_gdn_x3(const float* __restrict__ x, float* __restrict__ out,
                                                   const float* __restrict__ beta, const float* __restrict__ gamma,
                                                   const uint4* __restrict__ tw, float4 tosc, size_t npix,
                                                   int pcp, int* ovf) {
  __shared__ float4 sbeta[16];
  __shared__ uint4 sg[2 * 4 * 2 * 64];  // row-operand fragments [n][kb][hi, lo][lane]
  __shared__ uint4 stw[NPT > 0 ? NPT * 512 : 1];  // the tap pack (fvc_x3_tap_pack_weight layout)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  if (threadIdx.x < 64) reinterpret_cast<float*>(sbeta)[threadIdx.x] = beta[threadIdx.x];
  if constexpr (NPT > 0)
    for (int i = threadIdx.x; i < NPT * 512; i += 256) stw[i] = tw[i];
  // row operand: lane (li, lh) -> out channel 32n + li, k-block kb's 8 channels of half lh; every
  // wave reads all 4096 entries (the same scale in every wave of the launch), wave 0 stores them
  float gv[2][4][8];
  float gmax = 0.f;
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = 32 * (kb >> 1) + 16 * (kb & 1) + 4 * lh + (e < 4 ? e : 4 + e);
        gv[n][kb][e] = gamma[(32 * n + li) * 64 + ch];
        gmax = fmaxf(gmax, fabsf(gv[n][kb][e]));
      }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) gmax = fmaxf(gmax, __shfl_xor(gmax, o, 64));
  int ge = 0;
  (void)frexpf(gmax, &ge);
  const int kw = gmax > 0.f ? max(-60, min(60, 14 - ge)) : 0;
  if (wave == 0) {
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        gh8 h8, l8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float s = ldexpf(gv[n][kb][e], kw);
          const _Float16 h = (_Float16)s;
          h8[e] = h;
          l8[e] = (_Float16)((s - (float)h) * 2048.f);
        }
        sg[((n * 4 + kb) * 2) * 64 + lane] = __builtin_bit_cast(uint4, h8);
        sg[((n * 4 + kb) * 2 + 1) * 64 + lane] = __builtin_bit_cast(uint4, l8);
      }
  }
  const float ts[4] = {tosc.x, tosc.y, tosc.z, tosc.w};
  __syncthreads();
  const size_t ngroups = (npix + 31) / 32;
  float4 nx[8];  // nx[2 kb + h]: channels 32t + 16gp + 8h + 4lh + 0..3
  auto fetch = [&](size_t gi) {
    const size_t p = gi * 32 + li;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      nx[k] = p < npix ? *reinterpret_cast<const float4*>(x + p * 64 + 16 * (k >> 1) + 8 * (k & 1) + 4 * lh)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const size_t gstep = (size_t)gridDim.x * 4;
  size_t gi = (size_t)blockIdx.x * 4 + wave;
  float mx = 0.f;
  if (gi < ngroups) fetch(gi);
  for (; gi < ngroups; gi += gstep) {
    // keeps the loop-invariant fragment reads from LDS inside the loop (hoisted, they would take
    // 64 registers and spill)
    asm volatile("" ::: "memory");
    const size_t p = gi * 32 + li;
    // xr[t][r]: channel 32t + 8(r / 4) + 4lh + r % 4 (the accumulator layout)
    float xr[2][16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int t = k >> 2, r0 = 4 * (k & 3);
      xr[t][r0] = nx[k].x; xr[t][r0 + 1] = nx[k].y; xr[t][r0 + 2] = nx[k].z; xr[t][r0 + 3] = nx[k].w;
    }
    if (gi + gstep < ngroups) fetch(gi + gstep);
    // this pixel's scale: max |x| over its 64 channels (this lane's 32 and lane li + 32's)
    float ax = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) ax = fmaxf(ax, fabsf(xr[t][r]));
    ax = fmaxf(ax, __shfl_xor(ax, 32, 64));
    int pe = 0;
    (void)frexpf(ax * ax, &pe);
    const int es = ax > 0.f ? max(-60, min(60, 15 - pe)) : 0;  // max x^2 2^es in [2^14, 2^15)
    const float xsc = ldexpf(1.f, es);
    const float sc = ldexpf(1.f, -es - kw), scc = ldexpf(1.f, -es - kw - 11);
    gh8 sh[4], sl[4];
    bool big = false;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = xr[kb >> 1][8 * (kb & 1) + e];
        const float s = (v * v) * xsc;
        big |= !(s < 65000.f);
        const _Float16 h = (_Float16)s;
        sh[kb][e] = h;
        sl[kb][e] = (_Float16)((s - (float)h) * 2048.f);
      }
    // per N-tile: norm (x3 MFMAs, or the fp32 chain for a group out of fp16 range), then
    // y = x / sqrt(norm) (GDN) or x * sqrt(norm) (IGDN), norm = sum + beta, written over x (tile 0's
    // y is parked until tile 1's fp32 chain has read x)
    const bool slow = __any(big);
    float y0[16];
    const float s1 = slow ? 1.f : sc, s2 = slow ? 0.f : scc;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f32x16 a, c;
#pragma unroll
      for (int r = 0; r < 16; ++r) a[r] = c[r] = 0.f;
      if (!slow) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const gh8 wh = __builtin_bit_cast(gh8, sg[((n * 4 + kb) * 2) * 64 + lane]);
          const gh8 wl = __builtin_bit_cast(gh8, sg[((n * 4 + kb) * 2 + 1) * 64 + lane]);
          a = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, sh[kb], a, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, sh[kb], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, sl[kb], c, 0, 0, 0);
        }
      } else {
        // v_mfma_f32_32x32x2_f32, k = (register s of the lane, half lh)
#pragma unroll
        for (int s = 0; s < 32; ++s) {
          const int t = s >> 4, r = s & 15;
          const int ch = 32 * t + 8 * (r >> 2) + 4 * lh + (r & 3);
          const float v = xr[t][r];
          a = __builtin_amdgcn_mfma_f32_32x32x2f32(gamma[(32 * n + li) * 64 + ch], v * v, a, 0, 0, 0);
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = sbeta[8 * n + 2 * g + lh];
        const float bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float nv = sqrtf(fmaf(c[4 * g + i], s2, a[4 * g + i] * s1) + bb[i]);
          const float xv = xr[n][4 * g + i];
          const float yv = INV ? xv * nv : xv / nv;
          if (n == 0) y0[4 * g + i] = yv;
          else xr[1][4 * g + i] = yv;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) xr[0][r] = y0[r];
    float (&yr)[2][16] = xr;
    if constexpr (NPT == 0) {
      if (p < npix) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(out + p * 64 + 32 * t + 8 * g + 4 * lh) =
                make_float4(yr[t][4 * g], yr[t][4 * g + 1], yr[t][4 * g + 2], yr[t][4 * g + 3]);
      }
    } else {
      // the tap GEMM: y registers 8gp .. 8gp + 7 of tile t are the k16 block kb = 2t + gp
      const bool px_ok = p < npix;
      gh8 yh[4], yl[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = px_ok ? yr[kb >> 1][8 * (kb & 1) + e] : 0.f;
          const _Float16 h = (_Float16)f;
          yh[kb][e] = h;
          yl[kb][e] = (_Float16)((f - (float)h) * 2048.f);
          mx = fmaxf(mx, fabsf(f));
        }
#pragma unroll
      for (int pt = 0; pt < NPT; ++pt) {
        f32x16 pa, pc;
#pragma unroll
        for (int r = 0; r < 16; ++r) pa[r] = pc[r] = 0.f;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const uint4* f = stw + ((pt * 4 + kb) * 2) * 64 + lane;
          const gh8 wh = __builtin_bit_cast(gh8, f[0]), wl = __builtin_bit_cast(gh8, f[64]);
          pa = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yh[kb], pa, 0, 0, 0);
          pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, yh[kb], pc, 0, 0, 0);
          pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yl[kb], pc, 0, 0, 0);
        }
        const float s1 = ts[pt], s2 = ts[pt] * (1.0f / 2048.f);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int pp = pt * 32 + 8 * g + 4 * lh;
          if (px_ok && pp < pcp) {
            float o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = fmaf(pc[4 * g + i], s2, pa[4 * g + i] * s1);
            *reinterpret_cast<float4*>(out + p * pcp + pp) = make_float4(o[0], o[1], o[2], o[3]);
          }
        }
      }
    }
  }
  if (NPT > 0 && !(mx < 65000.f) && ovf) atomicOr(ovf, 1);
}

// ------------------------------------------------------------------ deterministic reductions
template <int K>
__device__ void block_reduce_store(double (&v)[K], double* out) {
  __shared__ double red[kBlk / 64][K];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = v[k];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0) red[wid][k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      double s = 0.0;
      for (int w = 0; w < kBlk / 64; ++w) s += red[w][k];
      out[blockIdx.x * K + k] = s;
    }
  }
}

template <int K>
__global__ void k_reduce_partials(const double* __restrict__ ws, int nblocks, double* __restrict__ out) {
  __shared__ double red[kBlk][K];
  double s[K];
#pragma unroll
  for (int k = 0; k < K; ++k) s[k] = 0.0;
  for (int i = threadIdx.x; i < nblocks; i += blockDim.x)
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] += ws[i * K + k];
#pragma unroll
  for (int k = 0; k < K; ++k) red[threadIdx.x][k] = s[k];
  __syncthreads();
  for (int st = kBlk / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st)
#pragma unroll
      for (int k = 0; k < K; ++k) red[threadIdx.x][k] += red[threadIdx.x + st][k];
    __syncthreads();
  }
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] = red[0][k];
}

__global__ __launch_bounds__(kBlk) void k_recon_finalize(const float* __restrict__ recon, const float* __restrict__ in,
                                                         const float* __restrict__ wf, const float* __restrict__ pred,
                                                         float* __restrict__ clipped, double* __restrict__ ws,
                                                         int B, int H, int W) {
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const size_t npix = (size_t)B * H * W;
  const size_t hw = (size_t)H * W;
  for (size_t p = grid_stride_start(); p < npix; p += (size_t)gridDim.x * blockDim.x) {
    const float4 r = reinterpret_cast<const float4*>(recon)[p];
    const float4 x = reinterpret_cast<const float4*>(in)[p];
    const float4 wv = reinterpret_cast<const float4*>(wf)[p];
    const float4 pv = reinterpret_cast<const float4*>(pred)[p];
    const float rr[3] = {r.x, r.y, r.z}, xx[3] = {x.x, x.y, x.z};
    const float ww[3] = {wv.x, wv.y, wv.z}, pp[3] = {pv.x, pv.y, pv.z};
    const size_t b = p / hw, q = p - b * hw;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float d0 = rr[c] - xx[c], d1 = ww[c] - xx[c], d2 = pp[c] - xx[c];
      acc[0] += (double)(d0 * d0);
      acc[1] += (double)(d1 * d1);
      acc[2] += (double)(d2 * d2);
      const float cv = fminf(fmaxf(rr[c], 0.f), 1.f);
      const float d3 = cv - xx[c];
      acc[3] += (double)(d3 * d3);
      clipped[(b * 3 + c) * hw + q] = cv;
    }
  }
  block_reduce_store<4>(acc, ws);
}

// Laplace bits (net.py:121-151): p = cdf(f+.5) - cdf(f-.5), cdf(v) = .5 - .5 sign(v) expm1(-|v|/s)
__device__ __forceinline__ float laplace_cdf(float v, float s) { return fvc_laplace_cdf(v, s); }

__device__ __forceinline__ float bits_of_prob(float p) {
  float b = -1.0f * logf(p + 1e-5f) / 0.6931471805599453f;
  return fminf(fmaxf(b, 0.f), 50.f);
}

__global__ __launch_bounds__(kBlk) void k_bits_laplace(const float* __restrict__ feat, const float* __restrict__ sigma,
                                                       double* __restrict__ ws, size_t npix, int C, int cp) {
  double acc[1] = {0.0};
  const size_t n = npix * C;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e / C;
    const int c = e - p * C;
    const float f = rintf(feat[p * cp + c]);
    const float s = fminf(fmaxf(sigma[p * cp + c], 1e-5f), 1e10f);
    const float prob = laplace_cdf(f + 0.5f, s) - laplace_cdf(f - 0.5f, s);
    acc[0] += (double)bits_of_prob(prob);
  }
  block_reduce_store<1>(acc, ws);
}

__device__ __forceinline__ float bitest_cdf(float x, const float* prm, int C, int c) {
  return fvc_bitest_cdf(x, prm, C, c);
}

__global__ __launch_bounds__(kBlk) void k_bits_factorized(const float* __restrict__ v, const float* __restrict__ prm,
                                                          double* __restrict__ ws, size_t npix, int C, int cp) {
  double acc[1] = {0.0};
  const size_t n = npix * C;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e / C;
    const int c = e - p * C;
    const float q = rintf(v[p * cp + c]);
    const float prob = bitest_cdf(q + 0.5f, prm, C, c) - bitest_cdf(q - 0.5f, prm, C, c);
    acc[0] += (double)bits_of_prob(prob);
  }
  block_reduce_store<1>(acc, ws);
}


// ------------------------------------------------------------------ RLVC path
// compressai.layers.GDN (models.py:23,529-538): norm = conv1x1(x^2, gamma) + beta,
// y = x * rsqrt(norm) (GDN) or x * sqrt(norm) (IGDN), any C (RLVC: 128). A block of C threads
// walks pixels in groups of kGcPix: the group's x rows go to LDS, thread i keeps row i of gamma
// in registers and sums gamma[i][j] x_j^2 over the LDS rows (broadcast reads).
constexpr int kGcPix = 8;

template <int C>
__global__ __launch_bounds__(C) void k_gdn_cai(const float* __restrict__ x, float* __restrict__ y,
                                               const float* __restrict__ beta, const float* __restrict__ gamma,
                                               size_t npix, int inverse) {
  __shared__ float xs[kGcPix][C];
  const int i = threadIdx.x;
  float g[C];
#pragma unroll
  for (int j = 0; j < C; ++j) g[j] = gamma[(size_t)i * C + j];
  const float b = beta[i];
  for (size_t p0 = (size_t)blockIdx.x * kGcPix; p0 < npix; p0 += (size_t)gridDim.x * kGcPix) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kGcPix; ++q) xs[q][i] = p0 + q < npix ? x[(p0 + q) * C + i] : 0.f;
    __syncthreads();
    float acc[kGcPix];
#pragma unroll
    for (int q = 0; q < kGcPix; ++q) acc[q] = 0.f;
#pragma unroll 8
    for (int j = 0; j < C; ++j) {
#pragma unroll
      for (int q = 0; q < kGcPix; ++q) {
        const float v = xs[q][j];
        acc[q] = fmaf(g[j], v * v, acc[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < kGcPix; ++q) {
      if (p0 + q >= npix) break;
      const float norm = acc[q] + b;
      const float xv = xs[q][i];
      y[(p0 + q) * C + i] = inverse ? xv * sqrtf(norm) : xv * (1.f / sqrtf(norm));
    }
  }
}

// ConvLSTM gates (entropy_models.py:367-378): f = sigmoid(f + forget_bias), i = sigmoid(i),
// c = c * f + i * relu(j), o = sigmoid(o), h = o * relu(c); NHWC tensors of C channels
__device__ __forceinline__ float sigmoid_t(float v) { return 1.f / (1.f + expf(-v)); }

__global__ void k_lstm_gates(const float* __restrict__ gj, const float* __restrict__ gi, const float* __restrict__ gf,
                             const float* __restrict__ go, const float* __restrict__ c_prev, float* __restrict__ c_out,
                             float* __restrict__ h_out, size_t n, float forget_bias) {
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const float f = sigmoid_t(gf[e] + forget_bias);
    const float ig = sigmoid_t(gi[e]);
    const float c = c_prev[e] * f + ig * fmaxf(gj[e], 0.f);
    const float o = sigmoid_t(go[e]);
    c_out[e] = c;
    h_out[e] = o * fmaxf(c, 0.f);
  }
}

// RecProbModel sigma (entropy_models.py:61-62): exp(max(sigma, -7)) / 10
__global__ void k_rpm_scale(const float* __restrict__ in, float* __restrict__ out, size_t n) {
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x)
    out[e] = expf(fmaxf(in[e], -7.f)) / 10.f;
}

__device__ __forceinline__ float bits_lb(float l) {  // likelihood_lower_bound(1e-9), then the bits clamp
  return bits_of_prob(fmaxf(l, 1e-9f));
}

// compressai EntropyBottleneck, filters (3,3,3,3) (compressai EB._logits_cumulative): per
// channel prm[c][kEbPrm] = softplus(matrix0..4) (3, 9, 9, 9, 3), bias0..4 (3, 3, 3, 3, 1),
// tanh(factor0..3) (3 x 4)
constexpr int kEbPrm = 58;
__device__ float eb_logits(float v, const float* __restrict__ p) {
  const float* m0 = p;
  const float* m1 = p + 3;
  const float* m2 = p + 12;
  const float* m3 = p + 21;
  const float* m4 = p + 30;
  const float* bs = p + 33;  // b0[3] b1[3] b2[3] b3[3] b4[1]
  const float* fs = p + 46;  // f0[3] f1[3] f2[3] f3[3]
  float a[3], t[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    a[r] = m0[r] * v + bs[r];
    a[r] += fs[r] * tanhf(a[r]);
  }
  const float* ms[3] = {m1, m2, m3};
#pragma unroll
  for (int l = 0; l < 3; ++l) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float acc = ms[l][3 * r] * a[0];
      acc = fmaf(ms[l][3 * r + 1], a[1], acc);
      acc = fmaf(ms[l][3 * r + 2], a[2], acc);
      t[r] = acc + bs[3 * (l + 1) + r];
      t[r] += fs[3 * (l + 1) + r] * tanhf(t[r]);
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) a[r] = t[r];
  }
  float o = m4[0] * a[0];
  o = fmaf(m4[1], a[1], o);
  o = fmaf(m4[2], a[2], o);
  return o + bs[12];
}

// x_hat = round(x - median) + median; likelihood = |sigmoid(s*upper) - sigmoid(s*lower)|,
// s = -sign(lower + upper) (compressai EB._likelihood); out: x_hat and the bits sum
__global__ __launch_bounds__(kBlk) void k_eb_forward(const float* __restrict__ x, const float* __restrict__ prm,
                                                     const float* __restrict__ med, float* __restrict__ xhat,
                                                     double* __restrict__ ws, size_t npix, int C, int cp) {
  double acc[1] = {0.0};
  const size_t n = npix * C;
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e / C;
    const int c = (int)(e - p * C);
    const float m = med[c];
    const float v = rintf(x[p * cp + c] - m) + m;
    xhat[p * cp + c] = v;
    const float lo = eb_logits(v - 0.5f, prm + (size_t)c * kEbPrm);
    const float up = eb_logits(v + 0.5f, prm + (size_t)c * kEbPrm);
    const float sum = lo + up;
    const float sg = sum > 0.f ? -1.f : (sum < 0.f ? 1.f : 0.f);
    acc[0] += (double)bits_lb(fabsf(sigmoid_t(sg * up) - sigmoid_t(sg * lo)));
  }
  block_reduce_store<1>(acc, ws);
}

// GaussianConditional with means (compressai GC._likelihood): x_hat = round(x - mu) + mu,
// v = |x_hat - mu|, s = max(scale, 0.11), l = Phi((.5 - v)/s) - Phi((-.5 - v)/s),
// Phi(t) = .5 erfc(-t / sqrt 2)
__global__ __launch_bounds__(kBlk) void k_gc_forward(const float* __restrict__ x, const float* __restrict__ scale,
                                                     const float* __restrict__ mu, float* __restrict__ xhat,
                                                     double* __restrict__ ws, size_t npix, int C, int cp) {
  double acc[1] = {0.0};
  const size_t n = npix * C;
  const float k = -0.70710678118654752f;  // -(2^-0.5)
  for (size_t e = grid_stride_start(); e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e / C;
    const int c = (int)(e - p * C);
    const size_t o = p * cp + c;
    const float m = mu[o];
    const float xh = rintf(x[o] - m) + m;
    xhat[o] = xh;
    const float v = fabsf(xh - m);
    const float s = fmaxf(scale[o], 0.11f);
    const float up = 0.5f * erfcf(k * ((0.5f - v) / s));
    const float lo = 0.5f * erfcf(k * ((-0.5f - v) / s));
    acc[0] += (double)bits_lb(up - lo);
  }
  block_reduce_store<1>(acc, ws);
}

static int env_flag(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && v[0]) ? atoi(v) : dflt;
}

static int grid_for(size_t n) {
  size_t g = (n + kBlk - 1) / kBlk;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int fvc_version(void) { return 1; }

int fvc_device_arch_ok(void) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 0;
  return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

int fvc_nchw_to_nhwc(const float* src, float* dst, int batch, int c, int h, int w, int cp, fvc_stream_t s) {
  if (!src || !dst || c > cp || cp % 4) return FVC_EINVAL;
  const size_t n = (size_t)batch * h * w;
  const unsigned long long hw = (unsigned long long)h * w;
  if (cp == 4 && hw >= 2 && 2ull * n < (1ull << 32)) {
    const unsigned m = (unsigned)(((1ull << 32) + hw - 1) / hw);
    hipLaunchKernelGGL(k_nchw_to_nhwc4, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, src, dst, batch, c,
                       (unsigned)hw, m);
  } else {
    hipLaunchKernelGGL(k_nchw_to_nhwc, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, src, dst, batch, c, h, w,
                       cp);
  }
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_nhwc_to_nchw(const float* src, float* dst, int batch, int c, int h, int w, int cp, int clamp01,
                     fvc_stream_t s) {
  if (!src || !dst || c > cp) return FVC_EINVAL;
  const size_t n = (size_t)batch * c * h * w;
  hipLaunchKernelGGL(k_nhwc_to_nchw, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, src, dst, batch, c, h, w, cp,
                     clamp01);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_avgpool2_nhwc(const float* src, float* dst, int batch, int h, int w, int cp, fvc_stream_t s) {
  if (!src || !dst || (h & 1) || (w & 1) || cp % 4) return FVC_EINVAL;
  const size_t n = (size_t)batch * (h / 2) * (w / 2) * (cp / 4);
  hipLaunchKernelGGL(k_avgpool2, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, src, dst, batch, h, w, cp);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_warp_nhwc(const float* im, const float* flow, float* out, int batch, int h, int w, int cp, fvc_stream_t s) {
  if (!im || !flow || !out || cp % 4 || h < 2 || w < 2) return FVC_EINVAL;
  const size_t n = (size_t)batch * h * w;
  hipLaunchKernelGGL(k_warp, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, im, flow, out, batch, h, w, cp);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_upsample2x_add_nhwc(const float* src, const float* skip, float* out, int batch, int h, int w, int cp,
                            int align_corners, float scale, fvc_stream_t s) {
  if (!src || !out || cp % 4) return FVC_EINVAL;
  const size_t n = (size_t)batch * 4 * h * w * (cp / 4);
  const unsigned long long H2 = 2ull * h, W2 = 2ull * w;
  // align_corners scales (in - 1) / (out - 1), one host float division each (as ATen's CPU kernel)
  const float usy = H2 > 1 ? (float)(h - 1) / (float)(H2 - 1) : 0.f;
  const float usx = W2 > 1 ? (float)(w - 1) / (float)(W2 - 1) : 0.f;
  if (cp == 64 && (unsigned long long)batch * H2 * W2 * 16ull < (1ull << 32) && env_flag("FVC_UP2_Q16", 1)) {
    const unsigned mW = (unsigned)(((1ull << 32) + W2 - 1) / W2), mH = (unsigned)(((1ull << 32) + H2 - 1) / H2);
    // (index arithmetic e + 2 * stride stays below 2^32: stride <= 8192 * kBlk)
    // two elements per thread, the skip tensor (read once: c0 / c1 are dead after this add) by
    // non-temporal loads: 1088x1920x64 at 8 frames 2.16 -> 1.99 ms (profiles/r5/up2_pair); same bits
    const bool nt = env_flag("FVC_UP2_NT", 1) != 0;
    if (n + (1ull << 24) < (1ull << 32) && env_flag("FVC_UP2_PAIR", 1) && nt)
      hipLaunchKernelGGL((k_up2_add_q16p<2, true>), dim3(grid_for((n + 1) / 2)), dim3(kBlk), 0, (hipStream_t)s, src, skip,
                         out, batch, h, w, align_corners, scale, mW, mH, usy, usx);
    else if (n + (1ull << 24) < (1ull << 32) && env_flag("FVC_UP2_PAIR", 1))
      hipLaunchKernelGGL((k_up2_add_q16p<2, false>), dim3(grid_for((n + 1) / 2)), dim3(kBlk), 0, (hipStream_t)s, src, skip,
                         out, batch, h, w, align_corners, scale, mW, mH, usy, usx);
    else
      hipLaunchKernelGGL(k_up2_add_q16, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, src, skip, out, batch, h, w,
                         align_corners, scale, mW, mH, usy, usx);
  } else {
    hipLaunchKernelGGL(k_up2_add, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, src, skip, out, batch, h, w, cp,
                       align_corners, scale, usy, usx);
  }
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_spynet_assemble(const float* im1, const float* im2, const float* flow_prev, float* flow_up, float* x8,
                        int batch, int h, int w, fvc_stream_t s) {
  if (!im1 || !im2 || !flow_up || !x8 || (h & 1) || (w & 1) || h < 2 || w < 2) return FVC_EINVAL;
  const size_t n = (size_t)batch * h * w;
  if (2ull * n < (1ull << 32) && env_flag("FVC_ASSEMBLE_Q", 1)) {
    // two pixels per thread per iteration: half as many threads as pixels
    const unsigned mW = (unsigned)(((1ull << 32) + w - 1) / w), mH = (unsigned)(((1ull << 32) + h - 1) / h);
    hipLaunchKernelGGL(k_spynet_assemble_q, dim3(grid_for((n + 1) / 2)), dim3(kBlk), 0, (hipStream_t)s, im1, im2, flow_prev,
                       flow_up, x8, batch, h, w, mW, mH);
  } else {
    hipLaunchKernelGGL(k_spynet_assemble, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, im1, im2, flow_prev,
                       flow_up, x8, batch, h, w);
  }
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_mc_assemble(const float* ref, const float* mv, float* warpframe, float* x8, int batch, int h, int w,
                    fvc_stream_t s) {
  if (!ref || !mv || !warpframe || !x8 || h < 2 || w < 2) return FVC_EINVAL;
  const size_t n = (size_t)batch * h * w;
  if (2ull * n < (1ull << 32) && env_flag("FVC_ASSEMBLE_Q", 1)) {
    const unsigned mW = (unsigned)(((1ull << 32) + w - 1) / w), mH = (unsigned)(((1ull << 32) + h - 1) / h);
    hipLaunchKernelGGL(k_mc_assemble_q, dim3(grid_for((n + 1) / 2)), dim3(kBlk), 0, (hipStream_t)s, ref, mv, warpframe, x8,
                       batch, h, w, mW, mH);
  } else {
    hipLaunchKernelGGL(k_mc_assemble, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, ref, mv, warpframe, x8,
                       batch, h, w);
  }
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_tap_gather_nhwc(const float* P, int pcp, const float* bias, const float* res, float* y, int batch,
                        int h, int w, int cout, int ksize, int stride, int transposed, int act, int post_op,
                        fvc_stream_t s) {
  if (!P || !bias || !y || batch <= 0 || h <= 0 || w <= 0 || cout < 1 || cout > 4 ||
      (ksize != 3 && ksize != 5) || pcp < ksize * ksize * cout || pcp % 4)
    return FVC_EINVAL;
  if (transposed ? stride != 2 : stride != 1) return FVC_EINVAL;
  const int Ho = transposed ? h * stride : h, Wo = transposed ? w * stride : w;
  const float slope = act == FVC_ACT_RELU ? 0.f : (act == FVC_ACT_LRELU ? 0.1f : 1.f);
  const size_t n = (size_t)batch * Ho * Wo;
  const dim3 g(grid_for(n)), bl(kBlk);
  hipStream_t st = (hipStream_t)s;
  if (!transposed && ksize == 3 && pcp <= 32) {
    // 8-row tiles: 39 KB of LDS at pcp 28, four blocks per CU (FVC_GATHER_TH=16: 18-row halo tiles)
    const char* th_env = getenv("FVC_GATHER_TH");
    const int th = (th_env && atoi(th_env) == 16) ? 16 : 8;
    const dim3 gt(fvc_cdiv(w, 32), fvc_cdiv(h, th), batch);
    const size_t lds = (size_t)(th + 2) * 34 * (pcp + 1) * 4;
#define FVC_TGL(CO, TH)                                                                                         \
    if (cout == CO && th == TH) {                                                                             \
      if (lds > 64 * 1024)                                                                                    \
        (void)hipFuncSetAttribute((const void*)k_tap_gather3_lds<CO, TH>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)lds);                                                                  \
      hipLaunchKernelGGL((k_tap_gather3_lds<CO, TH>), gt, dim3(256), lds, st, P, pcp, bias, res, y, h, w, slope, post_op); \
      FVC_CHECK_LAUNCH();                                                                                     \
      return 0;                                                                                               \
    }
    FVC_TGL(1, 8) FVC_TGL(2, 8) FVC_TGL(3, 8) FVC_TGL(4, 8)
    FVC_TGL(1, 16) FVC_TGL(2, 16) FVC_TGL(3, 16) FVC_TGL(4, 16)
#undef FVC_TGL
  }
  if (transposed && pcp <= 128) {
    // 8-row output tiles (6 x 19 input pixels in LDS: ~35 KB at pcp 76, four blocks per CU);
    // FVC_GATHER_TH=16: 16-row tiles
    const char* th_env = getenv("FVC_GATHER_TH");
    const int th = (th_env && atoi(th_env) == 16) ? 16 : 8;
    const dim3 gt(fvc_cdiv(Wo, 32), fvc_cdiv(Ho, th), batch);
    const size_t lds = (size_t)(th / 2 + 2) * 19 * (pcp + 1) * 4;
#define FVC_TGT(KS, CO)                                                                                        \
    if (ksize == KS && cout == CO) {                                                                          \
      const void* fn = th == 8 ? (const void*)k_tap_gather_t2_lds<KS, CO, 8> : (const void*)k_tap_gather_t2_lds<KS, CO, 16>; \
      if (lds > 64 * 1024) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      if (th == 8)                                                                                            \
        hipLaunchKernelGGL((k_tap_gather_t2_lds<KS, CO, 8>), gt, dim3(256), lds, st, P, pcp, bias, res, y, h, w, \
                           slope, post_op);                                                                   \
      else                                                                                                    \
        hipLaunchKernelGGL((k_tap_gather_t2_lds<KS, CO, 16>), gt, dim3(256), lds, st, P, pcp, bias, res, y, h, w, \
                           slope, post_op);                                                                   \
      FVC_CHECK_LAUNCH();                                                                                     \
      return 0;                                                                                               \
    }
    FVC_TGT(3, 1) FVC_TGT(3, 2) FVC_TGT(3, 3) FVC_TGT(3, 4)
    FVC_TGT(5, 1) FVC_TGT(5, 2) FVC_TGT(5, 3) FVC_TGT(5, 4)
#undef FVC_TGT
  }
#define FVC_TG(KS, CO, TR)                                                                                   \
  if (ksize == KS && cout == CO && transposed == TR) {                                                       \
    hipLaunchKernelGGL((k_tap_gather<KS, CO, TR>), g, bl, 0, st, P, pcp, bias, res, y, batch, h, w, Ho, Wo, \
                       slope, post_op);                                                                      \
    FVC_CHECK_LAUNCH();                                                                                      \
    return 0;                                                                                                \
  }
  FVC_TG(3, 1, 0) FVC_TG(3, 2, 0) FVC_TG(3, 3, 0) FVC_TG(3, 4, 0)
  FVC_TG(5, 1, 0) FVC_TG(5, 2, 0) FVC_TG(5, 3, 0) FVC_TG(5, 4, 0)
  FVC_TG(3, 1, 1) FVC_TG(3, 2, 1) FVC_TG(3, 3, 1) FVC_TG(3, 4, 1)
  FVC_TG(5, 1, 1) FVC_TG(5, 2, 1) FVC_TG(5, 3, 1) FVC_TG(5, 4, 1)
#undef FVC_TG
  return FVC_EINVAL;
}

int fvc_sub_f32(const float* a, const float* b, float* out, size_t n, fvc_stream_t s) {
  if (!a || !b || !out) return FVC_EINVAL;
  hipLaunchKernelGGL(k_sub, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, a, b, out, n);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_gdn_nhwc_cai(const float* x, float* y, const float* beta, const float* gamma, int batch, int h, int w, int c,
                     int inverse, fvc_stream_t s) {
  if (!x || !y || !beta || !gamma || (c != 64 && c != 128)) return FVC_EINVAL;
  const size_t npix = (size_t)batch * h * w;
  size_t nblk = (npix + kGcPix - 1) / kGcPix;
  if (nblk > 8192) nblk = 8192;
  if (nblk < 1) nblk = 1;
  if (c == 128)
    hipLaunchKernelGGL(k_gdn_cai<128>, dim3((unsigned)nblk), dim3(128), 0, (hipStream_t)s, x, y, beta, gamma, npix,
                       inverse);
  else
    hipLaunchKernelGGL(k_gdn_cai<64>, dim3((unsigned)nblk), dim3(64), 0, (hipStream_t)s, x, y, beta, gamma, npix,
                       inverse);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_lstm_gates(const float* gj, const float* gi, const float* gf, const float* go, const float* c_prev,
                   float* c_out, float* h_out, size_t n, float forget_bias, fvc_stream_t s) {
  if (!gj || !gi || !gf || !go || !c_prev || !c_out || !h_out) return FVC_EINVAL;
  hipLaunchKernelGGL(k_lstm_gates, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, gj, gi, gf, go, c_prev, c_out,
                     h_out, n, forget_bias);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_rpm_scale(const float* in, float* out, size_t n, fvc_stream_t s) {
  if (!in || !out) return FVC_EINVAL;
  hipLaunchKernelGGL(k_rpm_scale, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, in, out, n);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_eb_forward(const float* x, const float* params, const float* medians, float* xhat, double* out1, double* ws,
                   int batch, int h, int w, int c, int cp, fvc_stream_t s) {
  if (!x || !params || !medians || !xhat || !out1 || !ws || c > cp) return FVC_EINVAL;
  hipLaunchKernelGGL(k_eb_forward, dim3(kRedBlocks), dim3(kBlk), 0, (hipStream_t)s, x, params, medians, xhat, ws,
                     (size_t)batch * h * w, c, cp);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_reduce_partials<1>, dim3(1), dim3(kBlk), 0, (hipStream_t)s, ws, kRedBlocks, out1);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_gc_forward(const float* x, const float* scale, const float* mu, float* xhat, double* out1, double* ws,
                   int batch, int h, int w, int c, int cp, fvc_stream_t s) {
  if (!x || !scale || !mu || !xhat || !out1 || !ws || c > cp) return FVC_EINVAL;
  hipLaunchKernelGGL(k_gc_forward, dim3(kRedBlocks), dim3(kBlk), 0, (hipStream_t)s, x, scale, mu, xhat, ws,
                     (size_t)batch * h * w, c, cp);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_reduce_partials<1>, dim3(1), dim3(kBlk), 0, (hipStream_t)s, ws, kRedBlocks, out1);
  FVC_CHECK_LAUNCH();
  return 0;
}

// persistent grid of the split-precision GDN kernels: 4 groups of 32 pixels per block and pass
static unsigned gdn_x3_blocks(size_t npix) {
  static const int cap = env_flag("FVC_GDN_BLOCKS", 1024);
  size_t nb = ((npix + 31) / 32 + 3) / 4;
  if (nb > (size_t)cap) nb = (size_t)cap;
  return nb < 1 ? 1u : (unsigned)nb;
}

int fvc_gdn_nhwc(const float* x, float* y, const float* beta, const float* gamma, int batch, int h, int w, int c,
                 int inverse, fvc_stream_t s) {
  if (!x || !y || !beta || !gamma || c != 64) return FVC_EINVAL;
  const size_t npix = (size_t)batch * h * w;
  if (env_flag("FVC_GDN_X3", 1)) {
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (inverse)
      hipLaunchKernelGGL((k_gdn_x3<0, true>), dim3(gdn_x3_blocks(npix)), dim3(256), 0, (hipStream_t)s, x, y, beta, gamma,
                         (const uint4*)nullptr, z4, npix, 0, (int*)nullptr);
    else
      hipLaunchKernelGGL((k_gdn_x3<0, false>), dim3(gdn_x3_blocks(npix)), dim3(256), 0, (hipStream_t)s, x, y, beta,
                         gamma, (const uint4*)nullptr, z4, npix, 0, (int*)nullptr);
    FVC_CHECK_LAUNCH();
    return 0;
  }
  size_t nblk = ((npix + 31) / 32 + kGdnWaves - 1) / kGdnWaves;
  if (nblk > 2048) nblk = 2048;
  if (nblk < 1) nblk = 1;
  hipLaunchKernelGGL(k_gdn_mfma, dim3((unsigned)nblk), dim3(64 * kGdnWaves), 0, (hipStream_t)s, x, y, beta, gamma,
                     npix, inverse);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_gdn_tap_nhwc(const float* x, float* P, const float* beta, const float* gamma, const void* tap_wpack,
                     const float* tap_osc, int ntiles, int pcp, int batch, int h, int w, int c, int inverse,
                     int* overflow_flag, fvc_stream_t s) {
  if (!x || !P || !beta || !gamma || !tap_wpack || !tap_osc || c != 64 || ntiles < 1 || ntiles > 4 || pcp <= 0 ||
      pcp % 4 || pcp > 32 * ntiles)
    return FVC_EINVAL;
  const size_t npix = (size_t)batch * h * w;
  size_t nblk = ((npix + 31) / 32 + kGdnWaves - 1) / kGdnWaves;
  if (nblk > 2048) nblk = 2048;
  if (nblk < 1) nblk = 1;
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < ntiles; ++i) t[i] = tap_osc[i];
  const float4 tosc = make_float4(t[0], t[1], t[2], t[3]);
  const uint4* tw = (const uint4*)tap_wpack;
  if (env_flag("FVC_GDN_X3", 1)) {
    const unsigned nb = gdn_x3_blocks(npix);
#define FVC_GX(N, I)                                                                                           \
  if (ntiles == N && !!inverse == I)                                                                           \
    hipLaunchKernelGGL((k_gdn_x3<N, I>), dim3(nb), dim3(256), 0, (hipStream_t)s, x, P, beta, gamma, tw, tosc, npix, \
                       pcp, overflow_flag);
    FVC_GX(1, false) FVC_GX(2, false) FVC_GX(3, false) FVC_GX(4, false)
    FVC_GX(1, true) FVC_GX(2, true) FVC_GX(3, true) FVC_GX(4, true)
#undef FVC_GX
    FVC_CHECK_LAUNCH();
    return 0;
  }
#define FVC_GT(N)                                                                                               \
  if (ntiles == N) {                                                                                          \
    hipLaunchKernelGGL(k_gdn_tap_mfma<N>, dim3((unsigned)nblk), dim3(64 * kGdnWaves), 0, (hipStream_t)s, x, P, beta, \
                       gamma, tw, tosc, npix, inverse, pcp, overflow_flag);                                   \
    FVC_CHECK_LAUNCH();                                                                                       \
    return 0;                                                                                                 \
  }
  FVC_GT(1) FVC_GT(2) FVC_GT(3) FVC_GT(4)
#undef FVC_GT
  return FVC_EINVAL;
}

size_t fvc_reduce_ws_doubles(void) { return (size_t)kRedBlocks * 4; }

int fvc_recon_finalize(const float* recon, const float* input, const float* warpframe, const float* prediction,
                       float* clipped, double* out4, double* ws, int batch, int h, int w, fvc_stream_t s) {
  if (!recon || !input || !warpframe || !prediction || !clipped || !out4 || !ws) return FVC_EINVAL;
  hipLaunchKernelGGL(k_recon_finalize, dim3(kRedBlocks), dim3(kBlk), 0, (hipStream_t)s, recon, input, warpframe,
                     prediction, clipped, ws, batch, h, w);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_reduce_partials<4>, dim3(1), dim3(kBlk), 0, (hipStream_t)s, ws, kRedBlocks, out4);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_bits_laplace(const float* feature, const float* sigma, double* out1, double* ws, int batch, int h, int w,
                     int c, int cp, fvc_stream_t s) {
  if (!feature || !sigma || !out1 || !ws || c > cp) return FVC_EINVAL;
  hipLaunchKernelGGL(k_bits_laplace, dim3(kRedBlocks), dim3(kBlk), 0, (hipStream_t)s, feature, sigma, ws,
                     (size_t)batch * h * w, c, cp);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_reduce_partials<1>, dim3(1), dim3(kBlk), 0, (hipStream_t)s, ws, kRedBlocks, out1);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_bits_factorized(const float* v, const float* params, double* out1, double* ws, int batch, int h, int w,
                        int c, int cp, fvc_stream_t s) {
  if (!v || !params || !out1 || !ws || c > cp) return FVC_EINVAL;
  hipLaunchKernelGGL(k_bits_factorized, dim3(kRedBlocks), dim3(kBlk), 0, (hipStream_t)s, v, params, ws,
                     (size_t)batch * h * w, c, cp);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_reduce_partials<1>, dim3(1), dim3(kBlk), 0, (hipStream_t)s, ws, kRedBlocks, out1);
  FVC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
