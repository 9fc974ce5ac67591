// I-frame codec kernels (replaces the reference's BPG I-frame, models.py:412-429, whose
// bpgenc/bpgdec binaries are absent): 8-bit samples, JPEG 2000 reversible colour transform, L
// levels of the reversible LeGall 5/3 lifting wavelet (rows then columns, symmetric extension,
// Mallat layout), optional dead-zone quantisation of the high-pass subbands, and the per-block
// Laplace scale index the device rANS codes each coefficient with. Integer arithmetic only, so
// encoder and decoder reconstructions are bit-identical; the numpy restatement is
// oracle/iframe_ref.py. All kernels are HBM-bound elementwise / stencil passes over a few MB.
#include "fvc_common.h"

namespace {

constexpr int kBlk = 256;

int grid_for(size_t n) {
  size_t g = (n + kBlk - 1) / kBlk;
  if (g > 16384) g = 16384;
  return (int)(g < 1 ? 1 : g);
}

// q = clamp(rint(x * 255), 0, 255); Y = (R + 2G + B) >> 2, U = B - G, V = R - G
__global__ void k_rct_fwd(const float* __restrict__ x, int32_t* __restrict__ c, int B, size_t hw) {
  const size_t n = (size_t)B * hw;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t b = e / hw, i = e % hw;
    const float* xb = x + b * 3 * hw;
    int q[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v = rintf(xb[k * hw + i] * 255.f);
      q[k] = (int)fminf(fmaxf(v, 0.f), 255.f);
    }
    int32_t* cb = c + b * 3 * hw;
    cb[i] = (q[0] + 2 * q[1] + q[2]) >> 2;
    cb[hw + i] = q[2] - q[1];
    cb[2 * hw + i] = q[0] - q[1];
  }
}

__global__ void k_rct_inv(const int32_t* __restrict__ c, float* __restrict__ x, int B, size_t hw) {
  const size_t n = (size_t)B * hw;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t b = e / hw, i = e % hw;
    const int32_t* cb = c + b * 3 * hw;
    const int y = cb[i], u = cb[hw + i], v = cb[2 * hw + i];
    const int g = y - ((u + v) >> 2);
    const int rgb[3] = {v + g, g, u + g};
    float* xb = x + b * 3 * hw;
#pragma unroll
    for (int k = 0; k < 3; ++k) xb[k * hw + i] = (float)min(max(rgb[k], 0), 255) / 255.f;
  }
}

// One 5/3 lifting phase on the sub-rectangle [0,h) x [0,w) of P planes of row stride W, along
// columns-of-a-row (axis 0: index runs along W) or rows (axis 1: index runs along H). A line of
// length L = (axis ? h : w) has L/2 pairs; element k of a line sits at line_base + k * step.
struct Lift {
  int P, H, W, h, w, axis;
};

__device__ __forceinline__ void line_of(const Lift& g, size_t e, size_t& base, int& n, int& step, int& L) {
  const int half = (g.axis ? g.h : g.w) / 2;
  n = (int)(e % half);
  const size_t line = e / half;            // (plane, other coordinate)
  const int nlines = g.axis ? g.w : g.h;
  const size_t p = line / nlines;
  const int o = (int)(line % nlines);
  step = g.axis ? g.W : 1;
  L = g.axis ? g.h : g.w;
  base = p * (size_t)g.H * g.W + (g.axis ? (size_t)o : (size_t)o * g.W);
}

// forward predict: dst[L/2 + n] = x[2n+1] - ((x[2n] + x[2n+2]) >> 1)   (x[L] := x[L-2])
__global__ void k_lift_predict(const int32_t* __restrict__ src, int32_t* __restrict__ dst, Lift g) {
  const size_t n_all = (size_t)g.P * (g.axis ? g.w : g.h) * ((g.axis ? g.h : g.w) / 2);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    size_t base; int n, step, L;
    line_of(g, e, base, n, step, L);
    const int i0 = 2 * n, i2 = 2 * n + 2 < L ? 2 * n + 2 : L - 2;
    const int32_t x0 = src[base + (size_t)i0 * step], x1 = src[base + (size_t)(i0 + 1) * step];
    const int32_t x2 = src[base + (size_t)i2 * step];
    dst[base + (size_t)(L / 2 + n) * step] = x1 - ((x0 + x2) >> 1);
  }
}

// forward update: dst[n] = x[2n] + ((d[n-1] + d[n] + 2) >> 2)   (d[-1] := d[0]), d from dst
__global__ void k_lift_update(const int32_t* __restrict__ src, int32_t* __restrict__ dst, Lift g) {
  const size_t n_all = (size_t)g.P * (g.axis ? g.w : g.h) * ((g.axis ? g.h : g.w) / 2);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    size_t base; int n, step, L;
    line_of(g, e, base, n, step, L);
    const int half = L / 2;
    const int32_t d0 = dst[base + (size_t)(half + (n > 0 ? n - 1 : 0)) * step];
    const int32_t d1 = dst[base + (size_t)(half + n) * step];
    dst[base + (size_t)n * step] = src[base + (size_t)(2 * n) * step] + ((d0 + d1 + 2) >> 2);
  }
}

// inverse: even samples e[n] = s[n] - ((d[n-1] + d[n] + 2) >> 2) into dst[2n]
__global__ void k_unlift_even(const int32_t* __restrict__ src, int32_t* __restrict__ dst, Lift g) {
  const size_t n_all = (size_t)g.P * (g.axis ? g.w : g.h) * ((g.axis ? g.h : g.w) / 2);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    size_t base; int n, step, L;
    line_of(g, e, base, n, step, L);
    const int half = L / 2;
    const int32_t d0 = src[base + (size_t)(half + (n > 0 ? n - 1 : 0)) * step];
    const int32_t d1 = src[base + (size_t)(half + n) * step];
    dst[base + (size_t)(2 * n) * step] = src[base + (size_t)n * step] - ((d0 + d1 + 2) >> 2);
  }
}

// inverse: odd samples o[n] = d[n] + ((e[n] + e[n+1]) >> 1) into dst[2n+1] (e[half] := e[half-1])
__global__ void k_unlift_odd(const int32_t* __restrict__ src, int32_t* __restrict__ dst, Lift g) {
  const size_t n_all = (size_t)g.P * (g.axis ? g.w : g.h) * ((g.axis ? g.h : g.w) / 2);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    size_t base; int n, step, L;
    line_of(g, e, base, n, step, L);
    const int half = L / 2;
    const int32_t e0 = dst[base + (size_t)(2 * n) * step];
    const int32_t e1 = dst[base + (size_t)(n + 1 < half ? 2 * n + 2 : 2 * n) * step];
    dst[base + (size_t)(2 * n + 1) * step] = src[base + (size_t)(half + n) * step] + ((e0 + e1) >> 1);
  }
}

__global__ void k_copy_sub(const int32_t* __restrict__ src, int32_t* __restrict__ dst, int P, int H, int W, int h,
                           int w) {
  const size_t n_all = (size_t)P * h * w;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e / ((size_t)h * w);
    const int r = (int)((e / w) % h), c = (int)(e % w);
    const size_t o = p * (size_t)H * W + (size_t)r * W + c;
    dst[o] = src[o];
  }
}

// dead-zone quantisation of the high-pass coefficients (outside the level-L LL band)
__global__ void k_quant(int32_t* __restrict__ c, int P, int H, int W, int hl, int wl, int q, int inverse) {
  const size_t n_all = (size_t)P * H * W;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)((e / W) % H), col = (int)(e % W);
    if (r < hl && col < wl) continue;
    const int v = c[e];
    const int a = v < 0 ? -v : v;
    int out;
    if (!inverse) out = a / q;
    else out = a == 0 ? 0 : a * q + q / 2;
    c[e] = v < 0 ? -out : out;
  }
}

// per (plane, bs x bs block): mean |c| -> the Laplace table index compressai's build_indexes
// gives that scale (count of table entries >= s, s = max(mean, 0.11)); one wave per block, the
// sum in a fixed order (lane partials, then a fixed shuffle tree) so it is deterministic
__global__ void k_block_index(const int32_t* __restrict__ c, const float* __restrict__ table, int nt,
                              uint8_t* __restrict__ idx, int P, int H, int W, int bs) {
  const int bw = W / bs, bh = H / bs;
  const int blk = blockIdx.x;
  if (blk >= P * bh * bw) return;
  const int p = blk / (bh * bw), by = (blk / bw) % bh, bx = blk % bw;
  const int32_t* cb = c + (size_t)p * H * W + (size_t)by * bs * W + (size_t)bx * bs;
  long long s = 0;
  for (int i = threadIdx.x; i < bs * bs; i += 64) {
    const int v = cb[(size_t)(i / bs) * W + (i % bs)];
    s += v < 0 ? -v : v;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (threadIdx.x == 0) {
    const float m = fmaxf((float)((double)s / (double)(bs * bs)), 0.11f);
    int v = nt - 1;
    for (int k = 0; k < nt - 1; ++k) v -= (m <= table[k]) ? 1 : 0;
    idx[blk] = (uint8_t)v;
  }
}

// per-coefficient table index from the block indexes
__global__ void k_expand_index(const uint8_t* __restrict__ bidx, int32_t* __restrict__ idx, int P, int H, int W,
                               int bs) {
  const size_t n_all = (size_t)P * H * W;
  const int bw = W / bs, bh = H / bs;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n_all; e += (size_t)gridDim.x * blockDim.x) {
    const size_t p = e / ((size_t)H * W);
    const int r = (int)((e / W) % H), col = (int)(e % W);
    idx[e] = bidx[(p * bh + r / bs) * bw + col / bs];
  }
}

}  // namespace

extern "C" {

int fvc_iframe_rct_fwd(const float* x, int32_t* coeff, int batch, int h, int w, fvc_stream_t s) {
  if (!x || !coeff || batch <= 0 || h <= 0 || w <= 0) return FVC_EINVAL;
  const size_t hw = (size_t)h * w;
  hipLaunchKernelGGL(k_rct_fwd, dim3(grid_for(batch * hw)), dim3(kBlk), 0, (hipStream_t)s, x, coeff, batch, hw);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_iframe_rct_inv(const int32_t* coeff, float* x, int batch, int h, int w, fvc_stream_t s) {
  if (!x || !coeff || batch <= 0 || h <= 0 || w <= 0) return FVC_EINVAL;
  const size_t hw = (size_t)h * w;
  hipLaunchKernelGGL(k_rct_inv, dim3(grid_for(batch * hw)), dim3(kBlk), 0, (hipStream_t)s, coeff, x, batch, hw);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_iframe_dwt53(int32_t* coeff, int32_t* tmp, int planes, int h, int w, int levels, int inverse,
                     fvc_stream_t s) {
  if (!coeff || !tmp || planes <= 0 || levels < 0 || levels > 12) return FVC_EINVAL;
  if (h % (1 << levels) || w % (1 << levels)) return FVC_EINVAL;
  const hipStream_t st = (hipStream_t)s;
  auto launch = [&](void (*k)(const int32_t*, int32_t*, Lift), const int32_t* a, int32_t* b, const Lift& g) {
    const size_t n = (size_t)g.P * (g.axis ? g.w : g.h) * ((g.axis ? g.h : g.w) / 2);
    hipLaunchKernelGGL(k, dim3(grid_for(n)), dim3(kBlk), 0, st, a, b, g);
  };
  auto copy_back = [&](int hh, int ww) {
    const size_t n = (size_t)planes * hh * ww;
    hipLaunchKernelGGL(k_copy_sub, dim3(grid_for(n)), dim3(kBlk), 0, st, tmp, coeff, planes, h, w, hh, ww);
  };
  for (int i = 0; i < levels; ++i) {
    const int lv = inverse ? levels - 1 - i : i;
    const int hh = h >> lv, ww = w >> lv;
    // forward: rows then columns; inverse: columns then rows
    for (int a = 0; a < 2; ++a) {
      const int axis = inverse ? 1 - a : a;
      const Lift g{planes, h, w, hh, ww, axis};
      if (!inverse) {
        launch(k_lift_predict, coeff, tmp, g);
        launch(k_lift_update, coeff, tmp, g);
      } else {
        launch(k_unlift_even, coeff, tmp, g);
        launch(k_unlift_odd, coeff, tmp, g);
      }
      copy_back(hh, ww);
    }
  }
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_iframe_quant(int32_t* coeff, int planes, int h, int w, int levels, int q, int inverse, fvc_stream_t s) {
  if (!coeff || planes <= 0 || q < 1 || levels < 0) return FVC_EINVAL;
  if (q == 1) return 0;
  const size_t n = (size_t)planes * h * w;
  hipLaunchKernelGGL(k_quant, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, coeff, planes, h, w, h >> levels,
                     w >> levels, q, inverse);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_iframe_block_index(const int32_t* coeff, const float* scale_table, int n_scales, uint8_t* bidx,
                           int32_t* idx, int planes, int h, int w, int bs, fvc_stream_t s) {
  if (!coeff || !scale_table || !bidx || !idx || n_scales < 1 || n_scales > 256 || bs <= 0 || h % bs || w % bs)
    return FVC_EINVAL;
  const int nblk = planes * (h / bs) * (w / bs);
  hipLaunchKernelGGL(k_block_index, dim3(nblk), dim3(64), 0, (hipStream_t)s, coeff, scale_table, n_scales, bidx,
                     planes, h, w, bs);
  FVC_CHECK_LAUNCH();
  const size_t n = (size_t)planes * h * w;
  hipLaunchKernelGGL(k_expand_index, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, bidx, idx, planes, h, w,
                     bs);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_iframe_expand_index(const uint8_t* bidx, int32_t* idx, int planes, int h, int w, int bs, fvc_stream_t s) {
  if (!bidx || !idx || bs <= 0 || h % bs || w % bs) return FVC_EINVAL;
  const size_t n = (size_t)planes * h * w;
  hipLaunchKernelGGL(k_expand_index, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, bidx, idx, planes, h, w,
                     bs);
  FVC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
