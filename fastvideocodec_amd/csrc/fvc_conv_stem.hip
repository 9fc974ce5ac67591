// Split-precision direct convolution for the small-input "stem" layers, whose whole reduction
// (taps x input channels) is at most a few MFMA k-steps:
//   * Warp_net feature_ext, 3x3 s1 6 -> 64 on [warped frame, reference] (DVC/subnet/endecoder.py:
//     253-261, the first conv of Warp_net), at full resolution, twice per P-frame (encoder and decoder);
//   * mvEncoder conv1, 3x3 s2 2 -> 128 on the flow (DVC/subnet/analysis_mv.py:19-21, :58);
//   * resEncoder conv1, 5x5 s2 3 -> 64 on the residual (DVC/subnet/analysis.py:15-17, :44).
// Replaces the same ATen conv2d calls as fvc_conv_x3.hip, whose tiled kernel (input halo staged in
// LDS per channel chunk, 8-row tiles, the k-loop machinery of the 128-channel layers) runs these at
// 18-80 TF/s and 2.2-3.3 TB/s: their time is the output stream (64 or 128 channels per pixel from
// 2-8 input channels), and a plain store stream reaches 5.3 TB/s (profiles/r4/store_micro).
//
// Shape of the kernel: a block (4 waves) owns a tile of 4 output rows x 32 columns; its input
// window (e.g. 6 x 34 pixels for 3x3 s1) is loaded once, split into fp16 hi / lo planes in LDS
// (each input value split once, not once per tap that reads it), double-buffered so the next
// tile's loads fly during this tile's MFMAs and stores. Each wave builds its row's MFMA B operands
// for every k-step from LDS, then runs the output's N-tiles one after another (32 channels each,
// the accumulators reused), so the registers stay low and several blocks per CU keep the stores
// streaming. The weights (at most 7 k-steps x 4 N-tiles x hi/lo fragments = 56 KB) sit in LDS,
// loaded once per (persistent) block. (A first version fetched every tap per lane from global
// memory: 9x the load traffic at 3x3 s1, 43 % slower than the direct x3 kernel on 6 -> 64.)
//
// Reduction order: K index = tap * CINP + channel (tap = ky * k + kx, the input's pixel pitch
// CINP = 4 or 8 floats, channels past cin zero in the weights); one k-step = 16 K = two taps of
// 8 channels (CINP 8) or four taps of 4 (CINP 4). Numerics as fvc_conv_x3.hip: weights scaled by
// 2^kw (max in [2^13, 2^14)) and split hi + lo * 2^-11 on the host, activations split the same way
// in registers, main += w_hi x_hi and corr += w_lo x_hi + w_hi x_lo in two fp32 accumulators
// (v_mfma_f32_32x32x16_f16), y = main 2^-kw + corr 2^-kw-11 + bias. An input >= 65520 rounds to an
// infinite hi part: 0 * (every pre-activation output) is summed and a NaN raises the caller's
// overflow flag (the host then recomputes on the fp32 kernels), as the Winograd kernels do.
#include "fvc_common.h"
#include <math.h>
#include <stdlib.h>

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr float kLoScale = 2048.f;
constexpr unsigned kOob = 0xFFFFFF00u;
constexpr int kRsrcFlags = 0x00020000;

struct StemArgs {
  const float* x;     // [B][H][W][CINP]
  const uint4* w;     // [step][n][plane][lane] 16-B fragments
  const float* bias;  // [cout]
  float* y;           // [B][Ho][Wo][cout]
  int B, H, W, Ho, Wo, cin, cout;
  int tiles_x, tiles_y, ntiles;
  float osc, osc_c;
  int* ovf;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  const unsigned long long v = (unsigned long long)(uintptr_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* const q = (void*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), kRsrcFlags);
}

// v = hi + lo * 2^-11 for two values (the x3 / Winograd split)
__device__ __forceinline__ void split2(float v0, float v1, unsigned& hi, unsigned& lo) {
  float r0, r1;
  asm("v_cvt_pk_f16_f32 %0, %3, %4\n\t"
      "v_fma_mix_f32 %1, %0, -1.0, %3 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mix_f32 %2, %0, -1.0, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(hi), "=&v"(r0), "=&v"(r1)
      : "v"(v0), "v"(v1));
  asm("v_fma_mixlo_f16 %0, %1, %3, 0\n\t"
      "v_fma_mixhi_f16 %0, %2, %3, 0"
      : "=&v"(lo)
      : "v"(r0), "v"(r1), "s"(kLoScale));
}

__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, h8& hi, h8& lo) {
  unsigned hw[4], lw[4];
  split2(a[0], a[1], hw[0], lw[0]);
  split2(a[2], a[3], hw[1], lw[1]);
  split2(b[0], b[1], hw[2], lw[2]);
  split2(b[2], b[3], hw[3], lw[3]);
  hi = __builtin_bit_cast(h8, v4u{hw[0], hw[1], hw[2], hw[3]});
  lo = __builtin_bit_cast(h8, v4u{lw[0], lw[1], lw[2], lw[3]});
}

template <int CINP, int K>
struct StemGeom {
  static constexpr int kTaps = K * K;
  static constexpr int kTapsPerLane = CINP == 8 ? 1 : 2;  // one lane's 8 K values of a k-step
  static constexpr int kTapsPerStep = 2 * kTapsPerLane;
  static constexpr int kSteps = (kTaps + kTapsPerStep - 1) / kTapsPerStep;
};

// a block's tile: 4 output rows (one per wave) x 32 output columns; its input window staged in LDS
template <int CINP, int K, int S, int NW>
struct StemTile {
  static constexpr int kRows = (NW - 1) * S + K;
  static constexpr int kCols = 31 * S + K;
  static constexpr int kQ = CINP / 4;                          // 16-B channel quads per pixel
  static constexpr int kItems = kRows * kCols * kQ;
  static constexpr int kPer = (kItems + 64 * NW - 1) / (64 * NW);  // staging loads per thread
  static constexpr int kPlane = kRows * kCols * CINP * 2;          // bytes of one fp16 plane
};

template <int CINP, int NT, int K, int S, int ACT, int NW>
__global__ __launch_bounds__(64 * NW) void conv_stem_kernel(const StemArgs a) {
  constexpr int kThreads = 64 * NW;
  using G = StemGeom<CINP, K>;
  using T = StemTile<CINP, K, S, NW>;
  constexpr int NS = G::kSteps;
  constexpr int P = K / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* const sw = reinterpret_cast<uint4*>(smem);                  // [NS][NT][2][64]
  float* const sbias = reinterpret_cast<float*>(smem + NS * NT * 2 * 64 * 16);  // [32 NT]
  char* const tiles = smem + NS * NT * 2 * 64 * 16 + 32 * NT * 4;    // [buf][plane][pixel][CINP] fp16

  const int tid = threadIdx.x;
  for (int i = tid; i < NS * NT * 2 * 64; i += kThreads) sw[i] = a.w[i];
  for (int i = tid; i < 32 * NT; i += kThreads) sbias[i] = i < a.cout ? a.bias[i] : 0.f;

  const int lane = tid & 63;
  const int wave = tid >> 6;  // output row of the tile
  const int li = lane & 31;   // the lane's pixel in the strip (MFMA column)
  const int lh = lane >> 5;   // which 8 K values of a k-step the lane holds
  const int H = a.H, W = a.W;
  const unsigned img_bytes = (unsigned)H * (unsigned)W * CINP * 4u;
  f32x4 chk = {0.f, 0.f, 0.f, 0.f};

  struct Pos {
    int b, oy0, ox0;
  };
  auto decode = [&](int t) -> Pos {
    Pos q;
    const int per = a.tiles_y * a.tiles_x;
    q.b = t / per;
    const int r = t - q.b * per;
    const int ty = r / a.tiles_x;
    q.oy0 = NW * ty;
    q.ox0 = 32 * (r - ty * a.tiles_x);
    return q;
  };
  // staging: item e = (tile pixel, channel quad) -> one 16-B load (zeros outside the image
  // through the descriptor range), split into fp16 hi / lo planes once for every tap that reads it
  f32x4 v[T::kPer];
  auto fetch = [&](int t) {
    const Pos q = decode(t);
    const __amdgpu_buffer_rsrc_t rx = rsrc(a.x + (size_t)q.b * H * W * CINP, img_bytes);
#pragma unroll
    for (int j = 0; j < T::kPer; ++j) {
      const int e = tid + j * kThreads;
      const int pix = e / T::kQ, qd = e - pix * T::kQ;
      const int r = pix / T::kCols, c = pix - r * T::kCols;
      const int iy = q.oy0 * S - P + r, ix = q.ox0 * S - P + c;
      const bool ok = e < T::kItems && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      const unsigned off = ok ? (unsigned)((iy * W + ix) * CINP + 4 * qd) * 4u : kOob;
      v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
      // the pad channels (cin .. CINP-1) are masked here rather than trusted to be zero: their
      // weights are 0, but a NaN / Inf a producer left there would turn 0 * x into NaN
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * qd + i >= a.cin) v[j][i] = 0.f;
    }
  };
  auto stage = [&](int buf) {
    char* const th = tiles + (size_t)buf * 2 * T::kPlane;
#pragma unroll
    for (int j = 0; j < T::kPer; ++j) {
      const int e = tid + j * kThreads;
      if (e < T::kItems) {
        unsigned hw[2], lw[2];
        split2(v[j][0], v[j][1], hw[0], lw[0]);
        split2(v[j][2], v[j][3], hw[1], lw[1]);
        const int pix = e / T::kQ, qd = e - pix * T::kQ;
        const size_t o = ((size_t)pix * CINP + 4 * qd) * 2;
        *reinterpret_cast<uint2*>(th + o) = make_uint2(hw[0], hw[1]);
        *reinterpret_cast<uint2*>(th + T::kPlane + o) = make_uint2(lw[0], lw[1]);
      }
    }
  };

  int t = blockIdx.x;
  if (t < a.ntiles) {
    fetch(t);
    stage(0);
  }
  __syncthreads();
  int buf = 0;
  for (; t < a.ntiles; t += gridDim.x) {
    const int tn = t + (int)gridDim.x;
    if (tn < a.ntiles) fetch(tn);  // the next tile's loads fly during this tile's MFMAs and stores
    const Pos q = decode(t);
    const int oy = q.oy0 + wave, ox = q.ox0 + li;
    const bool out_ok = oy < a.Ho && ox < a.Wo;
    const char* const th = tiles + (size_t)buf * 2 * T::kPlane;

    // the lane's B operands of k-step st from the staged tile
    auto bop = [&](int st, h8& bhv, h8& blv) {
      if constexpr (CINP == 8) {
        const int tap = st * G::kTapsPerStep + lh;
        const int ky = tap / K, kx = tap - (tap / K) * K;
        const bool ok = tap < G::kTaps;
        const size_t o = ok ? (size_t)((wave * S + ky) * T::kCols + li * S + kx) * 16 : 0;
        const h8 hv = *reinterpret_cast<const h8*>(th + o);
        const h8 lv = *reinterpret_cast<const h8*>(th + T::kPlane + o);
        bhv = ok ? hv : h8{};
        blv = ok ? lv : h8{};
      } else {
        uint2 hp[2], lp[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int tap = st * G::kTapsPerStep + 2 * lh + u;
          const int ky = tap / K, kx = tap - (tap / K) * K;
          const bool ok = tap < G::kTaps;
          const size_t o = ok ? (size_t)((wave * S + ky) * T::kCols + li * S + kx) * 8 : 0;
          const uint2 hv = *reinterpret_cast<const uint2*>(th + o);
          const uint2 lv = *reinterpret_cast<const uint2*>(th + T::kPlane + o);
          hp[u] = ok ? hv : make_uint2(0u, 0u);
          lp[u] = ok ? lv : make_uint2(0u, 0u);
        }
        bhv = __builtin_bit_cast(h8, v4u{hp[0].x, hp[0].y, hp[1].x, hp[1].y});
        blv = __builtin_bit_cast(h8, v4u{lp[0].x, lp[0].y, lp[1].x, lp[1].y});
      }
    };
    // short reductions keep every k-step's B operands in registers across the N-tiles; long ones
    // (7x7: 25 k-steps) read them from LDS per k-step
    constexpr bool kHold = NS <= 8;
    h8 bh[kHold ? NS : 1], bl[kHold ? NS : 1];
    if constexpr (kHold) {
#pragma unroll
      for (int st = 0; st < NS; ++st) bop(st, bh[st], bl[st]);
    }

    const unsigned obase = (((unsigned)q.b * (unsigned)a.Ho + (unsigned)oy) * (unsigned)a.Wo + (unsigned)ox) *
                           (unsigned)a.cout;
#pragma unroll 1
    for (int n = 0; n < NT; ++n) {
      f32x16 acc, cor;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = cor[r] = 0.f;
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        const h8 wh = __builtin_bit_cast(h8, sw[((st * NT + n) * 2 + 0) * 64 + lane]);
        const h8 wl = __builtin_bit_cast(h8, sw[((st * NT + n) * 2 + 1) * 64 + lane]);
        h8 xh, xl;
        if constexpr (kHold) {
          xh = bh[st];
          xl = bl[st];
        } else {
          bop(st, xh, xl);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xh, acc, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, xh, cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, xl, cor, 0, 0, 0);
      }
      // lane (li, lh) register 4g + i: output channel 32 n + 8 g + 4 lh + i of pixel li
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = 32 * n + 8 * g + 4 * lh;
        const f32x4 bj = *reinterpret_cast<const f32x4*>(sbias + c0);
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pre = fmaf(cor[4 * g + i], a.osc_c, acc[4 * g + i] * a.osc);
          chk[i] = fmaf(pre, 0.f, chk[i]);
          float tv = pre + bj[i];
          if constexpr (ACT == FVC_ACT_RELU) tv = fmaxf(tv, 0.f);
          if constexpr (ACT == FVC_ACT_LRELU) tv = fmaxf(tv, tv * 0.1f);
          o[i] = tv;
        }
        if (out_ok) *reinterpret_cast<f32x4*>(a.y + (size_t)obase + c0) = o;
      }
    }
    if (tn < a.ntiles) stage(buf ^ 1);  // the other buffer: every wave left it at the last barrier
    __syncthreads();
    buf ^= 1;
  }
  if ((chk[0] != 0.f || chk[1] != 0.f || chk[2] != 0.f || chk[3] != 0.f) && a.ovf) atomicOr(a.ovf, 1);
}

int stem_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int CINP, int NT, int K, int S, int ACT>
int stem_launch(StemArgs a, hipStream_t st) {
  // waves per block = output rows per tile: 8 where the input window is large (8-float pixels, 5x5),
  // 4 for the 3x3 s2 4-float one (2 -> 128; 8 rows measured 4 % slower there, 10 % faster on 6 -> 64)
  // (8 only where weights + two tile buffers still fit the 160 KB of LDS: not 8-float 5x5 s2 128)
  constexpr int NS0 = StemGeom<CINP, K>::kSteps;
  constexpr size_t kLds8 = (size_t)NS0 * NT * 2 * 64 * 16 + 32 * NT * 4 + 4 * (size_t)StemTile<CINP, K, S, 8>::kPlane;
  constexpr int NW = ((CINP == 8 || K == 5) && kLds8 <= 160 * 1024) ? 8 : 4;
  constexpr int kThreads = 64 * NW;
  using G = StemGeom<CINP, K>;
  using T = StemTile<CINP, K, S, NW>;
  a.tiles_y = fvc_cdiv(a.Ho, NW);
  a.ntiles = a.B * a.tiles_y * a.tiles_x;
  const size_t lds = (size_t)G::kSteps * NT * 2 * 64 * 16 + 32 * NT * 4 + 2 * 2 * (size_t)T::kPlane;
  static_assert((size_t)G::kSteps * NT * 2 * 64 * 16 + 32 * NT * 4 + 4 * (size_t)T::kPlane <= 160 * 1024,
                "stem LDS over 160 KB");
  const hipError_t e = hipFuncSetAttribute((const void*)conv_stem_kernel<CINP, NT, K, S, ACT, NW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  // persistent: as many blocks as fit on every CU at once (3-4 per CU: 12-16 waves keep the store
  // stream full), strips dealt round-robin to the waves
  static int per_cu = 0;
  if (!per_cu) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)conv_stem_kernel<CINP, NT, K, S, ACT, NW>, kThreads,
                                                     lds) != hipSuccess || nb <= 0)
      nb = 2;
    per_cu = nb;
  }
  const long long want = a.ntiles;
  const long long cap = (long long)per_cu * stem_cus();
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL((conv_stem_kernel<CINP, NT, K, S, ACT, NW>), dim3(grid), dim3(kThreads), lds, st, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

template <int CINP, int NT, int K, int S>
int stem_act(const StemArgs& a, int act, hipStream_t st) {
  if (act == FVC_ACT_RELU) return stem_launch<CINP, NT, K, S, FVC_ACT_RELU>(a, st);
  if (act == FVC_ACT_LRELU) return stem_launch<CINP, NT, K, S, FVC_ACT_LRELU>(a, st);
  return stem_launch<CINP, NT, K, S, FVC_ACT_NONE>(a, st);
}

int stem_cinp(int cin) { return cin <= 4 ? 4 : 8; }

int stem_steps(int cinp, int k) {
  const int tps = cinp == 8 ? 2 : 4;
  return (k * k + tps - 1) / tps;
}

}  // namespace

extern "C" {

// the instantiated geometries: 3x3 s1 and s2, 5x5 s2; 1 <= cin <= 8; cout 64 or 128
int fvc_conv_stem_supported(int cin, int cout, int ksize, int stride, int transposed) {
  if (transposed || cin < 1 || cin > 8) return 0;
  // (SpyNet's first layer, 7x7 8 -> 32, ran correctly here in isolation -- tests vs float64 and the
  // direct kernel -- but with it on this kernel the overlapped 8-view / 4K pipelines lost
  // encoder == decoder bit-exactness at a late P-frame, not root-caused in r5: it stays on x3;
  // -DFVC_STEM_K7 experiment builds re-enable it)
#ifdef FVC_STEM_K7
  if (ksize == 7) return cout == 32 && stride == 1;
#endif
  if (cout != 64 && cout != 128) return 0;
  return (ksize == 3 && (stride == 1 || stride == 2)) || (ksize == 5 && stride == 2);
}

size_t fvc_conv_stem_wpack_bytes(int cin, int cout, int ksize) {
  if (!fvc_conv_stem_supported(cin, cout, ksize, ksize == 5 ? 2 : 1, 0)) return 0;
  return (size_t)stem_steps(stem_cinp(cin), ksize) * (cout / 32) * 2 * 64 * 16;
}

// w: OIHW fp32 [cout][cin][k][k] -> [step][n][plane][lane][8] fp16: lane l holds output channel
// 32 n + (l & 31) and K values 16 step + 8 (l >> 5) + e, K = tap * cinp + ci (the MFMA A operand);
// scaled by 2^kw (max |w| 2^kw in [2^13, 2^14)), plane 1 = (v - hi) * 2^11
int fvc_conv_stem_pack_weight(const float* w, int cin, int cout, int ksize, void* wp, float* osc_out) {
  if (!w || !wp || !osc_out || !fvc_conv_stem_wpack_bytes(cin, cout, ksize)) return FVC_EINVAL;
  const int cinp = stem_cinp(cin), ns = stem_steps(cinp, ksize), nt = cout / 32, kt = ksize * ksize;
  double mx = 0.0;
  for (int i = 0; i < cout * cin * kt; ++i) mx = fabs((double)w[i]) > mx ? fabs((double)w[i]) : mx;
  int kw = 0;
  if (mx > 0.0 && isfinite(mx)) {
    int e;
    frexp(mx, &e);
    kw = 14 - e;
    kw = kw < -100 ? -100 : (kw > 100 ? 100 : kw);
  }
  const float sc = ldexpf(1.f, kw);
  *osc_out = ldexpf(1.f, -kw);
  _Float16* out = (_Float16*)wp;
  for (int st = 0; st < ns; ++st)
    for (int n = 0; n < nt; ++n)
      for (int lane = 0; lane < 64; ++lane) {
        const int co = 32 * n + (lane & 31);
        for (int e = 0; e < 8; ++e) {
          const int kidx = 16 * st + 8 * (lane >> 5) + e;
          const int tap = kidx / cinp, ci = kidx - tap * cinp;
          const float v = (tap < kt && ci < cin) ? w[((size_t)co * cin + ci) * kt + tap] * sc : 0.f;
          const _Float16 hi = (_Float16)v;
          const size_t base = ((((size_t)st * nt + n) * 2) * 64 + lane) * 8;
          out[base + e] = hi;
          out[base + 64 * 8 + e] = (_Float16)((v - (float)hi) * 2048.f);
        }
      }
  return 0;
}

// x: NHWC with pixel pitch cinp = 4 (cin <= 4) or 8; y: NHWC [batch][h/stride][w/stride][cout];
// act as fvc_conv2d_nhwc_x3 (none / ReLU / LeakyReLU 0.1); no input op, residual or post-op
int fvc_conv2d_nhwc_stem(const float* x, const void* wpack, float osc, const float* bias, float* y, int batch, int h,
                         int w, int cin, int cout, int ksize, int stride, int act, int* overflow_flag,
                         fvc_stream_t stream) {
  if (!x || !wpack || !bias || !y || batch <= 0 || h <= 0 || w <= 0) return FVC_EINVAL;
  if (!fvc_conv_stem_supported(cin, cout, ksize, stride, 0)) return FVC_EINVAL;
  if (act != FVC_ACT_NONE && act != FVC_ACT_RELU && act != FVC_ACT_LRELU) return FVC_EINVAL;
  if (stride == 2 && ((h & 1) || (w & 1))) return FVC_EINVAL;
  const int cinp = stem_cinp(cin);
  // one image's input within a 32-bit buffer range; output offsets in 32 bits per launch
  if ((unsigned long long)h * w * cinp * 4ull >= (1ull << 31)) return FVC_EINVAL;
  StemArgs a;
  a.x = x;
  a.w = (const uint4*)wpack;
  a.bias = bias;
  a.y = y;
  a.B = batch;
  a.H = h;
  a.W = w;
  a.Ho = h / stride;
  a.Wo = w / stride;
  a.cin = cin;
  a.cout = cout;
  if ((unsigned long long)batch * a.Ho * a.Wo * cout >= (1ull << 32)) return FVC_EINVAL;
  a.tiles_x = fvc_cdiv(a.Wo, 32);
  a.tiles_y = fvc_cdiv(a.Ho, 4);  // per launch: the block height of the instantiation (stem_launch)
  const long long nt = (long long)batch * a.tiles_y * a.tiles_x;
  if (nt >= (1ll << 31)) return FVC_EINVAL;
  a.ntiles = (int)nt;
  a.osc = osc;
  a.osc_c = osc * (1.f / 2048.f);
  a.ovf = overflow_flag;
  const hipStream_t st = (hipStream_t)stream;
  if (cinp == 8 && ksize == 3 && stride == 1 && cout == 64) return stem_act<8, 2, 3, 1>(a, act, st);
  if (cinp == 8 && ksize == 3 && stride == 1 && cout == 128) return stem_act<8, 4, 3, 1>(a, act, st);
  if (cinp == 4 && ksize == 3 && stride == 1 && cout == 64) return stem_act<4, 2, 3, 1>(a, act, st);
  if (cinp == 4 && ksize == 3 && stride == 2 && cout == 128) return stem_act<4, 4, 3, 2>(a, act, st);
  if (cinp == 4 && ksize == 3 && stride == 2 && cout == 64) return stem_act<4, 2, 3, 2>(a, act, st);
  if (cinp == 8 && ksize == 3 && stride == 2 && cout == 128) return stem_act<8, 4, 3, 2>(a, act, st);
  if (cinp == 8 && ksize == 3 && stride == 2 && cout == 64) return stem_act<8, 2, 3, 2>(a, act, st);
  if (cinp == 4 && ksize == 3 && stride == 1 && cout == 128) return stem_act<4, 4, 3, 1>(a, act, st);
  if (cinp == 4 && ksize == 5 && stride == 2 && cout == 64) return stem_act<4, 2, 5, 2>(a, act, st);
  if (cinp == 4 && ksize == 5 && stride == 2 && cout == 128) return stem_act<4, 4, 5, 2>(a, act, st);
  if (cinp == 8 && ksize == 5 && stride == 2 && cout == 64) return stem_act<8, 2, 5, 2>(a, act, st);
  if (cinp == 8 && ksize == 5 && stride == 2 && cout == 128) return stem_act<8, 4, 5, 2>(a, act, st);
#ifdef FVC_STEM_K7
  if (cinp == 8 && ksize == 7 && stride == 1 && cout == 32) return stem_act<8, 1, 7, 1>(a, act, st);
#endif
  return FVC_EINVAL;
}

}  // extern "C"
