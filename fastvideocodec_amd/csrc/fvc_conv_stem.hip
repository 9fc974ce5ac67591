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
// Shape of the kernel: no LDS staging of activations. A wave owns a strip of 32 output pixels of
// one row; each lane fetches its own pixel's input taps straight from global memory (neighbouring
// lanes' taps overlap in L1), splits them into fp16 hi / lo once into registers (the MFMA B
// operands of every k-step), then runs the N-tiles of the output one after another (32 channels
// each, the accumulators reused), so the registers stay low and several waves per SIMD keep the
// stores streaming. The weights (at most 7 k-steps x 4 N-tiles x hi/lo fragments = 56 KB) sit in
// LDS, loaded once per block.
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
constexpr int kThreads = 256;  // 4 waves

struct StemArgs {
  const float* x;     // [B][H][W][CINP]
  const uint4* w;     // [step][n][plane][lane] 16-B fragments
  const float* bias;  // [cout]
  float* y;           // [B][Ho][Wo][cout]
  int B, H, W, Ho, Wo, cout;
  int strips_per_row, nstrips;
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

template <int CINP, int NT, int K, int S, int ACT>
__global__ __launch_bounds__(kThreads) void conv_stem_kernel(const StemArgs a) {
  using G = StemGeom<CINP, K>;
  constexpr int NS = G::kSteps;
  constexpr int P = K / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint4* const sw = reinterpret_cast<uint4*>(smem);                  // [NS][NT][2][64]
  float* const sbias = reinterpret_cast<float*>(smem + NS * NT * 2 * 64 * 16);  // [32 NT]

  const int tid = threadIdx.x;
  for (int i = tid; i < NS * NT * 2 * 64; i += kThreads) sw[i] = a.w[i];
  for (int i = tid; i < 32 * NT; i += kThreads) sbias[i] = i < a.cout ? a.bias[i] : 0.f;
  __syncthreads();

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 31;  // the lane's pixel in the strip (MFMA column)
  const int lh = lane >> 5;  // which 8 K values of a k-step the lane holds
  const int H = a.H, W = a.W;
  const unsigned img_bytes = (unsigned)H * (unsigned)W * CINP * 4u;
  f32x4 chk = {0.f, 0.f, 0.f, 0.f};

  for (int s = blockIdx.x * 4 + wave; s < a.nstrips; s += gridDim.x * 4) {
    const int row = s / a.strips_per_row;  // b * Ho + oy
    const int ox = (s - row * a.strips_per_row) * 32 + li;
    const int b = row / a.Ho;
    const int oy = row - b * a.Ho;
    const bool ox_ok = ox < a.Wo;
    const __amdgpu_buffer_rsrc_t rx = rsrc(a.x + (size_t)b * H * W * CINP, img_bytes);

    // the lane's B operands of every k-step: its pixel's taps, split once
    h8 bh[NS], bl[NS];
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      f32x4 v[2];
#pragma unroll
      for (int t = 0; t < G::kTapsPerLane; ++t) {
        const int tap = st * G::kTapsPerStep + lh * G::kTapsPerLane + t;
        const int ky = tap / K, kx = tap - (tap / K) * K;
        const int iy = oy * S + ky - P, ix = ox * S + kx - P;
        const bool ok = tap < G::kTaps && ox_ok && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const unsigned off = ok ? (unsigned)((iy * W + ix) * CINP) * 4u : kOob;
        if constexpr (CINP == 8) {
          v[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
          v[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, ok ? off + 16u : kOob, 0, 0));
        } else {
          v[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
        }
      }
      split8(v[0], v[1], bh[st], bl[st]);
    }

    const unsigned obase = ((unsigned)row * (unsigned)a.Wo + (unsigned)ox) * (unsigned)a.cout;
#pragma unroll 1
    for (int n = 0; n < NT; ++n) {
      f32x16 acc, cor;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = cor[r] = 0.f;
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        const h8 wh = __builtin_bit_cast(h8, sw[((st * NT + n) * 2 + 0) * 64 + lane]);
        const h8 wl = __builtin_bit_cast(h8, sw[((st * NT + n) * 2 + 1) * 64 + lane]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, bh[st], acc, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, bh[st], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, bl[st], cor, 0, 0, 0);
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
          float t = pre + bj[i];
          if constexpr (ACT == FVC_ACT_RELU) t = fmaxf(t, 0.f);
          if constexpr (ACT == FVC_ACT_LRELU) t = fmaxf(t, t * 0.1f);
          o[i] = t;
        }
        float* const dst = a.y + (size_t)obase + c0;
        if (ox_ok && c0 < a.cout) *reinterpret_cast<f32x4*>(dst) = o;
      }
    }
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
int stem_launch(const StemArgs& a, hipStream_t st) {
  using G = StemGeom<CINP, K>;
  const size_t lds = (size_t)G::kSteps * NT * 2 * 64 * 16 + 32 * NT * 4;
  const hipError_t e = hipFuncSetAttribute((const void*)conv_stem_kernel<CINP, NT, K, S, ACT>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  // persistent: as many blocks as fit on every CU at once (3-4 per CU: 12-16 waves keep the store
  // stream full), strips dealt round-robin to the waves
  static int per_cu = 0;
  if (!per_cu) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)conv_stem_kernel<CINP, NT, K, S, ACT>, kThreads,
                                                     lds) != hipSuccess || nb <= 0)
      nb = 2;
    per_cu = nb;
  }
  const long long want = ((long long)a.nstrips + 3) / 4;
  const long long cap = (long long)per_cu * stem_cus();
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL((conv_stem_kernel<CINP, NT, K, S, ACT>), dim3(grid), dim3(kThreads), lds, st, a);
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
  if (cout != 64 && cout != 128) return 0;
  return (ksize == 3 && (stride == 1 || stride == 2)) || (ksize == 5 && stride == 2);
}

size_t fvc_conv_stem_wpack_bytes(int cin, int cout, int ksize) {
  if (cin < 1 || cin > 8 || (cout != 64 && cout != 128) || (ksize != 3 && ksize != 5)) return 0;
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
  a.cout = cout;
  if ((unsigned long long)batch * a.Ho * a.Wo * cout >= (1ull << 32)) return FVC_EINVAL;
  a.strips_per_row = fvc_cdiv(a.Wo, 32);
  const long long ns = (long long)batch * a.Ho * a.strips_per_row;
  if (ns >= (1ll << 31)) return FVC_EINVAL;
  a.nstrips = (int)ns;
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
  return FVC_EINVAL;
}

}  // extern "C"
