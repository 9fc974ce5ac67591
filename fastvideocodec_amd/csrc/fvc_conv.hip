// Implicit-GEMM convolution / transposed convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the ATen conv2d / conv_transpose2d calls of the reference DVC forward
// (DVC/subnet/endecoder.py:142-169 MEBasic 7x7, :228-296 Warp_net/ResBlock 3x3,
// analysis_mv.py / synthesis_mv.py 3x3 (s2), analysis.py / synthesis.py / analysis_prior.py /
// synthesis_prior.py 5x5 s2 / 3x3).
//
// GEMM view: M = output pixels, N = output channels, K = taps x input channels.
//  * activations NHWC fp32, channels padded to 4 (cp);
//  * a block owns TH = 4*WM output rows x 32 output columns ("strips" of 32 pixels, one per
//    MFMA M-tile) and WN*32 output channels; 4 waves stacked vertically, each WM strips x WN
//    N-tiles (WM*WN accumulators of 16 VGPRs);
//  * K is walked in "k-blocks" = (tap, 4 consecutive input channels). One MFMA quad (4 x
//    32x32x2) consumes two k-blocks: lanes 0-31 take k-block 2q, lanes 32-63 take 2q+1, and
//    instruction e of the quad uses element e of each lane's float4 (a fixed permutation of the
//    K order shared by A and B, so results are deterministic);
//  * the input halo tile of one channel chunk (CC channels) lives in LDS (row stride padded so
//    CS/4 is odd: conflict-free ds_read_b128 across the 32 pixels of a strip); the packed weights
//    stream from L2 straight to VGPRs (16 B per lane, 1 KB per wave instruction, coalesced),
//    software-pipelined one quad ahead together with the LDS reads;
//  * transposed convs are split into stride^2 output-parity classes, each a stride-1 conv over
//    the input with a subset of taps (blockIdx.z = batch*classes + class); no zero-insertion.
//  * epilogue: bias, activation (ReLU / LeakyReLU 0.1), residual add, exp; pad channels = 0.
#include "fvc_common.h"
#include <stdlib.h>

namespace {

constexpr int kMaxTaps = 49;
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int kThreads = 256;

struct ConvArgs {
  const float* x;
  const float* w;
  const float* bias;
  const float* res;
  float* y;
  int B, H, W, cinp;       // input tensor
  int Ho, Wo, coutp, cout; // output tensor
  int Hq, Wq;              // virtual output grid (per class)
  int sin;                 // input step per virtual-grid step
  int sout;                // output step per virtual-grid step
  int nclass;
  int nchunks;
  int ntp;                 // padded N-tiles in the weight pack (cdiv(coutp,32))
  int dymin, dxmin;        // halo origin offset (union over classes)
  int ir, ic;              // halo tile rows / cols
  int in_op, act, post_op;
  int kbc[4];              // k-blocks per chunk per class (even)
  int ntaps[4];
  int oy0[4], ox0[4];
  long long wcls[4];       // float offset of each class in the weight pack
  short tdy[4][kMaxTaps];
  short tdx[4][kMaxTaps];
  int gy0[4], gny[4], gx0[4], gnx[4];  // per class: tap offsets form [gy0, gy0+gny) x [gx0, gx0+gnx)
};

template <int CC>
struct ChunkGeom {
  static constexpr int CC4 = CC / 4;
  static constexpr int CS = (CC4 % 2 == 1) ? CC : CC + 4;  // LDS pixel stride (floats)
};

template <int CC, int WM, int WN, int BPF>
__global__ __launch_bounds__(kThreads) void conv_mfma_f32_kernel(const ConvArgs a) {
  using G = ChunkGeom<CC>;
  constexpr int CC4 = G::CC4;
  constexpr int CS = G::CS;
  constexpr int TH = 4 * WM;
  constexpr int TW = 32;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* tap_off = reinterpret_cast<int*>(smem);  // kMaxTaps ints (64 reserved)
  float* tile = smem + 64;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 31;
  const int lh = lane >> 5;

  const int cls = blockIdx.z % a.nclass;
  const int b = blockIdx.z / a.nclass;
  const int tiles_x = (a.Wq + TW - 1) / TW;
  const int qy0 = (blockIdx.x / tiles_x) * TH;
  const int qx0 = (blockIdx.x % tiles_x) * TW;
  const int nt0 = blockIdx.y * WN;
  const int ntaps = a.ntaps[cls];
  const int kbc = a.kbc[cls];

  if (tid < ntaps) {
    tap_off[tid] = ((a.tdy[cls][tid] - a.dymin) * a.ic + (a.tdx[cls][tid] - a.dxmin)) * CS;
  }

  f32x16 acc[WM][WN];
#pragma unroll
  for (int m = 0; m < WM; ++m)
#pragma unroll
    for (int n = 0; n < WN; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

  const int iy0 = qy0 * a.sin + a.dymin;
  const int ix0 = qx0 * a.sin + a.dxmin;
  const int tile_elems = a.ir * a.ic * CC4;
  const float* xb = a.x + (size_t)b * a.H * a.W * a.cinp;

  // per-lane LDS base of each strip pixel (row = wave*WM+m, col = li)
  int pix_base[WM];
#pragma unroll
  for (int m = 0; m < WM; ++m) pix_base[m] = (((wave * WM + m) * a.sin) * a.ic + li * a.sin) * CS;

  const float* wcls = a.w + a.wcls[cls];
  const int nq = kbc >> 1;

  for (int ch = 0; ch < a.nchunks; ++ch) {
    // ---- stage the input halo tile of this channel chunk (zero padded, in_op applied)
    for (int e = tid; e < tile_elems; e += kThreads) {
      const int c4 = e % CC4;
      const int p = e / CC4;
      const int r = p / a.ic;
      const int c = p - r * a.ic;
      const int iy = iy0 + r;
      const int ix = ix0 + c;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
        v = *reinterpret_cast<const float4*>(xb + ((size_t)iy * a.W + ix) * a.cinp + ch * CC + c4 * 4);
        v = fvc_in_op_sel4(v, a.in_op);
      }
      *reinterpret_cast<float4*>(tile + p * CS + c4 * 4) = v;
    }
    __syncthreads();

    const float* wch = wcls + (size_t)ch * kbc * a.ntp * 128;
    float4 A[WM], Bv[WN], An[WM], Bn[WN], Bnn[WN];
    auto loadA = [&](int q, float4 (&Ar)[WM]) {
      const int kb = 2 * q + lh;
      const int t = kb / CC4;
      const int c4 = kb - t * CC4;
      const int toff = (t < ntaps ? tap_off[t] : 0) + c4 * 4;
#pragma unroll
      for (int m = 0; m < WM; ++m) Ar[m] = *reinterpret_cast<const float4*>(tile + pix_base[m] + toff);
    };
    auto loadB = [&](int q, float4 (&Br)[WN]) {
      const int kb = 2 * q + lh;
      const float* wk = wch + ((size_t)kb * a.ntp + nt0) * 128 + li * 4;
#pragma unroll
      for (int n = 0; n < WN; ++n) Br[n] = *reinterpret_cast<const float4*>(wk + n * 128);
    };
    loadA(0, A);
    loadB(0, Bv);
    if (BPF == 2 && nq > 1) loadB(1, Bn);
    for (int q = 0; q < nq; ++q) {
      if (q + 1 < nq) loadA(q + 1, An);
      if (BPF == 2) {
        if (q + 2 < nq) loadB(q + 2, Bnn);
      } else {
        if (q + 1 < nq) loadB(q + 1, Bn);
      }
      // element-major issue order: consecutive MFMAs hit different accumulators (no RAW chain).
      // Weights are the row operand and pixels the column operand, so each lane ends with 4
      // consecutive channels of one pixel per register group (16-B epilogue stores); the two
      // products of each MFMA and their order are the same either way.
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(Bv[n].x, A[m].x, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(Bv[n].y, A[m].y, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(Bv[n].z, A[m].z, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(Bv[n].w, A[m].w, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m) A[m] = An[m];
#pragma unroll
      for (int n = 0; n < WN; ++n) {
        Bv[n] = Bn[n];
        if (BPF == 2) Bn[n] = Bnn[n];
      }
    }
    __syncthreads();
  }

  // ---- epilogue: lane (li, lh) holds pixel qx0 + li; register group g holds output channels
  // N-tile*32 + 8g + 4lh + {0..3} -> one 16-B store (and residual load) per group
  const int oy0 = a.oy0[cls], ox0 = a.ox0[cls];
  const int qx = qx0 + li;
  if (qx >= a.Wq) return;
  const int ox = qx * a.sout + ox0;
#pragma unroll
  for (int m = 0; m < WM; ++m) {
    const int qy = qy0 + wave * WM + m;
    if (qy >= a.Hq) continue;
    const int oy = qy * a.sout + oy0;
    const size_t obase = (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.coutp;
#pragma unroll
    for (int n = 0; n < WN; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j0 = (nt0 + n) * 32 + 8 * g + 4 * lh;
        if (j0 >= a.coutp) continue;  // coutp is a multiple of 4: whole groups
        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.res) rv = *reinterpret_cast<const float4*>(a.res + obase + j0);
        const float rr[4] = {rv.x, rv.y, rv.z, rv.w};
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool real = j0 + i < a.cout;
          float v = acc[m][n][4 * g + i] + (real ? a.bias[j0 + i] : 0.f);
          if (a.act == FVC_ACT_RELU) v = v > 0.f ? v : 0.f;
          else if (a.act == FVC_ACT_LRELU) v = v > 0.f ? v : 0.1f * v;
          if (a.res) v += rr[i];
          if (a.post_op == FVC_POST_EXP) v = expf(v);
          o[i] = real ? v : 0.f;
        }
        *reinterpret_cast<float4*>(a.y + obase + j0) = make_float4(o[0], o[1], o[2], o[3]);
      }
  }
}

// Pipelined variant for stride-1 convs: two LDS halo-tile buffers; while the waves run the
// MFMAs of channel chunk ch out of one buffer, each thread stages one float4 of chunk ch+1 per
// MFMA quad into the other (global load issued before the quad's MFMAs, LDS write after), so
// the staging latency hides under the matrix work and only one barrier per chunk remains.
template <int CC, int WM, int WN, int NW>
__global__ __launch_bounds__(NW * 64) void conv_mfma_pipe_kernel(const ConvArgs a) {
  using G = ChunkGeom<CC>;
  constexpr int CC4 = G::CC4;
  constexpr int CS = G::CS;
  constexpr int TH = NW * WM;
  constexpr int TW = 32;
  constexpr int NT = NW * 64;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* tap_off = reinterpret_cast<int*>(smem);
  const int tile_floats = (a.ir * a.ic * CS + 3) & ~3;
  float* const tile0 = smem + 64;  // buffers at tile0 and tile0 + tile_floats (no pointer array:
                                   // it would turn the LDS accesses into flat ones)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int cls = blockIdx.z % a.nclass;
  const int b = blockIdx.z / a.nclass;
  const int tiles_x = (a.Wq + TW - 1) / TW;
  const int qy0 = (blockIdx.x / tiles_x) * TH;
  const int qx0 = (blockIdx.x % tiles_x) * TW;
  const int nt0 = blockIdx.y * WN;
  const int ntaps = a.ntaps[cls];
  const int kbc = a.kbc[cls];
  const int nq = kbc >> 1;

  if (tid < ntaps) tap_off[tid] = ((a.tdy[cls][tid] - a.dymin) * a.ic + (a.tdx[cls][tid] - a.dxmin)) * CS;

  const int iy0 = qy0 * a.sin + a.dymin;
  const int ix0 = qx0 * a.sin + a.dxmin;
  const int tile_elems = a.ir * a.ic * CC4;
  const float* xb = a.x + (size_t)b * a.H * a.W * a.cinp;

  auto fetch = [&](int e, int ch, float4& v, int& dst) {
    const int c4 = e % CC4;
    const int p = e / CC4;
    const int r = p / a.ic;
    const int c = p - r * a.ic;
    const int iy = iy0 + r, ix = ix0 + c;
    v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
      v = *reinterpret_cast<const float4*>(xb + ((size_t)iy * a.W + ix) * a.cinp + ch * CC + c4 * 4);
    dst = p * CS + c4 * 4;
  };  // in_op is applied at the LDS write (after the MFMAs), see below

  // prologue: chunk 0
  for (int e = tid; e < tile_elems; e += NT) {
    float4 v;
    int d;
    fetch(e, 0, v, d);
    *reinterpret_cast<float4*>(tile0 + d) = fvc_in_op_sel4(v, a.in_op);
  }

  f32x16 acc[WM][WN];
#pragma unroll
  for (int m = 0; m < WM; ++m)
#pragma unroll
    for (int n = 0; n < WN; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

  int pix_base[WM];
#pragma unroll
  for (int m = 0; m < WM; ++m) pix_base[m] = ((wave * WM + m) * a.ic + li) * CS;
  const float* wcls = a.w + a.wcls[cls];
  const int nstage = (tile_elems + NT - 1) / NT;
  __syncthreads();

  for (int ch = 0; ch < a.nchunks; ++ch) {
    const float* cur = tile0 + (ch & 1) * tile_floats;
    float* nxt = tile0 + ((ch + 1) & 1) * tile_floats;
    const bool has_next = ch + 1 < a.nchunks;
    const float* wch = wcls + (size_t)ch * kbc * a.ntp * 128;
    float4 A[WM], Bv[WN], An[WM], Bn[WN];
    auto load = [&](int q, float4 (&Ar)[WM], float4 (&Br)[WN]) {
      const int kb = 2 * q + lh;
      const int t = kb / CC4;
      const int c4 = kb - t * CC4;
      const int toff = (t < ntaps ? tap_off[t] : 0) + c4 * 4;
#pragma unroll
      for (int m = 0; m < WM; ++m) Ar[m] = *reinterpret_cast<const float4*>(cur + pix_base[m] + toff);
      const float* wk = wch + ((size_t)kb * a.ntp + nt0) * 128 + li * 4;
#pragma unroll
      for (int n = 0; n < WN; ++n) Br[n] = *reinterpret_cast<const float4*>(wk + n * 128);
    };
    load(0, A, Bv);
    for (int q = 0; q < nq; ++q) {
      float4 sv;
      int sd = -1;
      if (has_next && q < nstage) {
        const int e = tid + q * NT;
        if (e < tile_elems) fetch(e, ch + 1, sv, sd);
      }
      if (q + 1 < nq) load(q + 1, An, Bn);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[m].x, Bv[n].x, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[m].y, Bv[n].y, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[m].z, Bv[n].z, acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[m].w, Bv[n].w, acc[m][n], 0, 0, 0);
      if (sd >= 0) *reinterpret_cast<float4*>(nxt + sd) = fvc_in_op_sel4(sv, a.in_op);
#pragma unroll
      for (int m = 0; m < WM; ++m) A[m] = An[m];
#pragma unroll
      for (int n = 0; n < WN; ++n) Bv[n] = Bn[n];
    }
    if (has_next) {
      for (int q = nq; q < nstage; ++q) {
        const int e = tid + q * NT;
        if (e < tile_elems) {
          float4 v;
          int d;
          fetch(e, ch + 1, v, d);
          *reinterpret_cast<float4*>(nxt + d) = fvc_in_op_sel4(v, a.in_op);
        }
      }
    }
    __syncthreads();
  }

  const int oy0 = a.oy0[cls], ox0 = a.ox0[cls];
#pragma unroll
  for (int n = 0; n < WN; ++n) {
    const int j = (nt0 + n) * 32 + li;
    if (j >= a.coutp) continue;
    const bool real = j < a.cout;
    const float bj = real ? a.bias[j] : 0.f;
#pragma unroll
    for (int m = 0; m < WM; ++m) {
      const int qy = qy0 + wave * WM + m;
      if (qy >= a.Hq) continue;
      const int oy = qy * a.sout + oy0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qx = qx0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (qx >= a.Wq) continue;
        const int ox = qx * a.sout + ox0;
        const size_t o = (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.coutp + j;
        float v = acc[m][n][r] + bj;
        if (a.act == FVC_ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (a.act == FVC_ACT_LRELU) v = v > 0.f ? v : 0.1f * v;
        if (a.res) v += a.res[o];
        if (a.post_op == FVC_POST_EXP) v = expf(v);
        a.y[o] = real ? v : 0.f;
      }
    }
  }
}

// Stride-2 transposed conv with all four output-parity classes in one block: the four
// classes read the same input window, so the halo tile of a channel chunk is staged once and
// consumed by 1+2+2+4 (k=3) or 4+6+6+9 (k=5) taps instead of being re-staged per class.
// acc[class][WM][WN] stays in registers (WM=1: 4 waves x one 32-pixel strip each).
template <int CC, int WN>
__global__ __launch_bounds__(kThreads) void deconv2_mfma_f32_kernel(const ConvArgs a) {
  using G = ChunkGeom<CC>;
  constexpr int CC4 = G::CC4;
  constexpr int CS = G::CS;
  constexpr int TH = 4;
  constexpr int TW = 32;
  constexpr int NCL = 4;
  constexpr int MAXT = 16;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  int* tap_off = reinterpret_cast<int*>(smem);  // [NCL][MAXT]
  float* tile = smem + NCL * MAXT;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int b = blockIdx.z;
  const int tiles_x = (a.Wq + TW - 1) / TW;
  const int qy0 = (blockIdx.x / tiles_x) * TH;
  const int qx0 = (blockIdx.x % tiles_x) * TW;
  const int nt0 = blockIdx.y * WN;

  if (tid < NCL * MAXT) {
    const int cl = tid / MAXT, t = tid % MAXT;
    tap_off[tid] = t < a.ntaps[cl] ? ((a.tdy[cl][t] - a.dymin) * a.ic + (a.tdx[cl][t] - a.dxmin)) * CS : 0;
  }

  f32x16 acc[NCL][WN];
#pragma unroll
  for (int cl = 0; cl < NCL; ++cl)
#pragma unroll
    for (int n = 0; n < WN; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[cl][n][r] = 0.f;

  const int iy0 = qy0 + a.dymin;
  const int ix0 = qx0 + a.dxmin;
  const int tile_elems = a.ir * a.ic * CC4;
  const float* xb = a.x + (size_t)b * a.H * a.W * a.cinp;
  const int pix_base = (wave * a.ic + li) * CS;

  for (int ch = 0; ch < a.nchunks; ++ch) {
    for (int e = tid; e < tile_elems; e += kThreads) {
      const int c4 = e % CC4;
      const int p = e / CC4;
      const int r = p / a.ic;
      const int c = p - r * a.ic;
      const int iy = iy0 + r;
      const int ix = ix0 + c;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
        v = *reinterpret_cast<const float4*>(xb + ((size_t)iy * a.W + ix) * a.cinp + ch * CC + c4 * 4);
        v = fvc_in_op_sel4(v, a.in_op);
      }
      *reinterpret_cast<float4*>(tile + p * CS + c4 * 4) = v;
    }
    __syncthreads();
#pragma unroll
    for (int cl = 0; cl < NCL; ++cl) {
      const int kbc = a.kbc[cl];
      const int ntaps = a.ntaps[cl];
      const int nq = kbc >> 1;
      const float* wch = a.w + a.wcls[cl] + (size_t)ch * kbc * a.ntp * 128;
      const int* toffs = tap_off + cl * MAXT;
      float4 A, An, Bv[WN], Bn[WN];
      auto load = [&](int q, float4& Ar, float4 (&Br)[WN]) {
        const int kb = 2 * q + lh;
        const int t = kb / CC4;
        const int c4 = kb - t * CC4;
        const int toff = (t < ntaps ? toffs[t] : 0) + c4 * 4;
        Ar = *reinterpret_cast<const float4*>(tile + pix_base + toff);
        const float* wk = wch + ((size_t)kb * a.ntp + nt0) * 128 + li * 4;
#pragma unroll
        for (int n = 0; n < WN; ++n) Br[n] = *reinterpret_cast<const float4*>(wk + n * 128);
      };
      load(0, A, Bv);
      for (int q = 0; q < nq; ++q) {
        if (q + 1 < nq) load(q + 1, An, Bn);
#pragma unroll
        for (int n = 0; n < WN; ++n) {
          acc[cl][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A.x, Bv[n].x, acc[cl][n], 0, 0, 0);
          acc[cl][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A.y, Bv[n].y, acc[cl][n], 0, 0, 0);
          acc[cl][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A.z, Bv[n].z, acc[cl][n], 0, 0, 0);
          acc[cl][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(A.w, Bv[n].w, acc[cl][n], 0, 0, 0);
        }
        A = An;
#pragma unroll
        for (int n = 0; n < WN; ++n) Bv[n] = Bn[n];
      }
    }
    __syncthreads();
  }

  const int qy = qy0 + wave;
  if (qy >= a.Hq) return;
#pragma unroll
  for (int cl = 0; cl < NCL; ++cl) {
    const int oy = qy * 2 + a.oy0[cl];
#pragma unroll
    for (int n = 0; n < WN; ++n) {
      const int j = (nt0 + n) * 32 + li;
      if (j >= a.coutp) continue;
      const bool real = j < a.cout;
      const float bj = real ? a.bias[j] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qx = qx0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (qx >= a.Wq) continue;
        const int ox = qx * 2 + a.ox0[cl];
        const size_t o = (((size_t)b * a.Ho + oy) * a.Wo + ox) * a.coutp + j;
        float v = acc[cl][n][r] + bj;
        if (a.act == FVC_ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (a.act == FVC_ACT_LRELU) v = v > 0.f ? v : 0.1f * v;
        if (a.res) v += a.res[o];
        if (a.post_op == FVC_POST_EXP) v = expf(v);
        a.y[o] = real ? v : 0.f;
      }
    }
  }
}

// Small-N variant (cout <= 4: SpyNet conv5, Warp_net conv6, mvDecoder conv8, resDecoder deconv4;
// stride-1 input steps, i.e. stride-1 convs and the parity classes of transposed convs). Padding
// N to an MFMA tile would waste 8-16x of the matrix work, so this path is VALU. Each lane owns a
// column of PY output rows; a class's taps form a contiguous ny x nx grid of input offsets, so
// for every tap column dx the lane loads the PY + KMAX - 1 input pixels of its column once from
// the LDS halo tile and reuses each for all tap rows and output rows. The chunk's weights sit in
// LDS as [KMAX][nx][CC][COUT] (rows past ny zero-filled, so the unrolled tap loop has no branches)
// and are read as wave-uniform broadcasts. The next chunk's halo is prefetched into registers
// while the current one is multiplied.
// Block tile = 8 lane-rows x PY rows x 32 columns. Wide inputs use CC = 32 channels per chunk
// (a pixel's chunk is one full 128-B line, so no line is fetched once per 8-channel slice) with
// PY = 2 to keep the halo tile in LDS; narrow inputs use PY = 4.
template <int CC, int COUT, int KMAX, int PY>
__global__ __launch_bounds__(kThreads) void conv_smalln_f32_kernel(const ConvArgs a) {
  using G = ChunkGeom<CC>;
  constexpr int CC4 = G::CC4;
  constexpr int CS = G::CS;
  constexpr int TW = 32;
  constexpr int TH = (kThreads / TW) * PY;
  constexpr int NV = PY + KMAX - 1;
  constexpr int NPF = ((TH + KMAX - 1) * (TW + KMAX - 1) * CC4 + kThreads - 1) / kThreads;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nx = a.gnx[blockIdx.z % a.nclass];
  float* const wl = smem;                                          // [KMAX][nx][CC][COUT]
  float* const tile = smem + ((KMAX * nx * CC * COUT + 3) & ~3);   // + KMAX-1 spare rows

  const int tid = threadIdx.x;
  const int tx = tid & (TW - 1);
  const int ty = tid / TW;
  const int cls = blockIdx.z % a.nclass;
  const int b = blockIdx.z / a.nclass;
  const int tiles_x = (a.Wq + TW - 1) / TW;
  const int qy0 = (blockIdx.x / tiles_x) * TH;
  const int qx0 = (blockIdx.x % tiles_x) * TW;
  const int ny = a.gny[cls];
  const int coutp = a.coutp;

  float acc[PY][COUT];
#pragma unroll
  for (int k = 0; k < PY; ++k)
#pragma unroll
    for (int j = 0; j < COUT; ++j) acc[k][j] = 0.f;

  const int iy0 = qy0 + a.dymin;
  const int ix0 = qx0 + a.dxmin;
  const int tile_elems = a.ir * a.ic * CC4;
  const float* xb = a.x + (size_t)b * a.H * a.W * a.cinp;
  // LDS base of this lane's column at the class grid origin
  const int col0 = ((ty * PY + a.gy0[cls] - a.dymin) * a.ic + tx + a.gx0[cls] - a.dxmin) * CS;
  const int row_step = a.ic * CS;
  const float* __restrict__ wcls = a.w + a.wcls[cls];
  const int wl_n = KMAX * nx * CC * COUT;

  float4 pf[NPF];
  auto fetch = [&](int ch) {
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int e = tid + k * kThreads;
      pf[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < tile_elems) {
        const int c4 = e % CC4;
        const int p = e / CC4;
        const int r = p / a.ic;
        const int c = p - r * a.ic;
        const int iy = iy0 + r;
        const int ix = ix0 + c;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          pf[k] = *reinterpret_cast<const float4*>(xb + ((size_t)iy * a.W + ix) * a.cinp + ch * CC + c4 * 4);
      }
    }
  };
  auto put = [&](int ch) {
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const int e = tid + k * kThreads;
      if (e < tile_elems) {
        const int c4 = e % CC4;
        const int p = e / CC4;
        *reinterpret_cast<float4*>(tile + p * CS + c4 * 4) = fvc_in_op_sel4(pf[k], a.in_op);
      }
    }
    // weights of this chunk: pack [dy][dx][cin][coutp] -> LDS [KMAX][nx][CC][COUT], zero rows past ny
    const float* wch = wcls + (size_t)ch * ny * nx * CC * coutp;
    for (int e = tid; e < wl_n; e += kThreads) {
      const int j = e % COUT;
      const int r = e / COUT;  // (dy * nx + dx) * CC + c
      wl[e] = r < ny * nx * CC ? wch[(size_t)r * coutp + j] : 0.f;
    }
  };

  // spare rows below the halo tile: read (times zero weights) by the branch-free tap loop, so
  // they must hold finite values
  for (int e = tile_elems * 4 + tid; e < (a.ir + KMAX - 1) * a.ic * CS; e += kThreads) tile[e] = 0.f;
  fetch(0);
  for (int ch = 0; ch < a.nchunks; ++ch) {
    put(ch);
    __syncthreads();
    if (ch + 1 < a.nchunks) fetch(ch + 1);
    for (int dxi = 0; dxi < nx; ++dxi) {
      const float* colp = tile + col0 + dxi * CS;
#pragma unroll
      for (int c4 = 0; c4 < CC4; ++c4) {
        float4 v[NV];
#pragma unroll
        for (int r = 0; r < NV; ++r) v[r] = *reinterpret_cast<const float4*>(colp + r * row_step + c4 * 4);
#pragma unroll
        for (int dyi = 0; dyi < KMAX; ++dyi) {
          const float* wt = wl + ((dyi * nx + dxi) * CC + c4 * 4) * COUT;
          float wv[4 * COUT];
#pragma unroll
          for (int u = 0; u < 4 * COUT; ++u) wv[u] = wt[u];
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int k = 0; k < PY; ++k) {
              const float4 xv = v[k + dyi];
              const float xs = e == 0 ? xv.x : (e == 1 ? xv.y : (e == 2 ? xv.z : xv.w));
              if constexpr (COUT % 2 == 0) {
                // channel pairs as one packed FMA (v_pk_fma_f32): the same fp32 fma per channel
#pragma unroll
                for (int j = 0; j < COUT; j += 2) {
                  const f2v xx = {xs, xs};
                  const f2v ww = {wv[e * COUT + j], wv[e * COUT + j + 1]};
                  const f2v aa = {acc[k][j], acc[k][j + 1]};
                  const f2v rr = __builtin_elementwise_fma(xx, ww, aa);
                  acc[k][j] = rr[0];
                  acc[k][j + 1] = rr[1];
                }
              } else {
#pragma unroll
                for (int j = 0; j < COUT; ++j) acc[k][j] = __builtin_fmaf(xs, wv[e * COUT + j], acc[k][j]);
              }
            }
        }
      }
    }
    __syncthreads();
  }

  const int qx = qx0 + tx;
  if (qx >= a.Wq) return;
  const int ox = qx * a.sout + a.ox0[cls];
#pragma unroll
  for (int k = 0; k < PY; ++k) {
    const int qy = qy0 + ty * PY + k;
    if (qy >= a.Hq) continue;
    const int oy = qy * a.sout + a.oy0[cls];
    const size_t o = (((size_t)b * a.Ho + oy) * a.Wo + ox) * coutp;
    float r4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = j < COUT ? acc[k][j < COUT ? j : 0] + a.bias[j] : 0.f;
      if (j < COUT) {
        if (a.act == FVC_ACT_RELU) v = v > 0.f ? v : 0.f;
        else if (a.act == FVC_ACT_LRELU) v = v > 0.f ? v : 0.1f * v;
        if (a.res) v += a.res[o + j];
        if (a.post_op == FVC_POST_EXP) v = expf(v);
      }
      r4[j] = v;
    }
    *reinterpret_cast<float4*>(a.y + o) = make_float4(r4[0], r4[1], r4[2], r4[3]);
  }
}

// ------------------------------------------------------------------ host-side geometry
struct Cfg {
  int cinp, coutp, ntp, cc, wm, wn, nclass, nchunks, smalln, sn_py, fused, th, pipe, nw, lds_bufs;
  int sin, sout;
  int ntaps[4], kbc[4], oy0[4], ox0[4];
  int tky[4][kMaxTaps], tkx[4][kMaxTaps];  // kernel tap (ky,kx)
  int tdy[4][kMaxTaps], tdx[4][kMaxTaps];  // input offsets
  int dymin, dymax, dxmin, dxmax;
  int gy0[4], gny[4], gx0[4], gnx[4];
  long long wcls[4];
  long long wtotal;
};

static int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

static bool make_cfg(int cin, int cout, int ks, int stride, int transposed, Cfg& c) {
  if (cin <= 0 || cout <= 0 || (ks != 1 && ks != 3 && ks != 5 && ks != 7) || (stride != 1 && stride != 2))
    return false;
  c.cinp = fvc_rup(cin, 4);
  c.coutp = fvc_rup(cout, 4);
  c.ntp = fvc_cdiv(c.coutp, 32);
  if (c.ntp > 4) return false;
  const int pad = ks / 2;
  if (!transposed) {
    c.nclass = 1;
    c.sin = stride;
    c.sout = 1;
    c.ntaps[0] = 0;
    for (int ky = 0; ky < ks; ++ky)
      for (int kx = 0; kx < ks; ++kx) {
        int t = c.ntaps[0]++;
        c.tky[0][t] = ky; c.tkx[0][t] = kx;
        c.tdy[0][t] = ky - pad; c.tdx[0][t] = kx - pad;
      }
    c.oy0[0] = c.ox0[0] = 0;
  } else {
    c.nclass = stride * stride;
    c.sin = 1;
    c.sout = stride;
    for (int py = 0; py < stride; ++py)
      for (int px = 0; px < stride; ++px) {
        const int cl = py * stride + px;
        c.ntaps[cl] = 0;
        c.oy0[cl] = py; c.ox0[cl] = px;
        for (int ky = 0; ky < ks; ++ky) {
          if (((py + pad - ky) % stride + stride) % stride) continue;
          for (int kx = 0; kx < ks; ++kx) {
            if (((px + pad - kx) % stride + stride) % stride) continue;
            int t = c.ntaps[cl]++;
            c.tky[cl][t] = ky; c.tkx[cl][t] = kx;
            c.tdy[cl][t] = floordiv(py + pad - ky, stride);
            c.tdx[cl][t] = floordiv(px + pad - kx, stride);
          }
        }
      }
  }
  c.dymin = c.dxmin = 1 << 20;
  c.dymax = c.dxmax = -(1 << 20);
  for (int cl = 0; cl < c.nclass; ++cl)
    for (int t = 0; t < c.ntaps[cl]; ++t) {
      c.dymin = c.tdy[cl][t] < c.dymin ? c.tdy[cl][t] : c.dymin;
      c.dymax = c.tdy[cl][t] > c.dymax ? c.tdy[cl][t] : c.dymax;
      c.dxmin = c.tdx[cl][t] < c.dxmin ? c.tdx[cl][t] : c.dxmin;
      c.dxmax = c.tdx[cl][t] > c.dxmax ? c.tdx[cl][t] : c.dxmax;
    }
  for (int cl = 0; cl < c.nclass; ++cl) {
    int y0 = 1 << 20, y1 = -(1 << 20), x0 = 1 << 20, x1 = -(1 << 20);
    for (int t = 0; t < c.ntaps[cl]; ++t) {
      y0 = c.tdy[cl][t] < y0 ? c.tdy[cl][t] : y0;
      y1 = c.tdy[cl][t] > y1 ? c.tdy[cl][t] : y1;
      x0 = c.tdx[cl][t] < x0 ? c.tdx[cl][t] : x0;
      x1 = c.tdx[cl][t] > x1 ? c.tdx[cl][t] : x1;
    }
    c.gy0[cl] = y0; c.gny[cl] = y1 - y0 + 1;
    c.gx0[cl] = x0; c.gnx[cl] = x1 - x0 + 1;
    if (c.gny[cl] * c.gnx[cl] != c.ntaps[cl]) return false;  // taps always form a full grid
  }
  c.wn = c.ntp;
  // cout 2/3: MFMA N-tile padding would waste 8-16x -> VALU kernel (stride-1 input steps only)
  c.smalln = (c.coutp <= 4 && c.sin == 1) ? 1 : 0;
  c.fused = (transposed && stride == 2 && !c.smalln && c.cinp % 8 == 0 && ks <= 5) ? 1 : 0;
  {
    // measured: the per-class launch with WN<=2 beats the 4-class fused block (register-bound
    // at 1 wave/SIMD); keep the fused kernel behind FVC_DECONV_FUSED=1 for experiments.
    const char* f = getenv("FVC_DECONV_FUSED");
    c.fused = (f && f[0] == '1') ? c.fused : 0;
  }
  c.wm = ((!transposed && stride == 2) || c.fused) ? 1 : 2;
  {
    const char* w4 = getenv("FVC_CONV_WM4");
    if (w4 && w4[0] == '1' && !transposed && stride == 1 && ks == 3 && c.ntp <= 2) c.wm = 4;
  }
  if (c.fused) c.wn = (c.ntp % 2 == 0) ? 2 : 1;
  // channel chunk: largest of {32,16,8,4} dividing cinp whose LDS footprint fits 64 KB
  int maxt = 0;
  for (int cl = 0; cl < c.nclass; ++cl) maxt = c.ntaps[cl] > maxt ? c.ntaps[cl] : maxt;
  // pipelined (double-buffered) path for stride-1 convs with >= 2 channel chunks
  // measured (scripts/conv_micro.py, MI355X): 3x3 128->128 gains +31 % from the 8-wave
  // pipelined kernel; 3x3 64->64 and the 7x7 layers are faster on the 4-wave single-buffer one.
  c.pipe = (!transposed && stride == 1 && !c.smalln && c.cinp >= 128 && ks <= 3) ? 1 : 0;
  c.nw = 8;
  {
    const char* v = getenv("FVC_CONV_PIPE");
    if (v && v[0] == '0') c.pipe = 0;
    const char* v7 = getenv("FVC_CONV_PIPE7");
    if (v7 && v7[0] == '1' && !transposed && stride == 1 && !c.smalln && c.cinp >= 32) c.pipe = 1;
    const char* w = getenv("FVC_CONV_NW");
    if (c.pipe && w && w[0] == '4') c.nw = 4;
    const char* p1 = getenv("FVC_CONV_PIPE");
    if (p1 && p1[0] == '1' && !transposed && stride == 1 && !c.smalln && c.cinp >= 32 && ks <= 3) c.pipe = 1;
    const char* wn2 = getenv("FVC_CONV_WN2");
    if (wn2 && wn2[0] == '1' && !c.pipe && !c.smalln && !c.fused && c.ntp == 4) c.wn = 2;
    const char* wn1 = getenv("FVC_CONV_WN1");
    if (wn1 && wn1[0] == '1' && !c.smalln) c.wn = 1;
  }
  c.lds_bufs = c.pipe ? 2 : 1;
  c.sn_py = (c.smalln && c.cinp % 32 == 0) ? 2 : 4;
  c.th = c.smalln ? (kThreads / 32) * c.sn_py : (c.pipe ? c.nw * c.wm : 4 * c.wm);
  int cc = 32;
  for (;; cc >>= 1) {
    if (cc == 4) break;
    if (c.cinp % cc) continue;
    const int ir = (c.th - 1) * c.sin + 1 + (c.dymax - c.dymin);
    const int ic = 31 * c.sin + 1 + (c.dxmax - c.dxmin);
    const int cs = ((cc / 4) % 2 == 1) ? cc : cc + 4;
    size_t wbytes = 0;
    if (c.smalln) {
      int kmx = 0, nxm = 0;
      for (int cl = 0; cl < c.nclass; ++cl) {
        kmx = c.gny[cl] > kmx ? c.gny[cl] : kmx;
        nxm = c.gnx[cl] > nxm ? c.gnx[cl] : nxm;
      }
      const int kt = kmx <= 3 ? 3 : (kmx <= 5 ? 5 : 7);
      wbytes = (size_t)((kt * nxm * cc * 4 + 3) & ~3) * 4 + (size_t)(kt - 1) * ic * cs * 4;
    }
    const size_t budget = (c.pipe && c.nw == 8) ? 100 * 1024 : (c.smalln && c.sn_py == 2 ? 112 * 1024 : 64 * 1024);
    if ((size_t)c.lds_bufs * (((size_t)ir * ic * cs + 3) & ~(size_t)3) * 4 + 256 + wbytes <= budget) break;
  }
  {
    const char* vcc = getenv("FVC_CONV_CC");  // experiment override (must stay fixed per process)
    if (vcc && !c.smalln && !c.fused) {
      const int want = atoi(vcc);
      if ((want == 8 || want == 16 || want == 32) && c.cinp % want == 0) cc = want;
    }
  }
  c.cc = cc;
  c.nchunks = c.cinp / cc;
  long long off = 0;
  for (int cl = 0; cl < c.nclass; ++cl) {
    c.kbc[cl] = fvc_rup(c.ntaps[cl] * (cc / 4), 2);
    c.wcls[cl] = off;
    if (c.smalln)  // [chunk][dy][dx][cin in chunk][coutp] (tap grid order)
      off += (long long)c.nchunks * c.ntaps[cl] * cc * c.coutp;
    else           // [chunk][k-block][n-tile][32][4]
      off += (long long)c.nchunks * c.kbc[cl] * c.ntp * 128;
  }
  c.wtotal = off;
  return true;
}

static int g_bpf = -1;

template <int CC, int WM, int WN>
static int launch_t(const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  if (g_bpf < 0) {
    const char* v = getenv("FVC_CONV_BPF");
    g_bpf = (v && v[0] == '2') ? 2 : 1;  // measured: 2-deep weight prefetch is 2-4 % slower
  }
  if (g_bpf == 2)
    hipLaunchKernelGGL((conv_mfma_f32_kernel<CC, WM, WN, 2>), grid, dim3(kThreads), lds, s, a);
  else
    hipLaunchKernelGGL((conv_mfma_f32_kernel<CC, WM, WN, 1>), grid, dim3(kThreads), lds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

template <int CC, int WM>
static int launch_wn(int wn, const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  switch (wn) {
    case 1: return launch_t<CC, WM, 1>(a, grid, lds, s);
    case 2: return launch_t<CC, WM, 2>(a, grid, lds, s);
    case 3: return launch_t<CC, WM, 3>(a, grid, lds, s);
    case 4: return launch_t<CC, WM, 4>(a, grid, lds, s);
  }
  return FVC_EINVAL;
}

template <int CC>
static int launch_wm(int wm, int wn, const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  if (wm == 1) return launch_wn<CC, 1>(wn, a, grid, lds, s);
  if (wm == 4) {
    if (wn == 1) return launch_t<CC, 4, 1>(a, grid, lds, s);
    if (wn == 2) return launch_t<CC, 4, 2>(a, grid, lds, s);
    return FVC_EINVAL;
  }
  return launch_wn<CC, 2>(wn, a, grid, lds, s);
}

template <int CC, int COUT, int KMAX>
static int launch_sn_t(int py, const ConvArgs& a, dim3 grid, dim3 blk, size_t lds, hipStream_t s) {
  if (py == 2) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)conv_smalln_f32_kernel<CC, COUT, KMAX, 2>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((conv_smalln_f32_kernel<CC, COUT, KMAX, 2>), grid, blk, lds, s, a);
  } else {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)conv_smalln_f32_kernel<CC, COUT, KMAX, 4>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((conv_smalln_f32_kernel<CC, COUT, KMAX, 4>), grid, blk, lds, s, a);
  }
  FVC_CHECK_LAUNCH();
  return 0;
}

template <int CC, int COUT>
static int launch_sn_k(int kmax, int py, const ConvArgs& a, dim3 grid, dim3 blk, size_t lds, hipStream_t s) {
  if (kmax <= 3) return launch_sn_t<CC, COUT, 3>(py, a, grid, blk, lds, s);
  if (kmax <= 5) return launch_sn_t<CC, COUT, 5>(py, a, grid, blk, lds, s);
  return launch_sn_t<CC, COUT, 7>(py, a, grid, blk, lds, s);
}

template <int CC>
static int launch_sn_n(int cout, int kmax, int py, const ConvArgs& a, dim3 grid, dim3 blk, size_t lds,
                       hipStream_t s) {
  switch (cout) {
    case 1: return launch_sn_k<CC, 1>(kmax, py, a, grid, blk, lds, s);
    case 2: return launch_sn_k<CC, 2>(kmax, py, a, grid, blk, lds, s);
    case 3: return launch_sn_k<CC, 3>(kmax, py, a, grid, blk, lds, s);
    case 4: return launch_sn_k<CC, 4>(kmax, py, a, grid, blk, lds, s);
  }
  return FVC_EINVAL;
}

template <int CC, int WN, int NW>
static int launch_pp_t(const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)conv_mfma_pipe_kernel<CC, 2, WN, NW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((conv_mfma_pipe_kernel<CC, 2, WN, NW>), grid, dim3(NW * 64), lds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

template <int CC, int NW>
static int launch_pp_wn(int wn, const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  switch (wn) {
    case 1: return launch_pp_t<CC, 1, NW>(a, grid, lds, s);
    case 2: return launch_pp_t<CC, 2, NW>(a, grid, lds, s);
    case 3: return launch_pp_t<CC, 3, NW>(a, grid, lds, s);
    case 4: return launch_pp_t<CC, 4, NW>(a, grid, lds, s);
  }
  return FVC_EINVAL;
}

static int launch_pipe(int cc, int wn, int nw, const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  if (nw == 8) {
    switch (cc) {
      case 8: return launch_pp_wn<8, 8>(wn, a, grid, lds, s);
      case 16: return launch_pp_wn<16, 8>(wn, a, grid, lds, s);
      case 32: return launch_pp_wn<32, 8>(wn, a, grid, lds, s);
    }
  } else {
    switch (cc) {
      case 8: return launch_pp_wn<8, 4>(wn, a, grid, lds, s);
      case 16: return launch_pp_wn<16, 4>(wn, a, grid, lds, s);
      case 32: return launch_pp_wn<32, 4>(wn, a, grid, lds, s);
    }
  }
  return FVC_EINVAL;
}

template <int CC, int WN>
static int launch_fd_t(const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((deconv2_mfma_f32_kernel<CC, WN>), grid, dim3(kThreads), lds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

static int launch_fused(int cc, int wn, const ConvArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  if (wn == 1) {
    switch (cc) {
      case 8: return launch_fd_t<8, 1>(a, grid, lds, s);
      case 16: return launch_fd_t<16, 1>(a, grid, lds, s);
      case 32: return launch_fd_t<32, 1>(a, grid, lds, s);
    }
  } else {
    switch (cc) {
      case 8: return launch_fd_t<8, 2>(a, grid, lds, s);
      case 16: return launch_fd_t<16, 2>(a, grid, lds, s);
      case 32: return launch_fd_t<32, 2>(a, grid, lds, s);
    }
  }
  return FVC_EINVAL;
}

static int launch_smalln(int cc, int cout, int kmax, int py, const ConvArgs& a, dim3 grid, dim3 blk, size_t lds,
                         hipStream_t s) {
  switch (cc) {
    case 4: return launch_sn_n<4>(cout, kmax, py, a, grid, blk, lds, s);
    case 8: return launch_sn_n<8>(cout, kmax, py, a, grid, blk, lds, s);
    case 16: return launch_sn_n<16>(cout, kmax, py, a, grid, blk, lds, s);
    case 32: return launch_sn_n<32>(cout, kmax, py, a, grid, blk, lds, s);
  }
  return FVC_EINVAL;
}

static int run_conv(const float* x, const float* wpack, const float* bias, const float* res,
                    float* y, int batch, int h, int w, int cin, int cout, int ks, int stride,
                    int transposed, int in_op, int act, int post_op, hipStream_t s) {
  Cfg c;
  if (!make_cfg(cin, cout, ks, stride, transposed, c)) return FVC_EINVAL;
  if (!x || !wpack || !bias || !y || batch <= 0 || h <= 0 || w <= 0) return FVC_EINVAL;
  ConvArgs a;
  a.x = x; a.w = wpack; a.bias = bias; a.res = res; a.y = y;
  a.B = batch; a.H = h; a.W = w; a.cinp = c.cinp;
  a.coutp = c.coutp; a.cout = cout;
  if (!transposed) {
    if (stride == 2 && ((h & 1) || (w & 1))) return FVC_EINVAL;
    a.Ho = h / stride; a.Wo = w / stride;
    a.Hq = a.Ho; a.Wq = a.Wo;
  } else {
    a.Ho = h * stride; a.Wo = w * stride;
    a.Hq = h; a.Wq = w;
  }
  a.sin = c.sin; a.sout = c.sout; a.nclass = c.nclass; a.nchunks = c.nchunks; a.ntp = c.ntp;
  a.dymin = c.dymin; a.dxmin = c.dxmin;
  const int TH = c.th;
  a.ir = (TH - 1) * c.sin + 1 + (c.dymax - c.dymin);
  a.ic = 31 * c.sin + 1 + (c.dxmax - c.dxmin);
  a.in_op = in_op; a.act = act; a.post_op = post_op;
  for (int cl = 0; cl < 4; ++cl) {
    a.kbc[cl] = cl < c.nclass ? c.kbc[cl] : 0;
    a.ntaps[cl] = cl < c.nclass ? c.ntaps[cl] : 0;
    a.oy0[cl] = cl < c.nclass ? c.oy0[cl] : 0;
    a.ox0[cl] = cl < c.nclass ? c.ox0[cl] : 0;
    a.wcls[cl] = cl < c.nclass ? c.wcls[cl] : 0;
    a.gy0[cl] = cl < c.nclass ? c.gy0[cl] : 0;
    a.gny[cl] = cl < c.nclass ? c.gny[cl] : 0;
    a.gx0[cl] = cl < c.nclass ? c.gx0[cl] : 0;
    a.gnx[cl] = cl < c.nclass ? c.gnx[cl] : 0;
    for (int t = 0; t < kMaxTaps; ++t) {
      const bool v = cl < c.nclass && t < c.ntaps[cl];
      a.tdy[cl][t] = (short)(v ? c.tdy[cl][t] : 0);
      a.tdx[cl][t] = (short)(v ? c.tdx[cl][t] : 0);
    }
  }
  const int cs = ((c.cc / 4) % 2 == 1) ? c.cc : c.cc + 4;
  int maxt = 0;
  for (int cl = 0; cl < c.nclass; ++cl) maxt = c.ntaps[cl] > maxt ? c.ntaps[cl] : maxt;
  int kmx = 0, nxm = 0;
  for (int cl = 0; cl < c.nclass; ++cl) {
    kmx = c.gny[cl] > kmx ? c.gny[cl] : kmx;
    nxm = c.gnx[cl] > nxm ? c.gnx[cl] : nxm;
  }
  const int kmax_t = kmx <= 3 ? 3 : (kmx <= 5 ? 5 : 7);
  const size_t wbytes = c.smalln ? ((size_t)((kmax_t * nxm * c.cc * cout + 3) & ~3) * 4 +
                                    (size_t)(kmax_t - 1) * a.ic * cs * 4)
                                 : 0;
  const size_t lds = 256 + wbytes + (size_t)c.lds_bufs * (((size_t)a.ir * a.ic * cs + 3) & ~(size_t)3) * 4;
  const int tiles_x = fvc_cdiv(a.Wq, 32);
  const int tiles_y = fvc_cdiv(a.Hq, TH);
  // N-split heuristic (measured, scripts/conv_micro.py): fewer N-tiles per block when the grid
  // would not fill the chip, and at most 2 for the per-class transposed launch.
  if (!c.smalln && !c.fused && !getenv("FVC_CONV_WN1") && !getenv("FVC_CONV_WN2")) {
    int wn = c.ntp;
    if (transposed && wn == 4) wn = 2;
    const long long base = (long long)tiles_x * tiles_y * batch * c.nclass;
    const long long want = c.pipe ? 512 : 1024;
    while (wn > 1 && base * (c.ntp / wn) < want) {
      int w2 = wn - 1;
      while (w2 > 1 && c.ntp % w2) --w2;
      wn = w2;
    }
    c.wn = wn;
  }
  if (c.smalln) {
    dim3 grid(tiles_x * tiles_y, 1, batch * c.nclass);
    int kmax = 0;
    for (int cl = 0; cl < c.nclass; ++cl) kmax = c.gny[cl] > kmax ? c.gny[cl] : kmax;
    return launch_smalln(c.cc, cout, kmax, c.sn_py, a, grid, dim3(kThreads), lds, s);
  }
  if (c.fused) {
    dim3 grid(tiles_x * tiles_y, c.ntp / c.wn, batch);
    return launch_fused(c.cc, c.wn, a, grid, lds, s);
  }
  if (c.pipe) {
    dim3 grid(tiles_x * tiles_y, c.ntp / c.wn, batch * c.nclass);
    return launch_pipe(c.cc, c.wn, c.nw, a, grid, lds, s);
  }
  dim3 grid(tiles_x * tiles_y, c.ntp / c.wn, batch * c.nclass);
  switch (c.cc) {
    case 4: return launch_wm<4>(c.wm, c.wn, a, grid, lds, s);
    case 8: return launch_wm<8>(c.wm, c.wn, a, grid, lds, s);
    case 16: return launch_wm<16>(c.wm, c.wn, a, grid, lds, s);
    case 32: return launch_wm<32>(c.wm, c.wn, a, grid, lds, s);
  }
  return FVC_EINVAL;
}

}  // namespace

extern "C" {

size_t fvc_conv_wpack_floats(int cin, int cout, int ksize, int stride, int transposed) {
  Cfg c;
  if (!make_cfg(cin, cout, ksize, stride, transposed, c)) return 0;
  return (size_t)c.wtotal;
}

// w_host: conv OIHW [cout][cin][k][k]; deconv IOHW [cin][cout][k][k]
int fvc_conv_pack_weight(const float* w, float* wp, int cin, int cout, int ks, int stride,
                         int transposed) {
  Cfg c;
  if (!make_cfg(cin, cout, ks, stride, transposed, c) || !w || !wp) return FVC_EINVAL;
  const int cc4 = c.cc / 4;
  for (long long i = 0; i < c.wtotal; ++i) wp[i] = 0.f;
  for (int cl = 0; cl < c.nclass; ++cl)
    for (int ch = 0; ch < c.nchunks; ++ch)
      for (int kb = 0; kb < c.ntaps[cl] * cc4; ++kb) {
        const int t = kb / cc4, c4 = kb % cc4;
        const int ky = c.tky[cl][t], kx = c.tkx[cl][t];
        for (int j = 0; j < cout; ++j)
          for (int e = 0; e < 4; ++e) {
            const int ci = ch * c.cc + c4 * 4 + e;
            if (ci >= cin) continue;
            const float v = transposed ? w[(((size_t)ci * cout + j) * ks + ky) * ks + kx]
                                       : w[(((size_t)j * cin + ci) * ks + ky) * ks + kx];
            size_t o;
            if (c.smalln) {
              const int g = (c.tdy[cl][t] - c.gy0[cl]) * c.gnx[cl] + (c.tdx[cl][t] - c.gx0[cl]);
              o = (size_t)c.wcls[cl] + (((size_t)ch * c.ntaps[cl] + g) * c.cc + c4 * 4 + e) * c.coutp + j;
            }
            else
              o = (size_t)c.wcls[cl] + (((size_t)ch * c.kbc[cl] + kb) * c.ntp * 32 + j) * 4 + e;
            wp[o] = v;
          }
      }
  return 0;
}

int fvc_conv2d_nhwc_f32(const float* x, const float* wpack, const float* bias, const float* res,
                        float* y, int batch, int h, int w, int cin, int cout, int ksize,
                        int stride, int in_op, int act, int post_op, fvc_stream_t stream) {
  return run_conv(x, wpack, bias, res, y, batch, h, w, cin, cout, ksize, stride, 0, in_op, act,
                  post_op, (hipStream_t)stream);
}

int fvc_deconv2d_nhwc_f32(const float* x, const float* wpack, const float* bias,
                          const float* res, float* y, int batch, int h, int w, int cin, int cout,
                          int ksize, int stride, int in_op, int act, int post_op,
                          fvc_stream_t stream) {
  return run_conv(x, wpack, bias, res, y, batch, h, w, cin, cout, ksize, stride, 1, in_op, act,
                  post_op, (hipStream_t)stream);
}

}  // extern "C"
