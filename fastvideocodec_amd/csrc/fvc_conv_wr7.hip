// Winograd-rows F(2,7) split-precision convolution for SpyNet's 7x7 stride-1 layers
// (DVC/subnet/endecoder.py:142-169, MEBasic conv2 32->64, conv3 64->32, conv4 32->16) on the fp16
// matrix cores (v_mfma_f32_16x16x32_f16), at the direct split kernel's accuracy. Replaces the same
// ATen conv2d calls as fvc_conv_x3.hip for those geometries: along each image row the 1-D minimal
// filtering algorithm F(2,7) computes 2 outputs of a 7-tap row filter from 8 products instead of 14,
// and the 7 kernel rows stay a direct sum, so 28 instead of 49 products per output and channel pair
// (1.75x fewer matrix instructions for the same algorithmic work).
//
// Algorithm (Lavin & Gray 2016 / Toom-Cook, interpolation points 0, +-1, +-2, +-1/2 and infinity):
// for a 2-pixel output tile at columns (2t, 2t+1) the 8 input columns x[0..7] = in[2t-3 .. 2t+4] of
// every input row are transformed, V[j] = sum_l B^T[j][l] x[l]; position j is an independent
// 7x1 convolution over (kernel row dy, input channel) with the transformed weights
// U[j][dy] = sum_k G[j][k] w[dy][k]: M[j] = sum_{dy,c} U[j][dy][c] V[j][row + dy][c]; the tile is
// Y[i] = sum_j A^T[i][j] M[j]. B^T pairs the positions: V[1], V[2] = e +- o with e / o the even /
// odd columns (likewise 3/4 and 5/6); V[0] and V[7] are the two 4-tap end rows.
// Accuracy (CPU emulation of this arithmetic, scripts/wino_accuracy.py spynet, seeded SpyNet L4):
// max error 4.4e-7 / 5.3e-7 of output scale against float64, equal to the direct split kernel's
// 4.5e-7 / 5.4e-7 (the fp32 FMA chain: 1.2e-6 / 1.3e-6); F(4x4,3x3) fails the same gate
// (profiles/r5/wino_accuracy.txt).
//
// Numerics as fvc_conv_x3.hip: U scaled by 2^kw (max |U| in [2^13, 2^14)) and V (fp32, scaled by
// 2^-4 so |V| stays within the fp16 range wherever |x| does: the B^T rows sum to <= 15 in
// absolute value) are split exactly into fp16 hi + lo * 2^-11; main += U_hi V_hi and
// corr += U_lo V_hi + U_hi V_lo in two fp32 accumulators. A transformed value >= 65520 rounds to
// an infinite hi part whose products reach the tile's outputs as inf / NaN; the kernel sums
// 0 * output and raises the caller's overflow flag on a NaN (the host then recomputes the frame on
// the fp32 kernels). NaN inputs raise it as well.
//
// One launch covers 32 input channels (one MFMA K block per kernel row) and 16 * NT <= 32 output
// channels, so that every transformed weight stays in registers: one 256-thread block per CU, one
// wave per SIMD; wave w owns the position pair P(w) = (1,2), (3,4), (5,6), (0,7) for all 7 kernel
// rows (2 x 7 x NT x hi/lo fragments = 224 AGPRs at NT = 2). A 64-channel input runs as two launches
// (the second adds the first's partial sum before bias and activation), 64 output channels as two.
// A work item is a 32-column strip (16 tiles) of up to kRows output rows, walked top to bottom: each
// step transforms ONE new input row into a ring of 8 transformed rows held in VGPRs (2 positions x
// hi/lo per lane, the MFMA B operands), so every transformed row feeds all 7 output rows that use
// it; raw input rows arrive by LDS-DMA into an 8-row ring, one row per step, 5 rows ahead. The
// waves combine their two positions' M into partial outputs, exchange them through LDS (one barrier
// per output row, double-buffered) and wave w finishes one (output column parity, 16-channel tile)
// pair: bias, activation (or the partial-sum forms), 16-B stores.
#include "fvc_common.h"
#include <math.h>
#include <stdlib.h>

#include <type_traits>

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kCi = 32;                         // input channels per launch
constexpr int kQ = kCi / 4;                     // channel quads
constexpr int kSlots = 40;                      // column slots per (row, quad) line: 19 even + 19 odd used
constexpr int kRowEntries = kQ * kSlots;        // 16-B entries per staged row (320 = 5 DMA pieces)
constexpr int kRawRing = 8;                     // staged raw rows
constexpr int kRawBytes = kRawRing * kRowEntries * 16;  // 40,960
constexpr int kZBytes = 4 * 2 * 2 * 64 * 16;            // partial outputs: [wave][i][n][lane] f32x4
constexpr int kHdr = 256;                               // bias (128 B) + work-item word
constexpr int kLds = kHdr + kRawBytes + 2 * kZBytes;    // 73,984
constexpr int kRows = 128;                      // output rows per work item
constexpr float kLoScale = 2048.f;
constexpr unsigned kOob = 0xFFFFFF00u;
constexpr int kRsrcFlags = 0x00020000;
constexpr int kModeFull = 0;     // y = act(conv + bias)
constexpr int kModePartial = 1;  // y = conv (first input-channel half)
constexpr int kModeAdd = 2;      // y = act(conv + bias + y) (second input-channel half)

struct Wr7Args {
  const float* x;    // first input channel of this launch's 32 (pixel pitch xp floats)
  const uint4* u;    // packed U: [wave][pp][dy][n][plane][lane] 16-B fragments
  const float* bias; // this launch's 16 * NT biases (unused in the partial mode)
  float* y;          // first output channel of this launch (pixel pitch yp floats)
  int B, H, W, xp, yp;
  int ngroups, chunks_per_col, nchunks;
  float osc, osc_c;  // 2^(4-kw), 2^(4-kw-11): undo the U and V scales
  int* sched;        // [0] blocks finished, [1] next item: zero on entry, reset by the last block
  int* ovf;
};

typedef __attribute__((address_space(3))) void* lds_ptr;

// raw buffer descriptor over [p, p + bytes): offsets at or past bytes read 0 / drop the store
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  const unsigned long long v = (unsigned long long)(uintptr_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* const q = (void*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), kRsrcFlags);
}

// The three split-precision products of one (position, kernel row, 16-channel tile):
// acc += U_hi V_hi, cor += U_lo V_hi + U_hi V_lo. U is an AGPR operand (hipcc does not place MFMA
// A / B operands in AGPRs, hence asm). Wait states (cdna_hip_programming.md §5.7 item 2): the first
// block of each kernel row opens with s_nop 1 (a VALU-written V or a v_accvgpr_write of U right
// before); accumulate chains need none; wr7_drain fences the VALU readers of acc / cor.
#define WR7_MFMA3_BODY(C0, C1)                     \
  "v_mfma_f32_16x16x32_f16 %0, %2, %4, " C0 "\n\t" \
  "v_mfma_f32_16x16x32_f16 %1, %3, %4, " C1 "\n\t" \
  "v_mfma_f32_16x16x32_f16 %1, %2, %5, %1"
template <bool FIRST, bool NOP>
__device__ __forceinline__ void wr7_mfma3(f32x4& acc, f32x4& cor, const h8& uh, const h8& ul, const h8& vh,
                                          const h8& vl) {
  if constexpr (FIRST) {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\t" WR7_MFMA3_BODY("0", "0") : "=&v"(acc), "=&v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
    else
      asm volatile(WR7_MFMA3_BODY("0", "0") : "=&v"(acc), "=&v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
  } else {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\t" WR7_MFMA3_BODY("%0", "%1") : "+v"(acc), "+v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
    else
      asm volatile(WR7_MFMA3_BODY("%0", "%1") : "+v"(acc), "+v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
  }
}

// y = hi + lo * 2^-11 for two values (fvc_conv_wino.hip's split2: 5 VALU per pair)
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

__device__ __forceinline__ float relu1(float x) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  return r;
}

template <int I>
using ic = std::integral_constant<int, I>;

template <int NT, int MODE, int ACT>
__global__ __launch_bounds__(256, 1) void conv_wr7_kernel(const Wr7Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* const sbias = reinterpret_cast<float*>(smem);
  int* const sitem = reinterpret_cast<int*>(smem + 128);
  char* const raw = smem + kHdr;
  char* const zbuf = raw + kRawBytes;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = lane & 15;  // tile (MFMA B / D column): output columns 2t, 2t + 1 of the strip
  const int o = lane >> 4;  // channel octet of the lane (B operand K rows 8o .. 8o + 7)
  const int W = a.W, H = a.H;

  // resident U: u[pp][dy][n][plane] (AGPRs: the MFMA asm's "a" operands)
  h8 u[2][7][NT][2];
  {
    const uint4* src = a.u + (size_t)wave * (2 * 7 * NT * 2 * 64) + lane;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp)
#pragma unroll
      for (int dy = 0; dy < 7; ++dy)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            u[pp][dy][n][pl] = __builtin_bit_cast(h8, src[(((pp * 7 + dy) * NT + n) * 2 + pl) * 64]);
  }
  if (tid < 16 * NT) sbias[tid] = (MODE != kModePartial && a.bias) ? a.bias[tid] : 0.f;

  // the wave's position pair (a, b) = (1,2), (3,4), (5,6), (0,7): e / o = the even / odd input
  // columns' weighted sums (B^T rows, with the 2^-4 V scale), V_a = e + qa o, V_b = pb e + qb o;
  // its share of the output transform: Y_i += ya_i M_a + yb_i M_b (A^T columns a, b)
  const float s = 1.f / 16.f;
  float E0, E1, E2, E3, O0, O1, O2, O3, qa, pb, qb, ya0, yb0, ya1, yb1;
  if (wave == 0) {
    E0 = 0.f; E1 = s; E2 = -4.25f * s; E3 = s; O0 = s; O1 = -4.25f * s; O2 = s; O3 = 0.f;
    qa = 1.f; pb = 1.f; qb = -1.f; ya0 = 1.f; yb0 = 1.f; ya1 = 1.f; yb1 = -1.f;
  } else if (wave == 1) {
    E0 = 0.f; E1 = 0.25f * s; E2 = -1.25f * s; E3 = s; O0 = 0.5f * s; O1 = -2.5f * s; O2 = 2.f * s; O3 = 0.f;
    qa = 1.f; pb = 1.f; qb = -1.f; ya0 = 1.f; yb0 = 1.f; ya1 = 2.f; yb1 = -2.f;
  } else if (wave == 2) {
    E0 = 0.f; E1 = 4.f * s; E2 = -5.f * s; E3 = s; O0 = 2.f * s; O1 = -2.5f * s; O2 = 0.5f * s; O3 = 0.f;
    qa = 1.f; pb = 1.f; qb = -1.f; ya0 = 1.f; yb0 = 1.f; ya1 = 0.5f; yb1 = -0.5f;
  } else {
    E0 = -s; E1 = 5.25f * s; E2 = -5.25f * s; E3 = s; O0 = -s; O1 = 5.25f * s; O2 = -5.25f * s; O3 = s;
    qa = 0.f; pb = 0.f; qb = 1.f; ya0 = 1.f; yb0 = 0.f; ya1 = 0.f; yb1 = 1.f;
  }

  // DMA pieces of a staged row: piece k of 5 -> wave k & 3 (wave 0 also piece 4); the lane's entry
  // (quad, column slot) -> input column and channel-quad offset. Column slots of a (row, quad) line:
  // even strip columns 0..36 at 0..18, odd 1..37 at 19..37 (a tile's 8 columns are 2t + l)
  int dma_c[2], dma_q[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int e = (wave + 4 * m) * 64 + lane;
    const int q = e / kSlots, cs = e - q * kSlots;
    dma_c[m] = cs < 19 ? 2 * cs : (cs < 38 ? 2 * (cs - 19) + 1 : -(1 << 20));
    dma_q[m] = 4 * q;
  }
  const int npiece = wave == 0 ? 2 : 1;
  const unsigned row_bytes = (unsigned)W * a.xp * 4u;
  const unsigned rowe = (unsigned)W * a.xp;
  unsigned vo[2];
  auto row_offsets = [&](int g) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int ix = 32 * g - 3 + dma_c[m];
      vo[m] = (unsigned)ix < (unsigned)W ? (unsigned)(ix * a.xp + dma_q[m]) * 4u : kOob;
    }
  };
  // raw input row iy of image b into ring slot s (0 bytes for a padding row: the DMA lands zeros)
  auto stage_row = [&](const float* ximg, int iy, int slot) {
    const bool ok = (unsigned)iy < (unsigned)H;
    const __amdgpu_buffer_rsrc_t rx = rsrc(ximg + (size_t)(unsigned)(ok ? iy : 0) * rowe, ok ? row_bytes : 0u);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (m >= npiece) break;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rx, (lds_ptr)(raw + ((size_t)slot * kRowEntries + (wave + 4 * m) * 64) * 16), 16, vo[m], 0, 0, 0);
    }
  };

  // the transformed-row ring (MFMA B operands, 2 positions x hi / lo): slot of input row r =
  // (r - y0 + 3) & 7, the same as its raw slot
  h8 vh[8][2], vl[8][2];
  // transform raw slot RS into V slot RS: lane (t, o), channels 8o .. 8o + 7, positions a, b
  auto transform = [&](auto RS_c) {
    constexpr int RS = decltype(RS_c)::value;
    const char* const row = raw + (size_t)RS * kRowEntries * 16;
    float va[8], vb[8];
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      const char* const line = row + (size_t)(2 * o + hq) * kSlots * 16;
      float4 x[8];
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const int slot = (l & 1) ? 19 + t + (l >> 1) : t + (l >> 1);
        x[l] = *reinterpret_cast<const float4*>(line + slot * 16);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        auto ch = [&](const float4& v) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); };
        const float e = fmaf(E3, ch(x[6]), fmaf(E2, ch(x[4]), fmaf(E1, ch(x[2]), E0 * ch(x[0]))));
        const float od = fmaf(O3, ch(x[7]), fmaf(O2, ch(x[5]), fmaf(O1, ch(x[3]), O0 * ch(x[1]))));
        va[4 * hq + c] = fmaf(qa, od, e);
        vb[4 * hq + c] = fmaf(qb, od, pb * e);
      }
    }
    unsigned hwa[4], lwa[4], hwb[4], lwb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      split2(va[2 * i], va[2 * i + 1], hwa[i], lwa[i]);
      split2(vb[2 * i], vb[2 * i + 1], hwb[i], lwb[i]);
    }
    vh[RS][0] = __builtin_bit_cast(h8, v4u{hwa[0], hwa[1], hwa[2], hwa[3]});
    vl[RS][0] = __builtin_bit_cast(h8, v4u{lwa[0], lwa[1], lwa[2], lwa[3]});
    vh[RS][1] = __builtin_bit_cast(h8, v4u{hwb[0], hwb[1], hwb[2], hwb[3]});
    vl[RS][1] = __builtin_bit_cast(h8, v4u{lwb[0], lwb[1], lwb[2], lwb[3]});
  };
  // pin a transformed slot here in program order (its VALU writes may not sink towards the MFMAs
  // that read it, which carry no wait states of their own past the first block of a kernel row)
  auto pin = [&](auto RS_c) {
    constexpr int RS = decltype(RS_c)::value;
    h8& h0 = vh[RS][0];  // (asm operands do not capture: name the ring slots through references)
    h8& l0 = vl[RS][0];
    h8& h1 = vh[RS][1];
    h8& l1 = vl[RS][1];
    asm volatile("" : "+v"(h0), "+v"(l0), "+v"(h1), "+v"(l1));
  };

  // ---- schedule: items = (image, 32-column group, chunk of kRows output rows), chunk fastest
  int* const ctr = a.sched ? a.sched + 1 : nullptr;
  int k_item = 0;
  float chk = 0.f;
  const unsigned yrow_bytes = (unsigned)W * a.yp * 4u;
  // this lane's finishing share: output column parity fi and 16-channel tile fn (wave w -> (w & 1,
  // w >> 1)); NT = 1 leaves waves 2 and 3 without one
  const int fi = wave & 1, fn = wave >> 1;
  const bool fin = fn < NT;
  int zb = 0;

  for (;;) {
    if (tid == 0) sitem[0] = ctr ? atomicAdd(ctr, 1) : (int)blockIdx.x + k_item * (int)gridDim.x;
    ++k_item;
    __syncthreads();
    const int it = __builtin_amdgcn_readfirstlane(sitem[0]);
    if (it >= a.nchunks) break;
    const int col = it / a.chunks_per_col;
    const int y0 = (it - col * a.chunks_per_col) * kRows;
    const int y1 = min(y0 + kRows, H);
    const int b = col / a.ngroups;
    const int g = col - b * a.ngroups;
    const float* const ximg = a.x + (size_t)b * H * rowe;
    float* const yimg = a.y + (size_t)b * H * W * a.yp;
    row_offsets(g);
    // output byte offset of the finishing lane within an output row (past the row when the pixel
    // is outside the image)
    const int ox = 32 * g + 2 * t + fi;
    const unsigned so = ox < W ? (unsigned)(ox * a.yp + 16 * fn + 4 * o) * 4u : kOob;

    // prologue: raw rows y0-3 .. y0+4 into slots 0..7, then the first 7 transformed rows
#pragma unroll
    for (int i = 0; i < 8; ++i) stage_row(ximg, y0 - 3 + i, i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    transform(ic<0>{}); transform(ic<1>{}); transform(ic<2>{}); transform(ic<3>{});
    transform(ic<4>{}); transform(ic<5>{}); transform(ic<6>{});
    pin(ic<0>{}); pin(ic<1>{}); pin(ic<2>{}); pin(ic<3>{}); pin(ic<4>{}); pin(ic<5>{}); pin(ic<6>{});
    __syncthreads();  // every wave is done with raw slot 0 before step 0 stages into it

    int y = y0;
    // one output row: S = (y - y0) & 7 (compile-time: the loop is unrolled by 8)
    auto step = [&](auto S_c) {
      constexpr int S = decltype(S_c)::value;
      // raw row y + 5 into raw slot S (held row y - 3, transformed 7 steps ago)
      stage_row(ximg, y + 5, S);
      // the previous partial sum (second input-channel half): loaded now, used after the barrier
      const __amdgpu_buffer_rsrc_t ry = rsrc(yimg + (size_t)(unsigned)y * ((unsigned)W * a.yp), yrow_bytes);
      f32x4 rv = {0.f, 0.f, 0.f, 0.f};
      if constexpr (MODE == kModeAdd)
        if (fin) rv = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, so, 0, 0));

      f32x4 acc[2][NT], cor[2][NT];
      auto row_mfmas = [&](auto DY_c) {
        constexpr int DY = decltype(DY_c)::value;
        constexpr int VS = (S + DY) & 7;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            if (pp == 0 && n == 0)
              wr7_mfma3<DY == 0, true>(acc[pp][n], cor[pp][n], u[pp][DY][n][0], u[pp][DY][n][1], vh[VS][pp],
                                       vl[VS][pp]);
            else
              wr7_mfma3<DY == 0, false>(acc[pp][n], cor[pp][n], u[pp][DY][n][0], u[pp][DY][n][1], vh[VS][pp],
                                        vl[VS][pp]);
          }
      };
      row_mfmas(ic<0>{});
      row_mfmas(ic<1>{});
      row_mfmas(ic<2>{});
      // the next step's transformed row y + 4 (raw slot (S + 7) & 7, landed at the last barrier) into
      // V slot (S + 7) & 7, which no kernel row of this step reads
      transform(ic<(S + 7) & 7>{});
      row_mfmas(ic<3>{});
      row_mfmas(ic<4>{});
      row_mfmas(ic<5>{});
      row_mfmas(ic<6>{});
      pin(ic<(S + 7) & 7>{});
      // 12 wait states after the last MFMA before any VALU reads an accumulator
      if constexpr (NT == 2)
        asm volatile("s_nop 11" : "+v"(acc[0][0]), "+v"(acc[0][NT - 1]), "+v"(acc[1][0]), "+v"(acc[1][NT - 1]),
                     "+v"(cor[0][0]), "+v"(cor[0][NT - 1]), "+v"(cor[1][0]), "+v"(cor[1][NT - 1]));
      else
        asm volatile("s_nop 11" : "+v"(acc[0][0]), "+v"(acc[1][0]), "+v"(cor[0][0]), "+v"(cor[1][0]));

      // partial outputs of this wave's two positions -> LDS [wave][i][n][lane]
      char* const zw = zbuf + zb * kZBytes;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        f32x4 p0, p1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ma = fmaf(cor[0][n][r], 1.f / kLoScale, acc[0][n][r]);
          const float mb = fmaf(cor[1][n][r], 1.f / kLoScale, acc[1][n][r]);
          p0[r] = fmaf(yb0, mb, ya0 * ma);
          p1[r] = fmaf(yb1, mb, ya1 * ma);
        }
        *reinterpret_cast<f32x4*>(zw + (((wave * 2 + 0) * 2 + n) * 64 + lane) * 16) = p0;
        *reinterpret_cast<f32x4*>(zw + (((wave * 2 + 1) * 2 + n) * 64 + lane) * 16) = p1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA piece of raw row y + 5
      __syncthreads();
      if (fin) {
        f32x4 sum = *reinterpret_cast<const f32x4*>(zw + (((0 * 2 + fi) * 2 + fn) * 64 + lane) * 16);
#pragma unroll
        for (int w = 1; w < 4; ++w) sum += *reinterpret_cast<const f32x4*>(zw + (((w * 2 + fi) * 2 + fn) * 64 + lane) * 16);
        const f32x4 bj = *reinterpret_cast<const f32x4*>(sbias + 16 * fn + 4 * o);
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          chk = fmaf(sum[r], 0.f, chk);
          float tv = MODE == kModePartial ? sum[r] * a.osc : fmaf(sum[r], a.osc, bj[r]);
          if constexpr (MODE == kModeAdd) tv += rv[r];
          if constexpr (MODE != kModePartial) {
            if constexpr (ACT == FVC_ACT_RELU) tv = relu1(tv);
            if constexpr (ACT == FVC_ACT_LRELU) tv = fmaxf(tv, tv * 0.1f);
          }
          v[r] = tv;
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), ry, so, 0, 0);
      }
      zb ^= 1;
      ++y;
    };
    for (;;) {
      step(ic<0>{}); if (y >= y1) break;
      step(ic<1>{}); if (y >= y1) break;
      step(ic<2>{}); if (y >= y1) break;
      step(ic<3>{}); if (y >= y1) break;
      step(ic<4>{}); if (y >= y1) break;
      step(ic<5>{}); if (y >= y1) break;
      step(ic<6>{}); if (y >= y1) break;
      step(ic<7>{}); if (y >= y1) break;
    }
  }
  if (chk != 0.f && a.ovf) atomicOr(a.ovf, 1);
  if (a.sched && tid == 0) {
    __threadfence();
    if (atomicAdd(a.sched, 1) == (int)gridDim.x - 1) {
      atomicExch(a.sched + 1, 0);
      atomicExch(a.sched, 0);
    }
  }
}

static int wr7_num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

static int env_int(const char* n, int dflt) {
  const char* v = getenv(n);
  return (v && v[0]) ? atoi(v) : dflt;
}

template <int NT, int MODE, int ACT>
static int wr7_launch3(const Wr7Args& a, int grid, hipStream_t s) {
  const hipError_t e = hipFuncSetAttribute((const void*)conv_wr7_kernel<NT, MODE, ACT>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((conv_wr7_kernel<NT, MODE, ACT>), dim3(grid), dim3(256), kLds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

template <int NT, int MODE>
static int wr7_launch2(const Wr7Args& a, int act, int grid, hipStream_t s) {
  if (MODE == kModePartial || act == FVC_ACT_NONE) return wr7_launch3<NT, MODE, FVC_ACT_NONE>(a, grid, s);
  if (act == FVC_ACT_RELU) return wr7_launch3<NT, MODE, FVC_ACT_RELU>(a, grid, s);
  return wr7_launch3<NT, MODE, FVC_ACT_LRELU>(a, grid, s);
}

template <int NT>
static int wr7_launch1(const Wr7Args& a, int mode, int act, int grid, hipStream_t s) {
  if (mode == kModePartial) return wr7_launch2<NT, kModePartial>(a, act, grid, s);
  if (mode == kModeAdd) return wr7_launch2<NT, kModeAdd>(a, act, grid, s);
  return wr7_launch2<NT, kModeFull>(a, act, grid, s);
}

// F(2,7) G (8 x 7) for the points 0, 1, -1, 2, -2, 1/2, -1/2, infinity (exact fractions)
static void wr7_G(double G[8][7]) {
  for (int j = 0; j < 8; ++j)
    for (int k = 0; k < 7; ++k) G[j][k] = 0.0;
  G[0][0] = -1.0;
  for (int k = 0; k < 7; ++k) {
    G[1][k] = -2.0 / 9.0;
    G[2][k] = (k & 1 ? 2.0 : -2.0) / 9.0;
    G[3][k] = ldexp(1.0, k) / 90.0;
    G[4][k] = (k & 1 ? -1.0 : 1.0) * ldexp(1.0, k) / 90.0;
    G[5][k] = ldexp(1.0, 6 - k) / 90.0;
    G[6][k] = (k & 1 ? -1.0 : 1.0) * ldexp(1.0, 6 - k) / 90.0;
  }
  G[7][6] = 1.0;
}

}  // namespace

extern "C" {

int fvc_conv_wr7_supported(int cin, int cout, int ksize, int stride, int transposed) {
  if (ksize != 7 || stride != 1 || transposed) return 0;
  return (cin == 32 || cin == 64) && (cout == 16 || cout == 32 || cout == 64) && !(cin == 64 && cout == 64);
}

size_t fvc_conv_wr7_wpack_bytes(int nt) { return (nt == 1 || nt == 2) ? (size_t)4 * 2 * 7 * nt * 2 * 64 * 16 : 0; }

// w: [cout][cin][7][7] (OIHW fp32). Packs the sub-block of input channels ci0 .. ci0+31 and output
// channels co0 .. co0 + 16 nt - 1: U[j][dy][co][ci] = sum_k G[j][k] w[co][ci][dy][k] in double,
// scaled by 2^kw (max |U| of the block in [2^13, 2^14)), split into fp16 hi / lo * 2^11, laid out
// per wave w (positions (1,2), (3,4), (5,6), (0,7)) as [pp][dy][n][plane][lane][8]: lane l holds
// output channel co0 + 16n + (l & 15), input channels ci0 + 8 (l >> 4) + 0..7 (the MFMA A operand).
// osc_out = 2^(4 - kw): undoes the U scale and the kernel's 2^-4 V scale.
int fvc_conv_wr7_pack_weight(const float* w, int cin, int cout, int ci0, int co0, int nt, void* wp,
                             float* osc_out) {
  if (!w || !wp || !osc_out || (nt != 1 && nt != 2) || ci0 < 0 || ci0 + kCi > cin || co0 < 0 || co0 + 16 * nt > cout)
    return FVC_EINVAL;
  double G[8][7];
  wr7_G(G);
  const int ncol = 16 * nt;
  double* U = (double*)malloc(sizeof(double) * 8 * 7 * ncol * kCi);  // [j][dy][co][ci]
  if (!U) return FVC_EINVAL;
  double mx = 0.0;
  for (int j = 0; j < 8; ++j)
    for (int dy = 0; dy < 7; ++dy)
      for (int co = 0; co < ncol; ++co)
        for (int ci = 0; ci < kCi; ++ci) {
          const float* g = w + (((size_t)(co0 + co) * cin + ci0 + ci) * 7 + dy) * 7;
          double v = 0.0;
          for (int k = 0; k < 7; ++k) v += G[j][k] * (double)g[k];
          U[((size_t)(j * 7 + dy) * ncol + co) * kCi + ci] = v;
          mx = fabs(v) > mx ? fabs(v) : mx;
        }
  int kw = 0;
  if (mx > 0.0 && isfinite(mx)) {
    int e;
    frexp(mx, &e);
    kw = 14 - e;
    kw = kw < -100 ? -100 : (kw > 100 ? 100 : kw);
  }
  const double sc = ldexp(1.0, kw);
  *osc_out = ldexpf(1.f, 4 - kw);
  static const int pos[4][2] = {{1, 2}, {3, 4}, {5, 6}, {0, 7}};
  _Float16* out = (_Float16*)wp;
  for (int wv = 0; wv < 4; ++wv)
    for (int pp = 0; pp < 2; ++pp)
      for (int dy = 0; dy < 7; ++dy)
        for (int n = 0; n < nt; ++n)
          for (int lane = 0; lane < 64; ++lane) {
            const int co = 16 * n + (lane & 15);
            const size_t base = (((((size_t)(wv * 2 + pp) * 7 + dy) * nt + n) * 2) * 64 + lane) * 8;
            for (int e = 0; e < 8; ++e) {
              const int ci = 8 * (lane >> 4) + e;
              const float v = (float)(U[((size_t)(pos[wv][pp] * 7 + dy) * ncol + co) * kCi + ci] * sc);
              const _Float16 hi = (_Float16)v;
              out[base + e] = hi;
              out[base + 64 * 8 + e] = (_Float16)((v - (float)hi) * 2048.f);
            }
          }
  free(U);
  return 0;
}

// One launch: x points at input channel ci0 (pixel pitch xp), y at output channel co0 (pitch yp),
// bias at bias[co0] (unused when mode = 1). mode 0: y = act(conv + bias); 1: y = conv (the first
// 32-channel input half of a 64-channel layer); 2: y = act(conv + bias + y) (the second half).
int fvc_conv2d_nhwc_wr7(const float* x, int xp, const void* upack, int nt, float osc, const float* bias, float* y,
                        int yp, int batch, int h, int w, int mode, int act, int cu_reserve, int* overflow_flag,
                        int* sched, int sched_len, fvc_stream_t stream) {
  if (!x || !upack || !y || (nt != 1 && nt != 2) || batch <= 0 || h <= 0 || w <= 0 || cu_reserve < 0 ||
      sched_len < 0 || mode < 0 || mode > 2 || (mode != kModePartial && !bias))
    return FVC_EINVAL;
  if (act != FVC_ACT_NONE && act != FVC_ACT_RELU && act != FVC_ACT_LRELU) return FVC_EINVAL;
  if (xp < kCi || (xp & 3) || yp < 16 * nt || (yp & 3)) return FVC_EINVAL;
  // every buffer descriptor spans one row: 32-bit offsets hold for any batch
  if ((unsigned long long)w * (xp > yp ? xp : yp) * 4ull >= (1ull << 31)) return FVC_EINVAL;
  Wr7Args a;
  a.x = x;
  a.u = (const uint4*)upack;
  a.bias = bias;
  a.y = y;
  a.B = batch;
  a.H = h;
  a.W = w;
  a.xp = xp;
  a.yp = yp;
  a.ngroups = fvc_cdiv(w, 32);
  a.chunks_per_col = fvc_cdiv(h, kRows);
  const long long nch = (long long)batch * a.ngroups * a.chunks_per_col;
  if (nch >= (1ll << 30)) return FVC_EINVAL;
  a.nchunks = (int)nch;
  a.osc = osc;
  a.osc_c = osc * (1.f / 2048.f);
  a.ovf = overflow_flag;
  const int reserve = env_int("FVC_X3_RESERVE", -1) >= 0 ? env_int("FVC_X3_RESERVE", 0) : cu_reserve;
  const int ncu = wr7_num_cus() - (reserve < wr7_num_cus() / 2 ? reserve : wr7_num_cus() / 2);
  const int grid = ncu < a.nchunks ? ncu : a.nchunks;
  a.sched = (sched && sched_len >= 2 && env_int("FVC_X3_DYN", 1)) ? sched : nullptr;
  if (nt == 2) return wr7_launch1<2>(a, mode, act, grid, (hipStream_t)stream);
  return wr7_launch1<1>(a, mode, act, grid, (hipStream_t)stream);
}

}  // extern "C"
