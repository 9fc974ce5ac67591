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
// A work item is a 32-column strip (16 tiles) of up to 128 output rows, walked top to bottom: each
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

// experiment knobs (compile-time; the product build uses the defaults): the gap after which quad
// 1's raw columns are read, and whether waves 0..2 use the 3 + 3-term transform (branch) or every
// wave the general 4 + 4-term one (branch-free)
#ifndef FVC_WR7_Q1GAP
#define FVC_WR7_Q1GAP 4
#endif
#ifndef FVC_WR7_SPEC
#define FVC_WR7_SPEC 0
#endif
#ifndef FVC_WR7_DIST
#define FVC_WR7_DIST 2
#endif
// knock-outs (experiment builds only; results wrong): bit 0 no transform (raw reads + VALU),
// bit 1 no finishing (partial reads, stores), bit 2 no per-step barrier, bit 3 no MFMAs, bit 4 no
// partial-output writes (combine + ds_write)
#ifndef FVC_WR7_KO
#define FVC_WR7_KO 0
#endif
#ifndef FVC_WR7_SPREAD
#define FVC_WR7_SPREAD 0
#endif

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kCi = 32;                         // input channels per launch
constexpr int kQ = kCi / 4;                     // channel quads
constexpr int kSlots = 40;                      // column slots per (row, quad) line: 19 even + 19 odd used
constexpr int kRowEntries = kQ * kSlots;        // 16-B entries per staged row (320 = 5 DMA pieces)
constexpr int kRawRing = 16;                    // staged raw rows
constexpr int kRawBytes = kRawRing * kRowEntries * 16;  // 81,920
constexpr int kZBytes = 4 * 2 * 2 * 64 * 16;            // partial outputs: [wave][i][n][lane] f32x4
constexpr int kHdr = 256;                               // bias (128 B) + work-item word
constexpr int kResBytes = 4 * 3 * 64 * 16;             // residual rows (mode 2): [wave][3 slots][lane] f32x4
constexpr int kLds = kHdr + kRawBytes + 2 * kZBytes + 1024 + kResBytes;  // 128,256 (+ the dummy-DMA sink)
constexpr int kRowsMax = 128;                   // output rows per work item, at most (wr7_rows)
constexpr int kDist = FVC_WR7_DIST;             // raw rows are staged kDist steps before their transform
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
  int ngroups, rows, chunks_per_col, nchunks;  // rows: output rows per work item (wr7_rows)
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

// One LDS-DMA piece (buffer_load_dwordx4 ... lds: 16 B per lane into LDS at M0 + 16 lane) in
// inline asm. The builtin form makes hipcc wait for every pending LDS-DMA before each later
// ds_read (it cannot tell the addresses apart), which would drain this kernel's row prefetch at
// the first read of every step; in asm the DMA is invisible to hipcc's counters and the kernel
// waits for it itself (the counted vmcnt + barrier at the end of each step). M0 is compiler-
// reserved: set and restored inside the statement; s_nop 4 after the descriptor / M0 writes
// (cdna_hip_programming.md §5.7 items 1-2).
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t rx, unsigned voff, const char* lds_dst) {
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds_dst);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 4\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rx), "s"(base)
      : "memory");
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
  char* const sink = zbuf + 2 * kZBytes;
  char* const resb = sink + 1024;

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
  // columns' weighted sums (B^T rows, with the 2^-4 V scale).
  const float s = 1.f / 16.f;
  // The partials a wave writes are P0 = M_a + M_b, P1 = M_a - M_b (waves 0..2) or P0 = M0, P1 = M7
  // (wave 3); the A^T weights of P1 (1, 2, 1/2, 1 for waves 0..3) are applied by the finishing sum.
  float E0, E1, E2, E3, O0, O1, O2, O3;
  if (wave == 0) {
    E0 = 0.f; E1 = s; E2 = -4.25f * s; E3 = s; O0 = s; O1 = -4.25f * s; O2 = s; O3 = 0.f;
  } else if (wave == 1) {
    E0 = 0.f; E1 = 0.25f * s; E2 = -1.25f * s; E3 = s; O0 = 0.5f * s; O1 = -2.5f * s; O2 = 2.f * s; O3 = 0.f;
  } else if (wave == 2) {
    E0 = 0.f; E1 = 4.f * s; E2 = -5.f * s; E3 = s; O0 = 2.f * s; O1 = -2.5f * s; O2 = 0.5f * s; O3 = 0.f;
  } else {
    E0 = -s; E1 = 5.25f * s; E2 = -5.25f * s; E3 = s; O0 = -s; O1 = 5.25f * s; O2 = -5.25f * s; O3 = s;
  }

  // DMA pieces of a staged row: pieces 0..4 (320 entries); wave w issues piece w and, wave 0 only,
  // piece 4 -- waves 1..3 issue a second, dummy piece into a sink so that every wave has the same
  // number of vector-memory operations per step (the counted vmcnt below). The lane's entry
  // (quad, column slot) -> input column and channel-quad offset. Column slots of a (row, quad)
  // line: even strip columns 0..36 at 0..18, odd 1..37 at 19..37 (a tile's 8 columns are 2t + l)
  int dma_c[2], dma_q[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int e = (wave + 4 * m) * 64 + lane;
    const int q = e / kSlots, cs = e - q * kSlots;
    dma_c[m] = (m == 1 && wave != 0) ? -(1 << 20) : (cs < 19 ? 2 * cs : (cs < 38 ? 2 * (cs - 19) + 1 : -(1 << 20)));
    dma_q[m] = 4 * q;
  }
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
  // raw input row iy of image b into raw ring slot `slot` (0 bytes for a padding row: the DMA
  // lands zeros); two operations per wave
  auto stage_row = [&](const float* ximg, int iy, int slot) {
    const bool ok = (unsigned)iy < (unsigned)H;
    const __amdgpu_buffer_rsrc_t rx = rsrc(ximg + (size_t)(unsigned)(ok ? iy : 0) * rowe, ok ? row_bytes : 0u);
    char* const rowp = raw + (size_t)slot * kRowEntries * 16;
    dma_piece(rx, vo[0], rowp + (size_t)wave * 64 * 16);
    dma_piece(rx, vo[1], wave == 0 ? rowp + 4 * 64 * 16 : sink);
  };

  // the transformed-row ring (MFMA B operands, 2 positions x hi / lo): V slot of input row r =
  // (r - y0 + 3) & 7 (compile-time in the 8-way unrolled row loop); raw slot (r - y0 + 3) & 15
  h8 vh[8][2], vl[8][2];
  // the transform of one input row in pieces, so that its VALU can sit between the MFMA blocks
  // of a step: reads of one channel quad, the four channels of a quad, the splits
  struct Tx {
    float4 x0[8], x1[8];  // the lane's 8 columns of channel quads 2o and 2o + 1 (never live together)
    float va[8], vb[8];
    unsigned hwa[4], lwa[4], hwb[4], lwb[4];
  };
  auto tx_read = [&](Tx& T, const char* row, int hq) {
    const char* const line = row + (size_t)(2 * o + hq) * kSlots * 16;
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const int slot = (l & 1) ? 19 + t + (l >> 1) : t + (l >> 1);
      (hq ? T.x1 : T.x0)[l] = *reinterpret_cast<const float4*>(line + slot * 16);
    }
  };
  // waves 0..2: V_a, V_b = e +- o over 3 + 3 columns (E0 = O3 = 0); wave 3: V0 = e, V7 = o over
  // 4 + 4 columns (a wave-uniform branch: 8 VALU per channel either way)
  auto tx_chan = [&](Tx& T, int hq, int c) {
    const float4* const x = hq ? T.x1 : T.x0;
    auto ch = [&](const float4& v) { return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)); };
    // (the empty asm keeps hipcc from if-converting the uniform branch into both paths + selects)
    if (!FVC_WR7_SPEC) {
      const float e = fmaf(E3, ch(x[6]), fmaf(E2, ch(x[4]), fmaf(E1, ch(x[2]), E0 * ch(x[0]))));
      const float od = fmaf(O3, ch(x[7]), fmaf(O2, ch(x[5]), fmaf(O1, ch(x[3]), O0 * ch(x[1]))));
      const bool w3 = wave == 3;
      T.va[4 * hq + c] = w3 ? e : e + od;
      T.vb[4 * hq + c] = w3 ? od : e - od;
    } else if (wave != 3) {
      asm volatile("");
      const float e = fmaf(E3, ch(x[6]), fmaf(E2, ch(x[4]), E1 * ch(x[2])));
      const float od = fmaf(O2, ch(x[5]), fmaf(O1, ch(x[3]), O0 * ch(x[1])));
      T.va[4 * hq + c] = e + od;
      T.vb[4 * hq + c] = e - od;
    } else {
      asm volatile("");
      T.va[4 * hq + c] = fmaf(E3, ch(x[6]), fmaf(E2, ch(x[4]), fmaf(E1, ch(x[2]), E0 * ch(x[0]))));
      T.vb[4 * hq + c] = fmaf(O3, ch(x[7]), fmaf(O2, ch(x[5]), fmaf(O1, ch(x[3]), O0 * ch(x[1]))));
    }
  };
  auto tx_split = [&](Tx& T, int i) {  // i < 4: V_a pair i, else V_b pair i - 4
    if (i < 4) split2(T.va[2 * i], T.va[2 * i + 1], T.hwa[i], T.lwa[i]);
    else split2(T.vb[2 * (i - 4)], T.vb[2 * (i - 4) + 1], T.hwb[i - 4], T.lwb[i - 4]);
  };
  auto tx_store = [&](Tx& T, auto RS_c) {
    constexpr int RS = decltype(RS_c)::value;
    vh[RS][0] = __builtin_bit_cast(h8, v4u{T.hwa[0], T.hwa[1], T.hwa[2], T.hwa[3]});
    vl[RS][0] = __builtin_bit_cast(h8, v4u{T.lwa[0], T.lwa[1], T.lwa[2], T.lwa[3]});
    vh[RS][1] = __builtin_bit_cast(h8, v4u{T.hwb[0], T.hwb[1], T.hwb[2], T.hwb[3]});
    vl[RS][1] = __builtin_bit_cast(h8, v4u{T.lwb[0], T.lwb[1], T.lwb[2], T.lwb[3]});
    // pin the slot here in program order: its VALU writes may not sink towards the MFMAs that read
    // it (asm operands do not capture: name the ring slots through references)
    h8& h0 = vh[RS][0];
    h8& l0 = vl[RS][0];
    h8& h1 = vh[RS][1];
    h8& l1 = vl[RS][1];
    asm volatile("" : "+v"(h0), "+v"(l0), "+v"(h1), "+v"(l1));
  };
  auto transform = [&](const char* row, auto RS_c) {  // whole row (prologue)
    Tx T;
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      tx_read(T, row, hq);
#pragma unroll
      for (int c = 0; c < 4; ++c) tx_chan(T, hq, c);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) tx_split(T, i);
    tx_store(T, RS_c);
  };

  // ---- schedule: items = (image, 32-column group, chunk of kRows output rows), chunk fastest
  int* const ctr = a.sched ? a.sched + 1 : nullptr;
  int k_item = 0;
  float chk = 0.f;
  const unsigned yrow_bytes = (unsigned)W * a.yp * 4u;
  // this lane's finishing share: output column parity fi and 16-channel tile fn (wave w -> (w & 1,
  // w >> 1)); NT = 1 leaves waves 2 and 3 without one (their stores / loads go to kOob)
  const int fi = wave & 1, fn = wave >> 1;
  const bool fin = fn < NT;
  int zb = 0;
  // finishing of output row yf from the partial outputs in zbuf[zbf]: the four waves' partials
  // summed in a fixed order, then scale, bias, the mode's partial sum, activation, 16-B store;
  // live = false (no row before the item's first) issues the same memory operations to kOob
  // the residual partial sum of output row yf (mode 2) into this wave's LDS slot yf % 3, by
  // LDS-DMA like the raw rows (one operation per wave: the finishing lanes' 16 B each)
  auto dma_res = [&](float* yimg, int yf, unsigned so_) {
    if constexpr (MODE == kModeAdd) {
      const bool ok = yf < H;
      const __amdgpu_buffer_rsrc_t ry = rsrc(yimg + (size_t)(unsigned)(ok ? yf : 0) * ((unsigned)W * a.yp),
                                             ok ? yrow_bytes : 0u);
      dma_piece(ry, so_, resb + (size_t)(wave * 3 + (yf + 3) % 3) * 64 * 16);
    }
  };
  auto res_of = [&](int yf) -> f32x4 {
    if constexpr (MODE == kModeAdd) return *reinterpret_cast<const f32x4*>(resb + ((size_t)(wave * 3 + (yf + 3) % 3) * 64 + lane) * 16);
    return f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto finish_read = [&](int zbf, int yf, f32x4 (&P)[4], f32x4& bj, f32x4& rv) {
    const char* const zr = zbuf + zbf * kZBytes;
#pragma unroll
    for (int w = 0; w < 4; ++w) P[w] = *reinterpret_cast<const f32x4*>(zr + (((w * 2 + fi) * 2 + (fn & 1)) * 64 + lane) * 16);
    bj = *reinterpret_cast<const f32x4*>(sbias + 16 * (fn & 1) + 4 * o);
    rv = res_of(yf);
  };
  // Y_fi = sum over waves of c_w P_w in a fixed order (c = 1 for Y0; 1, 2, 1/2, 1 for Y1), then
  // scale, bias, the mode's partial sum, activation, 16-B store; live = false (no row before the
  // item's first) issues the same memory operation to kOob
  const float c1 = fi ? 2.f : 1.f, c2 = fi ? 0.5f : 1.f;
  auto finish_row = [&](float* yimg, int yf, unsigned so, bool live, const f32x4 (&P)[4], const f32x4& bj,
                        const f32x4& rv) {
    const __amdgpu_buffer_rsrc_t ry = rsrc(yimg + (size_t)(unsigned)yf * ((unsigned)W * a.yp), yrow_bytes);
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float sum = fmaf(c2, P[2][r], fmaf(c1, P[1][r], P[0][r])) + P[3][r];
      if (live && fin) chk = fmaf(sum, 0.f, chk);
      float tv = MODE == kModePartial ? sum * a.osc : fmaf(sum, a.osc, bj[r]);
      if constexpr (MODE == kModeAdd) tv += rv[r];
      if constexpr (MODE != kModePartial) {
        if constexpr (ACT == FVC_ACT_RELU) tv = relu1(tv);
        if constexpr (ACT == FVC_ACT_LRELU) tv = fmaxf(tv, tv * 0.1f);
      }
      v[r] = tv;
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), ry, live ? so : kOob, 0, 0);
  };
  for (;;) {
    if (tid == 0) sitem[0] = ctr ? atomicAdd(ctr, 1) : (int)blockIdx.x + k_item * (int)gridDim.x;
    ++k_item;
    __syncthreads();
    const int it = __builtin_amdgcn_readfirstlane(sitem[0]);
    if (it >= a.nchunks) break;
    const int col = it / a.chunks_per_col;
    const int y0 = (it - col * a.chunks_per_col) * a.rows;
    const int y1 = min(y0 + a.rows, H);
    const int b = col / a.ngroups;
    const int g = col - b * a.ngroups;
    const float* const ximg = a.x + (size_t)b * H * rowe;
    float* const yimg = a.y + (size_t)b * H * W * a.yp;
    row_offsets(g);
    // output byte offset of the finishing lane within an output row (past the row when the pixel
    // is outside the image or the wave finishes nothing)
    const int ox = 32 * g + 2 * t + fi;
    const unsigned so = (ox < W && fin) ? (unsigned)(ox * a.yp + 16 * fn + 4 * o) * 4u : kOob;
    auto raw_row = [&](int r) { return raw + (size_t)((r - y0 + 3) & (kRawRing - 1)) * kRowEntries * 16; };

    // prologue: raw rows y0-3 .. y0+5 (the first step's transform reads y0+4, the second's y0+5),
    // then the first 7 transformed rows
#pragma unroll
    for (int i = 0; i < 7 + kDist; ++i) stage_row(ximg, y0 - 3 + i, i);
    dma_res(yimg, y0, so);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    transform(raw_row(y0 - 3), ic<0>{}); transform(raw_row(y0 - 2), ic<1>{});
    transform(raw_row(y0 - 1), ic<2>{}); transform(raw_row(y0), ic<3>{});
    transform(raw_row(y0 + 1), ic<4>{}); transform(raw_row(y0 + 2), ic<5>{});
    transform(raw_row(y0 + 3), ic<6>{});
    __syncthreads();  // every wave is done with the prologue's raw slots before the steps stage

    int y = y0;
    // one output row y, S = (y - y0) & 7 (compile-time: the loop is unrolled by 8). Program order:
    // stage raw row y + 6; the previous row's residual; the 28 MFMA blocks of this row with, between
    // them, the finishing of row y - 1 and the transform of raw row y + 4 into V slot (S + 7) & 7
    // (a slot no kernel row of this step reads); drain; this row's partial outputs into zbuf[zb];
    // counted vmcnt (raw row y + 5 landed) and the step's one barrier.
    auto step = [&](auto S_c) {
      constexpr int S = decltype(S_c)::value;
      // the next row's partial sum (mode 2), finished two steps from now, then raw row y + 6
      dma_res(yimg, y + 1, so);
      stage_row(ximg, y + 4 + kDist, (y + 7 + kDist - y0) & (kRawRing - 1));
      const bool prev = y > y0;
      const char* const rrow = raw_row(y + 4);
      Tx T;

      f32x4 acc[2][NT], cor[2][NT];
      int blk = 0;
      // the VALU work placed after MFMA block k of the step (28 blocks)
      f32x4 P[4], bj, rv;
      auto gap = [&](int k) {
        // LDS reads two blocks ahead of their first use; quad 1's columns are read once quad 0's
        // are consumed (the two sets never live together: VGPR budget)
        if ((FVC_WR7_KO & 1) && k != 3 && k != 0) return;
        if ((FVC_WR7_KO & 2) && k == 3) return;
        if (k == 0) {
          if (!(FVC_WR7_KO & 1)) tx_read(T, rrow, 0);
          if (!(FVC_WR7_KO & 2)) finish_read(zb ^ 1, y - 1, P, bj, rv);
        } else if (k == 2) tx_chan(T, 0, 0);
        else if (k == 3) finish_row(yimg, y - 1, so, prev, P, bj, rv);
        else if (k >= 4 && k <= 6) tx_chan(T, 0, k - 3);
        else if (!FVC_WR7_SPREAD && k >= 8 && k <= 11) tx_chan(T, 1, k - 8);
        else if (FVC_WR7_SPREAD && k >= 8 && k <= 14 && !(k & 1)) tx_chan(T, 1, (k - 8) >> 1);
        else if (!FVC_WR7_SPREAD && k >= 12 && k <= 19) tx_split(T, k - 12);
        else if (FVC_WR7_SPREAD && k >= 15 && k <= 26 && k != 17 && k != 20 && k != 23 && k != 26)
          tx_split(T, k - 15 - (k > 17) - (k > 20) - (k > 23));
        else if (k == (FVC_WR7_SPREAD ? 27 : 20)) tx_store(T, ic<(S + 7) & 7>{});
        if (k == FVC_WR7_Q1GAP) tx_read(T, rrow, 1);
      };
      auto row_mfmas = [&](auto DY_c) {
        constexpr int DY = decltype(DY_c)::value;
        constexpr int VS = (S + DY) & 7;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            if (FVC_WR7_KO & 8) {
              if (DY == 0) acc[pp][n] = cor[pp][n] = f32x4{0.f, 0.f, 0.f, 0.f};
              asm volatile("" : "+v"(acc[pp][n]), "+v"(cor[pp][n]) : "v"(vh[VS][pp]), "v"(vl[VS][pp]));
            } else if (DY == 0 && pp == 0 && n == 0)
              wr7_mfma3<true, true>(acc[pp][n], cor[pp][n], u[pp][DY][n][0], u[pp][DY][n][1], vh[VS][pp], vl[VS][pp]);
            else
              wr7_mfma3<DY == 0, false>(acc[pp][n], cor[pp][n], u[pp][DY][n][0], u[pp][DY][n][1], vh[VS][pp],
                                        vl[VS][pp]);
            gap(blk);
            // NT = 1 has 14 blocks: two gaps' work per block
            if constexpr (NT == 1) gap(blk + 1);
            blk += NT == 1 ? 2 : 1;
          }
      };
      row_mfmas(ic<0>{});
      row_mfmas(ic<1>{});
      row_mfmas(ic<2>{});
      row_mfmas(ic<3>{});
      row_mfmas(ic<4>{});
      row_mfmas(ic<5>{});
      row_mfmas(ic<6>{});
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
        if (FVC_WR7_KO & 16) {
          asm volatile("" :: "v"(acc[0][n]), "v"(acc[1][n]), "v"(cor[0][n]), "v"(cor[1][n]));
          continue;
        }
        f32x4 ma, mb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ma[r] = fmaf(cor[0][n][r], 1.f / kLoScale, acc[0][n][r]);
          mb[r] = fmaf(cor[1][n][r], 1.f / kLoScale, acc[1][n][r]);
        }
        f32x4 p0 = ma, p1 = mb;
        if (wave != 3) {
          asm volatile("");
          p0 = ma + mb;
          p1 = ma - mb;
        }
        *reinterpret_cast<f32x4*>(zw + (((wave * 2 + 0) * 2 + n) * 64 + lane) * 16) = p0;
        *reinterpret_cast<f32x4*>(zw + (((wave * 2 + 1) * 2 + n) * 64 + lane) * 16) = p1;
      }
      // raw row y + 5 (staged one step ago) must have landed before the next step transforms it,
      // and (mode 2) row y's partial sum, staged one step ago just before it: every wave issues per
      // step [1 residual DMA,] 2 raw-row DMA operations and 1 store, so the ones younger than that
      // row's DMA are the previous step's store and this step's 3 (4)
      if constexpr (kDist == 3) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else if constexpr (MODE == kModeAdd) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      if (!(FVC_WR7_KO & 4)) __syncthreads();
      zb ^= 1;
      ++y;
    };
    // the item's last row, after step S
    auto last = [&](auto) {
      f32x4 P[4], bj, rv;
      finish_read(zb ^ 1, y1 - 1, P, bj, rv);
      finish_row(yimg, y1 - 1, so, true, P, bj, rv);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    for (;;) {
      step(ic<0>{}); if (y >= y1) { last(ic<0>{}); break; }
      step(ic<1>{}); if (y >= y1) { last(ic<1>{}); break; }
      step(ic<2>{}); if (y >= y1) { last(ic<2>{}); break; }
      step(ic<3>{}); if (y >= y1) { last(ic<3>{}); break; }
      step(ic<4>{}); if (y >= y1) { last(ic<4>{}); break; }
      step(ic<5>{}); if (y >= y1) { last(ic<5>{}); break; }
      step(ic<6>{}); if (y >= y1) { last(ic<6>{}); break; }
      step(ic<7>{}); if (y >= y1) { last(ic<7>{}); break; }
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

// Output rows per work item. An item pays a prologue (9 raw rows staged, 7 transformed) worth
// about kPrologueRows steady-state rows, so long items amortise it; but a launch's makespan is
// ceil(items / blocks) item lengths, and one block per CU over 128-row items leaves most of the
// chip idle at batch 1 (a 544x960 level is 150 items for 256 CUs; VERDICT r5: the batch-1 SpyNet
// stage went 4.6 -> 5.9 ms). Pick the item height that minimises that estimate. The result of
// every output row is the same for any item height (each row sums the same transformed rows in
// the same order), so the choice never changes the numbers. FVC_WR7_ROWS forces one (A/B).
static int wr7_rows(int batch, int h, int ngroups, int blocks) {
  const int forced = env_int("FVC_WR7_ROWS", 0);
  if (forced > 0) return forced < kRowsMax ? forced : kRowsMax;
  constexpr int kPrologueRows = 8;
  int best = kRowsMax;
  long long best_cost = -1;
  for (int r = kRowsMax; r >= 16; r /= 2) {
    const long long items = (long long)batch * ngroups * fvc_cdiv(h, r);
    const long long rounds = (items + blocks - 1) / blocks;
    const long long cost = rounds * ((r < h ? r : h) + kPrologueRows);
    if (best_cost < 0 || cost < best_cost) best = r, best_cost = cost;
  }
  return best;
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
  const int reserve = env_int("FVC_X3_RESERVE", -1) >= 0 ? env_int("FVC_X3_RESERVE", 0) : cu_reserve;
  const int ncu = wr7_num_cus() - (reserve < wr7_num_cus() / 2 ? reserve : wr7_num_cus() / 2);
  a.rows = wr7_rows(batch, h, a.ngroups, ncu);
  a.chunks_per_col = fvc_cdiv(h, a.rows);
  const long long nch = (long long)batch * a.ngroups * a.chunks_per_col;
  if (nch >= (1ll << 30)) return FVC_EINVAL;
  a.nchunks = (int)nch;
  a.osc = osc;
  a.osc_c = osc * (1.f / 2048.f);
  a.ovf = overflow_flag;
  const int grid = ncu < a.nchunks ? ncu : a.nchunks;
  a.sched = (sched && sched_len >= 2 && env_int("FVC_X3_DYN", 1)) ? sched : nullptr;
  if (nt == 2) return wr7_launch1<2>(a, mode, act, grid, (hipStream_t)stream);
  return wr7_launch1<1>(a, mode, act, grid, (hipStream_t)stream);
}

}  // extern "C"
