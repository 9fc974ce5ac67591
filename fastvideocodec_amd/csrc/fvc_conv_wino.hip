// Winograd F(2x2, 3x3) split-precision convolution for the 64 -> 64-channel, 3x3, stride-1 layers
// (Warp_net's ResBlocks, DVC/subnet/endecoder.py:228-296) on the fp16 matrix cores
// (v_mfma_f32_16x16x32_f16), at fp32-level accuracy. Replaces the same ATen conv2d calls as
// fvc_conv_x3.hip for that geometry: 16 products per (2x2 output tile, channel pair) instead of 36,
// i.e. 2.25x fewer matrix instructions for the same algorithmic work.
//
// Algorithm (Lavin & Gray 2016): for each 2x2 output tile the 4x4 input patch d is transformed,
// V = B^T d B; every transformed position p is an independent GEMM over the input channels with the
// transformed weights U[p] = (G g G^T)[p]: M[p] = sum_c U[p][c] V[p][c]; the tile is Y = A^T M A,
// then bias, activation and residual as the direct kernel. F(2,3) matrices:
//   B^T rows (1,0,-1,0) (0,1,1,0) (0,-1,1,0) (0,1,0,-1)   (input: additions only)
//   G   rows (1,0,0) (1/2,1/2,1/2) (1/2,-1/2,1/2) (0,0,1) (weights, on the host in double)
//   A^T rows (1,1,1,0) (0,1,-1,-1)                        (output: additions only)
//
// Numerics as fvc_conv_x3.hip: U (scaled by 2^kw so max|U| is in [2^13, 2^14)) and V (fp32 here)
// are split exactly into fp16 hi + lo * 2^-11; main += U_hi V_hi and corr += U_lo V_hi + U_hi V_lo
// in two fp32 accumulators. |V| <= 4 max|x|: a transformed value >= 65520 rounds to an infinite hi
// part, whose products reach every output of its tile that lies in the image as inf / NaN (the
// B^T / A^T patterns leave no overflowing position feeding only clipped outputs); the kernel sums
// 0 * output and raises the caller's overflow flag on a NaN (the host then recomputes on the fp32
// kernels). NaN inputs raise it as well.
//
// Resident weights: one 256-thread block per CU, one wave per SIMD with 512 registers. Wave r owns
// row r of the 4x4 transform domain (positions (r, q), q = 0..3) for all 64 output channels: its
// 64 KB of U (hi and lo planes) is loaded once per launch and stays in registers, so the k-loop
// reads no weights at all. A work item is a row of 16 tiles (2 output rows x 32 columns); per item
// each lane transforms the input of its tile (lane & 15) and 8 channels straight into the MFMA B
// operand of its wave's 4 positions (no V in memory). The waves then exchange the column-combined
// partial results Z[r][j] = sum_q M[r][q] A[q][j] through LDS (double-buffered: one barrier per
// item) and wave w finishes output channels 16w .. 16w+15: Y[i][j] = sum_r A^T[i][r] Z[r][j].
// Input: a ring of 8 raw fp32 input rows in LDS filled by LDS-DMA (buffer_load_dwordx4 ... lds, one
// descriptor per row: padding rows and columns read past it and land as zeros); consecutive items of a block walk down one tile column, so each item
// stages the 2 new rows of its 4-row window while the previous item computes.
// LDS input layout (r6): row slot -> 34 columns -> 16 channel quads, the quad index XORed with
// (column >> 1) & 15 (ring_entry): the LDS image of a row is its 34 pixels as they lie in memory, up
// to that swizzle, so each LDS-DMA instruction reads 4 whole pixels (1 KB contiguous), and the
// transform's ds_read_b128 of 16 tiles (columns 2t + d) x a quad still covers every bank group
// once per 16 lanes. (r3-r5: quad-major lines with even / odd column halves; -DFVC_WINO_PIX=0.)
// Epilogue forms: plain (bias, ReLU / LeakyReLU, residual add), and POOL, which also writes the
// 2x2 average pool of the output (each pool window is one Winograd tile: ATen's ((x00 + x01) + x10)
// + x11) / 4, bit-identical to k_avgpool2).
#include "fvc_common.h"
#include <math.h>
#include <stdlib.h>

namespace {

// cache policy of the activation stores (aux operand of buffer_store; experiment builds only,
// e.g. 2 = non-temporal on gfx950)
#ifndef FVC_STORE_AUX
#define FVC_STORE_AUX 0
#endif

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kC = 64;             // input and output channels
constexpr int kQ = kC / 4;         // channel quads per pixel
constexpr int kTiles = 16;         // tiles per item: one tile row x 16 tile columns
constexpr int kCols = 2 * kTiles + 2;  // input columns an item reads
// staged-row layout. FVC_WINO_PIX 1 (default, r6): pixel-major, entry (local column c, quad Q) at
// c * 16 + (Q ^ ((c >> 1) & 15)), 34 columns padded to 36 (9 LDS-DMA pieces): every DMA instruction
// reads 4 whole pixels (1 KB of consecutive bytes). 0 (r3-r5): quad-major, even columns in slots
// 0..16 and odd ones in 17..33 of a 40-slot line per quad: each DMA instruction gathered 16 B from
// ~40 pixels. Both give conflict-free ds_read_b128 for the transform's reads (16 tiles x a quad).
#ifndef FVC_WINO_PIX
#define FVC_WINO_PIX 1
#endif
constexpr bool kPix = FVC_WINO_PIX != 0;
constexpr int kSlots = 40;         // quad-major form: column slots per (row, quad) line (34 used)
constexpr int kRowEntries = kPix ? 36 * kQ : kQ * kSlots;   // 16-B entries per staged row (576 / 640)
constexpr int kRowPieces = kRowEntries / 64;                // LDS-DMA pieces per row (9 / 10)
constexpr int kRing = 8;           // staged input rows
constexpr int kRingBytes = kRing * kRowEntries * 16;  // 73,728 (quad-major: 81,920)
constexpr int kZBytes = 4 * 8 * 1024;                 // one Z buffer: 4 waves x 8 planes x 1 KB
constexpr int kHdr = 512;                             // bias (256 B) + schedule words
constexpr int kLds = kHdr + kRingBytes + 2 * kZBytes; // 139,776 B (quad-major: 148,480)
// fused upsample-add input (UP): the low-resolution rows one item's fix-up reads, [row][pixel][quad]
// (up to 4 source rows x 20 source columns, the span 4 output rows x 34 output columns of a 2x
// align_corners=True upsample can reach); Z single-buffered (two barriers per item)
constexpr int kLowRows = 4;
constexpr int kLowCols = 20;
constexpr int kLowRowEnt = kLowCols * kQ;                  // 16-B entries per low row (320)
constexpr int kLowBytes = kLowRows * kLowRowEnt * 16;      // 20,480
constexpr int kLdsUp = kHdr + kRingBytes + kZBytes + kLowBytes;  // 127,488 B
// items per schedule chunk (consecutive tile rows of one column): 16 (32 as an experiment switch)
constexpr int kChunkMin = 16, kChunkMax = 32;
constexpr float kLoScale = 2048.f;
// knock-outs (experiment builds only; results wrong): FVC_WINO_KO bit 1 = no k-step-1 MFMAs,
// 2 = no k-step-0 MFMAs (their split VALU kept), 4 = no item barrier, 8 = no finishing pass,
// 16 = finishing pass without its output stores, 32 = finishing pass without its Z reads,
// 64 = no staging of the next item's input rows (LDS-DMA issue and its scalar addressing)
#ifndef FVC_WINO_KO
#define FVC_WINO_KO 0
#endif
// UP knock-outs / forms (experiment builds only): FVC_UP_KO bit 1 = no fix-up body, 2 = no second
// barrier, 4 = no xu stores, 8 = no LDS write-back, 16 = no low-row DMA; FVC_UP_FORM 1 = per-entry
// lerp (four low taps per entry) instead of the shared horizontal lerps
#ifndef FVC_UP_KO
#define FVC_UP_KO 0
#endif
#ifndef FVC_UP_FORM
#define FVC_UP_FORM 0
#endif
#ifndef FVC_UP_FIRST
#define FVC_UP_FIRST 0
#endif
#ifndef FVC_WINO_KO_WAIT
#define FVC_WINO_KO_WAIT 0
#endif
#ifndef FVC_WINO_ALLNOP
#define FVC_WINO_ALLNOP 0
#endif
constexpr bool kAllNop = FVC_WINO_ALLNOP;  // every MFMA block opens with s_nop 1 (diagnostic)
constexpr unsigned kOob = 0xFFFFFF00u;
constexpr int kRsrcFlags = 0x00020000;
constexpr int kPostPool = 1;
constexpr int kPostTap = 2;
constexpr int kResPost = 1;
constexpr int kResPre = 2;


struct WinoArgs {
  const float* x;
  const uint4* u;        // packed U: [wave r][q][n][kk][plane][lane] 16-B fragments
  const float* bias;
  const float* res;
  float* y;
  float* pool;
  int B, H, W;
  int tiles_y, ngroups;  // tile rows, 32-column groups
  int nchunks, chunks_per_col, chunk;  // chunk: items (tile rows) per schedule chunk
  float osc, osc_c;      // 2^-kw, 2^-kw-11
  int* sched;            // [0] blocks finished, [1] next chunk; zero on entry, reset by the last block
  int* ovf;
  // kPostTap: y receives P [B][H][W][pcp] = T . y per pixel (the next layer's tap partials, T
  // [np <= 32][64] packed by fvc_wino_tap_pack_weight, scaled by 2^kt)
  const uint4* tw;
  float tosc, tosc_c;    // 2^-kt, 2^-kt-11
  int pcp;
  // pixel pitch (floats) of x and of y / res: 64, or 128 for a quarter of a 128 -> 128 conv
  // (x, y, res then point at the first channel of their 64-channel half)
  int xp, yp;
  // UP: x is the skip tensor S (full resolution, pitch 64); the input the conv reads is
  // X = S + up2(L) (bilinear, align_corners=True, L = xl [B][hl][wl][64], H = 2 hl, W = 2 wl), formed
  // in LDS after each row's LDS-DMA and written to xu (every pixel once) for the caller's residual
  const float* xl;
  float* xu;
  int hl, wl;
  float usy, usx;  // (hl - 1) / (H - 1), (wl - 1) / (W - 1), one correctly rounded float division each
};

typedef __attribute__((address_space(3))) void* lds_ptr;

// 16-B entry of (local column c = 0..33, channel quad Q) within a staged row
__device__ __forceinline__ int ring_entry(int c, int Q) {
  if constexpr (kPix) return c * kQ + (Q ^ ((c >> 1) & 15));
  return Q * kSlots + ((c & 1) ? 17 + (c >> 1) : (c >> 1));
}

// UP: quad swizzle of the low rows' LDS image (pixel p's quad q at slot q ^ low_swz(p))
__device__ __forceinline__ int low_swz(int p) { return (p & 3) << 2; }

// a raw buffer descriptor over [p, p + bytes): offsets at or past `bytes` read 0 / drop the store.
// The inputs go through readfirstlane (free on values already in SGPRs): the compiler must see the
// descriptor as uniform or it wraps every access in a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  const unsigned long long v = (unsigned long long)(uintptr_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  void* const q = (void*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), kRsrcFlags);
}

// The three split-precision products of one (position, 16-channel N-tile) pair:
//   acc += U_hi V_hi, cor += U_lo V_hi, cor += U_hi V_lo
// U is an AGPR operand ("a": the 256 resident U registers fill the accumulator half of the file,
// the k-loop's VGPRs stay free for the transforms); hipcc does not place MFMAs with A/B operands
// in AGPRs, hence inline asm. Wait states (cdna_hip_programming.md §5.7): a VALU write of vh / vl
// or a v_accvgpr_write of U right before -> 2 states (s_nop 1, opening the string); the
// accumulate chains need none; the VALU reads of acc / cor after the item's last MFMA are fenced
// by wino_mfma_drain.
// NOP: open with the 2 states (s_nop 1) a VALU-written vh / vl needs; blocks whose operands were
// written three or more instructions earlier skip it (scripts/check_wino_hazards.py audits the
// built .s for VALU writes of MFMA sources within 2 states).
#define WINO_MFMA3_BODY(C0, C1)                    \
  "v_mfma_f32_16x16x32_f16 %0, %2, %4, " C0 "\n\t" \
  "v_mfma_f32_16x16x32_f16 %1, %3, %4, " C1 "\n\t" \
  "v_mfma_f32_16x16x32_f16 %1, %2, %5, %1"
template <bool FIRST, bool NOP>
__device__ __forceinline__ void wino_mfma3(f32x4& acc, f32x4& cor, const h8& uh, const h8& ul, const h8& vh,
                                           const h8& vl) {
  if constexpr (FIRST) {  // first k-step of an item: the chains start from C = 0
    if constexpr (NOP)
      asm volatile("s_nop 1\n\t" WINO_MFMA3_BODY("0", "0") : "=&v"(acc), "=&v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
    else
      asm volatile(WINO_MFMA3_BODY("0", "0") : "=&v"(acc), "=&v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
  } else {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\t" WINO_MFMA3_BODY("%0", "%1") : "+v"(acc), "+v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
    else
      asm volatile(WINO_MFMA3_BODY("%0", "%1") : "+v"(acc), "+v"(cor) : "a"(uh), "a"(ul), "v"(vh), "v"(vl));
  }
}

// wino_mfma3 (first k-step) followed by the split of two values of the next k-step (split2's
// instructions): the split's VALU issues while this block's MFMAs run instead of in a cluster of
// its own. Its outputs feed MFMAs of the next k-step, blocks later.
#define WINO_MFMA3S_BODY                                                     \
  "v_mfma_f32_16x16x32_f16 %0, %7, %9, 0\n\t"                              \
  "v_cvt_pk_f16_f32 %2, %11, %12\n\t"                                      \
  "v_mfma_f32_16x16x32_f16 %1, %8, %9, 0\n\t"                              \
  "v_fma_mix_f32 %4, %2, -1.0, %11 op_sel_hi:[1,0,0]\n\t"                  \
  "v_fma_mix_f32 %5, %2, -1.0, %12 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"   \
  "v_mfma_f32_16x16x32_f16 %1, %7, %10, %1\n\t"                            \
  "v_fma_mixlo_f16 %3, %4, %6, 0\n\t"                                      \
  "v_fma_mixhi_f16 %3, %5, %6, 0"
template <bool NOP>
__device__ __forceinline__ void wino_mfma3_split(f32x4& acc, f32x4& cor, const h8& uh, const h8& ul, const h8& vh,
                                                 const h8& vl, float v0, float v1, unsigned& hi, unsigned& lo) {
  float r0, r1;
  if constexpr (NOP)
    asm volatile("s_nop 1\n\t" WINO_MFMA3S_BODY
                 : "=&v"(acc), "=&v"(cor), "=&v"(hi), "=&v"(lo), "=&v"(r0), "=&v"(r1)
                 : "s"(kLoScale), "a"(uh), "a"(ul), "v"(vh), "v"(vl), "v"(v0), "v"(v1));
  else
    asm volatile(WINO_MFMA3S_BODY
                 : "=&v"(acc), "=&v"(cor), "=&v"(hi), "=&v"(lo), "=&v"(r0), "=&v"(r1)
                 : "s"(kLoScale), "a"(uh), "a"(ul), "v"(vh), "v"(vl), "v"(v0), "v"(v1));
}

// 12 wait states after the last MFMA of an item (the 8-pass XDL bound, cdna_hip_programming.md
// §5.7 item 2) before any VALU reads an accumulator; the accumulators are operands so no reader is
// scheduled above it
__device__ __forceinline__ void wino_mfma_drain(f32x4 (&acc)[4][4], f32x4 (&cor)[4][4]) {
  asm volatile("s_nop 11" : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[0][2]), "+v"(acc[0][3]),
               "+v"(acc[1][0]), "+v"(acc[1][1]), "+v"(acc[1][2]), "+v"(acc[1][3]));
  asm volatile("" : "+v"(acc[2][0]), "+v"(acc[2][1]), "+v"(acc[2][2]), "+v"(acc[2][3]), "+v"(acc[3][0]),
               "+v"(acc[3][1]), "+v"(acc[3][2]), "+v"(acc[3][3]));
  asm volatile("" : "+v"(cor[0][0]), "+v"(cor[0][1]), "+v"(cor[0][2]), "+v"(cor[0][3]), "+v"(cor[1][0]),
               "+v"(cor[1][1]), "+v"(cor[1][2]), "+v"(cor[1][3]));
  asm volatile("" : "+v"(cor[2][0]), "+v"(cor[2][1]), "+v"(cor[2][2]), "+v"(cor[2][3]), "+v"(cor[3][0]),
               "+v"(cor[3][1]), "+v"(cor[3][2]), "+v"(cor[3][3]));
}

// max(x, 0) as one v_max_f32 (fmaxf compiles to a NaN-quieting v_max x, x first)
__device__ __forceinline__ float relu1(float x) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  return r;
}

// y = hi + lo * 2^-11 for two values: hi by one packed round-to-nearest conversion, the residual
// y - hi by v_fma_mix (hi read as f16 inside the FMA: exact), lo rounded straight to f16 by
// v_fma_mix{lo,hi} (5 VALU per pair instead of 8 for convert / convert back / subtract / scale /
// convert). Pure VALU asm: the hardware interlocks VALU dependencies.
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

// RES: 0 none, kResPost = y = act(conv + bias) + res (ResBlock), kResPre = y = act(conv + bias + res)
// (the second input half of a 128 -> 128 conv adding the first half's partial sum)
template <int IOP, int POST, int RES, int ACT, bool UP = false>
__global__ __launch_bounds__(256, 1) void conv_wino_kernel(const WinoArgs a) {
  static_assert(!UP || (POST == 0 && RES == 0), "the fused upsample-add input is a plain-conv form");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* const sbias = reinterpret_cast<float*>(smem);
  int* const sq = reinterpret_cast<int*>(smem + 256);  // [0..1] first chunks, [2..3] chunk after next
  char* const ring = smem + kHdr;
  char* const zbuf = ring + kRingBytes;
  char* const low = zbuf + (UP ? 1 : 2) * kZBytes;  // UP: the low-resolution rows of the next fix-up

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = row r of the transform domain
  const int t = lane & 15;    // tile of this lane (MFMA B column / D column)
  const int o = lane >> 4;    // channel octet of this lane within a 32-channel k-step
  // kPix: byte offset of column 2t in a staged row, and the quad swizzles of columns 2t, 2t + 1
  // ((2t >> 1) & 15 = t) and 2t + 2, 2t + 3 ((t + 1) & 15), each XORed with the octet's 2 o, x 16 B
  const int pix_b = 2 * t * kQ * 16;
  const int pix_x0 = ((2 * o) ^ t) * 16, pix_x1 = ((2 * o) ^ ((t + 1) & 15)) * 16;
  const int W = a.W, H = a.H;

  // resident U: u[q][n][kk][plane], 4 registers each (AGPRs: the MFMA asm's "a" operands)
  h8 u[4][4][2][2];
  {
    const uint4* src = a.u + (size_t)wave * (4 * 4 * 2 * 2 * 64) + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            u[q][n][kk][pl] = __builtin_bit_cast(h8, src[(((q * 4 + n) * 2 + kk) * 2 + pl) * 64]);
  }
  if (tid < kC) sbias[tid] = a.bias ? a.bias[tid] : 0.f;

  // rows of the 4x4 patch this wave's transform row combines: E = d[ra] + sb * d[rb]
  // (B^T rows (1,0,-1,0) (0,1,1,0) (0,-1,1,0) (0,1,0,-1)), then V[r][.] = E B (x-transform)
  const int ra = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int rb = wave == 0 ? 2 : (wave == 1 ? 2 : (wave == 2 ? 1 : 3));
  const float sb = wave == 1 ? 1.f : -1.f;

  // DMA pieces of a staged row this wave issues (piece k of 10 -> wave k & 3) and the lane's
  // part of each: local input column (or a pad slot) and channel-quad offset
  int dma_lc[3], dma_ch[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int e = (wave + 4 * m) * 64 + lane;
    if constexpr (kPix) {
      const int c = e >> 4, qq = e & 15;
      dma_lc[m] = c < 34 ? c : -(1 << 20);
      dma_ch[m] = 4 * (qq ^ ((c >> 1) & 15));
    } else {
      const int c4 = e / kSlots, cs = e - c4 * kSlots;
      dma_lc[m] = cs < 17 ? 2 * cs : (cs < 34 ? 2 * (cs - 17) + 1 : -(1 << 20));
      dma_ch[m] = 4 * c4;
    }
  }
  const int npiece = wave < kRowPieces - 8 ? 3 : 2;  // 9 / 10 pieces over 4 waves
  // byte offsets of the lane's pieces within an input row of column group g (past the row for
  // padding columns and pad slots: the buffer unit returns zeros)
  auto row_offsets = [&](int g, unsigned (&vo)[3]) {
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int ix = 32 * g - 1 + dma_lc[m];
      vo[m] = (unsigned)ix < (unsigned)W ? (unsigned)(ix * a.xp + dma_ch[m]) * 4u : kOob;
    }
  };
  const unsigned row_bytes = (unsigned)W * a.xp * 4u;   // one input row
  const unsigned yrow_bytes = (unsigned)W * a.yp * 4u;  // one output (and residual) row
  // stage input row iy of image b into ring slot s: one descriptor per row (0 bytes for a
  // padding row), the lane offsets of its column group
  // (ximg: the image's base; a row is one 32 x 32-bit product from it: per-row scalar work stays a
  // handful of instructions, the 64-bit image offset is formed once per chunk)
  const unsigned rowe = (unsigned)W * a.xp;
  auto stage_row = [&](const float* ximg, int iy, int s, const unsigned (&vo)[3]) {
    const bool row_ok = (unsigned)iy < (unsigned)H;
    const __amdgpu_buffer_rsrc_t rx = rsrc(ximg + (size_t)(unsigned)(row_ok ? iy : 0) * rowe, row_ok ? row_bytes : 0u);
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      if (m >= npiece) break;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rx, (lds_ptr)(ring + ((size_t)s * kRowEntries + (wave + 4 * m) * 64) * 16), 16, vo[m], 0, 0, 0);
    }
  };

  // ---- schedule: chunks of kChunk consecutive tile rows of one (image, 32-column group)
  int* const ctr = a.sched ? a.sched + 1 : nullptr;
  auto take = [&](int k) -> int {  // thread 0: the k-th chunk this block takes
    if (ctr) return atomicAdd(ctr, 1);
    return (int)blockIdx.x + k * (int)gridDim.x;
  };
  struct Pos {
    int b, g, ty0, ty1;  // tile rows [ty0, ty1) of column group g of image b; empty = no chunk
  };
  auto decode = [&](int ch) -> Pos {  // once per chunk (two scalar divisions)
    ch = __builtin_amdgcn_readfirstlane(ch);  // an LDS word: make it provably uniform
    Pos p{0, 0, 0, 0};
    if (ch < a.nchunks) {
      const int col = ch / a.chunks_per_col;
      p.ty0 = (ch - col * a.chunks_per_col) * a.chunk;
      p.ty1 = min(p.ty0 + a.chunk, a.tiles_y);
      p.b = col / a.ngroups;
      p.g = col - p.b * a.ngroups;
    }
    return p;
  };
  // ---- UP: the fix-up X = S + up2(L) of the rows an item adds to the ring. The rows land by
  // LDS-DMA as S; the low-resolution rows they need land in `low` by LDS-DMA as well (issued with the
  // rows, during the previous item's k-loop); after the item barrier every thread rewrites its
  // entries in place (ring entry = S + lerp of four low taps, the same arithmetic as the standalone
  // k_up2_add_q16p), writes the ones its chunk owns to xu, and a second barrier publishes them.
  struct Fix {
    int b, g, r0, nr, sbase;  // output rows [r0, r0 + nr) of column group g of image b, at ring slot sbase..
    int own0, own1;           // rows [own0, own1) are this chunk's to write to xu
    int lr0, nlow, lc0, ncol; // low rows / columns staged in `low` (nlow = 0: nothing to do)
  };
  auto make_fix = [&](const Pos& p, int ty, bool contd, int sb) -> Fix {
    Fix f;
    f.b = p.b;
    f.g = p.g;
    f.r0 = contd ? 2 * ty + 1 : 2 * ty - 1;
    f.nr = contd ? 2 : 4;
    f.sbase = contd ? (sb + 2) & (kRing - 1) : sb;
    f.own0 = 2 * p.ty0;
    f.own1 = 2 * p.ty1;
    const int rf = max(f.r0, 0), rl = min(f.r0 + f.nr - 1, H - 1);
    const int cf = max(32 * p.g - 1, 0), cl = min(32 * p.g + 32, W - 1);
    f.lr0 = fvc_up_index_scaled(rf, a.hl, a.usy).i0;
    f.nlow = rf <= rl ? fvc_up_index_scaled(rl, a.hl, a.usy).i1 - f.lr0 + 1 : 0;
    f.lc0 = fvc_up_index_scaled(cf, a.wl, a.usx).i0;
    f.ncol = fvc_up_index_scaled(cl, a.wl, a.usx).i1 - f.lc0 + 1;
    f.lr0 = __builtin_amdgcn_readfirstlane(f.lr0);
    f.nlow = __builtin_amdgcn_readfirstlane(f.nlow);
    f.lc0 = __builtin_amdgcn_readfirstlane(f.lc0);
    f.ncol = __builtin_amdgcn_readfirstlane(f.ncol);
    return f;
  };
  // the low rows of fix-up f into `low`: 4 rows x 5 pieces of 64 x 16 B (4 pixels each), piece
  // wave + 4 m of this wave; bytes past the row's ncol pixels read as zeros (never used). Entry
  // (pixel p, quad q) sits at p * 16 + (q ^ low_swz(p)): the fix-up's lanes read 16 pixels x 4 quads
  // at once, which unswizzled (256-B pixel pitch = all 64 banks) would hit the same 4 banks 16 times
  // over; the swizzle is applied on the global side (each lane's 16-B source), so the LDS-DMA image
  // stays lane-linear and every piece still reads 1 KB of consecutive bytes
  auto stage_low = [&](const Fix& f) {
    if constexpr ((FVC_UP_KO & 16) != 0) return;
    const int e = lane >> 4, qq = lane & 15;  // pixel within the piece, LDS quad slot
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int pc = wave + 4 * m, row = pc / 5, pr = pc - 5 * row;
      if (row < f.nlow) {
        const __amdgpu_buffer_rsrc_t rl =
            rsrc(a.xl + ((size_t)((unsigned)f.b * a.hl + f.lr0 + row) * a.wl + f.lc0) * kC, (unsigned)f.ncol * kC * 4u);
        const int px = 4 * pr + e;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_ptr)(low + ((size_t)row * kLowRowEnt + pr * 64) * 16), 16,
                                                 (unsigned)(px * kQ + (qq ^ low_swz(px))) * 16u, 0, 0, 0);
      }
    }
  };
  auto fixup_entry = [&](const Fix& f) {  // FVC_UP_FORM 1
    if (f.nlow <= 0) return;
    for (int cmb = tid; cmb < 4 * 34 * 4; cmb += 256) {
      const int qlo = cmb & 3, rest = cmb >> 2;
      const int qhi = rest / 34, sl = rest - 34 * qhi;
      const int q = 4 * qhi + qlo;
      const int c = sl < 17 ? 2 * sl : 2 * (sl - 17) + 1;
      const int ox = 32 * f.g - 1 + c;
      if ((unsigned)ox >= (unsigned)W) continue;
      const FvcUpIdx ux = fvc_up_index_scaled(ox, a.wl, a.usx);
      const int pa = ux.i0 - f.lc0, pb = ux.i1 - f.lc0;
      const int xa = pa * kQ + (q ^ low_swz(pa)), xb = pb * kQ + (q ^ low_swz(pb));
      const bool own_c = c >= 1 && c <= 32;
      for (int ri = 0; ri < f.nr; ++ri) {
        const int r = f.r0 + ri;
        if ((unsigned)r >= (unsigned)H) continue;
        const FvcUpIdx uy = fvc_up_index_scaled(r, a.hl, a.usy);
        const int ya = (uy.i0 - f.lr0) * kLowRowEnt, yb = (uy.i1 - f.lr0) * kLowRowEnt;
        float4* const pe =
            reinterpret_cast<float4*>(ring + ((size_t)((f.sbase + ri) & (kRing - 1)) * kRowEntries + ring_entry(c, q)) * 16);
        const float4* const lw = reinterpret_cast<const float4*>(low);
        const float4 sk = *pe;
        const float4 v = fvc_lerp2d4(lw[ya + xa], lw[ya + xb], lw[yb + xa], lw[yb + xb], uy, ux);
        const float4 xs = make_float4(sk.x + v.x, sk.y + v.y, sk.z + v.z, sk.w + v.w);
        if constexpr (!(FVC_UP_KO & 8)) *pe = xs;
        if constexpr (!(FVC_UP_KO & 4)) {
          if (own_c && r >= f.own0 && r < f.own1)
            *reinterpret_cast<float4*>(a.xu + (((size_t)f.b * H + r) * W + ox) * kC + 4 * q) = xs;
        } else {
          asm volatile("" ::"v"(xs.x), "v"(xs.y), "v"(xs.z), "v"(xs.w));
        }
      }
    }
  };
  // rows ri0, ri0 + 1 of fix-up f, all of this thread's entries at once: every LDS read (the entries
  // and the low taps) is issued before the first result is formed, so the reads' latency is paid
  // once per pair of rows instead of once per entry. A fix-up's row pairs (2m + 1, 2m + 2) of a 2x
  // align_corners upsample share their two low rows (both floor to m); then (SHARED) each low row's
  // horizontal lerp a l0x + b l1x is formed once for both rows: 4 low taps per column
  // instead of 8. Invalid entries (past the 544 (column slot, quad) pairs, outside the image) read
  // a safe address and write nothing.
  // this lane's fix-up columns for column group g: (column slot, quad) pairs tid, tid + 256,
  // tid + 512 (544 in all), their ring / xu offsets, low taps and weights. They depend on the group
  // only, so they are formed when the fix-ups' group changes (once per chunk), not per item.
  struct FixCols {
    unsigned lo[3], xo[3];
    int xa[3], xb[3];
    float l0[3], l1[3];
    bool ok[3], own[3];
  };
  auto fix_cols = [&](int g, int lc0) {
    FixCols fc;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int cmb0 = tid + 256 * j;
      fc.ok[j] = cmb0 < 4 * 34 * 4;
      const int cmb = fc.ok[j] ? cmb0 : tid;
      const int qlo = cmb & 3, rest = cmb >> 2;
      const int qhi = rest / 34, sl = rest - 34 * qhi;
      const int q = 4 * qhi + qlo;
      const int c = sl < 17 ? 2 * sl : 2 * (sl - 17) + 1;
      const int ox = 32 * g - 1 + c;
      fc.ok[j] = fc.ok[j] && (unsigned)ox < (unsigned)W;
      fc.own[j] = c >= 1 && c <= 32;
      const int oxc = min(max(ox, 0), W - 1);
      const FvcUpIdx ux = fvc_up_index_scaled(oxc, a.wl, a.usx);
      const int pa = ux.i0 - lc0, pb = ux.i1 - lc0;
      fc.xa[j] = pa * kQ + (q ^ low_swz(pa));
      fc.xb[j] = pb * kQ + (q ^ low_swz(pb));
      fc.l0[j] = ux.l0;
      fc.l1[j] = ux.l1;
      fc.lo[j] = (unsigned)ring_entry(c, q) * 16u;
      fc.xo[j] = (unsigned)(oxc * kC + 4 * q) * 4u;
    }
    return fc;
  };
  FixCols fcols = {};
  int fcols_g = -1;

  auto fixup_rows = [&](const Fix& f, int ri0) {
    bool rv[2], ro[2];
    int ya[2], yb[2];
    float ly0[2], ly1[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ri = ri0 + k, r = f.r0 + ri;
      rv[k] = ri < f.nr && (unsigned)r < (unsigned)H;
      ro[k] = rv[k] && r >= f.own0 && r < f.own1;
      const FvcUpIdx uy = fvc_up_index_scaled(rv[k] ? r : max(f.r0, 0), a.hl, a.usy);
      ya[k] = __builtin_amdgcn_readfirstlane((uy.i0 - f.lr0) * kLowRowEnt);
      yb[k] = __builtin_amdgcn_readfirstlane((uy.i1 - f.lr0) * kLowRowEnt);
      ly0[k] = uy.l0;
      ly1[k] = uy.l1;
    }
    if (!rv[0] && !rv[1]) return;
    // the pair's xu rows (32-bit lane offsets; bytes past the image drop)
    const int rxf = f.r0 + ri0 + (rv[0] ? 0 : 1);
    const __amdgpu_buffer_rsrc_t rxu = rsrc(a.xu + ((size_t)f.b * H + rxf) * W * kC, (unsigned)(min(H - rxf, 2) * W) * kC * 4u);
    const float4* const lw = reinterpret_cast<const float4*>(low);
    const bool shared = rv[0] && rv[1] && ya[0] == ya[1] && yb[0] == yb[1];  // wave-uniform
    const FixCols& fc = fcols;
    const unsigned* const lo = fc.lo;
    const unsigned* const xo = fc.xo;
    const int* const xa = fc.xa;
    const int* const xb = fc.xb;
    const bool* const ok = fc.ok;
    const bool* const own = fc.own;
    FvcUpIdx ux[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ux[j].l0 = fc.l0[j];
      ux[j].l1 = fc.l1[j];
    }
    char* const rw0 = ring + (size_t)((f.sbase + ri0) & (kRing - 1)) * kRowEntries * 16;
    char* const rw1 = ring + (size_t)((f.sbase + ri0 + 1) & (kRing - 1)) * kRowEntries * 16;
    auto put = [&](int j, int k, const float4& sk, const float4& v) {
      const float4 xs = make_float4(sk.x + v.x, sk.y + v.y, sk.z + v.z, sk.w + v.w);
      if (ok[j] && rv[k]) {
        if constexpr (!(FVC_UP_KO & 8)) *reinterpret_cast<float4*>((k ? rw1 : rw0) + lo[j]) = xs;
        if constexpr (!(FVC_UP_KO & 4)) {
          if (own[j] && ro[k])
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, xs), rxu,
                                                   (unsigned)(f.r0 + ri0 + k - rxf) * (unsigned)W * kC * 4u + xo[j], 0, 0);
        } else {
          asm volatile("" ::"v"(xs.x), "v"(xs.y), "v"(xs.z), "v"(xs.w));
        }
      }
    };
    auto hlerp = [&](const float4& ta, const float4& tb, const FvcUpIdx& u) {  // fvc_lerp2d's inner steps
      return make_float4(fvc_lerp1(ta.x, tb.x, u.l0, u.l1), fvc_lerp1(ta.y, tb.y, u.l0, u.l1),
                         fvc_lerp1(ta.z, tb.z, u.l0, u.l1), fvc_lerp1(ta.w, tb.w, u.l0, u.l1));
    };
    auto vlerp = [&](const float4& h0, const float4& h1, int k) {  // = fvc_lerp2d's outer step
      return make_float4(fvc_lerp1(h0.x, h1.x, ly0[k], ly1[k]), fvc_lerp1(h0.y, h1.y, ly0[k], ly1[k]),
                         fvc_lerp1(h0.z, h1.z, ly0[k], ly1[k]), fvc_lerp1(h0.w, h1.w, ly0[k], ly1[k]));
    };
    if (shared) {
      float4 t[3][6];  // two entries, then the four taps
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        t[j][0] = *reinterpret_cast<const float4*>(rw0 + lo[j]);
        t[j][1] = *reinterpret_cast<const float4*>(rw1 + lo[j]);
        t[j][2] = lw[ya[0] + xa[j]];
        t[j][3] = lw[ya[0] + xb[j]];
        t[j][4] = lw[yb[0] + xa[j]];
        t[j][5] = lw[yb[0] + xb[j]];
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float4 h0 = hlerp(t[j][2], t[j][3], ux[j]), h1 = hlerp(t[j][4], t[j][5], ux[j]);
        put(j, 0, t[j][0], vlerp(h0, h1, 0));
        put(j, 1, t[j][1], vlerp(h0, h1, 1));
      }
    } else {
      float4 t[3][2][5];
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          t[j][k][0] = *reinterpret_cast<const float4*>((k ? rw1 : rw0) + lo[j]);
          t[j][k][1] = lw[ya[k] + xa[j]];
          t[j][k][2] = lw[ya[k] + xb[j]];
          t[j][k][3] = lw[yb[k] + xa[j]];
          t[j][k][4] = lw[yb[k] + xb[j]];
        }
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int k = 0; k < 2; ++k)
          put(j, k, t[j][k][0], vlerp(hlerp(t[j][k][1], t[j][k][2], ux[j]), hlerp(t[j][k][3], t[j][k][4], ux[j]), k));
    }
  };
  auto fixup = [&](const Fix& f) {
    if constexpr ((FVC_UP_KO & 1) != 0) return;
    if (f.nlow <= 0) return;
    if constexpr (FVC_UP_FORM == 1) {
      fixup_entry(f);
      return;
    }
    if (f.g != fcols_g) {  // wave-uniform: a new column group (at most once per chunk)
      fcols = fix_cols(f.g, f.lc0);
      fcols_g = f.g;
    }
    fixup_rows(f, 0);
    if (f.nr > 2) fixup_rows(f, 2);
  };

  // the block knows its current and next chunk; the first item of every chunk takes the one
  // after (thread 0, into LDS word 2 + parity, decoded by everyone after that item's barrier)
  if (tid == 0) {
    sq[0] = take(0);
    sq[1] = take(1);
  }
  __syncthreads();
  Pos cur = decode(sq[0]);
  Pos nxt = decode(sq[1]);
  Pos nnp{0, 0, 0, 0};
  int ntaken = 2;

  // overflow check: 0 * (pre-activation output) summed over every output; a transformed input
  // >= 65520 rounds to an infinite hi part whose products reach the outputs as inf / NaN
  f2v chk2 = {0.f, 0.f};  // overflow check, two channels per instruction
  float mxy = 0.f;  // kPostTap: max |y| (y is split into fp16 halves for the tap GEMM)
  // the lane's output byte offsets within an item's 2-row band of column group g, and within a
  // pooled row (past the band for columns outside the image)
  const int cbase = 16 * wave + 4 * o;
  const int Hp = H >> 1, Wp = W >> 1;
  unsigned yo[2][2], po = 0;
  auto out_offsets = [&](int g) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ox = 32 * g + 2 * t + j;
#pragma unroll
      for (int i = 0; i < 2; ++i) yo[i][j] = ox < W ? (unsigned)((i * W + ox) * a.yp + cbase) * 4u : kOob;
    }
    if constexpr (POST == kPostPool) {
      const int px = 16 * g + t;
      po = px < Wp ? (unsigned)(px * kC + cbase) * 4u : kOob;
    }
  };
  unsigned vo_cur[3];
  // image bases of the current chunk (x, the output y / tap partials P, the residual)
  const unsigned ype = POST == kPostTap ? (unsigned)a.pcp : (unsigned)a.yp;
  const size_t ximg_e = (size_t)H * W * a.xp, yimg_e = (size_t)H * W * ype;
  const float* xi_cur = a.x + (size_t)cur.b * ximg_e;
  float* yi_cur = a.y + (size_t)cur.b * yimg_e;
  const float* ri_cur = RES ? a.res + (size_t)cur.b * H * W * a.yp : nullptr;

  if (cur.ty0 < cur.ty1) {
    // first item of the block: its whole 4-row window into ring slots 0..3
    row_offsets(cur.g, vo_cur);
    out_offsets(cur.g);
    for (int i = 0; i < 4; ++i) stage_row(xi_cur, 2 * cur.ty0 - 1 + i, i, vo_cur);
    Fix f0 = {};
    if constexpr (UP) {
      f0 = make_fix(cur, cur.ty0, false, 0);
      stage_low(f0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (UP) {
      fixup(f0);
      __syncthreads();
    }
    int ty = cur.ty0;
    int base = 0;  // ring slot of the current item's first row
    int zb = 0;    // Z buffer
    for (;;) {
      const bool first = ty == cur.ty0;
      const bool cont = ty + 1 < cur.ty1;  // the next item continues down this column: 2 new rows
      const Pos& np = cont ? cur : nxt;
      const int nty = cont ? ty + 1 : nxt.ty0;
      const bool nvalid = cont || nxt.ty0 < nxt.ty1;
      const int nbase = (base + (cont ? 2 : 4)) & (kRing - 1);
      Fix nf = {};  // UP: the fix-up of the next item's new rows (nothing when there is no next item)
      if constexpr (UP) {
        if (nvalid) nf = make_fix(np, nty, cont, nbase);
      }
      // the next item's new input rows (2, or 4 after a chunk change), issued between the MFMA
      // blocks of the k-loop (k-th pair of rows at point k) where their issue cost overlaps them
      auto stage_next = [&](int k) {
        if constexpr (FVC_WINO_KO & 64) return;  // knock-out: no staging of the next item's rows
        if (!nvalid) return;
        if (k == 0 && cont) return;
        const int i0 = 2 * k;
        if (cont) {
          for (int i = i0; i < i0 + 2; ++i) stage_row(xi_cur, 2 * nty - 1 + i, (nbase + i) & (kRing - 1), vo_cur);
        } else {
          unsigned vo[3];
          row_offsets(np.g, vo);
          const float* xi_np = a.x + (size_t)np.b * ximg_e;
          for (int i = i0; i < i0 + 2; ++i) stage_row(xi_np, 2 * nty - 1 + i, (nbase + i) & (kRing - 1), vo);
        }
        if constexpr (UP) {
          if (k == 1) stage_low(nf);
        }
      };
      if (first && tid == 0) sq[2 + (ntaken & 1)] = take(ntaken);  // chunk after next

      // this lane's 4 output pixels in the finishing pass (channels 16 wave + 4 o .. +3): one
      // descriptor per item over its 2-row band (1 row at an odd image's last tile row); the
      // residual is loaded now so its latency hides behind the k-loop
      const unsigned band_rows = 2 * ty + 1 < H ? 2u : 1u;
      const unsigned band_bytes = band_rows * yrow_bytes;
      const __amdgpu_buffer_rsrc_t ry = rsrc(yi_cur + (size_t)(unsigned)(2 * ty) * ((unsigned)W * ype),
                                             band_rows * (unsigned)W * ype * 4u);
      f32x4 rv[2][2];
      if constexpr (RES) {
        const __amdgpu_buffer_rsrc_t rr = rsrc(ri_cur + (size_t)(unsigned)(2 * ty) * ((unsigned)W * a.yp), band_bytes);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            rv[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, yo[i][j], 0, 0));
      }

      // ---- k-loop: 2 steps of 32 input channels, 48 MFMAs each
      f32x4 acc[4][4], cor[4][4];
      const char* rowa = ring + (size_t)((base + ra) & (kRing - 1)) * kRowEntries * 16;
      const char* rowb = ring + (size_t)((base + rb) & (kRing - 1)) * kRowEntries * 16;
      // software-pipelined: the next k-step's LDS reads and transform sit between this k-step's
      // MFMA blocks (source order is issue order around the asm blocks)
      auto read_raw = [&](int kk, int hh, float4 (&da)[4], float4 (&db)[4]) {
        (void)pix_b;
        // patch columns 0..3 of tile t: slots t, 17 + t, t + 1, 18 + t (even / odd column halves)
        const int Q = 8 * kk + 2 * o + hh;
        int e[4];
        if constexpr (kPix) {  // = ring_entry(2t + d, Q) * 16: (8 kk + hh) ^ (2 o ^ swizzle), per-lane parts hoisted
          const int cq = (8 * kk + hh) * 16;
          e[0] = pix_b + (cq ^ pix_x0);
          e[1] = e[0] + 256;
          e[2] = pix_b + 512 + (cq ^ pix_x1);
          e[3] = e[2] + 256;
        } else {
          const int e0 = (Q * kSlots + t) * 16;
          e[0] = e0;
          e[1] = e0 + 17 * 16;
          e[2] = e0 + 16;
          e[3] = e0 + 18 * 16;
        }
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          da[d] = *reinterpret_cast<const float4*>(rowa + e[d]);
          db[d] = *reinterpret_cast<const float4*>(rowb + e[d]);
        }
      };
      // V[q] = E B of the lane's tile for 4 channels (E = d[ra] + sb d[rb]), two channels per packed
      // instruction (v_pk_fma_f32 / v_pk_add_f32; a lone wave issues one VALU per ~4 cycles whether
      // packed or not: packing the transform, the column combination and the finishing pass, the
      // parts outside the MFMA blocks, gained 2-3 %, profiles/r4/wino_pk)
      auto transform_pk = [&](const float4 (&da)[4], const float4 (&db)[4], int hh, float (&v)[4][8]) {
        const f2v sb2 = {sb, sb};
#pragma unroll
        for (int cp = 0; cp < 2; ++cp) {
          f2v e[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            f2v xa = cp ? f2v{da[jj].z, da[jj].w} : f2v{da[jj].x, da[jj].y};
            f2v xb = cp ? f2v{db[jj].z, db[jj].w} : f2v{db[jj].x, db[jj].y};
            if constexpr (IOP == FVC_IN_RELU) {
              xa = f2v{relu1(xa.x), relu1(xa.y)};
              xb = f2v{relu1(xb.x), relu1(xb.y)};
            }
            e[jj] = __builtin_elementwise_fma(sb2, xb, xa);
          }
          const f2v q0 = e[0] - e[2], q1 = e[1] + e[2], q2 = e[2] - e[1], q3 = e[1] - e[3];
          v[0][4 * hh + 2 * cp] = q0.x; v[0][4 * hh + 2 * cp + 1] = q0.y;
          v[1][4 * hh + 2 * cp] = q1.x; v[1][4 * hh + 2 * cp + 1] = q1.y;
          v[2][4 * hh + 2 * cp] = q2.x; v[2][4 * hh + 2 * cp + 1] = q2.y;
          v[3][4 * hh + 2 * cp] = q3.x; v[3][4 * hh + 2 * cp + 1] = q3.y;
        }
      };
      auto split_all = [&](const float (&v)[4][8], h8 (&vh)[4], h8 (&vl)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          unsigned hw[4], lw[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            split2(v[q][2 * i], v[q][2 * i + 1], hw[i], lw[i]);
          }
          vh[q] = __builtin_bit_cast(h8, v4u{hw[0], hw[1], hw[2], hw[3]});
          vl[q] = __builtin_bit_cast(h8, v4u{lw[0], lw[1], lw[2], lw[3]});
        }
      };
      auto mfma_q1 = [&](int q, const h8 (&vh)[4], const h8 (&vl)[4]) {  // k-step 1 of position q
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          if (n == 0 || kAllNop) wino_mfma3<false, true>(acc[q][n], cor[q][n], u[q][n][1][0], u[q][n][1][1], vh[q], vl[q]);
          else wino_mfma3<false, false>(acc[q][n], cor[q][n], u[q][n][1][0], u[q][n][1][1], vh[q], vl[q]);
        }
      };
      float v0[4][8], v1[4][8];
      h8 vh0[4], vl0[4], vh1[4], vl1[4];
      // LDS reads one channel half ahead of their transform (two raw buffers): each batch of
      // ds_reads is in flight while the previous half is transformed instead of waited for
      float4 da[4], db[4], ea[4], eb[4];
      read_raw(0, 0, da, db);
      read_raw(0, 1, ea, eb);
      transform_pk(da, db, 0, v0);
      read_raw(1, 0, da, db);
      transform_pk(ea, eb, 1, v0);
      read_raw(1, 1, ea, eb);
      split_all(v0, vh0, vl0);
      transform_pk(da, db, 0, v1);
      stage_next(0);
      transform_pk(ea, eb, 1, v1);
      unsigned hw1[4][4], lw1[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int n = 0; n < 4; ++n)
          if constexpr (FVC_WINO_KO & 2) {
            split2(v1[n][2 * q], v1[n][2 * q + 1], hw1[n][q], lw1[n][q]);
            acc[q][n] = cor[q][n] = f32x4{0.f, 0.f, 0.f, 0.f};
            asm volatile("" : "+v"(acc[q][n]) : "v"(vh0[q]), "v"(vl0[q]));
          } else {
          ((q == 0 && n == 0) || kAllNop ? wino_mfma3_split<true> : wino_mfma3_split<false>)(acc[q][n], cor[q][n], u[q][n][0][0], u[q][n][0][1], vh0[q], vl0[q], v1[n][2 * q],
                           v1[n][2 * q + 1], hw1[n][q], lw1[n][q]);
          }
        if (q == 1) stage_next(1);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        vh1[q] = __builtin_bit_cast(h8, v4u{hw1[q][0], hw1[q][1], hw1[q][2], hw1[q][3]});
        vl1[q] = __builtin_bit_cast(h8, v4u{lw1[q][0], lw1[q][1], lw1[q][2], lw1[q][3]});
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (FVC_WINO_KO & 1) {
          asm volatile("" : "+v"(acc[q][0]), "+v"(cor[q][0]) : "v"(vh1[q]), "v"(vl1[q]));
        } else {
          mfma_q1(q, vh1, vl1);
        }
      }
      wino_mfma_drain(acc, cor);

      // ---- column combination Z[r][j] = sum_q M[r][q] A[q][j] (M in units of 2^kw: the scale is
      // applied once on Y) -> LDS plane (r, j, n), lane-linear
      char* const zw = zbuf + zb * kZBytes;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        f32x4 z0, z1;
        const f2v ls2 = {1.f / kLoScale, 1.f / kLoScale};
#pragma unroll
        for (int cp = 0; cp < 2; ++cp) {
          f2v m[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f2v c2 = cp ? f2v{cor[q][n][2], cor[q][n][3]} : f2v{cor[q][n][0], cor[q][n][1]};
            const f2v a2 = cp ? f2v{acc[q][n][2], acc[q][n][3]} : f2v{acc[q][n][0], acc[q][n][1]};
            m[q] = __builtin_elementwise_fma(c2, ls2, a2);
          }
          const f2v p0 = (m[0] + m[1]) + m[2], p1 = (m[1] - m[2]) - m[3];
          z0[2 * cp] = p0.x; z0[2 * cp + 1] = p0.y;
          z1[2 * cp] = p1.x; z1[2 * cp + 1] = p1.y;
        }
        *reinterpret_cast<f32x4*>(zw + ((wave * 2 + 0) * 4 + n) * 1024 + lane * 16) = z0;
        *reinterpret_cast<f32x4*>(zw + ((wave * 2 + 1) * 4 + n) * 1024 + lane * 16) = z1;
      }
#if FVC_WINO_KO_WAIT
      asm volatile("" ::: "memory");  // knock-out (experiment builds only): no wait for the next item's rows
#else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces of the next item
#endif
      if constexpr (!(FVC_WINO_KO & 4)) __syncthreads();
      if (first) nnp = decode(sq[2 + (ntaken & 1)]);  // published by this item's barrier
      if constexpr (UP && FVC_UP_FIRST) fixup(nf);  // experiment: the fix-up before the finishing pass

      // ---- finishing pass: wave w -> output channels 16w..16w+15 of the item's 16 tiles
      if constexpr (!(FVC_WINO_KO & 8)) {
      f32x4 z[4][2];
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if constexpr (FVC_WINO_KO & 32) {
            z[p][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            asm volatile("" : "+v"(z[p][j]));
          } else {
            z[p][j] = *reinterpret_cast<const f32x4*>(zw + ((p * 2 + j) * 4 + wave) * 1024 + lane * 16);
          }
      const f32x4 bj = *reinterpret_cast<const f32x4*>(sbias + cbase);
      f32x4 yv[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 vv;
#pragma unroll
          for (int cp = 0; cp < 2; ++cp) {
            auto pr = [&](const f32x4& x) { return cp ? f2v{x[2], x[3]} : f2v{x[0], x[1]}; };
            const f2v ys = i == 0 ? (pr(z[0][j]) + pr(z[1][j])) + pr(z[2][j]) : (pr(z[1][j]) - pr(z[2][j])) - pr(z[3][j]);
            chk2 = __builtin_elementwise_fma(ys, f2v{0.f, 0.f}, chk2);
            f2v tv = __builtin_elementwise_fma(ys, f2v{a.osc, a.osc}, pr(bj));
            if constexpr (RES == kResPre) tv += pr(rv[i][j]);
            if constexpr (ACT == FVC_ACT_RELU) tv = f2v{relu1(tv.x), relu1(tv.y)};
            if constexpr (ACT == FVC_ACT_LRELU) {
              const f2v t1 = tv * f2v{0.1f, 0.1f};
              tv = f2v{fmaxf(tv.x, t1.x), fmaxf(tv.y, t1.y)};
            }
            if constexpr (RES == kResPost) tv += pr(rv[i][j]);
            vv[2 * cp] = tv.x;
            vv[2 * cp + 1] = tv.y;
          }
          yv[i][j] = vv;
          if constexpr (POST != kPostTap) {
            if constexpr (FVC_WINO_KO & 16) asm volatile("" ::"v"(vv));
            else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, vv), ry, yo[i][j], 0, FVC_STORE_AUX);
          }
        }
      if constexpr (POST == kPostPool) {
        f32x4 pv;
#pragma unroll
        for (int c = 0; c < 4; ++c) pv[c] = (((yv[0][0][c] + yv[0][1][c]) + yv[1][0][c]) + yv[1][1][c]) / 4.f;
        const __amdgpu_buffer_rsrc_t rp =
            rsrc(a.pool + ((size_t)cur.b * Hp + ty) * Wp * kC, ty < Hp ? (unsigned)Wp * kC * 4u : 0u);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, pv), rp, po, 0, 0);
      }
      if constexpr (POST == kPostTap) {
        // y never reaches HBM: each wave parks its 16 channels of the item's 64 pixels in its own
        // planes of this item's Z buffer (no other wave read them), then wave v multiplies the
        // 64-channel y of pixel (i, j) = (v >> 1, v & 1) of the 16 tiles with the next layer's tap
        // weights: P [16 partials x 16 tiles] per row tile on v_mfma_f32_16x16x32_f16, split
        // precision (main = T_hi y_hi, corr = T_lo y_hi + T_hi y_lo), P = main 2^-kt + corr 2^-kt-11.
        // Z(zb) is next written two items later, behind the next item's barrier.
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            *reinterpret_cast<f32x4*>(zw + ((i * 2 + j) * 4 + wave) * 1024 + lane * 16) = yv[i][j];
#pragma unroll
            for (int c = 0; c < 4; ++c) mxy = fmaxf(mxy, fabsf(yv[i][j][c]));
          }
        __syncthreads();
        const int pi = wave >> 1, pj = wave & 1;
        h8 th[2], tl[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          // B operand: lane (t, q = lane >> 4) holds channels 32 kk + 8 q .. + 7 of tile t = quads
          // 2 (q & 1), +1 of wave 2 kk + (q >> 1)
          const char* src = zw + ((pi * 2 + pj) * 4 + 2 * kk + (lane >> 5)) * 1024 + ((2 * ((lane >> 4) & 1)) * 16 + t) * 16;
          const f32x4 q0 = *reinterpret_cast<const f32x4*>(src);
          const f32x4 q1 = *reinterpret_cast<const f32x4*>(src + 256);
          unsigned hw[4], lw[4];
          split2(q0[0], q0[1], hw[0], lw[0]);
          split2(q0[2], q0[3], hw[1], lw[1]);
          split2(q1[0], q1[1], hw[2], lw[2]);
          split2(q1[2], q1[3], hw[3], lw[3]);
          th[kk] = __builtin_bit_cast(h8, v4u{hw[0], hw[1], hw[2], hw[3]});
          tl[kk] = __builtin_bit_cast(h8, v4u{lw[0], lw[1], lw[2], lw[3]});
        }
        const int ox = 32 * cur.g + 2 * t + pj;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          f32x4 pa = {0.f, 0.f, 0.f, 0.f}, pc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const uint4* const tw = a.tw + (size_t)((rt * 2 + kk) * 2) * 64 + lane;
            const h8 wh = __builtin_bit_cast(h8, tw[0]);
            const h8 wl = __builtin_bit_cast(h8, tw[64]);
            pa = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, th[kk], pa, 0, 0, 0);
            pc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, th[kk], pc, 0, 0, 0);
            pc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, tl[kk], pc, 0, 0, 0);
          }
          const int p0 = rt * 16 + 4 * (lane >> 4);
          f32x4 o;
#pragma unroll
          for (int c = 0; c < 4; ++c) o[c] = fmaf(pc[c], a.tosc_c, pa[c] * a.tosc);
          const unsigned so = (ox < W && p0 < a.pcp) ? (unsigned)((pi * W + ox) * a.pcp + p0) * 4u : kOob;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, o), ry, so, 0, 0);
        }
      }

      }  // FVC_WINO_KO & 8

      if constexpr (UP) {  // the next item's new rows: S -> X in place (and to xu), then published
        if constexpr (!FVC_UP_FIRST) fixup(nf);
        if constexpr (!(FVC_UP_KO & 2)) __syncthreads();
      }

      // ---- advance
      if (!nvalid) break;
      if (!cont) {
        cur = nxt;
        nxt = nnp;
        ++ntaken;
        row_offsets(cur.g, vo_cur);
        out_offsets(cur.g);
        xi_cur = a.x + (size_t)cur.b * ximg_e;
        yi_cur = a.y + (size_t)cur.b * yimg_e;
        if constexpr (RES != 0) ri_cur = a.res + (size_t)cur.b * H * W * a.yp;
      }
      ty = nty;
      base = nbase;
      if constexpr (!UP) zb ^= 1;
    }
  }
  {
    if ((chk2.x != 0.f || chk2.y != 0.f || !(mxy < 65000.f)) && a.ovf) atomicOr(a.ovf, 1);
  }
  if (a.sched && tid == 0) {
    __threadfence();
    const int nblk = (int)gridDim.x;
    if (atomicAdd(a.sched, 1) == nblk - 1) {
      atomicExch(a.sched + 1, 0);
      atomicExch(a.sched, 0);
    }
  }
}

static int wino_num_cus() {
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

template <int IOP, int POST, int RES, int ACT, bool UP = false>
static int wino_launch4(const WinoArgs& a, int grid, hipStream_t s) {
  const int lds = UP ? kLdsUp : kLds;
  const hipError_t e = hipFuncSetAttribute((const void*)conv_wino_kernel<IOP, POST, RES, ACT, UP>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((conv_wino_kernel<IOP, POST, RES, ACT, UP>), dim3(grid), dim3(256), lds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

// the fused upsample-add input form: plain conv (no residual, no pool / tap epilogue)
template <int IOP>
static int wino_launch_up(const WinoArgs& a, int act, hipStream_t s, int grid) {
  if (act == FVC_ACT_NONE) return wino_launch4<IOP, 0, 0, FVC_ACT_NONE, true>(a, grid, s);
  if (act == FVC_ACT_RELU) return wino_launch4<IOP, 0, 0, FVC_ACT_RELU, true>(a, grid, s);
  return wino_launch4<IOP, 0, 0, FVC_ACT_LRELU, true>(a, grid, s);
}

// instantiated: Warp_net's forms (ResBlock conv1: ReLU in, ReLU act; conv2: residual, with or
// without the pool), plus no-activation / LeakyReLU plain convs for the general entry point
template <int IOP, int POST>
static int wino_launch(const WinoArgs& a, int act, hipStream_t s, int grid) {
  if constexpr (POST == kPostTap && IOP != FVC_IN_NONE) return FVC_EINVAL;
  if (a.res) {
    if (act == FVC_ACT_NONE) return wino_launch4<IOP, POST, kResPost, FVC_ACT_NONE>(a, grid, s);
    if (act == FVC_ACT_RELU) return wino_launch4<IOP, POST, kResPost, FVC_ACT_RELU>(a, grid, s);
    return wino_launch4<IOP, POST, kResPost, FVC_ACT_LRELU>(a, grid, s);
  }
  if (act == FVC_ACT_NONE) return wino_launch4<IOP, POST, 0, FVC_ACT_NONE>(a, grid, s);
  if (act == FVC_ACT_RELU) return wino_launch4<IOP, POST, 0, FVC_ACT_RELU>(a, grid, s);
  return wino_launch4<IOP, POST, 0, FVC_ACT_LRELU>(a, grid, s);
}

// the second input half of a 128 -> 128 quarter pair: residual (the first half's partial sum)
// added before the activation
template <int IOP>
static int wino_launch_pre(const WinoArgs& a, int act, hipStream_t s, int grid) {
  if (act == FVC_ACT_NONE) return wino_launch4<IOP, 0, kResPre, FVC_ACT_NONE>(a, grid, s);
  if (act == FVC_ACT_RELU) return wino_launch4<IOP, 0, kResPre, FVC_ACT_RELU>(a, grid, s);
  return wino_launch4<IOP, 0, kResPre, FVC_ACT_LRELU>(a, grid, s);
}

// pitch = 128: x / y / res point at the first channel of a 64-channel half of 128-channel tensors;
// res_pre adds res before the activation (bias may then be null: zeros)
static int run_wino(const float* x, const void* upack, float osc, const float* bias, const float* res, float* y,
                    float* pool, int batch, int h, int w, int in_op, int act, int cu_reserve, int* ovf, int* sched,
                    int sched_len, hipStream_t s, const void* tw = nullptr, float tosc = 0.f, int pcp = 0,
                    int pitch = kC, bool res_pre = false, const float* xl = nullptr, float* xu = nullptr) {
  if (tw && (pool || in_op != FVC_IN_NONE || pcp <= 0 || pcp > 32 || (pcp & 3))) return FVC_EINVAL;
  // UP: x is the skip S, xl the half-resolution source, xu receives S + up2(xl)
  if ((xl != nullptr) != (xu != nullptr)) return FVC_EINVAL;
  if (xl && (tw || pool || res || pitch != kC || (h & 1) || (w & 1))) return FVC_EINVAL;
  if (!x || !upack || (!bias && pitch == kC) || !y || batch <= 0 || h <= 0 || w <= 0 || cu_reserve < 0 ||
      sched_len < 0)
    return FVC_EINVAL;
  if (pitch != kC && (pitch != 2 * kC || tw || pool)) return FVC_EINVAL;
  if (res_pre && (!res || pitch != 2 * kC)) return FVC_EINVAL;
  if (in_op != FVC_IN_NONE && in_op != FVC_IN_RELU) return FVC_EINVAL;
  // every buffer descriptor spans one input row or one 2-row output band: 32-bit offsets hold
  // for any batch, only a band must stay below 4 GB
  if ((unsigned long long)w * pitch * 4ull * 2ull >= (1ull << 31)) return FVC_EINVAL;
  WinoArgs a;
  a.x = x;
  a.u = (const uint4*)upack;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.pool = pool;
  a.B = batch;
  a.H = h;
  a.W = w;
  a.tiles_y = (h + 1) / 2;
  a.ngroups = fvc_cdiv(w, 32);
  // 16 tile rows per chunk. Longer chunks re-stage fewer halo rows (a chunk's first item stages 4
  // rows, later ones 2): FVC_WINO_CHUNK=32 (experiments) measured equal on the 1088x1920 and
  // 544x960 layers and 4-5 % slower on the 272x480 quarters (profiles/r6/wino_ko/chunk.txt).
  // The result does not depend on it.
  a.chunk = env_int("FVC_WINO_CHUNK", kChunkMin) == kChunkMax ? kChunkMax : kChunkMin;
  a.chunks_per_col = fvc_cdiv(a.tiles_y, a.chunk);
  a.nchunks = batch * a.ngroups * a.chunks_per_col;
  a.osc = osc;
  a.osc_c = osc * (1.0f / 2048.f);
  a.ovf = ovf;
  a.tw = (const uint4*)tw;
  a.tosc = tosc;
  a.tosc_c = tosc * (1.0f / 2048.f);
  a.pcp = pcp;
  a.xp = a.yp = pitch;
  a.xl = xl;
  a.xu = xu;
  a.hl = h / 2;
  a.wl = w / 2;
  // ATen's align_corners=True scale (in - 1) / (out - 1), as k_up2_add_q16p computes it
  a.usy = h > 1 ? (float)(a.hl - 1) / (float)(h - 1) : 0.f;
  a.usx = w > 1 ? (float)(a.wl - 1) / (float)(w - 1) : 0.f;
  const int reserve = env_int("FVC_X3_RESERVE", -1) >= 0 ? env_int("FVC_X3_RESERVE", 0) : cu_reserve;
  const int ncu = wino_num_cus() - (reserve < wino_num_cus() / 2 ? reserve : wino_num_cus() / 2);
  int grid = ncu < a.nchunks ? ncu : a.nchunks;
  a.sched = (sched && sched_len >= 2 && env_int("FVC_X3_DYN", 1)) ? sched : nullptr;
  if (act != FVC_ACT_NONE && act != FVC_ACT_RELU && act != FVC_ACT_LRELU) return FVC_EINVAL;
  if (tw) return wino_launch<FVC_IN_NONE, kPostTap>(a, act, s, grid);
  if (xl) {
    if (in_op == FVC_IN_NONE) return wino_launch_up<FVC_IN_NONE>(a, act, s, grid);
    return wino_launch_up<FVC_IN_RELU>(a, act, s, grid);
  }
  if (res_pre) {
    if (in_op == FVC_IN_NONE) return wino_launch_pre<FVC_IN_NONE>(a, act, s, grid);
    return wino_launch_pre<FVC_IN_RELU>(a, act, s, grid);
  }
  if (pool) {
    if (in_op == FVC_IN_NONE) return wino_launch<FVC_IN_NONE, kPostPool>(a, act, s, grid);
    return wino_launch<FVC_IN_RELU, kPostPool>(a, act, s, grid);
  }
  if (in_op == FVC_IN_NONE) return wino_launch<FVC_IN_NONE, 0>(a, act, s, grid);
  return wino_launch<FVC_IN_RELU, 0>(a, act, s, grid);
}

static int x3w_kw(const double* u, size_t n) {
  double mx = 0.0;
  for (size_t i = 0; i < n; ++i) mx = fabs(u[i]) > mx ? fabs(u[i]) : mx;
  if (!(mx > 0.0) || !isfinite(mx)) return 0;
  int e;
  frexp(mx, &e);
  const int kw = 14 - e;  // mx * 2^kw in [2^13, 2^14)
  return kw < -100 ? -100 : (kw > 100 ? 100 : kw);
}

}  // namespace

extern "C" {

int fvc_conv_wino_supported(int cin, int cout, int ksize, int stride, int transposed) {
  return cin == kC && cout == kC && ksize == 3 && stride == 1 && !transposed;
}

size_t fvc_conv_wino_wpack_bytes(void) { return (size_t)16 * kC * kC * 2 * 2; }

// w: [64][64][3][3] (OIHW, fp32). U[p = (r, q)][ci][co] = (G g G^T)[r][q] in double, scaled by 2^kw,
// split into fp16 hi / lo*2^11 and laid out per wave r as [q][n][kk][plane][lane][8]: lane l holds
// output channel 16n + (l & 15), input channels 32kk + 8(l >> 4) + 0..7 (the MFMA A operand).
int fvc_conv_wino_pack_weight(const float* w, void* wp, float* osc_out) {
  if (!w || !wp || !osc_out) return FVC_EINVAL;
  static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  double* U = (double*)malloc(sizeof(double) * 16 * kC * kC);  // [p][co][ci]
  if (!U) return FVC_EINVAL;
  for (int co = 0; co < kC; ++co)
    for (int ci = 0; ci < kC; ++ci) {
      const float* g = w + ((size_t)co * kC + ci) * 9;
      double tmp[4][3];  // G g
      for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 3; ++k) tmp[i][k] = G[i][0] * g[0 * 3 + k] + G[i][1] * g[1 * 3 + k] + G[i][2] * g[2 * 3 + k];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
          U[((size_t)(i * 4 + j) * kC + co) * kC + ci] = tmp[i][0] * G[j][0] + tmp[i][1] * G[j][1] + tmp[i][2] * G[j][2];
    }
  const int kw = x3w_kw(U, (size_t)16 * kC * kC);
  const double sc = ldexp(1.0, kw);
  *osc_out = ldexpf(1.f, -kw);
  _Float16* out = (_Float16*)wp;
  for (int r = 0; r < 4; ++r)
    for (int q = 0; q < 4; ++q)
      for (int n = 0; n < 4; ++n)
        for (int kk = 0; kk < 2; ++kk)
          for (int lane = 0; lane < 64; ++lane) {
            const int co = 16 * n + (lane & 15);
            for (int e = 0; e < 8; ++e) {
              const int ci = 32 * kk + 8 * (lane >> 4) + e;
              const float v = (float)(U[((size_t)(r * 4 + q) * kC + co) * kC + ci] * sc);
              const _Float16 hi = (_Float16)v;
              const size_t base = ((((((size_t)r * 4 + q) * 4 + n) * 2 + kk) * 2) * 64 + lane) * 8;
              out[base + e] = hi;                                               // plane 0
              out[base + 64 * 8 + e] = (_Float16)((v - (float)hi) * 2048.f);   // plane 1
            }
          }
  free(U);
  return 0;
}

size_t fvc_wino_tap_wpack_bytes(int np) { return np > 0 && np <= 32 ? (size_t)2 * 2 * 2 * 64 * 16 : 0; }

// T [np][64] (row t*cout' + co of the next layer's tap-partial form) -> [row tile][k-step][hi|lo][lane]
// 16-B fragments: lane l holds row 16 rt + (l & 15), channels 32 kk + 8 (l >> 4) + 0..7 (the
// v_mfma_f32_16x16x32_f16 A operand), scaled by 2^kt (max |T| 2^kt in [2^13, 2^14))
int fvc_wino_tap_pack_weight(const float* w, void* wp, float* osc_out, int np) {
  if (!w || !wp || !osc_out || !fvc_wino_tap_wpack_bytes(np)) return FVC_EINVAL;
  double mx = 0.0;
  for (int i = 0; i < np * kC; ++i) mx = fabs((double)w[i]) > mx ? fabs((double)w[i]) : mx;
  int kt = 0;
  if (mx > 0.0 && isfinite(mx)) {
    int e;
    frexp(mx, &e);
    kt = 14 - e;
    kt = kt < -100 ? -100 : (kt > 100 ? 100 : kt);
  }
  const float sc = ldexpf(1.f, kt);
  *osc_out = ldexpf(1.f, -kt);
  _Float16* out = (_Float16*)wp;
  for (int rt = 0; rt < 2; ++rt)
    for (int kk = 0; kk < 2; ++kk)
      for (int lane = 0; lane < 64; ++lane) {
        const int r = rt * 16 + (lane & 15);
        for (int e = 0; e < 8; ++e) {
          const int ci = 32 * kk + 8 * (lane >> 4) + e;
          const float v = r < np ? w[(size_t)r * kC + ci] * sc : 0.f;
          const _Float16 hi = (_Float16)v;
          const size_t base = ((size_t)((rt * 2 + kk) * 2) * 64 + lane) * 8;
          out[base + e] = hi;
          out[base + 64 * 8 + e] = (_Float16)((v - (float)hi) * 2048.f);
        }
      }
  return 0;
}

int fvc_conv2d_nhwc_wino_tap(const float* x, const void* wpack, float osc, const float* bias, const float* res,
                             float* P, int batch, int h, int w, int act, const void* tap_wpack, float tap_osc, int pcp,
                             int cu_reserve, int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream) {
  if (!tap_wpack) return FVC_EINVAL;
  return run_wino(x, wpack, osc, bias, res, P, nullptr, batch, h, w, FVC_IN_NONE, act, cu_reserve, overflow_flag,
                  sched, sched_len, (hipStream_t)stream, tap_wpack, tap_osc, pcp);
}

int fvc_conv_wino128_supported(int cin, int cout, int ksize, int stride, int transposed) {
  return cin == 2 * kC && cout == 2 * kC && ksize == 3 && stride == 1 && !transposed;
}

size_t fvc_conv_wino128_wpack_bytes(void) { return 4 * fvc_conv_wino_wpack_bytes(); }

// w: [128][128][3][3] (OIHW) -> four 64 -> 64 packs, quarter (co half, ci half) at index
// 2 * co_half + ci_half, each with its own scale (osc4[quarter])
int fvc_conv_wino128_pack_weight(const float* w, void* wp, float* osc4) {
  if (!w || !wp || !osc4) return FVC_EINVAL;
  float* qw = (float*)malloc(sizeof(float) * kC * kC * 9);
  if (!qw) return FVC_EINVAL;
  for (int qd = 0; qd < 4; ++qd) {
    const int oh = qd >> 1, ih = qd & 1;
    for (int co = 0; co < kC; ++co)
      for (int ci = 0; ci < kC; ++ci)
        for (int k = 0; k < 9; ++k)
          qw[((size_t)co * kC + ci) * 9 + k] = w[(((size_t)(kC * oh + co)) * 2 * kC + kC * ih + ci) * 9 + k];
    const int r = fvc_conv_wino_pack_weight(qw, (char*)wp + qd * fvc_conv_wino_wpack_bytes(), osc4 + qd);
    if (r) {
      free(qw);
      return r;
    }
  }
  free(qw);
  return 0;
}

// A 128 -> 128 3x3 stride-1 conv as four 64 -> 64 Winograd launches: per output half, the first
// input half's sum (no bias, no activation) is written into y's half, then the second input half
// adds bias and that partial sum before the activation (in place: each lane reads its residual
// and writes the same bytes). Same stream order, no extra buffer.
int fvc_conv2d_nhwc_wino128(const float* x, const void* wpack, const float* osc4, const float* bias, float* y,
                            int batch, int h, int w, int in_op, int act, int cu_reserve, int* overflow_flag,
                            int* sched, int sched_len, fvc_stream_t stream) {
  if (!x || !wpack || !osc4 || !bias || !y) return FVC_EINVAL;
  const size_t qb = fvc_conv_wino_wpack_bytes();
  for (int oh = 0; oh < 2; ++oh) {
    float* yh = y + kC * oh;
    int r = run_wino(x, (const char*)wpack + (2 * oh) * qb, osc4[2 * oh], nullptr, nullptr, yh, nullptr, batch, h, w,
                     in_op, FVC_ACT_NONE, cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream, nullptr,
                     0.f, 0, 2 * kC, false);
    if (r) return r;
    r = run_wino(x + kC, (const char*)wpack + (2 * oh + 1) * qb, osc4[2 * oh + 1], bias + kC * oh, yh, yh, nullptr,
                 batch, h, w, in_op, act, cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream, nullptr,
                 0.f, 0, 2 * kC, true);
    if (r) return r;
  }
  return 0;
}

// y = conv(in_op(X)) with X = skip + up2(low) (bilinear, align_corners=True; Warp_net's
// c3_u = c1 + up(c3) and c4_u = c0 + up(c4), endecoder.py:288-293) formed in the kernel's staging
// and written to xsum (bit-identical to fvc_upsample2x_add_nhwc's output) for the consumer's residual
int fvc_conv2d_nhwc_wino_up(const float* skip, const float* low, float* xsum, const void* wpack, float osc,
                            const float* bias, float* y, int batch, int h, int w, int in_op, int act, int cu_reserve,
                            int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream) {
  if (!skip || !low || !xsum) return FVC_EINVAL;
  return run_wino(skip, wpack, osc, bias, nullptr, y, nullptr, batch, h, w, in_op, act, cu_reserve, overflow_flag,
                  sched, sched_len, (hipStream_t)stream, nullptr, 0.f, 0, kC, false, low, xsum);
}

int fvc_conv2d_nhwc_wino(const float* x, const void* wpack, float osc, const float* bias, const float* res,
                         float* y, float* pool, int batch, int h, int w, int in_op, int act, int cu_reserve,
                         int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream) {
  return run_wino(x, wpack, osc, bias, res, y, pool, batch, h, w, in_op, act, cu_reserve, overflow_flag, sched,
                  sched_len, (hipStream_t)stream);
}

}  // extern "C"
