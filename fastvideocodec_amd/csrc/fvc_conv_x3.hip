// Split-precision implicit-GEMM convolution / transposed convolution on the fp16 matrix cores
// (v_mfma_f32_32x32x16_f16), at fp32-level accuracy.
//
// Replaces the same ATen conv2d / conv_transpose2d calls as fvc_conv.hip (DVC/subnet/
// endecoder.py:142-169 MEBasic 7x7, :228-296 Warp_net/ResBlock 3x3, analysis_mv.py /
// synthesis_mv.py 3x3, analysis.py / synthesis.py / prior nets 5x5 s2) for every layer whose
// padded input channel count is a multiple of 8.
//
// Numerics ("fp16 x3"): every fp32 operand v is split exactly as v = hi + lo * 2^-11 with
// hi = fp16(v), lo = fp16((v - hi) * 2^11) (the residual scaled back into fp16's normal range,
// so the split keeps ~22 significant bits for any |v| in [6.1e-5, 65504]). Weights are first
// scaled by a per-layer power of two 2^kw so that max|w| 2^kw lies in [2^13, 2^14). A 32x32 output
// tile keeps two fp32 accumulators:
//     main += hi_x * hi_w                       (one MFMA)
//     corr += hi_x * lo_w + lo_x * hi_w         (two MFMAs)
// and the epilogue forms (main + corr * 2^-11) * 2^-kw + bias. The omitted lo*lo term is
// ~2^-22 relative; fp16 products are exact in the fp32 accumulator, so the result tracks an
// fp32 conv to ~1e-6 relative (tests/test_gpu_kernels.py bounds it like the fp32 kernel).
// Three fp16 MFMAs (3 x 32 cycles per K=16) replace eight fp32 ones (8 x 64 cycles): 5.3x
// less matrix time per MAC. An activation with |v| >= 65000 (or NaN) cannot be represented:
// the staging code ORs 1 into the caller's device flag (overflow_flag argument) instead of
// silently saturating; the host layer checks it and recomputes on the fp32 kernels.
//
// Tiling: GEMM M = output pixels (32-pixel strips), N = output channels (32-channel N-tiles),
// K = taps x input channels walked in k8-blocks = (tap, 8 consecutive channels). One MFMA
// consumes two k8-blocks: lanes 0-31 hold k8-block 2s, lanes 32-63 hold 2s+1, 8 fp16 each.
//  * a block = NW waves stacked vertically, each WM strips x WN N-tiles (2 accumulators per
//    tile); grid = (spatial tiles, N-tile groups, batch x parity classes);
//  * the input halo tile of one channel chunk (CC channels) is staged in LDS as
//    [pixel][hi CC | lo CC] fp16 with the pixel stride padded to 16 x odd bytes, so the
//    ds_read_b128 of 32 strip pixels is conflict-free; stride-2 convs store the tile columns
//    parity-split (even columns, then odd) so their strips also read consecutive pixels;
//  * two LDS buffers: while chunk c is multiplied, every thread stages one item of chunk c+1 per
//    k-step (global load before the MFMAs, split + LDS write after) -> one barrier per chunk;
//  * weights are pre-split at pack time into [class][chunk][k-step][N-tile][hi|lo][lane] 16-B
//    fragments, read from L2 straight into VGPRs (1 KB contiguous per wave instruction),
//    software-pipelined one k-step ahead together with the LDS reads;
//  * transposed convs: stride^2 output-parity classes, each a stride-1 conv with a tap subset;
//  * epilogue: scale + bias, ReLU / LeakyReLU(0.1), residual add, exp; pad channels = 0.
#include "fvc_common.h"
#include "fvc_dx.h"
#include <math.h>
#include <stdlib.h>

namespace {

// cache policy of the activation stores (aux operand of buffer_store; experiment builds only,
// e.g. 2 = non-temporal on gfx950)
#ifndef FVC_STORE_AUX
#define FVC_STORE_AUX 0
#endif

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int kMaxTapsX = 49;

// Accumulation: two weight planes (hi, lo*2^11) and activations split as hi + lo*2^-11; the
// correction products go to a second accumulator scaled by 2^-11 at the end. (Measured and
// rejected, r2: one accumulator with UNSCALED residual halves -- 64 fewer VGPRs, same speed on
// every geometry (scripts/gpu_x3_variants.sh), but an activation residual below 2^-14 is an
// fp16 subnormal and small-activation layers lose accuracy: 4.8e-4 relative at |x| ~ 1e-4.)
constexpr float kLoScale = 2048.f;
// FVC_X3_KO (compile-time, experiment builds only -- wrong results): knock out parts of the k-loop to
// find the binding unit. bit 0: no weight loads (registers), bit 1: no staging of later chunks,
// bit 2: no LDS operand reads (registers), bit 3: no MFMAs, bit 4: weights always from k-step 0
// (L1-resident), bit 5: staging always from tile 0 / chunk 0 (cache-resident).
#ifndef FVC_X3_KO
#define FVC_X3_KO 0
#endif
constexpr int kKO = FVC_X3_KO;  // activation residual scale
// FVC_X3_SCHED (compile-time, experiments): how each half-step's instruction stream is ordered.
// 0: sched_barrier pins [next operands' loads] then [MFMAs]; 1: compiler's own order within a
// half-step; 2: sched_group_barrier interleave, one load between consecutive MFMAs
// (profiles/r2/x3_experiments: 1 and 2 within +-5 % per geometry, 1 -1 % in the pipelined bench)
#ifndef FVC_X3_SCHED
#define FVC_X3_SCHED 0
#endif
constexpr int kSched = FVC_X3_SCHED;
// FVC_X3_ACC1 (compile-time variant): one accumulator. The weight pack carries three planes, hi,
// (w - hi) and hi * 2^-11 (the last two may be fp16 subnormals: their absolute error 2^-25 is
// 2^-39 of the layer's largest weight, which the pack scales into [2^13, 2^14)), so
//     acc += hi_w * hi_x + (w - hi)_w * hi_x + (hi_w 2^-11) * (lo_x 2^11)
// sums the same three products in one fp32 accumulator: half the accumulator registers and one
// FMA per output in the epilogue, for 1.5x the weight operand bytes.
#ifndef FVC_X3_ACC1
#define FVC_X3_ACC1 0
#endif
constexpr int kAcc1 = FVC_X3_ACC1;
constexpr int kNPL = kAcc1 ? 3 : 2;        // weight planes per (k-step, N-tile): hi, lo [, hi 2^-11]
constexpr int kFrag = 64 * kNPL;          // uint4 per (k-step, N-tile)
// internal post-op of the fused tap path (fvc_conv2d_nhwc_x3_tap): not part of the public enum
constexpr int kPostTap = 2;
// internal post-op of fvc_conv2d_nhwc_x3_pool: y and its 2x2 average pool (stride-1 convs, WM = 2)
constexpr int kPostPool = 3;

struct X3Args {
  const float* x;
  const uint4* w;
  const float* bias;
  const float* res;
  float* y;
  int B, H, W, cinp;
  int Ho, Wo, coutp, cout;
  int Hq, Wq;
  int sin, sout, nclass, nchunks, ntp;
  int dymin, dxmin, ir, ic, half;  // half > 0: parity-split tile columns (stride-2 conv)
  int in_op, act, post_op;
  float osc, osc_c;                // 2^-kw, 2^-kw-11
  float inv_ic;                    // 1 / ic
  float act_slope;                 // 0 (ReLU), 0.1 (LeakyReLU), 1 (none)
  int nks[4];                      // k-steps per chunk, per class
  int ntaps[4];
  int oy0[4], ox0[4];
  long long wcls[4];               // uint4 offset of each class in the pack
  int ps;                          // LDS plane stride (halves): 8 x (pixels rounded to 8 mod 16)
  unsigned y_bytes;                // bytes of y (and res): < 4 GB - 4 KB, the buffer range
  unsigned x_bytes;                // bytes of one input image: < 4 GB - 4 KB
  int xcd;                         // XCD-aware mapping of blocks to tile runs (static schedule)
  int* sched;                      // dynamic schedule (may be null: static runs): sched[0] = blocks
                                   // finished, sched[1 + y * B + z] = next work item of group (y, z);
                                   // zero on entry, reset to zero by the last block
  int prio;                        // static priority 1 for the second-dispatched half (waves 4-7)
  int* ovf;                        // caller's overflow flag (device int; may be null)
  int wl_h;                        // WL: halves per LDS weight buffer (the chunk's fragments)
  unsigned res_bytes;              // bytes of res (its own descriptor range)
  // POST == kPostTap: the epilogue applies the next layer's 1x1 tap-partial GEMM to the finished
  // output tile and writes P [B][Ho][Wo][pcp] to y instead of the tile itself
  const uint4* tw;                 // tap weights [k16 block][hi|lo][lane] (fvc_x3_tap_pack_weight)
  float tosc, tosc_c;              // 2^-kt, 2^-kt-11
  int pcp;                         // P channels (partials rounded up to 4, <= 32)
  // POST == kPostPool: the epilogue also writes avg_pool2d(y) (2x2, stride 2) to pool
  float* pool;
  unsigned pool_bytes;
  int toff[4][kMaxTapsX + 1];      // LDS offset (halves) of each tap's window; 0 past ntaps
  // pair-tap form (stride-1 convs with 16 output channels): an N-tile's rows 16-31 hold the same 16
  // channels' weights of the odd tap (ky, kx + 1) of each (ky, even kx) pair, multiplied with the even
  // tap's window: row 16 + c of pixel p is tap (ky, kx + 1)'s product for output pixel p - 1, so the
  // epilogue adds it from lane p + 1 and every strip of 32 pixels finishes 31 output columns
  int pt;
};

typedef float f2v __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

template <int IOP>
__device__ __forceinline__ float in_op_t(float v) {
  if (IOP == FVC_IN_RELU) return fmaxf(v, 0.f);
  if (IOP == FVC_IN_ABS) return fabsf(v);
  if (IOP == FVC_IN_ROUND) return rintf(v);  // torch.round: half-to-even
  return v;
}

// v = hi + lo * 2^-11 for 8 values (packed fp16 conversions); mx tracks max |v| for the
// representability check (|v| < 65000)
__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo, float& mx) {
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const f2v x = {v[i], v[i + 1]};
    const h2v h = __builtin_convertvector(x, h2v);
    const f2v back = __builtin_convertvector(h, f2v);
    const h2v l = __builtin_convertvector((x - back) * kLoScale, h2v);
    hi[i] = h[0];
    hi[i + 1] = h[1];
    lo[i] = l[0];
    lo[i + 1] = l[1];
  }
  mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))),
                       fmaxf(fmaxf(fabsf(v[4]), fabsf(v[5])), fmaxf(fabsf(v[6]), fabsf(v[7])))));
}

// FVC_X3_TRACE (compile-time, diagnostic builds only): per wave, s_memtime sums of the k-loop's
// segments (0 prologue, 1 operand/staging load issue, 2 MFMA blocks, 3 staging split + LDS write,
// 4 chunk end: leftover staging + barrier, 5 epilogue, 6 whole wave) into g_x3_trace. Each stamp
// drains lgkmcnt, so read shares, not lengths.
#ifndef FVC_X3_TRACE
#define FVC_X3_TRACE 0
#endif
constexpr int kTraceVals = 8;
constexpr int kTraceSlots = 1 << 16;
#if FVC_X3_TRACE
__device__ unsigned long long g_x3_trace[kTraceSlots * kTraceVals];
#endif
__device__ __forceinline__ unsigned long long x3_stamp() {
  unsigned long long t = 0;
#if FVC_X3_TRACE
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
  return t;
}

// One 1-KB LDS-DMA piece: lane l's 16 B at g land at LDS byte lds + 16 l. Inline asm (M0 saved
// and restored around it) so the compiler neither sees an LDS write it must drain with vmcnt(0)
// before every later ds_read nor counts it: the kernel orders it itself (vmcnt(0) before the
// barrier that precedes the first read of the buffer it fills).
__device__ __forceinline__ void glds16(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p));
}

// x and y / res are addressed through buffer descriptors with 32-bit offsets (the host keeps
// each image's input and each launch's output under 4 GB): a halo pixel outside the image gets an
// offset past the descriptor's range and loads zeros (the conv's zero padding, no select), and a
// store whose lane is outside the output is dropped by the same range check -- no branches.
constexpr unsigned kOob = 0xFFFFFF00u;
constexpr int kRsrcFlags = 0x00020000;

// Wave grid: the 8 waves form WG groups along N; the 8/WG waves of a group stack vertically,
// each WM strips x WN N-tiles, and group g owns N-tiles nt0 + g*WN .. +WN-1 of the block. With
// WG = 2, WM = 4, WN = 1 a wave re-uses each weight fragment on 4 strips: half the weight bytes
// per MFMA of WG = 1, WM = 2, WN = 2 through the vector-memory return path (TD), which the PMC
// passes show as the kernel's binding unit (scripts/gpu_pmc_x3.sh: TD busy 77 % at 40 % MFMA).
// WL = 1: the block's weight fragments of each chunk are copied once into LDS by LDS-DMA
// (global_load_lds, no VGPRs, issued with the chunk's activation staging one chunk ahead) and the
// waves read them with ds_read_b128 instead of each wave fetching the same 1-KB fragments from L2
// through the vector-memory return path (8 waves x WN x 2 KB per k-step).
template <int CC, int WM, int WN, int WG, int IOP, int POST, int NWV, int WL>
__global__ __launch_bounds__(NWV * 64) void conv_x3_kernel(const X3Args a) {
  constexpr int NW = NWV / WG;       // waves stacked vertically per N-group
  constexpr int C8 = CC / 8;
  constexpr int TH = NW * WM;
  constexpr int TW = 32;
  constexpr int NT = NWV * 64;       // threads staging the first tile
  constexpr int NTS = NWV * 64;      // threads staging later chunks

  extern __shared__ __attribute__((aligned(16))) _Float16 smh[];
  const int tile_h = 2 * C8 * a.ps;  // halves per A buffer: 2*C8 planes (hi octets, lo octets)
  _Float16* const tile0 = smh + 512;  // two buffers at tile0 and tile0 + tile_h (LDS pointers;
                                      // no pointer array, which would degrade them to flat)
  _Float16* const wbase = tile0 + 2 * tile_h;  // WL: two weight buffers of a.wl_h halves
  // LDS header (1 KB): bias of this block's N-tiles [WN * 32] floats at bytes 0..511, the staging
  // sink at 512..543, the work-item queue at 576..591
  float* const sbias = reinterpret_cast<float*>(smh);
  static_assert(WG * WN * 32 * 4 <= 512, "bias area");
  _Float16* const sdump = smh + 256;  // 32 B sink for staging writes of items past the tile
  int* const squeue = reinterpret_cast<int*>(smh) + 144;  // item k of this block at squeue[k & 3]

  unsigned long long tr[kTraceVals] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tr_t0 = x3_stamp();
  const unsigned long long tr_begin = tr_t0;
  auto TR = [&](int i) {  // close the running segment, attributing it to i
    if constexpr (FVC_X3_TRACE != 0) {
      const unsigned long long t1 = x3_stamp();
      tr[i] += t1 - tr_t0;
      tr_t0 = t1;
    }
  };
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar branches)
  const int li = lane & 31;
  const int lh = lane >> 5;
  const int b = blockIdx.z;
  const int TWo = a.pt ? TW - 1 : TW;  // output columns per tile
  const int tiles_x = (a.Wq + TWo - 1) / TWo;
  const int ntiles = tiles_x * ((a.Hq + TH - 1) / TH);
  // persistent over a contiguous run of work items w = tile * nclass + class (row-major tiles:
  // neighbours share halo rows and columns in this CU's L2; all parity classes of a transposed
  // conv's tile run back to back on one CU, so their shared input tile is fetched from HBM once
  // and every block gets the same mix of 4- / 2- / 1-tap classes); the staging pipeline runs on
  // across item boundaries
  const int nitems = ntiles * a.nclass;
  // Work items are taken from the group's counter (a.sched: dynamic schedule; a block that
  // starts late -- its CU held by another stream's kernel -- just takes fewer items), or as a
  // static contiguous run per block. The queue holds items k .. k+2 of this block: item k+2 is
  // taken (one atomic by thread 0) when item k starts and published at the end of its first
  // chunk, so item k+1 is in LDS before its chunk 0 is staged during item k's last chunk.
  // Static runs are XCD-aware: consecutive block ids are dispatched round-robin to the 8 XCDs,
  // so logical run lb = (b % 8)-major gives each XCD's blocks one contiguous band of the image.
  int* const ctr = a.sched ? a.sched + 1 + blockIdx.z * gridDim.y + blockIdx.y : nullptr;
  int lb = blockIdx.x;
  if (a.xcd) {
    const int G = gridDim.x, q8 = G / 8, r8 = G % 8, x8 = lb % 8;
    lb = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + lb / 8;
  }
  const int run_begin = (int)(((long long)nitems * lb) / gridDim.x);
  const int run_end = (int)(((long long)nitems * (lb + 1)) / gridDim.x);
  auto take = [&](int k) -> int {  // thread 0 only
    if (ctr) return atomicAdd(ctr, 1);
    return run_begin + k < run_end ? run_begin + k : nitems;
  };
  auto finish = [&]() {  // every block, once: the last one leaves the schedule zeroed
    if (ctr && tid == 0) {
      __threadfence();
      const int nblk = (int)(gridDim.x * gridDim.y * gridDim.z);
      if (atomicAdd(a.sched, 1) == nblk - 1) {
        for (int g = 0; g < (int)(gridDim.y * gridDim.z); ++g) atomicExch(a.sched + 1 + g, 0);
        atomicExch(a.sched, 0);
      }
    }
  };
  if (tid == 0) {
    squeue[0] = take(0);
    squeue[1] = take(1);
  }
  __syncthreads();
  const int w_first = squeue[0];
  if (w_first >= nitems) {
    finish();
    return;
  }
  const int nt0 = blockIdx.y * (WG * WN);  // first N-tile of the block
  int cls = w_first % a.nclass;
  int nq = a.nks[cls];
  const int hf = a.half;
  const int nch = a.nchunks;
  const int tile_items = a.ir * a.ic * C8;
  const int nstage = (tile_items + NTS - 1) / NTS;
  const int stid = tid;  // staging thread index
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (size_t)b * a.H * a.W * a.cinp), (short)0, (int)a.x_bytes, kRsrcFlags);
  const uint4* wcls = a.w + a.wcls[cls];  // (cls, nq, wcls, tap_tab: updated per work item)
  float mx = 0.f;  // max |staged value| (fp16 representability check)

  // one staging item = 8 channels of one halo pixel: 2 x 16-B buffer loads -> hi/lo h8 in LDS.
  // fetch always issues its two loads (halo pixels outside the image read zeros through the
  // descriptor's range check), so the k-loop has no divergent branches and the compiler can
  // count vmcnt exactly; in_op, the split and the LDS write happen in store, after the MFMAs.
  struct Stage {
    float4 v0, v1;
    int dst;
    bool ok;
  };
  auto fetch = [&](int e, int tile, int ch, Stage& st) {
    if constexpr ((kKO & 2) != 0) return;
    st.ok = e < tile_items;  // past the end: loads of a clamped index, no LDS write
    e = st.ok ? e : tile_items - 1;
    const int o = e & (C8 - 1);
    const int p = e / C8;
    const int r = (int)(((float)p + 0.5f) * a.inv_ic);  // exact: p < 2^14, ic <= 128
    const int c = p - r * a.ic;
    if constexpr ((kKO & 32) != 0) { tile = 0; ch = 0; }
    const int iy = (tile / tiles_x) * TH * a.sin + a.dymin + r;
    const int ix = (tile % tiles_x) * TWo * a.sin + a.dxmin + c;
    const bool inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    const unsigned off = inb ? ((unsigned)(iy * a.W + ix) * (unsigned)a.cinp + (unsigned)(ch * CC + o * 8)) * 4u : kOob;
    st.v0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    // 4-channel inputs (cin 2 / 3): the octet's upper half is zero padding -- the second load goes past
    // the descriptor's range and returns zeros (no branch)
    st.v1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, a.cinp == 4 ? kOob : off + 16u, 0, 0));
    const int cpos = hf ? ((c & 1) * hf + (c >> 1)) : c;
    st.dst = o * a.ps + (r * a.ic + cpos) * 8;  // plane o (hi), pixel-minor
  };
  auto store = [&](_Float16* t, const Stage& st) {
    if constexpr ((kKO & 2) != 0) return;
    float v[8] = {st.v0.x, st.v0.y, st.v0.z, st.v0.w, st.v1.x, st.v1.y, st.v1.z, st.v1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = in_op_t<IOP>(v[i]);  // zero padding stays zero
    h8 hi, lo;
    split8(v, hi, lo, mx);
    // branch-free (keeps the split in the MFMA basic block for interleaving): items past the
    // tile write to a sink
    _Float16* const ph = st.ok ? t + st.dst : sdump;
    _Float16* const pl = st.ok ? t + st.dst + C8 * a.ps : sdump + 8;
    *reinterpret_cast<h8*>(ph) = hi;
    *reinterpret_cast<h8*>(pl) = lo;
  };

  // WL: chunk ch_ of class cls_ -> LDS [k-step][N-tile][hi|lo][lane], one 1-KB piece per
  // wave-instruction (the LDS destination is the wave-uniform base + 16 B x lane)
  // piece p = (k-step q, N-tile n, plane pl) of the chunk whose fragments start at src (+ lane)
  auto w_piece = [&](int p, const uint4* src, _Float16* wdst) {
    if constexpr (WL != 0) {
      const int q = p / (WN * kNPL), r = p - q * (WN * kNPL);
      const int n = r / kNPL, pl = r - n * kNPL;
      const uint4* g = src + ((size_t)q * a.ntp + nt0 + n) * kFrag + pl * 64;
      glds16(g, lds_addr(wdst + p * 512));
    }
  };
  auto w_src = [&](int cls_, int ch_) {
    return a.w + a.wcls[cls_] + (size_t)ch_ * a.nks[cls_] * a.ntp * kFrag + lane;
  };
  auto stage_w = [&](int cls_, int ch_, _Float16* wdst) {
    if constexpr (WL != 0) {
      const int np = a.nks[cls_] * WN * kNPL;
      const uint4* src = w_src(cls_, ch_);
      for (int p = wave; p < np; p += NWV) w_piece(p, src, wdst);
    }
  };

  for (int e = tid; e < tile_items; e += NT) {
    Stage st;
    fetch(e, w_first / a.nclass, 0, st);
    store(tile0, st);
  }
  stage_w(cls, 0, wbase);
  if constexpr (WL != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (tid < WG * WN * 32) {
    const int j = nt0 * 32 + tid;
    sbias[tid] = j < a.cout ? a.bias[j] : 0.f;
  }

  if (a.prio && wave >= NWV / 2) __builtin_amdgcn_s_setprio(1);
  const int wm_ = wave % NW;                // vertical position of this wave in its group
  const int wg_ = wave / NW;                // N-group of this wave
  const int ntw = nt0 + wg_ * WN;           // first N-tile of this wave
  const int pix0 = (((wm_ * WM) * a.sin) * a.ic + li) * 8;  // strip m adds m * pix_m (halves)
  const int pix_m = a.sin * a.ic * 8;
  // tap window offsets live one per lane; v_readlane turns them into wave-uniform scalars
  // without a memory wait inside the k-loop
  int tap_tab = a.toff[cls][lane <= kMaxTapsX ? lane : kMaxTapsX];
  __syncthreads();
  TR(0);

  struct Ops {
    h8 ah[WM], al[WM];
    uint4 bh[WN], bl[WN], bm[kAcc1 ? WN : 1];
  };
  f32x16 acc[WM][WN], cor[kAcc1 ? 1 : WM][kAcc1 ? 1 : WN];
  uint4 ko_w = a.w[lane];
  h8 ko_a = *reinterpret_cast<const h8*>(tile0 + 8 * lane);
  int buf = 0;  // LDS buffer holding the chunk being multiplied
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, (int)a.y_bytes, kRsrcFlags);
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.res, (short)0, (int)a.res_bytes, kRsrcFlags);
  for (int k = 0;; ++k) {
    const int w = squeue[k & 3];
    if (w >= nitems) break;
    int taken = 0;
    if (tid == 0) taken = take(k + 2);
    const int tile = w / a.nclass;
    if (k != 0) {
      cls = w % a.nclass;
      nq = a.nks[cls];
      wcls = a.w + a.wcls[cls];
      tap_tab = a.toff[cls][lane <= kMaxTapsX ? lane : kMaxTapsX];
    }
#pragma unroll
    for (int m = 0; m < WM; ++m)
#pragma unroll
      for (int n = 0; n < WN; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          acc[m][n][r] = 0.f;
          if constexpr (!kAcc1) cor[m][n][r] = 0.f;
        }

    // K loop over channel chunks. Two operand register sets (ping-pong, no copies). Each
    // half-step issues the LDS and global loads of the next k-step (index clamped: the last
    // prefetch is a harmless repeat) and, in the first k-steps of a chunk, one staging load of
    // the next chunk (of this tile, or chunk 0 of the next tile); then its MFMAs; then the staging
    // LDS write. All loads are unconditional and sched_barrier pins the order, so every load has
    // a full k-step of MFMA work to land behind.
    for (int ch = 0; ch < nch; ++ch) {
      const _Float16* cur = tile0 + buf * tile_h;
      _Float16* nxt = tile0 + (buf ^ 1) * tile_h;
      const uint4* wcur = reinterpret_cast<const uint4*>(wbase + buf * a.wl_h);
      const bool last = ch + 1 == nch;
      const int s_item = last ? squeue[(k + 1) & 3] : w;
      const int s_tile = s_item / a.nclass;
      const int s_ch = last ? 0 : ch + 1;
      const bool stage_next = s_item < nitems;
      const uint4* wch = wcls + (size_t)ch * nq * a.ntp * kFrag;
      // WL: this wave's pieces of the next chunk's weights (issued after the chunk's first operand
      // reads, landed by the vmcnt(0) before the chunk's closing barrier)
      const int s_cls = s_item % a.nclass;
      const uint4* wsrc = WL ? w_src(stage_next ? s_cls : 0, s_ch) : nullptr;
      _Float16* const wdst = wbase + (buf ^ 1) * a.wl_h;
      const int wnp = (WL && stage_next) ? a.nks[s_cls] * WN * kNPL : 0;
      int wp = wave;
      auto w_issue = [&]() {
        if constexpr (WL != 0) {
          if (wp < wnp) {
            w_piece(wp, wsrc, wdst);
            wp += NWV;
          }
        }
      };
      // k-step q: lane half lh takes k8-block kb = 2q + lh = (tap kb / C8, octet kb % C8)
      auto load = [&](int q, Ops& op) {
        int toff;
        if (C8 == 1) {
          const int t0 = __builtin_amdgcn_readlane(tap_tab, 2 * q);
          const int t1 = __builtin_amdgcn_readlane(tap_tab, 2 * q + 1);
          toff = lh ? t1 : t0;
        } else {
          toff = __builtin_amdgcn_readlane(tap_tab, (2 * q) / C8) + (((2 * q) & (C8 - 1)) + lh) * a.ps;
        }
#pragma unroll
        for (int m = 0; m < WM; ++m) {
          if constexpr ((kKO & 4) != 0) {
            op.ah[m] = ko_a + (_Float16)(q + m);
            op.al[m] = ko_a;
            continue;
          }
          op.ah[m] = *reinterpret_cast<const h8*>(cur + pix0 + m * pix_m + toff);
          op.al[m] = *reinterpret_cast<const h8*>(cur + pix0 + m * pix_m + toff + C8 * a.ps);
        }
        const uint4* wk = WL ? wcur + (size_t)q * WN * kFrag + lane
                             : ((kKO & 16) ? wcls : wch) + ((size_t)((kKO & 16) ? 0 : q) * a.ntp + ntw) * kFrag + lane;
#pragma unroll
        for (int n = 0; n < WN; ++n) {
          if constexpr ((kKO & 1) != 0) {
            op.bh[n] = ko_w + (unsigned)(q + n);
            op.bl[n] = ko_w;
            continue;
          }
          op.bh[n] = wk[n * kFrag];
          op.bl[n] = wk[n * kFrag + 64];
          if constexpr (kAcc1) op.bm[n] = wk[n * kFrag + 128];
        }
      };
      // weights as the A (row) operand, pixels as B: the 32x32 result is channel x pixel, so
      // each lane ends up with 4 consecutive channels of one pixel per register group (16-B
      // epilogue stores)
      auto mfmas = [&](const Ops& op) {
        if constexpr ((kKO & 8) != 0) {
#pragma unroll
          for (int m = 0; m < WM; ++m)
#pragma unroll
            for (int n = 0; n < WN; ++n) acc[m][n][0] += (float)op.ah[m][0] + (float)__builtin_bit_cast(h8, op.bh[n])[0];
          return;
        }
#pragma unroll
        for (int m = 0; m < WM; ++m)
#pragma unroll
          for (int n = 0; n < WN; ++n) {
            const h8 wh = __builtin_bit_cast(h8, op.bh[n]);
            const h8 wl = __builtin_bit_cast(h8, op.bl[n]);
            if constexpr (kAcc1) {
              const h8 wm = __builtin_bit_cast(h8, op.bm[n]);
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, op.ah[m], acc[m][n], 0, 0, 0);
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, op.ah[m], acc[m][n], 0, 0, 0);
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wm, op.al[m], acc[m][n], 0, 0, 0);
            } else {
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, op.ah[m], acc[m][n], 0, 0, 0);
              cor[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, op.ah[m], cor[m][n], 0, 0, 0);
              cor[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, op.al[m], cor[m][n], 0, 0, 0);
            }
          }
      };
      // order pins inside a half-step (kSched 0) and the interleave pattern closing it (kSched 2)
      auto pin = [&]() {
        if constexpr (kSched == 0) __builtin_amdgcn_sched_barrier(0);
      };
      auto close = [&]() {
        if constexpr (kSched == 2) {
#pragma unroll
          for (int i = 0; i < 3 * WM * WN; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x120, 1, 0);  // then one DS or VMEM read
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      auto half_plain = [&](int q, const Ops& use, Ops& nxt_ops) {
        load(q + 1 < nq ? q + 1 : nq - 1, nxt_ops);
        pin();
        TR(1);
        mfmas(use);
        close();
        TR(2);
      };
      int staged = 0;
      Ops S0, S1;
      load(0, S0);
      while (wp < wnp) w_issue();  // WL: the next chunk's weights, a whole chunk ahead
      // staging items of the next chunk are spread evenly over the k-step pairs (one per staged
      // pair) so their VALU work interleaves with MFMA-only steps instead of bunching up at the
      // chunk start, where every wave would be VALU-bound at once
      const int npair = nq >> 1;
      const int nst = stage_next ? min(nstage, npair) : 0;
      const int spread = nst ? max(1, npair / nst) : 1;
      int q = 0;
      for (; staged < nst; ++staged) {
        // the staged item's split + LDS write come after the pair's second half-step, so its
        // loads have two half-steps of MFMAs (both waves of the SIMD) to land behind
        load(q + 1 < nq ? q + 1 : nq - 1, S1);
        Stage st;
        fetch(stid + staged * NTS, s_tile, s_ch, st);
        pin();
        TR(1);
        mfmas(S0);
        close();
        TR(2);
        load(q + 2 < nq ? q + 2 : nq - 1, S0);
        pin();
        TR(1);
        mfmas(S1);
        close();
        TR(2);
        store(nxt, st);
        TR(3);
        q += 2;
        for (int r = 1; r < spread; ++r, q += 2) {
          half_plain(q, S0, S1);
          half_plain(q + 1, S1, S0);
        }
      }
      for (; q + 1 < nq; q += 2) {
        half_plain(q, S0, S1);
        half_plain(q + 1, S1, S0);
      }
      if (nq & 1) mfmas(S0);
      TR(2);
      if (stage_next) {
        for (int qs = staged; qs < nstage; ++qs) {
          Stage st;
          fetch(stid + qs * NTS, s_tile, s_ch, st);
          store(nxt, st);
        }
      }
      if (ch == 0 && tid == 0) squeue[(k + 2) & 3] = taken;
      if constexpr (WL != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight DMA
      __syncthreads();
      buf ^= 1;
      TR(4);
    }

    // epilogue of this tile (its global stores drain while the next tile's k-loop runs).
    // Lane (li, lh) holds pixel qx0 + li of strip m; register group g (r = 4g..4g+3) holds output
    // channels N-tile*32 + 8g + 4lh + {0..3} -> one 16-B store (and residual load) per group.
    // Activation as one max: relu = max(v, 0*v), lrelu = max(v, 0.1*v), none = max(v, 1*v).
    // Pad channels need no select: their weights and bias are 0 and every residual tensor's pad
    // channels are 0, so they come out 0 -- except after exp (POST), which selects them to 0.
    const int qy0 = (tile / tiles_x) * TH, qx0 = (tile % tiles_x) * TWo;
    const bool px_ok = qx0 + li < a.Wq && li < TWo;
    auto pix_of = [&](int m) {  // output pixel index of this lane in strip m
      const unsigned qy = qy0 + wm_ * WM + m;
      return ((unsigned)b * a.Ho + qy * a.sout + a.oy0[cls]) * a.Wo + a.ox0[cls] + (unsigned)(qx0 + li) * a.sout;
    };
    auto voff_of = [&](int m, int n) {
      return pix_of(m) * (unsigned)a.coutp * 4u + (unsigned)((ntw + n) * 32 + 4 * lh) * 4u;
    };
    if constexpr (POST == kPostTap) {
      // Fused tap-partial epilogue (the next layer is a cout <= 4 conv computed as a 1x1 GEMM to
      // P = k*k*cout tap partials per pixel + fvc_tap_gather_nhwc). This wave holds every output
      // channel of its strips (WG = 1, WN = all N-tiles): lane (li, lh) has channel
      // 32n + 8g + 4lh + i of pixel li in register 4g + i of tile (m, n), so registers 8gp..8gp+7
      // of tile n are exactly the B operand of the k16 block kb = 2n + gp (channels
      // 32n + 16gp + {0-3, 8-11 | 4-7, 12-15} for lane half 0 | 1; the tap pack uses the same order).
      // The finished values y are split hi/lo like staged activations and multiplied with the
      // same three MFMAs per block; P = main * 2^-kt + corr * 2^-kt-11.
#pragma unroll
      for (int m = 0; m < WM; ++m) {
        const unsigned pix = pix_of(m);
        const bool row_ok = qy0 + wm_ * WM + m < a.Hq && px_ok;
        f32x16 pa, pc;
#pragma unroll
        for (int r = 0; r < 16; ++r) pa[r] = pc[r] = 0.f;
        // tile by tile: finish y of N-tile n (bias, act, residual), then its two k16 blocks, so
        // only one tile's y is live next to the partial accumulators
#pragma unroll
        for (int n = 0; n < WN; ++n) {
          float yv[16];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float4 rq = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.res) rq = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rr, voff_of(m, n) + 32u * g, 0, 0));
            const float4 bj = *reinterpret_cast<const float4*>(sbias + n * 32 + 8 * g + 4 * lh);
            const float bb[4] = {bj.x, bj.y, bj.z, bj.w};
            const float rr4[4] = {rq.x, rq.y, rq.z, rq.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 4 * g + i;
              const float tv = fmaf(cor[kAcc1 ? 0 : m][kAcc1 ? 0 : n][r], kAcc1 ? 0.f : a.osc_c, fmaf(acc[m][n][r], a.osc, bb[i]));
              yv[r] = fmaxf(tv, tv * a.act_slope) + rr4[i];
            }
          }
#pragma unroll
          for (int gp = 0; gp < 2; ++gp) {
            float v8[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) v8[t] = yv[8 * gp + t];
            h8 yh, yl;
            split8(v8, yh, yl, mx);
            const uint4* tw = a.tw + (size_t)((n * 2 + gp) * 2) * 64 + lane;
            const h8 wh = __builtin_bit_cast(h8, tw[0]);
            const h8 wl = __builtin_bit_cast(h8, tw[64]);
            pa = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yh, pa, 0, 0, 0);
            pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, yh, pc, 0, 0, 0);
            pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yl, pc, 0, 0, 0);
          }
        }
        const unsigned po = pix * (unsigned)a.pcp * 4u + (unsigned)(4 * lh) * 4u;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int p0 = 8 * g + 4 * lh;
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = fmaf(pc[4 * g + i], a.tosc_c, pa[4 * g + i] * a.tosc);
          const unsigned so = (row_ok && p0 < a.pcp) ? po + 32u * g : kOob;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_float4(o[0], o[1], o[2], o[3])), ry, so, 0, 0);
        }
      }
      TR(5);
      continue;
    }
    // residual: the 4 groups of output tile t+1 are loaded before tile t is finished and stored,
    // so each wait covers loads issued one tile earlier (vmcnt is in order and counts the stores);
    // WM = WN = 2 has no registers for the second set: its 4 loads are waited for together
    constexpr int NTL = WM * WN;
    constexpr bool kResPipe = NTL < 4;
    float4 rv[2][4];
    auto load_res = [&](int t, float4 (&r)[4]) {
      const unsigned vo = voff_of(t / WN, t % WN);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        r[g] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rr, vo + 32u * g, 0, 0));
    };
    if (a.res && kResPipe) load_res(0, rv[0]);
    // kPostPool: strips 0 and 1 of a wave are output rows 2r and 2r+1 and lanes li, li^1 are
    // columns 2c, 2c+1, so each 2x2 window is in one wave: strip 0's values are kept, strip 1
    // adds them with a DPP quad swap, and the even lanes store the pooled pixel (ATen order
    // ((x00 + x01) + x10) + x11, / 4: the same bits as k_avgpool2)
    float keep[POST == kPostPool ? WN : 1][4][4];
    const __amdgpu_buffer_rsrc_t rpool =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.pool, (short)0, (int)a.pool_bytes, kRsrcFlags);
    auto swap1 = [](float x) {  // value of lane li ^ 1 (quad_perm [1, 0, 3, 2])
      return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
    };
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      const int m = t / WN, n = t % WN;
      if (a.res) {
        if (!kResPipe) load_res(t, rv[t & 1]);
        else if (t + 1 < NTL) load_res(t + 1, rv[(t + 1) & 1]);
      }
      // pair-tap form: the odd taps' products of this lane's output pixel sit in rows 16-31
      // (register groups 2, 3) of the next lane
      float sh[8];
      if (a.pt) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float bv = kAcc1 ? acc[m][n][8 + r] * a.osc
                                 : fmaf(cor[kAcc1 ? 0 : m][kAcc1 ? 0 : n][8 + r], a.osc_c, acc[m][n][8 + r] * a.osc);
          sh[r] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(((lane + 1) & 63) * 4, __builtin_bit_cast(int, bv)));
        }
      }
      const unsigned vo = voff_of(m, n);
      const bool row_ok = qy0 + wm_ * WM + m < a.Hq && px_ok;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int jl = 8 * g + 4 * lh;       // channel within the N-tile
        const int j0 = (ntw + n) * 32 + jl;  // first of this lane's 4 channels
        const float4 bj = *reinterpret_cast<const float4*>(sbias + (wg_ * WN + n) * 32 + jl);
        const float bb[4] = {bj.x, bj.y, bj.z, bj.w};
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          float tv = kAcc1 ? fmaf(acc[m][n][r], a.osc, bb[i])
                           : fmaf(cor[kAcc1 ? 0 : m][kAcc1 ? 0 : n][r], a.osc_c, fmaf(acc[m][n][r], a.osc, bb[i]));
          if (a.pt && g < 2) tv += sh[r];
          v[i] = fmaxf(tv, tv * a.act_slope);
        }
        if (a.res) {
          const float4 q4 = rv[t & 1][g];
          v[0] += q4.x; v[1] += q4.y; v[2] += q4.z; v[3] += q4.w;
        }
        if constexpr (POST == FVC_POST_EXP) {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = j0 + i < a.cout ? expf(v[i]) : 0.f;
        }
        const unsigned so = (row_ok && j0 < a.coutp) ? vo + 32u * g : kOob;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_float4(v[0], v[1], v[2], v[3])),
                                               ry, so, 0, FVC_STORE_AUX);
        if constexpr (POST == kPostPool) {
          if (m == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) keep[n][g][i] = v[i];
          } else {
            // pooled values on the even lanes; groups g (even) and g + 1 go out in one store: the
            // odd lane li + 1 takes group g + 1 of its even neighbour (channels 8 further)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float x00 = keep[n][g][i], x10 = v[i];
              keep[n][g][i] = (((x00 + swap1(x00)) + x10) + swap1(x10)) / 4.f;
            }
            if (g & 1) {
              // the swap runs on every lane (a DPP read from a lane switched off by a branch
              // would return 0), then a bitwise select keeps the branch out
              float pv[4];
              const int odd = -(li & 1);
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int sw = __builtin_bit_cast(int, swap1(keep[n][g][i]));
                const int ev = __builtin_bit_cast(int, keep[n][g - 1][i]);
                pv[i] = __builtin_bit_cast(float, (sw & odd) | (ev & ~odd));
              }
              const int Hp = a.Hq >> 1, Wp = a.Wq >> 1;
              const int prow = (qy0 + wm_ * WM) >> 1, pcol = (qx0 + li) >> 1;
              const int jp = (ntw + n) * 32 + 8 * (g - 1 + (li & 1)) + 4 * lh;  // this lane's channels
              const bool pok = prow < Hp && pcol < Wp && jp < a.coutp;
              const unsigned po = (((unsigned)b * Hp + prow) * Wp + pcol) * (unsigned)a.coutp * 4u + (unsigned)jp * 4u;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_float4(pv[0], pv[1], pv[2], pv[3])),
                                                     rpool, pok ? po : kOob, 0, 0);
            }
          }
        }
      }
    }
    TR(5);
  }
  if (!(mx < 65000.f) && a.ovf) atomicOr(a.ovf, 1);
#if FVC_X3_TRACE
  {
    const unsigned long long tr_end = x3_stamp();
    tr[6] = tr_end - tr_begin;
    tr[7] = 1;
    const unsigned slot = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * NWV + wave;
    if (lane < kTraceVals && slot < (unsigned)kTraceSlots) {
      unsigned long long v = tr[0];
#pragma unroll
      for (int i = 1; i < kTraceVals; ++i) v = lane == i ? tr[i] : v;
      atomicAdd(&g_x3_trace[(size_t)slot * kTraceVals + lane], v);
    }
  }
#endif
  finish();
}

// ------------------------------------------------------------------ host-side geometry
struct X3Cfg {
  int cinp, coutp, ntp, cc, wm, wn, nw, nclass, nchunks, th, sin, sout;
  int pt;     // pair-tap form (16 output channels, stride 1): (ky, even kx) pairs, see X3Args::pt
  int dx;     // stride-2 transposed conv on fvc_deconv_x3.hip (all classes per staged tile, one chunk)
  int wl;     // weights staged in LDS by LDS-DMA (FVC_X3_WL; chosen at pack time: it can shrink cc)
  int wnmax;  // N-tiles per block the LDS weight buffers are sized for
  int ntaps[4], nks[4], oy0[4], ox0[4];
  int tky[4][kMaxTapsX], tkx[4][kMaxTapsX];
  int tdy[4][kMaxTapsX], tdx[4][kMaxTapsX];
  int dymin, dymax, dxmin, dxmax;
  long long wcls[4];
  long long wtotal;  // uint4 (16-B) units
};

static int x3_floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// LDS A tile: 2*CC/8 planes (hi octets, then lo octets) of ir*ic 16-B pixel entries. The plane
// stride is the pixel count rounded up to 4 mod 16 entries (64 B mod 256 B), so the staging
// writes of consecutive items (octets of one pixel go to different planes) do not collide, while
// a strip read (32 consecutive pixels of one plane, 16 B each) is conflict-free by construction.
static int x3_plane_pix(int ir, int ic) { return ((ir * ic + 15) & ~15) + 4; }
static size_t x3_tile_bytes(int ir, int ic, int cc) { return (size_t)4 * cc * x3_plane_pix(ir, ic); }

static int env_int(const char* n, int dflt) {
  const char* v = getenv(n);
  return (v && v[0]) ? atoi(v) : dflt;
}

// Geometry and tile choice. Returns false for layers the x3 path does not take (cinp % 8 != 0,
// cout <= 4 -> the VALU small-N kernel, > 128 output channels).
static bool x3_cfg(int cin, int cout, int ks, int stride, int transposed, X3Cfg& c) {
  if (cin <= 0 || cout <= 0 || (ks != 1 && ks != 3 && ks != 5 && ks != 7) || (stride != 1 && stride != 2))
    return false;
  c.cinp = fvc_rup(cin, 4);
  c.coutp = fvc_rup(cout, 4);
  // cin padded to 4 (cin 2 / 3: mvEncoder conv1, resEncoder conv1) runs as one zero-extended octet:
  // the staging loads 4 channels per pixel and pads the other 4 with zeros, so no widened copy of
  // the input is needed (FVC_X3_CIN4=0 keeps these layers on the fp32 kernels)
  if (c.cinp % 8 && !(c.cinp == 4 && env_int("FVC_X3_CIN4", 1))) return false;
  // cout <= 4 (N padded to one 32-wide tile): measured faster than the VALU small-N kernel for the
  // 3x3 / 5x5 layers (Warp_net conv6, mvDecoder conv8, resDecoder deconv4), slower for SpyNet's
  // 7x7 16->2 (scripts/conv_micro.py); FVC_X3_SMALLN=0/1 forces either way
  if (c.coutp <= 4) {
    const int sn = env_int("FVC_X3_SMALLN", -1);
    if (sn == 0 || (sn < 0 && ks > 5)) return false;
  }
  c.ntp = fvc_cdiv(c.coutp, 32);
  if (c.ntp > 4) return false;
  const int pad = ks / 2;
  c.pt = (!transposed && stride == 1 && c.coutp == 16 && ks >= 3 && env_int("FVC_X3_PT", 1)) ? 1 : 0;
  if (!transposed) {
    c.nclass = 1;
    c.sin = stride;
    c.sout = 1;
    c.ntaps[0] = 0;
    for (int ky = 0; ky < ks; ++ky)
      for (int kx = 0; kx < ks; kx += c.pt ? 2 : 1) {
        const int t = c.ntaps[0]++;
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
            const int t = c.ntaps[cl]++;
            c.tky[cl][t] = ky; c.tkx[cl][t] = kx;
            c.tdy[cl][t] = x3_floordiv(py + pad - ky, stride);
            c.tdx[cl][t] = x3_floordiv(px + pad - kx, stride);
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
  // stride-2 transposed convs with 64 / 96 / 128 input and 64 / 128 output channels: the
  // all-classes kernel (fvc_deconv_x3.hip) when two full-channel tile buffers fit in LDS; its pack
  // is this pack with one channel chunk. FVC_DX=0 keeps them on this kernel (at pack AND launch).
  c.dx = 0;
  c.wl = 0;
  if (transposed && stride == 2 && c.nclass == 4 && env_int("FVC_DX", 1) &&
      (c.cinp == 64 || c.cinp == 96 || c.cinp == 128) && (c.ntp == 2 || c.ntp == 4)) {
    int maxt = 0;
    for (int cl = 0; cl < 4; ++cl) maxt = c.ntaps[cl] > maxt ? c.ntaps[cl] : maxt;
    // items of R input rows x sw columns: 128 channels 8 x 16 (four 2 x 16-pixel strips), fewer
    // channels 2 x 32 (4 N-tiles) or 4 x 32 (2 N-tiles): 8 wave-tiles of 2 strips x 2 N-tiles or more
    const int sw = fvc_dx::strip_width(c.cinp);
    const int R = sw == 16 ? 8 : (c.ntp == 4 ? 2 : 4);
    const int ir = R + (c.dymax - c.dymin), ic = sw + (c.dxmax - c.dxmin);
    if (maxt <= fvc_dx::kMaxTaps && fvc_dx::lds_bytes(c.cinp, fvc_dx::plane_pix(ir, ic)) <= 160 * 1024) {
      c.dx = 1;
      c.cc = c.cinp;
      c.nchunks = 1;
      c.nw = 8;
      c.wm = 2;
      c.wn = 2;
      c.wnmax = 2;
      c.th = R;
      long long off = 0;
      for (int cl = 0; cl < 4; ++cl) {
        c.nks[cl] = fvc_cdiv(c.ntaps[cl] * (c.cc / 8), 2);
        c.wcls[cl] = off;
        off += (long long)c.nks[cl] * c.ntp * kFrag;
      }
      c.wtotal = off;
      return true;
    }
  }
  // channel chunk: the largest of 32 / 16 / 8 dividing cinp (shrunk below if the two LDS tile
  // buffers do not fit); FVC_X3_CC overrides for experiments
  c.cc = (c.cinp % 32 == 0) ? 32 : ((c.cinp % 16 == 0) ? 16 : 8);
  const int want_cc = env_int("FVC_X3_CC", 0);
  if ((want_cc == 8 || want_cc == 16 || want_cc == 32) && c.cinp % want_cc == 0) c.cc = want_cc;
  // block shape: 8 waves x 2 strips (16 output rows x 32 columns), 2 waves per SIMD;
  // FVC_X3_NW / FVC_X3_WM override for experiments (WM=4 only with 4 waves)
  c.nw = 8;
  // stride-2 convs: one strip per wave (measured 0.22 vs 0.35 ms on the 544x960 128-channel layer:
  // two strips double the halo rows each staged chunk carries)
  c.wm = env_int("FVC_X3_WM", (!transposed && stride == 2) ? 1 : 2) == 1 ? 1 : 2;
  // weight buffers in LDS (WL): two chunks of the block's fragments, sized for its widest N
  c.wl = env_int("FVC_X3_WL", 0) ? 1 : 0;
  c.wnmax = (c.wm == 1 && !transposed && stride == 2 && c.ntp % 4 == 0) ? 4 : (c.ntp >= 2 ? 2 : 1);
  // shrink the channel chunk, then the strips per wave, until two tile buffers fit in LDS
  for (;;) {
    c.th = c.nw * c.wm;
    const int ir = (c.th - 1) * c.sin + 1 + (c.dymax - c.dymin);
    const int ic = 31 * c.sin + 1 + (c.dxmax - c.dxmin);
    size_t lds = 1024 + 2 * x3_tile_bytes(ir, ic, c.cc);
    if (c.wl) {
      int nkmax = 0;
      for (int cl = 0; cl < c.nclass; ++cl) {
        const int nk = fvc_cdiv(c.ntaps[cl] * (c.cc / 8), 2);
        nkmax = nk > nkmax ? nk : nkmax;
      }
      lds += 2 * (size_t)nkmax * c.wnmax * kFrag * 16;
    }
    if (lds <= 160 * 1024) break;
    if (c.cc > 8 && c.cinp % (c.cc / 2) == 0) c.cc /= 2;
    else if (c.wm > 1) c.wm /= 2;
    else return false;
  }
  c.nchunks = c.cinp == 4 ? 1 : c.cinp / c.cc;
  c.wn = 1;
  long long off = 0;
  for (int cl = 0; cl < c.nclass; ++cl) {
    c.nks[cl] = fvc_cdiv(c.ntaps[cl] * (c.cc / 8), 2);
    c.wcls[cl] = off;
    off += (long long)c.nchunks * c.nks[cl] * c.ntp * kFrag;  // kFrag uint4 per (k-step, N-tile)
  }
  c.wtotal = off;
  return true;
}

static int x3_num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

static int x3_kw(const float* w, size_t n) {
  float mx = 0.f;
  for (size_t i = 0; i < n; ++i) mx = fabsf(w[i]) > mx ? fabsf(w[i]) : mx;
  if (!(mx > 0.f) || !isfinite(mx)) return 0;
  int e;
  frexpf(mx, &e);  // mx = m * 2^e, m in [0.5, 1)
  int kw = 14 - e;  // mx * 2^kw in [2^13, 2^14)
  return kw < -100 ? -100 : (kw > 100 ? 100 : kw);
}

template <int CC, int WM, int WN, int WG, int IOP, int POST, int NWV, int WL>
static int x3_launch(const X3Args& a, dim3 grid, size_t lds, hipStream_t s) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)conv_x3_kernel<CC, WM, WN, WG, IOP, POST, NWV, WL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((conv_x3_kernel<CC, WM, WN, WG, IOP, POST, NWV, WL>), grid, dim3(NWV * 64), lds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

// exp after the epilogue is only ever taken with an untransformed input (Synthesis_prior_net
// deconv3, synthesis_prior.py:25,57): instantiated for IN_NONE only
template <int CC, int WM, int WN, int WG, int WL, int NWV = 8>
static int x3_launch_iop(int iop, int post, const X3Args& a, dim3 grid, size_t lds, hipStream_t s) {
  if (post == kPostPool) {  // fused 2x2 pool epilogue: strip pairs per wave (run_x3)
    if constexpr (WG == 1 && WL == 0 && WM == 2 && WN <= 2)
      return iop == FVC_IN_NONE ? x3_launch<CC, WM, WN, WG, FVC_IN_NONE, kPostPool, NWV, WL>(a, grid, lds, s) : FVC_EINVAL;
    return FVC_EINVAL;
  }
  if (post == kPostTap) {  // fused tap epilogue: every output channel in one wave (run_x3)
    if constexpr (WG == 1 && WL == 0 && ((WM == 2 && WN <= 2) || (WM == 1 && WN == 4)))
      return iop == FVC_IN_NONE ? x3_launch<CC, WM, WN, WG, FVC_IN_NONE, kPostTap, NWV, WL>(a, grid, lds, s) : FVC_EINVAL;
    return FVC_EINVAL;
  }
  if (post == FVC_POST_EXP)
    return iop == FVC_IN_NONE ? x3_launch<CC, WM, WN, WG, FVC_IN_NONE, FVC_POST_EXP, NWV, WL>(a, grid, lds, s) : FVC_EINVAL;
  switch (iop) {
    case FVC_IN_NONE: return x3_launch<CC, WM, WN, WG, FVC_IN_NONE, FVC_POST_NONE, NWV, WL>(a, grid, lds, s);
    case FVC_IN_RELU: return x3_launch<CC, WM, WN, WG, FVC_IN_RELU, FVC_POST_NONE, NWV, WL>(a, grid, lds, s);
    case FVC_IN_ABS: return x3_launch<CC, WM, WN, WG, FVC_IN_ABS, FVC_POST_NONE, NWV, WL>(a, grid, lds, s);
    case FVC_IN_ROUND: return x3_launch<CC, WM, WN, WG, FVC_IN_ROUND, FVC_POST_NONE, NWV, WL>(a, grid, lds, s);
  }
  return FVC_EINVAL;
}

// instantiated wave grids (8 waves, 2 per SIMD, <= 256 registers: scripts/kres.sh):
// WG = 1 with WM, WN in {1, 2} or WM = 1, WN = 4; WG = 2 with WM = 4, WN = 1
template <int CC, int WL>
static int x3_launch_cc(int nwv, int wm, int wn, int wg, int iop, int post, const X3Args& a, dim3 grid,
                        size_t lds, hipStream_t s) {
  if (nwv != 8) return FVC_EINVAL;
  if (wg == 2) return (wm == 4 && wn == 1 && !WL) ? x3_launch_iop<CC, 4, 1, 2, 0>(iop, post, a, grid, lds, s) : FVC_EINVAL;
  if (wm == 2 && wn == 2) return x3_launch_iop<CC, 2, 2, 1, WL>(iop, post, a, grid, lds, s);
  if (wm == 2 && wn == 1) return x3_launch_iop<CC, 2, 1, 1, WL>(iop, post, a, grid, lds, s);
  if (wm == 1 && wn == 2) return x3_launch_iop<CC, 1, 2, 1, WL>(iop, post, a, grid, lds, s);
  if (wm == 1 && wn == 1) return x3_launch_iop<CC, 1, 1, 1, WL>(iop, post, a, grid, lds, s);
  if (wm == 1 && wn == 4) return x3_launch_iop<CC, 1, 4, 1, WL>(iop, post, a, grid, lds, s);
  return FVC_EINVAL;
}

// A stride-2 transposed conv on the all-classes kernel (fvc_deconv_x3.hip): R input rows x 32
// columns per work item, the item's (class, strip pair, N-tile pair) wave-tiles dealt to the 8 waves
// so that SIMD partners w and w + 4 together carry an equal share of taps (largest first, to the
// least-loaded SIMD, then to its less-loaded wave). Tap form: one strip x all 4 N-tiles per wave-tile.
static int run_dx(const X3Cfg& c, const float* x, const void* wpack, float osc, const float* bias, const float* res,
                  float* y, int batch, int h, int w, int cout, int in_op, int act, int post_op, int cu_reserve,
                  int* ovf, int* sched, int sched_len, hipStream_t s, const void* tw, float tosc, int pcp,
                  unsigned y_bytes, unsigned x_bytes) {
  const bool tap = tw != nullptr;
  if (tap && res) return FVC_EINVAL;
  const int R = c.th;
  const int sw = fvc_dx::strip_width(c.cinp);
  const int S = R / (32 / sw);  // strips per item
  const int wm = tap ? 1 : 2, wn = tap ? c.ntp : 2;
  fvc_dx::DxArgs d;
  d.x = x;
  d.w = (const uint4*)wpack;
  d.bias = bias;
  d.res = res;
  d.y = y;
  d.post_exp = post_op == FVC_POST_EXP ? 1 : 0;
  d.B = batch;
  d.H = h;
  d.W = w;
  d.cout = cout;
  d.coutp = c.coutp;
  d.ntp = c.ntp;
  d.R = R;
  d.sw = sw;
  d.ir = R + (c.dymax - c.dymin);
  d.ic = sw + (c.dxmax - c.dxmin);
  d.ps = fvc_dx::plane_pix(d.ir, d.ic);
  d.dymin = c.dymin;
  d.dxmin = c.dxmin;
  d.inv_ic = 1.0f / (float)d.ic;
  d.tiles_x = fvc_cdiv(w, sw);
  d.tiles_y = fvc_cdiv(h, R);
  const long long nitems = (long long)batch * d.tiles_x * d.tiles_y;
  if (nitems >= (1LL << 30)) return FVC_EINVAL;
  d.nitems = (int)nitems;
  d.osc = osc;
  d.osc_c = osc * (1.0f / 2048.f);
  d.act_slope = act == FVC_ACT_RELU ? 0.f : (act == FVC_ACT_LRELU ? 0.1f : 1.f);
  for (int cl = 0; cl < 4; ++cl) {
    d.nks[cl] = c.nks[cl];
    d.oy0[cl] = c.oy0[cl];
    d.ox0[cl] = c.ox0[cl];
    d.wcls[cl] = c.wcls[cl];
    for (int t = 0; t <= fvc_dx::kMaxTaps; ++t)
      d.toff[cl][t] = t < c.ntaps[cl] ? (c.tdy[cl][t] - c.dymin) * d.ic + (c.tdx[cl][t] - c.dxmin) : 0;
  }
  // wave-tiles (class, first strip, first N-tile), cost = the class's taps. Two assignments:
  // unpaired -- largest first to the least-loaded SIMD, then to its less-loaded wave; paired -- the
  // wave-tiles of one (class, N-tiles) in pairs of strip groups as one job on SIMD partners w and
  // w + 4 at the same list position, so the two waves stream the same weight fragments together
  // (one L2 read feeds both through L1). Paired is taken unless its busiest SIMD carries > 15 % more
  // taps (FVC_DX_PAIR=0/1 forces either).
  struct WT {
    int cl, m0, n0, cost;
  };
  WT wt[64];
  int n = 0;
  for (int cl = 0; cl < 4; ++cl)
    for (int n0 = 0; n0 < c.ntp; n0 += wn)
      for (int m0 = 0; m0 < S; m0 += wm) {
        if (n >= 64) return FVC_EINVAL;
        wt[n++] = {cl, m0, n0, c.ntaps[cl]};
      }
  auto enc = [](const WT& t) { return t.cl | (t.m0 << 4) | (t.n0 << 8); };
  auto by_cost = [](WT* v, int k) {  // stable insertion sort, descending
    for (int i = 1; i < k; ++i)
      for (int j = i; j > 0 && v[j].cost > v[j - 1].cost; --j) {
        const WT t = v[j];
        v[j] = v[j - 1];
        v[j - 1] = t;
      }
  };
  int up[fvc_dx::kWaves][fvc_dx::kMaxWT], upc[fvc_dx::kWaves] = {0};
  int pp[fvc_dx::kWaves][fvc_dx::kMaxWT], ppc[fvc_dx::kWaves] = {0};
  int up_max = 0, pp_max = 1 << 30;
  {  // unpaired
    WT v[64];
    for (int i = 0; i < n; ++i) v[i] = wt[i];
    by_cost(v, n);
    int sl[4] = {0, 0, 0, 0}, wl[fvc_dx::kWaves] = {0};
    for (int i = 0; i < n; ++i) {
      int sm = 0;
      for (int q = 1; q < 4; ++q) sm = sl[q] < sl[sm] ? q : sm;
      int wv = wl[sm + 4] < wl[sm] ? sm + 4 : sm;
      if (upc[wv] == fvc_dx::kMaxWT) wv = wv == sm ? sm + 4 : sm;
      if (upc[wv] == fvc_dx::kMaxWT) return FVC_EINVAL;
      up[wv][upc[wv]++] = enc(v[i]);
      sl[sm] += v[i].cost;
      wl[wv] += v[i].cost;
    }
    for (int q = 0; q < 4; ++q) up_max = sl[q] > up_max ? sl[q] : up_max;
  }
  if ((S / wm) % 2 == 0) {  // paired: jobs = consecutive wave-tile pairs of one (class, N-tiles)
    WT jobs[32];
    int nj = 0;
    for (int i = 0; i + 1 < n; i += 2) jobs[nj++] = wt[i];  // wt[i + 1]: same class / N-tiles, next strips
    int jidx[32];
    for (int i = 0; i < nj; ++i) jidx[i] = i;
    for (int i = 1; i < nj; ++i)
      for (int j = i; j > 0 && jobs[jidx[j]].cost > jobs[jidx[j - 1]].cost; --j) {
        const int t = jidx[j];
        jidx[j] = jidx[j - 1];
        jidx[j - 1] = t;
      }
    int sl[4] = {0, 0, 0, 0};
    bool ok = true;
    for (int i = 0; i < nj && ok; ++i) {
      const int j = jidx[i];
      int sm = 0;
      for (int q = 1; q < 4; ++q) sm = sl[q] < sl[sm] ? q : sm;
      if (ppc[sm] == fvc_dx::kMaxWT) {
        ok = false;
        break;
      }
      pp[sm][ppc[sm]++] = enc(wt[2 * j]);
      pp[sm + 4][ppc[sm + 4]++] = enc(wt[2 * j + 1]);
      sl[sm] += 2 * jobs[j].cost;
    }
    if (ok) {
      pp_max = 0;
      for (int q = 0; q < 4; ++q) pp_max = sl[q] > pp_max ? sl[q] : pp_max;
    }
  }
  const int pair_env = env_int("FVC_DX_PAIR", -1);
  const bool paired = pp_max < (1 << 30) && (pair_env == 1 || (pair_env != 0 && pp_max * 100 <= up_max * 115));
  for (int wv = 0; wv < fvc_dx::kWaves; ++wv)
    for (int j = 0; j < fvc_dx::kMaxWT; ++j)
      d.wt[wv][j] = paired ? (j < ppc[wv] ? pp[wv][j] : -1) : (j < upc[wv] ? up[wv][j] : -1);
  d.y_bytes = y_bytes;
  d.x_bytes = x_bytes;
  d.ovf = ovf;
  d.tw = (const uint4*)tw;
  d.tosc = tosc;
  d.tosc_c = tosc * (1.0f / 2048.f);
  d.pcp = pcp;
  const int reserve = env_int("FVC_X3_RESERVE", -1) >= 0 ? env_int("FVC_X3_RESERVE", 0) : cu_reserve;
  const int ncu = x3_num_cus() - (reserve < x3_num_cus() / 2 ? reserve : x3_num_cus() / 2);
  const int grid = ncu < d.nitems ? ncu : d.nitems;
  d.sched = (sched && sched_len >= 2 && env_int("FVC_X3_DYN", 1)) ? sched : nullptr;
  const size_t lds = fvc_dx::lds_bytes(c.cinp, d.ps);
  return fvc_dx::launch(d, c.cinp, wm, wn, in_op, tap, grid, lds, s);
}

// tw != null: fused tap epilogue (y receives P [batch][Ho][Wo][pcp], see kPostTap)
static int run_x3(const float* x, const void* wpack, float osc, const float* bias, const float* res,
                  float* y, int batch, int h, int w, int cin, int cout, int ks, int stride, int transposed,
                  int in_op, int act, int post_op, int cu_reserve, int* ovf, int* sched, int sched_len,
                  hipStream_t s, const void* tw = nullptr, float tosc = 0.f, int pcp = 0, float* pool = nullptr) {
  X3Cfg c;
  if (!x3_cfg(cin, cout, ks, stride, transposed, c)) return FVC_EINVAL;
  if (!x || !wpack || !bias || !y || batch <= 0 || h <= 0 || w <= 0) return FVC_EINVAL;
  if (tw) {
    // every output channel in one wave: N-tiles 1, 2 (2 strips per wave) or 4 (1 strip); the
    // channel chunk (and so the weight pack) stays what x3_cfg chose: fewer strips only shrink LDS
    if (post_op != FVC_POST_NONE || in_op != FVC_IN_NONE || c.wl || c.ntp == 3 || c.ntp > 4 || pcp <= 0 ||
        pcp > 32 || (pcp & 3) || (c.dx && c.ntp != 4))
      return FVC_EINVAL;
    if (!c.dx) {
      if (c.ntp == 4) c.wm = 1;
      c.th = c.nw * c.wm;
    }
    post_op = kPostTap;
  }
  if (pool) {
    // y and avg_pool2d(y): stride-1 conv, two strips per wave (rows 2r, 2r + 1), one N-group
    if (tw || transposed || stride != 1 || post_op != FVC_POST_NONE || in_op != FVC_IN_NONE || c.wl || c.wm != 2 ||
        c.ntp > 2)
      return FVC_EINVAL;
    post_op = kPostPool;
  }
  const int ych = tw ? pcp : c.coutp;  // channels of the tensor y points to
  X3Args a;
  a.x = x; a.w = (const uint4*)wpack; a.bias = bias; a.res = res; a.y = y;
  a.tw = (const uint4*)tw; a.pcp = pcp;
  a.tosc = tosc; a.tosc_c = tosc * (1.0f / 2048.f);
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
  // y and res are addressed through buffer descriptors with 32-bit offsets: split batches whose
  // output tensor reaches 4 GB into launches over sub-batches
  const unsigned long long ybytes = (unsigned long long)batch * a.Ho * a.Wo * ych * 4ull;
  const unsigned long long rbytes = (unsigned long long)batch * a.Ho * a.Wo * a.coutp * 4ull;
  const long long split_env = env_int("FVC_X3_SPLIT_BYTES", 0);  // tests: force the split path
  const unsigned long long split_at = split_env > 0 ? (unsigned long long)split_env : (1ull << 32) - 4096;
  if (ybytes >= split_at || (res && rbytes >= split_at)) {
    if (batch == 1) return FVC_EINVAL;
    const int b1 = batch / 2;
    const size_t xs = (size_t)h * w * c.cinp, ys = (size_t)a.Ho * a.Wo * ych, rs = (size_t)a.Ho * a.Wo * c.coutp;
    const int post_in = (tw || pool) ? FVC_POST_NONE : post_op;
    const size_t pls = (size_t)(a.Ho / 2) * (a.Wo / 2) * c.coutp;
    int rc = run_x3(x, wpack, osc, bias, res, y, b1, h, w, cin, cout, ks, stride, transposed, in_op, act,
                    post_in, cu_reserve, ovf, sched, sched_len, s, tw, tosc, pcp, pool);
    if (rc) return rc;
    return run_x3(x + b1 * xs, wpack, osc, bias, res ? res + b1 * rs : nullptr, y + b1 * ys, batch - b1, h, w, cin, cout, ks,
                  stride, transposed, in_op, act, post_in, cu_reserve, ovf, sched, sched_len, s, tw, tosc, pcp,
                  pool ? pool + b1 * pls : nullptr);
  }
  a.y_bytes = (unsigned)ybytes;
  a.res_bytes = (unsigned)rbytes;
  a.pool = pool;
  a.pool_bytes = (unsigned)((unsigned long long)batch * (a.Ho / 2) * (a.Wo / 2) * c.coutp * 4ull);
  // the input is addressed per image (blockIdx.z) through a 32-bit-range descriptor too
  const unsigned long long xbytes = (unsigned long long)h * w * c.cinp * 4ull;
  if (xbytes >= (1ull << 32) - 4096) return FVC_EINVAL;
  a.x_bytes = (unsigned)xbytes;
  a.ovf = ovf;
  if (c.dx)
    return run_dx(c, x, wpack, osc, bias, res, y, batch, h, w, cout, in_op, act, post_op, cu_reserve, ovf, sched,
                  sched_len, s, tw, tosc, pcp, a.y_bytes, a.x_bytes);
  a.sin = c.sin; a.sout = c.sout; a.nclass = c.nclass; a.nchunks = c.nchunks; a.ntp = c.ntp;
  a.dymin = c.dymin; a.dxmin = c.dxmin;
  const int th = c.th;
  a.ir = (th - 1) * c.sin + 1 + (c.dymax - c.dymin);
  a.xcd = env_int("FVC_X3_XCD", 1) ? 1 : 0;
  a.prio = env_int("FVC_X3_PRIO", 0) ? 1 : 0;
  a.ic = 31 * c.sin + 1 + (c.dxmax - c.dxmin);
  a.pt = c.pt;
  if (c.pt && (tw || pool)) return FVC_EINVAL;
  a.half = c.sin == 2 ? (a.ic + 1) / 2 : 0;
  a.inv_ic = 1.0f / (float)a.ic;
  a.act_slope = act == FVC_ACT_RELU ? 0.f : (act == FVC_ACT_LRELU ? 0.1f : 1.f);
  a.in_op = in_op; a.act = act; a.post_op = post_op;
  a.osc = osc;
  a.osc_c = osc * (1.0f / 2048.f);
  for (int cl = 0; cl < 4; ++cl) {
    const bool v = cl < c.nclass;
    a.nks[cl] = v ? c.nks[cl] : 0;
    a.ntaps[cl] = v ? c.ntaps[cl] : 0;
    a.oy0[cl] = v ? c.oy0[cl] : 0;
    a.ox0[cl] = v ? c.ox0[cl] : 0;
    a.wcls[cl] = v ? c.wcls[cl] : 0;
  }
  a.ps = x3_plane_pix(a.ir, a.ic) * 8;
  for (int cl = 0; cl < 4; ++cl)
    for (int t = 0; t <= kMaxTapsX; ++t) {
      int off = 0;
      if (cl < c.nclass && t < c.ntaps[cl]) {
        const int cdy = c.tdy[cl][t] - c.dymin;
        const int cdx = c.tdx[cl][t] - c.dxmin;
        const int cpos = a.half ? ((cdx & 1) * a.half + (cdx >> 1)) : cdx;
        off = (cdy * a.ic + cpos) * 8;
      }
      a.toff[cl][t] = off;
    }
  size_t lds = 1024 + 2 * x3_tile_bytes(a.ir, a.ic, c.cc);
  const int tiles_x = fvc_cdiv(a.Wq, 32);
  const int tiles_y = fvc_cdiv(a.Hq, th);
  // N-tiles per block: 2 (each staged input element feeds 64 output channels) unless the layer
  // has too few spatial tiles x N-groups to give every CU of the persistent grid some work
  // stride-2 convs (one strip per wave) with 4 N-tiles take all 128 channels per block: the
  // input tile is staged once instead of twice (3x3 s2 128->128 at 544x960: 0.214 -> 0.191 ms)
  int wn = (c.wm == 1 && !transposed && stride == 2 && c.ntp % 4 == 0) ? 4 : (c.ntp >= 2 ? 2 : 1);
  const int want_wn = (tw || pool) ? c.ntp : env_int("FVC_X3_WN", 0);
  if (want_wn == 1 || want_wn == 2 || (want_wn == 4 && c.wm == 1)) wn = want_wn;
  while (wn > 1 && c.ntp % wn) wn >>= 1;
  const long long base = (long long)tiles_x * tiles_y * batch * c.nclass;
  if (!want_wn)
    while (wn > 1 && base * (c.ntp / wn) < 2LL * x3_num_cus()) wn >>= 1;
  if ((tw || pool) && wn != c.ntp) return FVC_EINVAL;
  // two N-groups of 4 waves x 4 strips instead of 8 waves x 2 strips x 2 N-tiles (same block
  // tile: 16 rows x 32 pixels x 64 channels): each weight fragment feeds 4 strips
  int wm = c.wm, wg = 1;
  if (c.nw == 8 && !c.wl && !tw && !pool && env_int("FVC_X3_WG", 0) == 2 && c.wm == 2 && wn == 2) {
    wm = 4;
    wn = 1;
    wg = 2;
  }
  const int nb = wn * wg;  // N-tiles per block
  if (wn > c.wnmax && c.wl) return FVC_EINVAL;
  a.wl_h = 0;
  if (c.wl) {
    int nkmax = 0;
    for (int cl = 0; cl < c.nclass; ++cl) nkmax = c.nks[cl] > nkmax ? c.nks[cl] : nkmax;
    a.wl_h = nkmax * wn * kFrag * 8;  // halves
    lds += 2 * (size_t)a.wl_h * 2;
  }
  if (lds > 160 * 1024) return FVC_EINVAL;
  // persistent grid: ~one 8-wave block per CU (FVC_X3_BPC blocks per CU), each walking a
  // contiguous run of spatial tiles
  // cu_reserve CUs are left out of the persistent grid for kernels of other streams (the
  // latency-bound rANS chains): a block that cannot find a free CU would start only when another
  // block has finished its whole run, doubling the launch's time (FVC_X3_RESERVE overrides)
  const int reserve = env_int("FVC_X3_RESERVE", -1) >= 0 ? env_int("FVC_X3_RESERVE", 0) : cu_reserve;
  const int ncu = x3_num_cus() - (reserve < x3_num_cus() / 2 ? reserve : x3_num_cus() / 2);
  const long long yz = (long long)(c.ntp / nb) * batch;
  const int bpc = env_int("FVC_X3_BPC", 1);
  long long gx = ((long long)ncu * bpc + yz - 1) / yz;  // blocks over all (tile, class) items
  if (gx > (long long)tiles_x * tiles_y * c.nclass) gx = (long long)tiles_x * tiles_y * c.nclass;
  if (gx < 1) gx = 1;
  dim3 grid((unsigned)gx, c.ntp / nb, batch);
  // dynamic schedule when the caller's scratch holds the group counters (FVC_X3_DYN=0: static runs)
  a.sched = (sched && sched_len >= 1 + (long long)grid.y * grid.z && env_int("FVC_X3_DYN", 1)) ? sched : nullptr;
  if (c.wl) {
    switch (c.cc) {
      case 8: return x3_launch_cc<8, 1>(c.nw, wm, wn, wg, in_op, post_op, a, grid, lds, s);
      case 16: return x3_launch_cc<16, 1>(c.nw, wm, wn, wg, in_op, post_op, a, grid, lds, s);
      case 32: return x3_launch_cc<32, 1>(c.nw, wm, wn, wg, in_op, post_op, a, grid, lds, s);
    }
    return FVC_EINVAL;
  }
  switch (c.cc) {
    case 8: return x3_launch_cc<8, 0>(c.nw, wm, wn, wg, in_op, post_op, a, grid, lds, s);
    case 16: return x3_launch_cc<16, 0>(c.nw, wm, wn, wg, in_op, post_op, a, grid, lds, s);
    case 32: return x3_launch_cc<32, 0>(c.nw, wm, wn, wg, in_op, post_op, a, grid, lds, s);
  }
  return FVC_EINVAL;
}

}  // namespace

extern "C" {

#if FVC_X3_TRACE
// diagnostic builds: copy (and clear) the per-wave segment sums [slot][8]
int fvc_x3_trace_read(unsigned long long* host, int nslots) {
  if (nslots > kTraceSlots) nslots = kTraceSlots;
  if (hipDeviceSynchronize() != hipSuccess) return FVC_EINVAL;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_x3_trace), (size_t)nslots * kTraceVals * 8) != hipSuccess) return FVC_EINVAL;
  static unsigned long long zeros[kTraceSlots * kTraceVals];
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_x3_trace), zeros, sizeof(zeros)) != hipSuccess) return FVC_EINVAL;
  return 0;
}
#endif

int fvc_conv_x3_supported(int cin, int cout, int ksize, int stride, int transposed) {
  X3Cfg c;
  return x3_cfg(cin, cout, ksize, stride, transposed, c) ? 1 : 0;
}

int fvc_deconv_x3_all_classes(int cin, int cout, int ksize, int stride) {
  X3Cfg c;
  return x3_cfg(cin, cout, ksize, stride, 1, c) && c.dx ? 1 : 0;
}

// The pack layout the current configuration gives this geometry (a hash of every X3Cfg field the
// pack's fragment order depends on: kernel family, channel chunk, pair-tap form, taps and k-steps
// per class, total size), or 0 when the x3 path does not take the layer. The env switches that
// choose these (FVC_DX, FVC_X3_PT, FVC_X3_CIN4, FVC_X3_CC, FVC_X3_SMALLN) are read at pack AND at
// launch: callers record the id with a pack and compare it before each launch, so a switch
// flipped in between is refused instead of running on a pack of another layout.
unsigned fvc_conv_x3_layout_id(int cin, int cout, int ksize, int stride, int transposed) {
  X3Cfg c;
  if (!x3_cfg(cin, cout, ksize, stride, transposed, c)) return 0u;
  unsigned h = 2166136261u;
  auto mix = [&](long long v) {
    for (int i = 0; i < 8; ++i) {
      h ^= (unsigned)(v >> (8 * i)) & 0xffu;
      h *= 16777619u;
    }
  };
  mix(c.dx);
  mix(c.cc);
  mix(c.pt);
  mix(c.nchunks);
  mix(c.ntp);
  mix(c.nclass);
  for (int cl = 0; cl < c.nclass; ++cl) {
    mix(c.ntaps[cl]);
    mix(c.nks[cl]);
  }
  mix(c.wtotal);
  return h ? h : 1u;
}

size_t fvc_conv_x3_wpack_bytes(int cin, int cout, int ksize, int stride, int transposed) {
  X3Cfg c;
  if (!x3_cfg(cin, cout, ksize, stride, transposed, c)) return 0;
  return (size_t)c.wtotal * 16;
}

int fvc_conv_x3_pack_weight(const float* w, void* wp, float* osc_out, int cin, int cout, int ks,
                            int stride, int transposed) {
  X3Cfg c;
  if (!x3_cfg(cin, cout, ks, stride, transposed, c) || !w || !wp || !osc_out) return FVC_EINVAL;
  const size_t nw = (size_t)cin * cout * ks * ks;
  const int kw = x3_kw(w, nw);
  const float sc = ldexpf(1.f, kw);
  *osc_out = ldexpf(1.f, -kw);
  _Float16* out = (_Float16*)wp;
  const int c8n = c.cc / 8;
  for (long long i = 0; i < c.wtotal * 8; ++i) out[i] = (_Float16)0.f;
  for (int cl = 0; cl < c.nclass; ++cl)
    for (int ch = 0; ch < c.nchunks; ++ch)
      for (int q = 0; q < c.nks[cl]; ++q)
        for (int nt = 0; nt < c.ntp; ++nt)
          for (int lane = 0; lane < 64; ++lane) {
            const int li = lane & 31, lh = lane >> 5;
            const int kb = 2 * q + lh;
            const int t = kb / c8n, o = kb % c8n;
            const int j = nt * 32 + li;
            if (t >= c.ntaps[cl] || (!c.pt && j >= cout)) continue;
            const int ky = c.tky[cl][t];
            const int kx = c.tkx[cl][t] + (c.pt && li >= 16 ? 1 : 0);  // pair-tap: rows 16-31 = odd tap
            const int jo = c.pt ? (li & 15) : j;                          // output channel of row li
            if (kx >= ks || jo >= cout) continue;
            const size_t frag = ((((size_t)c.wcls[cl] + (((size_t)ch * c.nks[cl] + q) * c.ntp + nt) * kFrag)) + lane) * 8;
            for (int e = 0; e < 8; ++e) {
              const int ci = ch * c.cc + o * 8 + e;
              if (ci >= cin) continue;
              const float v = (transposed ? w[(((size_t)ci * cout + jo) * ks + ky) * ks + kx]
                                          : w[(((size_t)jo * cin + ci) * ks + ky) * ks + kx]) * sc;
              const _Float16 hi = (_Float16)v;
              out[frag + e] = hi;  // plane 0 (hi): lanes 0..63
              if (kAcc1) {
                out[frag + 64 * 8 + e] = (_Float16)(v - (float)hi);                 // plane 1: w - hi
                out[frag + 128 * 8 + e] = (_Float16)((float)hi * (1.f / 2048.f));  // plane 2: hi 2^-11
              } else {
                out[frag + 64 * 8 + e] = (_Float16)((v - (float)hi) * 2048.f);  // plane 1: lo * 2^11
              }
            }
          }
  return 0;
}

// tap weights for the fused epilogue: w [np][cin] (np = k*k*cout partials of the next layer,
// row t*cout + co), cin = this conv's cout. Layout [k16 block kb][hi|lo][lane] of 16-B fragments;
// lane (li, lh) of block kb holds row li, channels 16kb + 4lh + {0,1,2,3,8,9,10,11} (the
// accumulator order of the producing tile, kPostTap), scaled by 2^kt like the conv packs.
static int x3_tap_blocks(int cin) { return 2 * fvc_cdiv(fvc_rup(cin, 4), 32); }

size_t fvc_x3_tap_wpack_bytes(int np, int cin) {
  if (np <= 0 || np > 32 || cin <= 0 || cin > 128) return 0;
  return (size_t)x3_tap_blocks(cin) * 2 * 64 * 16;
}

int fvc_x3_tap_pack_weight(const float* w, void* wp, float* osc_out, int np, int cin) {
  if (!w || !wp || !osc_out || !fvc_x3_tap_wpack_bytes(np, cin)) return FVC_EINVAL;
  const int kw = x3_kw(w, (size_t)np * cin);
  const float sc = ldexpf(1.f, kw);
  *osc_out = ldexpf(1.f, -kw);
  _Float16* out = (_Float16*)wp;
  const int nkb = x3_tap_blocks(cin);
  for (int kb = 0; kb < nkb; ++kb)
    for (int lane = 0; lane < 64; ++lane) {
      const int li = lane & 31, lh = lane >> 5;
      for (int t = 0; t < 8; ++t) {
        const int ci = 16 * kb + (t < 4 ? t : t + 4) + 4 * lh;
        const float v = (li < np && ci < cin) ? w[(size_t)li * cin + ci] * sc : 0.f;
        const _Float16 hi = (_Float16)v;
        out[((size_t)(kb * 2 + 0) * 64 + lane) * 8 + t] = hi;
        out[((size_t)(kb * 2 + 1) * 64 + lane) * 8 + t] = (_Float16)((v - (float)hi) * 2048.f);
      }
    }
  return 0;
}

int fvc_conv_x3_tap_supported(int cin, int cout, int ksize, int stride, int transposed, int pcp) {
  X3Cfg c;
  if (!x3_cfg(cin, cout, ksize, stride, transposed, c) || c.wl || c.pt || pcp <= 0 || pcp > 32 || (pcp & 3)) return 0;
  if (c.dx) return c.ntp == 4;  // the all-classes kernel's tap form: 1 strip x 4 N-tiles
  const int wm = c.ntp == 4 ? 1 : c.wm;
  return (wm == 2 && c.ntp <= 2) || (wm == 1 && c.ntp == 4);
}

int fvc_conv2d_nhwc_x3_tap(const float* x, const void* wpack, float osc, const float* bias, const float* res,
                           float* P, int batch, int h, int w, int cin, int cout, int ksize, int stride, int act,
                           const void* tap_wpack, float tap_osc, int pcp, int cu_reserve, int* overflow_flag,
                           int* sched, int sched_len, fvc_stream_t stream) {
  if (cu_reserve < 0 || sched_len < 0 || !tap_wpack || !fvc_conv_x3_tap_supported(cin, cout, ksize, stride, 0, pcp))
    return FVC_EINVAL;
  return run_x3(x, wpack, osc, bias, res, P, batch, h, w, cin, cout, ksize, stride, 0, FVC_IN_NONE, act,
                FVC_POST_NONE, cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream, tap_wpack, tap_osc,
                pcp);
}

int fvc_deconv2d_nhwc_x3_tap(const float* x, const void* wpack, float osc, const float* bias, const float* res,
                             float* P, int batch, int h, int w, int cin, int cout, int ksize, int stride, int act,
                             const void* tap_wpack, float tap_osc, int pcp, int cu_reserve, int* overflow_flag,
                             int* sched, int sched_len, fvc_stream_t stream) {
  if (cu_reserve < 0 || sched_len < 0 || !tap_wpack || !fvc_conv_x3_tap_supported(cin, cout, ksize, stride, 1, pcp))
    return FVC_EINVAL;
  return run_x3(x, wpack, osc, bias, res, P, batch, h, w, cin, cout, ksize, stride, 1, FVC_IN_NONE, act,
                FVC_POST_NONE, cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream, tap_wpack, tap_osc,
                pcp);
}

int fvc_conv_x3_pool_supported(int cin, int cout, int ksize) {
  X3Cfg c;
  return x3_cfg(cin, cout, ksize, 1, 0, c) && !c.wl && !c.pt && c.wm == 2 && c.ntp <= 2;
}

int fvc_conv2d_nhwc_x3_pool(const float* x, const void* wpack, float osc, const float* bias, const float* res,
                            float* y, float* pool, int batch, int h, int w, int cin, int cout, int ksize, int act,
                            int cu_reserve, int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream) {
  if (cu_reserve < 0 || sched_len < 0 || !pool || !fvc_conv_x3_pool_supported(cin, cout, ksize)) return FVC_EINVAL;
  return run_x3(x, wpack, osc, bias, res, y, batch, h, w, cin, cout, ksize, 1, 0, FVC_IN_NONE, act, FVC_POST_NONE,
                cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream, nullptr, 0.f, 0, pool);
}

int fvc_conv2d_nhwc_x3(const float* x, const void* wpack, float osc, const float* bias,
                       const float* res, float* y, int batch, int h, int w, int cin, int cout,
                       int ksize, int stride, int in_op, int act, int post_op, int cu_reserve,
                       int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream) {
  if (cu_reserve < 0 || sched_len < 0) return FVC_EINVAL;
  return run_x3(x, wpack, osc, bias, res, y, batch, h, w, cin, cout, ksize, stride, 0, in_op, act,
                post_op, cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream);
}

int fvc_deconv2d_nhwc_x3(const float* x, const void* wpack, float osc, const float* bias,
                         const float* res, float* y, int batch, int h, int w, int cin, int cout,
                         int ksize, int stride, int in_op, int act, int post_op, int cu_reserve,
                         int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream) {
  if (cu_reserve < 0 || sched_len < 0) return FVC_EINVAL;
  return run_x3(x, wpack, osc, bias, res, y, batch, h, w, cin, cout, ksize, stride, 1, in_op, act,
                post_op, cu_reserve, overflow_flag, sched, sched_len, (hipStream_t)stream);
}

}  // extern "C"
