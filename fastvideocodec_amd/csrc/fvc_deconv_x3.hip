// Split-precision stride-2 transposed convolution with all four output-parity classes computed from
// ONE staged input tile (DVC/subnet/synthesis_mv.py:15-41 mvDecoder 3x3 128->128 deconvs,
// synthesis.py:14-27 resDecoder and synthesis_prior.py hyperprior 5x5 64/96->64 deconvs; the ATen
// conv_transpose2d calls with stride 2, padding k//2, output_padding 1).
//
// A stride-2 transposed conv splits into four stride-1 convs, one per output parity (py, px), over
// disjoint tap subsets (3x3: 1, 2, 2 and 4 taps; 5x5: 9, 6, 6, 4). fvc_conv_x3.hip runs them as four
// work items per tile, each re-staging the same input tile and each with a short K (one 3x3 tap of
// 128 channels = 8 k-steps): staging, chunk ends and barriers dominate (d3_128_half at 150-190 TF/s
// vs 320 for a stride-1 conv of equal work). Here a work item is R input rows x 32 input columns,
// all cin channels staged once into LDS (fp16 hi/lo octet planes, as fvc_conv_x3.hip), and the 8
// waves share out the item's (class, strip pair, N-tile pair) wave-tiles: wave w and its SIMD
// partner w + 4 together get an equal number of taps (host-side LPT assignment), so every SIMD's
// matrix pipe has the same work per item. Two tile buffers: the next item's tile is staged during
// the current item's k-loops (one barrier per item).
//
// Numerics are fvc_conv_x3.hip's: weights scaled by 2^kw and split hi + lo 2^-11 at pack time (the
// x3 pack with one channel chunk), activations split at staging, main += w_hi x_hi and
// corr += w_lo x_hi + w_hi x_lo in two fp32 accumulators; an activation >= 65000 raises the caller's
// overflow flag. Epilogue: scale + bias, ReLU / LeakyReLU, optional residual and exp, 16-B stores;
// or (tap form, 1 strip x all N-tiles per wave-tile) the next layer's tap partials, exactly as
// fvc_conv_x3.hip's kPostTap.
#include "fvc_dx.h"
#include <math.h>

namespace fvc_dx {

// cache policy of the activation stores (aux operand of buffer_store; experiment builds only,
// e.g. 2 = non-temporal on gfx950)
#ifndef FVC_STORE_AUX
#define FVC_STORE_AUX 0
#endif
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr float kLoScale = 2048.f;
constexpr unsigned kOob = 0xFFFFFF00u;
constexpr int kRsrcFlags = 0x00020000;
constexpr int kNT = 512;     // threads per block (8 waves, 2 per SIMD)
constexpr int kFrag = 128;   // uint4 per (k-step, N-tile): hi and lo planes x 64 lanes
constexpr int kHdr = 1024;   // LDS header: bias (512 B), staging sink, work-item queue
// FVC_DX_KO (compile-time, experiment builds only -- wrong results): knock out parts of the item to
// find the binding unit. bit 0: weight loads (registers), bit 1: staging of the next tile, bit 2:
// LDS operand reads (registers), bit 3: MFMAs, bit 4: epilogue stores
#ifndef FVC_DX_KO
#define FVC_DX_KO 0
#endif
constexpr int kKO = FVC_DX_KO;

template <int IOP>
__device__ __forceinline__ float in_op_t(float v) {
  if (IOP == FVC_IN_RELU) return fmaxf(v, 0.f);
  if (IOP == FVC_IN_ABS) return fabsf(v);
  if (IOP == FVC_IN_ROUND) return rintf(v);  // torch.round: half-to-even
  return v;
}

// v = hi + lo * 2^-11 for 8 values; mx tracks max |v| (fp16 representability, |v| < 65000)
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, kRsrcFlags);
}

template <int CIN, int WM, int WN, int IOP, bool TAP, int SW>
__global__ __launch_bounds__(kNT) void conv_dx_kernel(const DxArgs a) {
  static_assert(SW == 32 || SW == 16, "strip shapes: 1 x 32 or 2 x 16 input pixels");
  constexpr int SR = 32 / SW;   // input rows per strip
  constexpr int C8 = CIN / 8;   // channel octets (LDS planes per hi / lo half)
  constexpr int KPT = C8 / 2;   // k-steps per tap (one k-step = two octets of one tap)
  static_assert(C8 % 2 == 0, "a k-step's two octets must belong to one tap");

  extern __shared__ __attribute__((aligned(16))) _Float16 smh[];
  float* const sbias = reinterpret_cast<float*>(smh);          // bytes 0..511
  _Float16* const sdump = smh + 256;                           // bytes 512..543: staging sink
  int* const squeue = reinterpret_cast<int*>(smh) + 144;       // bytes 576..591: items k .. k+3
  _Float16* const tile0 = smh + kHdr / 2;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31;
  const int lh = lane >> 5;
  // the lane's pixel in its strip (MFMA column li): 1 x 32 strips take column li; 2 x 16 strips take
  // row li >> 4 and, on the second row, the columns rotated by one ((li - 17) & 15) so that each
  // 16-lane group of a ds_read_b128 hits 16 distinct bank quads with the odd row pitch of 17 pixels
  const int sdr = SW == 32 ? 0 : (li >> 4);
  const int sdc = SW == 32 ? li : (li < 16 ? li : ((li - 17) & 15));
  const int psh = a.ps * 8;           // halves per LDS plane
  const int tile_h = 2 * C8 * psh;    // halves per tile buffer
  const int Ho = 2 * a.H, Wo = 2 * a.W;
  const int tile_items = a.ir * a.ic * C8;
  const int nstage = (tile_items + kNT - 1) / kNT;
  float mx = 0.f;

  // ---- work items: (image, tile row, tile column), row-major, from the launch's counter (or a
  // static stride); item k + 2 is taken when item k starts and published at item k's barrier
  int* const ctr = a.sched ? a.sched + 1 : nullptr;
  auto take = [&](int k) -> int {  // thread 0 only
    if (ctr) return atomicAdd(ctr, 1);
    return (int)blockIdx.x + k * (int)gridDim.x;
  };
  auto finish = [&]() {  // every block once: the last one leaves the counters zeroed
    if (ctr && tid == 0) {
      __threadfence();
      if (atomicAdd(a.sched, 1) == (int)gridDim.x - 1) {
        atomicExch(a.sched + 1, 0);
        atomicExch(a.sched, 0);
      }
    }
  };
  auto decode = [&](int it, int& b, int& ty0, int& tx0) {
    const int per = a.tiles_x * a.tiles_y;
    b = it / per;
    const int r = it - b * per;
    const int ty = r / a.tiles_x;
    ty0 = ty * a.R;
    tx0 = (r - ty * a.tiles_x) * SW;
  };

  // ---- staging: item e = (tile pixel p, octet o) -> two 16-B loads (halo pixels outside the
  // image read zeros through the descriptor range), in_op + split + LDS write after the MFMAs
  struct Stage {
    float4 v0, v1;
    int dst;
    bool ok;
  };
  auto fetch = [&](int e, const __amdgpu_buffer_rsrc_t& rx, int iy0, int ix0, Stage& st) {
    if constexpr ((kKO & 2) != 0) return;
    st.ok = e < tile_items;
    e = st.ok ? e : tile_items - 1;
    const int p = e / C8;
    const int o = e - p * C8;
    const int r = (int)(((float)p + 0.5f) * a.inv_ic);  // exact: p < 2^14
    const int c = p - r * a.ic;
    const int iy = iy0 + r, ix = ix0 + c;
    const bool inb = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    const unsigned off = inb ? ((unsigned)(iy * a.W + ix) * (unsigned)CIN + (unsigned)(o * 8)) * 4u : kOob;
    st.v0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
    st.v1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rx, off + 16u, 0, 0));
    st.dst = o * psh + p * 8;
  };
  auto store = [&](_Float16* t, const Stage& st) {
    if constexpr ((kKO & 2) != 0) return;
    float v[8] = {st.v0.x, st.v0.y, st.v0.z, st.v0.w, st.v1.x, st.v1.y, st.v1.z, st.v1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = in_op_t<IOP>(v[i]);
    h8 hi, lo;
    split8(v, hi, lo, mx);
    _Float16* const ph = st.ok ? t + st.dst : sdump;
    _Float16* const pl = st.ok ? t + st.dst + C8 * psh : sdump + 8;
    *reinterpret_cast<h8*>(ph) = hi;
    *reinterpret_cast<h8*>(pl) = lo;
  };
  auto image_rsrc = [&](int b) {
    return rsrc(a.x + (size_t)b * a.H * a.W * CIN, a.x_bytes);
  };

  if (tid == 0) {
    squeue[0] = take(0);
    squeue[1] = take(1);
  }
  if (tid < a.coutp) sbias[tid] = tid < a.cout ? a.bias[tid] : 0.f;
  __syncthreads();
  const int first = squeue[0];
  if (first >= a.nitems) {
    finish();
    return;
  }
  int b, ty0, tx0;
  decode(first, b, ty0, tx0);
  {
    const __amdgpu_buffer_rsrc_t rx = image_rsrc(b);
    for (int e = tid; e < tile_items; e += kNT) {
      Stage st;
      fetch(e, rx, ty0 + a.dymin, tx0 + a.dxmin, st);
      store(tile0, st);
    }
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t ry = rsrc(a.y, a.y_bytes);
  const __amdgpu_buffer_rsrc_t rr = rsrc(a.res, a.res ? a.y_bytes : 0u);
  int buf = 0;
  for (int k = 0;; ++k) {
    const int it = squeue[k & 3];
    if (it >= a.nitems) break;
    int taken = 0;
    if (tid == 0) taken = take(k + 2);
    decode(it, b, ty0, tx0);
    const int s_it = squeue[(k + 1) & 3];
    const bool stage_next = s_it < a.nitems;
    int sb = 0, sty0 = 0, stx0 = 0;
    if (stage_next) decode(s_it, sb, sty0, stx0);
    const __amdgpu_buffer_rsrc_t rxs = image_rsrc(sb);
    const int siy0 = sty0 + a.dymin, six0 = stx0 + a.dxmin;
    const _Float16* const cur = tile0 + buf * tile_h;
    _Float16* const nxt = tile0 + (buf ^ 1) * tile_h;
    int staged = 0;

    for (int j = 0; j < kMaxWT; ++j) {
      const int ent = a.wt[wave][j];
      if (ent < 0) break;
      const int cls = ent & 15, m0 = (ent >> 4) & 15, n0 = (ent >> 8) & 15;
      const int nq = a.nks[cls];
      // tap window offsets one per lane; v_readlane makes them wave-uniform in the k-loop
      const int tap_tab = a.toff[cls][lane <= kMaxTaps ? lane : kMaxTaps];
      const uint4* const wcl = a.w + a.wcls[cls] + lane;
      int pix[WM];
#pragma unroll
      for (int m = 0; m < WM; ++m) pix[m] = (((m0 + m) * SR + sdr) * a.ic + sdc) * 8;

      f32x16 acc[WM][WN], cor[WM][WN];
#pragma unroll
      for (int m = 0; m < WM; ++m)
#pragma unroll
        for (int n = 0; n < WN; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[m][n][r] = cor[m][n][r] = 0.f;

      struct Ops {
        h8 ah[WM], al[WM];
        uint4 bh[WN], bl[WN];
      };
      // k-step q = tap q / KPT, octets 2 (q % KPT) + lh of that tap
      auto load = [&](int q, Ops& op) {
        const int t = q / KPT;
        const int toffh = __builtin_amdgcn_readlane(tap_tab, t) * 8 + (2 * (q - t * KPT) + lh) * psh;
#pragma unroll
        for (int m = 0; m < WM; ++m) {
          if constexpr ((kKO & 4) != 0) {
            op.ah[m] = h8{} + (_Float16)(q + m + toffh);
            op.al[m] = h8{} + (_Float16)(q);
            continue;
          }
          op.ah[m] = *reinterpret_cast<const h8*>(cur + toffh + pix[m]);
          op.al[m] = *reinterpret_cast<const h8*>(cur + toffh + pix[m] + C8 * psh);
        }
        const uint4* const wk = wcl + ((size_t)q * a.ntp + n0) * kFrag;
#pragma unroll
        for (int n = 0; n < WN; ++n) {
          if constexpr ((kKO & 1) != 0) {
            op.bh[n] = uint4{(unsigned)(q + n), 1u, 2u, 3u};
            op.bl[n] = uint4{(unsigned)q, 5u, 6u, 7u};
            continue;
          }
          op.bh[n] = wk[n * kFrag];
          op.bl[n] = wk[n * kFrag + 64];
        }
      };
      // weights as the A (row) operand, pixels as B: lane (li, lh) ends with 4 consecutive
      // channels of pixel li per register group
      auto mfmas = [&](const Ops& op) {
        if constexpr ((kKO & 8) != 0) {
#pragma unroll
          for (int m = 0; m < WM; ++m)
#pragma unroll
            for (int n = 0; n < WN; ++n)
              acc[m][n][0] += (float)op.ah[m][0] + (float)op.al[m][1] + __builtin_bit_cast(float, op.bh[n].x) +
                              __builtin_bit_cast(float, op.bl[n].y);
          return;
        }
#pragma unroll
        for (int m = 0; m < WM; ++m)
#pragma unroll
          for (int n = 0; n < WN; ++n) {
            const h8 wh = __builtin_bit_cast(h8, op.bh[n]);
            const h8 wl = __builtin_bit_cast(h8, op.bl[n]);
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, op.ah[m], acc[m][n], 0, 0, 0);
            cor[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, op.ah[m], cor[m][n], 0, 0, 0);
            cor[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, op.al[m], cor[m][n], 0, 0, 0);
          }
      };
      auto pin = []() { __builtin_amdgcn_sched_barrier(0); };
      // nq is even (KPT is); each pair of half-steps: load q+1 / MFMAs q / load q+2 / MFMAs q+1
      // (the last prefetch repeats q = nq - 1, harmlessly); one staging item of the next tile per
      // pair while this wave's share is not done, its split + LDS write after the pair
      Ops S0, S1;
      load(0, S0);
      const int npair = nq >> 1;
      const int nst = stage_next ? min(nstage - staged, npair) : 0;
      const int spread = nst ? max(1, npair / nst) : 1;
      int q = 0;
      for (int s = 0; s < nst; ++s) {
        load(q + 1, S1);
        Stage st;
        fetch(tid + (staged + s) * kNT, rxs, siy0, six0, st);
        pin();
        mfmas(S0);
        pin();
        load(q + 2 < nq ? q + 2 : nq - 1, S0);
        pin();
        mfmas(S1);
        pin();
        store(nxt, st);
        q += 2;
        for (int r = 1; r < spread && q < nq; ++r, q += 2) {
          load(q + 1, S1);
          pin();
          mfmas(S0);
          pin();
          load(q + 2 < nq ? q + 2 : nq - 1, S0);
          pin();
          mfmas(S1);
          pin();
        }
      }
      staged += nst;
      for (; q < nq; q += 2) {
        load(q + 1, S1);
        pin();
        mfmas(S0);
        pin();
        load(q + 2 < nq ? q + 2 : nq - 1, S0);
        pin();
        mfmas(S1);
        pin();
      }

      // ---- epilogue of this wave-tile: input position (row, col) of strip m, lane li ->
      // output pixel (2 row + py, 2 col + px); lane (li, lh) holds channels 8g + 4lh + {0..3}
      const int oyc = a.oy0[cls], oxc = a.ox0[cls];
      const int col = tx0 + sdc;
      if constexpr (TAP) {
#pragma unroll
        for (int m = 0; m < WM; ++m) {
          const int row = ty0 + (m0 + m) * SR + sdr;
          const bool ok = row < a.H && col < a.W;
          const unsigned pixo = ((unsigned)b * Ho + 2 * row + oyc) * (unsigned)Wo + 2 * col + oxc;
          f32x16 pa, pc;
#pragma unroll
          for (int r = 0; r < 16; ++r) pa[r] = pc[r] = 0.f;
#pragma unroll
          for (int n = 0; n < WN; ++n) {
            float yv[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const float4 bj = *reinterpret_cast<const float4*>(sbias + (n0 + n) * 32 + 8 * g + 4 * lh);
              const float bb[4] = {bj.x, bj.y, bj.z, bj.w};
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int r = 4 * g + i;
                const float tv = fmaf(cor[m][n][r], a.osc_c, fmaf(acc[m][n][r], a.osc, bb[i]));
                yv[r] = fmaxf(tv, tv * a.act_slope);
              }
            }
            // registers 8gp..8gp+7 of N-tile n are the B operand of k16 block 2n + gp (the tap
            // pack's channel order, fvc_x3_tap_pack_weight)
#pragma unroll
            for (int gp = 0; gp < 2; ++gp) {
              float v8[8];
#pragma unroll
              for (int t = 0; t < 8; ++t) v8[t] = yv[8 * gp + t];
              h8 yh, yl;
              split8(v8, yh, yl, mx);
              const uint4* const tw = a.tw + (size_t)(((n0 + n) * 2 + gp) * 2) * 64 + lane;
              const h8 wh = __builtin_bit_cast(h8, tw[0]);
              const h8 wl = __builtin_bit_cast(h8, tw[64]);
              pa = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yh, pa, 0, 0, 0);
              pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl, yh, pc, 0, 0, 0);
              pc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh, yl, pc, 0, 0, 0);
            }
          }
          const unsigned po = pixo * (unsigned)a.pcp * 4u + (unsigned)(4 * lh) * 4u;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int p0 = 8 * g + 4 * lh;
            float o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = fmaf(pc[4 * g + i], a.tosc_c, pa[4 * g + i] * a.tosc);
            const unsigned so = (ok && p0 < a.pcp && !(kKO & 16)) ? po + 32u * g : kOob;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_float4(o[0], o[1], o[2], o[3])), ry,
                                                   so, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int m = 0; m < WM; ++m) {
          const int row = ty0 + (m0 + m) * SR + sdr;
          const bool ok = row < a.H && col < a.W;
          const unsigned pixo = ((unsigned)b * Ho + 2 * row + oyc) * (unsigned)Wo + 2 * col + oxc;
#pragma unroll
          for (int n = 0; n < WN; ++n) {
            const unsigned vo = pixo * (unsigned)a.coutp * 4u + (unsigned)((n0 + n) * 32 + 4 * lh) * 4u;
            float4 rq[4];
            if (a.res) {
#pragma unroll
              for (int g = 0; g < 4; ++g)
                rq[g] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rr, vo + 32u * g, 0, 0));
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int j0 = (n0 + n) * 32 + 8 * g + 4 * lh;
              const float4 bj = *reinterpret_cast<const float4*>(sbias + j0);
              const float bb[4] = {bj.x, bj.y, bj.z, bj.w};
              float v[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int r = 4 * g + i;
                const float tv = fmaf(cor[m][n][r], a.osc_c, fmaf(acc[m][n][r], a.osc, bb[i]));
                v[i] = fmaxf(tv, tv * a.act_slope);
              }
              if (a.res) {
                v[0] += rq[g].x;
                v[1] += rq[g].y;
                v[2] += rq[g].z;
                v[3] += rq[g].w;
              }
              if (a.post_exp) {
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = j0 + i < a.cout ? expf(v[i]) : 0.f;
              }
              const unsigned so = (ok && j0 < a.coutp && !(kKO & 16)) ? vo + 32u * g : kOob;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_float4(v[0], v[1], v[2], v[3])),
                                                     ry, so, 0, FVC_STORE_AUX);
            }
          }
        }
      }
    }
    // the rest of this thread's share of the next tile
    if (stage_next) {
      for (; staged < nstage; ++staged) {
        Stage st;
        fetch(tid + staged * kNT, rxs, siy0, six0, st);
        store(nxt, st);
      }
    }
    if (tid == 0) squeue[(k + 2) & 3] = taken;
    __syncthreads();
    buf ^= 1;
  }
  if (!(mx < 65000.f) && a.ovf) atomicOr(a.ovf, 1);
  finish();
}

template <int CIN, int WM, int WN, int IOP, bool TAP>
int launch_t(const DxArgs& a, int grid, size_t lds, hipStream_t s) {
  // 128-channel layers: 2 x 16-pixel strips (8-row items: two full-channel buffers still fit);
  // fewer channels: 1 x 32-pixel strips
  constexpr int SW = CIN == 128 ? 16 : 32;
  if (a.sw != SW) return FVC_EINVAL;
  const hipError_t e = hipFuncSetAttribute((const void*)conv_dx_kernel<CIN, WM, WN, IOP, TAP, SW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return -(int)e;
  hipLaunchKernelGGL((conv_dx_kernel<CIN, WM, WN, IOP, TAP, SW>), dim3(grid), dim3(kNT), lds, s, a);
  FVC_CHECK_LAUNCH();
  return 0;
}

template <int CIN>
int launch_cin(const DxArgs& a, int wm, int wn, int iop, bool tap, int grid, size_t lds, hipStream_t s) {
  if (tap) {
    if constexpr (CIN == 128)
      if (wm == 1 && wn == 4 && iop == FVC_IN_NONE) return launch_t<CIN, 1, 4, FVC_IN_NONE, true>(a, grid, lds, s);
    return FVC_EINVAL;
  }
  if (wm != 2 || wn != 2) return FVC_EINVAL;
  switch (iop) {
    case FVC_IN_NONE: return launch_t<CIN, 2, 2, FVC_IN_NONE, false>(a, grid, lds, s);
    case FVC_IN_RELU: return launch_t<CIN, 2, 2, FVC_IN_RELU, false>(a, grid, lds, s);
    case FVC_IN_ABS: return launch_t<CIN, 2, 2, FVC_IN_ABS, false>(a, grid, lds, s);
    case FVC_IN_ROUND: return launch_t<CIN, 2, 2, FVC_IN_ROUND, false>(a, grid, lds, s);
  }
  return FVC_EINVAL;
}

}  // namespace

size_t lds_bytes(int cinp, int ps) { return (size_t)kHdr + 2 * (size_t)cinp * 4 * (size_t)ps; }

int plane_pix(int ir, int ic) { return (ir * ic) | 1; }

int launch(const DxArgs& a, int cinp, int wm, int wn, int iop, bool tap, int grid, size_t lds, hipStream_t s) {
  if (grid <= 0 || lds > 160 * 1024) return FVC_EINVAL;
  switch (cinp) {
    case 64: return launch_cin<64>(a, wm, wn, iop, tap, grid, lds, s);
    case 96: return launch_cin<96>(a, wm, wn, iop, tap, grid, lds, s);
    case 128: return launch_cin<128>(a, wm, wn, iop, tap, grid, lds, s);
  }
  return FVC_EINVAL;
}

}  // namespace fvc_dx
