// Entropy-coding kernels: latent <-> symbol streams, scale-table indexes, and a batched
// device rANS coder that is byte-compatible, stream for stream, with compressai's
// RansEncoder/RansDecoder.{encode,decode}_with_indexes (ryg_rans 64-bit state, 32-bit words,
// precision 16, 4-bit bypass for escapes), the C++ coder the reference reaches through
// entropy_models.py:80-94 (RecProbModel.compress/decompress).
//
// Parallelism: one lane per independent stream (a stream = one channel of one latent of one
// frame); a stream's symbol loop is inherently sequential (rANS state chain).
#include "fvc_common.h"
#include <stdlib.h>

namespace {

constexpr int kBlk = 256;
constexpr uint64_t kRansL = 1ull << 31;
constexpr int kPrec = 16;
constexpr int kBypassPrec = 4;
constexpr int kMaxBypass = (1 << kBypassPrec) - 1;

__global__ void k_latent_to_symbols(const float* __restrict__ lat, int32_t* __restrict__ sym, int B, int HW, int C,
                                    int cp) {
  const size_t n = (size_t)B * C * HW;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t i = e % HW;
    const size_t bc = e / HW;
    const size_t c = bc % C, b = bc / C;
    sym[e] = (int32_t)rintf(lat[(b * HW + i) * cp + c]);
  }
}

__global__ void k_symbols_to_latent(const int32_t* __restrict__ sym, float* __restrict__ lat, int B, int HW, int C,
                                    int cp) {
  const size_t n = (size_t)B * HW * cp;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const int c = e % cp;
    const size_t p = e / cp;
    const size_t b = p / HW, i = p % HW;
    lat[e] = c < C ? (float)sym[(b * C + c) * HW + i] : 0.f;
  }
}

// compressai GaussianConditional.build_indexes: s = max(scale, 0.11);
// idx = (n-1) - #{t in table[:-1] : s <= t}
__global__ void k_build_indexes(const float* __restrict__ sigma, const float* __restrict__ table, int nt,
                                int32_t* __restrict__ idx, int B, int HW, int C, int cp) {
  const size_t n = (size_t)B * C * HW;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const size_t i = e % HW;
    const size_t bc = e / HW;
    const size_t c = bc % C, b = bc / C;
    const float s = fmaxf(sigma[(b * HW + i) * cp + c], 0.11f);
    int v = nt - 1;
    for (int k = 0; k < nt - 1; ++k) v -= (s <= table[k]) ? 1 : 0;
    idx[e] = v;
  }
}

__global__ void k_channel_indexes(int32_t* __restrict__ idx, int B, int HW, int C) {
  const size_t n = (size_t)B * C * HW;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    idx[e] = (int32_t)((e / HW) % C);
}

// compressai EntropyModel.quantize(x, "symbols", means) = round(x - means).int() and
// dequantize(symbols, means) = symbols + means, elementwise over any contiguous layout
__global__ void k_quantize_symbols(const float* __restrict__ x, const float* __restrict__ means,
                                   int32_t* __restrict__ sym, size_t n) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    sym[e] = (int32_t)rintf(means ? x[e] - means[e] : x[e]);
}

__global__ void k_dequantize_symbols(const int32_t* __restrict__ sym, const float* __restrict__ means,
                                     float* __restrict__ out, size_t n) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x)
    out[e] = means ? (float)sym[e] + means[e] : (float)sym[e];
}

__global__ void k_build_indexes_flat(const float* __restrict__ scales, const float* __restrict__ table, int nt,
                                     int32_t* __restrict__ idx, size_t n) {
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const float s = fmaxf(scales[e], 0.11f);
    int v = nt - 1;
    for (int k = 0; k < nt - 1; ++k) v -= (s <= table[k]) ? 1 : 0;
    idx[e] = v;
  }
}

// ---- ryg_rans 64-bit primitives (rans64.h) + compressai bypass extension
__device__ __forceinline__ bool enc_put_bits(uint64_t& x, uint32_t*& ptr, const uint32_t* lo, uint32_t val) {
  const uint32_t freq = 1u << (16 - kBypassPrec);
  const uint64_t x_max = ((kRansL >> 16) << 32) * freq;
  if (x >= x_max) {
    if (ptr <= lo) return false;
    *--ptr = (uint32_t)x;
    x >>= 32;
  }
  x = (x << kBypassPrec) | val;
  return true;
}

// Phase 1 (fully parallel over all symbols): table lookups plus ryg_rans' reciprocal form of
// the division (Rans64EncSymbolInit: q = mulhi64(x, rcp) >> shift, exact for every x the coder
// can hold), so the sequential phase has no divide on its critical path.
struct EncSym {
  uint64_t rcp;     // rcp_freq
  uint32_t sf;      // start | freq << 16
  uint32_t shift;   // rcp_shift | escape flag << 8
};

__device__ __forceinline__ EncSym make_enc_sym(uint32_t start, uint32_t freq, bool esc) {
  EncSym e;
  e.sf = start | (freq << 16);
  if (freq < 2) {
    e.rcp = ~0ull;
    e.shift = 0;
  } else {
    uint32_t shift = 0;
    while (freq > (1u << shift)) shift++;
    uint64_t x0 = freq - 1, x1 = 1ull << (shift + 31);
    const uint64_t t1 = x1 / freq;
    x0 += (x1 % freq) << 32;
    const uint64_t t0 = x0 / freq;
    e.rcp = t0 + (t1 << 32);
    e.shift = shift - 1;
  }
  if (esc) e.shift |= 0x100u;
  return e;
}

__global__ void k_rans_prep(const int32_t* __restrict__ symbols, const int32_t* __restrict__ indexes, int64_t n,
                            const int32_t* __restrict__ cdfs, int cdf_stride, const int32_t* __restrict__ cdf_sizes,
                            const int32_t* __restrict__ offsets, EncSym* __restrict__ prep,
                            uint32_t* __restrict__ raw_out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t ci = indexes[i];
    const int32_t* cdf = cdfs + (size_t)ci * cdf_stride;
    const int32_t max_value = cdf_sizes[ci] - 2;
    int32_t value = symbols[i] - offsets[ci];
    uint32_t raw = 0;
    if (value < 0) {
      raw = (uint32_t)(-2 * value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw = (uint32_t)(2 * (value - max_value));
      value = max_value;
    }
    const uint32_t start = (uint32_t)cdf[value];
    const uint32_t freq = (uint32_t)(cdf[value + 1] - cdf[value]);  // < 65536: every table has >= 2 bins
    prep[i] = make_enc_sym(start, freq, value == max_value);
    raw_out[i] = raw;
  }
}

__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// Phase 2: one lane per stream walks its symbols backward (compressai's BufferedRansEncoder
// pushes forward and flushes backward; each symbol's sub-symbols are put in reverse push order).
// The per-symbol records are independent of the state chain, so they are fetched kPf ahead in
// register blocks: the chain then runs at ALU latency instead of one memory latency per symbol.
constexpr int kPf = 8;

__global__ void k_rans_encode(const EncSym* __restrict__ prep, const uint32_t* __restrict__ raw_in,
                              const int64_t* __restrict__ sym_off, int nstreams, uint32_t* __restrict__ words,
                              const int64_t* __restrict__ word_off, int32_t* __restrict__ nwords) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  uint32_t* const lo = words + word_off[s];
  uint32_t* const hi = words + word_off[s + 1];
  uint32_t* ptr = hi;
  uint64_t x = kRansL;
  bool ok = true;
  const int64_t b = sym_off[s];
  EncSym cur[kPf], nxt[kPf];
  int64_t i = sym_off[s + 1] - 1;  // symbol index of cur[0]; cur[k] = prep[i - k]
#pragma unroll
  for (int k = 0; k < kPf; ++k)
    if (i - k >= b) cur[k] = prep[i - k];
  for (; ok && i >= b; i -= kPf) {
#pragma unroll
    for (int k = 0; k < kPf; ++k)
      if (i - kPf - k >= b) nxt[k] = prep[i - kPf - k];
#pragma unroll
    for (int k = 0; k < kPf; ++k) {
      const int64_t ik = i - k;
      if (!ok || ik < b) break;
      const EncSym p = cur[k];
      const uint32_t start = p.sf & 0xFFFFu, freq = p.sf >> 16;
      if (p.shift & 0x100u) {  // escape bin: bypass-coded payload
        const uint32_t raw = raw_in[ik];
        int32_t nb = 0;
        while (nb < 8 && (raw >> (nb * kBypassPrec)) != 0) ++nb;
        for (int32_t j = nb - 1; ok && j >= 0; --j)
          ok = enc_put_bits(x, ptr, lo, (raw >> (j * kBypassPrec)) & kMaxBypass);
        const int32_t q = nb / kMaxBypass, r = nb - q * kMaxBypass;
        if (ok) ok = enc_put_bits(x, ptr, lo, (uint32_t)r);
        for (int32_t kk = 0; ok && kk < q; ++kk) ok = enc_put_bits(x, ptr, lo, kMaxBypass);
        if (!ok) break;
      }
      const uint64_t x_max = ((kRansL >> kPrec) << 32) * freq;
      if (x >= x_max) {
        if (ptr <= lo) {
          ok = false;
          break;
        }
        *--ptr = (uint32_t)x;
        x >>= 32;
      }
      // Rans64EncPutSymbol: x = x + bias + q * (2^prec - freq), q = mulhi(x, rcp) >> shift
      const uint64_t q = mulhi64(x, p.rcp) >> (p.shift & 0xFFu);
      const uint64_t bias = freq < 2 ? (uint64_t)start + (1u << kPrec) - 1 : (uint64_t)start;
      x = x + bias + q * (uint64_t)((1u << kPrec) - freq);
    }
#pragma unroll
    for (int k = 0; k < kPf; ++k) cur[k] = nxt[k];
  }
  if (ok && ptr - lo >= 2) {
    ptr -= 2;
    ptr[0] = (uint32_t)x;
    ptr[1] = (uint32_t)(x >> 32);
    nwords[s] = (int32_t)(hi - ptr);
  } else {
    nwords[s] = -1;
  }
}

__global__ void k_pack_scan(const int32_t* __restrict__ nwords, int n, int64_t* __restrict__ pack_off,
                            int32_t* __restrict__ status) {
  // single block, fixed-order exclusive scan; a stream whose encode ran out of space (nwords < 0)
  // packs as empty and sets status = FVC_ENOSPC
  __shared__ int64_t part[kBlk];
  __shared__ int bad[kBlk];
  const int per = (n + kBlk - 1) / kBlk;
  const int b0 = threadIdx.x * per;
  int64_t s = 0;
  int nbad = 0;
  for (int i = b0; i < b0 + per && i < n; ++i) {
    s += nwords[i] > 0 ? nwords[i] : 0;
    nbad += nwords[i] < 0 ? 1 : 0;
  }
  part[threadIdx.x] = s;
  bad[threadIdx.x] = nbad;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    int any = 0;
    for (int t = 0; t < kBlk; ++t) {
      const int64_t v = part[t];
      part[t] = run;
      run += v;
      any |= bad[t];
    }
    pack_off[n] = run;
    if (status) status[0] = any ? FVC_ENOSPC : 0;
  }
  __syncthreads();
  int64_t run = part[threadIdx.x];
  for (int i = b0; i < b0 + per && i < n; ++i) {
    pack_off[i] = run;
    run += nwords[i] > 0 ? nwords[i] : 0;
  }
}

__global__ void k_pack_copy(const uint32_t* __restrict__ words, const int64_t* __restrict__ word_off,
                            const int32_t* __restrict__ nwords, const int64_t* __restrict__ pack_off,
                            uint32_t* __restrict__ out) {
  const int s = blockIdx.x;
  const int32_t n = nwords[s];
  if (n <= 0) return;
  const uint32_t* src = words + word_off[s + 1] - n;
  uint32_t* dst = out + pack_off[s];
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}


// Decode tables: a compact image per table, copied into the decoder's LDS table cache
// (k_rans_decode) or read from L2 when it does not fit. Table t occupies
// img_off[t] .. img_off[t+1] words = kL2N bucket entries of 2 words, then n_t = cdf_sizes[t] - 1
// start|freq<<16 words (padded to an even count). Bucket u covers cum in [u << kL2Shift, (u+1) << kL2Shift): its entry is
// {lo | hi << 16, start|freq<<16 of lo} with lo / hi the symbols holding the bucket's first / last
// cum; lo == hi (most of the cum space) decodes from the entry alone.
constexpr int kL2Shift = 9;
constexpr int kL2N = 1 << (kPrec - kL2Shift);
constexpr int kL2Words = 2 * kL2N;

__global__ void k_build_img_off(const int32_t* __restrict__ cdf_sizes, int ntables, uint32_t* __restrict__ img_off) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t o = 0;
  for (int t = 0; t < ntables; ++t) {
    img_off[t] = o;
    o += kL2Words + (uint32_t)((cdf_sizes[t] - 1 + 1) & ~1);  // even: 8-B aligned bucket entries
  }
  img_off[ntables] = o;
}

__global__ void k_build_img(const int32_t* __restrict__ cdfs, int cdf_stride, const int32_t* __restrict__ cdf_sizes,
                            int ntables, const uint32_t* __restrict__ img_off, uint32_t* __restrict__ img) {
  const int t = blockIdx.y;
  const int n = cdf_sizes[t] - 1;
  const int32_t* cdf = cdfs + (size_t)t * cdf_stride;
  auto sft = [&](int s) { return (uint32_t)cdf[s] | ((uint32_t)(cdf[s + 1] - cdf[s]) << 16); };
  uint32_t* out = img + img_off[t];
  auto holder = [&](uint32_t cum) {  // last symbol with cdf[s] <= cum
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if ((uint32_t)cdf[mid] <= cum) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < kL2N + n; e += gridDim.x * blockDim.x) {
    if (e < kL2N) {
      const int lo = holder((uint32_t)e << kL2Shift);
      const int hi = holder((((uint32_t)e + 1) << kL2Shift) - 1);
      out[2 * e] = (uint32_t)lo | ((uint32_t)hi << 16);
      out[2 * e + 1] = sft(lo);
    } else {
      out[kL2Words + e - kL2N] = sft(e - kL2N);
    }
  }
}

// One block per 64 streams, two waves (r2). Wave 0 (the decoder) runs the state chains, one lane per stream; wave 1
// (the loader) keeps the decoder's inputs in LDS one phase (kJ symbols) ahead -- per symbol a
// record {table index, offset, LDS address of the table's image or ~0} and a ring of the
// stream's next kR bitstream words -- and writes the previous phase's decoded symbols out. The
// decoder reads only LDS for a symbol of a cached table: its chain is one bucket-entry read
// (plus a binary search in the rare buckets that span several symbols), the rANS arithmetic
// and, on renormalisation, one ring read -- no L2 latency, no in-order vmcnt wait behind an HBM
// index fetch or a store (r1's one-wave kernel had both: 4.5 -> 3.7-4.2 ms for 1,152 streams of
// 8,160 low-rate symbols, scripts/coder_micro.py).
//
// Table cache: the block copies the contiguous run of table images [t_lo, t_hi) into LDS (t_lo
// = the smallest table index among its streams' first kJ symbols; as many tables as fit in
// kTabWords). Channel framing puts one table per stream (mv, z: a block's 64 channels) or the
// Laplace scale table, smallest scales first (feature), in the cache; a symbol of another table
// reads the same image from L2 (its global offset travels in the record).
//
// The loader hides its own latencies: table indexes are fetched two phases ahead (registers),
// offsets of cached tables come from LDS, and the ring is refilled kRB words at a time.
//
// Ring protocol: the decoder publishes its word position pos(B_p) at barrier B_p and the loader
// its fill mark (double-buffered by phase parity); during phase p the loader may write words [fill, fill + kRB) into slots w % kR
// if fill + kRB <= pos(B_p) + kR (those slots held consumed words). During phase p the decoder
// reads ring words below the fill mark published at B_p; a word past it is read from global.
constexpr int kJ = 16;                // symbols per phase
constexpr int kR = 64;                // ring words per stream
constexpr int kRB = 32;               // ring refill batch
constexpr int kTabDir = 256;          // cached tables at most
constexpr int kTabWords = 25600;      // 100 KB of table images
constexpr size_t kDec2Lds =
    (size_t)(2 * kJ * 64 * 4 + 2 * kJ * 64 + kR * 64 + 3 * 64 + 4 + 2 * kTabDir + kTabWords) * 4;
static_assert(kDec2Lds <= 160 * 1024, "k_rans_decode's LDS image must fit gfx950's 160 KB per CU");
constexpr uint32_t kGlobTab = 0x80000000u;  // record flag: table image read from global memory
constexpr int kDecSpb = 64;                 // streams per decode block when the caller passes 0
constexpr int kRsrcFlags = 0x00020000;  // buffer descriptor dword 3 (raw 32-bit, as fvc_conv_x3.hip)

// Global reads that sit next to LDS reads of the same value go through buffer descriptors: a
// plain pointer would let the compiler merge the two into one generic (flat) load, which waits on
// both counters and serialises the chain.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dec_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, kRsrcFlags);
}
__device__ __forceinline__ uint32_t bload(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0);
}

__global__ __launch_bounds__(128) void k_rans_decode(
    const uint32_t* __restrict__ packed, const int64_t* __restrict__ pack_off, const int32_t* __restrict__ indexes,
    const int64_t* __restrict__ sym_off, int nstreams, const int32_t* __restrict__ cdf_sizes,
    const int32_t* __restrict__ offsets, int ntables, const uint32_t* __restrict__ img_off, const uint32_t* __restrict__ img,
    int32_t* __restrict__ symbols, int32_t* __restrict__ status, int spb) {
  extern __shared__ int32_t lds[];
  uint4* const s_rec = reinterpret_cast<uint4*>(lds);          // [2][kJ][64] {ci, off, tab, -}
  int32_t* const s_out = lds + 2 * kJ * 64 * 4;                // [2][kJ][64] decoded symbols
  uint32_t* const s_ring = (uint32_t*)(s_out + 2 * kJ * 64);   // [kR][64]
  int32_t* const s_pos = (int32_t*)(s_ring + kR * 64);         // [64] published word positions
  int32_t* const s_fill = s_pos + 64;                          // [2][64] ring fill marks by phase parity
  int32_t* const s_trange = s_fill + 2 * 64;                   // t_lo, t_hi
  uint32_t* const s_dir = (uint32_t*)(s_trange + 4);           // [kTabDir] LDS word offset of cached table
  int32_t* const s_doff = (int32_t*)(s_dir + kTabDir);         // [kTabDir] its offset
  uint32_t* const s_tab = (uint32_t*)(s_doff + kTabDir);       // [kTabWords] table images
  const int lane = threadIdx.x & 63;
  const bool loader = threadIdx.x >= 64;
  // spb streams per block (lanes >= spb idle): with fewer streams a block's table cache holds the
  // tables of all of them, so no lane of the decoder wave waits on L2 per symbol
  const int s = blockIdx.x * spb + lane;
  const bool live = lane < spb && s < nstreams;
  const int64_t w0 = live ? pack_off[s] : 0;
  const int nw = live ? (int)(pack_off[s + 1] - w0) : 0;
  const int64_t b = live ? sym_off[s] : 0;
  const int len = live ? (int)(sym_off[s + 1] - b) : 0;
  int maxlen = len;
  for (int o = 32; o > 0; o >>= 1) maxlen = max(maxlen, __shfl_xor(maxlen, o, 64));
  const int nph = (maxlen + kJ - 1) / kJ;
  const __amdgpu_buffer_rsrc_t r_packed = dec_rsrc(packed), r_offsets = dec_rsrc(offsets);
  const __amdgpu_buffer_rsrc_t r_img = dec_rsrc(img), r_imgoff = dec_rsrc(img_off);

  // ---- loader helpers
  int32_t ci[kJ], cn[kJ];  // table indexes of the next phase and the one after
  auto load_ci = [&](int32_t (&dst)[kJ], int base) {
#pragma unroll
    for (int j = 0; j < kJ; ++j) dst[j] = base + j < len ? indexes[b + base + j] : 0;
  };
  auto put_recs = [&](int buf, int t_lo, int t_hi) {
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const int c = ci[j];
      const bool cached = (unsigned)(c - t_lo) < (unsigned)(t_hi - t_lo);
      const int di = cached ? c - t_lo : 0;  // separate LDS and global loads (no generic pointer)
      uint32_t tab = s_dir[di];
      int32_t off = s_doff[di];
      if (!cached) {  // the table's image in global memory (L2-resident)
        tab = kGlobTab | bload(r_imgoff, (uint32_t)c * 4u);
        off = (int32_t)bload(r_offsets, (uint32_t)c * 4u);
      }
      s_rec[(buf * kJ + j) * 64 + lane] = make_uint4((uint32_t)c, (uint32_t)off, tab, 0u);
    }
  };
  auto flush = [&](int buf, int base) {
    int32_t v[kJ];
#pragma unroll
    for (int j = 0; j < kJ; ++j) v[j] = s_out[(buf * kJ + j) * 64 + lane];
#pragma unroll
    for (int j = 0; j < kJ; ++j)
      if (base + j < len) symbols[b + base + j] = v[j];
  };
  int fill_end = 0;
  auto refill = [&](int pub) {  // one batch of kRB words if their slots are free
    if (fill_end >= nw || fill_end + kRB > pub + kR) return;
    uint32_t v[kRB];
#pragma unroll
    for (int k = 0; k < kRB; ++k) v[k] = fill_end + k < nw ? packed[w0 + fill_end + k] : 0u;
#pragma unroll
    for (int k = 0; k < kRB; ++k) s_ring[((unsigned)(fill_end + k) & (kR - 1)) * 64 + lane] = v[k];
    fill_end = min(fill_end + kRB, nw);
  };

  // ---- prologue: cache range, table images, phase-0 records, first ring words
  if (loader) {
    load_ci(ci, 0);
    int tmin = ntables;
#pragma unroll
    for (int j = 0; j < kJ; ++j)
      if (j < len) tmin = min(tmin, ci[j]);
    for (int o = 32; o > 0; o >>= 1) tmin = min(tmin, __shfl_xor(tmin, o, 64));
    int nfit = 0;  // tables tmin .. tmin + nfit - 1 fit (the test is monotone in t)
    if (tmin < ntables) {
      const uint32_t base = img_off[tmin];
      for (int k0 = 0; k0 < kTabDir; k0 += 64) {
        const int t = tmin + k0 + lane;
        nfit += __popcll(__ballot(t < ntables && img_off[t + 1] - base <= (uint32_t)kTabWords));
      }
    }
    if (lane == 0) {
      s_trange[0] = tmin;
      s_trange[1] = tmin + nfit;
    }
  } else {
    s_pos[lane] = 0;
  }
  __syncthreads();
  const int t_lo = s_trange[0], t_hi = s_trange[1];
  if (t_hi > t_lo) {
    const uint32_t base = img_off[t_lo];
    const uint32_t nwd = img_off[t_hi] - base;
    for (uint32_t i = threadIdx.x; i < nwd; i += 128) s_tab[i] = img[base + i];
    for (int t = threadIdx.x; t < t_hi - t_lo; t += 128) {
      s_dir[t] = (uint32_t)(s_tab - (uint32_t*)lds) + img_off[t_lo + t] - base;
      s_doff[t] = offsets[t_lo + t];
    }
  }
  __syncthreads();
  if (loader) {
    put_recs(0, t_lo, t_hi);
    if (nph > 1) load_ci(cn, kJ);
    refill(0);
    refill(0);
    s_fill[lane] = fill_end;  // parity 0: read after B_0
  }
  __syncthreads();  // B_0

  if (loader) {
    for (int p = 0; p < nph; ++p) {
      const int pub = s_pos[lane];  // pos(B_p)
      if (p + 1 < nph) {
#pragma unroll
        for (int j = 0; j < kJ; ++j) ci[j] = cn[j];
        if (p + 2 < nph) load_ci(cn, (p + 2) * kJ);
        put_recs((p + 1) & 1, t_lo, t_hi);
      }
      if (p >= 1) flush((p - 1) & 1, (p - 1) * kJ);
      refill(pub);
      s_fill[((p + 1) & 1) * 64 + lane] = fill_end;  // read by the decoder right after B_{p+1}
      __syncthreads();  // B_{p+1}
    }
    if (nph > 0) flush((nph - 1) & 1, (nph - 1) * kJ);
    return;
  }

  // ---- decoder. Each phase's kJ records are read into registers at its start (one LDS wait per
  // phase); the symbol loop is unrolled so every later LDS read on the chain is an explicit
  // ds_read (ring reads and global fallbacks are separate loads, never one generic pointer).
  const uint32_t* const L = (const uint32_t*)lds;
  int valid_end = s_fill[lane];  // ring words readable in this phase
  auto word = [&](int w) -> uint32_t {
    uint32_t v = s_ring[((unsigned)w & (kR - 1)) * 64 + lane];
    if (w >= valid_end) v = bload(r_packed, (uint32_t)(w0 + w) * 4u);
    return v;
  };
  bool ok = live && nw >= 2;
  uint64_t x = 0;
  int pos = 0;
  if (ok) {
    x = (uint64_t)word(0) | ((uint64_t)word(1) << 32);
    pos = 2;
  }
  uint32_t wnext = pos < nw ? word(pos) : 0u;
  auto renorm = [&]() {
    if (x < kRansL) {
      if (pos >= nw) return false;
      x = (x << 32) | wnext;
      ++pos;
      wnext = pos < nw ? word(pos) : 0u;
    }
    return true;
  };
  const uint32_t mask = (1u << kPrec) - 1;
  for (int p = 0; p < nph; ++p) {
    const int buf = p & 1;
    uint4 rec[kJ];
#pragma unroll
    for (int j = 0; j < kJ; ++j) rec[j] = s_rec[(buf * kJ + j) * 64 + lane];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const uint4 cur = rec[j];
      int32_t value = 0;
      if (p * kJ + j < len && ok) {
        const int32_t c = (int32_t)cur.x;
        const uint32_t cum = (uint32_t)x & mask;
        const bool glob = (cur.z & kGlobTab) != 0u;
        const uint32_t tb = cur.z & ~kGlobTab;
        auto tword = [&](uint32_t i) -> uint32_t {  // word i of the table image
          uint32_t v = L[glob ? 0u : tb + i];
          if (glob) v = bload(r_img, (tb + i) * 4u);
          return v;
        };
        uint2 ent;
        if (!glob) {
          ent = *reinterpret_cast<const uint2*>(L + tb + 2 * (cum >> kL2Shift));
        } else {
          ent.x = bload(r_img, (tb + 2 * (cum >> kL2Shift)) * 4u);
          ent.y = bload(r_img, (tb + 2 * (cum >> kL2Shift) + 1) * 4u);
        }
        int32_t sidx = (int32_t)(ent.x & 0xFFFFu);
        uint32_t sf = ent.y;
        int hi = (int32_t)(ent.x >> 16);
        if (hi != sidx) {  // bucket spans symbols sidx .. hi
          while (sidx < hi) {
            const int mid = (sidx + hi + 1) >> 1;
            if ((tword(kL2Words + mid) & 0xFFFFu) <= cum) sidx = mid; else hi = mid - 1;
          }
          sf = tword(kL2Words + sidx);
        }
        const uint32_t start = sf & 0xFFFFu, freq = sf >> 16;
        x = (uint64_t)freq * (x >> kPrec) + (cum - start);
        ok = renorm();
        value = sidx;
        if (ok && start + freq == (1u << kPrec)) {  // escape bin (== max_value)
          auto getbits = [&](int32_t& v) {
            v = (int32_t)(x & kMaxBypass);
            x >>= kBypassPrec;
            return renorm();
          };
          int32_t v = 0;
          ok = getbits(v);
          int32_t nb = v;
          while (ok && v == kMaxBypass && nb < 64) {
            ok = getbits(v);
            nb += v;
          }
          if (nb > 8) ok = false;
          uint32_t raw = 0;
          for (int32_t t = 0; ok && t < nb; ++t) {
            ok = getbits(v);
            raw |= (uint32_t)v << (t * kBypassPrec);
          }
          const int32_t max_value = cdf_sizes[c] - 2;
          value = (int32_t)(raw >> 1);
          if (raw & 1) value = -value - 1;
          else value += max_value;
        }
        value += (int32_t)cur.y;
      }
      s_out[(buf * kJ + j) * 64 + lane] = value;
    }
    s_pos[lane] = pos;  // pos(B_{p+1})
    __syncthreads();    // B_{p+1}
    valid_end = s_fill[((p + 1) & 1) * 64 + lane];  // wnext stays valid: unconsumed words stay put
  }
  if (live) status[s] = ok ? 0 : FVC_ECORRUPT;
}

static int grid_for(size_t n) {
  size_t g = (n + kBlk - 1) / kBlk;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int fvc_latent_to_symbols(const float* lat, int32_t* sym, int batch, int h, int w, int c, int cp, fvc_stream_t s) {
  if (!lat || !sym || c > cp) return FVC_EINVAL;
  const size_t n = (size_t)batch * c * h * w;
  hipLaunchKernelGGL(k_latent_to_symbols, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, lat, sym, batch, h * w,
                     c, cp);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_symbols_to_latent(const int32_t* sym, float* lat, int batch, int h, int w, int c, int cp, fvc_stream_t s) {
  if (!lat || !sym || c > cp) return FVC_EINVAL;
  const size_t n = (size_t)batch * cp * h * w;
  hipLaunchKernelGGL(k_symbols_to_latent, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, sym, lat, batch, h * w,
                     c, cp);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_build_indexes(const float* sigma, const float* table, int nt, int32_t* idx, int batch, int h, int w, int c,
                      int cp, fvc_stream_t s) {
  if (!sigma || !table || !idx || nt < 1 || c > cp) return FVC_EINVAL;
  const size_t n = (size_t)batch * c * h * w;
  hipLaunchKernelGGL(k_build_indexes, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, sigma, table, nt, idx, batch,
                     h * w, c, cp);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_channel_indexes(int32_t* idx, int batch, int hw, int c, fvc_stream_t s) {
  if (!idx) return FVC_EINVAL;
  const size_t n = (size_t)batch * c * hw;
  hipLaunchKernelGGL(k_channel_indexes, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, idx, batch, hw, c);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_quantize_symbols(const float* x, const float* means, int32_t* sym, size_t n, fvc_stream_t s) {
  if ((!x || !sym) && n) return FVC_EINVAL;
  if (!n) return 0;
  hipLaunchKernelGGL(k_quantize_symbols, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, x, means, sym, n);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_dequantize_symbols(const int32_t* sym, const float* means, float* out, size_t n, fvc_stream_t s) {
  if ((!sym || !out) && n) return FVC_EINVAL;
  if (!n) return 0;
  hipLaunchKernelGGL(k_dequantize_symbols, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, sym, means, out, n);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_build_indexes_flat(const float* scales, const float* table, int nt, int32_t* idx, size_t n,
                           fvc_stream_t s) {
  if ((!scales || !idx) && n) return FVC_EINVAL;
  if (!table || nt < 1) return FVC_EINVAL;
  if (!n) return 0;
  hipLaunchKernelGGL(k_build_indexes_flat, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, scales, table, nt,
                     idx, n);
  FVC_CHECK_LAUNCH();
  return 0;
}

size_t fvc_rans_encode_ws_bytes(int64_t nsymbols) { return (size_t)nsymbols * (sizeof(EncSym) + 4); }

int fvc_rans_encode(const int32_t* symbols, const int32_t* indexes, const int64_t* sym_off, int nstreams,
                    int64_t nsymbols, const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes,
                    const int32_t* offsets, void* ws, uint32_t* words, const int64_t* word_off, int32_t* nwords,
                    fvc_stream_t s) {
  if (!symbols || !indexes || !sym_off || !cdfs || !cdf_sizes || !offsets || !ws || !words || !word_off ||
      !nwords || nstreams <= 0 || nsymbols < 0)
    return FVC_EINVAL;
  EncSym* prep = (EncSym*)ws;
  uint32_t* raw = (uint32_t*)(prep + nsymbols);
  if (nsymbols > 0) {
    hipLaunchKernelGGL(k_rans_prep, dim3(grid_for((size_t)nsymbols)), dim3(kBlk), 0, (hipStream_t)s, symbols, indexes,
                       nsymbols, cdfs, cdf_stride, cdf_sizes, offsets, prep, raw);
    FVC_CHECK_LAUNCH();
  }
  const int blk = 64;
  hipLaunchKernelGGL(k_rans_encode, dim3((nstreams + blk - 1) / blk), dim3(blk), 0, (hipStream_t)s, prep, raw,
                     sym_off, nstreams, words, word_off, nwords);
  FVC_CHECK_LAUNCH();
  return 0;
}

size_t fvc_rans_lut_bytes(int ntables, int cdf_stride) {
  if (ntables <= 0 || cdf_stride <= 1) return 0;
  return ((size_t)ntables + 1) * 4 + (size_t)ntables * ((size_t)cdf_stride + 1 + kL2Words) * 4;
}

// layout of the decode-table buffer: img_off [ntables + 1] u32 | img (compact images, k_build_img)
int fvc_rans_build_lut(const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes, int ntables, void* lut,
                       fvc_stream_t s) {
  if (!cdfs || !cdf_sizes || !lut || ntables <= 0 || cdf_stride <= 1) return FVC_EINVAL;
  uint32_t* img_off = (uint32_t*)lut;
  hipLaunchKernelGGL(k_build_img_off, dim3(1), dim3(64), 0, (hipStream_t)s, cdf_sizes, ntables, img_off);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_build_img, dim3(fvc_cdiv(cdf_stride + kL2N, kBlk), ntables), dim3(kBlk), 0,
                     (hipStream_t)s, cdfs, cdf_stride, cdf_sizes, ntables, img_off, img_off + ntables + 1);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_rans_pack(const uint32_t* words, const int64_t* word_off, const int32_t* nwords, int nstreams,
                  int64_t* pack_off, uint32_t* out, int32_t* status, fvc_stream_t s) {
  if (!words || !word_off || !nwords || !pack_off || !out || nstreams <= 0) return FVC_EINVAL;
  hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(kBlk), 0, (hipStream_t)s, nwords, nstreams, pack_off, status);
  FVC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_pack_copy, dim3(nstreams), dim3(kBlk), 0, (hipStream_t)s, words, word_off, nwords, pack_off,
                     out);
  FVC_CHECK_LAUNCH();
  return 0;
}

int fvc_rans_decode(const uint32_t* packed, const int64_t* pack_off, const int32_t* indexes, const int64_t* sym_off,
                    int nstreams, int ntables, int cdf_stride, const int32_t* cdf_sizes, const int32_t* offsets,
                    const void* lut, int32_t* symbols, int32_t* status, int streams_per_block, fvc_stream_t s) {
  if (!packed || !pack_off || !indexes || !sym_off || !cdf_sizes || !offsets || !lut || !symbols || !status ||
      nstreams <= 0 || ntables <= 0 || cdf_stride <= 1)
    return FVC_EINVAL;
  const uint32_t* img_off = (const uint32_t*)lut;
  if (streams_per_block < 0 || streams_per_block > 64) return FVC_EINVAL;
  // kDec2Lds (static_assert'ed against gfx950's 160 KB per CU above) needs the opt-in: a device
  // that refuses it cannot run this kernel, so report that instead of a generic launch failure
  const hipError_t attr =
      hipFuncSetAttribute((const void*)k_rans_decode, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDec2Lds);
  if (attr != hipSuccess) return -(int)attr;
  const int spb = streams_per_block ? streams_per_block : kDecSpb;
  hipLaunchKernelGGL(k_rans_decode, dim3((nstreams + spb - 1) / spb), dim3(128), kDec2Lds, (hipStream_t)s, packed,
                     pack_off, indexes, sym_off, nstreams, cdf_sizes, offsets, ntables, img_off, img_off + ntables + 1,
                     symbols, status, spb);
  FVC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------ host: CDF quantisation
// compressai cpp_exts/ops/ops.cpp pmf_to_quantized_cdf (called by EntropyModel._pmf_to_cdf).
// Table build happens once per weight load (EntropyBottleneck/GaussianConditional.update),
// on the host in the reference too.
#include <cmath>
#include <vector>

extern "C" int fvc_pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf_out) {
  if (!pmf || !cdf_out || n <= 0 || precision <= 0 || precision > 16) return FVC_EINVAL;
  for (int i = 0; i < n; ++i)
    if (pmf[i] < 0 || !std::isfinite(pmf[i])) return FVC_EINVAL;
  std::vector<uint32_t> cdf(n + 1);
  cdf[0] = 0;
  for (int i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)std::round(pmf[i] * (float)(1 << precision));
  int acc = 0;  // std::accumulate(..., 0) accumulates in int
  for (int i = 0; i <= n; ++i) acc += (int)cdf[i];
  const uint32_t total = (uint32_t)acc;
  if (total == 0) return FVC_EINVAL;
  for (int i = 0; i <= n; ++i) cdf[i] = (uint32_t)(((uint64_t)(1 << precision) * cdf[i]) / total);
  for (int i = 1; i <= n; ++i) cdf[i] += cdf[i - 1];
  cdf[n] = 1u << precision;
  for (int i = 0; i < n; ++i) {
    if (cdf[i] == cdf[i + 1]) {
      uint32_t best_freq = ~0u;
      int best_steal = -1;
      for (int j = 0; j < n; ++j) {
        const uint32_t freq = cdf[j + 1] - cdf[j];
        if (freq > 1 && freq < best_freq) {
          best_freq = freq;
          best_steal = j;
        }
      }
      if (best_steal < 0) return FVC_EINVAL;
      if (best_steal < i) {
        for (int j = best_steal + 1; j <= i; ++j) cdf[j]--;
      } else {
        for (int j = i + 1; j <= best_steal; ++j) cdf[j]++;
      }
    }
  }
  for (int i = 0; i < n; ++i)
    if (cdf[i + 1] <= cdf[i]) return FVC_EINVAL;
  for (int i = 0; i <= n; ++i) cdf_out[i] = cdf[i];
  return 0;
}
