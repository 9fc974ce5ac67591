// Entropy-coding kernels: latent <-> symbol streams, scale-table indexes, and a batched
// device rANS coder that is byte-compatible, stream for stream, with compressai's
// RansEncoder/RansDecoder.{encode,decode}_with_indexes (ryg_rans 64-bit state, 32-bit words,
// precision 16, 4-bit bypass for escapes), the C++ coder the reference reaches through
// entropy_models.py:80-94 (RecProbModel.compress/decompress).
//
// Parallelism: one lane per independent stream (a stream = one channel of one latent of one
// frame); a stream's symbol loop is inherently sequential (rANS state chain).
#include "fvc_common.h"

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


// Decode tables, small enough to stay L2-resident: per table t
//   lut[t][u]  (u = cum >> kLutShift, 4096 buckets): the symbol s with cdf[s] <= u << kLutShift
//              < cdf[s+1], i.e. the first candidate for any cum in that bucket;
//   sf[t][s]   = cdf[s] | (cdf[s+1] - cdf[s]) << 16.
// A decoded symbol costs two dependent L2 hits (bucket, then its start/freq) plus a short
// forward step when the bucket straddles a symbol boundary; the old 2^16-entry LUT was one
// random access into 256 KB per table, missing in L2 almost every time.
constexpr int kLutShift = 4;
constexpr int kLutN = 1 << (kPrec - kLutShift);

__global__ void k_build_lut(const int32_t* __restrict__ cdfs, int cdf_stride, const int32_t* __restrict__ cdf_sizes,
                            int ntables, uint16_t* __restrict__ lut, uint32_t* __restrict__ sf) {
  const int64_t nl = (int64_t)ntables * kLutN;
  const int64_t ns = (int64_t)ntables * cdf_stride;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nl + ns; e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nl) {
      const int t = (int)(e / kLutN);
      const uint32_t cum = (uint32_t)(e % kLutN) << kLutShift;
      const int32_t* cdf = cdfs + (size_t)t * cdf_stride;
      int lo = 0, hi = cdf_sizes[t] - 1;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if ((uint32_t)cdf[mid] <= cum) lo = mid; else hi = mid;
      }
      lut[e] = (uint16_t)lo;
    } else {
      const int64_t f = e - nl;
      const int t = (int)(f / cdf_stride);
      const int sidx = (int)(f % cdf_stride);
      const int32_t* cdf = cdfs + (size_t)t * cdf_stride;
      sf[f] = sidx < cdf_sizes[t] - 1 ? ((uint32_t)cdf[sidx] | ((uint32_t)(cdf[sidx + 1] - cdf[sidx]) << 16)) : 0u;
    }
  }
}

// One lane per stream (64-lane blocks). The next bitstream word and the next kPf table indexes
// are held in registers ahead of need, so the only memory accesses on the state chain are the
// two table hits. Decoded symbols go to an LDS ring (kRing per lane) and are written to global
// memory in bursts: a global store outstanding in vmcnt would make every later load wait for it
// (the compiler cannot order a load behind a store), i.e. one store latency per symbol.
constexpr int kRing = 64;

__global__ __launch_bounds__(64) void k_rans_decode(
    const uint32_t* __restrict__ packed, const int64_t* __restrict__ pack_off, const int32_t* __restrict__ indexes,
    const int64_t* __restrict__ sym_off, int nstreams, int cdf_stride, const int32_t* __restrict__ cdf_sizes,
    const int32_t* __restrict__ offsets, const uint16_t* __restrict__ lut, const uint32_t* __restrict__ sft,
    int32_t* __restrict__ symbols, int32_t* __restrict__ status) {
  __shared__ int32_t ring[kRing * 64];
  const int lane = threadIdx.x;
  const int s = blockIdx.x * 64 + lane;
  const bool live = s < nstreams;
  const uint32_t* ptr = packed + (live ? pack_off[s] : 0);
  const uint32_t* end = packed + (live ? pack_off[s + 1] : 0);
  bool ok = live && end - ptr >= 2;
  uint64_t x = 0;
  if (ok) {
    x = (uint64_t)ptr[0] | ((uint64_t)ptr[1] << 32);
    ptr += 2;
  }
  uint32_t wnext = ptr < end ? *ptr : 0u;  // next renormalisation word, loaded ahead
  auto renorm = [&]() {
    if (x < kRansL) {
      if (ptr >= end) return false;
      x = (x << 32) | wnext;
      ++ptr;
      wnext = ptr < end ? *ptr : 0u;
    }
    return true;
  };
  const uint64_t mask = (1ull << kPrec) - 1;
  const int64_t b = live ? sym_off[s] : 0;
  const int64_t e = live ? sym_off[s + 1] : 0;
  // all lanes walk the same number of steps (the wave's longest stream); shorter ones idle
  int64_t len = e - b, maxlen = len;
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t v = __shfl_xor(maxlen, o, 64);
    maxlen = v > maxlen ? v : maxlen;
  }
  int32_t cur[kPf], nxt[kPf], off[kPf];
#pragma unroll
  for (int k = 0; k < kPf; ++k) cur[k] = k < len ? indexes[b + k] : 0;
#pragma unroll
  for (int k = 0; k < kPf; ++k) off[k] = offsets[cur[k]];
  auto flush = [&](int64_t base, int n) {  // symbols [base, base+n) of this lane from the ring
    for (int j = 0; j < n; ++j)
      if (base + j < len) symbols[b + base + j] = ring[j * 64 + lane];
  };
  for (int64_t i = 0; i < maxlen; i += kPf) {
#pragma unroll
    for (int k = 0; k < kPf; ++k) nxt[k] = i + kPf + k < len ? indexes[b + i + kPf + k] : 0;
#pragma unroll
    for (int k = 0; k < kPf; ++k) {
      const int64_t ik = i + k;
      const int32_t ci = cur[k];
      int32_t value = 0;
      if (ik < len && ok) {
        const uint32_t cum = (uint32_t)(x & mask);
        const uint32_t* sfc = sft + (size_t)ci * cdf_stride;
        int32_t sidx = lut[(size_t)ci * kLutN + (cum >> kLutShift)];
        uint32_t sf = sfc[sidx];
        while (cum >= (sf & 0xFFFFu) + (sf >> 16)) sf = sfc[++sidx];
        const uint32_t start = sf & 0xFFFFu, freq = sf >> 16;
        x = freq * (x >> kPrec) + cum - start;
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
          for (int32_t j = 0; ok && j < nb; ++j) {
            ok = getbits(v);
            raw |= (uint32_t)v << (j * kBypassPrec);
          }
          const int32_t max_value = cdf_sizes[ci] - 2;
          value = (int32_t)(raw >> 1);
          if (raw & 1) value = -value - 1;
          else value += max_value;
        }
        value += off[k];
      }
      ring[(int)(ik % kRing) * 64 + lane] = value;
    }
    if ((i + kPf) % kRing == 0) flush(i + kPf - kRing, kRing);
#pragma unroll
    for (int k = 0; k < kPf; ++k) cur[k] = nxt[k];
#pragma unroll
    for (int k = 0; k < kPf; ++k) off[k] = offsets[cur[k]];
  }
  const int64_t done = (maxlen + kPf - 1) / kPf * kPf;  // steps written to the ring
  if (done % kRing) flush(done - done % kRing, (int)(done % kRing));
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
  return (size_t)ntables * ((size_t)cdf_stride * 4 + (size_t)kLutN * 2);
}

int fvc_rans_build_lut(const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes, int ntables, void* lut,
                       fvc_stream_t s) {
  if (!cdfs || !cdf_sizes || !lut || ntables <= 0 || cdf_stride <= 1) return FVC_EINVAL;
  uint32_t* sf = (uint32_t*)lut;
  uint16_t* lut16 = (uint16_t*)(sf + (size_t)ntables * cdf_stride);
  const size_t n = (size_t)ntables * (kLutN + cdf_stride);
  hipLaunchKernelGGL(k_build_lut, dim3(grid_for(n)), dim3(kBlk), 0, (hipStream_t)s, cdfs, cdf_stride, cdf_sizes,
                     ntables, lut16, sf);
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
                    const void* lut, int32_t* symbols, int32_t* status, fvc_stream_t s) {
  if (!packed || !pack_off || !indexes || !sym_off || !cdf_sizes || !offsets || !lut || !symbols || !status ||
      nstreams <= 0 || ntables <= 0 || cdf_stride <= 1)
    return FVC_EINVAL;
  const uint32_t* sf = (const uint32_t*)lut;
  const uint16_t* lut16 = (const uint16_t*)(sf + (size_t)ntables * cdf_stride);
  const int blk = 64;
  hipLaunchKernelGGL(k_rans_decode, dim3((nstreams + blk - 1) / blk), dim3(blk), 0, (hipStream_t)s, packed, pack_off,
                     indexes, sym_off, nstreams, cdf_stride, cdf_sizes, offsets, lut16, sf, symbols, status);
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
