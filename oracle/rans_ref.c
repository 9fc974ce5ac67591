/*
 * ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline). Never linked
 * into libfvc.
 *
 * Plain-C restatement of the compressai 1.2 entropy-coder C++ extension, which is absent
 * from /root/reference and this image:
 *   - cpp_exts/ops/ops.cpp              pmf_to_quantized_cdf
 *   - cpp_exts/rans/rans_interface.cpp  BufferedRansEncoder::encode_with_indexes + flush,
 *                                       RansDecoder::decode_with_indexes
 *   - third_party/ryg_rans/rans64.h     Rans64Enc and Rans64Dec primitives (+ compressai PutBits/GetBits)
 * Reference call sites: entropy_models.py:80-94 (RecProbModel.compress/decompress).
 * Written the way compressai structures it (forward push into a symbol queue, then a
 * reverse flush) so it independently checks the device kernel's reverse walk.
 *
 * Independence from the product: the product's host quantiser (fvc_coder.hip,
 * fvc_pmf_to_quantized_cdf) follows ops.cpp literally, editing the cumulative table in place.
 * This one works on the per-bin frequency array instead. ops.cpp's repair of an empty bin i
 * ("steal one count from the lowest bin j with freq > 1": cdf[j+1..i] -= 1 if j < i, else
 * cdf[i+1..j] += 1) changes exactly two frequencies, freq[i] += 1 and freq[j] -= 1, so the
 * repair loop below is a different program with the same output by construction; the two are
 * compared table for table in tests/test_coder_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PREC 16
#define BYPASS_PREC 4
#define MAX_BYPASS ((1 << BYPASS_PREC) - 1)
#define RANS64_L (1ull << 31)

/* half away from zero, as std::round on the float product */
static uint32_t round_half_away(float v) {
  const double d = (double)v;
  return (uint32_t)(d >= 0 ? floor(d + 0.5) : -floor(-d + 0.5));
}

int ref_pmf_to_quantized_cdf(const float *pmf, int n, int precision, uint32_t *cdf) {
  if (n <= 0) return -1;
  const uint64_t one = 1ull << precision;
  uint64_t *freq = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
  if (!freq) return -1;
  /* 1. scaled, rounded probabilities (float product, as ops.cpp multiplies floats) */
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (!(pmf[i] >= 0) || !isfinite(pmf[i])) { free(freq); return -1; }
    freq[i] = round_half_away(pmf[i] * (float)one);
    total += freq[i];
  }
  if (total == 0 || total > 0x7fffffffull) { free(freq); return -1; }
  /* 2. renormalise each bin by integer division; the last bin absorbs what the floors lost
   *    (ops.cpp forces the final cumulative value to 2^precision) */
  uint64_t run = 0;
  for (int i = 0; i < n; ++i) {
    freq[i] = (one * freq[i]) / total;
    run += freq[i];
  }
  if (run > one) { free(freq); return -1; }
  freq[n - 1] += one - run;
  /* 3. give every empty bin one count, taken from the first smallest bin with more than one */
  for (int i = 0; i < n; ++i) {
    if (freq[i] != 0) continue;
    int donor = -1;
    for (int j = 0; j < n; ++j)
      if (freq[j] > 1 && (donor < 0 || freq[j] < freq[donor])) donor = j;
    if (donor < 0) { free(freq); return -1; }
    freq[donor] -= 1;
    freq[i] += 1;
  }
  /* 4. cumulative table */
  cdf[0] = 0;
  for (int i = 0; i < n; ++i) cdf[i + 1] = cdf[i] + (uint32_t)freq[i];
  free(freq);
  return 0;
}

typedef struct { uint16_t start, range; int bypass; } RansSym;

/* returns number of 32-bit words written to out (the stream bytes, little-endian), or -1 */
int ref_rans_encode(const int32_t *symbols, const int32_t *indexes, int n, const int32_t *cdfs,
                    int stride, const int32_t *sizes, const int32_t *offsets, uint32_t *out, int cap) {
  RansSym *q = (RansSym *)malloc(sizeof(RansSym) * (size_t)(n * 20 + 4));
  size_t nq = 0;
  for (int i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    const int32_t *cdf = cdfs + (size_t)ci * stride;
    const int32_t max_value = sizes[ci] - 2;
    int32_t value = symbols[i] - offsets[ci];
    uint32_t raw = 0;
    if (value < 0) { raw = (uint32_t)(-2 * value - 1); value = max_value; }
    else if (value >= max_value) { raw = (uint32_t)(2 * (value - max_value)); value = max_value; }
    q[nq].start = (uint16_t)cdf[value];
    q[nq].range = (uint16_t)(cdf[value + 1] - cdf[value]);
    q[nq++].bypass = 0;
    if (value == max_value) {
      int32_t nb = 0;
      while (nb < 8 && (raw >> (nb * BYPASS_PREC)) != 0) ++nb;
      int32_t val = nb;
      while (val >= MAX_BYPASS) { q[nq].start = MAX_BYPASS; q[nq].range = MAX_BYPASS + 1; q[nq++].bypass = 1; val -= MAX_BYPASS; }
      q[nq].start = (uint16_t)val; q[nq].range = (uint16_t)(val + 1); q[nq++].bypass = 1;
      for (int32_t j = 0; j < nb; ++j) {
        const int32_t v = (raw >> (j * BYPASS_PREC)) & MAX_BYPASS;
        q[nq].start = (uint16_t)v; q[nq].range = (uint16_t)(v + 1); q[nq++].bypass = 1;
      }
    }
  }
  uint32_t *buf = (uint32_t *)malloc(sizeof(uint32_t) * (nq + 4));
  uint32_t *end = buf + nq + 4;
  uint32_t *ptr = end;
  uint64_t x = RANS64_L;
  while (nq > 0) {
    const RansSym s = q[--nq];
    if (!s.bypass) {
      const uint64_t x_max = ((RANS64_L >> PREC) << 32) * s.range;
      if (x >= x_max) { *--ptr = (uint32_t)x; x >>= 32; }
      x = ((x / s.range) << PREC) + (x % s.range) + s.start;
    } else {
      const uint32_t freq = 1u << (16 - BYPASS_PREC);
      const uint64_t x_max = ((RANS64_L >> 16) << 32) * freq;
      if (x >= x_max) { *--ptr = (uint32_t)x; x >>= 32; }
      x = (x << BYPASS_PREC) | s.start;
    }
  }
  ptr -= 2;
  ptr[0] = (uint32_t)x;
  ptr[1] = (uint32_t)(x >> 32);
  const int nw = (int)(end - ptr);
  int ret = -1;
  if (nw <= cap) { memcpy(out, ptr, sizeof(uint32_t) * nw); ret = nw; }
  free(buf);
  free(q);
  return ret;
}

static int dec_renorm(uint64_t *x, const uint32_t **ptr, const uint32_t *end) {
  if (*x < RANS64_L) {
    if (*ptr >= end) return -1;
    *x = (*x << 32) | **ptr;
    (*ptr)++;
  }
  return 0;
}

int ref_rans_decode(const uint32_t *words, int nwords, const int32_t *indexes, int n,
                    const int32_t *cdfs, int stride, const int32_t *sizes, const int32_t *offsets,
                    int32_t *out) {
  if (nwords < 2) return -1;
  const uint32_t *ptr = words + 2, *end = words + nwords;
  uint64_t x = (uint64_t)words[0] | ((uint64_t)words[1] << 32);
  for (int i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    const int32_t *cdf = cdfs + (size_t)ci * stride;
    const int32_t max_value = sizes[ci] - 2;
    const uint32_t cum = (uint32_t)(x & ((1u << PREC) - 1));
    int s = 0;  /* std::find_if(cdf, cdf_end, v > cum) - 1 */
    while (s + 1 < sizes[ci] && (uint32_t)cdf[s + 1] <= cum) ++s;
    x = (uint64_t)(cdf[s + 1] - cdf[s]) * (x >> PREC) + (x & ((1u << PREC) - 1)) - (uint32_t)cdf[s];
    if (dec_renorm(&x, &ptr, end)) return -1;
    int32_t value = s;
    if (value == max_value) {
      int32_t val = (int32_t)(x & MAX_BYPASS); x >>= BYPASS_PREC;
      if (dec_renorm(&x, &ptr, end)) return -1;
      int32_t nb = val;
      while (val == MAX_BYPASS) {
        val = (int32_t)(x & MAX_BYPASS); x >>= BYPASS_PREC;
        if (dec_renorm(&x, &ptr, end)) return -1;
        nb += val;
      }
      uint32_t raw = 0;
      for (int32_t j = 0; j < nb; ++j) {
        val = (int32_t)(x & MAX_BYPASS); x >>= BYPASS_PREC;
        if (dec_renorm(&x, &ptr, end)) return -1;
        raw |= (uint32_t)val << (j * BYPASS_PREC);
      }
      value = (int32_t)(raw >> 1);
      if (raw & 1) value = -value - 1; else value += max_value;
    }
    out[i] = value + offsets[ci];
  }
  return 0;
}
