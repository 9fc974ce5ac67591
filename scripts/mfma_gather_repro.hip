// r6: minimal standalone reproducer (no libfvc, no torch, no LDS, no shared data) of the fault that
// the r5/r6 race probes traced to the warp gathers (profiles/r6/race/README.md):
//   stream A: k_mfma  -- a persistent grid whose waves issue back-to-back dependent MFMAs on
//             register operands only (no memory traffic in the loop)
//   stream B: k_gather -- reads a fixed image at data-dependent addresses (4 taps per pixel, two
//             pixels per thread, every load issued before the first use), writes one pixel each;
//             then k_compare counts pixels that differ from a golden output made with stream A idle
// On MI355X (gfx950, ROCm 7.2) the gathers return zeros for some lanes 48..63 of a wave while k_mfma
// runs; coalesced loads in the same setting, and gathers beside a VALU-only antagonist, are exact.
// build: hipcc --offload-arch=gfx950 -O2 scripts/mfma_gather_repro.hip -o mfma_gather_repro
// run:   ./mfma_gather_repro ITERS KIND THREADS BLOCKS_PER_CU NLOADS
//   KIND 0 VALU-only antagonist (control), 1 v_mfma_f32_32x32x16_f16, 2 v_mfma_f32_16x16x32_f16,
//        3 v_mfma_f32_32x32x2_f32, 4 none (victim alone)
//   THREADS antagonist block size (64..1024), BLOCKS_PER_CU antagonist blocks per CU,
//   NLOADS gathers in flight per thread before the first use: 4 (one pixel) or 8 (two pixels)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ void k_mfma(float* out, int rounds) {
  f32x16 acc = {};
  f32x4 acc4 = {};
  float s = (float)threadIdx.x;
  const h8 a = {1, 1, 1, 1, 1, 1, 1, 1};
  h8 b = {(_Float16)(threadIdx.x & 7), 1, 2, 3, 4, 5, 6, 7};
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
      if constexpr (KIND == 2) acc4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc4, 0, 0, 0);
      if constexpr (KIND == 3) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(s, 1.0f, acc, 0, 0, 0);
      if constexpr (KIND == 0) s = fmaf(s, 1.0001f, 0.5f);
    }
  }
  float t = s;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += acc[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) t += acc4[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

// bilinear 4-tap gather of a W x H image of float4 pixels by a per-pixel offset (clamped)
__device__ __forceinline__ float4 tap4(const float4* __restrict__ img, const float4 f, unsigned q, int W, int H,
                                       float4 (&v)[4], float (&w)[4]) {
  const int y = (int)(q / W), x = (int)(q - (unsigned)y * W);
  const float fx = fminf(fmaxf(x + f.x, 0.f), (float)(W - 1)), fy = fminf(fmaxf(y + f.y, 0.f), (float)(H - 1));
  const int x0 = (int)fx, y0 = (int)fy;
  const unsigned dx = x0 + 1 < W ? 1u : 0u, dy = y0 + 1 < H ? (unsigned)W : 0u;
  const float ax = fx - x0, ay = fy - y0;
  const unsigned r0 = (unsigned)y0 * W + x0;
  v[0] = img[r0];
  v[1] = img[r0 + dx];
  v[2] = img[r0 + dy];
  v[3] = img[r0 + dy + dx];
  w[0] = (1 - ax) * (1 - ay);
  w[1] = ax * (1 - ay);
  w[2] = (1 - ax) * ay;
  w[3] = ax * ay;
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ float4 combine(const float4 (&v)[4], const float (&w)[4]) {
  float4 o;
  o.x = v[0].x * w[0] + v[1].x * w[1] + v[2].x * w[2] + v[3].x * w[3];
  o.y = v[0].y * w[0] + v[1].y * w[1] + v[2].y * w[2] + v[3].y * w[3];
  o.z = v[0].z * w[0] + v[1].z * w[1] + v[2].z * w[2] + v[3].z * w[3];
  o.w = 0.f;
  return o;
}

template <int NLOADS>
__global__ void k_gather(const float4* __restrict__ img, const float4* __restrict__ off, float4* __restrict__ out,
                         int H, int W) {
  const unsigned npix = (unsigned)H * W, st = gridDim.x * blockDim.x;
  if constexpr (NLOADS == 8) {
    for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += 2 * st) {
      const unsigned p2 = p + st < npix ? p + st : p;
      const float4 f1 = off[p], f2 = off[p2];
      float4 v1[4], v2[4];
      float w1[4], w2[4];
      tap4(img, f1, p, W, H, v1, w1);
      tap4(img, f2, p2, W, H, v2, w2);
      out[p] = combine(v1, w1);
      out[p2] = combine(v2, w2);
    }
  } else {
    for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += st) {
      float4 v[4];
      float w[4];
      tap4(img, off[p], p, W, H, v, w);
      out[p] = combine(v, w);
    }
  }
}

// stats: [0] mismatching pixels, [1..4] by lane quarter of the thread that wrote the pixel
__global__ void k_compare(const float4* __restrict__ a, const float4* __restrict__ gold, unsigned n, unsigned st,
                          int* stats) {
  for (unsigned q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const float4 x = a[q], g = gold[q];
    if (__float_as_uint(x.x) != __float_as_uint(g.x) || __float_as_uint(x.y) != __float_as_uint(g.y) ||
        __float_as_uint(x.z) != __float_as_uint(g.z)) {
      atomicAdd(stats, 1);
      atomicAdd(stats + 1 + ((q % st) & 63) / 16, 1);
    }
  }
}

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return (float)(s >> 8) * (1.f / 16777216.f);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const int kind = argc > 2 ? atoi(argv[2]) : 1;
  const int threads = argc > 3 ? atoi(argv[3]) : 512;
  const int per_cu = argc > 4 ? atoi(argv[4]) : 1;
  const int nloads = argc > 5 ? atoi(argv[5]) : 8;
  const int H = 2176, W = 3840;
  const size_t npix = (size_t)H * W;
  unsigned seed = 777u;
  std::vector<float> img(npix * 4), off(npix * 4);
  for (size_t p = 0; p < npix; ++p) {
    for (int c = 0; c < 3; ++c) img[p * 4 + c] = frand(seed);
    img[p * 4 + 3] = 0.f;
    off[p * 4 + 0] = (frand(seed) - 0.5f) * 6.f;
    off[p * 4 + 1] = (frand(seed) - 0.5f) * 6.f;
    off[p * 4 + 2] = off[p * 4 + 3] = 0.f;
  }
  float4 *dimg, *doff, *dout, *dgold;
  float* dant;
  int* dstats;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipMalloc(&dimg, npix * 16));
  CK(hipMalloc(&doff, npix * 16));
  CK(hipMalloc(&dout, npix * 16));
  CK(hipMalloc(&dgold, npix * 16));
  CK(hipMalloc(&dant, (size_t)ncu * per_cu * threads * 4));
  CK(hipMalloc(&dstats, 5 * sizeof(int)));
  CK(hipMemcpy(dimg, img.data(), npix * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(doff, off.data(), npix * 16, hipMemcpyHostToDevice));
  CK(hipMemset(dstats, 0, 5 * sizeof(int)));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  const unsigned gg = (unsigned)((npix / (nloads == 8 ? 2 : 1) + 255) / 256 > 8192 ? 8192
                                                                                   : (npix / (nloads == 8 ? 2 : 1) + 255) / 256);
  const unsigned st = gg * 256;
  auto victim = [&](float4* o) {
    if (nloads == 8) hipLaunchKernelGGL(k_gather<8>, dim3(gg), dim3(256), 0, sb, dimg, doff, o, H, W);
    else hipLaunchKernelGGL(k_gather<4>, dim3(gg), dim3(256), 0, sb, dimg, doff, o, H, W);
    CK(hipGetLastError());
  };
  victim(dgold);
  CK(hipDeviceSynchronize());
  const int rounds = 2000;
  for (int it = 0; it < iters; ++it) {
    const dim3 g(ncu * per_cu), b(threads);
    if (kind == 0) hipLaunchKernelGGL(k_mfma<0>, g, b, 0, sa, dant, rounds);
    if (kind == 1) hipLaunchKernelGGL(k_mfma<1>, g, b, 0, sa, dant, rounds);
    if (kind == 2) hipLaunchKernelGGL(k_mfma<2>, g, b, 0, sa, dant, rounds);
    if (kind == 3) hipLaunchKernelGGL(k_mfma<3>, g, b, 0, sa, dant, rounds);
    CK(hipGetLastError());
    for (int r = 0; r < 4; ++r) {
      victim(dout);
      hipLaunchKernelGGL(k_compare, dim3(4096), dim3(256), 0, sb, dout, dgold, (unsigned)npix, st, dstats);
      CK(hipGetLastError());
    }
  }
  CK(hipDeviceSynchronize());
  int s[5];
  CK(hipMemcpy(s, dstats, sizeof(s), hipMemcpyDeviceToHost));
  printf("RESULT kind=%d threads=%d blocks_per_cu=%d nloads=%d victim_launches=%d px_checked=%zu mismatching_px=%d "
         "lane_quarters=[%d,%d,%d,%d]\n",
         kind, threads, per_cu, nloads, iters * 4, (size_t)iters * 4 * npix, s[0], s[1], s[2], s[3], s[4]);
  return 0;
}
