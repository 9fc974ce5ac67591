// r6: standalone reproducer for the K7-stem / warp-gather hazard (profiles/r6/race/README.md).
// No torch, no pipeline: two HIP streams and two C-ABI entry points of an experiment build of
// libfvc (-DFVC_STEM_K7, which puts SpyNet's 7x7 8 -> 32 layer on conv_stem_kernel).
//   stream A: fvc_conv2d_nhwc_stem 7x7 8->32 over a 5-level pyramid (the SpyNet launch pattern)
//   stream B: fvc_mc_assemble (k_mc_assemble_q: bilinear 4-tap gathers, two pixels per thread) on
//             fixed inputs, then a compare kernel against a golden output made with stream A idle
// Every mismatching pixel is counted by wave-lane quarter and by which of the thread's pixels
// (first / second of its pair) it is.
// build: hipcc --offload-arch=gfx950 -O2 -Iinclude scripts/race_repro.hip -o gpurun_out/race_repro \
//          -Lfastvideocodec_amd -l:libfvc_k7.so -Wl,-rpath,$PWD/fastvideocodec_amd
// run:   gpurun_out/race_repro ITERS STEM(0|1)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "fvc.h"

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                     \
    }                                                                              \
  } while (0)
#define CF(x)                                                   \
  do {                                                          \
    int r_ = (x);                                               \
    if (r_ != 0) {                                              \
      fprintf(stderr, "%s:%d %s returned %d\n", __FILE__, __LINE__, #x, r_); \
      exit(2);                                                  \
    }                                                           \
  } while (0)

// stats: [0] mismatching pixels, [1..4] by lane quarter, [5..6] by pair member, [7] first bad pixel + 1
__global__ void k_compare(const float4* __restrict__ a, const float4* __restrict__ gold, unsigned n, unsigned st,
                          int* stats) {
  for (unsigned q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const float4 x = a[q], g = gold[q];
    if (__float_as_uint(x.x) != __float_as_uint(g.x) || __float_as_uint(x.y) != __float_as_uint(g.y) ||
        __float_as_uint(x.z) != __float_as_uint(g.z)) {
      const unsigned th = q % st, j = q / st;
      atomicAdd(stats, 1);
      atomicAdd(stats + 1 + (th & 63) / 16, 1);
      atomicAdd(stats + 5 + (j & 1), 1);
      atomicMax(stats + 7, (int)q + 1);
    }
  }
}

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return (float)(s >> 8) * (1.f / 16777216.f);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  const int use_stem = argc > 2 ? atoi(argv[2]) : 1;
  const int H = 2176, W = 3840;
  const size_t npix = (size_t)H * W;
  unsigned seed = 12345u;

  // ---- motion compensation inputs: ref in [0, 1] (clamped recon-like, with exact zeros), flow ~ +-3 px
  std::vector<float> ref(npix * 4), mv(npix * 4);
  for (size_t p = 0; p < npix; ++p) {
    for (int c = 0; c < 3; ++c) {
      const float v = frand(seed) * 1.6f - 0.3f;
      ref[p * 4 + c] = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
    }
    ref[p * 4 + 3] = 0.f;
    mv[p * 4 + 0] = (frand(seed) - 0.5f) * 6.f;
    mv[p * 4 + 1] = (frand(seed) - 0.5f) * 6.f;
    mv[p * 4 + 2] = mv[p * 4 + 3] = 0.f;
  }
  float *dref, *dmv, *dwf, *dx8, *dgold;
  int* dstats;
  CK(hipMalloc(&dref, npix * 16));
  CK(hipMalloc(&dmv, npix * 16));
  CK(hipMalloc(&dwf, npix * 16));
  CK(hipMalloc(&dx8, npix * 32));
  CK(hipMalloc(&dgold, npix * 16));
  CK(hipMalloc(&dstats, 8 * sizeof(int)));
  CK(hipMemcpy(dref, ref.data(), npix * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dmv, mv.data(), npix * 16, hipMemcpyHostToDevice));
  CK(hipMemset(dstats, 0, 8 * sizeof(int)));

  // ---- the 7x7 8 -> 32 stem over five pyramid levels
  const int cin = 8, cout = 32, k = 7;
  if (use_stem && !fvc_conv_stem_supported(cin, cout, k, 1, 0)) {
    fprintf(stderr, "this library has no 7x7 stem (build with -DFVC_STEM_K7)\n");
    return 2;
  }
  std::vector<float> w((size_t)cout * cin * k * k), bias(cout);
  for (auto& v : w) v = (frand(seed) - 0.5f) * 0.1f;
  for (auto& v : bias) v = (frand(seed) - 0.5f) * 0.1f;
  const size_t wbytes = fvc_conv_stem_wpack_bytes(cin, cout, k);
  std::vector<char> wp(wbytes > 0 ? wbytes : 16);
  float osc = 1.f;
  void* dwp = nullptr;
  float* dbias = nullptr;
  int* dovf = nullptr;
  if (use_stem) {
    CF(fvc_conv_stem_pack_weight(w.data(), cin, cout, k, wp.data(), &osc));
    CK(hipMalloc(&dwp, wbytes));
    CK(hipMemcpy(dwp, wp.data(), wbytes, hipMemcpyHostToDevice));
    CK(hipMalloc(&dbias, cout * 4));
    CK(hipMemcpy(dbias, bias.data(), cout * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dovf, 4));
    CK(hipMemset(dovf, 0, 4));
  }
  float *sx[5] = {}, *sy[5] = {};
  for (int l = 0; l < 5 && use_stem; ++l) {
    const size_t n = (size_t)(H >> l) * (W >> l);
    std::vector<float> xh(n * 8);
    for (auto& v : xh) v = frand(seed);
    CK(hipMalloc(&sx[l], n * 32));
    CK(hipMalloc(&sy[l], n * 128));
    CK(hipMemcpy(sx[l], xh.data(), n * 32, hipMemcpyHostToDevice));
  }

  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));

  // golden with stream A idle
  CF(fvc_mc_assemble(dref, dmv, dgold, dx8, 1, H, W, (fvc_stream_t)sb));
  CK(hipStreamSynchronize(sb));
  // k_mc_assemble_q's grid: min(8192, ceil(npix / 2 / 256)) blocks of 256 threads
  size_t g = (npix / 2 + 255) / 256;
  if (g > 8192) g = 8192;
  const unsigned st = (unsigned)(g * 256);

  for (int it = 0; it < iters; ++it) {
    if (use_stem)
      for (int rep = 0; rep < 2; ++rep)
        for (int l = 4; l >= 0; --l)
          CF(fvc_conv2d_nhwc_stem(sx[l], dwp, osc, dbias, sy[l], 1, H >> l, W >> l, cin, cout, k, 1, 1 /*relu*/,
                                  dovf, (fvc_stream_t)sa));
    for (int rep = 0; rep < 4; ++rep) {
      CF(fvc_mc_assemble(dref, dmv, dwf, dx8, 1, H, W, (fvc_stream_t)sb));
      hipLaunchKernelGGL(k_compare, dim3(4096), dim3(256), 0, sb, (const float4*)dwf, (const float4*)dgold,
                         (unsigned)npix, st, dstats);
      CK(hipGetLastError());
    }
    if ((it + 1) % 16 == 0) {
      CK(hipDeviceSynchronize());
      int s[8];
      CK(hipMemcpy(s, dstats, sizeof(s), hipMemcpyDeviceToHost));
      printf("iter %d: mismatching px %d (lane quarters %d %d %d %d; pair first %d second %d)\n", it + 1, s[0], s[1],
             s[2], s[3], s[4], s[5], s[6]);
      fflush(stdout);
    }
  }
  CK(hipDeviceSynchronize());
  int s[8];
  CK(hipMemcpy(s, dstats, sizeof(s), hipMemcpyDeviceToHost));
  printf("RESULT stem=%d iters=%d mc_launches=%d mismatching_px=%d lane_quarters=[%d,%d,%d,%d] pair=[%d,%d]\n",
         use_stem, iters, iters * 4, s[0], s[1], s[2], s[3], s[4], s[5], s[6]);
  return 0;
}
