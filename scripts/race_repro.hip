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
// run:   gpurun_out/race_repro ITERS ANTAGONIST VICTIM
//   ANTAGONIST 0 none, 1 the library's 7x7 stem (fvc_conv2d_nhwc_stem), else a synthetic persistent
//              kernel (k_antagonist) given as MF,LDSREAD,LDS_BYTES,LO,SPAN, e.g. 1,1,85376,0,85360 =
//              32x32x16 MFMAs on ds_read_b128 operands over all of an 85 KB allocation
//   VICTIM     0 the library's fvc_mc_assemble (12-B gathers: global_load_dwordx3), 1 a local copy of
//              its gather loop with 12-B loads, 2 the same copy with 16-B loads (global_load_dwordx4),
//              3 a coalesced two-input copy (no gathers)
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

// local copy of k_mc_assemble_q's gather loop (two pixels per thread, every load issued before the
// stores), simplified tap math; W16: keep the fourth channel so every gather is a 16-B load
template <bool W16>
__global__ void k_gather(const float4* __restrict__ ref, const float4* __restrict__ mv, float4* __restrict__ out,
                         int H, int W) {
  const unsigned npix = (unsigned)H * W, st = gridDim.x * blockDim.x;
  for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += 2 * st) {
    const unsigned p2 = p + st < npix ? p + st : p;
    const float4 f1 = mv[p], f2 = mv[p2];
    float4 o[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const unsigned q = k ? p2 : p;
      const float4 f = k ? f2 : f1;
      const int y = (int)(q / W), x = (int)(q - (unsigned)y * W);
      const float fx = fminf(fmaxf(x + f.x, 0.f), (float)(W - 1)), fy = fminf(fmaxf(y + f.y, 0.f), (float)(H - 1));
      const int x0 = (int)fx, y0 = (int)fy;
      const unsigned dx = x0 + 1 < W ? 1u : 0u, dy = y0 + 1 < H ? (unsigned)W : 0u;
      const float ax = fx - x0, ay = fy - y0;
      const unsigned r0 = (unsigned)y0 * W + x0;
      const float4 a = ref[r0], b = ref[r0 + dx], c = ref[r0 + dy], d = ref[r0 + dy + dx];
      const float wa = (1 - ax) * (1 - ay), wb = ax * (1 - ay), wc = (1 - ax) * ay, wd = ax * ay;
      o[k].x = a.x * wa + b.x * wb + c.x * wc + d.x * wd;
      o[k].y = a.y * wa + b.y * wb + c.y * wc + d.y * wd;
      o[k].z = a.z * wa + b.z * wb + c.z * wc + d.z * wd;
      o[k].w = W16 ? a.w * wa + b.w * wb + c.w * wc + d.w * wd : 0.f;
    }
    out[p] = o[0];
    out[p2] = o[1];
  }
}

// coalesced victim: out = ref + mv, pixel-contiguous 16-B loads and stores (two pixels per thread)
__global__ void k_copy2(const float4* __restrict__ ref, const float4* __restrict__ mv, float4* __restrict__ out,
                        unsigned npix) {
  const unsigned st = gridDim.x * blockDim.x;
  for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += 2 * st) {
    const unsigned p2 = p + st < npix ? p + st : p;
    const float4 a = ref[p], b = mv[p], c = ref[p2], d = mv[p2];
    out[p] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, 0.f);
    out[p2] = make_float4(c.x + d.x, c.y + d.y, c.z + d.z, 0.f);
  }
}

// synthetic antagonists: one 512-thread block per CU, each wave issuing, for `rounds` iterations,
// 8 x (ds_read_b128 from [lo, lo + span) of its LDS when LDSREAD, and MF = 1: v_mfma_f32_32x32x16_f16,
// 2: v_mfma_f32_16x16x32_f16, 0: a plain f32 add). No global memory in the loop; one store per lane
// at the end keeps the work alive.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <int MF, bool LDSREAD>
__global__ __launch_bounds__(512) void k_antagonist(float* out, int rounds, int lds_bytes, int lo, int span) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  for (int i = tid; i < lds_bytes / 16; i += 512) reinterpret_cast<uint4*>(smem)[i] = make_uint4(i, i * 3, i * 5, i * 7);
  __syncthreads();
  f32x16 acc = {};
  f32x4v acc4 = {};
  float sum = 0.f;
  const h8 w = {1, 1, 1, 1, 1, 1, 1, 1};
  h8 x = {(_Float16)tid, 1, 2, 3, 4, 5, 6, 7};
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if constexpr (LDSREAD) {
        const int o = lo + (((tid * 7 + r * 13 + s * 29) * 16) % span);
        x = *reinterpret_cast<const h8*>(smem + (o & ~15));
      } else {
        x[0] = x[0] + (_Float16)1;
      }
      if constexpr (MF == 1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w, x, acc, 0, 0, 0);
      if constexpr (MF == 2) acc4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w, x, acc4, 0, 0, 0);
      if constexpr (MF == 0) sum += (float)x[0] + (float)x[7];
    }
  }
  float t = sum;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += acc[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) t += acc4[i];
  out[blockIdx.x * 512 + tid] = t;
}

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return (float)(s >> 8) * (1.f / 16777216.f);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  int antagonist = 1, amf = 1, ardl = 1, abytes = 85376, alo = 0, aspan = 85360;
  if (argc > 2) {
    if (strchr(argv[2], ',')) {
      antagonist = 2;
      sscanf(argv[2], "%d,%d,%d,%d,%d", &amf, &ardl, &abytes, &alo, &aspan);
    } else {
      antagonist = atoi(argv[2]);
    }
  }
  const int victim = argc > 3 ? atoi(argv[3]) : 0;
  const int use_stem = antagonist == 1;
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

  float* dant = nullptr;
  CK(hipMalloc(&dant, 256 * 512 * 4));
  const void* kant = nullptr;
  if (antagonist == 2) {
    const void* tab[3][2] = {{(const void*)k_antagonist<0, false>, (const void*)k_antagonist<0, true>},
                             {(const void*)k_antagonist<1, false>, (const void*)k_antagonist<1, true>},
                             {(const void*)k_antagonist<2, false>, (const void*)k_antagonist<2, true>}};
    kant = tab[amf][ardl ? 1 : 0];
    CK(hipFuncSetAttribute(kant, hipFuncAttributeMaxDynamicSharedMemorySize, abytes));
  }
  auto run_victim = [&](float* outp, hipStream_t s) {
    const unsigned gg = (unsigned)((npix / 2 + 255) / 256 > 8192 ? 8192 : (npix / 2 + 255) / 256);
    if (victim == 0) {
      CF(fvc_mc_assemble(dref, dmv, outp, dx8, 1, H, W, (fvc_stream_t)s));
    } else if (victim == 1) {
      hipLaunchKernelGGL(k_gather<false>, dim3(gg), dim3(256), 0, s, (const float4*)dref, (const float4*)dmv,
                         (float4*)outp, H, W);
    } else if (victim == 3) {
      hipLaunchKernelGGL(k_copy2, dim3(gg), dim3(256), 0, s, (const float4*)dref, (const float4*)dmv, (float4*)outp,
                         (unsigned)npix);
    } else {
      hipLaunchKernelGGL(k_gather<true>, dim3(gg), dim3(256), 0, s, (const float4*)dref, (const float4*)dmv,
                         (float4*)outp, H, W);
    }
    CK(hipGetLastError());
  };
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));

  // golden with stream A idle
  run_victim(dgold, sb);
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
    if (antagonist == 2) {
      int rounds = 4000;
      void* args[] = {&dant, &rounds, &abytes, &alo, &aspan};
      CK(hipLaunchKernel(kant, dim3(256), dim3(512), args, abytes, sa));
    }
    for (int rep = 0; rep < 4; ++rep) {
      run_victim(dwf, sb);
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
  printf("RESULT antagonist=%s victim=%d iters=%d victim_launches=%d mismatching_px=%d lane_quarters=[%d,%d,%d,%d] "
         "pair=[%d,%d]\n", argc > 2 ? argv[2] : "1", victim, iters, iters * 4, s[0], s[1], s[2], s[3], s[4], s[5], s[6]);
  return 0;
}
