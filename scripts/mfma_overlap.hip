// Does a wave's independent VALU issue inside its own MFMAs' execution? (round 5; the question
// behind profiles/r5/wino_pipe). Each wave runs a loop of blocks: three v_mfma_f32_16x16x32_f16 in
// the split-precision pattern of the Winograd kernels (acc = A0 B0; cor = A1 B0; cor += A0 B1),
// then K VALU instructions on registers no MFMA touches. Timed per configuration on the whole
// chip with 1 or 2 waves per SIMD; cycles per block from the measured time and the clock under
// load (s_memrealtime is not the shader clock: time x 1.76 GHz is printed as an estimate).
// If VALU overlapped the MFMAs, MFMA + K VALU would cost max(MFMA, VALU), not the sum.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/mfma_overlap.hip -o scripts/mfma_overlap
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

// MODE 0: MFMA blocks + K VALU (v_fma_f32); 1: VALU only; 2: MFMA only (K ignored);
// 3: MFMA blocks + K packed VALU (v_pk_fma_f32); 4: MFMA blocks with independent accumulators
// (three chains, no C dependency inside a block) + K VALU
template <int MODE, int K>
__global__ __launch_bounds__(512) void loop(const h8* in, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  h8 a0 = in[t & 4095], a1 = in[(t + 7) & 4095], b0 = in[(t + 1000) & 4095], b1 = in[(t + 2000) & 4095];
  f32x4 acc = {}, cor = {}, c2 = {};
  float v[8];
  f2v p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = (float)(t + i) * 1e-3f;
    p[i] = f2v{v[i], -v[i]};
  }
  const float m = 0.999f;
  const f2v m2 = {m, m};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
      if constexpr (MODE == 0 || MODE == 2 || MODE == 3) {
        asm volatile(
            "v_mfma_f32_16x16x32_f16 %0, %2, %4, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %1, %3, %4, %1\n\t"
            "v_mfma_f32_16x16x32_f16 %1, %2, %5, %1"
            : "+v"(acc), "+v"(cor)
            : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
      }
      if constexpr (MODE == 4) {
        asm volatile(
            "v_mfma_f32_16x16x32_f16 %0, %3, %5, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %1, %4, %5, %1\n\t"
            "v_mfma_f32_16x16x32_f16 %2, %3, %6, %2"
            : "+v"(acc), "+v"(cor), "+v"(c2)
            : "v"(a0), "v"(a1), "v"(b0), "v"(b1));
      }
      if constexpr (MODE == 0 || MODE == 1 || MODE == 4) {
#pragma unroll
        for (int k = 0; k < K; ++k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[k & 7]) : "s"(m), "v"(v[(k + 3) & 7]));
      }
      if constexpr (MODE == 3) {
#pragma unroll
        for (int k = 0; k < K; ++k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[k & 7]) : "v"(m2), "v"(p[(k + 3) & 7]));
      }
    }
  }
  asm volatile("s_nop 11" : "+v"(acc), "+v"(cor), "+v"(c2));  // MFMA results -> VALU reads
  float s = acc[0] + acc[1] + cor[2] + cor[3] + c2[0];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += v[i] + p[i].x;
  out[t] = s;
}

template <int MODE, int K>
static void run(const char* name, const h8* in, float* out, int blocks, int threads, int iters) {
  hipLaunchKernelGGL((loop<MODE, K>), dim3(blocks), dim3(threads), 0, 0, in, out, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((loop<MODE, K>), dim3(blocks), dim3(threads), 0, 0, in, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double blocks_per_wave = (double)iters * 8;
  const double ns_per_block = ms * 1e6 / blocks_per_wave;
  printf("%-34s waves/SIMD %d  %7.2f ns/block  ~%6.1f cycles/block at 1.76 GHz\n", name, threads / 256, ns_per_block,
         ns_per_block * 1.76);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  h8* in;
  float* out;
  hipMalloc(&in, 4096 * sizeof(h8));
  hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
  hipMemset(in, 0, 4096 * sizeof(h8));
  for (int threads = 256; threads <= 512; threads += 256) {
    run<2, 0>("mfma x3 only", in, out, cus, threads, iters);
    run<1, 6>("valu x6 only", in, out, cus, threads, iters);
    run<1, 12>("valu x12 only", in, out, cus, threads, iters);
    run<0, 2>("mfma x3 + valu x2", in, out, cus, threads, iters);
    run<0, 6>("mfma x3 + valu x6", in, out, cus, threads, iters);
    run<0, 12>("mfma x3 + valu x12", in, out, cus, threads, iters);
    run<3, 6>("mfma x3 + pk valu x6", in, out, cus, threads, iters);
    run<4, 0>("mfma x3 indep only", in, out, cus, threads, iters);
    run<4, 6>("mfma x3 indep + valu x6", in, out, cus, threads, iters);
    run<4, 12>("mfma x3 indep + valu x12", in, out, cus, threads, iters);
  }
  hipFree(in);
  hipFree(out);
  return 0;
}
