// Sustained v_mfma_f32_32x32x16_f16 rate on the whole chip with register operands (random fp16
// data, 8 waves per CU, 4 accumulators per wave, no memory in the loop): the practical MFMA
// ceiling the conv kernels are compared against (clock under matrix load, not the 2.4 GHz peak).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/mfma_peak.hip -o scripts/mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(512) void mfma_loop(const h8* in, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  h8 a = in[t & 4095], b = in[(t + 1000) & 4095];
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x16{};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[t] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus;  // one 512-thread block (8 waves) per CU
  h8* in;
  float* out;
  hipMalloc(&in, 4096 * sizeof(h8));
  hipMalloc(&out, (size_t)blocks * 512 * sizeof(float));
  _Float16 host[4096 * 8];
  srand(1);
  for (int i = 0; i < 4096 * 8; ++i) host[i] = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  hipMemcpy(in, host, sizeof(host), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(512), 0, 0, in, out, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(512), 0, 0, in, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)blocks * 8 * iters * 3 * 4 * (32.0 * 32 * 16 * 2);
    const double tfs = flops / (ms * 1e-3) / 1e12;
    // 4 SIMDs x (32x32x16x2 flop per 32 cycles) per CU
    const double ghz = tfs * 1e12 / (cus * 4.0 * (32 * 32 * 16 * 2) / 32.0) / 1e9;
    printf("mfma_f32_32x32x16_f16: %.3f ms  %.1f TF/s dense  (x3 ceiling %.1f TF/s)  implied clock %.2f GHz\n",
           ms, tfs, tfs / 3, ghz);
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
