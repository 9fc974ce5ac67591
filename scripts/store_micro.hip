// Store-pattern micro-benchmark (MI355X): the same 535 MB output (1088 x 1920 pixels x 64 fp32
// channels) written with the x3 epilogue's lane layout (lane = pixel, one 16-B group of 4 channels
// per store: 32-B pieces per pixel per instruction) vs 128-B coalesced pieces (8 lanes per pixel
// per instruction) vs fully contiguous 1-KB wave stores. Prints GB/s per pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

// pattern 0: x3 layout. wave covers 32 pixels x 32 channels (an N-tile): lane (li, lh) -> pixel
// li, groups g = 0..3 -> channels 8g + 4lh .. +3: 4 stores, each 32 pixels x 32 B
// pattern 1: coalesced: store s -> pixels 8s .. 8s + 7, lane -> pixel 8s + (lane >> 3), quad lane & 7
// pattern 2: contiguous: store s -> bytes [1 KB s, 1 KB (s + 1)) of the wave's 4 KB tile... (pixel-major)
template <int PAT>
__global__ __launch_bounds__(256) void k_store(float* __restrict__ y, int npix, int C) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntile = C / 32;
  const long long wtiles = (long long)(npix / 32) * ntile;
  for (long long wt = (long long)blockIdx.x * 4 + wave; wt < wtiles; wt += (long long)gridDim.x * 4) {
    const int n = (int)(wt % ntile);
    const long long p0 = (wt / ntile) * 32;
    const f4 v = {1.f, 2.f, 3.f, 4.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      long long off;
      if (PAT == 0) {
        const int li = lane & 31, lh = lane >> 5;
        off = (p0 + li) * C + n * 32 + 8 * s + 4 * lh;
      } else if (PAT == 1) {
        off = (p0 + 8 * s + (lane >> 3)) * C + n * 32 + 4 * (lane & 7);
      } else {
        off = (p0 + 8 * s + (lane >> 3)) * C + n * 32 + 4 * (lane & 7);  // same bytes as 1 ...
        if (C == 32) off = p0 * C + (long long)(s * 64 + lane) * 4;        // ... or a flat 1-KB run
      }
      *reinterpret_cast<f4*>(y + off) = v;
    }
  }
}

int main() {
  const int npix = 1088 * 1920 * 4, C = 64;
  float* y;
  hipMalloc(&y, (size_t)npix * C * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int pat = 0; pat < 2; ++pat)
    for (int grid : {1024, 4096}) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        for (int it = 0; it < 5; ++it) {
          if (pat == 0) hipLaunchKernelGGL(k_store<0>, dim3(grid), dim3(256), 0, 0, y, npix, C);
          else hipLaunchKernelGGL(k_store<1>, dim3(grid), dim3(256), 0, 0, y, npix, C);
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep) printf("pattern %d grid %d: %.3f ms per write of %.0f MB, %.1f GB/s\n", pat, grid, ms / 5,
                        (double)npix * C * 4 / 1e6, (double)npix * C * 4 / (ms / 5 * 1e-3) / 1e9);
      }
    }
  hipFree(y);
  return 0;
}
