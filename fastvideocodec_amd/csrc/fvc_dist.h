// Device CDFs shared by the bit estimators (fvc_elem.hip) and the torchac-compatible coder's
// tables (fvc_torchac.hip), float32 in the order torch evaluates them.
#pragma once
#include <hip/hip_runtime.h>

// torch.distributions.Laplace(0, s).cdf(v) = 0.5 - 0.5 * sign(v) * expm1(-|v| / s)  (net.py:143)
__device__ __forceinline__ float fvc_laplace_cdf(float v, float s) {
  const float sg = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
  return 0.5f - 0.5f * sg * expm1f(-fabsf(v) / s);
}

__device__ __forceinline__ float fvc_softplus(float v) { return v > 20.f ? v : log1pf(expf(v)); }

// DVC BitEstimator CDF of channel c (bitEstimator.py:18-42); prm [11][C] = (h, b, a) x 3, h4, b4
__device__ __forceinline__ float fvc_bitest_cdf(float x, const float* prm, int C, int c) {
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const float h = prm[(3 * f) * C + c], b = prm[(3 * f + 1) * C + c], a = prm[(3 * f + 2) * C + c];
    x = x * fvc_softplus(h) + b;
    x = x + tanhf(x) * tanhf(a);
  }
  const float h = prm[9 * C + c], b = prm[10 * C + c];
  const float t = x * fvc_softplus(h) + b;
  return 1.f / (1.f + expf(-t));
}
