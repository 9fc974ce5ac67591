// Shared helpers for libfvc (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/fvc.h"

#define FVC_CHECK_LAUNCH()                                   \
  do {                                                       \
    hipError_t e__ = hipGetLastError();                      \
    if (e__ != hipSuccess) return -(int)e__;                 \
  } while (0)

static inline int fvc_cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int fvc_rup(int a, int b) { return fvc_cdiv(a, b) * b; }

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float fvc_apply_in_op(float v, int op) {
  switch (op) {
    case FVC_IN_RELU: return v > 0.f ? v : 0.f;
    case FVC_IN_ABS: return fabsf(v);
    case FVC_IN_ROUND: return rintf(v);  // torch.round = half-to-even
    default: return v;
  }
}

// Branch-free form for staging code: selects on a wave-uniform op keep the compiler from
// splitting the staging path into per-element branches (each with its own s_waitcnt).
__device__ __forceinline__ float fvc_in_op_sel(float v, int op) {
  float t = (op == FVC_IN_ROUND) ? rintf(v) : v;
  t = (op == FVC_IN_ABS) ? fabsf(t) : t;
  t = (op == FVC_IN_RELU) ? fmaxf(t, 0.f) : t;
  return t;
}

__device__ __forceinline__ float4 fvc_in_op_sel4(float4 v, int op) {
  return make_float4(fvc_in_op_sel(v.x, op), fvc_in_op_sel(v.y, op), fvc_in_op_sel(v.z, op),
                     fvc_in_op_sel(v.w, op));
}

__device__ __forceinline__ float4 fvc_apply_in_op4(float4 v, int op) {
  v.x = fvc_apply_in_op(v.x, op);
  v.y = fvc_apply_in_op(v.y, op);
  v.z = fvc_apply_in_op(v.z, op);
  v.w = fvc_apply_in_op(v.w, op);
  return v;
}

// ------------------------------------------------------------------ bilinear upsampling (shared)
// ATen compute_indices_weights_linear for align_corners=True with the scale (in-1)/(out-1)
// precomputed (the caller computes it the same way: one correctly rounded float division), and the
// bilinear combination in ATen's order (a l0x + b l1x) l0y + (c l0x + d l1x) l1y, every product and
// sum rounded on its own (no contraction: the form the standalone upsample kernel has always
// computed), so the standalone upsample-add kernel (fvc_elem.hip) and the Winograd kernel's fused
// upsample-add staging (fvc_conv_wino.hip) produce the same bits.
struct FvcUpIdx {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ FvcUpIdx fvc_up_index_scaled(int d, int in, float scale) {
#pragma clang fp contract(off)
  const float src = scale * (float)d;
  int i0 = (int)floorf(src);
  const float lam = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  if (i0 > in - 1) i0 = in - 1;
  FvcUpIdx u;
  u.i0 = i0;
  u.i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  u.l1 = lam;
  u.l0 = 1.f - lam;
  return u;
}

// one row's horizontal step a l0 + b l1 and the vertical step h0 l0y + h1 l1y (both unfused)
__device__ __forceinline__ float fvc_lerp1(float a, float b, float l0, float l1) {
#pragma clang fp contract(off)
  return a * l0 + b * l1;
}

__device__ __forceinline__ float fvc_lerp2d(float a, float b, float c, float d, float l0x, float l1x, float l0y,
                                            float l1y) {
  return fvc_lerp1(fvc_lerp1(a, b, l0x, l1x), fvc_lerp1(c, d, l0x, l1x), l0y, l1y);
}

__device__ __forceinline__ float4 fvc_lerp2d4(const float4& a, const float4& b, const float4& c, const float4& d,
                                              const FvcUpIdx& uy, const FvcUpIdx& ux) {
  return make_float4(fvc_lerp2d(a.x, b.x, c.x, d.x, ux.l0, ux.l1, uy.l0, uy.l1),
                     fvc_lerp2d(a.y, b.y, c.y, d.y, ux.l0, ux.l1, uy.l0, uy.l1),
                     fvc_lerp2d(a.z, b.z, c.z, d.z, ux.l0, ux.l1, uy.l0, uy.l1),
                     fvc_lerp2d(a.w, b.w, c.w, d.w, ux.l0, ux.l1, uy.l0, uy.l1));
}
