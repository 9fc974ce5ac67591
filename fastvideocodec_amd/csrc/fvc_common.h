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
