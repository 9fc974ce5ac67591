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

__device__ __forceinline__ float4 fvc_apply_in_op4(float4 v, int op) {
  v.x = fvc_apply_in_op(v.x, op);
  v.y = fvc_apply_in_op(v.y, op);
  v.z = fvc_apply_in_op(v.z, op);
  v.w = fvc_apply_in_op(v.w, op);
  return v;
}
