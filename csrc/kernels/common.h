// Shared device helpers for the jax_raft_amd gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define JR_DEVICE __device__ __forceinline__

JR_DEVICE float bf2f(bf16 v) { return (float)v; }
JR_DEVICE bf16 f2bf(float v) { return (bf16)v; }

JR_DEVICE float rcpf_(float x) { return __builtin_amdgcn_rcpf(x); }
JR_DEVICE float sigmoidf_(float x) { return rcpf_(1.0f + __expf(-x)); }
JR_DEVICE float tanhf_(float x) {
  // tanh(x) = 1 - 2 / (exp(2x) + 1); saturates cleanly for large |x|.
  float e = __expf(2.0f * x);
  return 1.0f - 2.0f * rcpf_(e + 1.0f);
}

// Activation codes shared with the host side (jax_raft_amd/ops/native.py).
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3, ACT_SPLIT_TANH_RELU = 4 };

JR_DEVICE float apply_act(float v, int act, int c, int split) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.0f);
    case ACT_SIGMOID: return sigmoidf_(v);
    case ACT_TANH: return tanhf_(v);
    case ACT_SPLIT_TANH_RELU: return c < split ? tanhf_(v) : fmaxf(v, 0.0f);
    default: return v;
  }
}

#define HIP_LAUNCH_CHECK() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
