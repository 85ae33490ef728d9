// fused_common.h -- wave-uniform helpers shared by the MFMA on-the-fly kernels
// (fused_box.hip, fused_proj.hip).
#pragma once

#include "common.h"

namespace dvc {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int buni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long long buni64(long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
template <typename T> __device__ __forceinline__ T *buniptr(T *p) { return (T *)buni64((long long)p); }
__device__ __forceinline__ int bwave_min(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return buni(v);
}
__device__ __forceinline__ int bwave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return buni(v);
}

template <int n> struct BRun {
    f32x2 p[n / 2];
    float t;
};

}  // namespace dvc
