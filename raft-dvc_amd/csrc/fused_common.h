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

// 16-bit operand policy of the MFMA on-the-fly kernels: bf16, or fp16 -- the reference's CorrBlockOnTheFly under
// its Trainer's autocast runs the einsum in fp16 (corr_otf.py:198-237, trainer.py:249-257).  The window dots are
// rounded to E exactly as the materialised build rounds its E pyramid (build_gemm.hip Mma16<E>: the same
// f32x2 -> E x 2 conversion), so the on-the-fly lookup equals the materialised E path.
template <typename E> struct E16;
template <> struct E16<bf16_t> {
    static __device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ unsigned pack2(f32x2 v) {
        return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
    }
    static __device__ __forceinline__ float lo(unsigned w) { return __uint_as_float(w << 16); }
    static __device__ __forceinline__ float hi(unsigned w) { return __uint_as_float(w & 0xffff0000u); }
};
template <> struct E16<f16_t> {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ unsigned pack2(f32x2 v) {
        return __builtin_bit_cast(unsigned, __builtin_convertvector(v, h2));
    }
    static __device__ __forceinline__ float lo(unsigned w) { return bits16_to_f32<f16_t>(w); }
    static __device__ __forceinline__ float hi(unsigned w) { return bits16_to_f32<f16_t>(w >> 16); }
};

// The box group each XCD runs at once in the on-the-fly box kernels (k_fused_box, k_fused_box_f32): 32 boxes (one per
// CU of an XCD) as 8 x 4 x 1 boxes of 2 x 2 x 16 queries = a 16 x 8 x 16 query block, whose level-0 union of windows
// is ~11 % smaller than the 4 x 4 x 2 group's (8 x 8 x 32 queries).  Round 6 A/B at config #5 (gpurun_out/r6l):
// bf16 10.70 / 10.68 -> 10.38 / 10.32 ms per lookup; fp32 unchanged.  Kernels and host grids share these.
constexpr int kBoxGY = 8, kBoxGX = 4, kBoxGZ = 1;

template <int n> struct BRun {
    f32x2 p[n / 2];
    float t;
};

}  // namespace dvc
