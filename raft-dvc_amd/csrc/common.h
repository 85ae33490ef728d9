// common.h -- shared device helpers for the gfx950 correlation kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "dvccorr.h"

// DVC_DIAG = 1: the diagnostics library (libdvccorr_diag.so, `make diag`) -- ablation, timeline and store-policy
// kernel instances reachable through dvc_set_tuning, for A/B tools only (DVCCORR_LIB selects it).  The product
// library (libdvccorr.so) is built with DVC_DIAG = 0 and carries only product kernels.
#ifndef DVC_DIAG
#define DVC_DIAG 0
#endif
// 1: the convc1-fused tile lookup prefetches each next level under the current one's last row (lookup_tile.h XLP;
// round 6 A/B, gpurun_out/r6g: 0.137 ms against 0.108 without -- the prefetch's live state spills 45 VGPRs at two
// waves per SIMD and the next level's first plane waits a full latency in the last row; off)
#ifndef DVC_PROJ_XLP
#define DVC_PROJ_XLP 0
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short bf16_t;   // storage type of one bf16 value
typedef _Float16 f16_t;          // storage type of one fp16 value (the AMP pyramid, trainer.py:249-252)
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace dvc {

constexpr int kWave = 64;

// A dvc_set_tuning knob: process-global (relaxed atomic), so a value set on the caller's thread also governs the
// launches PyTorch's autograd engine makes from its own per-device worker thread (round 6; the knobs were
// thread_local before, which left a backward under loss.backward() on the defaults).
template <typename T> struct Knob {
    std::atomic<T> v;
    explicit constexpr Knob(T x) : v(x) {}
    operator T() const { return v.load(std::memory_order_relaxed); }
    Knob &operator=(T x) {
        v.store(x, std::memory_order_relaxed);
        return *this;
    }
};

// Geometry of the correlation pyramid, passed by value to kernels.
struct Geo {
    int L;
    int H[DVC_MAX_LEVELS], W[DVC_MAX_LEVELS], D[DVC_MAX_LEVELS], Dp[DVC_MAX_LEVELS];
    int zero[DVC_MAX_LEVELS];
    long long off[DVC_MAX_LEVELS];
    long long row_stride;
};

// {p, p} in two registers.  A packed-FP32 op whose low lane reads the high element of a source (op_sel
// [1, ..], the compiler's way to broadcast the high half of a pair) returned wrong low-lane values in
// lanes 48-63 now and then while another wave of the same workgroup ran MFMAs (k_fused_proj, round 2,
// found with dump instances of the kernel; tests/test_gpu_proj_fused.py::test_repeatable_under_poisoned_memory guards it).  The empty asm hides that the
// halves are equal, so no such broadcast is formed.  Used for every broadcast pair (VGPR or SGPR source) in a
// kernel that issues MFMAs; tools/isa_check.py fails the build check on any that is left.
__device__ __forceinline__ f32x2 splat2(float p) {
    f32x2 v = {p, p};
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ float bf16_bits_to_f32(unsigned int h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ bf16_t f32_to_bf16(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// 16-bit storage types (bf16_t, f16_t): two values (round to nearest even) packed into one dword, low first,
// and one value's 16 bits (low half of h) widened to float.
template <typename T> __device__ __forceinline__ unsigned pack2_16(float a, float b);
template <> __device__ __forceinline__ unsigned pack2_16<bf16_t>(float a, float b) {
    return (unsigned)f32_to_bf16(a) | ((unsigned)f32_to_bf16(b) << 16);
}
template <> __device__ __forceinline__ unsigned pack2_16<f16_t>(float a, float b) {
    return (unsigned)__builtin_bit_cast(unsigned short, (f16_t)a) |
           ((unsigned)__builtin_bit_cast(unsigned short, (f16_t)b) << 16);
}
template <typename T> __device__ __forceinline__ float bits16_to_f32(unsigned h);
template <> __device__ __forceinline__ float bits16_to_f32<bf16_t>(unsigned h) { return __uint_as_float(h << 16); }
template <> __device__ __forceinline__ float bits16_to_f32<f16_t>(unsigned h) {
    return (float)__builtin_bit_cast(f16_t, (unsigned short)(h & 0xffffu));
}

// Arguments of the lookup kernels (materialised pyramid or fused window buffer).
// A launch covers queries [q0, q0 + nq) of every batch element and levels
// [l0, l0 + nl); out/coords are indexed with the full Nq and Ltot.
struct LookupArgs {
    const void *corr;        // pyramid rows [B][Nq][row_stride], or window buffer [B][nq][NB]
    const float *coords;     // (B, 3, Nq)
    float *out;              // (B, Ltot*n^3, Nq)
    long long Nq, q0, nq, nqb, row_stride;
    int B, Ltot, l0, nl, legacy, nach, ach, r;
    int H[DVC_MAX_LEVELS], W[DVC_MAX_LEVELS], D[DVC_MAX_LEVELS], Dp[DVC_MAX_LEVELS], zero[DVC_MAX_LEVELS];
    int generic[DVC_MAX_LEVELS];   // level handled by a separate per-output launch (legacy, W != D)
    int ablate;                    // diagnostics only: 1 = skip output stores, 2 = skip run loads
    int order;                     // tile kernel: 1 = odd tiles walk the levels coarse-to-fine
    int ldpol;                     // tile kernel: cache-policy bits of the plane loads
    int split_levels;              // tile kernel: one level per workgroup (blockIdx.y), for launches whose
                                   // query tiles alone cannot fill the chip (one rank's slab)
    int brick;                     // tile kernel: bit l = level l stored in (1, 8, 8) bricks (DVC_BRICKED)
    long long off[DVC_MAX_LEVELS];
    // tile kernel with the motion encoder's convc1 fused (PROJ instances only):
    // packed bf16 weights (dvc_proj_pack), bias[96], out (B, 96, Nq)
    const void *proj_w;
    const float *proj_b;
    float *proj_out;
    unsigned long long *trace;   // diagnostics only (tile kernel ABL & 8): per-workgroup s_memrealtime stamps
};

template <typename T> struct StoreT;
template <> struct StoreT<float> {
    static __device__ __forceinline__ float load(const float *p) { return *p; }
    static __device__ __forceinline__ void store(float *p, float v) { *p = v; }
};
template <> struct StoreT<bf16_t> {
    static __device__ __forceinline__ float load(const bf16_t *p) { return bf16_bits_to_f32(*p); }
    static __device__ __forceinline__ void store(bf16_t *p, float v) { *p = f32_to_bf16(v); }
};
template <> struct StoreT<f16_t> {
    static __device__ __forceinline__ float load(const f16_t *p) { return (float)*p; }
    static __device__ __forceinline__ void store(f16_t *p, float v) { *p = (f16_t)v; }
};

// ---------------------------------------------------------------------------
// Sampling-coordinate arithmetic of the reference, in float32, no FMA
// contraction, IEEE division (reference src/core/corr.py:41-44 then
// grid_sample's align_corners unnormalise): x -> 2x/(S-1) - 1 -> ((g+1)/2)*(S'-1).
// Bit-identical to the CPU reference (checked by the oracle, see
// oracle/corr_oracle.c header).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float norm_coord(float x, float snm1) {
#pragma clang fp contract(off)
    float t = 2.0f * x;
    float u = t / snm1;
    return u - 1.0f;
}
__device__ __forceinline__ float unnorm_coord(float g, float sum1) {
#pragma clang fp contract(off)
    float t = g + 1.0f;
    float u = t / 2.0f;
    return u * sum1;
}
__device__ __forceinline__ float roundtrip(float x, float snm1, float sum1) {
    return unnorm_coord(norm_coord(x, snm1), sum1);
}

// Trilinear sample at grid_sample source indices (ix: W axis, iy: H axis,
// iz: D axis) of one level in the padded row layout; out-of-range corners
// contribute nothing (padding_mode='zeros').  Weight products and term order
// follow grid_sample (tnw, tne, tsw, tse, bnw, bne, bsw, bse).
template <typename T>
__device__ __forceinline__ float tri_sample(const T *lvl, int Hl, int Wl, int Dl, int Dpl, float ix, float iy,
                                            float iz) {
#pragma clang fp contract(off)
    if (!(fabsf(ix) < 1e7f) || !(fabsf(iy) < 1e7f) || !(fabsf(iz) < 1e7f)) return 0.0f;   // NaN/inf/huge: all OOB
    const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
    const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
    const float wx1 = ix - fx, wx0 = (fx + 1.0f) - ix;
    const float wy1 = iy - fy, wy0 = (fy + 1.0f) - iy;
    const float wz1 = iz - fz, wz0 = (fz + 1.0f) - iz;
    float acc = 0.0f;
#pragma unroll
    for (int cz = 0; cz < 2; ++cz)
#pragma unroll
        for (int cy = 0; cy < 2; ++cy)
#pragma unroll
            for (int cx = 0; cx < 2; ++cx) {
                const int x = x0 + cx, y = y0 + cy, z = z0 + cz;
                if (x < 0 || x >= Wl || y < 0 || y >= Hl || z < 0 || z >= Dl) continue;
                const float w = ((cx ? wx1 : wx0) * (cy ? wy1 : wy0)) * (cz ? wz1 : wz0);
                acc += StoreT<T>::load(lvl + ((long long)y * Wl + x) * Dpl + z) * w;
            }
    return acc;
}

// Geometry of k_pack_pyramid (pack.hip): every packed target level of fmap2 in one pass.  The source is nslab
// H-slabs of (B, C, maxh, W, D) float32, slab r holding planes [h0(r), h0(r + 1)) of the balanced split
// h0(r) = r sbase + min(r, srem) (dvccorr/sharded.py slab_bounds) zero-padded to maxh planes: an all-gather's receive
// buffer as it lands.  One slab (nslab = 1, maxh = H) is the plain (B, C, H, W, D) tensor.
struct PyrGeo {
    int L, C, Cp, H[4], W[4], D[4], Dp[4];
    long long off[4];
    long long row_stride;
    int ncx, ncy, ncz;   // cells per axis (level 0, ceil)
    int brick;           // bit l: level l in (1, 8, 8) bricks (DVC_BRICKED, include/dvccorr.h)
    int B, nslab, maxh, sbase, srem;
};

// Stream-ordered zero fill of `bytes` (a multiple of 4) by a kernel.  Round 5: a backward captured in a HIP graph
// (torch.cuda.CUDAGraph) and replayed twice returned garbage d fmap2 from the second replay on -- the zero guard
// and the cell counts its hipMemsetAsync calls clear were not cleared again (tools/graph_bwd_diag.py) -- so the
// library's clears are kernels, which every replay runs in stream order.
template <typename = void>
__global__ __launch_bounds__(256) void k_zero_dwords(unsigned *__restrict__ p, long long n) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = 0u;
}
inline hipError_t zero_async(void *p, size_t bytes, hipStream_t s) {
    const long long n = (long long)(bytes / 4);
    if (n <= 0) return hipSuccess;
    const long long blocks = std::min<long long>((n + 255) / 256, 8192);
    k_zero_dwords<><<<(unsigned)blocks, 256, 0, s>>>(reinterpret_cast<unsigned *>(p), n);
    return hipGetLastError();
}

}  // namespace dvc
