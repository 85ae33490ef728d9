// flow.hip -- the per-iteration flow bookkeeping around the correlation lookup
// (SURVEY §8(f) row 4):
//   k_coords_grid   coords_grid_3d                         src/core/corr.py:71-99
//   k_upflow        upflow_3d(flow, target_shape)          src/core/corr.py:211-253
//                   fused with RAFTDVC.forward's coords update and flow
//                   difference: coords1 += delta_flow; upflow_3d(coords1 - coords0)
//                                                          src/core/raft_dvc.py:482-485
//
// All HBM-bound elementwise work; the upsampled flow (B, 3, H, W, D) float32 is
// the only large stream (25 MB at a 128^3 input), written once with one dword per
// lane over consecutive z (256-byte segments per wave).  The low-resolution input
// (<= 0.4 MB at 32^3) stays in L2 for the 8-corner gathers.
//
// Trilinear weights follow ATen's CPU upsample_trilinear3d with align_corners=True:
// ratio = float(in - 1) / (out - 1) (0 when out == 1), src = ratio * o, i0 = trunc(src),
// i1 = i0 + (i0 < in - 1), l1 = clamp(src - i0, 0, 1), l0 = 1 - l1; the value is nested
// h-outer: l0h*(l0w*(l0d*v000 + l1d*v001) + l1w*(..)) + l1h*(..), then channel c < 3 is
// multiplied by float(target/in) along its axis (corr.py:242-251).  Each pair is one
// explicit fma(l1, v1, l0 * v0), so every template instance rounds identically.  The coords0 grid
// is the identity (corr.py:91-97), so coords1 - coords0 is formed on the fly and the
// flow difference is never materialised.
#include "common.h"

namespace dvc {

struct AxisW {
    int i0, i1;
    float l0, l1;
};

__device__ __forceinline__ AxisW axis_weights(int o, int in, float ratio) {
    const float src = ratio * (float)o;
    AxisW a;
    a.i0 = (int)src;
    a.i1 = a.i0 + (a.i0 < in - 1 ? 1 : 0);
    a.l1 = fminf(fmaxf(src - (float)a.i0, 0.0f), 1.0f);
    a.l0 = 1.0f - a.l1;
    return a;
}

// out (B, 3, H, W, D): channel c holds the index along axis c.
__global__ __launch_bounds__(256) void k_coords_grid(float *__restrict__ out, long long B, int H, int W, int D) {
    const long long vox = (long long)H * W * D;
    const long long total = B * 3 * vox;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long v = i % vox;
        const int c = (int)((i / vox) % 3);
        const int z = (int)(v % D);
        const int x = (int)((v / D) % W);
        const int y = (int)(v / ((long long)W * D));
        out[i] = (float)(c == 0 ? y : (c == 1 ? x : z));
    }
}

// Low-resolution value of channel c at (y, x, z): lo (+ delta) (- index on axis c).
template <bool DELTA, bool SUBGRID>
__device__ __forceinline__ float lo_value(const float *__restrict__ lo, const float *__restrict__ delta, long long idx,
                                          int c, int y, int x, int z) {
    float v = lo[idx];
    if (DELTA) v = v + delta[idx];
    if (SUBGRID) v = v - (float)(c == 0 ? y : (c == 1 ? x : z));
    return v;
}

// One output value: trilinear over the 8 low-resolution corners, then the axis scale.
template <bool DELTA, bool SUBGRID>
__device__ __forceinline__ float upflow_value(const float *__restrict__ lo, const float *__restrict__ delta,
                                              long long base, int c, int w, int d, const AxisW &ay, const AxisW &ax,
                                              const AxisW &az, float scale) {
    float acc_y[2];
#pragma unroll
    for (int ty = 0; ty < 2; ++ty) {
        const int y = ty ? ay.i1 : ay.i0;
        float acc_x[2];
#pragma unroll
        for (int tx = 0; tx < 2; ++tx) {
            const int x = tx ? ax.i1 : ax.i0;
            const long long row = base + ((long long)y * w + x) * d;
            const float v0 = lo_value<DELTA, SUBGRID>(lo, delta, row + az.i0, c, y, x, az.i0);
            const float v1 = lo_value<DELTA, SUBGRID>(lo, delta, row + az.i1, c, y, x, az.i1);
            acc_x[tx] = __builtin_fmaf(az.l1, v1, az.l0 * v0);   // pinned: identical in every instance
        }
        acc_y[ty] = __builtin_fmaf(ax.l1, acc_x[1], ax.l0 * acc_x[0]);
    }
    return __builtin_fmaf(ay.l1, acc_y[1], ay.l0 * acc_y[0]) * scale;
}

constexpr int kUpRows = 4;   // output rows (oy) per workgroup

// up (B, C, H, W, D) = upflow_3d(lo (+ delta) (- coords0)); channels 0..2 scaled.
// lo_out (nullable) receives lo + delta at low resolution (the updated coords1).
// Grid: x = chunks of one output (W, D) plane (256 lanes x VEC consecutive z),
// y = groups of kUpRows output rows, z = b*C + c; the h-axis weights and the channel
// are uniform per workgroup, lanes store VEC consecutive z (16-byte stores for VEC 4,
// D % 4 == 0), and each workgroup covers kUpRows rows so the grid stays ~1-2 K groups.
template <bool DELTA, bool SUBGRID, int VEC>
__global__ __launch_bounds__(256) void k_upflow(const float *__restrict__ lo, const float *__restrict__ delta,
                                                float *__restrict__ lo_out, float *__restrict__ up, long long B, int C,
                                                int h, int w, int d, int H, int W, int D, float rh, float rw, float rd,
                                                float sh, float sw, float sd) {
    const int bc = blockIdx.z;
    const int c = bc % C;
    if (lo_out != nullptr) {   // coords1 + delta, spread over the whole grid
        const long long total_lo = B * C * (long long)h * w * d;
        const long long nthr = (long long)gridDim.x * gridDim.y * gridDim.z * blockDim.x;
        for (long long i = (((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * blockDim.x +
                           threadIdx.x;
             i < total_lo; i += nthr)
            lo_out[i] = DELTA ? lo[i] + delta[i] : lo[i];
    }
    const int p = (blockIdx.x * blockDim.x + threadIdx.x) * VEC;   // first z of this lane's VEC outputs
    if (p >= W * D) return;
    const int ox = p / D, oz0 = p - ox * D;
    const float scale = c == 0 ? sh : (c == 1 ? sw : (c == 2 ? sd : 1.0f));
    const AxisW ax = axis_weights(ox, w, rw);
    AxisW az[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) az[k] = axis_weights(oz0 + k, d, rd);
    const long long base = (long long)bc * h * w * d;
    const long long plane = (long long)W * D;
    const int y0 = blockIdx.y * kUpRows;
    for (int oy = y0; oy < y0 + kUpRows && oy < H; ++oy) {
        const AxisW ay = axis_weights(oy, h, rh);
        float *dst = up + ((long long)bc * H + oy) * plane + p;
        if (VEC == 4) {
            float4 v;
            v.x = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, az[0], scale);
            v.y = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, az[VEC > 1 ? 1 : 0], scale);
            v.z = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, az[VEC > 2 ? 2 : 0], scale);
            v.w = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, az[VEC > 3 ? 3 : 0], scale);
            *reinterpret_cast<float4 *>(dst) = v;
        } else {
            dst[0] = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, az[0], scale);
        }
    }
}

template __global__ void k_upflow<false, false, 1>(const float *, const float *, float *, float *, long long, int,
    int, int, int, int, int, int, float, float, float, float, float, float);
template __global__ void k_upflow<false, true, 1>(const float *, const float *, float *, float *, long long, int,
    int, int, int, int, int, int, float, float, float, float, float, float);
template __global__ void k_upflow<true, true, 1>(const float *, const float *, float *, float *, long long, int,
    int, int, int, int, int, int, float, float, float, float, float, float);
template __global__ void k_upflow<false, false, 4>(const float *, const float *, float *, float *, long long, int,
    int, int, int, int, int, int, float, float, float, float, float, float);
template __global__ void k_upflow<false, true, 4>(const float *, const float *, float *, float *, long long, int,
    int, int, int, int, int, int, float, float, float, float, float, float);
template __global__ void k_upflow<true, true, 4>(const float *, const float *, float *, float *, long long, int,
    int, int, int, int, int, int, float, float, float, float, float, float);

}  // namespace dvc
