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
    // src is rounded to float before the weight is taken, as the reference's upsample kernel
    // does; without this clang may fuse ratio * o - i0 into one fma in some inlined call sites
    // and not in others, and the two k_upflow forms would differ in the last bits.
#pragma clang fp contract(off)
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

constexpr int kZRun = 5;     // low-res z values covering 4 consecutive outputs when upsampling (ratio <= 1)

__device__ __forceinline__ float pick5(const float (&v)[kZRun], int j) {
    return j == 0 ? v[0] : (j == 1 ? v[1] : (j == 2 ? v[2] : (j == 3 ? v[3] : v[4])));
}

// Row cache of the z-run path: T[k] = the x- and z-interpolated value of low-res row y
// for this lane's 4 outputs -- exactly acc_y[ty] of upflow_value, so the rounding is
// identical; each low-res (y, x) row is gathered once (kZRun values) per lane and row.
// load(x, j) returns the low-res value at (y, x, min(zlo + j, last z)) -- clamped entries
// are never picked.
template <class Load>
__device__ __forceinline__ void upflow_row_from(Load load, int zlo, const AxisW &ax, const AxisW (&az)[4],
                                                float (&T)[4]) {
    float acc_x[2][4];
#pragma unroll
    for (int tx = 0; tx < 2; ++tx) {
        const int x = tx ? ax.i1 : ax.i0;
        float v[kZRun];
#pragma unroll
        for (int j = 0; j < kZRun; ++j) v[j] = load(x, j);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            acc_x[tx][k] = __builtin_fmaf(az[k].l1, pick5(v, az[k].i1 - zlo), az[k].l0 * pick5(v, az[k].i0 - zlo));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) T[k] = __builtin_fmaf(ax.l1, acc_x[1][k], ax.l0 * acc_x[0][k]);
}

template <bool DELTA, bool SUBGRID>
__device__ __forceinline__ void upflow_row(const float *__restrict__ lo, const float *__restrict__ delta,
                                           long long base, int c, int y, int w, int d, int zlo, const AxisW &ax,
                                           const AxisW (&az)[4], float (&T)[4]) {
    upflow_row_from(
        [&](int x, int j) {
            const int zz = min(zlo + j, d - 1);
            return lo_value<DELTA, SUBGRID>(lo, delta, base + ((long long)y * w + x) * d + zz, c, y, x, zz);
        },
        zlo, ax, az, T);
}

// Row-cache walk over output rows y0 .. ylast for one lane's 4 outputs: row(y, T) fills T
// for low-res row y; emit(oy, v) stores the 4 outputs of row oy.
template <class Row, class Emit>
__device__ __forceinline__ void upflow_rows_cached(Row row, Emit emit, int y0, int ylast, int h, float rh,
                                                   float scale) {
    int cy0 = -1, cy1 = -1;
    float T0[4], T1[4];
    for (int oy = y0; oy <= ylast; ++oy) {
        const AxisW ay = axis_weights(oy, h, rh);
        if (ay.i0 != cy0) {
            if (ay.i0 == cy1) {
#pragma unroll
                for (int k = 0; k < 4; ++k) T0[k] = T1[k];
            } else {
                row(ay.i0, T0);
            }
            cy0 = ay.i0;
        }
        if (ay.i1 != cy1) {
            if (ay.i1 == cy0) {
#pragma unroll
                for (int k = 0; k < 4; ++k) T1[k] = T0[k];
            } else {
                row(ay.i1, T1);
            }
            cy1 = ay.i1;
        }
        float4 v;
        v.x = __builtin_fmaf(ay.l1, T1[0], ay.l0 * T0[0]) * scale;
        v.y = __builtin_fmaf(ay.l1, T1[1], ay.l0 * T0[1]) * scale;
        v.z = __builtin_fmaf(ay.l1, T1[2], ay.l0 * T0[2]) * scale;
        v.w = __builtin_fmaf(ay.l1, T1[3], ay.l0 * T0[3]) * scale;
        emit(oy, v);
    }
}

// up (B, C, H, W, D) = upflow_3d(lo (+ delta) (- coords0)); channels 0..2 scaled.
// lo_out (nullable) receives lo + delta at low resolution (the updated coords1).
// Grid: x = chunks of one output (W, D) plane (256 lanes x VEC consecutive z),
// y = groups of `rows` output rows, z = b*C + c; the h-axis weights and the channel
// are uniform per workgroup, lanes store VEC consecutive z (16-byte stores for VEC 4,
// D % 4 == 0), and each workgroup covers `rows` consecutive rows (dvc_set_tuning "upflow_rows").
template <bool DELTA, bool SUBGRID, int VEC>
__device__ __forceinline__ void upflow_item(const float *__restrict__ lo, const float *__restrict__ delta,
                                            float *__restrict__ up, int bc, int xc, int y0, int rows, int C, int h,
                                            int w, int d, int H, int W, int D, float rh, float rw, float rd, float sh,
                                            float sw, float sd) {
    const int c = bc % C;
    const int p = (xc * (int)blockDim.x + (int)threadIdx.x) * VEC;   // first z of this lane's VEC outputs
    if (p >= W * D) return;
    const int ox = p / D, oz0 = p - ox * D;
    const float scale = c == 0 ? sh : (c == 1 ? sw : (c == 2 ? sd : 1.0f));
    const AxisW ax = axis_weights(ox, w, rw);
    AxisW az[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) az[k] = axis_weights(oz0 + k, d, rd);
    const long long base = (long long)bc * h * w * d;
    const long long plane = (long long)W * D;
    // upsampling in z: z-run loads + low-res row cache (per-lane guard: the run must cover every corner)
    if (VEC == 4 && rd <= 1.0f && az[VEC - 1].i1 - az[0].i0 < kZRun) {
        const AxisW (&az4)[4] = *reinterpret_cast<const AxisW(*)[4]>(&az[0]);
        const int zlo = az[0].i0;
        upflow_rows_cached(
            [&](int y, float (&T)[4]) { upflow_row<DELTA, SUBGRID>(lo, delta, base, c, y, w, d, zlo, ax, az4, T); },
            [&](int oy, const float4 &v) {
                *reinterpret_cast<float4 *>(up + ((long long)bc * H + oy) * plane + p) = v;
            },
            y0, min(y0 + rows, H) - 1, h, rh, scale);
        return;
    }
    for (int oy = y0; oy < y0 + rows && oy < H; ++oy) {
        const AxisW ay = axis_weights(oy, h, rh);
        float *dst = up + ((long long)bc * H + oy) * plane + p;
        if (VEC == 4) {   // downsampling in z (rare): one value at a time keeps the register count of the z-run path
#pragma unroll 1
            for (int k = 0; k < VEC; ++k)   // weights recomputed: indexing az[k] would go through scratch
                dst[k] = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax,
                                                      axis_weights(oz0 + k, d, rd), scale);
        } else {
            dst[0] = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, az[0], scale);
        }
    }
}

// up (B, C, H, W, D) = upflow_3d(lo (+ delta) (- coords0)); channels 0..2 scaled.
// lo_out (nullable) receives lo + delta at low resolution (the updated coords1).
// Work items: (chunk of one output (W, D) plane = 256 lanes x VEC consecutive z,
// group of `rows` output rows, b*C + c), chunk fastest; a grid of ~1-2 K
// workgroups strides over them (the workgroup dispatcher, not HBM, limits a
// one-item-per-workgroup grid here: 6 K groups took 47 us, 768 took 15 us).  The
// h-axis weights and the channel are uniform per item, lanes store VEC
// consecutive z (16-byte stores for VEC 4, D % 4 == 0).
// lo_out = lo (+ delta) (the updated coords1), spread over the whole grid.  16-byte
// accesses, two per lane in flight per pass: at the #5 tail (6.3 M values, 3 K workgroups)
// the scalar loop took 8 dependent load->store passes per lane ahead of the item.
template <bool DELTA>
__device__ __forceinline__ void upflow_lo_out(const float *__restrict__ lo, const float *__restrict__ delta,
                                              float *__restrict__ lo_out, long long total) {
    const long long nthr = (long long)gridDim.x * blockDim.x;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long done = 0;
    if ((((uintptr_t)lo | (uintptr_t)lo_out | (DELTA ? (uintptr_t)delta : 0)) & 15) == 0) {
        const long long n4 = total / 4;
        const float4 *l4 = reinterpret_cast<const float4 *>(lo);
        const float4 *d4 = reinterpret_cast<const float4 *>(delta);
        float4 *o4 = reinterpret_cast<float4 *>(lo_out);
        for (long long i = tid; i < n4; i += 2 * nthr) {
            const bool two = i + nthr < n4;
            float4 a = l4[i], b = two ? l4[i + nthr] : a;
            if (DELTA) {
                const float4 da = d4[i], db = two ? d4[i + nthr] : da;
                a = make_float4(a.x + da.x, a.y + da.y, a.z + da.z, a.w + da.w);
                b = make_float4(b.x + db.x, b.y + db.y, b.z + db.z, b.w + db.w);
            }
            o4[i] = a;
            if (two) o4[i + nthr] = b;
        }
        done = n4 * 4;
    }
    for (long long i = done + tid; i < total; i += nthr) lo_out[i] = DELTA ? lo[i] + delta[i] : lo[i];
}

constexpr int kStageCap = 8192;   // floats of the staged low-res box (32 KB of LDS)

// Lean per-output form of one VEC-4 item (the staged kernel's fallback when a box exceeds the
// tile -- the host picks the staged kernel only where its bound says every box fits, so this
// is for float edge cases): one value at a time keeps the staged kernel's register count.
template <bool DELTA, bool SUBGRID>
__device__ __forceinline__ void upflow_item_generic(const float *__restrict__ lo, const float *__restrict__ delta,
                                                    float *__restrict__ up, int bc, int xc, int y0, int rows, int C,
                                                    int h, int w, int d, int H, int W, int D, float rh, float rw,
                                                    float rd, float sh, float sw, float sd) {
    const int c = bc % C;
    const int p = (xc * (int)blockDim.x + (int)threadIdx.x) * 4;
    if (p >= W * D) return;
    const int ox = p / D, oz0 = p - ox * D;
    const float scale = c == 0 ? sh : (c == 1 ? sw : (c == 2 ? sd : 1.0f));
    const AxisW ax = axis_weights(ox, w, rw);
    const long long base = (long long)bc * h * w * d;
    for (int oy = y0; oy < y0 + rows && oy < H; ++oy) {
        const AxisW ay = axis_weights(oy, h, rh);
        float *dst = up + ((long long)bc * H + oy) * (long long)W * D + p;
#pragma unroll 1
        for (int k = 0; k < 4; ++k)
            dst[k] = upflow_value<DELTA, SUBGRID>(lo, delta, base, c, w, d, ay, ax, axis_weights(oz0 + k, d, rd),
                                                  scale);
    }
}

// Staged form of one item (VEC 4, every axis upsampled): the low-res box the item's 1024
// outputs x `rows` rows read -- (y rows) x (x rows) x (z run), lo (+ delta) (- index)
// formed once per element -- is loaded with coalesced loads into LDS, then each lane runs
// the same row-cache walk as upflow_item over LDS instead of global memory (same values,
// same order: bitwise equal), reading each corner at its precomputed tile offset (no z-run
// selects; any ratio <= 1).  Returns false (nothing done) when the box exceeds the LDS
// tile; the caller then runs the direct form.  Uniform per workgroup: every lane reaches
// both barriers.
template <bool DELTA, bool SUBGRID>
__device__ __forceinline__ bool upflow_item_staged(const float *__restrict__ lo, const float *__restrict__ delta,
                                                   float *__restrict__ up, float *__restrict__ tile, int bc, int xc,
                                                   int y0, int rows, int C, int h, int w, int d, int H, int W, int D,
                                                   float rh, float rw, float rd, float sh, float sw, float sd) {
    const int WD = W * D;
    const int p0 = xc * 1024, plast = min(p0 + 1023, WD - 1);
    const int ylast = min(y0 + rows, H) - 1;
    const int oxa = p0 / D, oxb = plast / D;
    const int ix0 = axis_weights(oxa, w, rw).i0, nlx = axis_weights(oxb, w, rw).i1 - ix0 + 1;
    int iz0 = 0, nlz = d;
    if (oxa == oxb) {
        iz0 = axis_weights(p0 - oxa * D, d, rd).i0;
        nlz = axis_weights(plast - oxa * D, d, rd).i1 - iz0 + 1;
    }
    const int iy0 = axis_weights(y0, h, rh).i0, nly = axis_weights(ylast, h, rh).i1 - iy0 + 1;
    const int nrow = nly * nlx;
    if ((long long)nrow * nlz > kStageCap) return false;
    const int c = bc % C;
    const long long base = (long long)bc * h * w * d;
    // stage: element e = (row, zz), rows (yy, xx) x-fastest; lanes step 256 elements at a time
    {
        const int sr = 256 / nlz, sz = 256 - sr * nlz;
        int zz = (int)threadIdx.x % nlz, rr = (int)threadIdx.x / nlz;
        int yy = rr / nlx, xx = rr - yy * nlx;
        for (int e = (int)threadIdx.x; e < nrow * nlz; e += 256) {
            const int y = iy0 + yy, x = ix0 + xx, z = iz0 + zz;
            tile[e] = lo_value<DELTA, SUBGRID>(lo, delta, base + ((long long)y * w + x) * d + z, c, y, x, z);
            zz += sz;
            xx += sr;
            if (zz >= nlz) {
                zz -= nlz;
                ++xx;
            }
            while (xx >= nlx) {
                xx -= nlx;
                ++yy;
            }
        }
    }
    __syncthreads();
    const int p = p0 + (int)threadIdx.x * 4;
    if (p < WD) {
        const int ox = p / D, oz0 = p - ox * D;
        const float scale = c == 0 ? sh : (c == 1 ? sw : (c == 2 ? sd : 1.0f));
        const AxisW ax = axis_weights(ox, w, rw);
        AxisW az[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) az[k] = axis_weights(oz0 + k, d, rd);
        // tile offsets of the 2 x 4 x 2 corners this lane reads from every staged y row (invariant)
        int off[2][4][2];
#pragma unroll
        for (int tx = 0; tx < 2; ++tx) {
            const int xo = ((tx ? ax.i1 : ax.i0) - ix0) * nlz - iz0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                off[tx][k][0] = xo + az[k].i0;
                off[tx][k][1] = xo + az[k].i1;
            }
        }
        const int ystride = nlx * nlz;
        const long long plane = (long long)WD;
        upflow_rows_cached(
            [&](int y, float (&T)[4]) {   // = upflow_row's T: the same corner values, the same fma order
                const float *trow = tile + (y - iy0) * ystride;
                float acc_x[2][4];
#pragma unroll
                for (int tx = 0; tx < 2; ++tx)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        acc_x[tx][k] =
                            __builtin_fmaf(az[k].l1, trow[off[tx][k][1]], az[k].l0 * trow[off[tx][k][0]]);
#pragma unroll
                for (int k = 0; k < 4; ++k) T[k] = __builtin_fmaf(ax.l1, acc_x[1][k], ax.l0 * acc_x[0][k]);
            },
            [&](int oy, const float4 &v) {
                *reinterpret_cast<float4 *>(up + ((long long)bc * H + oy) * plane + p) = v;
            },
            y0, ylast, h, rh, scale);
    }
    __syncthreads();   // the next item restages the tile
    return true;
}

// up (B, C, H, W, D) = upflow_3d(lo (+ delta) (- coords0)); channels 0..2 scaled.
// lo_out (nullable) receives lo + delta at low resolution (the updated coords1).
// Work items: (chunk of one output (W, D) plane = 256 lanes x VEC consecutive z,
// group of `rows` output rows, b*C + c), chunk fastest; by default one workgroup per
// item (dvc_set_tuning "upflow_wgs" caps the grid, which then strides over the items).
// The h-axis weights and the channel are uniform per item, lanes store VEC consecutive z
// (16-byte stores for VEC 4, D % 4 == 0).  STAGED (VEC 4, all ratios <= 1): the item's
// low-res box goes through LDS (upflow_item_staged) instead of per-lane global gathers.
template <bool DELTA, bool SUBGRID, int VEC, bool STAGED>
__global__ __launch_bounds__(256) void k_upflow(const float *__restrict__ lo, const float *__restrict__ delta,
                                                float *__restrict__ lo_out, float *__restrict__ up, long long B, int C,
                                                int h, int w, int d, int H, int W, int D, float rh, float rw, float rd,
                                                float sh, float sw, float sd, int nx, int ny, int rows) {
    if (lo_out != nullptr) upflow_lo_out<DELTA>(lo, delta, lo_out, B * C * (long long)h * w * d);
    __shared__ float tile[STAGED ? kStageCap : 1];
    const long long nitems = (long long)nx * ny * B * C;
    for (long long it = blockIdx.x; it < nitems; it += gridDim.x) {
        const int xc = (int)(it % nx);
        const long long r = it / nx;
        const int yg = (int)(r % ny);
        const int bc = (int)(r / ny);
        if constexpr (STAGED) {
            if (!upflow_item_staged<DELTA, SUBGRID>(lo, delta, up, tile, bc, xc, yg * rows, rows, C, h, w, d, H, W, D,
                                                    rh, rw, rd, sh, sw, sd))
                upflow_item_generic<DELTA, SUBGRID>(lo, delta, up, bc, xc, yg * rows, rows, C, h, w, d, H, W, D, rh, rw,
                                                    rd, sh, sw, sd);
        } else {
            upflow_item<DELTA, SUBGRID, VEC>(lo, delta, up, bc, xc, yg * rows, rows, C, h, w, d, H, W, D, rh, rw, rd,
                                             sh, sw, sd);
        }
    }
}

#define DVC_UPFLOW_INST(DL, SG, V, ST)                                                                          \
    template __global__ void k_upflow<DL, SG, V, ST>(const float *, const float *, float *, float *, long long, int, \
        int, int, int, int, int, int, float, float, float, float, float, float, int, int, int);
DVC_UPFLOW_INST(false, false, 1, false)
DVC_UPFLOW_INST(false, true, 1, false)
DVC_UPFLOW_INST(true, true, 1, false)
DVC_UPFLOW_INST(false, false, 4, false)
DVC_UPFLOW_INST(false, true, 4, false)
DVC_UPFLOW_INST(true, true, 4, false)
DVC_UPFLOW_INST(false, false, 4, true)
DVC_UPFLOW_INST(false, true, 4, true)
DVC_UPFLOW_INST(true, true, 4, true)
#undef DVC_UPFLOW_INST

}  // namespace dvc
