/*
 * corr_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of RAFT-DVC's correlation hot path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg to check the HIP
 * kernels.  Nothing under raft-dvc_amd/ may link, load or call this file.
 *
 * What it restates (reference = zachtong/RAFT-DVC, paths relative to it):
 *   - all-pairs correlation       src/core/corr.py:141-167  (matmul, / sqrt(C))
 *   - 2x2x2 avg-pool pyramid      src/core/corr.py:132-139  (F.avg_pool3d, floor)
 *   - radius-r trilinear lookup    src/core/corr.py:169-208  (delta meshgrid 'ij',
 *                                  centroid / 2**i, cat over levels)
 *   - bilinear_sampler_3d          src/core/corr.py:17-68    (normalise by (S-1),
 *                                  [1,0,2] / legacy [2,0,1] grid channel order,
 *                                  grid_sample bilinear, zeros, align_corners)
 *
 * Numerics: dot products, pooling and the interpolation sum are carried in
 * float64 ("exact" side of the comparison).  The sampling-coordinate
 * arithmetic (normalise -> grid_sample unnormalise -> floor -> corner
 * weights) is carried in float32 exactly as the reference does it, because
 * that arithmetic decides which corners are used; it was verified bit-exact
 * against torch.nn.functional.grid_sample (CPU, 3-D) while writing this file.
 *
 * Pinning: tests/test_oracle_golden.py checks this oracle against golden
 * vectors produced by importing the reference (tests/golden/gen_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_MAXL 16

/* Level dims: avg_pool3d(k=2,s=2) floors each axis (corr.py:138).  Pooling an
 * axis of size < 2 raises in the reference ("Output size is too small"):
 * return -1 for that case. */
int oracle_levels(int H, int W, int D, int L, int *dims)
{
    if (L < 1 || L > OR_MAXL || H < 1 || W < 1 || D < 1) return -1;
    int h = H, w = W, d = D;
    for (int l = 0; l < L; ++l) {
        if (l > 0) {
            if (h < 2 || w < 2 || d < 2) return -1;
            h /= 2; w /= 2; d /= 2;
        }
        dims[3 * l + 0] = h; dims[3 * l + 1] = w; dims[3 * l + 2] = d;
    }
    return 0;
}

long long oracle_pyr_elems(int H, int W, int D, int L)
{
    int dims[3 * OR_MAXL];
    if (oracle_levels(H, W, D, L, dims)) return -1;
    long long s = 0;
    for (int l = 0; l < L; ++l) s += (long long)dims[3 * l] * dims[3 * l + 1] * dims[3 * l + 2];
    return s;
}

/* Correlation pyramid rows (natural layout per level, levels concatenated).
 * rows[] are global query indices g = b*N + q, q = (h*W + w)*D + d.
 * out[nrows][Ptot] (double).  corr.py:155-167 then :136-139. */
int oracle_corr_rows(const float *f1, const float *f2, int B, int C, int H, int W, int D, int L,
                     const long long *rows, long long nrows, double *out)
{
    int dims[3 * OR_MAXL];
    if (oracle_levels(H, W, D, L, dims) || B < 1 || C < 1) return -1;
    const long long N = (long long)H * W * D;
    const long long Ptot = oracle_pyr_elems(H, W, D, L);
    const double inv = 1.0 / sqrt((double)C);
#pragma omp parallel for schedule(dynamic, 1)
    for (long long r = 0; r < nrows; ++r) {
        const long long g = rows[r];
        const long long b = g / N, q = g % N;
        double *o = out + r * Ptot;
        /* level 0: dot products over channels */
        double *acc = o;
        for (long long p = 0; p < N; ++p) acc[p] = 0.0;
        for (int c = 0; c < C; ++c) {
            const double a = (double)f1[(b * C + c) * N + q];
            const float *row2 = f2 + (b * C + c) * N;
            for (long long p = 0; p < N; ++p) acc[p] += a * (double)row2[p];
        }
        for (long long p = 0; p < N; ++p) acc[p] *= inv;
        /* pooled levels: mean over 2x2x2 of the previous level */
        long long off = 0;
        for (int l = 1; l < L; ++l) {
            const int h0 = dims[3 * (l - 1)], w0 = dims[3 * (l - 1) + 1], d0 = dims[3 * (l - 1) + 2];
            const int h1 = dims[3 * l], w1 = dims[3 * l + 1], d1 = dims[3 * l + 2];
            const double *src = o + off;
            double *dst = o + off + (long long)h0 * w0 * d0;
            for (int y = 0; y < h1; ++y)
                for (int x = 0; x < w1; ++x)
                    for (int z = 0; z < d1; ++z) {
                        double s = 0.0;
                        for (int dy = 0; dy < 2; ++dy)
                            for (int dx = 0; dx < 2; ++dx)
                                for (int dz = 0; dz < 2; ++dz)
                                    s += src[((long long)(2 * y + dy) * w0 + (2 * x + dx)) * d0 + (2 * z + dz)];
                        dst[((long long)y * w1 + x) * d1 + z] = s / 8.0;
                    }
            off += (long long)h0 * w0 * d0;
        }
    }
    return 0;
}

/* ---- float32 sampling-coordinate model (corr.py:41-63 + grid_sample CPU) --- */
static float norm_f32(float x, int S)    /* 2.0 * x / (S - 1) - 1.0, fp32 ops */
{
    volatile float t = 2.0f * x;
    volatile float u = t / (float)(S - 1);
    return u - 1.0f;
}
static float unnorm_f32(float g, int S)  /* ((g + 1) / 2) * (S - 1), fp32 ops */
{
    volatile float t = g + 1.0f;
    volatile float u = t / 2.0f;
    return u * (float)(S - 1);
}

/* One trilinear sample of a (Hv, Wv, Dv) double volume at grid_sample
 * unnormalised source indices (ix: W axis, iy: H axis, iz: D axis).
 * Weights in fp32 exactly as grid_sample, sum in double. */
static double tri_sample_d(const double *v, int Hv, int Wv, int Dv, float ix, float iy, float iz)
{
    if (!(ix == ix) || !(iy == iy) || !(iz == iz)) return 0.0;     /* NaN -> no corner in bounds */
    if (fabsf(ix) > 1e9f || fabsf(iy) > 1e9f || fabsf(iz) > 1e9f) return 0.0;
    const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
    const long long x0 = (long long)fx, y0 = (long long)fy, z0 = (long long)fz;
    volatile float wx1 = ix - fx, wx0 = (fx + 1.0f) - ix;
    volatile float wy1 = iy - fy, wy0 = (fy + 1.0f) - iy;
    volatile float wz1 = iz - fz, wz0 = (fz + 1.0f) - iz;
    const float wxs[2] = {wx0, wx1}, wys[2] = {wy0, wy1}, wzs[2] = {wz0, wz1};
    double acc = 0.0;
    /* grid_sample order: tnw tne tsw tse bnw bne bsw bse  (x fastest, then y, then z) */
    for (int cz = 0; cz < 2; ++cz)
        for (int cy = 0; cy < 2; ++cy)
            for (int cx = 0; cx < 2; ++cx) {
                const long long x = x0 + cx, y = y0 + cy, z = z0 + cz;
                if (x < 0 || x >= Wv || y < 0 || y >= Hv || z < 0 || z >= Dv) continue;
                volatile float wxy = wxs[cx] * wys[cy];
                volatile float w = wxy * wzs[cz];
                acc += v[(y * Wv + x) * Dv + z] * (double)w;
            }
    return acc;
}

/* Sampling indices for bilinear_sampler_3d at position (ph, pw, pd) of a
 * (Hv, Wv, Dv) volume.  Fixed convention: grid channels [1,0,2]; legacy:
 * [2,0,1] (corr.py:49-52). */
static void sample_indices(float ph, float pw, float pd, int Hv, int Wv, int Dv, int legacy,
                           float *ix, float *iy, float *iz)
{
    const float gh = norm_f32(ph, Hv), gw = norm_f32(pw, Wv), gd = norm_f32(pd, Dv);
    float gx, gy, gz;
    if (legacy) { gx = gd; gy = gh; gz = gw; }
    else        { gx = gw; gy = gh; gz = gd; }
    *ix = unnorm_f32(gx, Wv);
    *iy = unnorm_f32(gy, Hv);
    *iz = unnorm_f32(gz, Dv);
}

/* Lookup for selected query rows.  pyr: [nrows][Ptot] natural-layout
 * pyramid rows (from oracle_corr_rows); rows[]: their global query indices;
 * coords: (B, 3, H, W, D) float32.  out: [nrows][L*(2r+1)^3] double, channel
 * = l*n^3 + a*n^2 + b*n + e (corr.py:188-208). */
int oracle_lookup_rows(const double *pyr, const long long *rows, long long nrows, const float *coords,
                       int B, int H, int W, int D, int L, int r, int legacy, double *out)
{
    int dims[3 * OR_MAXL];
    if (oracle_levels(H, W, D, L, dims) || r < 0) return -1;
    (void)B;
    const long long N = (long long)H * W * D;
    const long long Ptot = oracle_pyr_elems(H, W, D, L);
    const int n = 2 * r + 1, n3 = n * n * n;
#pragma omp parallel for schedule(dynamic, 4)
    for (long long ri = 0; ri < nrows; ++ri) {
        const long long g = rows[ri], b = g / N, q = g % N;
        const float cy = coords[(b * 3 + 0) * N + q];
        const float cx = coords[(b * 3 + 1) * N + q];
        const float cz = coords[(b * 3 + 2) * N + q];
        long long off = 0;
        for (int l = 0; l < L; ++l) {
            const int Hl = dims[3 * l], Wl = dims[3 * l + 1], Dl = dims[3 * l + 2];
            const double *v = pyr + ri * Ptot + off;
            double *o = out + ri * (long long)L * n3 + (long long)l * n3;
            const float s = (float)(1 << l);
            volatile float py = cy / s, px = cx / s, pz = cz / s;    /* coords / 2**i */
            for (int a = 0; a < n; ++a)
                for (int bb = 0; bb < n; ++bb)
                    for (int e = 0; e < n; ++e) {
                        double val = 0.0;
                        if (Hl > 1 && Wl > 1 && Dl > 1) {   /* size-1 axis: 0/0 or x/0 -> all corners OOB */
                            volatile float ph = py + (float)(a - r);
                            volatile float pw = px + (float)(bb - r);
                            volatile float pd = pz + (float)(e - r);
                            float ix, iy, iz;
                            sample_indices(ph, pw, pd, Hl, Wl, Dl, legacy, &ix, &iy, &iz);
                            val = tri_sample_d(v, Hl, Wl, Dl, ix, iy, iz);
                        }
                        o[(a * n + bb) * n + e] = val;
                    }
            off += (long long)Hl * Wl * Dl;
        }
    }
    return 0;
}

/* bilinear_sampler_3d (corr.py:17-68): vol (B, C, Hv, Wv, Dv) float32,
 * pts (B, Hq, Wq, Dq, 3) float32 in (h, w, d) order -> out (B, C, Hq, Wq, Dq). */
int oracle_sample(const float *vol, int B, int C, int Hv, int Wv, int Dv, const float *pts, int Hq, int Wq,
                  int Dq, int legacy, double *out)
{
    const long long Nv = (long long)Hv * Wv * Dv, Nq = (long long)Hq * Wq * Dq;
    double *tmp = (double *)malloc(sizeof(double) * Nv);
    if (!tmp) return -1;
    for (int b = 0; b < B; ++b)
        for (int c = 0; c < C; ++c) {
            const float *src = vol + ((long long)b * C + c) * Nv;
            for (long long i = 0; i < Nv; ++i) tmp[i] = src[i];
            for (long long k = 0; k < Nq; ++k) {
                const float *p = pts + ((long long)b * Nq + k) * 3;
                double val = 0.0;
                if (Hv > 1 && Wv > 1 && Dv > 1) {
                    float ix, iy, iz;
                    sample_indices(p[0], p[1], p[2], Hv, Wv, Dv, legacy, &ix, &iy, &iz);
                    val = tri_sample_d(tmp, Hv, Wv, Dv, ix, iy, iz);
                }
                out[((long long)b * C + c) * Nq + k] = val;
            }
        }
    free(tmp);
    return 0;
}
