// lookup_common.h -- window geometry shared by the lookup walk (lookup.hip) and the
// fused window-dot stage (fused.hip); both must derive the same window origin.
#pragma once

#include "common.h"

namespace dvc {

struct Item {
    int l, ac, b;
    long long qi;   // query index inside the launch's range [0, nq) (may be >= nq in the last wave)
};

// item = ((l * nach + ac) * B + b) * nqb + qb, one wavefront each (4 per block).
__device__ __forceinline__ bool decode_item(const LookupArgs &A, Item &it) {
    // wave-uniform by construction; readfirstlane lets the compiler keep it in SGPRs
    const long long item = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const long long bq = (long long)A.B * A.nqb;
    const long long per_l = (long long)A.nach * bq;
    if (item >= per_l * A.nl) return false;
    const int li = (int)(item / per_l);
    long long rem = item - (long long)li * per_l;
    it.l = A.l0 + li;
    it.ac = (int)(rem / bq);
    rem -= (long long)it.ac * bq;
    it.b = (int)(rem / A.nqb);
    it.qi = (rem - (long long)it.b * A.nqb) * 64 + (threadIdx.x & 63);
    return true;
}

__device__ __forceinline__ void load_coords(const float *coords, int b, long long Nq, long long q, float &cy,
                                            float &cx, float &cz) {
    const float *cb = coords + (long long)b * 3 * Nq + q;
    cy = cb[0];
    cx = cb[Nq];
    cz = cb[2 * Nq];
}

// Window axes of one query at one level.  H axis <- h coordinate; U = memory W axis,
// V = memory D axis (contiguous).  Fixed convention: U <- w coordinate, V <- d;
// legacy (grid channels [2,0,1], corr.py:49-50): U <- d coordinate, V <- w, with the
// normalise/unnormalise sizes swapped accordingly.
struct WinAxes {
    float ph, pu, pv;         // level coordinates driving H, U, V
    float kh, ku, kv;         // floor of each
    float hs, un, uu, vn, vu; // (S-1) used to normalise / unnormalise per axis
    bool dead;                // NaN / huge coordinate: every corner out of range -> 0
};

__device__ __forceinline__ void window_axes(float py, float px, float pz, int Hl, int Wl, int Dl, int legacy,
                                            WinAxes &ax) {
    ax.ph = py;
    ax.pu = legacy ? pz : px;
    ax.pv = legacy ? px : pz;
    ax.dead = !(fabsf(ax.ph) < 1e6f) || !(fabsf(ax.pu) < 1e6f) || !(fabsf(ax.pv) < 1e6f);
    if (ax.dead) { ax.ph = -1e5f; ax.pu = -1e5f; ax.pv = -1e5f; }
    ax.hs = (float)(Hl - 1);
    ax.un = legacy ? (float)(Dl - 1) : (float)(Wl - 1);
    ax.uu = (float)(Wl - 1);
    ax.vn = legacy ? (float)(Wl - 1) : (float)(Dl - 1);
    ax.vu = (float)(Dl - 1);
    ax.kh = floorf(ax.ph);
    ax.ku = floorf(ax.pu);
    ax.kv = floorf(ax.pv);
}

// Corner weights of offset d along one axis: the reference's sample index
// ix = unnorm(norm(p + d)), weights (k+1 - ix, ix - k) with k = floor(p) + d.
__device__ __forceinline__ void axis_weights(float p, float kp, int d, float sn, float su, float &w0, float &w1) {
#pragma clang fp contract(off)
    const float x = roundtrip(p + (float)d, sn, su);
    const float k = kp + (float)d;
    w1 = x - k;
    w0 = (k + 1.0f) - x;
}

// Geometry of a legacy W != D level for k_lookup_stretch (lookup.hip), from the host: WX x DX the staged box of one
// wave's chunk of W-axis samples (WX columns, DX values along D, RB bytes per staged row, LS bytes per lane's LDS
// region); WINBUF (the on-the-fly path) reads a per-query window box of NYB x WXF x DX dots (boxe floats) instead of
// the pyramid row.
constexpr int kStretchSE = 3;   // W-axis samples per k_lookup_stretch wave
struct StretchGeo {
    int WX, DX, RB, LS, NYB, WXF;
    long long boxe;
};

}  // namespace dvc
