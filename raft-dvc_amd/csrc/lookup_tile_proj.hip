#include "lookup_tile.h"

namespace dvc {

// convc1-fused instances of k_lookup_tile (lookup_tile.h; radii whose (2r+1) x 3 row values fit one
// 32-k slice) and their weight packing
#define DVC_TILE_PROJ(T, R) template __global__ void k_lookup_tile<T, R, true, 0, 1, 0, 0, -1, DVC_PROJ_XLP>(LookupArgs);
// fp32 pyramids: the exact split consumer (PROJ 2, bf16 hi/lo operands, lookup_tile.h)
#define DVC_TILE_PROJX(R) template __global__ void k_lookup_tile<float, R, true, 0, 2, 0, 0, -1, DVC_PROJ_XLP>(LookupArgs);
DVC_TILE_PROJX(1) DVC_TILE_PROJX(2) DVC_TILE_PROJX(3) DVC_TILE_PROJX(4)
DVC_TILE_PROJ(bf16_t, 1) DVC_TILE_PROJ(bf16_t, 2) DVC_TILE_PROJ(bf16_t, 3) DVC_TILE_PROJ(bf16_t, 4)
DVC_TILE_PROJ(f16_t, 1) DVC_TILE_PROJ(f16_t, 2) DVC_TILE_PROJ(f16_t, 3) DVC_TILE_PROJ(f16_t, 4)

// Weight re-layout for the PROJ instances: W (96, L (2r+1)^3) fp32, the reference's
// convc1.weight viewed (96, L*(2r+1)^3) (update.py:222) -> fp16 in the consumer's
// MFMA A-operand order [l][a][wave][ot][lane][8].  Lane (m16, h4) of tile ot holds
// channel o = 16 ot + m16 at the slice positions k = 8 h4 .. 8 h4 + 7 (k order above);
// positions past the wave's values are 0.  Reference channel of (l, a, u, v):
// l (2r+1)^3 + a (2r+1)^2 + u chstep_u + v chstep_v (corr.py:188-208).
// split = 1 (dvc_proj_pack_exact, fp32 blocks): bf16 hi = bf16(w) at [idx], bf16 lo = bf16(w - hi) at [total + idx]
__global__ void k_proj_pack(const float *__restrict__ w, bf16_t *__restrict__ out, int L, int r, int legacy,
                            long long total, int split) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int n = 2 * r + 1, NP = n / 2, COLS = 3, NWV = (n + COLS - 1) / COLS, OT = ProjCfg::OT;
    const int e = (int)(idx & 7);
    long long t = idx >> 3;
    const int lane = (int)(t & 63); t >>= 6;
    const int ot = (int)(t % OT); t /= OT;
    const int w8 = (int)(t % NWV); t /= NWV;
    const int a = (int)(t % n); t /= n;
    const int l = (int)t;
    const int o = 16 * ot + (lane & 15);
    const int kk = 8 * (lane >> 4) + e;
    const int NU = w8 < NWV - 1 ? COLS : n - COLS * (NWV - 1);
    int uu = -1, v = 0;
    if (kk < 2 * NU * NP) {
        uu = kk / (2 * NP);
        v = kk % (2 * NP);
    } else if (kk < 2 * NU * NP + NU) {
        uu = kk - 2 * NU * NP;
        v = n - 1;
    }
    float val = 0.0f;
    if (uu >= 0) {
        const int u = w8 * COLS + uu;
        const long long ch = (long long)l * n * n * n + (long long)a * n * n + (legacy ? u + v * n : u * n + v);
        val = w[(long long)o * L * n * n * n + ch];
    }
    if (split) {
        const __bf16 hi = (__bf16)val;
        out[idx] = __builtin_bit_cast(bf16_t, hi);
        out[total + idx] = __builtin_bit_cast(bf16_t, (__bf16)(val - (float)hi));
        return;
    }
    out[idx] = __builtin_bit_cast(bf16_t, (_Float16)val);   // fp16 bits
}

}  // namespace dvc

