#include "lookup_tile.h"

namespace dvc {

// fp16 instances of k_lookup_tile (lookup_tile.h): the AMP pyramid (DVC_F16); see lookup_tile.hip
#define DVC_TILE_INST(T, R)                                                      \
    template __global__ void k_lookup_tile<T, R, false, 0, false, 0>(LookupArgs); \
    template __global__ void k_lookup_tile<T, R, true, 0, false, 0>(LookupArgs);  \
    template __global__ void k_lookup_tile<T, R, true, 0, false, 2>(LookupArgs);  \
    template __global__ void k_lookup_tile<T, R, true, 0, false, 3>(LookupArgs);  \
    template __global__ void k_lookup_tile<T, R, true, 0, false, 5>(LookupArgs);
DVC_TILE_INST(f16_t, 1) DVC_TILE_INST(f16_t, 2) DVC_TILE_INST(f16_t, 3)
DVC_TILE_INST(f16_t, 4) DVC_TILE_INST(f16_t, 5) DVC_TILE_INST(f16_t, 6)
// balanced four-wave instances (tuning "lookup_waves" = 4)
template __global__ void k_lookup_tile<f16_t, 4, true, 0, false, 0, 4>(LookupArgs);
template __global__ void k_lookup_tile<f16_t, 4, true, 0, false, 5, 4>(LookupArgs);

}  // namespace dvc
