#include "lookup_tile.h"

namespace dvc {

// diagnostics-only instances of k_lookup_tile (lookup_tile.h): ablations (tuning "lookup_ablate") and the
// output-store cache-policy A/B (tuning "lookup_stpol": plain, sc1, sc0 + sc1, nt + sc1)
template __global__ void k_lookup_tile<bf16_t, 4, true, 1, false, 0>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 4, false, 0>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 2, false, 0>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 3, false, 0>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 0, false, 0, 4, 0>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 0, false, 0, 4, 16>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 0, false, 0, 4, 18>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 0, false, 0, 4, 17>(LookupArgs);
// timeline stamps (tuning "lookup_trace", dvc_lookup_trace_buffer): the default four-wave r = 4 instances
template __global__ void k_lookup_tile<bf16_t, 4, true, 8, false, 0, 4>(LookupArgs);
template __global__ void k_lookup_tile<bf16_t, 4, true, 8, false, 5, 4>(LookupArgs);
// every-level timeline stamps of the convc1-fused instance (64 per workgroup; round 6, tools/trace_proj.py)
template __global__ void k_lookup_tile<bf16_t, 4, true, 16, 1, 0, 0, -1, DVC_PROJ_XLP>(LookupArgs);

}  // namespace dvc
