// fused_proj_r1.hip -- the r = 1 instances of k_fused_proj (fused_proj.hip), compiled without SLP vectorisation:
// with it hipcc forms one packed-FP32 add whose low lane reads the high half of a pair, the op that returned wrong
// low-lane values while another wave ran MFMAs (round 2; tools/isa_check.py).  The rest of fused_proj.hip compiles
// with SLP (round 6: 2.5 % faster at config #5).
#define DVC_FPROJ_R1_TU 1
#include "fused_proj.hip"

namespace dvc {
#define DVC_FPROJ_R1_INST(KS, E)                                                                                 \
    template __global__ void k_fused_proj<1, KS, 0, E>(const bf16_t *, const bf16_t *, LookupArgs,                \
                                                      const unsigned long long *, int, int, long long, float, float *);
DVC_FPROJ_R1_INST(1, bf16_t) DVC_FPROJ_R1_INST(2, bf16_t) DVC_FPROJ_R1_INST(4, bf16_t)
DVC_FPROJ_R1_INST(1, f16_t) DVC_FPROJ_R1_INST(2, f16_t) DVC_FPROJ_R1_INST(4, f16_t)
}  // namespace dvc
