"""ISA guard (CPU, cross-compiled code objects): no kernel that runs MFMAs may contain a packed-FP32 op
whose low lane reads the high element of a source register pair (VGPR or SGPR).  On gfx950 such ops
returned wrong low-lane values in lanes 48-63 now and then while another wave of the workgroup ran MFMAs
(k_fused_proj, round 2; tools/isa_check.py, splat2 in csrc/common.h).  Round 3: no exceptions -- the
SGPR-pair scale broadcasts of the build epilogues are materialised too."""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

LIB = os.path.join(ROOT, "raft-dvc_amd", "dvccorr", "libdvccorr.so")
CSRC = os.path.join(ROOT, "raft-dvc_amd", "csrc")


def test_library_is_current():
    """The guard disassembles the shipped library, so it must be built from the current sources."""
    assert os.path.exists(LIB), "libdvccorr.so missing: run __graft_entry__.build()"
    srcs = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) + \
        [os.path.join(ROOT, "include", "dvccorr.h"), os.path.join(CSRC, "Makefile")]
    stale = [os.path.basename(s) for s in srcs if os.path.getmtime(s) > os.path.getmtime(LIB)]
    assert not stale, f"libdvccorr.so is older than {stale}: rebuild before trusting the ISA guard"


def test_no_packed_fp32_opsel_beside_mfma():
    """Disassembles the shipped library's gfx950 code objects (seconds)."""
    assert os.path.exists("/opt/rocm/llvm/bin/llvm-objdump"), "llvm-objdump is part of the ROCm image"
    import isa_check
    res = isa_check.check_library(LIB)
    mfma_kernels = set().union(*(v[3] for v in res.values()))
    # the disassembly covers the kernels that matter, and the pattern is recognised in objdump syntax
    # (the MFMA-free fp32 backward kernels keep such ops: the hazard needs an MFMA wave beside them)
    for k in ("k_fused_proj", "k_lookup_tile", "k_build_bf16", "k_fused_box"):
        assert any(k in m for m in mfma_kernels), k
    # k_fused_proj r = 1 comes from its own no-SLP unit (fused_proj_r1.hip, round 6): present, and clean like the rest
    assert any("k_fused_projILi1E" in m for m in mfma_kernels)
    assert any(v[2] for v in res.values())
    bad = {f"{b}:{k}": v[0] for b, (pk, _mf, _q, _m) in res.items() for k, v in pk.items()}
    assert not bad, bad


def test_hidden_load_kernels_do_not_spill():
    """k_build_f32r and the k_build_bf16 / k_build_bf16_2b instances with NCH <= 16 issue their operand loads from
    inline asm, out of the compiler's s_waitcnt bookkeeping (build_gemm.hip, Hidden<NCH>).  That is only correct
    while none of those destination registers is ever spilled or reassigned before its load lands (the round-1
    fault: k_build_bf16_2b<32> spilled them).  The AMDGPU metadata of the shipped code objects must show no
    private segment and no VGPR / SGPR spills for every such kernel."""
    import isa_check
    res = isa_check.kernel_resources(LIB)
    hidden = [k for k in res if isa_check.HIDDEN_LOAD_KERNELS.search(k)]
    assert len(hidden) >= 12, hidden     # k_build_f32r x 6, k_build_bf16 x 6+, k_build_bf16_2b x 6
    assert any("k_build_f32r" in k for k in hidden) and any("k_build_bf16_2b" in k for k in hidden)
    assert not isa_check.spill_violations(res), isa_check.spill_violations(res)
    # the pattern recognises spills where they exist (the compiler-tracked NCH = 32 instances do spill)
    assert any(v.get(".vgpr_spill_count", 0) for k, v in res.items() if "k_build_bf16_2bILi32E" in k)


def test_product_library_has_no_diagnostics_instances():
    """The ablation / timeline / store-policy instances are built only into libdvccorr_diag.so (make diag,
    common.h DVC_DIAG); the shipped libdvccorr.so refuses their tuning knobs and carries none of them."""
    import ctypes
    import isa_check
    names = list(isa_check.kernel_resources(LIB))
    assert any("k_lookup_tile" in k for k in names) and any("k_fused_box" in k for k in names)
    # ablation template arguments: k_lookup_tile<bf16, 4, true, ABL != 0, ...>, k_fused_box<..., ABL != 0>,
    # k_build_bf16<16, false, ABL != 0>, k_fused_proj<4, 4, ABL != 0>
    diag = [k for k in names if "k_lookup_tileItLi4ELb1ELi1E" in k or "k_lookup_tileItLi4ELb1ELi8E" in k
            or "k_build_bf16ILi16ELb0ELi1E" in k or "k_fused_boxILi4ELi4ELi8ELi2ELi2ELi16ELi1E" in k
            or "k_fused_projILi4ELi4ELi1E" in k or "k_lookup_tileItLi4ELb1ELi0ELb0ELi0ELi4ELi16E" in k]
    assert not diag, diag
    lib = ctypes.CDLL(LIB)
    for key in (b"lookup_ablate", b"build_ablate", b"fused_ablate", b"lookup_stpol", b"lookup_trace_lo"):
        assert lib.dvc_set_tuning(key, 1) == 2, key   # DVC_ERR_UNSUPPORTED
    assert lib.dvc_set_tuning(b"lookup_variant", 2) == 0
