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
    assert any(v[2] for v in res.values())
    bad = {f"{b}:{k}": v[0] for b, (pk, _mf, _q, _m) in res.items() for k, v in pk.items()}
    assert not bad, bad
