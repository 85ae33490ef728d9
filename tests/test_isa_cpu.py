"""ISA guard (CPU, cross-compiles): no kernel that runs MFMAs may contain a packed-FP32 op whose low lane
reads the high element of a VGPR source.  On gfx950 such ops returned wrong low-lane values in lanes 48-63
now and then while another wave of the workgroup ran MFMAs (k_fused_proj, round 2; tools/isa_check.py,
splat2 in csrc/common.h)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                                reason="hipcc not available")


@pytest.mark.timeout(600)
def test_no_packed_fp32_opsel_beside_mfma():
    import isa_check
    csrc = isa_check.CSRC
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".hip"))
    res = isa_check.check(files)
    bad = {f"{f}:{k}": v[0] for f, (pk, _mf, _q) in res.items() for k, v in pk.items()}
    assert not bad, bad
