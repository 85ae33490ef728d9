"""A/B of k_upflow rows per work item and grid size (dvc_set_tuning "upflow_rows" /
"upflow_wgs", "upflow_staged") at the bench's
iteration-tail shape (coords 32^3 -> flow_up 128^3): HIP-event average over 50 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-dvc_amd"))
import dvccorr  # noqa: E402
from dvccorr import _lib  # noqa: E402

S, E = int(os.environ.get("S", 32)), int(os.environ.get("E", 4))
dev = torch.device("cuda:0")
c1 = torch.rand(1, 3, S, S, S, device=dev) * S
dl = torch.rand(1, 3, S, S, S, device=dev) - 0.5
new = torch.empty_like(c1)
up = torch.empty(1, 3, S * E, S * E, S * E, device=dev)
st = torch.cuda.current_stream(dev)
ref = None
for pf, rows, wgs in ((0, 8, 1 << 30), (1, 8, 1 << 30), (1, 8, 2048), (1, 12, 1 << 30), (1, 12, 2048),
                      (1, 16, 1 << 30), (1, 16, 2048), (1, 16, 1024), (1, 16, 4096), (1, 24, 2048)):
    _lib.set_tuning("upflow_staged", pf)
    _lib.set_tuning("upflow_rows", rows)
    _lib.set_tuning("upflow_wgs", wgs)
    call = lambda: _lib.check(_lib.lib().dvc_flow_step(c1.data_ptr(), dl.data_ptr(), new.data_ptr(), up.data_ptr(),
                                                        1, S, S, S, S * E, S * E, S * E, st.cuda_stream))
    for _ in range(5):
        call()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(50):
        call()
    b.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 50
    if ref is None:
        ref = up.clone()
    same = torch.equal(ref, up)
    print(f"staged {pf} rows {rows:2d} wgs {min(wgs, 99999):5d}: {ms * 1e3:.1f} us  {up.numel() * 4 * 1.0 / (ms * 1e-3) / 1e9:.0f} GB/s written  same={same}",
          flush=True)
