"""k_upflow alone at the #5 iteration-tail shape (coords 128^3 -> flow_up 256^3), for rocprofv3
kernel-trace / PMC passes: N calls of dvc_flow_step with the current tuning (env PF = upflow_staged,
ROWS = upflow_rows)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raft-dvc_amd"))
import dvccorr  # noqa: E402,F401
from dvccorr import _lib  # noqa: E402

S, E, N = int(os.environ.get("S", 128)), int(os.environ.get("E", 2)), int(os.environ.get("N", 10))
_lib.set_tuning("upflow_staged", int(os.environ.get("PF", 1)))
_lib.set_tuning("upflow_rows", int(os.environ.get("ROWS", 12)))
dev = torch.device("cuda:0")
c1 = torch.rand(1, 3, S, S, S, device=dev) * S
dl = torch.rand(1, 3, S, S, S, device=dev) - 0.5
new = torch.empty_like(c1)
up = torch.empty(1, 3, S * E, S * E, S * E, device=dev)
st = torch.cuda.current_stream(dev)
for _ in range(N):
    _lib.check(_lib.lib().dvc_flow_step(c1.data_ptr(), dl.data_ptr(), new.data_ptr(), up.data_ptr(),
                                         1, S, S, S, S * E, S * E, S * E, st.cuda_stream))
torch.cuda.synchronize()
print("done", flush=True)
