"""What the persistent block kernel's workgroup 0 sees (kernel arguments, first ticket) in eager
launches, a standalone captured graph with host work between the launch and the end of the
capture, and the engine's replayed MLM step (csrc/persist.hip persist_debug)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from perceiver_io_amd.ops import ext  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_persist_gpu import _block, _block_params, bf  # noqa: E402

K = ext.require()
DEV = "cuda"


def show(tag):
    torch.cuda.synchronize()
    d = K.persist_debug()
    print(f"{tag}: R={d[0]} N={d[1]} L={d[2]} sync={d[3]:#x} qkv0={d[4]:#x} ticket0={d[5]} wo0={d[6]:#x} x0={d[7]:#x} "
          f"err={K.persist_errors(True)}", flush=True)


B, N, L, C = 16, 256, 3, 64
R = B * N
qkv = bf(torch.randn(R, 3 * C, device=DEV))
x = torch.randn(R, C, device=DEV)
ps = _block_params(L, 64, seed=9)
print(f"expected qkv0={qkv.data_ptr():#x} x0={x.data_ptr():#x} wo0={ps['wo'][0].data_ptr():#x}")
ref = _block(K, qkv, x, N, ps, None, 0.0)
show("eager")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    _block(K, qkv, x, N, ps, None, 0.0)
torch.cuda.current_stream().wait_stream(s)
show("eager side stream")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = _block(K, qkv, x, N, ps, None, 0.0)
    junk = []
    for i in range(50):  # host work + allocations between the launch and the end of the capture
        junk.append(torch.empty(1000 + i, device=DEV).fill_(1.0) * 2)
for r in range(3):
    g.replay()
    show(f"replay {r}")
    print("  bitwise:", all(torch.equal(u, v) for u, v in zip(out, ref)), flush=True)
