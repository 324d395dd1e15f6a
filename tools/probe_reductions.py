import torch, sys
sys.path.insert(0, '.')
from perceiver_io_amd.ops import ext
K = ext.require()
x = torch.arange(64, dtype=torch.float32, device='cuda')
out = K.reduce_probe(x).cpu()
names = ["wave_sum", "wave_max", "half_sum", "half_max", "xor16_sum", "xor32_sum"]
for n, o in zip(names, out):
    print(n, o.tolist())
