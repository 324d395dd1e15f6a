"""Record the factored K/V projection outputs of one image-classifier forward under three
executors (HIP in-tree PE GEMM, HIP with the torch.mm fallback, emulation) and compare."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_model_gpu as T  # noqa: E402
from perceiver_io_amd import ops  # noqa: E402
from perceiver_io_amd.ops import ext, fused  # noqa: E402
from perceiver_io_amd.tasks import LitImageClassifier  # noqa: E402


class _NoPeGemm:
    def __getattr__(self, n):
        if n in ("pe_gemm", "pe_weight_prep"):
            raise AttributeError(n)
        return getattr(ext.require(), n)


rec = []
orig = fused._pe_proj_fwd


def spy(K, *a):
    out = orig(K, *a)
    rec.append([t.detach().float().clone() for t in out])
    return out


fused._pe_proj_fwd = spy
torch.manual_seed(1)
lit = LitImageClassifier(image_shape=(28, 28, 1), num_classes=10,
                         optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                         num_latents=32, num_latent_channels=128, num_encoder_layers=2,
                         num_encoder_self_attention_layers_per_block=2, num_decoder_cross_attention_heads=1).cuda()
x = torch.randn(4, 28, 28, 1, device="cuda")
y = torch.randint(0, 10, (4,), device="cuda")
res = {}
saved = ops.fused.kernels
for name in ("kernel", "torch_mm", "emu"):
    rec.clear()
    lit.zero_grad()
    if name == "emu":
        with ops.backend("hip"), T._emulated():
            l, _ = lit.step((x, y))
    else:
        if name == "torch_mm":
            ops.fused.kernels = lambda t: _NoPeGemm()
        with ops.backend("hip"):
            l, _ = lit.step((x, y))
        ops.fused.kernels = saved
    res[name] = (l.item(), [r for r in rec])
    print(name, "loss %.6f" % l.item(), "calls", len(rec), flush=True)
for name in ("kernel", "torch_mm"):
    for i, (a, b) in enumerate(zip(res[name][1], res["emu"][1])):
        print(name, "call", i, " ".join("%.3e/%.3e" % ((u - v).abs().max().item(), v.abs().max().item())
                                        for u, v in zip(a, b)))
