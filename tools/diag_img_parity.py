"""Per-tensor gradient errors of the image classifier (HIP kernels vs emulation vs fp32 eager)
for the LayerNorm parameters, optionally with torch batch sums instead of pio::batch_sum2."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_model_gpu as T  # noqa: E402
from perceiver_io_amd import ops  # noqa: E402
from perceiver_io_amd.ops import ext  # noqa: E402
from perceiver_io_amd.tasks import LitImageClassifier  # noqa: E402


class _NoPeGemm:
    """the HIP extension without the in-tree PE GEMM (torch.mm fallback in _pe_proj_fwd)"""

    def __getattr__(self, n):
        if n in ("pe_gemm", "pe_weight_prep"):
            raise AttributeError(n)
        return getattr(ext.require(), n)


for variant in ("kernel", "torch_mm"):
    for seed in (1, 2):
        torch.manual_seed(seed)
        lit = LitImageClassifier(image_shape=(28, 28, 1), num_classes=10,
                                 optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                 num_latents=32, num_latent_channels=128, num_encoder_layers=2,
                                 num_encoder_self_attention_layers_per_block=2, num_decoder_cross_attention_heads=1).cuda()
        x = torch.randn(4, 28, 28, 1, device="cuda")
        y = torch.randint(0, 10, (4,), device="cuda")
        res = {}
        saved = ops.fused.kernels
        for name in ("torch", "hip", "emu"):
            lit.zero_grad()
            if name == "emu":
                with ops.backend("hip"), T._emulated():
                    l, _ = lit.step((x, y))
                    l.backward()
            else:
                if variant == "torch_mm" and name == "hip":
                    ops.fused.kernels = lambda t: _NoPeGemm()
                with ops.backend(name):
                    l, _ = lit.step((x, y))
                    l.backward()
                ops.fused.kernels = saved
            res[name] = T._grads(lit)
        for n in res["torch"]:
            if "1.cross_attention.0.module.q_norm" in n:
                g0, g1, g2 = res["torch"][n], res["hip"][n], res["emu"][n]
                print(variant, seed, n, "hip-emu %.4f hip-torch %.4f emu-torch %.4f" % (
                    T._rel(g1, g2), T._rel(g1, g0), T._rel(g2, g0)), flush=True)
