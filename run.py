#!/usr/bin/env python
"""LArTPC per-pixel semantic segmentation with Perceiver IO (reference ``run.py``).

512×512 single-plane wire images → 3 classes per pixel.  Perceiver IO with a Fourier-encoded
image input (262,144 inputs, key-padding mask on zero pixels = sparse attention), 32×64
latents, 3 layers × (1 cross + 3 self-attention), and a decoder with 262,144 output queries
(one per pixel) → 3-way classifier.  A U-ResNet is constructed alongside (unused in forward,
as in the reference).  Weighted cross-entropy (background weight 0), Adam (lr 1e-3, wd 1e-4),
ReduceLROnPlateau stepped on the loss before backward, grad-norm clip 10, batch 4, per-class
accuracies, validation each epoch, checkpoint ``{'epoch','model_state_dict','optimizer_state_dict'}``.

Differences (documented): the larcv/ROOT reader is replaced by a synthetic track/shower
generator (``perceiver_io_amd.data.synthetic.lartpc_event``; larcv/ROOT are not available);
logits are permuted to (B, 3, H·W) instead of the reference's ``reshape(B, 3, -1)`` which
interleaves pixels and classes (defect D6); metrics go to JSONL/tfevents.

    python run.py [--epochs 10] [--events 64] [--size 512] [--batch-size 4]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from perceiver_io_amd.data.synthetic import SyntheticLArTPC  # noqa: E402
from perceiver_io_amd.models import (ClassificationOutputAdapter, ImageInputAdapter, PerceiverDecoder,  # noqa: E402
                                     PerceiverEncoder, PerceiverIO)
from perceiver_io_amd.models.uresnet import UResNet  # noqa: E402
from perceiver_io_amd.train.loggers import TensorBoardLogger  # noqa: E402


class LArPerceiver(torch.nn.Module):
    def __init__(self, size: int = 512, latents=(32, 64), bands: int = 32):
        super().__init__()
        n, c = latents
        enc = PerceiverEncoder(ImageInputAdapter((size, size, 1), bands), (n, c), num_layers=3,
                               num_cross_attention_heads=4, num_self_attention_heads=4,
                               num_self_attention_layers_per_block=3, dropout=0.0)
        dec = PerceiverDecoder(ClassificationOutputAdapter(num_classes=3, num_outputs=size * size, num_output_channels=c),
                               (n, c), num_cross_attention_heads=1, dropout=0.0)
        self.size = size
        self.perceiver = PerceiverIO(enc, dec)
        self.uresnet = UResNet(num_classes=3, input_channels=c, inplanes=16)

    def forward(self, img):
        b = img.shape[0]
        x = img.reshape(b, self.size, self.size, 1)
        mask = (x == 0).reshape(b, -1)  # zero pixels are padding keys (sparse attention)
        logits = self.perceiver(x, mask)  # (B, H*W, 3)
        return logits.permute(0, 2, 1)  # (B, 3, H*W)


def accuracies(pred, lab):
    out = {}
    for name, sel in (("acc", lab > 0), ("acc1", lab == 1), ("acc2", lab == 2)):
        n = sel.sum()
        out[name] = ((pred[sel] == lab[sel]).float().mean().item() if n > 0 else 0.0)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--events", type=int, default=64)
    ap.add_argument("--val-events", type=int, default=8)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--batch-size", type=int, default=4)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--max-steps", type=int, default=-1)
    ap.add_argument("--log-dir", default="runs")
    ap.add_argument("--ckpt-dir", default="ckpt")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args(argv)
    dev = torch.device(a.device)
    torch.manual_seed(0)
    model = LArPerceiver(a.size).to(dev)
    train = torch.utils.data.DataLoader(SyntheticLArTPC(a.events, a.size, seed=0), batch_size=a.batch_size,
                                        shuffle=True, drop_last=True, num_workers=1)
    val = torch.utils.data.DataLoader(SyntheticLArTPC(a.val_events, a.size, seed=1), batch_size=a.batch_size,
                                      drop_last=True)
    opt = torch.optim.Adam(model.parameters(), lr=a.lr, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, patience=5000, factor=0.1)
    weights = torch.tensor([0.0, 1.0, 1.0], device=dev)
    log = TensorBoardLogger(a.log_dir, name="lartpc")
    step = 0
    epoch = 0
    for epoch in range(a.epochs):
        model.train()
        for img, lab in train:
            t0 = time.perf_counter()
            img, lab = img.to(dev), lab.to(dev)
            opt.zero_grad()
            out = model(img)
            loss = F.cross_entropy(out, lab, weight=weights)
            sched.step(loss.item())  # stepped before backward, like the reference
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 10)
            opt.step()
            acc = accuracies(out.argmax(1), lab)
            log.log_metrics({"loss": loss.item(), "lr": opt.param_groups[0]["lr"],
                             **{f"train_{k}": v for k, v in acc.items()}}, step)
            print(f"epoch {epoch} step {step} loss {loss.item():.4f} {time.perf_counter() - t0:.3f}s", flush=True)
            step += 1
            if 0 < a.max_steps <= step:
                break
        model.eval()
        vl, va = [], []
        with torch.no_grad():
            for img, lab in val:
                img, lab = img.to(dev), lab.to(dev)
                out = model(img)
                vl.append(F.cross_entropy(out, lab, weight=weights).item())
                va.append(accuracies(out.argmax(1), lab)["acc"])
        if vl:
            log.log_metrics({"validation_loss": sum(vl) / len(vl), "val_acc": sum(va) / len(va)}, step)
            print(f"validation loss: {sum(vl) / len(vl):.4f}", flush=True)
        if 0 < a.max_steps <= step:
            break
    os.makedirs(a.ckpt_dir, exist_ok=True)
    torch.save({"epoch": epoch, "model_state_dict": model.state_dict(), "optimizer_state_dict": opt.state_dict()},
               os.path.join(a.ckpt_dir, f"model_{epoch}.ckpt"))
    log.close()


if __name__ == "__main__":
    main()
