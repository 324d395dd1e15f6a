"""BERT-style text masking (reference ``perceiver/model.py:265-293``).

The randomness is a counter hash (``text_mask_kernel``, ``csrc/elementwise.hip``): per token,
three uniforms and a replacement id derive from ``hash3(seed, counter)`` and the token index.
The per-device state ``{seed, counter, ticket}`` lives in device memory and the kernel itself
advances the counter, so a replayed hipGraph draws fresh masks every step with no torch RNG
kernels (and none of the generator's per-replay seed/offset fills) in the step.  The seed is
drawn once from torch's default generator (``torch.manual_seed`` makes runs reproducible).
An explicit ``generator`` draws a one-off seed from it instead (counter 0, state untouched).

The CPU path evaluates the same hash (``ops/emulation.py``), so both backends produce
identical masks from the same state.  Unlike the reference, the input ids are never modified
in place (defect D4).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import emulation, ext

_states: Dict[torch.device, torch.Tensor] = {}


def mask_state(device) -> torch.Tensor:
    """The persistent ``int64 (3,)`` masking RNG state of ``device`` (created on first use,
    which must precede any graph capture — the step engine's eager warm-up does)."""
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    st = _states.get(device)
    if st is None:
        if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("text masking state must be created before graph capture (run one eager step first)")
        seed = int(torch.randint(0, 2**62, (1,)).item())
        st = _states[device] = torch.tensor([seed, 0, 0], dtype=torch.int64, device=device)
    return st


def reset_mask_state(seed: Optional[int] = None):
    """Forget (or re-seed, on every device already in use) the masking RNG state."""
    if seed is None:
        _states.clear()
        return
    for st in _states.values():
        st.copy_(torch.tensor([seed, 0, 0], dtype=torch.int64))


def text_masking(x: torch.Tensor, pad_mask: Optional[torch.Tensor], vocab_size: int, unk_token_id: int,
                 mask_token_id: int, num_special_tokens: int, mask_p: float = 0.15,
                 generator: Optional[torch.Generator] = None):
    from . import use_hip

    if generator is not None:  # one-off seed from the caller's generator
        seed = int(torch.randint(0, 2**62, (1,), generator=generator, device=generator.device).item())
        state, advance = torch.tensor([seed, 0, 0], dtype=torch.int64, device=x.device), False
    else:
        state, advance = mask_state(x.device), True
    pm = pad_mask.to(torch.bool).contiguous() if pad_mask is not None else None
    K = ext.require() if use_hip(x) else emulation
    return K.text_mask(x.contiguous(), pm, state, unk_token_id, mask_token_id, mask_p, num_special_tokens, vocab_size,
                       advance)
