"""Portable seeded weights for random-init RAFT models.

The reference's random init (`core/extractor.py:147-154` kaiming-normal fan_out
for the encoders, PyTorch's default Conv2d init elsewhere) depends on the
global torch RNG stream and on module construction order.  Parity between the
build container (where the reference runs) and the GPU box (where it cannot)
needs weights that both sides regenerate bit-for-bit from a seed, so every
tensor here is drawn from its own numpy PCG64 stream keyed by (seed, key name).

The distributions mirror the reference's init:
  * encoder convs (`fnet.*`, `cnet.*`): N(0, 2 / (out_ch * kh * kw))  (kaiming fan_out, relu)
  * other convs: U(-1/sqrt(fan_in), 1/sqrt(fan_in))                 (PyTorch default)
  * conv biases: U(-1/sqrt(fan_in), 1/sqrt(fan_in))
  * BatchNorm: weight U(0.8, 1.2), bias U(-0.1, 0.1), running_mean N(0, 0.1^2),
    running_var U(0.8, 1.2) — perturbed from (1, 0, 0, 1) so BN folding is exercised.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch
import torch.nn as nn


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([int(seed), zlib.crc32(key.encode())])))


def seeded_state_dict(model: nn.Module, seed: int = 0) -> dict:
    """Return {state_dict key: torch.Tensor (CPU)} for every Conv2d / BatchNorm2d
    tensor of `model`, drawn deterministically from (seed, key)."""
    out = {}
    for name, mod in model.named_modules():
        pre = name + "." if name else ""
        if isinstance(mod, nn.Conv2d):
            o, c, kh, kw = mod.weight.shape
            fan_in = c * kh * kw
            key = pre + "weight"
            if name.startswith("fnet.") or name.startswith("cnet."):
                std = np.sqrt(2.0 / (o * kh * kw))
                w = _rng(seed, key).standard_normal((o, c, kh, kw)) * std
            else:
                bound = 1.0 / np.sqrt(fan_in)
                w = _rng(seed, key).uniform(-bound, bound, (o, c, kh, kw))
            out[key] = torch.from_numpy(w.astype(np.float32))
            if mod.bias is not None:
                key = pre + "bias"
                bound = 1.0 / np.sqrt(fan_in)
                out[key] = torch.from_numpy(_rng(seed, key).uniform(-bound, bound, (o,)).astype(np.float32))
        elif isinstance(mod, nn.BatchNorm2d):
            n = mod.num_features
            out[pre + "weight"] = torch.from_numpy(_rng(seed, pre + "weight").uniform(0.8, 1.2, n).astype(np.float32))
            out[pre + "bias"] = torch.from_numpy(_rng(seed, pre + "bias").uniform(-0.1, 0.1, n).astype(np.float32))
            out[pre + "running_mean"] = torch.from_numpy(
                (_rng(seed, pre + "running_mean").standard_normal(n) * 0.1).astype(np.float32))
            out[pre + "running_var"] = torch.from_numpy(
                _rng(seed, pre + "running_var").uniform(0.8, 1.2, n).astype(np.float32))
            out[pre + "num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    # Shared submodules (ResidualBlock.norm3 is also downsample.1, core/extractor.py:39-42)
    # appear under every alias in state_dict(); give aliases the canonical tensors.
    canon = {}
    for name, mod in model.named_modules():
        canon.setdefault(id(mod), name)
    for name, mod in model.named_modules(remove_duplicate=False):
        first = canon[id(mod)]
        if first != name:
            for k in list(out):
                if (k.startswith(first + ".") and "." not in k[len(first) + 1:]):
                    out[name + k[len(first):]] = out[k]
    return out


def seeded_images(batch: int, height: int, width: int, seed: int = 1):
    """Synthetic frame pair: uint8-valued float frames U[0,255) from a seeded
    torch CPU generator, img2 drawn after img1."""
    g = torch.Generator().manual_seed(seed)
    img1 = torch.randint(0, 256, (batch, 3, height, width), generator=g).float()
    img2 = torch.randint(0, 256, (batch, 3, height, width), generator=g).float()
    return img1, img2


def smooth_images(batch: int, height: int, width: int, seed: int = 1, shift=(3.0, -2.0)):
    """A textured frame and a shifted copy (real motion, so the recurrent
    refinement has structure to find).  Deterministic numpy construction."""
    rng = _rng(seed, "smooth_images")
    ys, xs = np.meshgrid(np.arange(height, dtype=np.float64), np.arange(width, dtype=np.float64), indexing="ij")
    imgs1, imgs2 = [], []
    for bi in range(batch):
        f = rng.uniform(0.02, 0.15, (6, 2))
        ph = rng.uniform(0, 2 * np.pi, (6, 3))

        def tex(x, y):
            ch = []
            for c in range(3):
                v = sum(np.sin(f[k, 0] * x + f[k, 1] * y + ph[k, c]) for k in range(6))
                ch.append(127.5 + 20.0 * v)
            return np.clip(np.stack(ch, 0), 0, 255)

        imgs1.append(tex(xs, ys))
        imgs2.append(tex(xs - shift[0] * (bi + 1), ys - shift[1]))
    i1 = torch.from_numpy(np.round(np.stack(imgs1)).astype(np.float32))
    i2 = torch.from_numpy(np.round(np.stack(imgs2)).astype(np.float32))
    return i1, i2
