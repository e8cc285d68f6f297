"""Deterministic synthetic weights and images (no checkpoints ship with the reference).

The reference loads `models/vgg_normalised.pth` (`config/rl/*.yaml` key `vgg:`) and
its own `checkpoints/<iter>` files; none are in the repo (`.gitignore:5`), and there is
no network here. Every test, golden fixture and benchmark therefore uses weights from
this counter-based generator, which is identical on every machine and every torch
version because it is plain uint64 arithmetic in numpy (splitmix64 -> uniform).

* conv weights: uniform with He variance, std = sqrt(2 / fan_in)  (fan_in = Cin*kh*kw)
* conv biases:  uniform in [-0.05, 0.05)
* images:       uniform in [0, 1), matching `ToTensor()` of the reference drivers
                (`test.py:49-54`, `train.py:41-46`)
"""
from __future__ import annotations

import hashlib
from typing import Dict, Iterable, Tuple

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _key_seed(seed: int, key: str) -> np.uint64:
    h = hashlib.sha256(f"{seed}:{key}".encode()).digest()
    return np.uint64(int.from_bytes(h[:8], "little"))


def uniform01(seed: int, key: str, n: int, offset: int = 0) -> np.ndarray:
    """n float64 values in [0,1) from splitmix64 over counter offset+1..offset+n."""
    base = _key_seed(seed, key)
    with np.errstate(over="ignore"):
        z = base + (np.arange(offset + 1, offset + n + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def conv_param(seed: int, key: str, shape: Tuple[int, ...]) -> np.ndarray:
    """He-uniform conv weight (4-D) or small uniform bias (1-D), float32."""
    n = int(np.prod(shape))
    u = uniform01(seed, key, n)
    if len(shape) == 4:
        fan_in = shape[1] * shape[2] * shape[3]
        bound = np.sqrt(3.0) * np.sqrt(2.0 / fan_in)
        v = (2.0 * u - 1.0) * bound
    else:
        v = (2.0 * u - 1.0) * 0.05
    return v.astype(np.float32).reshape(shape)


def synth_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int) -> Dict[str, np.ndarray]:
    """Fill every (key, shape) pair of a state_dict template."""
    return {k: conv_param(seed, k, tuple(s)) for k, s in shapes}


def synth_module_(module, seed: int) -> None:
    """In-place: overwrite every parameter of a torch module with generator values."""
    import torch

    sd = module.state_dict()
    new = synth_state_dict(((k, tuple(v.shape)) for k, v in sd.items()), seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in new.items()})


def image(seed: int, shape: Tuple[int, ...]) -> np.ndarray:
    """Synthetic image batch in [0,1), float32, NCHW."""
    return uniform01(seed, "image", int(np.prod(shape))).astype(np.float32).reshape(shape)


def image_range(seed: int, shape: Tuple[int, ...], start: int, end: int) -> np.ndarray:
    """Images [start, end) of image(seed, shape) without generating the others (the
    counter of element i is i + 1, so a batch slice is a counter range)."""
    per = int(np.prod(shape[1:]))
    return uniform01(seed, "image", (end - start) * per, offset=start * per).astype(
        np.float32).reshape((end - start,) + tuple(shape[1:]))


def checksum(arrs: Dict[str, np.ndarray]) -> Tuple[float, float]:
    s = 0.0
    s2 = 0.0
    for k in sorted(arrs):
        a = arrs[k].astype(np.float64)
        s += float(a.sum())
        s2 += float((a * a).sum())
    return s, s2


def conditioned_features(seed: int, C: int, HW: int, decades: float = 3.0) -> np.ndarray:
    """(C, HW) float64 ReLU features conditioned like encoder activations: channel scales
    spanning 10^-decades .. 1, neighbouring channels mixed, so the covariance's eigenvalues
    spread over ~2 * decades decades (WCT goldens at C = 256 / 512). Elementwise only:
    bit-identical on every machine."""
    z = (2.0 * uniform01(seed, "wctfeat", C * HW).reshape(C, HW) - 1.0) * np.sqrt(3.0)
    scale = 10.0 ** (-decades * np.arange(C, dtype=np.float64) / max(C - 1, 1))
    x = scale[:, None] * (z + 0.3)
    x[:-1] += 0.5 * x[1:]
    return np.maximum(x, 0.0)
