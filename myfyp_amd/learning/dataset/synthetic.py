"""Synthetic, learnable stand-ins for MNIST and CIFAR-10 (no network access on the build/GPU boxes).

Each class has a fixed random smooth prototype; a sample is its class prototype, randomly shifted
by up to ±2 px, plus per-pixel noise, clipped to uint8 — same dtype/shape/range as the real
datasets (MNIST ``uint8[28,28]`` in 0..255, CIFAR ``uint8[32,32,3]``), so the learners see the
reference's input pipeline (uint8 → float, no normalisation). Difficulty knobs, so that accuracy
climbs over several rounds instead of saturating instantly:

* ``similarity`` — every class prototype is blended with a shared pattern (classes overlap);
* ``noise`` — per-pixel stroke noise;
* ``modes`` — prototypes per class (a sample picks one: intra-class variety a model must cover);
* ``label_noise`` — fraction of TRAINING labels replaced by a uniformly random class (test labels
  stay clean, so the Bayes accuracy stays 1 but training sees conflicting targets).
"""

from __future__ import annotations

from typing import Tuple

import numpy as np

from myfyp_amd.learning.dataset.p2pfl_dataset import P2PFLDataset


def _smooth_prototypes(rng: np.random.Generator, num_classes: int, shape: Tuple[int, ...], similarity: float = 0.0) -> np.ndarray:
    """Smooth random 'stroke' images; ``similarity`` blends every class with a shared pattern
    (higher = classes overlap more = harder task)."""
    h, w = shape[0], shape[1]
    protos = []
    common = rng.random((7, 7) + shape[2:])
    for _ in range(num_classes):
        coarse = (1 - similarity) * rng.random((7, 7) + shape[2:]) + similarity * common
        # bilinear upsample of a 7x7 grid -> smooth blobs
        yi = np.linspace(0, 6, h)
        xi = np.linspace(0, 6, w)
        y0 = np.floor(yi).astype(int).clip(0, 5)
        x0 = np.floor(xi).astype(int).clip(0, 5)
        fy = (yi - y0)[:, None]
        fx = (xi - x0)[None, :]
        if coarse.ndim == 3:
            fy, fx = fy[..., None], fx[..., None]
        a = coarse[y0][:, x0]
        b = coarse[y0][:, x0 + 1]
        c = coarse[y0 + 1][:, x0]
        d = coarse[y0 + 1][:, x0 + 1]
        img = a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + c * fy * (1 - fx) + d * fy * fx
        img = np.clip((img - 0.45) * 3.0, 0, 1)  # sparse strokes like handwritten digits
        protos.append(img)
    return np.stack(protos).astype(np.float32)


def _make(rng: np.random.Generator, protos: np.ndarray, n: int, noise: float, max_shift: int, modes: int = 1,
          label_noise: float = 0.0) -> Tuple[np.ndarray, np.ndarray]:
    num_classes = protos.shape[0] // modes  # protos: [num_classes * modes, ...], class-major
    labels = rng.integers(0, num_classes, size=n)
    mode = rng.integers(0, modes, size=n) if modes > 1 else np.zeros(n, dtype=np.int64)
    out = np.empty((n,) + protos.shape[1:], dtype=np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = protos[labels[s:e] * modes + mode[s:e]].copy()
        # per-sample random translation (grouped by shift so it stays vectorised)
        shifts = rng.integers(-max_shift, max_shift + 1, size=(e - s, 2))
        for dy in range(-max_shift, max_shift + 1):
            for dx in range(-max_shift, max_shift + 1):
                sel = np.nonzero((shifts[:, 0] == dy) & (shifts[:, 1] == dx))[0]
                if len(sel):
                    base[sel] = np.roll(base[sel], (dy, dx), axis=(1, 2))
        # MNIST-like statistics: near-zero background, noisy strokes of varying intensity, plus
        # sparse background speckle. ``noise`` scales the stroke noise.
        gain = rng.uniform(0.6, 1.2, size=(e - s,) + (1,) * (base.ndim - 1))
        stroke = base > 0.05
        img = base * 255.0 * gain + rng.normal(0.0, noise * 255.0, size=base.shape) * np.where(stroke, 1.0, 0.15)
        img = np.where(rng.random(base.shape) < 0.02, rng.uniform(0, 255, size=base.shape), img)
        out[s:e] = np.clip(img, 0, 255).astype(np.uint8)
    if label_noise > 0:
        flip = rng.random(n) < label_noise
        labels = np.where(flip, rng.integers(0, num_classes, size=n), labels)
    return out, labels.astype(np.int64)


def synthetic_mnist(n_train: int = 60000, n_test: int = 10000, seed: int = 1234, noise: float = 1.0, max_shift: int = 3, similarity: float = 0.6) -> P2PFLDataset:
    """MNIST-shaped dataset: ``image`` uint8[N,28,28], ``label`` int64[N] in 0..9."""
    rng = np.random.default_rng(seed)
    protos = _smooth_prototypes(rng, 10, (28, 28), similarity)
    xtr, ytr = _make(rng, protos, n_train, noise, max_shift)
    xte, yte = _make(rng, protos, n_test, noise, max_shift)
    return P2PFLDataset.from_arrays({"image": xtr, "label": ytr}, {"image": xte, "label": yte})


def synthetic_cifar10(n_train: int = 50000, n_test: int = 10000, seed: int = 4321, noise: float = 1.0, max_shift: int = 3, similarity: float = 0.6,
                      modes: int = 1, label_noise: float = 0.0) -> P2PFLDataset:
    """CIFAR-10-shaped dataset: ``image`` uint8[N,32,32,3], ``label`` int64[N] in 0..9."""
    rng = np.random.default_rng(seed)
    protos = _smooth_prototypes(rng, 10 * modes, (32, 32, 3), similarity)
    xtr, ytr = _make(rng, protos, n_train, noise, max_shift, modes, label_noise)
    xte, yte = _make(rng, protos, n_test, noise, max_shift, modes)
    return P2PFLDataset.from_arrays({"image": xtr, "label": ytr}, {"image": xte, "label": yte})
