"""Seeded synthetic 16 kHz noisy/clean pairs (SURVEY.md §8 d).

The reference trains on LibriMix (absent here; ``distill.py:208-229``).  Bench and tests use
this recipe instead: clean = sum of 8 enveloped sinusoids, noise scaled to a random SNR.
"""
import numpy as np

from .weights import DATA_SEED


def synthetic_pairs(batch, num_samples, seed=DATA_SEED, fs=16000):
    """Returns (noisy, clean) float32 arrays of shape [batch, num_samples]."""
    g = np.random.default_rng(seed)
    t = np.arange(num_samples, dtype=np.float64) / fs
    env = 0.5 * (1.0 + np.sin(2 * np.pi * 3.0 * t))
    clean = np.zeros((batch, num_samples), np.float64)
    noisy = np.zeros((batch, num_samples), np.float64)
    for b in range(batch):
        f = g.uniform(80.0, 3800.0, 8)
        a = g.uniform(0.02, 0.1, 8)
        ph = g.uniform(0.0, 2 * np.pi, 8)
        c = (a[:, None] * np.sin(2 * np.pi * f[:, None] * t[None, :] + ph[:, None])).sum(0) * env
        n = g.standard_normal(num_samples)
        snr_db = g.uniform(0.0, 10.0)
        p_c = np.mean(c ** 2)
        p_n = np.mean(n ** 2)
        n *= np.sqrt(p_c / (p_n * 10 ** (snr_db / 10.0)))
        clean[b] = c
        noisy[b] = np.clip(c + n, -1.0, 1.0)
    return noisy.astype(np.float32), clean.astype(np.float32)
