"""Perturbation bound of one SPKD term (framework.py:150-172) under relative feature errors.

Test infrastructure ("bf16 bound"): the mixed-precision C2 step stores the frozen
teacher's and the ReviewKD fusions' features in bf16 and runs their GEMMs on bf16 MFMA operands,
so every tap row z_i (one sample, K features) reaches the SPKD Gram as z_i + e_i.  Given the
row-wise relative errors rho_i = ||e_i|| / ||z_i||, this module bounds the change of

    L = || N(Z_t Z_t^T) - N(Z_s Z_s^T) ||_F^2 / B^2,   N(G)_ij = G_ij / sum_j |G_ij|

(the reference's row L1 normalisation) without any linearisation:

  * Gram:  |dG_ij| = |<e_i,z_j> + <z_i,e_j> + <e_i,e_j>| <= (rho_i + rho_j + rho_i rho_j) n_i n_j
    =: D_ij  (Cauchy-Schwarz, n_i = ||z_i||);
  * row sums: |dr_i| <= sum_j D_ij =: D_i, so for D_i < r_i
    |N(G+dG)_ij - N(G)_ij| = |dG_ij r_i - G_ij dr_i| / (r_i (r_i + dr_i))
                          <= (D_ij r_i + |G_ij| D_i) / (r_i (r_i - D_i)) =: b_ij;
  * loss: with A = N(G_t), C = N(G_s) and a, c the perturbations (|a| <= b^t, |c| <= b^s),
    |L' - L| = |sum 2 (A - C)(a - c) + (a - c)^2| / B^2
            <= sum_ij [2 |A_ij - C_ij| (b^t_ij + b^s_ij) + (b^t_ij + b^s_ij)^2] / B^2.

Everything is evaluated in float64 on the oracle's own features.
"""
import numpy as np


def _gram(z):
    z = np.asarray(z, np.float64).reshape(z.shape[0], -1)
    return z @ z.T


def _row_bound(G, rho):
    n = np.sqrt(np.maximum(np.diag(G), 0.0))
    r = np.abs(G).sum(1)
    D = (rho[:, None] + rho[None, :] + rho[:, None] * rho[None, :]) * n[:, None] * n[None, :]
    Di = D.sum(1)
    if np.any(Di >= r):
        return None, r
    b = (D * r[:, None] + np.abs(G) * Di[:, None]) / (r * (r - Di))[:, None]
    return b, r


def spkd_term(Gs, Gt):
    """L from two (fp64) Grams, as framework.py:161-172 with batchmean."""
    A = Gt / np.abs(Gt).sum(1, keepdims=True)
    C = Gs / np.abs(Gs).sum(1, keepdims=True)
    return float(((A - C) ** 2).sum() / Gt.shape[0] ** 2)


def spkd_bound(Gs, Gt, rho_s, rho_t):
    """Upper bound on |L(perturbed) - L(exact)| for row relative errors rho_s, rho_t (scalars or
    per-row arrays).  Returns inf when a row's error could flip its normalisation (D_i >= r_i)."""
    B = Gt.shape[0]
    rho_s = np.broadcast_to(np.asarray(rho_s, np.float64), (B,))
    rho_t = np.broadcast_to(np.asarray(rho_t, np.float64), (B,))
    bs, rs = _row_bound(Gs, rho_s)
    bt, rt = _row_bound(Gt, rho_t)
    if bs is None or bt is None:
        return float("inf")
    A = Gt / rt[:, None]
    C = Gs / rs[:, None]
    bb = bs + bt
    return float((2 * np.abs(A - C) * bb + bb * bb).sum() / B ** 2)


def row_rel_err(approx, exact):
    """rho_i = ||approx_i - exact_i|| / ||exact_i|| per sample (float64)."""
    a = np.asarray(approx, np.float64).reshape(approx.shape[0], -1)
    e = np.asarray(exact, np.float64).reshape(exact.shape[0], -1)
    return np.sqrt(((a - e) ** 2).sum(1) / np.maximum((e ** 2).sum(1), 1e-300))
