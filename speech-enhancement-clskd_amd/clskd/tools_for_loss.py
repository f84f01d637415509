"""tools_for_loss.py drop-in for the hot path: l2_norm-based SI-SNR (tools_for_loss.py:22-47)."""
import torch

from . import ops


def si_snr(s1, s2, eps=1e-8):
    """Mean over rows of 10*log10(||s_t||^2 / (||e||^2 + eps) + eps), no DC removal
    (tools_for_loss.py:37-47).  Computed by clskd_sisnr_rows + clskd_sum_f32 on the device."""
    rows = ops.sisnr_rows(s1, s2, eps)
    out = torch.empty((), dtype=torch.float32, device=rows.device)
    return ops.sum_f32(rows, out, 1.0 / rows.numel())


def si_snr_rows(s1, s2, eps=1e-8):
    return ops.sisnr_rows(s1, s2, eps)
