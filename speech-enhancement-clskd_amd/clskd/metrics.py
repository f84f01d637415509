"""Validation metrics of the CLSKD drop-in: SI-SDR and STOI on the device.

``KnowledgeDistillation.validation_step`` (distill.py:149-199) scores each utterance with
``asteroid.metrics.get_metrics(mix, clean, estimate, sample_rate=16000)`` restricted to
``COMPUTE_METRICS = ["si_sdr", "stoi"]`` (distill.py:35) and logs the batch means of
``si_sdr``, ``stoi`` and their improvements over the unprocessed mixture.  Those metrics come
from third-party code (pb_bss_eval's si_sdr, pystoi's stoi — the function the reference's own
``tools_for_model.cal_stoi`` calls, tools_for_model.py:595-600); here both run in
libclskd_hip.so (``clskd_sisdr_f64``, ``clskd_stoi``), batched over utterances, float64.
"""
import torch

from . import ops
from ._lib import check, ptr


def _rows(x):
    x = x.float()
    if x.dim() == 1:
        x = x.unsqueeze(0)
    x = x.reshape(-1, x.shape[-1])
    if x.stride(-1) != 1:
        x = x.contiguous()
    return x


def si_sdr(reference, estimation):
    """pb_bss_eval.evaluation.si_sdr per row (float64 tensor [rows]): scale-invariant SDR in dB,
    no mean removal, no eps (the tools_for_loss.py:50-92 formula)."""
    r, e = _rows(reference), _rows(estimation)
    if r.shape != e.shape:
        raise ValueError(f"si_sdr: shapes {tuple(r.shape)} and {tuple(e.shape)} differ")
    out = torch.empty(r.shape[0], device=r.device, dtype=torch.float64)
    check(ops.lib().clskd_sisdr_f64(ptr(r), ptr(e), r.shape[0], r.shape[1], r.stride(0),
                                    e.stride(0), ptr(out), ops._stream()), "sisdr_f64")
    return out


def stoi(x, y, fs_sig, extended=False):
    """pystoi.stoi(clean x, processed y, fs_sig) per row (float64 tensor [rows]); the classic
    measure only (the reference calls it with extended=False)."""
    if extended:
        raise NotImplementedError("extended STOI is not used by the reference (extended=False)")
    c, e = _rows(x), _rows(y)
    if c.shape != e.shape:
        raise Exception("x and y should have the same length")
    L = ops.lib()
    B, n = c.shape
    nbytes = int(L.clskd_stoi_workspace(B, n, int(fs_sig)))
    if nbytes < 0:
        raise ValueError("stoi: bad shape")
    ws = torch.empty(nbytes, device=c.device, dtype=torch.uint8)
    out = torch.empty(B, device=c.device, dtype=torch.float64)
    check(L.clskd_stoi(ptr(c), ptr(e), B, n, c.stride(0), e.stride(0), int(fs_sig), ptr(ws),
                       nbytes, ptr(out), ops._stream()), "stoi")
    return out


def cal_stoi(dirty_wavs, clean_wavs, fs=16000):
    """tools_for_model.py:595-600: STOI of each processed row against its clean row."""
    return stoi(clean_wavs, dirty_wavs, fs).tolist()


COMPUTE_METRICS = ["si_sdr", "stoi"]


def get_metrics(mix, clean, estimate, sample_rate=16000, metrics_list=COMPUTE_METRICS):
    """asteroid.metrics.get_metrics for single-source rows: {"input_<m>": [rows], "<m>": [rows]}
    (float64 tensors on the device) for m in metrics_list ("si_sdr", "stoi")."""
    out = {}
    for m in metrics_list:
        if m == "si_sdr":
            out["input_si_sdr"] = si_sdr(clean, mix)
            out["si_sdr"] = si_sdr(clean, estimate)
        elif m == "stoi":
            out["input_stoi"] = stoi(clean, mix, sample_rate)
            out["stoi"] = stoi(clean, estimate, sample_rate)
        else:
            raise NotImplementedError(f"metric {m!r} is not on the reference's validation path")
    return out


def summarize(utt_metrics, metrics_list=COMPUTE_METRICS):
    """distill.py:185-192: batch means of each metric and of its improvement over the input."""
    res = {}
    for m in metrics_list:
        res[m] = utt_metrics[m].mean()
        res[m + "_imp"] = (utt_metrics[m] - utt_metrics["input_" + m]).mean()
    return res
