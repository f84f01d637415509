"""Import-time shims that let the reference's local-DCCRN path import in THIS container.

Used only by ``gen_golden.py`` (fixture generation, never on the GPU box).  SURVEY.md §8 c:
  1. stub modules for asteroid / asteroid_filterbanks / pesq / pystoi — only touched at import
     (DCCRN.py:11, tools_for_loss.py:5-6,258-259, tools_for_model.py:8-9);
  2. ``torch.stft`` without ``return_complex`` -> ``view_as_real(stft(..., return_complex=True))``
     (framework.py:27 predates torch 2);
  3. ``nn.Module.cuda`` / ``Tensor.cuda`` -> identity (framework.py:198-202; no GPU here).
"""
import sys
import types

REFERENCE = "/root/reference"


class _Dummy:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return None


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install():
    sys.dont_write_bytecode = True
    import torch
    import torch.nn as nn

    _stub("asteroid")
    _stub("asteroid.losses", SingleSrcPMSQE=_Dummy, PITLossWrapper=_Dummy)
    tr = _stub("asteroid_filterbanks.transforms")
    _stub("asteroid_filterbanks", STFTFB=_Dummy, Encoder=_Dummy, transforms=tr)
    _stub("pesq", pesq=lambda *a, **k: 0.0)
    _stub("pystoi", stoi=lambda *a, **k: 0.0)

    if not getattr(torch.stft, "_clskd_shim", False):
        _orig = torch.stft

        def stft(x, n_fft, hop_length=None, win_length=None, window=None, *a, **k):
            if "return_complex" not in k:
                k["return_complex"] = True
                return torch.view_as_real(_orig(x, n_fft, hop_length, win_length, window, *a, **k))
            return _orig(x, n_fft, hop_length, win_length, window, *a, **k)

        stft._clskd_shim = True
        torch.stft = stft

    nn.Module.cuda = lambda self, *a, **k: self
    torch.Tensor.cuda = lambda self, *a, **k: self
    if REFERENCE not in sys.path:
        sys.path.insert(0, REFERENCE)
