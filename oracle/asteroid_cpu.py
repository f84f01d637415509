"""CPU oracle of the asteroid ``DCCRNet_mini`` ('DCCRN-CL-test') forward, as the reference's
eval script runs it (eval.py:37-101) — fp32 PyTorch-CPU restatement.

TEST INFRASTRUCTURE ONLY (same contract as ``oracle/ref_cpu.py``).

The model class lives in an un-vendored asteroid fork (asteroid_version '0.6.1dev', absent).
Its structure is read off the reference's own artefacts: the 182 ``state_dict`` keys and shapes
of checkpoint/the_best_model.pth and the module print-out in test-asteroid.ipynb (cells 22, 27,
39): STFTFB encoder (conv1d, no padding) -> Nyquist bin dropped -> 6 DCUNetComplexEncoderBlocks
(ComplexConv2d (5,2) stride (2,1) padding (2,0), OnReIm BatchNorm2d, OnReIm PReLU) ->
DCCRMaskNetRNN_mini (2 per-layer complex LSTMs 128->32->32, batch-first, complex Linear 32->128)
-> Identity + 5 DCUNetComplexDecoderBlocks (ComplexConvTranspose2d output_padding (1,0)) with
BaseUNet skips cat([x, enc_out]) -> ComplexConvTranspose2d (with bias) -> BoundComplexMask('tanh')
-> mask * spectrum, Nyquist re-padded with 0 -> STFTFB decoder (conv_transpose1d).

Three choices the artefacts leave open were settled against the reference's own outputs, the
five example_CLSKD/*/s0_estimate.wav (tests/test_asteroid_oracle.py):
  * BatchNorm runs in TRAIN mode: eval.py builds the model with ``from_pretrained`` and never
    calls ``.eval()`` (eval.py:39), so every utterance is normalised by its own statistics;
  * the RNN block has no residual connection; the mask bound is 'tanh' (|M| -> tanh |M|);
  * eval.py's ``normalize_estimates`` (peak of the estimate set to the mixture's peak) and
    soundfile's float->PCM16 conversion (reproduced as floor(x * 32768)) give the int16 files.
With those, this restatement reproduces the shipped int16 estimates to within 2 LSB, >= 99 % of
samples bit-exact.
"""
import numpy as np
import torch
import torch.nn.functional as F

ENC = [(1, 4), (4, 8), (8, 16), (16, 32), (32, 32), (32, 32)]   # complex channels in, out
DEC = [(64, 32), (64, 32), (64, 16), (32, 8), (16, 4)]          # decoders 1..5
OUT = (8, 1)


def stftfb_filters(n_filters=512, kernel_size=400, stride=100):
    """asteroid_filterbanks.STFTFB filters [n+2, 1, kernel] (sqrt-Hann window, DFT rows scaled by
    1 / (0.5 sqrt(kernel n / stride)), DC and Nyquist rows / sqrt 2) — equals the checkpoint's
    ``encoder.filterbank._filters`` to 2e-9."""
    window = np.hanning(kernel_size + 1)[:-1] ** 0.5
    f = np.fft.fft(np.eye(n_filters))
    f /= 0.5 * np.sqrt(kernel_size * n_filters / stride)
    lpad = (n_filters - kernel_size) // 2
    idx = list(range(lpad, lpad + kernel_size))
    cut = n_filters // 2 + 1
    f = np.vstack([np.real(f[:cut, idx]), np.imag(f[:cut, idx])])
    f[0, :] /= np.sqrt(2)
    f[n_filters // 2, :] /= np.sqrt(2)
    return torch.from_numpy((f * window)[:, None, :].astype(np.float32))


def _cconv(xr, xi, sd, pre, transpose=False, **kw):
    """ComplexMultiplicationWrapper: re = R(xr) - I(xi), im = R(xi) + I(xr) (biases included)."""
    wr, wi = sd[pre + "re_module.weight"], sd[pre + "im_module.weight"]
    br, bi = sd.get(pre + "re_module.bias"), sd.get(pre + "im_module.bias")
    f = F.conv_transpose2d if transpose else F.conv2d
    return f(xr, wr, br, **kw) - f(xi, wi, bi, **kw), f(xi, wr, br, **kw) + f(xr, wi, bi, **kw)


def _bn(x, sd, pre, train):
    if train:
        return F.batch_norm(x, None, None, sd[pre + "weight"], sd[pre + "bias"], True, 0.1, 1e-5)
    return F.batch_norm(x, sd[pre + "running_mean"], sd[pre + "running_var"], sd[pre + "weight"],
                        sd[pre + "bias"], False, 0.1, 1e-5)


def _lstm(x, sd, pre):
    """nn.LSTM(batch_first=True), one layer, zero initial state: gates i, f, g, o."""
    wih, whh = sd[pre + "weight_ih_l0"], sd[pre + "weight_hh_l0"]
    b = sd[pre + "bias_ih_l0"] + sd[pre + "bias_hh_l0"]
    H = whh.shape[1]
    B, T, _ = x.shape
    gx = x @ wih.t() + b
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    out = []
    for t in range(T):
        g = gx[:, t] + h @ whh.t()
        i, f, gg, o = g.split(H, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        out.append(h)
    return torch.stack(out, 1)


def forward(sd, wav, train=True):
    """DCCRNet_mini forward: wav [B, L] -> estimate [B, L] (asteroid returns [B, 1, L])."""
    sd = {k: torch.as_tensor(v) for k, v in sd.items()}
    filt = sd["encoder.filterbank._filters"]
    spec = F.conv1d(wav[:, None], filt, stride=100)  # [B, 514, T]
    re, im = spec[:, :257], spec[:, 257:]
    xr, xi = re[:, None, :-1], im[:, None, :-1]     # DCCRNet.forward_encoder: Nyquist dropped
    enc = []
    for i in range(len(ENC)):
        p = f"masker.encoders.{i}."
        xr, xi = _cconv(xr, xi, sd, p + "conv.", stride=(2, 1), padding=(2, 0))
        xr = F.prelu(_bn(xr, sd, p + "norm.re_module.", train), sd[p + "activation.re_module.weight"])
        xi = F.prelu(_bn(xi, sd, p + "norm.im_module.", train), sd[p + "activation.im_module.weight"])
        enc.append((xr, xi))
    # DCCRMaskNetRNN_mini: [B, C, F, T] -> [B, T, C*F] -> 2 complex LSTM layers -> complex Linear
    B, C, Fq, T = xr.shape
    r = xr.permute(0, 3, 1, 2).reshape(B, T, C * Fq)
    i_ = xi.permute(0, 3, 1, 2).reshape(B, T, C * Fq)
    for l in range(2):
        p = f"masker.encoders.6.rnn.rnns.{l}."
        rr, ii = _lstm(r, sd, p + "re_module.rnn."), _lstm(i_, sd, p + "im_module.rnn.")
        ri, ir = _lstm(i_, sd, p + "re_module.rnn."), _lstm(r, sd, p + "im_module.rnn.")
        r, i_ = rr - ii, ri + ir
    p = "masker.encoders.6.linear."
    Lr = lambda z: F.linear(z, sd[p + "re_module.weight"], sd[p + "re_module.bias"])  # noqa: E731
    Li = lambda z: F.linear(z, sd[p + "im_module.weight"], sd[p + "im_module.bias"])  # noqa: E731
    lr, li = Lr(r) - Li(i_), Lr(i_) + Li(r)
    xr = lr.reshape(B, T, C, Fq).permute(0, 2, 3, 1)
    xi = li.reshape(B, T, C, Fq).permute(0, 2, 3, 1)
    # BaseUNet decoders [Identity, 1..5]: x = dec(x); x = cat([x, enc_out]) over reversed encoders
    for d in range(len(DEC) + 1):
        if d > 0:
            p = f"masker.decoders.{d}."
            xr, xi = _cconv(xr, xi, sd, p + "deconv.", transpose=True, stride=(2, 1),
                            padding=(2, 0), output_padding=(1, 0))
            xr = F.prelu(_bn(xr, sd, p + "norm.re_module.", train), sd[p + "activation.re_module.weight"])
            xi = F.prelu(_bn(xi, sd, p + "norm.im_module.", train), sd[p + "activation.im_module.weight"])
        er, ei = enc[len(ENC) - 1 - d]
        xr, xi = torch.cat([xr, er], 1), torch.cat([xi, ei], 1)
    mr, mi = _cconv(xr, xi, sd, "masker.output_layer.0.", transpose=True, stride=(2, 1),
                    padding=(2, 0), output_padding=(1, 0))
    # BoundComplexMask('tanh'): tanh(|M|) e^{i angle M}; DCCRNet.apply_masks: M * X, pad Nyquist
    mag = torch.tanh(torch.sqrt(mr ** 2 + mi ** 2))
    ph = torch.atan2(mi, mr)
    mr, mi = (mag * torch.cos(ph))[:, 0], (mag * torch.sin(ph))[:, 0]
    sr, si = re[:, :-1], im[:, :-1]
    er_, ei_ = mr * sr - mi * si, mr * si + mi * sr
    z = torch.zeros_like(er_[:, :1])
    est = torch.cat([er_, z, ei_, z], 1)
    out = F.conv_transpose1d(est, sd["decoder.filterbank._filters"], stride=100)[:, 0]
    L = wav.shape[-1]
    if out.shape[-1] < L:  # pad_x_to_y
        out = F.pad(out, (0, L - out.shape[-1]))
    return out[:, :L]


def state_dict_from_fixture(fx):
    """The checkpoint's state_dict from tests/golden/asteroid_mini.npz (decoder filterbank =
    encoder filterbank, stored once)."""
    sd = {k[2:]: torch.from_numpy(fx[k]) for k in fx.files if k.startswith("w/")}
    for k in ("_filters", "torch_window"):
        sd["decoder.filterbank." + k] = sd["encoder.filterbank." + k]
    return sd


def normalize_estimates(est, mix):
    """asteroid.dsp.normalization.normalize_estimates for one source: peak -> mixture peak."""
    return est * np.max(np.abs(mix)) / np.max(np.abs(est))


def to_pcm16(x):
    """soundfile float -> PCM_16 as the shipped WAVs show it: floor(x * 32768)."""
    return np.floor(np.asarray(x, np.float64) * 32768.0).astype(np.int64)


def mixture_from_wav(mix_i16):
    """eval.py wrote the mixture it read (LibriMix, int16 / 32768) back through soundfile: the
    stored ints are the originals up to the PCM scaling; the model input is int16 / 32768."""
    return np.asarray(mix_i16, np.float32) / 32768.0
