"""CPU oracle: an fp32 PyTorch-CPU restatement of the reference hot path, op for op.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / CPU baseline.  The product
path (``speech-enhancement-clskd_amd/clskd``) never imports it and has no CPU fallback.

Pinned by ``tests/golden/*.npz`` (written by ``tests/golden/gen_golden.py`` from the reference
itself, imported in this container) — see ``tests/test_oracle_golden.py``.

Everything is functional over a ``params`` dict keyed by the reference ``state_dict`` keys
(``clskd.weights.recipe_state_dict``).  Citations are file:line into the reference.
"""
import numpy as np
import torch
import torch.nn.functional as F
from scipy.signal import get_window


# --------------------------------------------------------------------------------------------
# ConvSTFT / ConviSTFT  (tools_for_model.py:15-109)
# --------------------------------------------------------------------------------------------
def init_kernels(win_len=400, win_inc=100, fft_len=512, win_type="hamming", invers=False):
    """tools_for_model.py:15-32: rfft(eye(N))[:win_len] real||imag, (pinv for inverse) * window."""
    window = get_window(win_type, win_len, fftbins=True)
    fourier_basis = np.fft.rfft(np.eye(fft_len))[:win_len]
    kernel = np.concatenate([np.real(fourier_basis), np.imag(fourier_basis)], 1).T
    if invers:
        kernel = np.linalg.pinv(kernel).T
    kernel = kernel * window
    return (torch.from_numpy(kernel[:, None, :].astype(np.float32)),
            torch.from_numpy(window[None, :, None].astype(np.float32)))


_KCACHE = {}


def _kernels():
    if "k" not in _KCACHE:
        fwd, _ = init_kernels()
        inv, win = init_kernels(invers=True)
        _KCACHE["k"] = (fwd, inv, win)
    return _KCACHE["k"]


def conv_stft(x, win_len=400, win_inc=100):
    """tools_for_model.py:53-67 ('complex'): zero pad win-hop both sides, conv1d stride hop."""
    fwd, _, _ = _kernels()
    if x.dim() == 2:
        x = x.unsqueeze(1)
    x = F.pad(x, [win_len - win_inc, win_len - win_inc])
    return F.conv1d(x, fwd, stride=win_inc)


def conv_istft(spec, win_len=400, win_inc=100):
    """tools_for_model.py:90-109: conv_transpose1d with pinv kernel / (OLA(window^2)+1e-8), trim."""
    _, inv, win = _kernels()
    out = F.conv_transpose1d(spec, inv, stride=win_inc)
    t = win.repeat(1, 1, spec.size(-1)) ** 2
    enframe = torch.eye(win_len)[:, None, :]
    coff = F.conv_transpose1d(t, enframe, stride=win_inc)
    out = out / (coff + 1e-8)
    return out[..., win_len - win_inc:-(win_len - win_inc)]


# --------------------------------------------------------------------------------------------
# complex layers  (tools_for_model.py:138-330)
# --------------------------------------------------------------------------------------------
def complex_conv2d(x, p, pre):
    """tools_for_model.py:236-262: causal time pad [1,0]; four real convs; real=rr-ii, imag=ri+ir."""
    x = F.pad(x, [1, 0, 0, 0])
    r, i = torch.chunk(x, 2, 1)
    wr, br = p[pre + "real_conv.weight"], p[pre + "real_conv.bias"]
    wi, bi = p[pre + "imag_conv.weight"], p[pre + "imag_conv.bias"]
    conv = lambda z, w, b: F.conv2d(z, w, b, stride=(2, 1), padding=(2, 0))
    real = conv(r, wr, br) - conv(i, wi, bi)
    imag = conv(r, wi, bi) + conv(i, wr, br)
    return torch.cat([real, imag], 1)


def complex_conv_transpose2d(x, p, pre):
    """tools_for_model.py:303-330 with ConvTranspose2d(k=(5,2), s=(2,1), p=(2,0), op=(1,0))."""
    r, i = torch.chunk(x, 2, 1)
    wr, br = p[pre + "real_conv.weight"], p[pre + "real_conv.bias"]
    wi, bi = p[pre + "imag_conv.weight"], p[pre + "imag_conv.bias"]
    convt = lambda z, w, b: F.conv_transpose2d(z, w, b, stride=(2, 1), padding=(2, 0),
                                               output_padding=(1, 0))
    real = convt(r, wr, br) - convt(i, wi, bi)
    imag = convt(r, wi, bi) + convt(i, wr, br)
    return torch.cat([real, imag], 1)


def complex_cat(inputs, axis=1):
    """tools_for_model.py:181-190: concatenate real halves, then imag halves."""
    reals, imags = zip(*[torch.chunk(z, 2, axis) for z in inputs])
    return torch.cat([torch.cat(reals, axis), torch.cat(imags, axis)], axis)


def batch_norm(x, p, pre, train, momentum=0.1, eps=1e-5, update_stats=False):
    """nn.BatchNorm2d semantics (DCCRN.py:80,124): train -> batch stats (biased var)."""
    rm, rv = p[pre + "running_mean"], p[pre + "running_var"]
    if update_stats:
        return F.batch_norm(x, rm, rv, p[pre + "weight"], p[pre + "bias"], train, momentum, eps)
    return F.batch_norm(x, rm.clone(), rv.clone(), p[pre + "weight"], p[pre + "bias"], train,
                        momentum, eps)


def prelu(x, alpha):
    return F.prelu(x, alpha)


def lstm(x, w_ih, w_hh, b_ih, b_hh):
    """nn.LSTM(1 layer, unidirectional, batch_first=False), zero initial state.  x [T,B,D]."""
    Tn, Bn, _ = x.shape
    H = w_hh.shape[1]
    gx = torch.matmul(x, w_ih.t()) + b_ih + b_hh
    h = x.new_zeros(Bn, H)
    c = x.new_zeros(Bn, H)
    out = []
    for t in range(Tn):
        g = gx[t] + torch.matmul(h, w_hh.t())
        i, f, gg, o = torch.chunk(g, 4, 1)
        i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
        c = f * c + i * gg
        h = o * torch.tanh(c)
        out.append(h)
    return torch.stack(out, 0)


def lstm_torch(x, w_ih, w_hh, b_ih, b_hh):
    """Same as ``lstm`` through torch's own nn.LSTM kernel (what the reference calls)."""
    m = torch.nn.LSTM(w_ih.shape[1], w_hh.shape[1], num_layers=1, batch_first=False)
    with torch.no_grad():
        m.weight_ih_l0.copy_(w_ih)
        m.weight_hh_l0.copy_(w_hh)
        m.bias_ih_l0.copy_(b_ih)
        m.bias_hh_l0.copy_(b_hh)
    return m(x)[0]


def naive_complex_lstm(real, imag, p, pre, project, lstm_fn=lstm_torch):
    """tools_for_model.py:159-174: real=R(r)-I(i), imag=R(i)+I(r); optional Linear per part."""
    R = [p[pre + "real_lstm." + k] for k in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    I = [p[pre + "imag_lstm." + k] for k in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    r2r = lstm_fn(real, *R)
    r2i = lstm_fn(real, *I)
    i2r = lstm_fn(imag, *R)
    i2i = lstm_fn(imag, *I)
    real_out = r2r - i2i
    imag_out = i2r + r2i
    if project:
        real_out = F.linear(real_out, p[pre + "r_trans.weight"], p[pre + "r_trans.bias"])
        imag_out = F.linear(imag_out, p[pre + "i_trans.weight"], p[pre + "i_trans.bias"])
    return real_out, imag_out


# --------------------------------------------------------------------------------------------
# DCCRN.forward  (DCCRN.py:149-240)
# --------------------------------------------------------------------------------------------
def dccrn_forward(p, inputs, train=True, n_layers=6, rnn_layers=2, fft_len=512,
                  lstm_fn=lstm_torch, update_stats=False):
    """Returns dict with outputs (mask_real, mask_imag, real, imag, out_wav) and the taps:
    enc (6 encoder block outputs), dec (6 decoder block outputs before [...,1:]) and the
    enhance output (real, imag) [T,B,D] (feature_extraction.py:3-50 hooks)."""
    specs = conv_stft(inputs)
    real = specs[:, :fft_len // 2 + 1]
    imag = specs[:, fft_len // 2 + 1:]
    spec_mags = torch.sqrt(real ** 2 + imag ** 2 + 1e-8)
    spec_phase = torch.atan2(imag, real)
    cspecs = torch.stack([real, imag], 1)[:, :, 1:]
    out = cspecs
    enc = []
    for i in range(n_layers):
        pre = f"encoder.{i}."
        out = complex_conv2d(out, p, pre + "0.")
        out = batch_norm(out, p, pre + "1.", train, update_stats=update_stats)
        out = prelu(out, p[pre + "2.weight"])
        enc.append(out)
    B, C, D, L = out.shape
    out = out.permute(3, 0, 1, 2)
    r_in = torch.reshape(out[:, :, :C // 2], [L, B, C // 2 * D])
    i_in = torch.reshape(out[:, :, C // 2:], [L, B, C // 2 * D])
    for li in range(rnn_layers):
        r_in, i_in = naive_complex_lstm(r_in, i_in, p, f"enhance.{li}.", li == rnn_layers - 1,
                                        lstm_fn=lstm_fn)
    clstm = (r_in, i_in)
    r_rnn = torch.reshape(r_in, [L, B, C // 2, D])
    i_rnn = torch.reshape(i_in, [L, B, C // 2, D])
    out = torch.cat([r_rnn, i_rnn], 2).permute(1, 2, 3, 0)
    lstm_out = out
    dec = []
    for d in range(n_layers):
        out = complex_cat([out, enc[-1 - d]], 1)
        pre = f"decoder.{d}."
        out = complex_conv_transpose2d(out, p, pre + "0.")
        if d != n_layers - 1:
            out = batch_norm(out, p, pre + "1.", train, update_stats=update_stats)
            out = prelu(out, p[pre + "2.weight"])
        dec.append(out)
        out = out[..., 1:]
    mask_real = F.pad(out[:, 0], [0, 0, 1, 0])
    mask_imag = F.pad(out[:, 1], [0, 0, 1, 0])
    # masking_mode 'E' (DCCRN.py:212-226)
    mask_mags = (mask_real ** 2 + mask_imag ** 2) ** 0.5
    real_phase = mask_real / (mask_mags + 1e-8)
    imag_phase = mask_imag / (mask_mags + 1e-8)
    mask_phase = torch.atan2(imag_phase, real_phase)
    mask_mags = torch.tanh(mask_mags)
    est_mags = mask_mags * spec_mags
    est_phase = spec_phase + mask_phase
    real = est_mags * torch.cos(est_phase)
    imag = est_mags * torch.sin(est_phase)
    out_spec = torch.cat([real, imag], 1)
    out_wav = torch.squeeze(conv_istft(out_spec), 1)
    out_wav = torch.clamp(out_wav, -1, 1)
    return dict(mask_real=mask_real, mask_imag=mask_imag, real=real, imag=imag, out_wav=out_wav,
                enc=enc, dec=dec, clstm=clstm, lstm_out=lstm_out, specs=specs)


# --------------------------------------------------------------------------------------------
# losses  (framework.py:16-172, tools_for_loss.py:22-47)
# --------------------------------------------------------------------------------------------
def stft_mag(x, fft_size, hop_size, win_length, window):
    """framework.py:16-32 (torch>=2 form): |STFT| clamped at 1e-7, transposed [B, frames, bins]."""
    s = torch.stft(x, fft_size, hop_size, win_length, window, return_complex=True)
    s = torch.view_as_real(s)
    return torch.sqrt(torch.clamp(s[..., 0] ** 2 + s[..., 1] ** 2, min=1e-7)).transpose(2, 1)


def mrstft_loss(x, y, fft_sizes=(512,), hop_sizes=(100,), win_lengths=(400,), factor_sc=0.1,
                factor_mag=0.1):
    """framework.py:104-146 (+ STFTLoss :85-101, SC :40-50, LogMag :58-68)."""
    sc = 0.0
    mag = 0.0
    for fs, ss, wl in zip(fft_sizes, hop_sizes, win_lengths):
        w = torch.hann_window(wl)
        xm = stft_mag(x, fs, ss, wl, w)
        ym = stft_mag(y, fs, ss, wl, w)
        sc = sc + torch.norm(ym - xm, p="fro") / torch.norm(ym, p="fro")
        mag = mag + F.l1_loss(torch.log(ym), torch.log(xm))
    sc = sc / len(fft_sizes)
    mag = mag / len(fft_sizes)
    return factor_sc * sc, factor_mag * mag


def spkd_gram(z, dtype=None):
    """framework.py:155-157: G = normalize(z z^T, 1) over flatten(z,1).

    NB the reference passes ``1`` positionally to ``torch.nn.functional.normalize(input, p, dim)``,
    i.e. p=1 along the default dim=1: rows are L1-normalised (G_ij / max(sum_j |G_ij|, 1e-12)),
    not L2.  Pinned by tests/golden/losses.npz and clskd_step.npz."""
    z = torch.flatten(z, 1)
    if dtype is not None:
        z = z.to(dtype)
    return F.normalize(torch.matmul(z, torch.t(z)), p=1, dim=1)


def spkd_loss(student, teacher, reduction="batchmean", dtype=None):
    """framework.py:150-172: ||G_t - G_s||_F^2 (/ B^2 for batchmean).

    dtype=torch.float64 evaluates the same math exactly enough to serve as the parity reference at
    full size: the reference's fp32 matmul over K ~ 2.6M elements carries ~1e-3 relative error in
    the loss (measured, tests/diag_spkd_precision.py)."""
    g_t = spkd_gram(teacher, dtype)
    g_s = spkd_gram(student, dtype)
    loss = torch.norm(g_t - g_s) ** 2
    b = teacher.shape[0]
    return loss / (b ** 2) if reduction == "batchmean" else loss


def l2_norm(s1, s2):
    """tools_for_loss.py:22-27."""
    return torch.sum(s1 * s2, -1, keepdim=True)


def si_snr(s1, s2, eps=1e-8):
    """tools_for_loss.py:37-47 (no DC removal)."""
    s1_s2 = l2_norm(s1, s2)
    s2_s2 = l2_norm(s2, s2)
    s_target = s1_s2 / (s2_s2 + eps) * s2
    e_noise = s1 - s_target
    snr = 10 * torch.log10(l2_norm(s_target, s_target) / (l2_norm(e_noise, e_noise) + eps) + eps)
    return torch.mean(snr)


def si_snr_rows(s1, s2, eps=1e-8):
    """Per-row values of ``si_snr`` before the mean."""
    s1_s2 = l2_norm(s1, s2)
    s2_s2 = l2_norm(s2, s2)
    s_target = s1_s2 / (s2_s2 + eps) * s2
    e_noise = s1 - s_target
    return (10 * torch.log10(l2_norm(s_target, s_target) / (l2_norm(e_noise, e_noise) + eps)
                             + eps))[..., 0]


# --------------------------------------------------------------------------------------------
# ReviewKD / ABF  (framework.py:176-284)
# --------------------------------------------------------------------------------------------
def abf_forward(p, pre, x, y=None, shape=None, out_shape=None, fuse=False):
    """framework.py:205-222.  BN layers are fresh modules in train mode (batch statistics)."""
    n, _, h, w = x.shape
    x = F.conv2d(x, p[pre + "conv1.0.weight"])
    x = batch_norm(x, p, pre + "conv1.1.", True)
    if fuse:
        y = F.interpolate(y, (shape, w), mode="nearest")
        z = torch.cat([x, y], 1)
        z = torch.sigmoid(F.conv2d(z, p[pre + "att_conv.0.weight"], p[pre + "att_conv.0.bias"]))
        x = x * z[:, 0].view(n, 1, h, w) + y * z[:, 1].view(n, 1, h, w)
    if x.shape[-1] != out_shape:
        x = F.interpolate(x, (out_shape, w), mode="nearest")
    out = F.conv2d(x, p[pre + "conv2.0.weight"], padding=1)
    out = batch_norm(out, p, pre + "conv2.1.", True)
    return out, x


def review_kd_forward(p, feature_maps, ft_type, shapes=(4, 8, 16, 32, 64, 128)):
    """framework.py:240-263 for build_review_kd(feature_maps, ft_type) (:266-284)."""
    pre = f"{ft_type}.abfs."
    n = len(feature_maps)
    xs = feature_maps[::-1] if ft_type == "encoder" else list(feature_maps)
    results = []
    out, res = abf_forward(p, pre + "0.", xs[0], out_shape=shapes[0])
    results.append(out)
    for j in range(1, n):
        out, res = abf_forward(p, pre + f"{j}.", xs[j], res, shapes[j], shapes[j], fuse=True)
        if ft_type == "encoder":
            results.insert(0, out)
        else:
            results.append(out)
    return results


# --------------------------------------------------------------------------------------------
# the CLSKD step  (distill.py:72-148) with the local DCCRN tap contract
# --------------------------------------------------------------------------------------------
def tap_contract(fwd):
    """Maps a dccrn_forward() result to the asteroid-equivalent taps used by distill.py:
    encoder = 6 encoder outputs; decoder = [LSTM output as [B,C,4,T], decoder outputs 0..4];
    clstm_real / clstm_img = enhance output halves transposed to batch-first [B,T,D]."""
    return dict(encoder=list(fwd["enc"]),
                decoder=[fwd["lstm_out"]] + list(fwd["dec"][:5]),
                clstm_real=fwd["clstm"][0].transpose(0, 1),
                clstm_img=fwd["clstm"][1].transpose(0, 1))


def clskd_step(pt, ps, pabf, X, y, lstm_fn=lstm_torch, gram_dtype=None):
    """distill.py:72-148 with local teacher/student.  Returns a dict of every loss term."""
    tf = dccrn_forward(pt, X, train=True, lstm_fn=lstm_fn)
    sf = dccrn_forward(ps, X, train=True, lstm_fn=lstm_fn)
    t = tap_contract(tf)
    s = tap_contract(sf)
    s_enc = review_kd_forward(pabf, s["encoder"], "encoder")
    s_dec = review_kd_forward(pabf, s["decoder"], "decoder")
    student_preds = sf["out_wav"]  # distill.py:100 (second student forward: identical output)
    base = mrstft_loss(student_preds.squeeze(), y.squeeze())[1]
    enc_terms = [spkd_loss(a, b, dtype=gram_dtype) for a, b in zip(s_enc, t["encoder"])]
    dec_terms = [spkd_loss(a, b, dtype=gram_dtype) for a, b in zip(s_dec, t["decoder"])]
    cr = spkd_loss(s["clstm_real"], t["clstm_real"], dtype=gram_dtype)
    ci = spkd_loss(s["clstm_img"], t["clstm_img"], dtype=gram_dtype)
    total = base + sum(enc_terms) + sum(dec_terms) + cr + ci
    return dict(total=total, base=base, enc=enc_terms, dec=dec_terms, clstm_real=cr,
                clstm_img=ci, student_wav=student_preds, teacher_wav=tf["out_wav"],
                s_enc=s_enc, s_dec=s_dec, t_taps=t, s_taps=s)


def spkd_output_step(pt, ps, X, y, lstm_fn=lstm_torch):
    """distill_SPKD.py:69-87: MRSTFT base + SPKD on the final waveforms."""
    s = dccrn_forward(ps, X, train=True, lstm_fn=lstm_fn)["out_wav"]
    with torch.no_grad():
        t = dccrn_forward(pt, X, train=True, lstm_fn=lstm_fn)["out_wav"]
    base = mrstft_loss(s.squeeze(), y.squeeze())[1]
    sp = spkd_loss(s, t)
    return dict(total=base + sp, base=base, spkd=sp)


def to_torch_params(d):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in d.items()}
