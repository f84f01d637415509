"""Model/loss constants and parameter-shape tables, mirroring the reference's ``config.py``.

Names follow ``config.py:22-48`` so ``import clskd.config as cfg`` reads like the reference.
``dccrn_param_shapes`` reproduces the reference ``DCCRN.state_dict()`` key order and shapes
(``DCCRN.py:63-147``; ``tools_for_model.py:138-330``) without importing the reference, so a
reference checkpoint loads key-for-key.
"""
from collections import OrderedDict

# STFT front end (config.py:22-31)
fs = 16000
win_len = 400
win_inc = 100
fft_len = 512
window_type = "hamming"

# teacher (config.py:33-38)
rnn_layers = 2
rnn_units = 256
masking_mode = "E"
use_clstm = True
kernel_num = [32, 64, 128, 256, 256, 256]
kernel_size = 5

# training (config.py:41-43)
max_epochs = 20
learning_rate = 0.0006
batch = 32

# student (config.py:46-48)
rnn_layers_student = 2
rnn_units_student = 64
kernel_num_student = [8, 16, 32, 64, 64, 64]

# CLSKD base loss: MultiResolutionSTFTLoss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100])
# (distill.py:58-59), hann window, factor 0.1.
mrstft_fft = 512
mrstft_hop = 100
mrstft_win = 400

# ReviewKD tables (framework.py:266-284)
REVIEW_IN = [8, 16, 32, 64, 64, 64]
REVIEW_OUT = [32, 64, 128, 256, 256, 256]
REVIEW_SHAPES = [4, 8, 16, 32, 64, 128]


def n_frames(num_samples, win=win_len, hop=win_inc):
    """ConvSTFT frame count: zero pad win-hop each side then stride hop (tools_for_model.py:61-62)."""
    return (num_samples + 2 * (win - hop) - win) // hop + 1


def dccrn_param_shapes(rnn_units, kernel_num, rnn_layers=2, ksize=5, fft=fft_len):
    """Ordered {state_dict key: shape} of the reference DCCRN (use_clstm=True, use_cbn=False)."""
    kn = [2] + list(kernel_num)
    s = OrderedDict()
    for i in range(len(kn) - 1):
        cin, cout = kn[i] // 2, kn[i + 1] // 2
        p = f"encoder.{i}."
        for part in ("real_conv", "imag_conv"):
            s[p + f"0.{part}.weight"] = (cout, cin, ksize, 2)
            s[p + f"0.{part}.bias"] = (cout,)
        for k in ("weight", "bias", "running_mean", "running_var"):
            s[p + f"1.{k}"] = (kn[i + 1],)
        s[p + "1.num_batches_tracked"] = ()
        s[p + "2.weight"] = (1,)
    hidden_dim = fft // (2 ** len(kn))
    feat = hidden_dim * kn[-1]
    enh = OrderedDict()  # registered after encoder/decoder ModuleLists (DCCRN.py:66-67 vs :88-99)
    for li in range(rnn_layers):
        p = f"enhance.{li}."
        din = (feat if li == 0 else rnn_units) // 2
        h = rnn_units // 2
        for part in ("real_lstm", "imag_lstm"):
            enh[p + f"{part}.weight_ih_l0"] = (4 * h, din)
            enh[p + f"{part}.weight_hh_l0"] = (4 * h, h)
            enh[p + f"{part}.bias_ih_l0"] = (4 * h,)
            enh[p + f"{part}.bias_hh_l0"] = (4 * h,)
        if li == rnn_layers - 1:
            for part in ("r_trans", "i_trans"):
                enh[p + f"{part}.weight"] = (feat // 2, h)
                enh[p + f"{part}.bias"] = (feat // 2,)
    for d, idx in enumerate(range(len(kn) - 1, 0, -1)):
        cin, cout = kn[idx] * 2 // 2, kn[idx - 1] // 2
        p = f"decoder.{d}."
        for part in ("real_conv", "imag_conv"):
            s[p + f"0.{part}.weight"] = (cin, cout, ksize, 2)  # ConvTranspose2d: [in, out, kh, kw]
            s[p + f"0.{part}.bias"] = (cout,)
        if idx != 1:
            for k in ("weight", "bias", "running_mean", "running_var"):
                s[p + f"1.{k}"] = (kn[idx - 1],)
            s[p + "1.num_batches_tracked"] = ()
            s[p + "2.weight"] = (1,)
    s.update(enh)
    return s


def review_param_shapes(ft_type, in_channels=REVIEW_IN, out_channels=REVIEW_OUT):
    """Ordered {key: shape} of ``build_review_kd(…, ft_type)`` (framework.py:176-284), keys prefixed
    with ``ft_type + '.'``.  ``abfs`` is reversed (framework.py:238), so ``abfs.0`` is the
    deepest level (in_channels[-1], no attention fuse)."""
    mid = min(512, in_channels[-1])
    n = len(in_channels)
    s = OrderedDict()
    for j in range(n):
        idx = n - 1 - j  # reversed list position j holds construction index idx
        cin, cout, fuse = in_channels[idx], out_channels[idx], idx < n - 1
        p = f"{ft_type}.abfs.{j}."
        s[p + "conv1.0.weight"] = (mid, cin, 1, 1)
        for k in ("weight", "bias", "running_mean", "running_var"):
            s[p + f"conv1.1.{k}"] = (mid,)
        s[p + "conv1.1.num_batches_tracked"] = ()
        s[p + "conv2.0.weight"] = (cout, mid, 3, 3)
        for k in ("weight", "bias", "running_mean", "running_var"):
            s[p + f"conv2.1.{k}"] = (cout,)
        s[p + "conv2.1.num_batches_tracked"] = ()
        if fuse:
            s[p + "att_conv.0.weight"] = (2, 2 * mid, 1, 1)
            s[p + "att_conv.0.bias"] = (2,)
    return s


TEACHER = dict(rnn_units=rnn_units, kernel_num=kernel_num)
STUDENT = dict(rnn_units=rnn_units_student, kernel_num=kernel_num_student)
