"""asteroid-compatible ``DCCRNet_mini`` ('DCCRN-CL-test') on MI355X — the model class the reference
actually distils and evaluates (distill.py:245-247, eval.py:39; SURVEY.md §8 f rank 2).

The module tree reproduces the 182 ``state_dict`` keys of the reference's checkpoints
(checkpoint/the_best_model.pth, checkpoint_SPKD/SPKD_best_model.pth: asteroid ``serialize()``
dicts), so ``DCCRNet_mini.from_pretrained(path)`` loads them unchanged; the forward runs in
libclskd_hip.so on BFTC buffers with the kernels of ``clskd.DCCRN`` (implicit-GEMM complex
convs / polyphase transposed convs, fused BatchNorm statistics, the LSTM recurrence kernel).

Semantics (asteroid's DCCRNet, structure from the checkpoint and test-asteroid.ipynb; the open
points were settled against the reference's shipped estimates, see oracle/asteroid_cpu.py):
STFTFB analysis without padding (T = (L - 400) / 100 + 1), Nyquist bin dropped; six complex
encoder blocks (5x2 kernel, stride (2, 1), padding (2, 0): T shrinks by one per block;
re / im BatchNorm and PReLU); two per-layer complex LSTMs (batch-first) + complex Linear;
Identity + five complex decoder blocks (transposed 5x2, output padding (1, 0): T grows by one)
with skips cat([x, enc_out]); output transposed conv with bias; BoundComplexMask('tanh') times
the spectrum, Nyquist re-padded with 0; STFTFB synthesis (plain overlap-add); pad to L.
``model.train()`` (the default, and what eval.py runs: it never calls ``.eval()``) normalises
with batch statistics — ``enhance`` therefore processes one utterance per call like eval.py.
"""
import json

import numpy as np
import torch
import torch.nn as nn

from . import ops
from ._lib import check, ptr
from .ops import OutMap, Seg, SegGeom, seg_bftc

ARCHITECTURES = {
    # (encoders (in, out) complex channels, decoders 1..n (in, out), output (in, out), rnn hidden)
    "DCCRN-CL-test": ([(1, 4), (4, 8), (8, 16), (16, 32), (32, 32), (32, 32)],
                      [(64, 32), (64, 32), (64, 16), (32, 8), (16, 4)], (8, 1), 32),
}


def _pv(*ts):
    return tuple((t.data_ptr(), t._version) for t in ts)


class _ReIm(nn.Module):
    """asteroid complex_nn.ComplexMultiplicationWrapper / OnReIm: re_module, im_module."""

    def __init__(self, cls, *args, **kwargs):
        super().__init__()
        self.re_module = cls(*args, **kwargs)
        self.im_module = cls(*args, **kwargs)


class STFTFB(nn.Module):
    """asteroid_filterbanks.STFTFB buffers: ``_filters`` [n+2, 1, kernel], ``torch_window``."""

    def __init__(self, n_filters=512, kernel_size=400, stride=100):
        super().__init__()
        self.n_filters, self.kernel_size, self.stride = n_filters, kernel_size, stride
        window = np.hanning(kernel_size + 1)[:-1] ** 0.5
        f = np.fft.fft(np.eye(n_filters))
        f /= 0.5 * np.sqrt(kernel_size * n_filters / stride)
        lpad = (n_filters - kernel_size) // 2
        idx = list(range(lpad, lpad + kernel_size))
        cut = n_filters // 2 + 1
        f = np.vstack([np.real(f[:cut, idx]), np.imag(f[:cut, idx])])
        f[0, :] /= np.sqrt(2)
        f[n_filters // 2, :] /= np.sqrt(2)
        self.register_buffer("_filters", torch.from_numpy((f * window)[:, None, :].astype(np.float32)))
        self.register_buffer("torch_window", torch.from_numpy(window.astype(np.float32)))


class _FB(nn.Module):
    def __init__(self, *args):
        super().__init__()
        self.filterbank = STFTFB(*args)


class DCUNetComplexEncoderBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = _ReIm(nn.Conv2d, cin, cout, (5, 2), (2, 1), (2, 0), bias=False)
        self.norm = _ReIm(nn.BatchNorm2d, cout)
        self.activation = _ReIm(nn.PReLU)


class DCUNetComplexDecoderBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.deconv = _ReIm(nn.ConvTranspose2d, cin, cout, (5, 2), (2, 1), (2, 0), (1, 0),
                            bias=False)
        self.norm = _ReIm(nn.BatchNorm2d, cout)
        self.activation = _ReIm(nn.PReLU)


class _SingleRNN(nn.Module):
    def __init__(self, cin, hid):
        super().__init__()
        self.rnn = nn.LSTM(cin, hid, batch_first=True)


class ComplexSingleRNN(nn.Module):
    def __init__(self, cin, hid, n_layers=2):
        super().__init__()
        self.rnns = nn.ModuleList([_ReIm(_SingleRNN, cin if i == 0 else hid, hid)
                                   for i in range(n_layers)])


class DCCRMaskNetRNN_mini(nn.Module):
    def __init__(self, in_size, hid):
        super().__init__()
        self.rnn = ComplexSingleRNN(in_size, hid)
        self.linear = _ReIm(nn.Linear, hid, in_size)


class DCCRMaskNet_mini(nn.Module):
    def __init__(self, architecture, n_freqs=256):
        super().__init__()
        enc, dec, out, hid = ARCHITECTURES[architecture]
        f_last = n_freqs // 2 ** len(enc)
        self.encoders = nn.ModuleList([DCUNetComplexEncoderBlock(a, b) for a, b in enc]
                                      + [DCCRMaskNetRNN_mini(enc[-1][1] * f_last, hid)])
        self.decoders = nn.ModuleList([nn.Identity()] + [DCUNetComplexDecoderBlock(a, b)
                                                         for a, b in dec])
        self.output_layer = nn.Sequential(
            _ReIm(nn.ConvTranspose2d, out[0], out[1], (5, 2), (2, 1), (2, 0), (1, 0), bias=True))


class DCCRNet_mini(nn.Module):
    """asteroid.models.DCCRNet_mini: forward(wav [B, L] or [B, 1, L]) -> [B, 1, L]."""

    _DEC_TAPS = {0: ((0, 1), (2, 0), (4, -1)), 1: ((1, 1), (3, 0))}  # parity -> (kf, dF)

    def __init__(self, architecture="DCCRN-CL-test", stft_n_filters=512, stft_kernel_size=400,
                 stft_stride=100, sample_rate=16000.0, n_freqs=256, **masknet_kwargs):
        super().__init__()
        if architecture not in ARCHITECTURES:
            raise NotImplementedError(f"DCCRNet_mini architecture {architecture!r}: only "
                                      f"{sorted(ARCHITECTURES)} (the reference's checkpoints)")
        if (stft_n_filters, stft_kernel_size, stft_stride, n_freqs) != (512, 400, 100, 256):
            raise NotImplementedError("built for the reference's STFT 512 / 400 / 100, 256 bins")
        self.model_args = dict(architecture=architecture, stft_n_filters=stft_n_filters,
                               stft_kernel_size=stft_kernel_size, stft_stride=stft_stride,
                               sample_rate=sample_rate, n_freqs=n_freqs)
        self.encoder = _FB(stft_n_filters, stft_kernel_size, stft_stride)
        self.masker = DCCRMaskNet_mini(architecture, n_freqs)
        self.decoder = _FB(stft_n_filters, stft_kernel_size, stft_stride)
        self.sample_rate = sample_rate
        self._wcache = {}

    # ------------------------------------------------------------------ asteroid BaseModel API
    @classmethod
    def from_pretrained(cls, pretrained_model_conf_or_path, *args, **kwargs):
        """A serialize() dict or a path to one (loaded with weights_only=True)."""
        conf = pretrained_model_conf_or_path
        if isinstance(conf, str):
            torch.serialization.add_safe_globals([torch.torch_version.TorchVersion])
            conf = torch.load(conf, map_location="cpu", weights_only=True)
        model = cls(*args, **conf["model_args"], **kwargs)
        model.load_state_dict(conf["state_dict"])
        return model

    def serialize(self):
        return dict(model_name=type(self).__name__, state_dict=self.state_dict(),
                    model_args=dict(self.model_args), infos={})

    # ------------------------------------------------------------------ packed operands
    def _packed(self, key, params, build):
        ent = self._wcache.get(key)
        ver = _pv(*params)
        tok = ops.capture_token()  # entries built inside a capture serve that capture only
        if ent is None or ent[0] != ver or not ops.cache_entry_usable(ent[2], tok):
            with torch.no_grad():
                ent = (ver, build(), tok)
            self._wcache[key] = ent
        ops.capture_keep(ent[1], tok)
        return ent[1]

    def _enc_w(self, i):
        cc = self.masker.encoders[i].conv

        def build():
            wr, wi = cc.re_module.weight, cc.im_module.weight  # [Co, Ci, 5, 2]
            w = torch.cat([torch.cat([wr, -wi], 1), torch.cat([wi, wr], 1)], 0)
            Co, Ci = w.shape[:2]
            return ops.pack_weight(w.permute(0, 2, 3, 1).reshape(Co, 10, Ci), 10 * Ci)
        return self._packed(("enc", i), (cc.re_module.weight, cc.im_module.weight), build)

    def _dec_w(self, mod, parity, nprev):
        """Transposed complex conv of a decoder (or the output layer): input channels per part
        [prev (nprev), skip]; K per tap [prev (re, im), skip (re, im)]; bias br - bi | br + bi."""
        rm, im_ = mod.re_module, mod.im_module

        def build():
            wr, wi = rm.weight, im_.weight  # [Ci, Co, 5, 2]
            top = torch.cat([wr, wi], 1)    # real input -> [real out | imag out]
            bot = torch.cat([-wi, wr], 1)   # imag input -> [real out | imag out]
            w = torch.cat([top, bot], 0)    # rows [prev_re, skip_re, prev_im, skip_im]
            ci = wr.shape[0]
            ns = ci - nprev
            w = torch.cat([w[0:nprev], w[ci:ci + nprev], w[nprev:ci], w[ci + nprev:ci + nprev + ns]], 0)
            taps = [(kf, kt) for kf, _ in self._DEC_TAPS[parity] for kt in (0, 1)]
            w = torch.stack([w[:, :, kf, kt] for kf, kt in taps], 0).permute(2, 0, 1)
            Co = w.shape[0]
            if rm.bias is not None:
                bias = torch.cat([rm.bias - im_.bias, im_.bias + rm.bias]).float().contiguous()
            else:
                bias = None
            return ops.pack_weight(w, len(taps) * 2 * ci), bias
        ps = [rm.weight, im_.weight] + ([rm.bias, im_.bias] if rm.bias is not None else [])
        return self._packed(("dec", id(mod), parity), ps, build)

    def _lstm_w(self, li):
        m = self.masker.encoders[-1].rnn.rnns[li]
        R, I = m.re_module.rnn, m.im_module.rnn

        def build():
            wih = torch.cat([R.weight_ih_l0, I.weight_ih_l0], 0)  # [8H, D]
            H = R.hidden_size
            if li == 0:  # input [B, T, C*F] (channel-major) gathered from BFTC taps over f
                D = wih.shape[1]
                w = wih.reshape(8 * H, D // 4, 4).permute(0, 2, 1)
            else:
                w = wih.unsqueeze(1)
            bias = torch.cat([R.bias_ih_l0 + R.bias_hh_l0, I.bias_ih_l0 + I.bias_hh_l0])
            whh = torch.stack([R.weight_hh_l0, I.weight_hh_l0], 0)
            return (ops.pack_weight(w, wih.shape[1]), bias.float().contiguous(),
                    whh.float().contiguous())
        return self._packed(("lstm", li), (R.weight_ih_l0, I.weight_ih_l0, R.weight_hh_l0,
                                           I.weight_hh_l0, R.bias_ih_l0, R.bias_hh_l0,
                                           I.bias_ih_l0, I.bias_hh_l0), build)

    def _lin_w(self):
        lin = self.masker.encoders[-1].linear
        Lr, Li = lin.re_module, lin.im_module

        def build():  # K segments (r, i): re = [Wr | -Wi] + (br - bi), im = [Wi | Wr] + (br + bi)
            wre = torch.cat([Lr.weight, -Li.weight], 1)
            wim = torch.cat([Li.weight, Lr.weight], 1)
            return (ops.pack_weight(wre.unsqueeze(1), wre.shape[1]),
                    (Lr.bias - Li.bias).float().contiguous(),
                    ops.pack_weight(wim.unsqueeze(1), wim.shape[1]),
                    (Lr.bias + Li.bias).float().contiguous())
        return self._packed(("lin",), (Lr.weight, Li.weight, Lr.bias, Li.bias), build)

    def _fb_w(self):
        ef, df = self.encoder.filterbank._filters, self.decoder.filterbank._filters

        def build():
            a = ops.pack_weight(ef[:, 0, :].float().unsqueeze(1), ef.shape[-1])  # [514, 400]
            w = df[:, 0, :].float().t().contiguous()                             # [400, 514]
            w = torch.cat([w, w.new_zeros(w.shape[0], 2)], 1)                   # K = 516
            return a, ops.pack_weight(w.unsqueeze(1), 516)
        return self._packed(("fb",), (ef, df), build)

    # ------------------------------------------------------------------ BatchNorm + PReLU
    def _bn_prelu(self, raw, norm, act, train, part, nblk):
        """OnReIm(BatchNorm2d) + OnReIm(PReLU) over BFTC [.., re | im] channels in place; the
        re / im modules' running statistics are updated as asteroid's train mode does."""
        C2 = raw.shape[-1]
        nr, ni = norm.re_module, norm.im_module
        g = torch.cat([nr.weight, ni.weight]).float().contiguous()
        b = torch.cat([nr.bias, ni.bias]).float().contiguous()
        rm = torch.cat([nr.running_mean, ni.running_mean]).float().contiguous()
        rv = torch.cat([nr.running_var, ni.running_var]).float().contiguous()
        coef = ops.batch_norm_bftc(raw, None, g, b, rm, rv, train, nr.momentum, nr.eps, 1,
                                   partial=(part, nblk) if train else None)
        if train:
            with torch.no_grad():
                nr.running_mean.copy_(rm[:C2 // 2])
                ni.running_mean.copy_(rm[C2 // 2:])
                nr.running_var.copy_(rv[:C2 // 2])
                ni.running_var.copy_(rv[C2 // 2:])
                nr.num_batches_tracked += 1
                ni.num_batches_tracked += 1
        alpha = torch.cat([act.re_module.weight, act.im_module.weight]).float().contiguous()
        rows = raw.numel() // C2
        sc = coef.data_ptr()
        check(ops.lib().clskd_bn_apply_reim(ptr(raw), ptr(raw), rows, C2, sc, sc + 4 * C2,
                                            ptr(alpha), ops._dt(raw), ops._stream()),
              "bn_apply_reim")
        return raw

    # ------------------------------------------------------------------ forward
    def forward(self, wav):
        x = wav
        if x.dim() == 3:
            x = x.squeeze(1)
        if x.dim() == 1:
            x = x.unsqueeze(0)
        return self.run(x, self.training)["wav"].unsqueeze(1)

    def run(self, x, train=True):
        if not x.is_cuda:
            raise RuntimeError("clskd DCCRNet_mini runs on the HIP device (no CPU fallback)")
        x = x.float().contiguous()
        B, L = x.shape
        if L < 400:
            raise ValueError("DCCRNet_mini needs at least one 400-sample frame")
        T = (L - 400) // 100 + 1
        dev = x.device
        f32 = dict(device=dev, dtype=torch.float32)
        wa, ws = self._fb_w()
        # ---- STFTFB analysis (conv1d, stride 100, no padding): 4 hops of 100 samples per frame
        spec = torch.empty(B, T, 514, **f32)
        ops.conv([Seg(x, 0, SegGeom(100, L, 0, 100, 1, L // 100))], [(0, kt) for kt in range(4)],
                 B, 1, T, 514, wa, None, spec, OutMap(T * 514, 0, 514))
        xin = ops.spec_bftc(spec, 0, 257, 256, torch.empty(B, 256, T, 2, **f32))  # Nyquist dropped
        # ---- complex encoders
        enc = []
        F, Ti, cur = 256, T, xin
        for i, blk in enumerate(self.masker.encoders[:-1]):
            Co = 2 * blk.conv.re_module.out_channels
            Fo, To = F // 2, Ti - 1
            raw = torch.empty(B, Fo, To, Co, **f32)
            nmb = ops.conv_mblocks(B, Fo, To)
            part = torch.empty(nmb * Co * 2, device=dev, dtype=torch.float64) if train else None
            ops.conv([seg_bftc(cur)], [(kf - 2, kt) for kf in range(5) for kt in range(2)], B, Fo,
                     To, Co, self._enc_w(i), None, raw, OutMap(Fo * To * Co, To * Co, Co),
                     stride_f=2, stats=part)
            cur = self._bn_prelu(raw, blk.norm, blk.activation, train, part, nmb)
            enc.append(cur)
            F, Ti = Fo, To
        # ---- DCCRMaskNetRNN_mini: two complex LSTM layers (batch-first) + complex Linear
        e6 = enc[-1]
        D4, C6 = e6.shape[1], e6.shape[-1]
        Ch = C6 // 2
        rnn = self.masker.encoders[-1].rnn
        H = rnn.rnns[0].re_module.rnn.hidden_size
        r_in = None
        for li in range(len(rnn.rnns)):
            wp, bias, whh = self._lstm_w(li)
            gx = torch.empty(2, B, Ti, 8 * H, **f32)
            for half in range(2):
                if li == 0:
                    segs, taps = [seg_bftc(e6, c0=half * Ch, C=Ch)], [(f, 0) for f in range(D4)]
                else:
                    segs, taps = [Seg(r_in[half], 0, SegGeom(H, Ti * H, 0, H, 1, Ti))], [(0, 0)]
                ops.conv(segs, taps, B, 1, Ti, 8 * H, wp, bias, gx[half],
                         OutMap(Ti * 8 * H, 0, 8 * H))
            hs = torch.empty(2, 2 * B, Ti, H, **f32)
            ops.lstm_recurrent(gx, 4 * H, Ti * 8 * H, 8 * H, whh, 2, 2 * B, Ti, H, hs,
                               2 * B * Ti * H, Ti * H, H)
            ro = torch.empty(B, Ti, H, **f32)
            io = torch.empty(B, Ti, H, **f32)
            ops.complex_combine(hs[0, :B], hs[1, B:], hs[0, B:], hs[1, :B], ro, io)
            r_in = (ro, io)
        wre, bre, wim, bim = self._lin_w()
        rnn_out = torch.empty(B, D4, Ti, C6, **f32)
        segs = [Seg(r_in[h], 0, SegGeom(H, Ti * H, 0, H, 1, Ti)) for h in range(2)]
        for half, (w, b) in enumerate(((wre, bre), (wim, bim))):
            ops.conv(segs, [(0, 0)], B, 1, Ti, Ch * D4, w, b, rnn_out,
                     OutMap(D4 * Ti * C6, 0, C6, 1, Ti * C6, D4), out_offset=half * Ch)
        # ---- decoders: [Identity, 1..n] with skips cat([x, enc_out]), then the output layer
        prev, F = rnn_out, D4
        nenc = len(enc)
        dec_mods = list(self.masker.decoders)[1:] + [self.masker.output_layer[0]]
        for d, mod in enumerate(dec_mods):
            skip = enc[nenc - 1 - d]
            is_out = d == len(dec_mods) - 1
            deconv = mod if is_out else mod.deconv
            Co = 2 * deconv.re_module.out_channels
            segs = [seg_bftc(prev), seg_bftc(skip)]
            raw = torch.empty(B, 2 * F, Ti + 1, Co, **f32)
            nmb = ops.conv_mblocks(B, F, Ti + 1)
            part = (torch.empty(2 * nmb * Co * 2, device=dev, dtype=torch.float64)
                    if (train and not is_out) else None)
            for parity in (0, 1):
                wp, bias = self._dec_w(deconv, parity, prev.shape[-1] // 2)
                taps = [(dF, -kt) for _, dF in self._DEC_TAPS[parity] for kt in (0, 1)]
                ops.conv(segs, taps, B, F, Ti + 1, Co, wp, bias, raw,
                         OutMap(2 * F * (Ti + 1) * Co, (Ti + 1) * Co, Co, of_mul=2, of_add=parity),
                         stats=part, stats_offset=parity * nmb * Co * 2)
            if not is_out:
                raw = self._bn_prelu(raw, mod.norm, mod.activation, train, part, 2 * nmb)
            prev, F, Ti = raw, 2 * F, Ti + 1
        mask = prev  # [B][256][T][2]
        # ---- BoundComplexMask('tanh') * spectrum, Nyquist 0; STFTFB synthesis; pad to L
        est = torch.empty(B, T, 516, **f32)
        check(ops.lib().clskd_mask_bdt(ptr(spec), 514, ptr(mask), T, B, T, ptr(est), 516,
                                       ops._stream()), "mask_bdt")
        frames = torch.empty(B, T, 400, **f32)
        ops.conv([Seg(est, 0, SegGeom(516, T * 516, 0, 516, 1, T))], [(0, 0)], B, 1, T, 400, ws,
                 None, frames, OutMap(T * 400, 0, 400))
        out = torch.empty(B, L, **f32)
        ops.ola_hop(frames, None, 100, L, 0, False, out)
        return dict(wav=out, mask=mask, spec=spec, enc=enc)


def normalize_estimates(est, mix):
    """asteroid.dsp.normalization.normalize_estimates (eval.py:75) on device tensors: each
    estimate row scaled so its peak equals the mixture's peak."""
    mmax = mix.abs().amax(-1, keepdim=True)
    return est * (mmax / est.abs().amax(-1, keepdim=True))


def enhance(model, mixtures):
    """eval.py:57-75 per utterance (batch 1, the model in whatever mode it is — eval.py leaves
    it in train mode), no grad: returns the normalised estimates (list of [L_i] tensors)."""
    outs = []
    with torch.no_grad():
        for mix in mixtures:
            m = mix.reshape(1, -1)
            est = model(m)[:, 0]
            outs.append(normalize_estimates(est, m)[0])
    return outs


def load_conf(npz):
    """serialize()-style dict from tests/golden/asteroid_mini.npz-like arrays (w/<key> entries)."""
    sd = {k[2:]: torch.from_numpy(npz[k]) for k in npz.files if k.startswith("w/")}
    for k in ("_filters", "torch_window"):
        sd.setdefault("decoder.filterbank." + k, sd["encoder.filterbank." + k])
    return dict(model_name=str(npz["model_name"]), state_dict=sd,
                model_args=json.loads(str(npz["model_args"])))
