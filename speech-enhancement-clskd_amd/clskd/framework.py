"""framework.py drop-in: MultiResolutionSTFTLoss, SPKDLoss, ABF / ReviewKD / build_review_kd.

Same class names, constructor arguments and return conventions as the reference
(``framework.py:16-284``); arithmetic runs in libclskd_hip.so.  Feature maps may be any NCHW
tensors; BFTC buffers produced by ``clskd.DCCRN`` (exposed as permuted NCHW views) are consumed
without copies.
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .ops import OutMap, Seg, SegGeom, seg_bftc

# ABF conv1 folded into its consumers (clskd_abf_*; CLSKD_ABF_FOLD=0: the materialising path)
_ABF_FOLD = os.environ.get("CLSKD_ABF_FOLD", "1") != "0"

# --------------------------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------------------------


def to_bftc(x):
    """NCHW tensor -> contiguous BFTC tensor (no copy when x is a permuted BFTC buffer)."""
    if x.dim() != 4:
        raise ValueError(f"expected an NCHW feature map, got shape {tuple(x.shape)}")
    B, Cn, Fn, Tn = x.shape
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    if x.stride() == (Fn * Tn * Cn, 1, Tn * Cn, Cn):
        return x.permute(0, 2, 3, 1)  # contiguous view of the underlying BFTC storage
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2)


def _pv(*ts):
    return tuple((t.data_ptr(), t._version) for t in ts)


# --------------------------------------------------------------------------------------------
# STFT losses (framework.py:16-146)
# --------------------------------------------------------------------------------------------
class _StftPlan:
    """Framing GEMM plan of one resolution: torch.stft(center=True, reflect, onesided) with a
    win_length window centred in fft_size, as a hop-grouped conv over the reflect-padded signal."""

    def __init__(self, fft_size, hop, win, window):
        self.fft, self.hop, self.win = fft_size, hop, win
        self.off = (fft_size - win) // 2
        self.KT = -(-win // hop)
        w = np.zeros(self.KT * hop, np.float64)
        w[:win] = window.double().cpu().numpy()
        n = np.arange(self.KT * hop, dtype=np.float64) + self.off
        f = np.arange(fft_size // 2 + 1, dtype=np.float64)[:, None]
        ang = 2.0 * np.pi * f * n[None, :] / fft_size
        basis = np.concatenate([np.cos(ang) * w, -np.sin(ang) * w], 0)  # [fft+2, KT*hop]
        self.basis_cpu = torch.from_numpy(basis.astype(np.float32))
        self._dev = {}

    def basis(self, dev):
        if dev not in self._dev:
            self._dev[dev] = ops.pack_weight(self.basis_cpu.to(dev).unsqueeze(1), self.KT * self.hop)
        return self._dev[dev]

    def spectrum(self, x):
        B, L = x.shape
        nb = self.fft // 2 + 1
        Tm = 1 + L // self.hop
        pad = self.fft // 2
        Lr = L + 2 * pad + self.KT * self.hop
        Lr += (-Lr) % 4
        xr = torch.empty(B, Lr, device=x.device, dtype=torch.float32)
        ops.frame_pad(x, pad, Lr, 1, xr)
        X = torch.empty(B, Tm, 2 * nb, device=x.device, dtype=torch.float32)
        seg = Seg(xr, self.off, SegGeom(self.hop, Lr, 0, self.hop, 1, Tm + self.KT))
        ops.conv([seg], [(0, kt) for kt in range(self.KT)], B, 1, Tm, 2 * nb,
                 self.basis(x.device), None, X, OutMap(Tm * 2 * nb, 0, 2 * nb))
        return X


class STFTLoss(nn.Module):
    """framework.py:72-101."""

    def __init__(self, fft_size=1024, shift_size=120, win_length=600, window="hann_window"):
        super().__init__()
        self.fft_size, self.shift_size, self.win_length = fft_size, shift_size, win_length
        self.register_buffer("window", getattr(torch, window)(win_length))
        self._plan = _StftPlan(fft_size, shift_size, win_length, self.window)

    def accumulate(self, x, y, out2, factor_sc, factor_mag, accumulate, tape=None):
        x = x.reshape(-1, x.shape[-1]).float().contiguous()
        y = y.reshape(-1, y.shape[-1]).float().contiguous()
        X = self._plan.spectrum(x)
        Y = self._plan.spectrum(y)
        nb = self.fft_size // 2 + 1
        if tape is not None:  # what backward.mrstft_backward needs
            L = x.shape[1]
            Lr = L + 2 * (self.fft_size // 2) + self._plan.KT * self._plan.hop
            Lr += (-Lr) % 4
            tape.append(dict(X=X, Y=Y, plan=self._plan, factor_mag=factor_mag,
                             count=X.shape[0] * X.shape[1] * nb, L=L, Lr=Lr))
        return ops.stft_mag_loss(X, Y, nb, factor_sc, factor_mag, out2, accumulate)

    def forward(self, x, y):
        out2 = self.accumulate(x, y, None, 1.0, 1.0, False)
        return out2[0], out2[1]


class MultiResolutionSTFTLoss(nn.Module):
    """framework.py:104-146: returns (factor_sc * mean sc, factor_mag * mean log-mag L1)."""

    def __init__(self, fft_sizes=[1024, 2048, 512], hop_sizes=[120, 240, 50],
                 win_lengths=[600, 1200, 240], window="hann_window", factor_sc=0.1,
                 factor_mag=0.1):
        super().__init__()
        assert len(fft_sizes) == len(hop_sizes) == len(win_lengths)
        self.stft_losses = nn.ModuleList()
        for fs, ss, wl in zip(fft_sizes, hop_sizes, win_lengths):
            self.stft_losses += [STFTLoss(fs, ss, wl, window)]
        self.factor_sc = factor_sc
        self.factor_mag = factor_mag

    def forward(self, x, y, out2=None, tape=None):
        R = len(self.stft_losses)
        for r, f in enumerate(self.stft_losses):
            out2 = f.accumulate(x, y, out2, self.factor_sc / R, self.factor_mag / R, r > 0, tape)
        return out2[0], out2[1]


# --------------------------------------------------------------------------------------------
# SPKD (framework.py:150-172)
# --------------------------------------------------------------------------------------------
class SPKDLoss(nn.Module):
    """Similarity-preserving KD: G = normalize(z z^T, p=1) per side, ||G_t - G_s||_F^2 (/ B^2).

    NB the reference's ``normalize(torch.matmul(z, torch.t(z)), 1)`` passes 1 as p (L1 rows)."""

    def __init__(self, student_output, teacher_output, reduction, **kwargs):
        super().__init__()
        self.student_outputs = student_output
        self.teacher_outputs = teacher_output
        self.reduction = reduction

    def matmul_and_normalize(self, z):
        _, gs, _ = ops.spkd_losses([(ops.gram_view(z), ops.gram_view(z))], z.shape[0], True, True)
        return gs[0]

    def compute_spkd_loss(self, teacher_outputs, student_outputs):
        B = teacher_outputs.shape[0]
        loss = ops.spkd_losses([(ops.gram_view(student_outputs), ops.gram_view(teacher_outputs))],
                               B, batchmean=False)
        return loss[0]

    def forward(self, *args, **kwargs):
        B = self.teacher_outputs.shape[0]
        loss = ops.spkd_losses([(ops.gram_view(self.student_outputs),
                                 ops.gram_view(self.teacher_outputs))], B,
                               batchmean=self.reduction == "batchmean")
        return loss[0]


# --------------------------------------------------------------------------------------------
# ABF / ReviewKD (framework.py:176-284)
# --------------------------------------------------------------------------------------------
class ABF(nn.Module):
    """framework.py:176-222.  Parameters are standard Conv2d/BatchNorm2d containers; forward
    runs conv1(1x1)+BN -> [nearest upsample + attention fuse] -> conv2(3x3)+BN in HIP."""

    def __init__(self, in_channel, mid_channel, out_channel, fuse):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv2d(in_channel, mid_channel, kernel_size=1, bias=False),
                                   nn.BatchNorm2d(mid_channel))
        self.conv2 = nn.Sequential(nn.Conv2d(mid_channel, out_channel, kernel_size=3, stride=1,
                                             padding=1, bias=False),
                                   nn.BatchNorm2d(out_channel))
        if fuse:
            self.att_conv = nn.Sequential(nn.Conv2d(mid_channel * 2, 2, kernel_size=1), nn.Sigmoid())
        else:
            self.att_conv = None
        nn.init.kaiming_uniform_(self.conv1[0].weight, a=1)
        nn.init.kaiming_uniform_(self.conv2[0].weight, a=1)
        self._wcache = {}
        self.compute = "fp32"  # MFMA operand type of conv1/conv2 ("fp32" | "bf16")

    @property
    def act_dtype(self):
        return torch.bfloat16 if self.compute == "bf16" else torch.float32

    def _params(self):
        ps = [self.conv1[0].weight, self.conv2[0].weight]
        if self.att_conv is not None:
            ps += [self.att_conv[0].weight, self.att_conv[0].bias]
        return ps

    def param_versions(self):
        return tuple(p._version for p in self._params())

    def redraw_jobs(self):
        """Draw jobs (clskd_uniform_redraw) re-initialising this ABF like framework.py:179-195:
        conv1/conv2 kaiming_uniform(a=1) -> U(+-sqrt(3/fan_in)); att_conv default Conv2d init ->
        weight and bias U(+-1/sqrt(fan_in)).  Targets the packed operands of the current
        weight cache as well, so no repack follows the draw."""
        ent = self._wcache.get("w")
        w1p = w2p = None
        if ent is not None:
            w1p, w2p, _ = ent[1]
        jobs = []
        for w, wp in ((self.conv1[0].weight, w1p), (self.conv2[0].weight, w2p)):
            N, Cin, kh, kw = w.shape
            jobs.append((w, wp, Cin, kh * kw, math.sqrt(3.0 / (Cin * kh * kw))))
        if self.att_conv is not None:
            aw, ab = self.att_conv[0].weight, self.att_conv[0].bias
            fan_in = aw.shape[1] * aw.shape[2] * aw.shape[3]
            jobs.append((aw, None, aw.shape[1], aw.shape[2] * aw.shape[3], 1.0 / math.sqrt(fan_in)))
            jobs.append((ab, None, 1, 1, 1.0 / math.sqrt(fan_in)))
        return jobs

    def after_redraw(self):
        """The parameters were rewritten in place by a kernel: advance their version counters
        (autograd / cache bookkeeping) and mark the packed operands (written by the same
        kernel) current."""
        ps = self._params()
        torch.autograd.graph.increment_version(ps)
        ent = self._wcache.get("w")
        if ent is not None:
            w1p, w2p, _ = ent[1]
            torch.autograd.graph.increment_version([w1p, w2p])  # invalidates derived layouts
            self._wcache["w"] = (_pv(*ps) + ent[0][-2:],) + tuple(ent[1:])

    def _weights(self, in_dtype):
        ps = self._params()
        ver = _pv(*ps) + (self.compute, in_dtype)
        ent = self._wcache.get("w")
        tok = ops.capture_token()  # entries built inside a capture serve that capture only
        if ent is None or ent[0] != ver or not ops.cache_entry_usable(ent[2] if len(ent) > 2 else None, tok):
            with torch.no_grad():
                c1 = "bf16" if in_dtype == torch.bfloat16 else "fp32"
                w1 = self.conv1[0].weight  # [mid, in, 1, 1]
                w1p = ops.pack_weight(w1.reshape(w1.shape[0], 1, w1.shape[1]), w1.shape[1], c1)
                w2 = self.conv2[0].weight  # [out, mid, 3, 3]
                w2p = ops.pack_weight(w2.permute(0, 2, 3, 1).reshape(w2.shape[0], 9, w2.shape[1]),
                                      9 * w2.shape[1], self.compute)
                att = None
                if self.att_conv is not None:
                    att = (self.att_conv[0].weight.reshape(2, -1).float().contiguous(),
                           self.att_conv[0].bias.float().contiguous())
            ent = (ver, (w1p, w2p, att), tok)
            self._wcache["w"] = ent
        ops.capture_keep(ent[1], tok)
        return ent[1]

    def forward_bftc(self, x, y=None, shape=None, out_shape=None, train=None, defer_bn=False,
                     tape=None, conv2_stream=None):
        """x: BFTC [B][F][T][Cin]; y: BFTC residual [B][Fr][Tr][mid].  Returns (out, x_fused) BFTC.
        defer_bn: conv2's BatchNorm is left unapplied — out is an ops.DeferredBN (raw output +
        coefficients) for a consumer that folds the affine into its loads (the SPKD Gram).
        tape: a dict receiving what ABF.backward_bftc needs (raw conv outputs, BN coefficients and
        batch statistics, the fused map and the residual).
        conv2_stream: run the 3x3 conv2 and its BatchNorm on this stream (after the fused map
        exists) — it is off the level-to-level residual chain, which then continues on the
        current stream; `out` belongs to conv2_stream."""
        train = self.training if train is None else train
        if tape is not None and not train:
            raise ValueError("ABF tape (backward) needs train-mode BatchNorm")
        B, Fn, Tn, Cin = x.shape
        w1p, w2p, att = self._weights(x.dtype)
        mid = w1p.shape[0]
        nmb = ops.conv_mblocks(B, Fn, Tn)
        if _ABF_FOLD and mid == 64 and ops.abf_tap_ok(x):
            x1 = self._level_folded(x, y, shape, att, train, tape)
        else:
            x1 = self._level_conv1(x, y, shape, w1p, att, train, tape, nmb)
        if Tn != out_shape and Fn != out_shape:
            raise NotImplementedError(
                f"ABF output interpolation to ({out_shape}, {Tn}) from F={Fn} is not on the CLSKD path")
        if conv2_stream is not None:
            ev = torch.cuda.Event()
            ev.record()
            x1.record_stream(conv2_stream)
            conv2_stream.wait_event(ev)
            with torch.cuda.stream(conv2_stream):
                return self._conv2_bftc(x1, w2p, train, defer_bn, tape, nmb)
        return self._conv2_bftc(x1, w2p, train, defer_bn, tape, nmb)

    def _level_folded(self, x, y, shape, att, train, tape):
        """conv1 + BN1 [+ attention fusion] with conv1 folded (clskd_abf_*): the BatchNorm
        statistics of W1 x come from x's moments and the fused kernel recomputes W1 x per row,
        so conv1's 64-channel output never reaches HBM (only the raw copy the tape keeps)."""
        B, Fn, Tn, Cin = x.shape
        dev = x.device
        act = dict(device=dev, dtype=self.act_dtype)
        w1 = self.conv1[0].weight
        bn = self.conv1[1]
        mv1 = torch.empty(2, 64, device=dev, dtype=torch.float32) if tape is not None else None
        coef = ops.abf_bn1_coef(x, w1, bn, train,
                                stats_out=(mv1[0], mv1[1]) if tape is not None else None)
        res = None
        if self.att_conv is not None:
            if shape != Fn:  # the reference's torch.cat would fail as well (framework.py:213-216)
                raise ValueError(f"ABF fuse: residual upsampled to F={shape} but x has F={Fn}")
            res = y if y.dtype == act["dtype"] else y.to(act["dtype"])
            res = res.contiguous()
        xf = torch.empty(B, Fn, Tn, 64, **act)
        x1_raw = torch.empty(B, Fn, Tn, 64, **act) if tape is not None else None
        ops.abf_conv1_fuse(x, w1, coef, res, att, xf, x1_raw)
        if tape is not None:
            # versions of the weights this forward used: a re-draw (abf_reinit='step') before the
            # backward rewrites them in place, which backward.review_backward refuses
            tape.update(x_in=x, x1=x1_raw, mv1=mv1, res=res, coef1=coef,
                        wver=self.param_versions())
        return xf

    def _level_conv1(self, x, y, shape, w1p, att, train, tape, nmb):
        """conv1 as a pointwise conv with its 64-channel output materialised (fallback for taps
        the folded kernels cannot read in place; CLSKD_ABF_FOLD=0 selects it everywhere)."""
        B, Fn, Tn, Cin = x.shape
        mid = w1p.shape[0]
        dev = x.device
        act = dict(device=dev, dtype=self.act_dtype)
        x1 = torch.empty(B, Fn, Tn, mid, **act)
        f64 = dict(device=dev, dtype=torch.float64)
        part = torch.empty(nmb * mid * 2, **f64) if train else None
        ops.conv([seg_bftc(x)], [(0, 0)], B, Fn, Tn, mid, w1p, None, x1,
                 OutMap(Fn * Tn * mid, Tn * mid, mid), stats=part)
        bn = self.conv1[1]
        mv1 = torch.empty(2, mid, device=dev, dtype=torch.float32) if tape is not None else None
        so1 = (mv1[0], mv1[1]) if tape is not None else None
        if tape is not None:
            # versions of the weights this forward used: a re-draw (abf_reinit='step') before the
            # backward rewrites them in place, which backward.review_backward refuses
            tape.update(x_in=x, x1=x1, mv1=mv1, res=y, wver=self.param_versions())
        if self.att_conv is not None:
            if shape != Fn:  # the reference's torch.cat would fail as well (framework.py:213-216)
                raise ValueError(f"ABF fuse: residual upsampled to F={shape} but x has F={Fn}")
            # conv1's BatchNorm is applied by the fuse kernel as it loads x1 (no extra pass)
            coef = ops.batch_norm_bftc(x1, None, bn.weight, bn.bias, bn.running_mean,
                                       bn.running_var, train, bn.momentum, bn.eps, 1,
                                       partial=(part, nmb) if train else None, stats_out=so1)
            if tape is not None:
                tape["coef1"] = coef
            if y.dtype != x1.dtype:  # user-supplied residual of another storage type
                y = y.to(x1.dtype).contiguous()
            xf = torch.empty_like(x1)
            ops.abf_fuse(x1, y, att[0], att[1], xf, x_coef=coef)
            if tape is not None:
                tape["res"] = y
            x1 = xf
        elif tape is not None:
            x1n = torch.empty_like(x1)
            _, coef = ops.batch_norm_bftc(x1, x1n, bn.weight, bn.bias, bn.running_mean,
                                          bn.running_var, train, bn.momentum, bn.eps, 1,
                                          partial=(part, nmb), stats_out=so1, return_coef=True)
            tape["coef1"] = coef
            x1 = x1n
        else:
            ops.batch_norm_bftc(x1, x1, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                train, bn.momentum, bn.eps, 1,
                                partial=(part, nmb) if train else None)
        return x1

    def _conv2_bftc(self, x1, w2p, train, defer_bn, tape, nmb):
        B, Fn, Tn, _ = x1.shape
        dev = x1.device
        act = dict(device=dev, dtype=self.act_dtype)
        f64 = dict(device=dev, dtype=torch.float64)
        Cout = w2p.shape[0]
        out = torch.empty(B, Fn, Tn, Cout, **act)
        bn = self.conv2[1]
        mv2 = torch.empty(2, Cout, device=dev, dtype=torch.float32) if tape is not None else None
        # train: conv2's BatchNorm statistics folded into the conv launch (ops.BnStats)
        st = (ops.BnStats(bn, Cout, B * Fn * Tn, 1, dev,
                          stats_out=(mv2[0], mv2[1]) if mv2 is not None else None)
              if train else None)
        ops.conv([seg_bftc(x1)], [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], B, Fn,
                 Tn, Cout, w2p, None, out, OutMap(Fn * Tn * Cout, Tn * Cout, Cout),
                 bn_stats=(st, True) if st is not None else None)
        if train:
            coef = st.coefficients()
        else:
            coef = ops.batch_norm_bftc(out, None, bn.weight, bn.bias, bn.running_mean,
                                       bn.running_var, False, bn.momentum, bn.eps, 1)
        if tape is not None:
            tape.update(xf=x1, out_raw=out, coef2=coef, mv2=mv2)
            d = ops.DeferredBN(out, coef)
            return (d if defer_bn else d.materialize()), x1
        if defer_bn:
            return ops.DeferredBN(out, coef), x1
        return ops.bn_apply(out, out, coef), x1

    def forward(self, x, y=None, shape=None, out_shape=None, feature_type=None):
        out, xf = self.forward_bftc(to_bftc(x), to_bftc(y) if y is not None else None, shape,
                                    out_shape)
        return nchw(out), nchw(xf)


class ReviewKD(nn.Module):
    """framework.py:226-263."""

    def __init__(self, in_channels, out_channels, shapes, out_shapes, feature_maps, ft_type):
        super().__init__()
        self.shapes = shapes
        self.out_shapes = shapes if out_shapes is None else out_shapes
        self.feature_maps = feature_maps
        self.ft_type = ft_type
        abfs = nn.ModuleList()
        mid_channel = min(512, in_channels[-1])
        for idx, in_channel in enumerate(in_channels):
            abfs.append(ABF(in_channel, mid_channel, out_channels[idx], idx < len(in_channels) - 1))
        self.abfs = abfs[::-1]

    def set_compute(self, compute):
        for abf in self.abfs:
            abf.compute = compute
        return self

    def forward_bftc(self, feats, defer_bn=False, tape=None, conv2_stream=None):
        """feats: BFTC student features in the reference's list order.  Returns BFTC outputs
        (ops.DeferredBN entries when defer_bn: the ABF output BatchNorms left for the consumer).
        tape: a list receiving one ABF tape dict per level, in processing order.
        conv2_stream: every level's conv2 + BatchNorm runs there (ABF.forward_bftc); the outputs
        belong to that stream."""
        xs = feats[::-1] if self.ft_type == "encoder" else list(feats)
        results = []
        tp = {} if tape is not None else None
        out, res = self.abfs[0].forward_bftc(xs[0], out_shape=self.out_shapes[0],
                                             defer_bn=defer_bn, tape=tp, conv2_stream=conv2_stream)
        if tape is not None:
            tape.append(tp)
        results.append(out)
        for feature, abf, shape, out_shape in zip(xs[1:], self.abfs[1:], self.shapes[1:],
                                                  self.out_shapes[1:]):
            tp = {} if tape is not None else None
            out, res = abf.forward_bftc(feature, res, shape, out_shape, defer_bn=defer_bn, tape=tp,
                                        conv2_stream=conv2_stream)
            if tape is not None:
                tape.append(tp)
            if self.ft_type == "encoder":
                results.insert(0, out)
            else:
                results.append(out)
        return results

    def forward(self, x=None):
        feats = [to_bftc(f) for f in self.feature_maps]
        return [nchw(r) for r in self.forward_bftc(feats)]


def build_review_kd(feature_maps, ft_type):
    """framework.py:266-284."""
    in_channels = [8, 16, 32, 64, 64, 64]
    out_channels = [32, 64, 128, 256, 256, 256]
    shapes = [4, 8, 16, 32, 64, 128]
    out_shapes = [4, 8, 16, 32, 64, 128]
    if ft_type not in ("encoder", "decoder"):
        raise ValueError(ft_type)
    model = ReviewKD(in_channels, out_channels, shapes, out_shapes, feature_maps, ft_type)
    dev = None
    for f in feature_maps or []:
        if torch.is_tensor(f):
            dev = f.device
            break
    if dev is not None:
        model = model.to(dev)
    return model
