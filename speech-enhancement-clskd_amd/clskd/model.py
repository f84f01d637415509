"""DCCRN on MI355X: reference-compatible module tree, HIP forward.

``DCCRN`` keeps the constructor signature, submodule names and ``state_dict`` keys of the
reference (``DCCRN.py:14-147``; ``tools_for_model.py:35-330``), so reference checkpoints load
unchanged and ``feature_extraction``-style taps are available.  The submodules (nn.Conv2d,
nn.LSTM, …) are parameter containers only: ``DCCRN.forward`` runs the whole network through
libclskd_hip.so on BFTC ([batch][freq][time][channel]) buffers, never through torch compute.

Supported configuration = the one the reference trains and distils: masking_mode 'E',
use_clstm=True, use_cbn=False, kernel_size 5, fft 512 / win 400 / hop 100.  Anything else raises.
"""
import os
import weakref

import numpy as np
import torch
import torch.nn as nn
from scipy.signal import get_window

from . import config as cfg
from . import ops
from .ops import OutMap, Seg, SegGeom, seg_bftc

# --------------------------------------------------------------------------------------------
# fixed STFT kernels (tools_for_model.py:15-32)
# --------------------------------------------------------------------------------------------


def init_kernels(win_len, win_inc, fft_len, win_type=None, invers=False):
    """Same construction as tools_for_model.py:15-32 (float64, then fp32)."""
    if win_type == "None" or win_type is None:
        window = np.ones(win_len)
    else:
        window = get_window(win_type, win_len, fftbins=True)
    basis = np.fft.rfft(np.eye(fft_len))[:win_len]
    kernel = np.concatenate([np.real(basis), np.imag(basis)], 1).T
    if invers:
        kernel = np.linalg.pinv(kernel).T
    kernel = kernel * window
    return (torch.from_numpy(kernel[:, None, :].astype(np.float32)),
            torch.from_numpy(window[None, :, None].astype(np.float32)))


class ConvSTFT(nn.Module):
    """tools_for_model.py:35-67 (buffer ``weight`` [N+2, 1, win])."""

    def __init__(self, win_len, win_inc, fft_len=None, win_type="hamming", feature_type="real",
                 fix=True):
        super().__init__()
        self.fft_len = fft_len if fft_len is not None else int(2 ** np.ceil(np.log2(win_len)))
        kernel, _ = init_kernels(win_len, win_inc, self.fft_len, win_type)
        self.register_buffer("weight", kernel)
        self.feature_type = feature_type
        self.stride = win_inc
        self.win_len = win_len
        self.dim = self.fft_len


class ConviSTFT(nn.Module):
    """tools_for_model.py:70-109 (buffers ``weight``, ``window``, ``enframe``)."""

    def __init__(self, win_len, win_inc, fft_len=None, win_type="hamming", feature_type="real",
                 fix=True):
        super().__init__()
        self.fft_len = fft_len if fft_len is not None else int(2 ** np.ceil(np.log2(win_len)))
        kernel, window = init_kernels(win_len, win_inc, self.fft_len, win_type, invers=True)
        self.register_buffer("weight", kernel)
        self.feature_type = feature_type
        self.win_type = win_type
        self.win_len = win_len
        self.stride = win_inc
        self.dim = self.fft_len
        self.register_buffer("window", window)
        self.register_buffer("enframe", torch.eye(win_len)[:, None, :])


class ComplexConv2d(nn.Module):
    """Parameter container for tools_for_model.py:193-262 (real_conv / imag_conv)."""

    def __init__(self, in_channels, out_channels, kernel_size=(1, 1), stride=(1, 1),
                 padding=(0, 0), dilation=1, groups=1, causal=True, complex_axis=1):
        super().__init__()
        self.in_channels = in_channels // 2
        self.out_channels = out_channels // 2
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.causal, self.complex_axis = causal, complex_axis
        self.real_conv = nn.Conv2d(self.in_channels, self.out_channels, kernel_size, stride,
                                   padding=[padding[0], 0], dilation=dilation, groups=groups)
        self.imag_conv = nn.Conv2d(self.in_channels, self.out_channels, kernel_size, stride,
                                   padding=[padding[0], 0], dilation=dilation, groups=groups)
        nn.init.normal_(self.real_conv.weight.data, std=0.05)
        nn.init.normal_(self.imag_conv.weight.data, std=0.05)
        nn.init.constant_(self.real_conv.bias, 0.0)
        nn.init.constant_(self.imag_conv.bias, 0.0)

    def forward(self, x):
        raise NotImplementedError("ComplexConv2d runs inside DCCRN.forward (HIP executor)")


class ComplexConvTranspose2d(nn.Module):
    """Parameter container for tools_for_model.py:265-330."""

    def __init__(self, in_channels, out_channels, kernel_size=(1, 1), stride=(1, 1),
                 padding=(0, 0), output_padding=(0, 0), causal=False, complex_axis=1, groups=1):
        super().__init__()
        self.in_channels = in_channels // 2
        self.out_channels = out_channels // 2
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.output_padding = output_padding
        self.real_conv = nn.ConvTranspose2d(self.in_channels, self.out_channels, kernel_size,
                                            stride, padding=padding,
                                            output_padding=output_padding, groups=groups)
        self.imag_conv = nn.ConvTranspose2d(self.in_channels, self.out_channels, kernel_size,
                                            stride, padding=padding,
                                            output_padding=output_padding, groups=groups)
        self.complex_axis = complex_axis
        nn.init.normal_(self.real_conv.weight, std=0.05)
        nn.init.normal_(self.imag_conv.weight, std=0.05)
        nn.init.constant_(self.real_conv.bias, 0.0)
        nn.init.constant_(self.imag_conv.bias, 0.0)

    def forward(self, x):
        raise NotImplementedError("ComplexConvTranspose2d runs inside DCCRN.forward (HIP executor)")


class NavieComplexLSTM(nn.Module):
    """Parameter container for tools_for_model.py:138-178 (name kept from the reference)."""

    def __init__(self, input_size, hidden_size, projection_dim=None, bidirectional=False,
                 batch_first=False):
        super().__init__()
        assert not bidirectional, "bidirectional complex LSTM is not on the DCCRN-CL path"
        self.input_dim = input_size // 2
        self.rnn_units = hidden_size // 2
        self.real_lstm = nn.LSTM(self.input_dim, self.rnn_units, num_layers=1, batch_first=False)
        self.imag_lstm = nn.LSTM(self.input_dim, self.rnn_units, num_layers=1, batch_first=False)
        if projection_dim is not None:
            self.projection_dim = projection_dim // 2
            self.r_trans = nn.Linear(self.rnn_units, self.projection_dim)
            self.i_trans = nn.Linear(self.rnn_units, self.projection_dim)
        else:
            self.projection_dim = None

    def forward(self, x):
        raise NotImplementedError("NavieComplexLSTM runs inside DCCRN.forward (HIP executor)")


def _pv(*tensors):
    """Cache key of a parameter group: storage pointers and in-place versions."""
    return tuple((t.data_ptr(), t._version) for t in tensors)


# A trained student's parameters live in one flat buffer (train.FlatParams) and every Adam step
# rewrites them, so each step re-packs every parameter group (cat / negate / permute / bias sums
# / pad: 3-12 torch launches and their host time per group).  Each packing is linear in the
# group's parameters with coefficients +-1 and at most a few terms per element, so after the
# first build the group is re-packed by ONE clskd_index_gather from the flat buffer into one
# buffer holding all of the group's outputs.  The map is probed once (device synchronised: the
# flat buffer holds +(flat index + 1) for one parameter at a time meanwhile) and kept only if
# the gather reproduces the real build bitwise (fp32 outputs; a + b summed in the build's order).
# CLSKD_PACK_MAPS=0 disables it (A/B).
_PACK_MAPS_ON = os.environ.get("CLSKD_PACK_MAPS", "1") == "1"
# the taped H = 32 recurrence stores its cell states for the backward (round 6; CLSKD_LSTM_CELLS=0:
# the backward re-derives them with its serial scan, A/B)
_LSTM_CELLS = os.environ.get("CLSKD_LSTM_CELLS", "1") == "1"
# the changed parameter groups re-packed in one batched gather at the start of a forward
# (DCCRN.prepack; CLSKD_PREPACK=0: one gather per group at its first use, A/B)
_PREPACK = os.environ.get("CLSKD_PREPACK", "1") == "1"


# packed outputs -> (model, group, slot): backward.tw_prebuild re-derives the data-gradient weights
# of the packed forward weights a step just made, all in one batched gather at the start of the
# backward (id -> (weak output, weak model, group key, slot); verified by identity on lookup)
_PACK_PROV = {}


def _note_pack_outputs(model, key, out):
    outs = [(out, None)] if isinstance(out, torch.Tensor) else [
        (t, i) for i, t in enumerate(out) if isinstance(t, torch.Tensor)]
    if len(_PACK_PROV) > 4096:
        for k in [k for k, v in _PACK_PROV.items() if v[0]() is None]:
            del _PACK_PROV[k]
    mref = weakref.ref(model)
    for t, i in outs:
        _PACK_PROV[id(t)] = (weakref.ref(t), mref, key, i)


def pack_provenance(t):
    """(model, group key, slot | None) of a packed output still current in its model's cache."""
    v = _PACK_PROV.get(id(t))
    if v is None or v[0]() is not t:
        return None
    m = v[1]()
    return None if m is None else (m, v[2], v[3])


def pack_output(model, key, slot, tok):
    """The model's current packed output (group key, slot) usable under capture token tok."""
    ent = model._wcache.get(key)
    if ent is None or not ops.cache_entry_usable(ent[2], tok):
        return None
    out = ent[1]
    return out if slot is None else out[slot]


def _flat_root(params):
    """A 1-D fp32 view of the one storage every parameter of the group lives in (the FlatParams
    buffer: parameters re-homed with `p.data = flat[off:off + k]` share its storage), else None."""
    st = None
    for p in params:
        if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
            return None
        s = p.untyped_storage()
        if st is None:
            st = s
        elif s.data_ptr() != st.data_ptr():
            return None
    if st is None or st.nbytes() // 4 >= (1 << 24):
        return None
    return torch.empty(0, dtype=torch.float32, device=params[0].device).set_(st, 0, (st.nbytes() // 4,))


def _pack_group(maps, key, params, build):
    m = maps.get(key)
    if m:
        root, idx, sgn, total, layout, kind = m
        r = _flat_root(params)
        if r is not None and r.data_ptr() == root.data_ptr() and r.numel() == root.numel():
            buf = torch.empty(total, dtype=torch.float32, device=root.device)
            ops.index_gather(root, idx, sgn, buf)
            outs = [buf[o:o + n].view(sh) for o, n, sh in layout]
            return outs[0] if kind == "tensor" else kind(outs)
    out = build()
    if (m is None and _PACK_MAPS_ON and not torch.cuda.is_current_stream_capturing()
            and any(p.requires_grad for p in params)):
        maps[key] = _probe_pack_map(params, build, out)
    return out


def _probe_pack_map(params, build, out):
    root = _flat_root(params)
    kind = "tensor" if isinstance(out, torch.Tensor) else type(out)
    outs = [out] if kind == "tensor" else list(out)
    if root is None or kind not in ("tensor", tuple, list) or not all(
            isinstance(o, torch.Tensor) and o.dtype == torch.float32 and o.is_contiguous()
            for o in outs):
        return False
    layout, total = [], 0
    for o in outs:  # every output on a 256-B boundary (16-B vector loads of the packed weights)
        layout.append((total, o.numel(), tuple(o.shape)))
        total += -(-o.numel() // 64) * 64
    dev = root.device
    base = root.data_ptr()
    if len(params) < 2 and params[0].numel() == root.numel():
        return False  # a parameter in its own storage: nothing shared to gather from
    torch.cuda.synchronize(dev)
    saved = root.clone()
    terms = []  # per probed parameter: the flat (index + 1) with sign of each output element
    try:
        for p in params:
            root.zero_()
            off = (p.data_ptr() - base) // 4
            p.view(-1).copy_(torch.arange(off + 1, off + p.numel() + 1, dtype=torch.float32, device=dev))
            po = build()
            po = [po] if isinstance(po, torch.Tensor) else list(po)
            flat = torch.zeros(total, dtype=torch.float32, device=dev)
            for (o, n, _), t in zip(layout, po):
                flat[o:o + n] = t.reshape(-1)
            terms.append(flat)
    finally:
        root.copy_(saved)
        torch.cuda.synchronize(dev)
    T = torch.stack(terms, 1)  # [total, nparams]
    nz = T != 0
    J = max(1, int(nz.sum(1).max()))
    # each element's non-zero terms in parameter order, padded with idx -1
    order = torch.argsort((~nz).to(torch.int8), dim=1, stable=True)[:, :J]
    v = torch.gather(T, 1, order)
    # values that are not flat indices of `root` (a build that reads other tensors, or one that is
    # not a ±1 selection): reject before the gather could read out of bounds
    if not ops.probe_values_are_indices(v, root.numel()):
        return False
    idx = torch.where(v != 0, v.abs() - 1, torch.full_like(v, -1)).to(torch.int32).contiguous()
    sgn = torch.sign(v).contiguous()
    buf = torch.empty(total, dtype=torch.float32, device=dev)
    ops.index_gather(root, idx, sgn, buf)
    for (o, n, _), t in zip(layout, outs):
        if not torch.equal(buf[o:o + n], t.reshape(-1)):
            return False
    return (root, idx, sgn, total, layout, kind)


# --------------------------------------------------------------------------------------------
# DCCRN
# --------------------------------------------------------------------------------------------
class DCCRN(nn.Module):
    def __init__(self, rnn_layers=cfg.rnn_layers, rnn_units=cfg.rnn_units, win_len=cfg.win_len,
                 win_inc=cfg.win_inc, fft_len=cfg.fft_len, win_type=cfg.window_type,
                 masking_mode="E", use_clstm=False, use_cbn=False, kernel_size=5,
                 kernel_num=[16, 32, 64, 128, 256, 256]):
        super().__init__()
        if masking_mode != "E" or not use_clstm or use_cbn or kernel_size != 5:
            raise NotImplementedError(
                "clskd.DCCRN builds the DCCRN-CL path of the reference (masking_mode='E', "
                "use_clstm=True, use_cbn=False, kernel_size=5)")
        if (win_len, win_inc, fft_len) != (400, 100, 512):
            raise NotImplementedError("clskd.DCCRN is built for win 400 / hop 100 / fft 512")
        self.win_len, self.win_inc, self.fft_len, self.win_type = win_len, win_inc, fft_len, win_type
        self.rnn_units = rnn_units
        self.input_dim = self.output_dim = win_len
        self.hidden_layers = rnn_layers
        self.kernel_size = kernel_size
        self.kernel_num = [2] + list(kernel_num)
        self.masking_mode = masking_mode
        self.use_clstm = use_clstm
        self.fix = True
        self.stft = ConvSTFT(win_len, win_inc, fft_len, win_type, "complex", fix=True)
        self.istft = ConviSTFT(win_len, win_inc, fft_len, win_type, "complex", fix=True)
        self.encoder = nn.ModuleList()
        self.decoder = nn.ModuleList()
        kn = self.kernel_num
        for idx in range(len(kn) - 1):
            self.encoder.append(nn.Sequential(
                ComplexConv2d(kn[idx], kn[idx + 1], kernel_size=(kernel_size, 2), stride=(2, 1),
                              padding=(2, 1)),
                nn.BatchNorm2d(kn[idx + 1]),
                nn.PReLU()))
        hidden_dim = fft_len // (2 ** len(kn))
        rnns = []
        for idx in range(rnn_layers):
            rnns.append(NavieComplexLSTM(
                input_size=hidden_dim * kn[-1] if idx == 0 else rnn_units,
                hidden_size=rnn_units,
                projection_dim=hidden_dim * kn[-1] if idx == rnn_layers - 1 else None))
        self.enhance = nn.Sequential(*rnns)
        for idx in range(len(kn) - 1, 0, -1):
            mods = [ComplexConvTranspose2d(kn[idx] * 2, kn[idx - 1], kernel_size=(kernel_size, 2),
                                           stride=(2, 1), padding=(2, 0), output_padding=(1, 0))]
            if idx != 1:
                mods += [nn.BatchNorm2d(kn[idx - 1]), nn.PReLU()]
            self.decoder.append(nn.Sequential(*mods))
        self._wcache = {}
        self._pmaps = {}  # parameter group -> packing index map (_pack_group)
        self._pgroups = {}
        self._pkparams = {}  # parameter group -> its resolved tensors (prepack)
        self._pkused = set()  # groups used since the last prepack (the next one re-packs these)
        self._refs = None
        self._tap_sinks = []
        # MFMA operand type of the large GEMMs: "fp32" (exact-f32 MFMA), "f32x3" (fp32 storage, 3 x
        # bf16 split-product MFMA for the fp32 convs), "bf16" / "fp16" (16-bit operands, fp32
        # accumulation).  STFT/iSTFT framing GEMMs run fp32 ("f32x3": split products).
        self.compute = "fp32"
        self.train_split = 0  # KnowledgeDistillation.set_precision: split products in training
        # a captured training step (clskd.graph.TrainStepGraph) records the packing of every
        # trainable parameter group, so each replay packs the weights its own optimizer step wrote
        self.repack_in_capture = False

    # ---------------------------------------------------------------- reference helpers
    def flatten_parameters(self):
        pass

    def get_params(self, weight_decay=0.0):
        """DCCRN.py:242-257."""
        weights, biases = [], []
        for name, param in self.named_parameters():
            (biases if "bias" in name else weights).append(param)
        return [{"params": weights, "weight_decay": weight_decay},
                {"params": biases, "weight_decay": 0.0}]

    def loss(self, inputs, labels, real_spec=None, img_spec=None, loss_mode="SI-SNR"):
        """DCCRN.py:259-411 — the SI-SNR / MSE modes (the others need asteroid PMSQE / mel)."""
        from .tools_for_loss import si_snr
        if loss_mode == "SI-SNR":
            return -si_snr(inputs, labels)
        raise NotImplementedError(f"loss_mode {loss_mode!r} is not on the CLSKD hot path")

    # ---------------------------------------------------------------- packed weights
    @staticmethod
    def _cmp(segs, K=None):
        """MFMA operand type of one GEMM = storage type of its input segments."""
        return {torch.bfloat16: "bf16", torch.float16: "fp16"}.get(segs[0].tensor.dtype, "fp32")

    @property
    def act_dtype(self):
        """Storage of the BFTC activations: bf16 when the model computes in bf16 (the frozen
        teacher in precision='mixed'), fp32 otherwise."""
        return {"bf16": torch.bfloat16, "fp16": torch.float16}.get(self.compute, torch.float32)

    def _packed(self, key, params, build):
        """Packed operands of a parameter group, rebuilt when a parameter's storage or in-place
        version changes.  params: the group's tensors, or a callable returning them (resolved
        once per key: the module tree is fixed after construction, and nn.Module attribute
        lookups are a measurable part of the step's host time)."""
        if callable(params):
            pg = self._pgroups.get(key)
            if pg is None:
                pg = self._pgroups[key] = tuple(params())
            params = pg
        self._pkparams[key] = params
        self._pkused.add(key)
        ent = self._wcache.get(key)
        ver = _pv(*params)
        tok = ops.capture_token()  # entries built inside a capture serve that capture only
        if ent is None or ent[0] != ver or not ops.cache_entry_usable(ent[2], tok) or (
                self.repack_in_capture and tok is not None and ent[3] is not tok
                and any(p.requires_grad for p in params)):
            with torch.no_grad():
                ent = (_pv(*params), _pack_group(self._pmaps, key, params, build), tok, None)
            self._wcache[key] = ent
            _note_pack_outputs(self, key, ent[1])
        ops.capture_keep(ent[1], tok)
        return ent[1]

    def prepack(self):
        """Re-pack every parameter group that has a packing map and changed since its entry (a
        training step's Adam rewrote them) in one batched gather (clskd_index_gather_jobs) at the
        start of a forward, instead of one launch per group at its first use.  Entries made
        here inside a capture are that capture's repacks (the graph replays the gather)."""
        if not _PREPACK or not self._pmaps:
            return
        tok = ops.capture_token()
        jobs, pend = [], []
        used, self._pkused = self._pkused, set()
        for key in used:
            m = self._pmaps.get(key)
            params = self._pkparams.get(key)
            if not m or params is None:
                continue
            root, idx, sgn, total, layout, kind = m
            r = _flat_root(params)
            if r is None or r.data_ptr() != root.data_ptr() or r.numel() != root.numel():
                continue
            ver = _pv(*params)
            ent = self._wcache.get(key)
            if not (self.repack_in_capture and tok is not None) and ent is not None and (
                    ent[0] == ver and ops.cache_entry_usable(ent[2], tok)):
                continue  # (a captured step re-packs every group: its replays follow Adam)
            buf = torch.empty(total, dtype=torch.float32, device=root.device)
            jobs.append((root, idx, sgn, buf))
            pend.append((key, ver, buf, layout, kind))
        if len(jobs) < 2:
            return
        ops.index_gather_jobs(jobs)
        for key, ver, buf, layout, kind in pend:
            outs = [buf[o:o + n].view(sh) for o, n, sh in layout]
            out = outs[0] if kind == "tensor" else kind(outs)
            self._wcache[key] = (ver, out, tok, tok)
            _note_pack_outputs(self, key, out)
            ops.capture_keep(out, tok)

    def _layer_refs(self):
        """Per-layer module references, resolved once: encoder (conv, bn, prelu), decoder
        (conv, bn | None, prelu | None), the LSTM stack."""
        if self._refs is None:
            enc = [(s[0], s[1], s[2]) for s in self.encoder]
            dec = [(s[0], s[1] if len(s) > 1 else None, s[2] if len(s) > 1 else None)
                   for s in self.decoder]
            self._refs = dict(enc=enc, dec=dec, lstm=list(self.enhance))
        return self._refs

    def _enc_w(self, i, compute="fp32"):
        cc = self._layer_refs()["enc"][i][0]

        def build():
            wr, wi = cc.real_conv.weight, cc.imag_conv.weight  # [Co/2, Ci/2, 5, 2]
            top = torch.cat([wr, -wi], 1)
            bot = torch.cat([wi, wr], 1)
            w = torch.cat([top, bot], 0)  # [Co, Ci, 5, 2]
            Co, Ci = w.shape[:2]
            w = w.permute(0, 2, 3, 1).reshape(Co, 10, Ci)  # tap = kf*2 + kt
            bias = torch.cat([cc.real_conv.bias - cc.imag_conv.bias,
                              cc.imag_conv.bias + cc.real_conv.bias]).float().contiguous()
            return ops.pack_weight(w, 10 * Ci, compute), bias
        return self._packed(("enc", i, compute), lambda: (cc.real_conv.weight, cc.imag_conv.weight,
                                                          cc.real_conv.bias, cc.imag_conv.bias), build)

    _DEC_TAPS = {0: ((0, 1), (2, 0), (4, -1)), 1: ((1, 1), (3, 0))}  # parity -> (kf, dF)

    def _dec_w(self, d, parity, compute="fp32"):
        cc = self._layer_refs()["dec"][d][0]

        def build():
            wr, wi = cc.real_conv.weight, cc.imag_conv.weight  # [Ci/2, Co/2, 5, 2]
            top = torch.cat([wr, wi], 1)   # real input -> [real out | imag out]
            bot = torch.cat([-wi, wr], 1)  # imag input -> [real out | imag out]
            w = torch.cat([top, bot], 0)   # [Ci, Co, 5, 2], rows [out_re, skip_re, out_im, skip_im]
            Ci, Co = w.shape[:2]
            # K order per tap: [out_t (re, im), skip (re, im)] — two contiguous segments (the
            # decoder input and the skip tensor, each whole): fewer, wider gather runs, and
            # 32-channel segments make narrow layers eligible for the halo kernel
            # (row blocks by slicing: an index tensor built on the host would be copied to the
            # device synchronously on every re-pack, i.e. every training step)
            h = Ci // 4
            w = torch.cat([w[0:h], w[2 * h:3 * h], w[h:2 * h], w[3 * h:4 * h]], 0)
            taps = [(kf, kt) for kf, _ in self._DEC_TAPS[parity] for kt in (0, 1)]
            w = torch.stack([w[:, :, kf, kt] for kf, kt in taps], 0)  # [ntap, Ci, Co]
            w = w.permute(2, 0, 1)  # [Co, ntap, Ci]
            bias = torch.cat([cc.real_conv.bias - cc.imag_conv.bias,
                              cc.imag_conv.bias + cc.real_conv.bias]).float().contiguous()
            return ops.pack_weight(w, len(taps) * Ci, compute), bias
        return self._packed(("dec", d, parity, compute),
                            lambda: (cc.real_conv.weight, cc.imag_conv.weight, cc.real_conv.bias,
                                     cc.imag_conv.bias), build)

    def _lstm_w(self, li, compute="fp32"):
        m = self._layer_refs()["lstm"][li]
        R, I = m.real_lstm, m.imag_lstm

        def build():
            H = R.hidden_size
            wih = torch.cat([R.weight_ih_l0, I.weight_ih_l0], 0)  # [8H, D]
            if li == 0:
                D = wih.shape[1]
                Ch = D // 4
                w = wih.reshape(8 * H, Ch, 4).permute(0, 2, 1)  # [8H, tap=f, Ch]
                wp = ops.pack_weight(w, D, compute)
            else:
                wp = ops.pack_weight(wih.unsqueeze(1), wih.shape[1], compute)
            bias = torch.cat([R.bias_ih_l0 + R.bias_hh_l0, I.bias_ih_l0 + I.bias_hh_l0]).float().contiguous()
            whh = torch.stack([R.weight_hh_l0, I.weight_hh_l0], 0).float().contiguous()
            out = [wp, bias, whh]
            if m.projection_dim is not None:
                for lin in (m.r_trans, m.i_trans):
                    out += [ops.pack_weight(lin.weight.unsqueeze(1), lin.weight.shape[1], compute),
                            lin.bias.float().contiguous()]
            return out
        def ps():
            p = [R.weight_ih_l0, I.weight_ih_l0, R.weight_hh_l0, I.weight_hh_l0, R.bias_ih_l0,
                 R.bias_hh_l0, I.bias_ih_l0, I.bias_hh_l0]
            if m.projection_dim is not None:
                p += [m.r_trans.weight, m.r_trans.bias, m.i_trans.weight, m.i_trans.bias]
            return p
        return self._packed(("lstm", li, compute), ps, build)

    def _stft_w(self):
        def build():  # [514, 400] -> K padded to the fp32 engine's multiple
            return ops.pack_weight(self.stft.weight[:, 0, :].float().unsqueeze(1), 400)
        return self._packed(("stft",), (self.stft.weight,), build)

    def _istft_w(self):
        def build():
            inv = self.istft.weight[:, 0, :].float()  # [514, 400]
            w = inv.t().contiguous()  # [400, 514]
            w = torch.cat([w, w.new_zeros(400, 2)], 1)  # K = 516 (est buffer has 2 zero columns)
            return ops.pack_weight(w.unsqueeze(1), 516), self.istft.window[0, :, 0].float().contiguous()
        return self._packed(("istft",), (self.istft.weight, self.istft.window), build)

    # ---------------------------------------------------------------- forward
    def forward(self, inputs, lens=None, is_feat=None):
        """DCCRN.py:149-240.  inputs [B, L] fp32 on the HIP device."""
        res = self.run(inputs, train=self.training, bn_updates=1 if self.training else 0)
        for sink in list(self._tap_sinks):
            sink(res)
        if is_feat:
            return res["out_wav"]
        return res["mask_real"], res["mask_imag"], res["real"], res["imag"], res["out_wav"]

    def spectrum(self, x):
        """ConvSTFT (tools_for_model.py:53-67) -> spec [B][T][514] (frame-major)."""
        B, L = x.shape
        T = cfg.n_frames(L)
        Lp = 100 * (T + 3)
        dev = x.device
        xp = torch.empty(B, Lp, device=dev, dtype=torch.float32)
        ops.frame_pad(x, 300, Lp, 0, xp)
        spec = torch.empty(B, T, 514, device=dev, dtype=torch.float32)
        seg = Seg(xp, 0, SegGeom(100, Lp, 0, 100, 1, T + 3))
        ops.conv([seg], [(0, kt) for kt in range(4)], B, 1, T, 514, self._stft_w(), None, spec,
                 OutMap(T * 514, 0, 514))
        return spec

    @staticmethod
    def _norm(raw, bn, pr, st, train, bn_updates, tape, key, mv, gram_taps, B):
        """BatchNorm + PReLU of a conv output (train: batch statistics from the conv launches'
        BnStats — folded into them or one finalize launch; eval: running statistics).  In place
        unless a tape keeps the raw output; gram_taps: the apply pass also computes the tap's
        SPKD Gram partials (ops.bn_apply_gram).  Returns the normalised tensor."""
        if not train:
            if tape is not None:
                post = torch.empty_like(raw)
                _, coef = ops.batch_norm_bftc(raw, post, bn.weight, bn.bias, bn.running_mean,
                                              bn.running_var, False, bn.momentum, bn.eps,
                                              bn_updates, alpha=pr.weight, return_coef=True)
                tape.setdefault(key, []).append((raw, coef, mv))
                return post
            return ops.batch_norm_bftc(raw, raw, bn.weight, bn.bias, bn.running_mean,
                                       bn.running_var, False, bn.momentum, bn.eps, bn_updates,
                                       alpha=pr.weight)
        coef = st.coefficients()
        if tape is not None:
            post = ops.bn_apply(raw, torch.empty_like(raw), coef, pr.weight)
            tape.setdefault(key, []).append((raw, coef, mv))
            return post
        if gram_taps is not None:
            gram_taps.append(ops.bn_apply_gram(raw, coef, pr.weight, B))
            return raw
        return ops.bn_apply(raw, raw, coef, pr.weight)

    def run(self, x, train=True, bn_updates=1, spec=None, want_masks=True, on_encoder=None,
            tape=None, taps_only=False, mark=None, on_decoder_tap=None, gram_taps=None):
        """See _run.  compute 'f32x3' (the student in precision 'mixed'): the fp32 convs of a
        forward without a tape run as 3 x bf16 split products (CLSKD_F32X3); a taped (training)
        forward too when train_split bit 1 or 2 is set (KnowledgeDistillation.set_precision),
        else on the exact fp32 engines."""
        split = self.compute == "f32x3" and (tape is None or bool(self.train_split & 6))
        self.prepack()
        with ops.split_products(split):
            return self._run(x, train, bn_updates, spec, want_masks, on_encoder, tape, taps_only,
                             mark, on_decoder_tap, gram_taps)

    def _run(self, x, train=True, bn_updates=1, spec=None, want_masks=True, on_encoder=None,
             tape=None, taps_only=False, mark=None, on_decoder_tap=None, gram_taps=None):
        """Full forward on the HIP device.  Returns a dict of BFTC buffers and NCHW views.
        on_encoder(enc): called (on the launching stream) right after the encoder, so a caller can
        fork work that only needs the encoder taps before the LSTM and decoder are enqueued.
        tape: a dict that receives what the backward pass (clskd.backward) needs — pre-BN conv
        outputs kept beside the activations, BN coefficients and batch statistics, the LSTM gate
        inputs and hidden histories, the iSTFT frames.
        on_decoder_tap(t): called (on the launching stream) as each decoder-side tap exists —
        dec_in, then decoder outputs 0..nl-2 — so a consumer (ReviewKD-decoder) can pipeline
        behind the decoder on another stream.
        taps_only: stop after the taps a distillation step reads (encoder outputs, dec_in,
        decoder outputs 0..nl-2): the last decoder layer, mask 'E' and ConviSTFT are dead for
        the CLSKD loss (SURVEY.md §8 d) and are skipped — out_wav is None.
        gram_taps: a list (train mode, no tape) that receives, for every BatchNorm'd SPKD tap —
        encoder outputs 0..nl-1, then decoder outputs 0..nl-2 — the GramSlabs of that tap: its
        BatchNorm + PReLU apply pass is fused with its SPKD Gram partials (ops.bn_apply_gram),
        so the step never reads the tap again for its Gram."""
        fuse_gram = gram_taps is not None and train and tape is None
        if not x.is_cuda:
            raise RuntimeError("clskd.DCCRN.forward needs inputs on the HIP device")
        x = x.float()
        if x.dim() == 3:
            x = x.squeeze(1)
        x = x.contiguous()
        B, L = x.shape
        T = cfg.n_frames(L)
        dev = x.device
        f32 = dict(device=dev, dtype=torch.float32)
        act = dict(device=dev, dtype=self.act_dtype)
        if spec is None:
            spec = self.spectrum(x)
        kn = self.kernel_num
        nl = len(kn) - 1
        # ---------------- encoder (DCCRN.py:171-176, tools_for_model.py:236-262)
        enc = []
        F = 256
        for i in range(nl):
            Co = kn[i + 1]
            Fo = F // 2
            if i == 0:
                # real = spec[:, 1:257], imag = spec[:, 258:514] (DCCRN.py:165-170) as the two
                # channels of a BFTC input: same K order (tap, re, im) as the packed weights
                spec_b = ops.spec_bftc(spec, 1, 258, 256, torch.empty(B, 256, T, 2, **f32))
                segs = [seg_bftc(spec_b)]
                if tape is not None:
                    tape["spec_b"] = spec_b
            else:
                segs = [seg_bftc(enc[-1])]
            wp, bias = self._enc_w(i, self._cmp(segs, 10 * kn[i]))
            taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
            raw = torch.empty(B, Fo, T, Co, **act)
            _, bn, pr = self._layer_refs()["enc"][i]
            mv = torch.empty(2, Co, **f32) if tape is not None else None
            st = (ops.BnStats(bn, Co, B * Fo * T, bn_updates, dev,
                              stats_out=(mv[0], mv[1]) if mv is not None else None)
                  if train else None)
            ops.conv(segs, taps, B, Fo, T, Co, wp, bias, raw, OutMap(Fo * T * Co, T * Co, Co),
                     stride_f=2, bn_stats=(st, True) if st is not None else None)
            enc.append(self._norm(raw, bn, pr, st, train, bn_updates, tape, "enc_bn", mv,
                                  gram_taps if fuse_gram else None, B))
            F = Fo
        if mark is not None:
            mark("encoder done")
        if on_encoder is not None:
            on_encoder(enc)
        # ---------------- complex LSTM (DCCRN.py:178-199, tools_for_model.py:159-174)
        C6 = kn[-1]
        Ch = C6 // 2
        act6 = enc[-1]
        D4 = act6.shape[1]
        H = self.rnn_units // 2
        r_in = None
        lstm_io = []
        for li in range(self.hidden_layers):
            gx = torch.empty(2, B, T, 8 * H, **f32)
            for half in range(2):
                if li == 0:
                    segs = [seg_bftc(act6, c0=half * Ch, C=Ch)]
                    taps = [(f, 0) for f in range(D4)]
                else:
                    src = r_in[half]
                    segs = [Seg(src, 0, SegGeom(H, T * H, 0, H, 1, T))]
                    taps = [(0, 0)]
                packs = self._lstm_w(li, self._cmp(segs, len(taps) * segs[0].geom.C))
                wp, bias, whh = packs[:3]
                ops.conv(segs, taps, B, 1, T, 8 * H, wp, bias, gx[half],
                         OutMap(T * 8 * H, 0, 8 * H))
            hs = torch.empty(2, 2 * B, T, H, **f32)
            # taped: the recurrence leaves the gate pre-activations in gx (the backward's `pre`)
            pre = tape is not None and ops.lstm_pre_capable(H)
            cells = None
            if pre:  # ... and its cell states (the backward then skips its cell-state scan)
                cells = torch.empty(2 * 2 * B * T * H, **f32) if _LSTM_CELLS else None
                ops.lstm_recurrent_pre(gx, 4 * H, T * 8 * H, 8 * H, whh, 2, 2 * B, T, H, hs,
                                       2 * B * T * H, T * H, H, cbuf=cells)
            else:
                ops.lstm_recurrent(gx, 4 * H, T * 8 * H, 8 * H, whh, 2, 2 * B, T, H, hs,
                                   2 * B * T * H, T * H, H)
            if tape is not None:
                tape.setdefault("lstm", []).append(dict(gx=gx, hs=hs, r_in=r_in, pre=pre,
                                                        cells=cells))
            # a 16-bit model (the frozen teacher in precision 'mixed' / 'fp16') stores the layer
            # output as the 16-bit operand of the next layer's input GEMM and the projection
            # (one rounding, as every other teacher activation); fp32 models and taped
            # (backward) forwards keep fp32
            lo = act if (self.compute != "fp32" and tape is None) else f32
            ro = torch.empty(B, T, H, **lo)
            io = torch.empty(B, T, H, **lo)
            ops.complex_combine(hs[0, :B], hs[1, B:], hs[0, B:], hs[1, :B], ro, io)
            r_in = (ro, io)
            lstm_io.append((ro, io))
        # projection into the decoder input [B][D4][T][C6] (DCCRN.py:188-199)
        dec_in = torch.empty(B, D4, T, C6, **act)
        m = self._layer_refs()["lstm"][self.hidden_layers - 1]
        P = m.projection_dim
        for half in range(2):
            segs = [Seg(r_in[half], 0, SegGeom(H, T * H, 0, H, 1, T))]
            packs = self._lstm_w(self.hidden_layers - 1, self._cmp(segs, H))
            wpp, bp = packs[3 + 2 * half], packs[4 + 2 * half]
            ops.conv(segs, [(0, 0)], B, 1, T, P, wpp, bp,
                     dec_in, OutMap(D4 * T * C6, 0, C6, 1, T * C6, D4), out_offset=half * Ch)
        if mark is not None:
            mark("lstm + projection done")
        if on_decoder_tap is not None:
            on_decoder_tap(dec_in)
        # ---------------- decoder (DCCRN.py:201-206, tools_for_model.py:303-330), polyphase
        dec = []
        out_t, out_t0, out_T = dec_in, 0, T
        F = D4
        for d in range(nl - 1 if taps_only else nl):
            skip = enc[-1 - d]
            Cof = out_t.shape[-1]
            Csk = skip.shape[-1]
            # complex_cat (DCCRN.py:203-204): real = [out_re, skip_re], imag = [out_im, skip_im];
            # the packed weights take K per tap as [out_t (re|im), skip (re|im)] (_dec_w)
            assert Cof == Csk, "DCCRN decoder: input and skip channel counts match"
            segs = [seg_bftc(out_t, 0, Cof, out_t0, out_T), seg_bftc(skip, 0, Csk)]
            dcv, dbn, dpr = self._layer_refs()["dec"][d]
            Co = dcv.out_channels * 2
            last = d == nl - 1
            raw = torch.empty(B, 2 * F, T + 1, Co, **(f32 if last else act))
            Ci = sum(sg.geom.C for sg in segs)
            has_bn = dbn is not None
            bn = pr = mv = st = None
            if has_bn:
                bn, pr = dbn, dpr
                mv = torch.empty(2, Co, **f32) if tape is not None else None
                if train:  # one BatchNorm over both polyphase parities (2 x B*F*(T+1) rows)
                    st = ops.BnStats(bn, Co, 2 * B * F * (T + 1), bn_updates, dev,
                                     stats_out=(mv[0], mv[1]) if mv is not None else None)
            launches = []
            for parity in (0, 1):
                taps = [(dF, -kt) for _, dF in self._DEC_TAPS[parity] for kt in (0, 1)]
                wp, bias = self._dec_w(d, parity, self._cmp(segs, len(taps) * Ci))
                launches.append((segs, taps, B, F, T + 1, Co, wp, bias, raw,
                                 OutMap(2 * F * (T + 1) * Co, (T + 1) * Co, Co, of_mul=2,
                                        of_add=parity)))
            if st is not None and not all(ops.conv_folds(*a) for a in launches):
                st.partials_only()  # the parities dispatch to different kernels: no fold
            for parity, a in enumerate(launches):
                ops.conv(*a, bn_stats=(st, parity == 1) if st is not None else None)
            if has_bn:
                raw = self._norm(raw, bn, pr, st, train, bn_updates, tape, "dec_bn", mv,
                                 gram_taps if (fuse_gram and d < nl - 1) else None, B)
            elif tape is not None:
                tape.setdefault("dec_bn", []).append(None)
            dec.append(raw)
            if on_decoder_tap is not None and d < nl - 1:
                on_decoder_tap(raw)
            out_t, out_t0, out_T = raw, 1, T
            F = 2 * F
        nchw = lambda t: t.permute(0, 3, 1, 2)
        if taps_only:
            return dict(out_wav=None, real=None, imag=None, mask_real=None, mask_imag=None,
                        enc=enc, dec=dec, dec_in=dec_in, spec=spec, est=None, T=T,
                        enc_nchw=[nchw(t) for t in enc], dec_nchw=[nchw(t) for t in dec],
                        lstm_io=lstm_io)
        # ---------------- mask 'E' + ConviSTFT + clamp (DCCRN.py:207-237)
        mask = dec[-1]  # [B][256][T+1][2]
        est = torch.empty(B, T, 516, **f32)
        mr = mi = None
        if want_masks:
            mr = torch.empty(B, T, 257, **f32)
            mi = torch.empty(B, T, 257, **f32)
        ops.mask_e(spec, mask, T, est, mr, mi)
        winv, window = self._istft_w()
        frames = torch.empty(B, T, 400, **f32)
        ops.conv([Seg(est, 0, SegGeom(516, T * 516, 0, 516, 1, T))], [(0, 0)], B, 1, T, 400, winv,
                 None, frames, OutMap(T * 400, 0, 400))
        out_len = (T + 1) * 100 - 400
        wav = torch.empty(B, out_len, **f32)
        ops.ola_hop(frames, window, 100, out_len, 300, True, wav)
        if tape is not None:
            tape.update(spec=spec, est=est, frames=frames, window=window, out_len=out_len, T=T,
                        B=B, train=train)
        return dict(
            out_wav=wav,
            real=est[:, :, :257].permute(0, 2, 1),
            imag=est[:, :, 257:514].permute(0, 2, 1),
            mask_real=mr.permute(0, 2, 1) if mr is not None else None,
            mask_imag=mi.permute(0, 2, 1) if mi is not None else None,
            enc=enc, dec=dec, dec_in=dec_in, spec=spec, est=est, T=T,
            enc_nchw=[nchw(t) for t in enc], dec_nchw=[nchw(t) for t in dec],
            lstm_io=lstm_io)

    @staticmethod
    def clstm_from_dec_in(dec_in):
        """[T,B,P] real/imag enhance outputs (DCCRN.py:186) from the BFTC decoder input."""
        B, D4, T, C6 = dec_in.shape
        Ch = C6 // 2
        r = dec_in[..., :Ch].permute(2, 0, 3, 1).reshape(T, B, Ch * D4)
        i = dec_in[..., Ch:].permute(2, 0, 3, 1).reshape(T, B, Ch * D4)
        return r, i
