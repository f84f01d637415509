"""Streaming DCCRN inference (config C5: 16 kHz, 25 ms window / 6.25 ms hop, hipGraph per hop).

The reference is offline only (``eval.py:47-60``); SURVEY.md §8 f rank 3 pins the streaming path
by equality with the offline eval-mode forward (``DCCRN.forward``, ``DCCRN.py:149-240``) on the
same input.  Per hop of 100 new samples (B streams in parallel):

* ConvSTFT of the newest 400-sample window (one framing GEMM row per stream);
* the encoder is causal in time (``F.pad(x, [1, 0])``, ``tools_for_model.py:237``): each layer keeps
  a 2-frame input window [t-1, t];
* the complex LSTMs carry (h, c) across hops (``clskd_lstm_cell``);
* each decoder layer looks ONE frame ahead (``ConvTranspose2d`` time kernel 2 + ``[..., 1:]``,
  ``DCCRN.py:201-206``), so layer d produces frame t-1-d at hop t from a 2-frame window of its
  input and its skip; the mask (and the enhanced frame) lags the input by ``LOOKAHEAD`` = 6 hops;
* mask 'E' + ConviSTFT frame + overlap-add over a 4-frame ring emits 100 final samples.

Output latency: 9 hops (900 samples = 56.25 ms): 6 decoder look-ahead frames + the 300-sample
STFT centring.  All per-hop buffers are time-major (``[slot][B][F][C]``) so each hop's newest
frame is one contiguous slot that kernels write directly; windows shift by slot copies.  The
steady-state hop (about 70 launches) is captured once as a hipGraph and replayed.

Eval-mode BatchNorm only (running statistics, as at inference).  Flush: after the last input
frame the decoder pipeline drains with zero frames (the offline decoder's out-of-range inputs).
"""
import torch

from . import config as cfg
from . import ops
from .ops import OutMap, Seg, SegGeom

HOP, WIN = 100, 400
LOOKAHEAD = 6  # decoder frames: layer d reads its input one frame ahead, 6 layers
LATENCY_HOPS = LOOKAHEAD + 3  # + the 300-sample centring of the STFT framing


def _seg_tm(buf, slot0=0, nslots=None, c0=0, C=None):
    """Segment over a time-major window buf[S][B][F][Ct] (slots slot0.. as time)."""
    S, B, F, Ct = buf.shape
    C = Ct - c0 if C is None else C
    nslots = S - slot0 if nslots is None else nslots
    return Seg(buf, slot0 * B * F * Ct + c0, SegGeom(C, F * Ct, Ct, B * F * Ct, F, nslots))


class StreamingDCCRN:
    """Hop-by-hop DCCRN enhancement of B parallel streams with a captured hipGraph per hop.

    step(x_hop [B][100]) -> [B][100] enhanced samples, delayed by LATENCY_HOPS hops (None while
    the pipeline fills); finish() drains the look-ahead; process(x [B][L]) runs a whole clip and
    returns the offline-aligned [B][L] output (equal to model.eval()(x) up to fp32 rounding)."""

    def __init__(self, model, batch, graph=True):
        if model.training:
            raise ValueError("StreamingDCCRN runs eval-mode BatchNorm: call model.eval() first")
        self.m = model
        self.B = B = batch
        dev = next(model.parameters()).device
        self.dev = dev
        f32 = dict(device=dev, dtype=torch.float32)
        kn = model.kernel_num
        self.nl = nl = len(kn) - 1
        self.H = H = model.rnn_units // 2
        C6 = kn[-1]
        self.D4 = D4 = 256 // (2 ** nl)
        # ---- buffers (all zero: the causal / centring pads of the first frames)
        self.x_in = torch.zeros(B, HOP, **f32)
        self.wav_out = torch.zeros(B, HOP, **f32)
        self.xwin = torch.zeros(B, WIN, **f32)
        self.xtmp = torch.zeros(B, WIN - HOP, **f32)
        self.spec = torch.zeros(LOOKAHEAD + 1, B, 514, **f32)     # spectra t-6 .. t
        self.spec_b = torch.zeros(B, 256, 1, 2, **f32)            # encoder-0 input frame (BFTC)
        Fi = [256 // (2 ** i) for i in range(nl + 1)]
        Cin = [2] + list(kn[1:-1])
        self.ewin = [torch.zeros(2, B, Fi[i], Cin[i], **f32) for i in range(nl)]   # enc inputs
        self.eraw = [torch.zeros(B, Fi[i + 1], 1, kn[i + 1], **f32) for i in range(nl)]
        # encoder output ring of depth 7 - i: decoder layer 5 - i reads frames (t-6+i, t-5+i)
        self.ering = [torch.zeros(nl + 1 - i, B, Fi[i + 1], kn[i + 1], **f32) for i in range(nl)]
        self.gx = torch.zeros(2, B, 8 * H, **f32)
        self.h = torch.zeros(model.hidden_layers, 2, 2 * B, H, **f32)
        self.c = torch.zeros(model.hidden_layers, 2, 2 * B, H, **f32)
        self.hs = torch.zeros(2, 2 * B, H, **f32)
        self.rio = [(torch.zeros(B, H, **f32), torch.zeros(B, H, **f32))
                    for _ in range(model.hidden_layers)]
        # decoder input windows: d = 0 the LSTM projection (dec_in), d > 0 decoder d-1 output
        Fd = [D4 * (2 ** d) for d in range(nl)]
        Co = [model.decoder[d][0].out_channels * 2 for d in range(nl)]
        self.dwin = [torch.zeros(2, B, D4, C6, **f32)] + \
                    [torch.zeros(2, B, 2 * Fd[d - 1], Co[d - 1], **f32) for d in range(1, nl)]
        self.draw = [torch.zeros(B, 2 * Fd[d], 1, Co[d], **f32) for d in range(nl - 1)]
        self.mask = torch.zeros(B, 256, 2, 2, **f32)   # last decoder output at time slot 1
        self.est = torch.zeros(B, 1, 516, **f32)
        self.frames = torch.zeros(B, 4, WIN, **f32)     # OLA ring u-3 .. u
        self.ftmp = torch.zeros(B, 3, WIN, **f32)
        self.tmp = {}
        self.Fd, self.Co, self.Fi, self.Cin = Fd, Co, Fi, Cin
        # ---- eval-mode BatchNorm coefficients [scale | shift] (fixed at inference)
        self.ebn = [self._bn_coef(model.encoder[i][1]) for i in range(nl)]
        self.dbn = [self._bn_coef(model.decoder[d][1]) for d in range(nl - 1)]
        self.t = 0
        self.graph = None
        self.use_graph = graph
        self.steps_run = 0

    def _bn_coef(self, bn):
        x = torch.empty(1, bn.num_features, device=self.dev)
        return ops.batch_norm_bftc(x, None, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                   False, bn.momentum, bn.eps)

    def _bn_apply(self, x, y, coef, alpha):
        Cn = x.shape[-1]
        sc = coef.data_ptr()
        ops.check(ops.lib().clskd_bn_apply(x.data_ptr(), y.data_ptr(), x.numel() // Cn, Cn, sc,
                                           sc + 4 * Cn, ops.ptr(alpha), ops._dt(x), ops._stream()),
                  "bn_apply")

    def _shift(self, buf):
        """Time-major window: slot k <- slot k+1 for all but the newest slot."""
        S = buf.shape[0]
        if S == 2:
            buf[0].copy_(buf[1])
            return
        tmp = self.tmp.get(id(buf))
        if tmp is None:
            tmp = self.tmp[id(buf)] = torch.empty_like(buf[1:])
        tmp.copy_(buf[1:])
        buf[:-1].copy_(tmp)

    # ------------------------------------------------------------------------------------
    def _hop(self, live_in=True, zero_from=None):
        """One hop.  live_in=False (flush): no new input frame (encoder / LSTM frames are the
        offline out-of-range zeros); zero_from = T: decoder outputs of frames >= T are zero."""
        m, B, nl, H = self.m, self.B, self.nl, self.H
        from .model import DCCRN
        t = self.t
        # ---- shift every window / ring by one frame
        self.xtmp.copy_(self.xwin[:, HOP:])
        self.xwin[:, :WIN - HOP].copy_(self.xtmp)
        self.xwin[:, WIN - HOP:].copy_(self.x_in)
        self._shift(self.spec)
        for w in self.ewin + self.ering + self.dwin:
            self._shift(w)
        self.ftmp.copy_(self.frames[:, 1:])
        self.frames[:, :3].copy_(self.ftmp)
        if live_in:
            # ---- ConvSTFT of the newest window (tools_for_model.py:53-67)
            ops.conv([Seg(self.xwin, 0, SegGeom(HOP, WIN, 0, HOP, 1, 4))],
                     [(0, kt) for kt in range(4)], B, 1, 1, 514, m._stft_w(), None, self.spec[-1],
                     OutMap(514, 0, 514))
            ops.spec_bftc(self.spec[-1].view(B, 1, 514), 1, 258, 256, self.spec_b)
            self.ewin[0][1].copy_(self.spec_b.view(B, 256, 2))
            # ---- encoder (DCCRN.py:171-176): window [t-1, t], taps (kf-2, kt)
            for i in range(nl):
                wp, bias = m._enc_w(i, "fp32")
                Fo, Co = self.Fi[i + 1], m.kernel_num[i + 1]
                ops.conv([_seg_tm(self.ewin[i])], [(kf - 2, kt) for kf in range(5) for kt in range(2)],
                         B, Fo, 1, Co, wp, bias, self.eraw[i], OutMap(Fo * Co, Co, Co), stride_f=2)
                bn, pr = m.encoder[i][1], m.encoder[i][2]
                dst = self.ewin[i + 1][1] if i + 1 < nl else self.ering[i][-1]
                self._bn_apply(self.eraw[i].view(B, Fo, Co), dst, self.ebn[i], pr.weight)
                if i + 1 < nl:
                    self.ering[i][-1].copy_(dst)
            # ---- complex LSTMs (DCCRN.py:178-199), state carried across hops
            C6, Ch, D4 = m.kernel_num[-1], m.kernel_num[-1] // 2, self.D4
            r_in = None
            for li in range(m.hidden_layers):
                packs = m._lstm_w(li, "fp32")
                wp, bias, whh = packs[:3]
                for half in range(2):
                    if li == 0:
                        # newest frame (slot 1) of the last encoder output's 2-frame ring
                        segs = [_seg_tm(self.ering[nl - 1], 1, 1, half * Ch, Ch)]
                        taps = [(f, 0) for f in range(D4)]
                    else:
                        segs = [Seg(r_in[half], 0, SegGeom(H, H, 0, H, 1, 1))]
                        taps = [(0, 0)]
                    ops.conv(segs, taps, B, 1, 1, 8 * H, wp, bias, self.gx[half], OutMap(8 * H, 0, 8 * H))
                ops.lstm_cell(self.gx, 4 * H, 8 * H, whh, 2, 2 * B, H, self.h[li], self.c[li],
                              2 * B * H, H, self.hs, 2 * B * H, H)
                ro, io = self.rio[li]
                ops.complex_combine(self.hs[0, :B], self.hs[1, B:], self.hs[0, B:], self.hs[1, :B], ro, io)
                r_in = (ro, io)
            last = m.enhance[m.hidden_layers - 1]
            packs = m._lstm_w(m.hidden_layers - 1, "fp32")
            for half in range(2):
                ops.conv([Seg(r_in[half], 0, SegGeom(H, H, 0, H, 1, 1))], [(0, 0)], B, 1, 1,
                         last.projection_dim, packs[3 + 2 * half], packs[4 + 2 * half], self.dwin[0][1],
                         OutMap(D4 * C6, 0, 0, 1, C6, D4), out_offset=half * Ch)
        else:
            for r in self.ering:
                r[-1].zero_()
            self.dwin[0][1].zero_()
        # ---- decoder (DCCRN.py:201-206): layer d emits frame t-1-d from [t-1-d, t-d]
        for d in range(nl):
            F, Co = self.Fd[d], self.Co[d]
            ring = self.ering[nl - 1 - d]   # depth d + 2: slots 0, 1 = frames t-1-d, t-d
            Cof, Csk = self.dwin[d].shape[-1], ring.shape[-1]
            last_layer = d == nl - 1
            out_frame = t - 1 - d
            dead = zero_from is not None and out_frame >= zero_from
            dst = self.mask if last_layer else self.draw[d]
            if dead:
                if last_layer:
                    self.mask[:, :, 1].zero_()
                else:
                    self.dwin[d + 1][1].zero_()
                continue
            segs = [_seg_tm(self.dwin[d], 0, 2), _seg_tm(ring, 0, 2)]
            for parity in (0, 1):
                taps = [(dF, 1 - kt) for _, dF in DCCRN._DEC_TAPS[parity] for kt in (0, 1)]
                wp, bias = m._dec_w(d, parity, "fp32")
                if last_layer:  # mask [B][256][2][2], written at time slot 1
                    omap, off = OutMap(256 * 2 * 2, 2 * 2, 2, of_mul=2, of_add=parity), 2
                else:
                    omap, off = OutMap(2 * F * Co, Co, Co, of_mul=2, of_add=parity), 0
                ops.conv(segs, taps, B, F, 1, Co, wp, bias, dst, omap, out_offset=off)
            if not last_layer:
                pr = m.decoder[d][2]
                self._bn_apply(self.draw[d].view(B, 2 * F, Co), self.dwin[d + 1][1], self.dbn[d],
                               pr.weight)
        # ---- mask 'E' on frame t-6, ConviSTFT frame, overlap-add (DCCRN.py:207-237)
        ops.mask_e(self.spec[0].view(B, 1, 514), self.mask, 1, self.est)
        winv, window = m._istft_w()
        ops.conv([Seg(self.est, 0, SegGeom(516, 516, 0, 516, 1, 1))], [(0, 0)], B, 1, 1, WIN, winv,
                 None, self.frames, OutMap(4 * WIN, 0, 0), out_offset=3 * WIN)
        ops.ola_hop(self.frames, window, HOP, HOP, 300, True, self.wav_out)
        self.t += 1

    def _capture(self):
        """Capture the steady-state hop once its kernels' launch plans exist (warm hops)."""
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        snap = self._snapshot()
        with torch.cuda.graph(g, stream=ops.capture_stream(self.dev)):
            self._hop()
        self._restore(snap)   # capture only records: the hop counter must not advance
        self.graph = g

    def _snapshot(self):
        return self.t

    def _restore(self, t):
        self.t = t

    def step(self, x_hop):
        """Feed 100 new samples per stream; returns the enhanced hop 9 hops behind (or None)."""
        self.x_in.copy_(x_hop)
        if self.graph is None and self.use_graph and self.steps_run >= 2:
            self._capture()
        if self.graph is not None:
            self.graph.replay()
            self.t += 1
        else:
            self._hop()
        self.steps_run += 1
        return self.wav_out.clone() if self.t - 1 - LOOKAHEAD >= 3 else None

    def process(self, x):
        """Whole clip x [B][L] (L % 100 == 0) through the hop loop + flush -> [B][L], aligned
        with the offline forward's output."""
        B, L = x.shape
        assert B == self.B and L % HOP == 0
        T = cfg.n_frames(L)
        outs = []
        for t in range(T):
            s = t * HOP
            hop = x[:, s:s + HOP] if s + HOP <= L else torch.zeros(B, HOP, device=x.device)
            y = self.step(hop)
            if y is not None:
                outs.append(y)
        for _ in range(LOOKAHEAD):   # drain the decoder look-ahead with zero frames (eager)
            self.x_in.zero_()
            self._hop(live_in=False, zero_from=T)
            outs.append(self.wav_out.clone())
        return torch.cat(outs, 1)[:, :L]


class FusedStreamingDCCRN(StreamingDCCRN):
    """The same hop as StreamingDCCRN, as ONE launch per hop (clskd_stream_hop,
    csrc/stream_hop.hip): one workgroup per stream walks the ConvSTFT row, encoder, complex
    LSTMs, projection, decoder, mask 'E', iSTFT row and overlap-add with each layer's current
    frame in LDS and the frames the causal convolutions / decoder look-ahead need in per-stream
    rings.  Same step() / process() contract and latency (9 hops); the ~70-launch hop becomes one
    launch, so the hop is no longer bound by launch and dependency latency.  Weights are the
    offline forward's packed fp32 operands in the kernel's k-quad layout [K/4][N][4] (built once;
    re-create the object after changing the model's parameters)."""

    def __init__(self, model, batch):
        super().__init__(model, batch, graph=False)
        m, B, dev = self.m, self.B, self.dev
        from . import _lib
        nl, H, D4 = self.nl, self.H, self.D4
        if nl != 6 or m.hidden_layers != 2:
            raise NotImplementedError("the fused hop is built for the 6-layer, 2-LSTM DCCRN")
        kn = m.kernel_num
        C6 = kn[-1]
        keep = []

        def q4(w, K, ci=None):
            """packed [N][Kp] (first K columns real) -> k-quad [K/4][N][4]; ci: pad each tap's ci
            input channels to a quad (encoder 0's (re, im))."""
            w = w.float()[:, :K]
            N = w.shape[0]
            if ci is not None:
                w = torch.nn.functional.pad(w.reshape(N, K // ci, ci), (0, 4 - ci)).reshape(N, -1)
                K = w.shape[1]
            assert K % 4 == 0, K
            t = w.reshape(N, K // 4, 4).permute(1, 0, 2).contiguous()
            keep.append(t)
            return t.data_ptr()

        def p(t):
            keep.append(t)
            return t.data_ptr()

        a = _lib.StreamHopArgs()
        a.stft_w = q4(m._stft_w(), WIN)
        winv, window = m._istft_w()
        a.istft_w, a.window = q4(winv, 516), p(window)
        for i in range(nl):
            wp, bias = m._enc_w(i, "fp32")
            a.enc_w[i], a.enc_b[i] = q4(wp, 10 * kn[i], ci=2 if i == 0 else None), p(bias)
            a.enc_coef[i], a.enc_alpha[i] = p(self.ebn[i]), p(m.encoder[i][2].weight.detach().float())
            a.enc_cin[i], a.enc_cout[i] = kn[i], kn[i + 1]
        for li in range(2):
            packs = m._lstm_w(li, "fp32")
            K = D4 * (C6 // 2) if li == 0 else H
            whh = packs[2].float().reshape(8 * H, H)  # [2][4H][H] -> n = ws*4H + g
            a.lstm_w[li], a.lstm_b[li], a.lstm_whh[li] = q4(packs[0], K), p(packs[1]), q4(whh, H)
            if li == 1:
                for half in range(2):
                    a.proj_w[half], a.proj_b[half] = q4(packs[3 + 2 * half], H), p(packs[4 + 2 * half])
        for d in range(nl):
            for parity in (0, 1):
                wp, bias = m._dec_w(d, parity, "fp32")
                ci = (C6 if d == 0 else self.Co[d - 1]) + kn[nl - d]
                a.dec_w[d][parity], a.dec_b[d][parity] = q4(wp, (6 if parity == 0 else 4) * ci), p(bias)
            if d < nl - 1:
                a.dec_coef[d], a.dec_alpha[d] = p(self.dbn[d]), p(m.decoder[d][2].weight.detach().float())
            a.dec_ca[d] = C6 if d == 0 else self.Co[d - 1]
            a.dec_cb[d] = kn[nl - d]
            a.dec_co[d] = self.Co[d]
        a.H, a.D4, a.B = H, D4, B
        # per-stream state layout (floats)
        off = 0

        def take(n):
            nonlocal off
            o = off
            off += (n + 3) // 4 * 4
            return o

        a.off_xwin = take(WIN)
        a.off_spec = take(7 * 514)
        for i in range(nl):
            a.off_enc[i] = take((7 - i) * (128 >> i) * kn[i + 1])
        a.off_decin = take(2 * D4 * C6)
        for d in range(nl - 1):
            a.off_dout[d] = take(2 * 2 * self.Fd[d] * self.Co[d])
        a.off_h = take(2 * 4 * H)
        a.off_c = take(2 * 4 * H)
        a.off_frames = take(4 * WIN)
        a.state_stride = off
        self.fstate = torch.zeros(B, off, device=dev, dtype=torch.float32)
        a.state = self.fstate.data_ptr()
        a.x_in, a.wav_out = self.x_in.data_ptr(), self.wav_out.data_ptr()
        self._args, self._keep = a, keep

    def _hop(self, live_in=True, zero_from=None):
        a = self._args
        a.t, a.live = self.t, int(live_in)
        a.zero_from = -1 if zero_from is None else int(zero_from)
        ops.check(ops.lib().clskd_stream_hop(a, ops._stream()), "stream_hop")
        self.t += 1

    def step(self, x_hop):
        self.x_in.copy_(x_hop)
        self._hop()
        self.steps_run += 1
        return self.wav_out.clone() if self.t - 1 - LOOKAHEAD >= 3 else None
