"""KnowledgeDistillation (distill.py:38-148) and the SPKD-output variant (distill_SPKD.py:37-87)
as MI355X-native training-step objects.

``KnowledgeDistillation.training_step((X, y), batch_idx)`` returns the same scalar loss as the
reference: MRSTFT log-magnitude base loss + 14 SPKD terms (6 encoder ReviewKD pairs, 6 decoder
ReviewKD pairs, clstm real/imag), with the local-DCCRN tap contract of SURVEY.md §8 a11.
The whole fwd+loss step is HIP kernels: one shared ConvSTFT, the teacher and student
forwards (train-mode BN), both ReviewKD fusions, ONE batched-Gram launch over all 28 taps,
one SPKD finalize launch, the MRSTFT GEMM + reduction and a final sum.

Deliberate equivalences (documented in DESIGN.md):
  * distill.py:85 and :100 run the student forward twice on the same input in train mode; the
    outputs are identical, so the step runs it once and applies the BN running-stat update twice.
  * Teacher and student share the fixed ConvSTFT kernel (tools_for_model.py:44-47), so the input
    spectrum is computed once.
  * The reference builds NEW random ABF modules each step (distill.py:92-96); here the ABF
    modules are re-drawn every step on the device (``abf_reinit='step'``, the default,
    kaiming_uniform(a=1) like framework.py:194-195) or, as an explicit opt-in for parity tests
    with injected ABF weights, kept fixed (``abf_reinit='once'``).
"""
import collections
import os

import torch
import torch.nn as nn

from . import config as cfg
from . import _lib, ops
from .framework import MultiResolutionSTFTLoss, SPKDLoss, build_review_kd
from .model import DCCRN


_SIDE = {}
# teacher_ahead (clskd_step): per device, the join events of the last two steps and the tensors
# of the last two steps (kept alive until every stream that reads them has passed them)
_AHEAD = {}
_MARKS = None  # diagnostics (tools/stream_marks.py): list collecting (label, event) per step


def _mark(label, stream):
    if _MARKS is not None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        _MARKS.append((label, ev))


# A/B switch: CLSKD_STUDENT_SPLIT=0 keeps the student of precision 'mixed' on the exact fp32 engines
_STUDENT_SPLIT = os.environ.get("CLSKD_STUDENT_SPLIT", "1") == "1"
# the training step of a 'mixed' student (C3): bit 0 — weight gradients on split products
# (csrc/wgrad_x3.hip, the default: 20.2 -> 19.0 ms per step); bit 1 — the taped forward's and the
# backward's data-gradient fp32 convs too (measured +0.2 ms on top: the split engine displaces
# the halo / pointwise kernels of the narrow layers); bit 2 — the taped forward only (the
# data gradients stay exact).  CLSKD_TRAIN_SPLIT=0: the whole training step exact (A/B,
# profiles/r5_train_split_ab.txt)
# default 5 = weight gradients + the taped forward (round 6: 14.93-15.04 -> 14.74-14.87 ms,
# profiles/r6_train_split_ab.txt); 1 = weight gradients only
_TRAIN_SPLIT = int(os.environ.get("CLSKD_TRAIN_SPLIT", "5"))
_SERIAL = os.environ.get("CLSKD_SERIAL_STREAMS") == "1"  # diagnostic: the whole step on one stream
# conv_gemm8's persistent grid inside the concurrent four-stream step: 7/8 of the CUs (224 of
# 256), so the wide teacher / ReviewKD GEMMs leave a CU per XCD group to the other streams'
# kernels instead of queueing them behind a full-chip grid (measured 5.31-5.32 vs 5.37-5.39 ms
# per C2 step, interleaved on one box; tools/grid_ab.sh).  The tile deal changes, not the tiles
# or their K order: results are bitwise the full grid's (tests/test_gpu_parity.py).  0 = every
# CU; a serialized step (the census: isolated kernel times) and taped training forwards keep the
# full grid.
_STEP_G8_GRID_FRAC = float(os.environ.get("CLSKD_STEP_G8_GRID_FRAC", "0.875"))
_NCU = {}


def _step_g8_grid(dev):
    if _STEP_G8_GRID_FRAC <= 0 or _STEP_G8_GRID_FRAC >= 1:
        return 0
    n = _NCU.get(dev.index)
    if n is None:
        n = _NCU[dev.index] = torch.cuda.get_device_properties(dev).multi_processor_count
    return max(8, int(n * _STEP_G8_GRID_FRAC) // 8 * 8)


class serialized_streams:
    """Context manager: every side stream of the step is the caller's stream (one serial
    stream) — used by bench.py for its per-kernel census, so kernel durations are isolated ones
    (as rocprofv3's kernel trace sees them) instead of times shared with concurrent streams."""

    def __enter__(self):
        global _SERIAL
        self._prev, _SERIAL = _SERIAL, True
        return self

    def __exit__(self, *exc):
        global _SERIAL
        _SERIAL = self._prev
        return False


def _side_stream(dev, which=0):
    """Extra HIP streams per device.  which = 0, 1: the student chain and the ReviewKD-encoder /
    MRSTFT chain run beside the teacher, overlapping the latency-bound LSTM recurrences and small
    kernels with the GEMMs.  which = 2: the teacher's stream (the step's critical path when the
    three share the CUs).  All at equal priority: a high-priority teacher stream measured 0.5-1 %
    slower on MI355X (the side chains' small kernels then queue behind the teacher's large
    GEMMs), CU-masked side streams (hipExtStreamCreateWithCUMask leaving 32-128 CUs to the
    teacher) 8.6-9.9 ms against 5.6 ms; both experiments were removed in round 4."""
    if _SERIAL:
        return torch.cuda.current_stream(dev)
    key = (torch.device(dev).index, which)
    if key not in _SIDE:
        _SIDE[key] = ops.prepare_stream(torch.cuda.Stream(device=dev))
    return _SIDE[key]




class _SlabRefs:
    """Slab ranges of several GramSlabs launches (kept alive together) in pair order."""

    def __init__(self, refs, owners):
        self.refs, self.owners = refs, owners


def _gram_bftc(t, c0=0, Cs=None):
    affine = None
    if isinstance(t, ops.DeferredBN):  # BatchNorm folded into the Gram's loads
        t, affine = t.raw, t.coef
    B, Fn, Tn, Ct = t.shape
    Cs = Ct if Cs is None else Cs
    return ops.GramView(t, 0, Fn * Tn * Ct, Fn * Tn, Ct, c0, Cs, affine)


def _validation_step(module, batch):
    """distill.py:149-199 (and distill_SPKD.py's copy): for every utterance of the batch the
    student's estimate (eval-mode forward, as Lightning's validation loop runs it, no grad; the
    one-source PIT of the reference is the identity), asteroid get_metrics' si_sdr and stoi of
    the estimate and of the unprocessed mixture against the clean source, then the batch means
    of si_sdr, stoi and their improvements — the dict the reference passes to self.log_dict.
    All metrics run on the device (clskd.metrics); returned as Python floats."""
    from . import metrics
    x, y = batch
    x = x.float().reshape(x.shape[0], -1).contiguous()
    y = y.float().reshape(x.shape[0], -1).contiguous()
    student = module.student
    was = student.training
    student.eval()
    try:
        with torch.no_grad():
            est = student(x, is_feat=True)
            utt = metrics.get_metrics(x, y, est, sample_rate=module.cfg.fs)
            res = metrics.summarize(utt)
    finally:
        student.train(was)
    module.last_val = {k: float(v) for k, v in res.items()}
    return module.last_val


class KnowledgeDistillation(nn.Module):
    """distill.py:38-229 without Lightning: same constructor and step signature.

    Limitation of abf_reinit='step' (the default): the ABF re-draw rewrites the ReviewKD weights
    in place at the start of every training_step, and the autograd tape of a step checks their
    version, so two forwards before one backward (e.g. loss1 + loss2 summed for manual gradient
    accumulation) raise a RuntimeError in the first step's backward instead of using the
    overwritten weights.  The reference builds fresh ABF modules per step (distill.py:92-96) and
    allows that pattern; here, call backward after each training_step (Lightning's automatic
    optimisation does), or use abf_reinit='once'."""

    def __init__(self, teacher, student, sftf_loss=MultiResolutionSTFTLoss, spkd_loss=SPKDLoss,
                 cfg=cfg, abf_reinit="step", precision="fp32"):
        super().__init__()
        self.automatic_optimization = True
        self.teacher = teacher
        for p in self.teacher.parameters():
            p.requires_grad = False
        self.student = student
        self.spkd_loss = spkd_loss
        self.stft_loss = sftf_loss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100])
        self.cfg = cfg
        self.abf_reinit = abf_reinit
        self.review_encoder = build_review_kd(None, "encoder")
        self.review_decoder = build_review_kd(None, "decoder")
        self.last = None
        # ABF re-draw: Philox keys from torch's CPU generator (torch.manual_seed reproducible)
        k = torch.randint(0, 2 ** 62, (2,), dtype=torch.int64)
        self._draw_seed = {"encoder": int(k[0]), "decoder": int(k[1])}
        self._draw_state = {}
        self._draw_jobs = {}
        self.set_precision(precision)

    def set_precision(self, precision):
        """"fp32": every GEMM on exact-f32 MFMA.  "mixed": the frozen teacher and the ReviewKD
        fusions (95 % of the step's FLOPs; they only feed the SPKD similarity Grams) run bf16
        MFMA operands with fp32 accumulation; the student — whose waveform is the product and
        the SI-SNR / RMS parity target — keeps fp32 storage and accumulation, its fp32 convs on
        3 x bf16 split products (compute 'f32x3': <= ~3 * 2^-18 relative per product, against the
        reference training script's TF32 at 2^-11; exact fp32 under a tape / in training)."""
        if precision not in ("fp32", "mixed"):
            raise ValueError(precision)
        self.precision = precision
        c = "bf16" if precision == "mixed" else "fp32"
        self.teacher.compute = c
        self.review_encoder.set_compute(c)
        self.review_decoder.set_compute(c)
        self.student.compute = "f32x3" if (precision == "mixed" and _STUDENT_SPLIT) else "fp32"
        self.student.train_split = _TRAIN_SPLIT if self.student.compute == "f32x3" else 0
        return self

    def forward(self, x):
        return self.student(x)

    def configure_optimizers(self):
        return torch.optim.Adam(self.student.parameters(), lr=self.cfg.learning_rate)

    def _reinit_abf(self, which=None):
        """Re-draw the ABF weights (framework.py:194-195 / distill.py:92-96) of one ReviewKD
        module (which = 'encoder' | 'decoder') or of both: one clskd_uniform_redraw launch per
        module on the current stream (parameters and packed operands written together)."""
        if self.abf_reinit != "step":
            return
        names = ("encoder", "decoder") if which is None else (which,)
        for name in names:
            rk = self.review_encoder if name == "encoder" else self.review_decoder
            jobs = [j for abf in rk.abfs for j in abf.redraw_jobs()]
            dev = jobs[0][0].device
            st = self._draw_state.get((name, dev))
            if st is None:  # {draw counter, ticket} per module: the two modules draw on
                st = torch.zeros(2, dtype=torch.int64, device=dev)  # different streams
                self._draw_state[(name, dev)] = st
            key = tuple((w.data_ptr(), wp.data_ptr() if wp is not None else 0) for w, wp, *_ in jobs)
            arr = self._draw_jobs.get((name, key))
            if arr is None:
                arr = (_lib.DrawJob * len(jobs))()
                for i, (w, wp, cin, ntap, bound) in enumerate(jobs):
                    assert w.dtype == torch.float32 and w.is_contiguous()
                    if wp is not None:
                        assert wp.is_contiguous() and wp.shape[0] == w.shape[0]
                    arr[i] = _lib.DrawJob(w.data_ptr(), wp.data_ptr() if wp is not None else None,
                                          w.numel(), cin, ntap, wp.shape[1] if wp is not None else 0,
                                          ops._dt(wp) if wp is not None else 0, bound, i)
                self._draw_jobs = {k: v for k, v in self._draw_jobs.items() if k[0] != name}
                self._draw_jobs[(name, key)] = arr
            ops.check(ops.lib().clskd_uniform_redraw(arr, len(jobs), self._draw_seed[name],
                                                     st.data_ptr(), ops._stream()), "uniform_redraw")
            for abf in rk.abfs:
                abf.after_redraw()

    def _wants_grad(self):
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.student.parameters())

    def training_step(self, batch, batch_idx=0, return_parts=False):
        """distill.py:72-148.  Under autograd (grad enabled, trainable student) the returned loss
        is connected to the student's parameters: loss.backward() runs the HIP backward
        (clskd.backward) and accumulates into .grad, as Lightning's automatic optimisation
        expects."""
        X, y = batch
        if self._wants_grad() and not return_parts:
            params = [p for p in self.student.parameters() if p.requires_grad]
            return _CLSKDLoss.apply(self, X, y, *params)
        out = clskd_step(self.teacher, self.student, self.review_encoder, self.review_decoder,
                         self.stft_loss, X, y, reinit=self._reinit_abf,
                         teacher_ahead=getattr(self, "teacher_ahead", False))
        self.last = out
        if return_parts:
            return out
        return out["loss"]

    def validation_step(self, batch, batch_idx=0):
        """distill.py:149-199: {si_sdr, si_sdr_imp, stoi, stoi_imp} over the batch."""
        return _validation_step(self, batch)

    def forward_with_tape(self, X, y):
        out = clskd_step(self.teacher, self.student, self.review_encoder, self.review_decoder,
                         self.stft_loss, X, y, reinit=self._reinit_abf, tape=True)
        self.last = out
        return out

    def backward_into(self, out, grads, accumulate=False, upstream=1.0):
        """Student gradients of upstream * out['loss'] into `grads` (parameter -> fp32 tensor)."""
        from .backward import clskd_backward
        ts = getattr(self.student, "train_split", 0)
        with ops.split_products(bool(ts & 2), wgrad=bool(ts & 1)):
            clskd_backward(out, self.student, self.review_encoder, self.review_decoder, grads,
                           acc_params=accumulate, upstream=upstream)

    def train_step(self, batch, flat, opt):
        """One C3 training step without autograd bookkeeping: fwd+loss (tape) -> HIP backward
        into the flat gradient buffer -> (multi-rank) one all-reduce -> one Adam launch.
        flat: train.FlatParams(self.student); opt: train.FlatAdam(flat, ...)."""
        from .train import allreduce_grads
        X, y = batch
        out = self.forward_with_tape(X, y)
        self.backward_into(out, flat.grad_dict())
        scale = allreduce_grads(flat)
        opt.step(grad_scale=scale)
        return out["loss"]


@torch.no_grad()
def clskd_step(teacher, student, review_encoder, review_decoder, stft_loss, X, y, reinit=None,
               tape=False, teacher_ahead=False):
    """One CLSKD fwd+loss step (distill.py:72-148).  Returns a dict of device tensors.
    tape=True additionally records what clskd.backward.clskd_backward needs (result['tape']).

    teacher_ahead=True (back-to-back steps over inputs already resident on the device: X and y
    must not be written on the caller's stream between steps): the frozen teacher's chain of
    this step — the step's critical path — does not wait for the previous step's join, only for
    the join of the step before it, so it runs while the previous step's ReviewKD / Gram / loss
    tail finishes.  Every other chain still starts after the previous step's join (the student's
    BatchNorm running statistics and the ABF re-draws stay step-ordered), and each step's tensors
    are held until two steps later, so no buffer is reused while another stream may read it.
    The work and the results are those of the serial schedule; only the overlap changes.  Not
    under graph capture, tapes or serialised streams."""
    if not (isinstance(teacher, DCCRN) and isinstance(student, DCCRN)):
        raise TypeError("clskd_step expects clskd.DCCRN teacher and student")
    if tape or not X.is_cuda:
        return _clskd_step(teacher, student, review_encoder, review_decoder, stft_loss, X, y,
                           reinit, tape, teacher_ahead)
    # the concurrent step's conv_gemm8 grid cap — also for the serialised census step
    # (serialized_streams), so the census times exactly the kernel instances the timed steps run
    # (a capped grid keeps the data-parallel tile deal: no stream-K)
    from . import _lib
    prev = _lib.set_g8_grid(_step_g8_grid(X.device))
    try:
        return _clskd_step(teacher, student, review_encoder, review_decoder, stft_loss, X, y,
                           reinit, tape, teacher_ahead)
    finally:
        _lib.set_g8_grid(prev)


def _clskd_step(teacher, student, review_encoder, review_decoder, stft_loss, X, y, reinit, tape,
                teacher_ahead):
    X0, y0 = X, y
    X = X.float()
    if X.dim() == 3:
        X = X.squeeze(1)
    X = X.contiguous()
    y = y.float().reshape(X.shape[0], -1).contiguous()
    B = X.shape[0]
    dev = X.device
    _mark("start", torch.cuda.current_stream(dev))
    capturing = torch.cuda.is_current_stream_capturing()
    ring = _AHEAD.setdefault(dev.index, dict(joins=collections.deque(maxlen=2),
                                             held=collections.deque(maxlen=2)))
    # ahead only when BOTH previous steps ran ahead-mode (their tensors are held in the ring): a
    # step run with teacher_ahead off freed its teacher-stream blocks at return, and an ahead
    # teacher that waited only for the join before it could reuse them while that step's Grams
    # still read them
    ahead = (teacher_ahead and not _SERIAL and not tape and not capturing
             and len(ring["joins"]) == 2 and all(h is not None for h in ring["held"]))
    if ahead and (X.data_ptr() != X0.data_ptr() or y.data_ptr() != y0.data_ptr()):
        # the conversions above were queued on the caller's stream, which the ahead teacher chain
        # does not wait for: the resident-input contract of teacher_ahead is fp32 contiguous X, y
        raise ValueError("clskd_step(teacher_ahead=True) needs fp32 contiguous [B, L] inputs "
                         "already resident on the device")
    spec_ev = None
    # teacher_ahead under graph capture: the ahead LAYOUT (the spectrum on the teacher stream,
    # the student waiting for it by event) with the teacher forked from the capture stream like
    # every branch; clskd.graph.AheadStepExecutor replays two such captures alternately, each
    # one's teacher stream waiting for the end of its own previous replay instead of the fork
    if ahead or (teacher_ahead and capturing and not _SERIAL and not tape):
        # the teacher chain (spectrum included) waits for the join of step i-1, not step i
        tstream = _side_stream(dev, 2)
        if ahead:
            tstream.wait_event(ring["joins"][0])
        else:
            tstream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(tstream):
            spec = teacher.spectrum(X)
        spec_ev = torch.cuda.Event()
        spec_ev.record(tstream)
    else:
        spec = teacher.spectrum(X)
    # both ConvSTFTs are the fixed (win 400, hop 100, fft 512) kernel of the same window type
    s_spec = spec if teacher.win_type == student.win_type else None
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev, 0)
    side2 = _side_stream(dev, 1)
    # spec ready; the previous step's work (joined into main) is done before buffers are reused
    side.wait_stream(main)
    side2.wait_stream(main)
    if spec_ev is not None:
        side.wait_event(spec_ev)
    buf = torch.empty(16, dtype=torch.float32, device=dev)  # [sc, mag, spkd x 14]
    # Everything that depends on the student alone runs beside the teacher forward (main):
    #   side : student forward -> decoder-ABF re-draw -> ReviewKD decoder fusions
    #   side2: encoder-ABF re-draw -> (student encoder done) ReviewKD encoder fusions ->
    #          (student done) MRSTFT base loss on (student wav, clean) (distill.py:100-101)
    # ReviewKD: distill.py:92-96, tap contract SURVEY.md §8 a11.
    held = {}
    tapes = dict(s={}, re=[], rd=[], ms=[]) if tape else None
    # the ReviewKD conv2s (+ BN, SPKD Grams) run on the caller's stream, which is otherwise idle
    # between the teacher's encoder Grams and the join: they are off the level-to-level residual
    # chain of the fusions (framework.py:254-261), which stays on side / side2
    c2 = main
    if reinit is not None:  # fresh ABF modules (distill.py:92-96): only ReviewKD reads them
        with torch.cuda.stream(side2):
            reinit("encoder")

    # SPKD Gram partials run on the stream that produced their features, as soon as those
    # exist (main: ReviewKD maps (conv2 fork) + student dec_in halves and the teacher's encoder
    # taps; tstream: teacher decoder taps); one finalize on main after the join
    # (framework.py:150-172).
    def fork_review_encoder(enc):
        ev = torch.cuda.Event()
        ev.record(side)
        with torch.cuda.stream(side2):
            side2.wait_event(ev)
            _mark("side2: student encoder ready", side2)
            s_enc = review_encoder.forward_bftc(enc, defer_bn=True,
                                                tape=tapes["re"] if tapes else None,
                                                conv2_stream=c2)
            _mark("side2: review encoder done", side2)
            held["s_enc"] = s_enc
        with torch.cuda.stream(c2):
            held["g_enc"] = ops.GramSlabs([_gram_bftc(a) for a in s_enc], B)
            _mark("enc grams done", c2)

    # ReviewKD-decoder pipelined behind the student decoder on the caller's stream: level j
    # (framework.py:254-261, forward order) starts as soon as its student tap exists
    rd = dict(res=None, outs=[], taps=[])

    def review_decoder_level(tap):
        ev = torch.cuda.Event()
        ev.record(side)
        with torch.cuda.stream(main):
            main.wait_event(ev)
            j = len(rd["outs"])
            if j == 0 and reinit is not None:
                reinit("decoder")
            abf = review_decoder.abfs[j]
            tp = {} if tapes else None
            if j == 0:
                out, res = abf.forward_bftc(tap, out_shape=review_decoder.out_shapes[0],
                                            defer_bn=True, tape=tp)
            else:
                out, res = abf.forward_bftc(tap, rd["res"], review_decoder.shapes[j],
                                            review_decoder.out_shapes[j], defer_bn=True, tape=tp)
            if tapes:
                tapes["rd"].append(tp)
            rd["res"] = res
            rd["outs"].append(out)
            rd["taps"].append(tap)

    def run_student():
        with torch.cuda.stream(side):
            sf = student.run(X, train=student.training, bn_updates=2 if student.training else 0,
                             spec=s_spec, want_masks=False, on_encoder=fork_review_encoder,
                             tape=tapes["s"] if tapes else None,
                             on_decoder_tap=review_decoder_level)
            student_done = torch.cuda.Event()
            student_done.record(side)
            _mark("side: student done", side)
        rstream = main
        with torch.cuda.stream(rstream):
            s_dec = rd["outs"]
            assert len(s_dec) == len(review_decoder.abfs)
            Chs = sf["dec_in"].shape[-1] // 2
            g_dec = ops.GramSlabs([_gram_bftc(a) for a in s_dec] +
                                  [_gram_bftc(sf["dec_in"], 0, Chs), _gram_bftc(sf["dec_in"], Chs, Chs)],
                                  B)
            _mark("review decoder + grams done", rstream)
        with torch.cuda.stream(side2):
            side2.wait_event(student_done)
            stft_loss(sf["out_wav"], y, out2=buf[0:2], tape=tapes["ms"] if tapes else None)
            _mark("side2: mrstft done", side2)
        out_s.update(sf=sf, s_dec=s_dec, g_dec=g_dec)

    def run_teacher():
        tstream = _side_stream(dev, 2)
        if not ahead:
            tstream.wait_stream(main)
        # train-mode teacher: every BatchNorm'd tap's apply pass is fused with its SPKD Gram
        # partials (DCCRN.run(gram_taps=...), ops.bn_apply_gram) — the teacher taps are never
        # read again for their Grams; dec_in (the LSTM projection, no BatchNorm) and its two
        # clstm halves get one Gram launch as soon as it exists
        fused = teacher.training
        tg, dg = [], {}

        def dec_in_grams(tap):
            if "g" not in dg:  # the first decoder-side tap is dec_in
                Cht = tap.shape[-1] // 2
                dg["g"] = ops.GramSlabs([_gram_bftc(tap), _gram_bftc(tap, 0, Cht),
                                         _gram_bftc(tap, Cht, Cht)], B)

        with torch.cuda.stream(tstream):
            # the teacher's last decoder layer, mask and iSTFT are dead for the loss: stop at its taps
            tf = teacher.run(X, train=teacher.training, bn_updates=1, spec=spec, want_masks=False,
                             taps_only=True, gram_taps=tg if fused else None,
                             on_decoder_tap=dec_in_grams if fused else None,
                             mark=(lambda lab: _mark("teacher: " + lab, tstream))
                             if _MARKS is not None else None)
            _mark("teacher: done", tstream)
            if fused:
                # taps in run order: the nl encoder outputs, then the first nl - 1 decoder
                # outputs (the last decoder layer is dead for the loss); any teacher depth
                nl = len(teacher.kernel_num) - 1
                assert len(tg) == 2 * nl - 1 and "g" in dg, (len(tg), nl)
                d = dg["g"]
                g_te = _SlabRefs([g.refs[0] for g in tg[:nl]], tg[:nl])
                g_td = _SlabRefs([d.refs[0]] + [g.refs[0] for g in tg[nl:]] + d.refs[1:],
                                 (d, tg[nl:]))
            else:  # eval-mode teacher: BatchNorm applied in place, Gram passes of their own
                g_te = ops.GramSlabs([_gram_bftc(a) for a in tf["enc"]], B)
                t_dec = [tf["dec_in"]] + tf["dec"][:5]
                Cht = tf["dec_in"].shape[-1] // 2
                g_td = ops.GramSlabs([_gram_bftc(a) for a in t_dec] +
                                     [_gram_bftc(tf["dec_in"], 0, Cht),
                                      _gram_bftc(tf["dec_in"], Cht, Cht)], B)
            _mark("teacher: grams done", tstream)
        out_t.update(tf=tf, g_td=g_td, g_te=g_te)

    out_s, out_t = {}, {}
    # host enqueue order: the teacher chain (the critical path) first — wait_stream dependencies
    # are taken at enqueue time (measured: student chain first = 7.29 ms vs 5.60 per C2 step)
    run_teacher()
    run_student()
    sf, s_dec, g_dec = out_s["sf"], out_s["s_dec"], out_s["g_dec"]
    tf, g_td, g_te = out_t["tf"], out_t["g_td"], out_t["g_te"]
    s_enc, g_enc = held["s_enc"], held["g_enc"]
    tstream = _side_stream(dev, 2)
    g_t = _SlabRefs(g_te.refs + g_td.refs, (g_te, g_td))
    main.wait_stream(tstream)
    main.wait_stream(side)
    main.wait_stream(side2)
    # returned side-stream tensors: their blocks must not be recycled by a later side-stream
    # allocation before the caller's reads on `main` are done
    sf["out_wav"].record_stream(main)
    _mark("main: joined", main)
    s_refs = g_enc.refs + g_dec.refs
    assert len(s_refs) == 14 and len(g_t.refs) == 14
    ops.spkd_finalize(s_refs, g_t.refs, B, batchmean=True, out=buf[2:])
    total = torch.empty((), dtype=torch.float32, device=dev)
    ops.sum_f32(buf[1:], total)
    _mark("main: end", main)
    if not capturing:
        join = torch.cuda.Event()
        join.record(main)
        ring["joins"].append(join)
        # held until two steps later (teacher_ahead: the next step's teacher may still overlap
        # this step's readers of these tensors on other streams)
        ring["held"].append((out_s, out_t, held, rd, spec, X, y) if teacher_ahead else None)
    return dict(loss=total, base=buf[1], sc=buf[0], spkd=buf[2:], enc=buf[2:8], dec=buf[8:14],
                clstm_real=buf[14], clstm_img=buf[15], student_wav=sf["out_wav"],
                teacher_wav=tf["out_wav"], s_enc=ops.MaterializingList(s_enc),
                s_dec=ops.MaterializingList(s_dec), t=tf, s=sf,
                gram_slabs=(g_enc, g_dec, g_t), s_enc_list=s_enc, s_dec_list=s_dec, tape=tapes)


class _CLSKDLoss(torch.autograd.Function):
    """Connects the HIP fwd+loss step to autograd: forward = clskd_step(tape=True), backward =
    clskd.backward over that tape, returning one gradient per student parameter."""

    @staticmethod
    def forward(ctx, kd, X, y, *params):
        out = kd.forward_with_tape(X, y)
        ctx.kd, ctx.out, ctx.params = kd, out, params
        return out["loss"].clone()

    @staticmethod
    def backward(ctx, gout):
        kd, out, params = ctx.kd, ctx.out, ctx.params
        up = float(gout.reshape(()).item()) if gout is not None else 1.0
        grads = {p: torch.empty_like(p, dtype=torch.float32) for p in params}
        kd.backward_into(out, grads, accumulate=False, upstream=up)
        ctx.out = None
        return (None, None, None) + tuple(grads[p] for p in params)


class SPKDDistillation(nn.Module):
    """distill_SPKD.py:37-87: MRSTFT base + SPKD on the output waveforms (config C4)."""

    def __init__(self, teacher, student, sftf_loss=MultiResolutionSTFTLoss, spkd_loss=SPKDLoss,
                 cfg=cfg, precision="fp32"):
        super().__init__()
        self.teacher = teacher
        for p in self.teacher.parameters():
            p.requires_grad = False
        self.student = student
        self.spkd_loss = spkd_loss
        self.stft_loss = sftf_loss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100])
        self.cfg = cfg
        self.set_precision(precision)

    def set_precision(self, precision):
        """As KnowledgeDistillation.set_precision: "mixed" runs the frozen teacher (no_grad in
        distill_SPKD.py:75-76; its waveform only feeds the SPKD Gram) on bf16 MFMA operands with
        fp32 accumulation; "fp16" the same on IEEE-half operands and fp16 feature storage
        (configuration C4 of BASELINE.json: "batch=32 x 4 s fp16"); the student stays fp32."""
        if precision not in ("fp32", "mixed", "fp16"):
            raise ValueError(precision)
        self.precision = precision
        self.teacher.compute = {"mixed": "bf16", "fp16": "fp16"}.get(precision, "fp32")
        self.student.compute = "fp32"
        return self

    def forward(self, x):
        return self.student(x)

    def validation_step(self, batch, batch_idx=0):
        """distill_SPKD.py's validation step (the same as distill.py:149-199)."""
        return _validation_step(self, batch)

    @torch.no_grad()
    def training_step(self, batch, batch_idx=0, return_parts=False):
        X, y = batch
        X = X.float().reshape(X.shape[0], -1).contiguous()
        y = y.float().reshape(X.shape[0], -1).contiguous()
        spec = self.teacher.spectrum(X)
        buf = torch.empty(3, dtype=torch.float32, device=X.device)
        # two chains joined before the SPKD Gram: the teacher forward (the critical path) on the
        # caller's stream, the student forward + MRSTFT base loss (distill_SPKD.py:73-79) beside
        # it on a side stream; the side stream first waits for spec and the previous step
        main = torch.cuda.current_stream(X.device)
        side = _side_stream(X.device, 0)
        side.wait_stream(main)
        t = self.teacher.run(X, train=self.teacher.training, bn_updates=1, spec=spec,
                             want_masks=False)["out_wav"]
        with torch.cuda.stream(side):
            s = self.student.run(X, train=self.student.training, bn_updates=1, spec=spec,
                                 want_masks=False)["out_wav"]
            self.stft_loss(s, y, out2=buf[0:2])
        main.wait_stream(side)
        s.record_stream(main)  # side-stream allocation read (and returned) on the caller's stream
        ops.spkd_losses([(ops.gram_view(s), ops.gram_view(t))], X.shape[0], out=buf[2:3])
        total = torch.empty((), dtype=torch.float32, device=X.device)
        ops.sum_f32(buf[1:], total)
        if return_parts:
            return dict(loss=total, base=buf[1], spkd=buf[2], student_wav=s, teacher_wav=t)
        return total
