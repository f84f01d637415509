"""Backward pass of the CLSKD step (student gradients) on libclskd_hip.so.

The reference trains with Lightning's automatic optimisation: ``loss.backward()`` through the
teacher-frozen graph of ``distill.py:72-148`` and ``Adam(student.parameters())``
(``distill.py:202-204``).  Here the backward is an explicit reverse schedule over a forward tape
(``DCCRN.run(tape=...)``, ``ReviewKD.forward_bftc(tape=...)``, ``MultiResolutionSTFTLoss(...,
tape=...)``):

* every data gradient of a GEMM (complex Conv2d, polyphase ConvTranspose2d, ABF 1x1 / 3x3,
  LSTM projections, the STFT framing GEMMs) is ANOTHER launch of the implicit-GEMM conv engine
  with transposed packed weights and a K table that reads the output gradient — stride-2 encoder
  convs become two polyphase launches, the decoder's polyphase pair becomes one stride-2 gather;
  contributions of several consumers sum in place (``accumulate``);
* every weight gradient is ``clskd_conv2d_wgrad`` over the forward's own descriptor;
* BatchNorm / PReLU / ABF fusion / mask / OLA / pad / log-magnitude / LSTM BPTT / SPKD have
  dedicated kernels (``csrc/norm_bwd.hip``, ``lstm.hip``, ``loss.hip``);
* packed-operand gradients map back onto the module parameters through index maps derived once
  from the packing transform (``clskd_index_gather``).

Gradients are fp32; every reduction has a fixed order, so a step's gradients are bitwise
repeatable.  Parity: ``tests/test_gpu_parity.py::test_clskd_backward_*`` against the CPU oracle's
autograd (``oracle/ref_cpu.py``).
"""
import os
import weakref

import numpy as np
import torch

from . import ops
from .ops import OutMap, Seg, SegGeom, seg_bftc

f32 = torch.float32


def _zeros(shape, dev):
    return torch.zeros(shape, device=dev, dtype=f32)


def _empty(shape, dev):
    return torch.empty(shape, device=dev, dtype=f32)


# ------------------------------------------------------------------------------------------
# packed-gradient -> parameter index maps
# ------------------------------------------------------------------------------------------
_MAPS = {}


def unpack_maps(key, fn, shapes, Kp, dev):
    """Index maps from a packed operand [N][Kp] (row-major) back to each parameter of `shapes`.

    fn(*tensors) must be the packing transform (cat / permute / negate) returning [N, K]; it is
    evaluated on float64 tensors holding +(flat parameter index + 1), so each packed entry names
    its source element and sign.  Returns one (idx [n_i, J] int32, sgn [n_i, J] fp32) per
    parameter (J = max multiplicity, idx = -1 padding)."""
    k = (key, tuple(tuple(s) for s in shapes), Kp, str(dev))
    if k in _MAPS:
        return _MAPS[k]
    offs = np.cumsum([0] + [int(np.prod(s)) for s in shapes])
    qs, ps, ss = [], [], []
    for i, s in enumerate(shapes):
        # the packing is linear: evaluate it with only parameter i non-zero, so packed entries
        # that sum several parameters (e.g. br - bi) still name one source each
        ts = [torch.zeros(sh, dtype=torch.float64) for sh in shapes]
        ts[i] = torch.arange(int(offs[i]) + 1, int(offs[i + 1]) + 1, dtype=torch.float64).reshape(s)
        packed = fn(*ts).detach().cpu().numpy()
        N, K = packed.shape
        full = np.zeros((N, Kp), np.float64)
        full[:, :K] = packed
        flat = full.ravel()
        nz = np.nonzero(flat)[0]
        qs.append(np.abs(flat[nz]).astype(np.int64) - 1)
        ps.append(nz)
        ss.append(np.sign(flat[nz]))
    q, pos, sg = np.concatenate(qs), np.concatenate(ps), np.concatenate(ss)
    order = np.argsort(q, kind="stable")
    q, pos, sg = q[order], pos[order], sg[order]
    total = int(offs[-1])
    counts = np.bincount(q, minlength=total)
    J = max(1, int(counts.max()))
    first = np.zeros(total + 1, np.int64)
    first[1:] = np.cumsum(counts)
    rank = np.arange(len(q)) - first[q]
    idx = -np.ones((total, J), np.int64)
    sgn = np.zeros((total, J), np.float32)
    idx[q, rank] = pos
    sgn[q, rank] = sg
    out = []
    for i in range(len(shapes)):
        a, b = int(offs[i]), int(offs[i + 1])
        out.append((torch.from_numpy(idx[a:b].astype(np.int32)).to(dev),
                    torch.from_numpy(sgn[a:b]).to(dev)))
    _MAPS[k] = out
    return out


# Packed-gradient -> parameter scatters of one backward pass (acc = False: every parameter's
# gradient is written once) are collected here and launched together at the end of the student's
# backward (ops.index_gather_jobs: ~70 launches -> 2); None: launch each one at once
_SCATTERS = None


def _scatter(src, maps, grads, acc):
    for (idx, sgn), g in zip(maps, grads):
        if g is not None:
            if _SCATTERS is not None and not acc:
                _SCATTERS.append((src, idx, sgn, g))
            else:
                ops.index_gather(src, idx, sgn, g, accumulate=acc)


# ------------------------------------------------------------------------------------------
# transposed (data-gradient) weights, cached per packed forward weight
# ------------------------------------------------------------------------------------------
_TW = {}
_TW_MAX = 512  # entries; a C3 step of one model uses ~60


def _tw(key, src, build):
    """Transposed/packed weight cache.  An entry is valid only for the very tensor object it was
    built from (weak reference) at the same in-place version: keys carry id()s of modules, and a
    module or tensor freed by an earlier step can hand its id and storage address to a new one
    (seen as a flaky mixed-precision gradient test: a new model's ABF backward ran with the
    previous model's re-drawn ABF weights; regression test
    tests/test_host_cpu.py::test_tw_cache_rebuilds_for_a_new_source_identity).  Entries whose
    source died are dropped on every insert, and the cache is bounded (oldest first), so freed
    models do not keep device copies of their weights alive."""
    k = (src.data_ptr(), src._version)
    tok = ops.capture_token()  # entries built inside a capture serve that capture only
    ent = _TW.get(key)
    if ent is not None and ent[0] == k and ent[2]() is src and ops.cache_entry_usable(ent[3], tok):
        ops.capture_keep(ent[1], tok)
        return ent[1]
    with torch.no_grad():
        w = _tw_build(key, src, build)
    _tw_install(key, src, w, tok)
    if _TW_PREBUILD and _TWMAP.get(key):  # how to find this entry's source next step
        from .model import pack_provenance
        prov = pack_provenance(src)
        _TW_PLAN[key] = ("pack", weakref.ref(prov[0]), prov[1], prov[2]) if prov else (
            "tensor", weakref.ref(src))
    return w


def _tw_install(key, src, w, tok):
    k = (src.data_ptr(), src._version)
    _TW.pop(key, None)
    for dead in [kk for kk, e in _TW.items() if e[2]() is None]:
        del _TW[dead]
    while len(_TW) >= _TW_MAX:
        del _TW[next(iter(_TW))]
    _TW[key] = (k, w, weakref.ref(src), tok)
    ops.capture_keep(w, tok)


# Every step re-derives the mapped entries whose sources changed (the packed forward weights an
# Adam step rewrote, the re-drawn ABF weights), one index_gather each at its first use.
# tw_prebuild, at the start of the backward, finds each such entry's current source from the
# previous step's plan (a packed output of the model: model.pack_provenance; else the same
# tensor object) and gathers them all in one batched launch (CLSKD_TW_PREBUILD=0: A/B).
_TW_PREBUILD = os.environ.get("CLSKD_TW_PREBUILD", "1") == "1"
_TW_PLAN = {}


def tw_prebuild():
    if not _TW_PREBUILD or not _TW_PLAN:
        return
    from .model import pack_output
    tok = ops.capture_token()
    jobs, pend = [], []
    for key, plan in list(_TW_PLAN.items()):
        m = _TWMAP.get(key)
        src = None
        if plan[0] == "pack":
            model = plan[1]()
            src = pack_output(model, plan[2], plan[3], tok) if model is not None else None
        else:
            src = plan[1]()
        if not m or src is None:
            _TW_PLAN.pop(key, None)
            continue
        if m[0] != (tuple(src.shape), src.dtype, str(src.device)):
            continue
        ent = _TW.get(key)
        if (ent is not None and ent[0] == (src.data_ptr(), src._version) and ent[2]() is src
                and ops.cache_entry_usable(ent[3], tok)):
            continue
        out = torch.empty(m[3], dtype=f32, device=src.device)
        jobs.append((src, m[1], m[2], out))
        pend.append((key, src, out))
    if len(jobs) < 2:
        return
    ops.index_gather_jobs(jobs)
    for key, src, out in pend:
        _tw_install(key, src, out, tok)


# A rebuilt entry (every step: Adam rewrote the packed forward weights, the ABFs were re-drawn) is
# a signed selection of its source's elements (cat / negate / permute / zero-pad / pack), so after
# its first build it runs as ONE index_gather launch from a map probed once, instead of the
# torch cat / permute / contiguous / pack chain (2-6 launches and their host time per entry).
# The probe evaluates `build` with the source holding +(flat index + 1) and keeps the map only if
# gathering the real source reproduces the real build bitwise; entries that read other tensors
# too, or change dtype, keep `build`.  CLSKD_TW_MAPS=0 disables the maps (A/B).
_TW_MAPS_ON = os.environ.get("CLSKD_TW_MAPS", "1") == "1"
_BATCH_SCATTERS = os.environ.get("CLSKD_BATCH_SCATTERS", "1") == "1"  # A/B: 0 = one launch each
# mixed-precision ReviewKD backward: the mid-channel gradient maps (conv2 data gradient, ABF
# fusion dx / dyup) stored bf16 — the ABF fusion backward's dominant bytes halved (C3 -0.28 ms;
# worst C3 parameter gradient vs the oracle 3.04e-3 against 3.23e-3 with fp32 maps,
# profiles/r6_rkd_grad_bf16.txt).  CLSKD_RKD_GRAD_BF16=0: fp32 storage (A/B)
_RKD_GRAD_BF16 = os.environ.get("CLSKD_RKD_GRAD_BF16", "1") == "1"
# the ABF conv1 BatchNorm backward fused into conv1's data gradient (clskd_bn_bwd_conv1x1;
# CLSKD_BN1_CONV1_FUSED=0: apply pass + the fp32 engine, A/B)
_BN1_CONV1_FUSED = os.environ.get("CLSKD_BN1_CONV1_FUSED", "1") == "1"
# split-product data gradients on the bf16 LDS-DMA engine (round 6): the raw-output gradient as
# bf16 hi / lo planes, the transposed weight tripled [W_hi | W_hi | W_lo] per tap (CLSKD_DGRAD_PLANES)
_DGRAD_PLANES = os.environ.get("CLSKD_DGRAD_PLANES", "1") == "1"
_PLANES_MIN_N = int(os.environ.get("CLSKD_PLANES_MIN_N", "33"))  # narrowest output on planes
_TWMAP = {}


def _planes_of(draw, geom):
    """draw [..][C] fp32 (channel-contiguous rows) -> (bf16 planes [..][2C], the two segments of
    the split K table: planes (hi | lo) and planes' hi half), or None when not eligible."""
    C = geom.C
    if not (_DGRAD_PLANES and C % 32 == 0 and draw.dtype == f32 and draw.is_contiguous()
            and geom.sT == C and draw.data_ptr() % 16 == 0):
        return None
    planes = torch.empty(draw.shape[:-1] + (2 * C,), dtype=torch.bfloat16, device=draw.device)
    ops.split_planes(draw, planes)
    g2 = SegGeom(2 * C, geom.sB * 2, geom.sF * 2, geom.sT * 2, geom.F, geom.T)
    g1 = SegGeom(C, geom.sB * 2, geom.sF * 2, geom.sT * 2, geom.F, geom.T)
    return planes, [Seg(planes, 0, g2), Seg(planes, 0, g1)]


def _split3_weight(wt, ntaps, C):
    """Packed fp32 data-gradient weight [N][ntaps*C (+pad)] -> bf16 [N][Kp] of the planes' K
    table (per tap [W_hi | W_hi | W_lo], Kp = ntaps*3C padded to 64)."""
    N = wt.shape[0]
    Kp = -(-ntaps * 3 * C // 64) * 64
    out = torch.empty(N, Kp, dtype=torch.bfloat16, device=wt.device)
    ops.pack_split3(wt, ntaps, C, out)
    return out


def _tw_build(key, src, build):
    m = _TWMAP.get(key)
    if not _TW_MAPS_ON or not isinstance(src, torch.Tensor):
        return build()
    sig = (tuple(src.shape), src.dtype, str(src.device))
    if m and m[0] == sig:
        _, idx, sgn, shape = m
        out = torch.empty(shape, dtype=f32, device=src.device)
        ops.index_gather(src, idx, sgn, out)
        return out
    w = build()
    if (m is None and src.is_cuda and src.dtype == f32 and w.dtype == f32
            and src.is_contiguous() and w.is_contiguous() and src.numel() < (1 << 24)
            and not torch.cuda.is_current_stream_capturing()):
        _TWMAP[key] = _tw_probe(src, build, w, sig)
    return w


def _tw_probe(src, build, w, sig):
    """Map of `build` over `src` (see above), or False.  Synchronises the device around the probe
    (first build of an entry only): the source is overwritten with indices meanwhile."""
    torch.cuda.synchronize(src.device)
    saved = src.clone()
    try:
        src.copy_(torch.arange(1, src.numel() + 1, dtype=f32, device=src.device).view_as(src))
        wp = build()
    finally:
        src.copy_(saved)
    torch.cuda.synchronize(src.device)
    if wp.shape != w.shape or wp.dtype != f32:
        return False
    v = wp.reshape(-1)
    # a build that reads tensors other than `src` (or is not a ±1 selection) yields values that
    # are not source indices: reject the map before any gather could read out of bounds
    if not ops.probe_values_are_indices(v, src.numel()):
        return False
    idx = torch.where(v != 0, v.abs() - 1, torch.full_like(v, -1)).to(torch.int32).reshape(-1, 1)
    sgn = torch.sign(v).reshape(-1, 1).contiguous()
    out = torch.empty(w.shape, dtype=f32, device=w.device)
    ops.index_gather(src, idx, sgn, out)
    if not torch.equal(out, w):
        return False
    return (sig, idx.contiguous(), sgn, tuple(w.shape))


# ------------------------------------------------------------------------------------------
# the student DCCRN
# ------------------------------------------------------------------------------------------
def _enc_pack_fn(wr, wi):
    """ComplexConv2d packing of DCCRN._enc_w: [Co, 10*Ci] (tap = kf*2 + kt, then channel)."""
    top = torch.cat([wr, -wi], 1)
    bot = torch.cat([wi, wr], 1)
    w = torch.cat([top, bot], 0)
    Co, Ci = w.shape[:2]
    return w.permute(0, 2, 3, 1).reshape(Co, 10 * Ci)


def _cbias_fn(br, bi):
    return torch.cat([br - bi, bi + br]).reshape(-1, 1)


def _dec_pack_fn(taps_kf):
    def fn(wr, wi):
        top = torch.cat([wr, wi], 1)
        bot = torch.cat([-wi, wr], 1)
        w = torch.cat([top, bot], 0)
        Ci = w.shape[0]
        h = Ci // 4
        perm = torch.cat([torch.arange(0, h), torch.arange(2 * h, 3 * h),
                          torch.arange(h, 2 * h), torch.arange(3 * h, 4 * h)])
        w = w[perm]
        taps = [(kf, kt) for kf in taps_kf for kt in (0, 1)]
        w = torch.stack([w[:, :, kf, kt] for kf, kt in taps], 0).permute(2, 0, 1)
        return w.reshape(w.shape[0], -1)
    return fn


def dccrn_backward(m, tape, enc, dec, dec_in, lstm_io, g, pg, acc_params=False, join=None):
    """Reverse of DCCRN.run for a student `m` (fp32 activations).
    tape: the forward tape; enc/dec/dec_in/lstm_io: the forward's activations.
    g: upstream gradient buffers (fp32): g['wav'] [B][L] or None; g['enc'][i] like enc[i];
       g['dec'][k] (k < 5) like dec[k]; g['dec_in'] like dec_in.  Consumed (accumulated into).
    pg: dict parameter -> fp32 gradient tensor (contiguous, same shape) receiving the gradients.
    join(): called before the first accumulation into g['enc'] / g['dec'] / g['dec_in'] (after
    the waveform tail and the last decoder layer's weight gradient), so a caller can produce
    those buffers' first contributions on other streams meanwhile."""
    from .model import DCCRN
    B, T = tape["B"], tape["T"]
    dev = tape["spec"].device
    kn = m.kernel_num
    nl = len(kn) - 1

    # ---------------- ConviSTFT + clamp + mask 'E' (DCCRN.py:207-237)
    dmask = None
    if g.get("wav") is not None:
        frames, window, out_len = tape["frames"], tape["window"], tape["out_len"]
        dframes = _empty((B, T, 400), dev)
        ops.ola_bwd(frames, window, g["wav"], 100, out_len, 300, True, dframes)
        winv, _ = m._istft_w()  # [400][516]
        wt = _tw(("istft_t", id(m)), winv,
                 lambda: ops.pack_weight(winv[:, :516].t().contiguous().unsqueeze(1), 400))
        dest = _empty((B, T, 516), dev)
        # (N = 516 on the exact engine: split products with the planes' data gradients)
        with ops.split_products(_DGRAD_PLANES and getattr(m, "compute", "fp32") == "f32x3",
                                wgrad=getattr(ops._SPLIT, "wgrad", False)):
            ops.conv([Seg(dframes, 0, SegGeom(400, T * 400, 0, 400, 1, T))], [(0, 0)], B, 1, T, 516,
                     wt, None, dest, OutMap(T * 516, 0, 516), mfma_only=True)
        dmask = _empty(dec[-1].shape, dev)
        ops.mask_e_bwd(tape["spec"], dec[-1], T, dest, dmask)

    # ---------------- decoder (DCCRN.py:201-206), reverse
    F_in = [dec_in.shape[1] * (2 ** d) for d in range(nl)]  # input freq of decoder layer d
    for d in range(nl - 1, -1, -1):
        mod = m.decoder[d]
        cc = mod[0]
        F = F_in[d]
        out_t = dec_in if d == 0 else dec[d - 1]
        out_t0 = 0 if d == 0 else 1
        skip = enc[-1 - d]
        Cof, Csk = out_t.shape[-1], skip.shape[-1]
        Co = cc.out_channels * 2
        Ci = Cof + Csk
        # gradient w.r.t. the raw (pre-BN) transposed-conv output
        if d == nl - 1:
            if dmask is None:
                if join is not None:
                    join()
                    join = None
                continue  # no waveform gradient: the last layer is dead for the loss
            draw = dmask
        else:
            raw, coef, mv = tape["dec_bn"][d]
            bn, pr = mod[1], mod[2]
            draw = _empty(raw.shape, dev)
            ops.bn_bwd(raw, g["dec"][d], coef[:Co], coef[Co:], mv[0], mv[1], bn.eps, bn.weight,
                       pr.weight, draw, pg.get(bn.weight), pg.get(bn.bias), pg.get(pr.weight),
                       accumulate_params=acc_params)
        segs = [seg_bftc(out_t, 0, Cof, out_t0, T), seg_bftc(skip, 0, Csk)]
        # weight gradients: both polyphase parities into one concatenated packed buffer
        packs = [m._dec_w(d, p, "fp32") for p in (0, 1)]
        Kps = [packs[p][0].shape[1] for p in (0, 1)]
        dwcat = _empty((Co * (Kps[0] + Kps[1]),), dev)
        dbias = _empty((Co,), dev)
        for p in (0, 1):
            taps = [(dF, -kt) for _, dF in DCCRN._DEC_TAPS[p] for kt in (0, 1)]
            dw = dwcat[Co * Kps[0] * p:Co * (Kps[0] + Kps[1] * p)].view(Co, Kps[p])
            ops.conv_wgrad(segs, taps, B, F, T + 1, Co, draw,
                           OutMap(2 * F * (T + 1) * Co, (T + 1) * Co, Co, of_mul=2, of_add=p), dw,
                           dbias, accumulate=False, accumulate_bias=p == 1)
        _dec_scatter(m, d, dwcat, Kps, dbias, pg, acc_params)
        if join is not None:
            join()
            join = None
        # data gradients: one stride-2 gather over the raw-output gradient, per destination
        dgeom = SegGeom(Co, 2 * F * (T + 1) * Co, (T + 1) * Co, Co, 2 * F, T + 1)
        dseg = Seg(draw, 0, dgeom)
        taps_b = [(p - 2 * dF, kt) for p in (0, 1) for _, dF in DCCRN._DEC_TAPS[p] for kt in (0, 1)]
        # planes where a destination is wider than 32 channels (the bf16 engine's 32-wide tile
        # loses to the exact engine: profiles/r6_planes_micro.txt)
        pl = _planes_of(draw, dgeom) if max(Cof, Csk) >= _PLANES_MIN_N else None
        for s0, Cs, dst, t0, Tt in ((0, Cof, g["dec_in"] if d == 0 else g["dec"][d - 1], out_t0,
                                     out_t.shape[2]),
                                    (Cof, Csk, g["enc"][nl - 1 - d], 0, T)):
            wt = _tw(("dec_t", id(m), d, s0), packs[0][0], lambda: _dec_dgrad_w(packs, Ci, s0, Cs))
            if pl is not None and Cs >= _PLANES_MIN_N:  # split products on the bf16 engine
                ops.conv(pl[1], taps_b, B, F, T, Cs, _split3_weight(wt, len(taps_b), Co), None, dst,
                         OutMap(F * Tt * Cs, Tt * Cs, Cs), out_offset=t0 * Cs, stride_f=2,
                         accumulate=True)
                continue
            ops.conv([dseg], taps_b, B, F, T, Cs, wt, None, dst, OutMap(F * Tt * Cs, Tt * Cs, Cs),
                     out_offset=t0 * Cs, stride_f=2, accumulate=True)

    # ---------------- LSTM projection + complex LSTMs (DCCRN.py:178-199), reverse
    C6 = kn[-1]
    Ch = C6 // 2
    D4 = dec_in.shape[1]
    H = m.rnn_units // 2
    last = m.enhance[m.hidden_layers - 1]
    P = last.projection_dim
    packs_last = m._lstm_w(m.hidden_layers - 1, "fp32")
    ro, io = lstm_io[-1]
    d_out = [_empty((B, T, H), dev), _empty((B, T, H), dev)]
    for half in range(2):
        wpp, bp = packs_last[3 + 2 * half], packs_last[4 + 2 * half]
        lin = last.r_trans if half == 0 else last.i_trans
        omap = OutMap(D4 * T * C6, 0, C6, 1, T * C6, D4)
        src = (ro, io)[half]
        segs = [Seg(src, 0, SegGeom(H, T * H, 0, H, 1, T))]
        dw = _empty(wpp.shape, dev)
        db = _empty((P,), dev)
        ops.conv_wgrad(segs, [(0, 0)], B, 1, T, P, g["dec_in"], omap, dw, db, dy_offset=half * Ch)
        maps = unpack_maps(("lin", P, H), lambda w: w, [(P, H)], wpp.shape[1], dev)
        _scatter(dw, maps, [pg.get(lin.weight)], acc_params)
        _scatter(db, [_ident_map(P, dev)], [pg.get(lin.bias)], acc_params)
        wt = _tw(("proj_t", id(m), half), wpp,
                 lambda: ops.pack_weight(wpp[:, :H].reshape(Ch, D4, H).permute(2, 1, 0).contiguous(),
                                         D4 * Ch))
        dseg = Seg(g["dec_in"], half * Ch, SegGeom(Ch, D4 * T * C6, T * C6, C6, D4, T))
        ops.conv([dseg], [(f, 0) for f in range(D4)], B, 1, T, H, wt, None, d_out[half],
                 OutMap(T * H, 0, H), mfma_only=True)
    for li in range(m.hidden_layers - 1, -1, -1):
        lt = tape["lstm"][li]
        gx, hs = lt["gx"], lt["hs"]
        mod = m.enhance[li]
        R, I = mod.real_lstm, mod.imag_lstm
        wp, bias, whh = m._lstm_w(li, "fp32")[:3]
        dh = _empty((2, 2 * B, T, H), dev)
        ops.complex_combine_bwd(d_out[0], d_out[1], dh)
        # gate pre-activations: gx + h_{t-1} W_hh^T over the saved history (in place in gx) —
        # unless the taped forward's recurrence left them there (clskd_lstm_recurrent_pre)
        whp = _tw(("whh_p", id(m), li), whh,
                  lambda: torch.stack([ops.pack_weight(whh[ws].unsqueeze(1), H) for ws in (0, 1)]))
        if not lt.get("pre", False):
            for ws in range(2):
                hseg = Seg(hs, ws * 2 * B * T * H, SegGeom(H, T * H, 0, H, 1, T))
                ops.conv([hseg], [(0, -1)], 2 * B, 1, T, 4 * H, whp[ws], None, gx,
                         OutMap(T * 8 * H, 0, 8 * H), out_offset=ws * 4 * H, accumulate=True)
        dg = _empty((2, B, T, 8 * H), dev)
        st = (4 * H, T * 8 * H, 8 * H)
        ops.lstm_bwd(gx, st, dh, (2 * B * T * H, T * H, H), whh, 2, 2 * B, T, H, dg, st,
                     cells=lt.get("cells"))
        # W_hh gradient per weight set: rows (seq, t) x history h_{t-1}
        Kh = whp.shape[2]
        dwhh = _empty((2, 4 * H, Kh), dev)
        for ws in range(2):
            hseg = Seg(hs, ws * 2 * B * T * H, SegGeom(H, T * H, 0, H, 1, T))
            ops.conv_wgrad([hseg], [(0, -1)], 2 * B, 1, T, 4 * H, dg, OutMap(T * 8 * H, 0, 8 * H),
                           dwhh[ws], dy_offset=ws * 4 * H)
        _scatter(dwhh, unpack_maps(("whh", H, Kh), lambda a, b: torch.cat([
            torch.cat([a, a.new_zeros(4 * H, Kh - H)], 1), torch.cat([b, b.new_zeros(4 * H, Kh - H)], 1)], 0),
            [(4 * H, H), (4 * H, H)], Kh, dev), [pg.get(R.weight_hh_l0), pg.get(I.weight_hh_l0)],
            acc_params)
        # W_ih / bias gradients (the two input halves accumulate) and the input gradient
        dwih = _empty(wp.shape, dev)
        dbias = _empty((8 * H,), dev)
        nxt = [_empty((B, T, H), dev), _empty((B, T, H), dev)] if li > 0 else None
        for half in range(2):
            if li == 0:
                segs = [seg_bftc(enc[-1], c0=half * Ch, C=Ch)]
                taps = [(f, 0) for f in range(D4)]
            else:
                segs = [Seg(lt["r_in"][half], 0, SegGeom(H, T * H, 0, H, 1, T))]
                taps = [(0, 0)]
            ops.conv_wgrad(segs, taps, B, 1, T, 8 * H, dg[half], OutMap(T * 8 * H, 0, 8 * H), dwih,
                           dbias, accumulate=half == 1)
            gseg = [Seg(dg[half], 0, SegGeom(8 * H, T * 8 * H, 0, 8 * H, 1, T))]
            if li == 0:
                wt = _tw(("ih_t", id(m), li), wp, lambda: ops.pack_weight(
                    wp[:, :D4 * Ch].t().contiguous().unsqueeze(1), 8 * H))
                ops.conv(gseg, [(0, 0)], B, 1, T, D4 * Ch, wt, None, g["enc"][-1],
                         OutMap(D4 * T * C6, 0, C6, T * C6, 1, Ch), out_offset=half * Ch,
                         accumulate=True)
            else:
                wt = _tw(("ih_t", id(m), li), wp, lambda: ops.pack_weight(
                    wp[:, :H].t().contiguous().unsqueeze(1), 8 * H))
                ops.conv(gseg, [(0, 0)], B, 1, T, H, wt, None, nxt[half], OutMap(T * H, 0, H),
                         mfma_only=True)
        D = R.weight_ih_l0.shape[1]
        if li == 0:
            fn = lambda a, b: torch.cat([a, b], 0).reshape(8 * H, D // 4, 4).permute(0, 2, 1).reshape(8 * H, D)
        else:
            fn = lambda a, b: torch.cat([a, b], 0)
        _scatter(dwih, unpack_maps(("wih", li, H, D), fn, [(4 * H, D), (4 * H, D)], wp.shape[1], dev),
                 [pg.get(R.weight_ih_l0), pg.get(I.weight_ih_l0)], acc_params)
        bmaps = unpack_maps(("lstm_b", H), lambda a, b, c, e: torch.cat([a + b, c + e]).reshape(-1, 1),
                            [(4 * H,)] * 4, 1, dev)
        _scatter(dbias, bmaps, [pg.get(R.bias_ih_l0), pg.get(R.bias_hh_l0), pg.get(I.bias_ih_l0),
                                pg.get(I.bias_hh_l0)], acc_params)
        d_out = nxt

    # ---------------- encoder (DCCRN.py:171-176), reverse
    for i in range(nl - 1, -1, -1):
        mod = m.encoder[i]
        bn, pr = mod[1], mod[2]
        raw, coef, mv = tape["enc_bn"][i]
        Co = raw.shape[-1]
        Fo = raw.shape[1]
        draw = _empty(raw.shape, dev)
        ops.bn_bwd(raw, g["enc"][i], coef[:Co], coef[Co:], mv[0], mv[1], bn.eps, bn.weight,
                   pr.weight, draw, pg.get(bn.weight), pg.get(bn.bias), pg.get(pr.weight),
                   accumulate_params=acc_params)
        src = tape["spec_b"] if i == 0 else enc[i - 1]
        Ci = src.shape[-1]
        wp, _ = m._enc_w(i, "fp32")
        taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
        dw = _empty(wp.shape, dev)
        db = _empty((Co,), dev)
        ops.conv_wgrad([seg_bftc(src)], taps, B, Fo, T, Co, draw, OutMap(Fo * T * Co, T * Co, Co),
                       dw, db, stride_f=2)
        cc = mod[0]
        maps = unpack_maps(("enc", Co, Ci), _enc_pack_fn,
                           [tuple(cc.real_conv.weight.shape), tuple(cc.imag_conv.weight.shape)],
                           wp.shape[1], dev)
        _scatter(dw, maps, [pg.get(cc.real_conv.weight), pg.get(cc.imag_conv.weight)], acc_params)
        bmaps = unpack_maps(("cbias", Co), _cbias_fn, [(Co // 2,), (Co // 2,)], 1, dev)
        _scatter(db, bmaps, [pg.get(cc.real_conv.bias), pg.get(cc.imag_conv.bias)], acc_params)
        if i == 0:
            continue
        dgeom = SegGeom(Co, Fo * T * Co, T * Co, Co, Fo, T)
        dseg = Seg(draw, 0, dgeom)
        pl = _planes_of(draw, dgeom) if Ci >= _PLANES_MIN_N else None
        for p in (0, 1):
            kfs = [kf for kf in range(5) if kf % 2 == p]
            taps_b = [((p - kf + 2) // 2, 1 - kt) for kf in kfs for kt in range(2)]
            # kfs = p, p+2, ...: a strided slice — a Python-list index would build an index
            # tensor and copy it host-to-device synchronously every step (host stalls on the GPU)
            wt = _tw(("enc_t", id(m), i, p), wp, lambda: ops.pack_weight(
                wp[:, :10 * Ci].reshape(Co, 5, 2, Ci)[:, p::2].permute(3, 1, 2, 0)
                .reshape(Ci, len(kfs) * 2, Co).contiguous(), len(kfs) * 2 * Co))
            if pl is not None:  # split products on the bf16 engine
                ops.conv(pl[1], taps_b, B, Fo, T, Ci, _split3_weight(wt, len(taps_b), Co), None,
                         g["enc"][i - 1], OutMap(2 * Fo * T * Ci, T * Ci, Ci, of_mul=2, of_add=p),
                         accumulate=True)
                continue
            ops.conv([dseg], taps_b, B, Fo, T, Ci, wt, None, g["enc"][i - 1],
                     OutMap(2 * Fo * T * Ci, T * Ci, Ci, of_mul=2, of_add=p), accumulate=True)


_IDENT = {}


def _ident_map(n, dev):
    k = (n, str(dev))
    if k not in _IDENT:
        _IDENT[k] = (torch.arange(n, dtype=torch.int32, device=dev).reshape(n, 1),
                     torch.ones(n, 1, dtype=f32, device=dev))
    return _IDENT[k]


def _dec_dgrad_w(packs, Ci, s0, Cs):
    """Data-gradient weight of one decoder input segment: [Cs][(tap over both parities, n)]."""
    from .model import DCCRN
    ws = []
    for p in (0, 1):
        wp = packs[p][0]
        nt = len(DCCRN._DEC_TAPS[p]) * 2
        ws.append(wp[:, :nt * Ci].reshape(wp.shape[0], nt, Ci)[:, :, s0:s0 + Cs])
    w = torch.cat(ws, 1)  # [Co, 10, Cs]
    Co = w.shape[0]
    return ops.pack_weight(w.permute(2, 1, 0).contiguous(), 10 * Co)


def _dec_scatter(m, d, dwcat, Kps, dbias, pg, acc):
    from .model import DCCRN
    cc = m.decoder[d][0]
    Co = cc.out_channels * 2
    shapes = [tuple(cc.real_conv.weight.shape), tuple(cc.imag_conv.weight.shape)]
    K0 = Kps[0]

    def fn(wr, wi):  # [Co, K0 | K1] with each parity padded to its Kp
        a = _dec_pack_fn([kf for kf, _ in DCCRN._DEC_TAPS[0]])(wr, wi)
        b = _dec_pack_fn([kf for kf, _ in DCCRN._DEC_TAPS[1]])(wr, wi)
        a = torch.cat([a, a.new_zeros(a.shape[0], K0 - a.shape[1])], 1)
        b = torch.cat([b, b.new_zeros(b.shape[0], Kps[1] - b.shape[1])], 1)
        # the gradient buffer holds parity 0 as [Co][K0] then parity 1 as [Co][K1]
        return torch.cat([a.reshape(-1), b.reshape(-1)]).reshape(1, -1)

    maps = unpack_maps(("dec", d, Co, tuple(Kps)), fn, shapes, Co * (K0 + Kps[1]), dwcat.device)
    _scatter(dwcat, maps, [pg.get(cc.real_conv.weight), pg.get(cc.imag_conv.weight)], acc)
    bmaps = unpack_maps(("cbias", Co), _cbias_fn, [(Co // 2,), (Co // 2,)], 1, dwcat.device)
    _scatter(dbias, bmaps, [pg.get(cc.real_conv.bias), pg.get(cc.imag_conv.bias)], acc)


# ------------------------------------------------------------------------------------------
# ReviewKD (framework.py:176-263), reverse — ABF weights are not trained (new modules per step)
# ------------------------------------------------------------------------------------------
def review_backward(review, tape, coef_m, d_feats, acc_feats):
    """tape: ReviewKD.forward_bftc's per-level tapes (processing order); coef_m[j]: the SPKD
    gradient coefficients M = dG + dG^T [B][B] of level j's output Gram; d_feats[j]: student-
    feature gradient buffer of level j, accumulated into when acc_feats[j].

    The SPKD gradient dz = M z of each output is fused into its conv2 BatchNorm backward
    (clskd_spkd_bn_bwd: dz never reaches HBM).  When the fusions ran in bf16 (precision='mixed')
    the raw-output gradient is stored bf16 and the conv2 data gradient — the heaviest GEMM of
    the backward — runs on the bf16 MFMA engine like its forward; fp32 otherwise."""
    n = len(tape)
    dyup_next = None  # level j+1's gradient w.r.t. its upsampled residual (= level j's fused map)
    for j in range(n - 1, -1, -1):
        tp = tape[j]
        abf = review.abfs[j]
        if "wver" in tp and tp["wver"] != abf.param_versions():
            # same contract as autograd's saved-tensor version check: the ABF weights this
            # tape's forward used were rewritten (a later step's re-draw) before its backward
            raise RuntimeError(
                "ReviewKD ABF weights were modified in place (abf_reinit='step' re-draw) after the "
                "forward that recorded this tape; run its backward before the next step's forward")
        dev = tp["x1"].device
        out_raw = tp["out_raw"]
        Bn, Fn, Tn, Cout = out_raw.shape
        mid = tp["x1"].shape[-1]
        bn2 = abf.conv2[1]
        lowp = out_raw.dtype == torch.bfloat16
        d_oraw = torch.empty(out_raw.shape, device=dev, dtype=out_raw.dtype if lowp else f32)
        ops.spkd_bn_bwd(out_raw, tp["coef2"], coef_m[j], tp["mv2"][0], tp["mv2"][1], bn2.eps,
                        bn2.weight, d_oraw)
        # levels with an attention fusion hand d_xf only to abf_fuse_bwd (any storage type);
        # the level without one accumulates the residual gradient into it (fp32)
        gdt = torch.bfloat16 if (lowp and _RKD_GRAD_BF16 and abf.att_conv is not None) else f32
        d_xf = torch.empty((Bn, Fn, Tn, mid), device=dev, dtype=gdt)
        w2 = abf.conv2[0].weight
        w2t = _tw(("abf2_t", id(abf), lowp), w2, lambda: ops.pack_weight(
            w2.permute(1, 2, 3, 0).reshape(mid, 9, Cout).contiguous().float(), 9 * Cout,
            "bf16" if lowp else "fp32"))
        ops.conv([seg_bftc(d_oraw)], [(1 - kf, 1 - kt) for kf in range(3) for kt in range(3)], Bn, Fn,
                 Tn, mid, w2t, None, d_xf, OutMap(Fn * Tn * mid, Tn * mid, mid))
        c1 = tp["coef1"]
        bn1 = abf.conv1[1]
        if abf.att_conv is not None:
            # one pass: residual path of level j+1 folded in on load, the attention-fusion
            # backward, and the conv1-BN statistics partials (no down-sum / BN-reduce passes)
            dxn = torch.empty(d_xf.shape, device=dev, dtype=gdt)
            dyup = torch.empty(d_xf.shape, device=dev, dtype=gdt)
            aw = abf.att_conv[0].weight.reshape(2, -1).float().contiguous()
            ab = abf.att_conv[0].bias.float().contiguous()
            part, nblk = ops.abf_fuse_bwd(tp["x1"], tp["res"], aw, ab, c1, d_xf, dxn, dyup,
                                          dnext=dyup_next, mv1=tp["mv1"], eps=bn1.eps)
            dyup_next = dyup
        else:
            if dyup_next is not None:  # residual path of level j+1 (nearest upsampling)
                ops.nearest_down_sum(dyup_next, d_xf, accumulate=True)
            dxn = d_xf
            dyup_next = None
            part, nblk = None, 0
        w1 = abf.conv1[0].weight  # [mid, Cin, 1, 1]
        Cin = w1.shape[1]
        w1m = w1.reshape(mid, Cin).float().contiguous()
        if _BN1_CONV1_FUSED and ops.bn_bwd_conv1x1_ok(tp["x1"], dxn, w1m, d_feats[j]):
            # conv1 BatchNorm backward applied inside conv1's data gradient: d_x1 (64 channels
            # at the tap's resolution, fp32) never reaches HBM
            k = ops.bn_bwd_coeffs(tp["x1"], dxn, c1[:mid], c1[mid:], tp["mv1"][0], tp["mv1"][1],
                                  bn1.eps, bn1.weight, part, nblk)
            ops.bn_bwd_conv1x1(tp["x1"], dxn, k, w1m, d_feats[j], accumulate=bool(acc_feats[j]))
            continue
        d_x1 = _empty(tp["x1"].shape, dev)
        if part is not None:
            ops.bn_bwd_from_partials(tp["x1"], dxn, c1[:mid], c1[mid:], tp["mv1"][0],
                                     tp["mv1"][1], bn1.eps, bn1.weight, part, nblk, d_x1)
        else:
            ops.bn_bwd(tp["x1"], dxn, c1[:mid], c1[mid:], tp["mv1"][0], tp["mv1"][1], bn1.eps,
                       bn1.weight, None, d_x1)
        w1t = _tw(("abf1_t", id(abf)), w1, lambda: ops.pack_weight(
            w1.reshape(mid, Cin).t().contiguous().unsqueeze(1).float(), mid))
        ops.conv([seg_bftc(d_x1)], [(0, 0)], Bn, Fn, Tn, Cin, w1t, None, d_feats[j],
                 OutMap(Fn * Tn * Cin, Tn * Cin, Cin), accumulate=bool(acc_feats[j]), mfma_only=True)


# ------------------------------------------------------------------------------------------
# MRSTFT log-magnitude base loss (framework.py:58-146), reverse
# ------------------------------------------------------------------------------------------
def mrstft_backward(tape, d_x, upstream=1.0):
    """tape: per-resolution dicts from MultiResolutionSTFTLoss(..., tape=...); d_x [B][L]
    (accumulated into): gradient of upstream * mag-loss w.r.t. the estimate x."""
    for t in tape:
        X, Y, plan = t["X"], t["Y"], t["plan"]
        B, Tm, W2 = X.shape
        nb = plan.fft // 2 + 1
        # the spectrum gradient gets a row pitch padded to a multiple of 4 (zero columns), so the
        # framing data gradient below gathers it with 16-B loads (vec4 K table)
        Wp = -(-W2 // 4) * 4
        dX = _empty((B, Tm, Wp), X.device)
        ops.stft_mag_loss_bwd(X, Y, nb, upstream * t["factor_mag"] / t["count"], dX)
        Lr, L = t["Lr"], t["L"]
        dxr = _zeros((B, Lr), X.device)
        basis = plan.basis(X.device)  # [2nb][KT*hop]
        KT, hop = plan.KT, plan.hop

        def build():
            w = basis[:, :KT * hop].reshape(W2, KT, hop)
            w = torch.cat([w, w.new_zeros(Wp - W2, KT, hop)], 0)  # zero rows for the pad columns
            return ops.pack_weight(w.permute(2, 1, 0).contiguous(), KT * Wp)
        wt = _tw(("stft_t", id(plan)), basis, build)
        ops.conv([Seg(dX, 0, SegGeom(Wp, Tm * Wp, 0, Wp, 1, Tm))], [(0, -kt) for kt in range(KT)], B, 1,
                 Tm + KT - 1, hop, wt, None, dxr, OutMap(Lr, 0, hop), out_offset=plan.off,
                 mfma_only=True)
        ops.frame_pad_bwd(dxr, L, plan.fft // 2, 1, d_x, accumulate=True)


# ------------------------------------------------------------------------------------------
# the CLSKD step (distill.py:72-148), reverse
# ------------------------------------------------------------------------------------------
def _gram_view_bftc(t, c0=0, Cs=None):
    affine = None
    if isinstance(t, ops.DeferredBN):
        t, affine = t.raw, t.coef
    B, Fn, Tn, Ct = t.shape
    Cs = Ct if Cs is None else Cs
    return ops.GramView(t, 0, Fn * Tn * Ct, Fn * Tn, Ct, c0, Cs, affine)


def clskd_backward(res, student, review_encoder, review_decoder, pg, acc_params=False,
                   upstream=1.0):
    """Gradients of upstream * res['loss'] (a clskd_step(..., tape=True) result) w.r.t. the
    student's parameters, written into pg (parameter -> fp32 tensor).  Teacher frozen, ABF
    modules untrained (distill.py:49-50, 92-96, 202-204): gradients flow through ReviewKD only
    to the student's taps.  Runs on the current stream."""
    tp = res["tape"]
    sf = res["s"]
    enc, dec, dec_in = sf["enc"], sf["dec"], sf["dec_in"]
    wav = sf["out_wav"]
    B = wav.shape[0]
    dev = wav.device
    g = dict(enc=[_empty(t.shape, dev) for t in enc], dec=[_empty(t.shape, dev) for t in dec[:5]],
             dec_in=_empty(dec_in.shape, dev), wav=_zeros(wav.shape, dev))
    # SPKD (framework.py:150-172): M = dG + dG^T per pair, then dz = M z per student tap
    g_enc, g_dec, g_t = res["gram_slabs"]
    s_refs = g_enc.refs + g_dec.refs
    M = ops.spkd_grad(s_refs, g_t.refs, B, True, upstream, device=dev)
    n_enc = len(res["s_enc_list"])
    _, D4, T, C6 = dec_in.shape
    Ch = C6 // 2
    # clstm real / imag taps = the two channel halves of dec_in (fp32, no BN): dz = M z directly
    ops.gram_bwd([(_gram_view_bftc(dec_in, h * Ch, Ch), M[2 * n_enc + h], g["dec_in"], D4 * T * C6,
                   C6, h * Ch, False) for h in range(2)], B)
    # Three independent branches on three streams, joined before the student's first accumulation
    # into the tap gradients: ReviewKD-decoder backward | ReviewKD-encoder backward (their
    # SPKD gradients fused into the output BN backward) | the waveform tail on the calling
    # stream (MRSTFT log-magnitude -> OLA -> iSTFT -> mask -> last decoder layer's wgrad).
    # ReviewKD decoder levels follow the feature order; encoder levels process the reversed
    # taps and insert results at the front (framework.py:245-261).
    from .distill import _side_stream
    main = torch.cuda.current_stream(dev)
    tw_prebuild()  # on main, before the branches fork: every consumer is ordered after it
    s_dec, s_enc = _side_stream(dev, 0), _side_stream(dev, 1)
    n = len(enc)
    for st in (s_dec, s_enc):
        st.wait_stream(main)
    with torch.cuda.stream(s_dec):
        review_backward(review_decoder, tp["rd"], [M[n_enc + j] for j in range(n_enc)],
                        [g["dec_in"]] + g["dec"], [True] + [False] * 5)
    with torch.cuda.stream(s_enc):
        review_backward(review_encoder, tp["re"], [M[n - 1 - j] for j in range(n)],
                        [g["enc"][n - 1 - j] for j in range(n)], [False] * n)
    # MRSTFT log-magnitude base loss (distill.py:100-101) -> d student waveform
    # the spectrum gradient's frame GEMM (N = hop, K = taps x 516: 23 TF/s on the exact engine,
    # at the head of the waveform tail every student gradient waits for) on split products when
    # the data gradients are (CLSKD_DGRAD_PLANES with a 'mixed' student)
    with ops.split_products(_DGRAD_PLANES and getattr(student, "compute", "fp32") == "f32x3",
                            wgrad=getattr(ops._SPLIT, "wgrad", False)):
        mrstft_backward(tp["ms"], g["wav"], upstream)

    def join():
        main.wait_stream(s_dec)
        main.wait_stream(s_enc)

    global _SCATTERS
    _SCATTERS = [] if (_BATCH_SCATTERS and not acc_params) else None
    try:
        dccrn_backward(student, tp["s"], enc, dec, dec_in, sf["lstm_io"], g, pg, acc_params, join=join)
        if _SCATTERS:
            ops.index_gather_jobs(_SCATTERS)  # on main: every scattered gradient was made there
    finally:
        _SCATTERS = None
    return g
