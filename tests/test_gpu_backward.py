"""GPU parity of the CLSKD training step's backward pass (config C3, SURVEY.md §8 f rank 1):
the HIP gradients (clskd.backward) against the CPU oracle's autograd (oracle/ref_cpu.py, the
fp32 PyTorch restatement of the reference pinned by tests/golden), plus the primitives
(wgrad / accumulate conv, LSTM BPTT, Adam) against torch.

Tolerance: relative L2 error ||g - g_ref|| / ||g_ref|| <= 2e-3 per parameter (fp32 on both
sides, different summation orders; BatchNorm backward over small batches amplifies rounding).
"""
import os

import numpy as np
import pytest
import torch

from clskd import config as cfg
from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, apply_recipe

pytestmark = pytest.mark.gpu

DEV = "cuda"
torch.set_num_threads(min(16, os.cpu_count() or 1))


def _rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _np(t):
    return t.detach().float().cpu().numpy()


def test_conv_wgrad_and_accumulate_against_torch():
    """wgrad through a forward descriptor (2 segments, 3x3, stride 2 in freq, N not a tile
    multiple) and an accumulating data-gradient launch, against torch autograd."""
    from clskd import ops
    g = torch.Generator().manual_seed(1)
    B, F, T, C1, C2, N = 2, 10, 23, 8, 4, 40
    a = torch.randn(B, F, T, C1, generator=g)
    b = torch.randn(B, F, T, C2, generator=g)
    w = (torch.randn(N, C1 + C2, 3, 3, generator=g) * 0.1).requires_grad_()
    bias = torch.randn(N, generator=g).requires_grad_()
    x = torch.cat([a, b], 3).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(x, w, bias, stride=(2, 1), padding=1)
    dy = torch.randn(ref.shape, generator=g)
    ref.backward(dy)
    Fo = ref.shape[2]
    taps = [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)]
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(DEV)
    segs = [ops.seg_bftc(a.to(DEV)), ops.seg_bftc(b.to(DEV))]
    Kp = -(-9 * (C1 + C2) // 16) * 16
    dw = torch.empty(N, Kp, device=DEV)
    db = torch.empty(N, device=DEV)
    ops.conv_wgrad(segs, taps, B, Fo, T, N, dyd, ops.OutMap(Fo * T * N, T * N, N), dw, db, stride_f=2)
    got = dw[:, :9 * (C1 + C2)].reshape(N, 3, 3, C1 + C2).permute(0, 3, 1, 2)
    assert _rel(_np(got), w.grad.numpy()) < 1e-5
    assert _rel(_np(db), bias.grad.numpy()) < 1e-5
    # accumulate: out = prior + conv
    out = torch.randn(B, Fo, T, N, generator=g).to(DEV)
    prior = out.clone()
    wp = ops.pack_weight(w.detach().permute(0, 2, 3, 1).reshape(N, 9, C1 + C2).to(DEV), 9 * (C1 + C2))
    ops.conv(segs, taps, B, Fo, T, N, wp, None, out, ops.OutMap(Fo * T * N, T * N, N),
             stride_f=2, accumulate=True)
    plain = torch.nn.functional.conv2d(x, w.detach(), None, stride=(2, 1), padding=1)
    np.testing.assert_allclose(_np(out - prior), plain.permute(0, 2, 3, 1).numpy(), rtol=1e-5,
                               atol=1e-5)


def _wgrad_ref(segs, taps, sf, Fo, dy):
    """fp64 dW[n, tap, c] and dbias[n] of the implicit-GEMM conv (zero padding)."""
    x = torch.cat([s.double() for s in segs], 3)
    B, Fi, T, Cin = x.shape
    dy = dy.double()
    dw = torch.zeros(dy.shape[-1], len(taps), Cin, dtype=torch.float64)
    for ti, (dF, dT) in enumerate(taps):
        fi = torch.arange(Fo) * sf + dF
        tt = torch.arange(T) + dT
        vf = (fi >= 0) & (fi < Fi)
        vt = (tt >= 0) & (tt < T)
        sub = torch.zeros(B, Fo, T, Cin, dtype=torch.float64)
        sub[:, vf.nonzero()[:, 0][:, None], vt.nonzero()[:, 0][None, :]] = \
            x[:, fi[vf][:, None], tt[vt][None, :]]
        dw[:, ti] = torch.einsum("bftn,bftc->nc", dy, sub)
    return dw, dy.sum((0, 1, 2))


X3_CASES = {
    # name: (segment channels, N, taps, stride_f, B, Fi, Fo, T)
    "n2_k96_2seg": ((16, 16), 2, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1, 3, 20, 20, 301),
    "n8_k20_cin2": ((2,), 8, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 2, 65, 33, 211),
    "n16_k80": ((8,), 16, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 2, 64, 32, 301),
    "n24_k384_2seg": ((32, 32), 24, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1, 2, 9, 9, 157),
    "n64_k320": ((32,), 64, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 2, 16, 8, 301),
    "n100_k48": ((12,), 100, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 1, 7, 7, 45),
}


@pytest.mark.parametrize("depth", [0, 1, 2])
@pytest.mark.parametrize("case", sorted(X3_CASES))
def test_conv_wgrad_split_products_against_fp64(case, depth):
    """The split-product weight gradient (csrc/wgrad_x3.hip: descriptors of compute CLSKD_F32X3,
    inside ops.split_products(..., wgrad=True)) against fp64 torch: every n-tile width (N 2 - 100,
    two n-tiles at 100), vec4 and scalar gathers (Cin 2), polyphase two-segment decoder taps,
    stride 2, several row splits (M up to 85 k) and partial chunks.  Bound: 3 x bf16 products
    drop terms <= ~3 * 2^-18 relative each; the sums over 1e4-1e5 rows of random-sign terms stay
    far inside rel L2 2e-5 (dbias sums the fp32 values: 2e-6).  Bitwise repeatable.  depth: row
    chunks in flight per wave (CLSKD_WGRAD_DEPTH; 0 = the per-instance default)."""
    from clskd import _lib, ops
    prev = _lib.set_knob("CLSKD_WGRAD_DEPTH", depth)
    try:
        _x3_case(case)
    finally:
        _lib.set_knob("CLSKD_WGRAD_DEPTH", prev)


@pytest.mark.parametrize("case", sorted(X3_CASES))
def test_conv_wgrad_xcd_order_is_bitwise_identical(case):
    """CLSKD_WGRAD_XCD (each XCD walks a contiguous run of (row chunk, n-tile, k-tile) work items)
    only reassigns work items to workgroups: dW and dbias bitwise equal to the grid order."""
    from clskd import _lib, ops
    segc, N, taps, sf, B, Fi, Fo, T = X3_CASES[case]
    g = torch.Generator().manual_seed(9)
    dsegs = [ops.seg_bftc((torch.randn(B, Fi, T, c, generator=g) * 1.3).to(DEV)) for c in segc]
    dyd = torch.randn(B, Fo, T, N, generator=g).to(DEV)
    Kp = -(-len(taps) * sum(segc) // 16) * 16
    outs = []
    for xcd in (0, 1):
        prev = _lib.set_knob("CLSKD_WGRAD_XCD", xcd)
        try:
            dw = torch.empty(N, Kp, device=DEV)
            db = torch.empty(N, device=DEV)
            with ops.split_products(False, wgrad=True):
                ops.conv_wgrad(dsegs, taps, B, Fo, T, N, dyd, ops.OutMap(Fo * T * N, T * N, N), dw,
                               db, stride_f=sf)
            torch.cuda.synchronize()
            outs.append((dw, db))
        finally:
            _lib.set_knob("CLSKD_WGRAD_XCD", prev)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def _x3_case(case):
    from clskd import ops
    segc, N, taps, sf, B, Fi, Fo, T = X3_CASES[case]
    g = torch.Generator().manual_seed(7)
    segs = [torch.randn(B, Fi, T, c, generator=g) * 1.3 + 0.1 for c in segc]
    dy = torch.randn(B, Fo, T, N, generator=g)
    ref_w, ref_b = _wgrad_ref(segs, taps, sf, Fo, dy)
    Cin = sum(segc)
    Kp = -(-len(taps) * Cin // 16) * 16
    dyd = dy.to(DEV)
    dsegs = [ops.seg_bftc(s.to(DEV)) for s in segs]
    outs = []
    for _ in range(2):
        dw = torch.full((N, Kp), float("nan"), device=DEV)
        db = torch.full((N,), float("nan"), device=DEV)
        with ops.split_products(False, wgrad=True):
            ops.conv_wgrad(dsegs, taps, B, Fo, T, N, dyd, ops.OutMap(Fo * T * N, T * N, N), dw, db,
                           stride_f=sf)
        outs.append((dw.clone(), db.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    dw, db = outs[0]
    got = dw[:, :len(taps) * Cin].reshape(N, len(taps), Cin)
    assert torch.isfinite(dw).all()
    ew, eb = _rel(_np(got), ref_w.numpy()), _rel(_np(db), ref_b.numpy())
    print(f"{case}: rel L2 dW {ew:.2e} dbias {eb:.2e}")
    assert ew < 2e-5, ew
    assert eb < 2e-6, eb
    # the exact engine on the same descriptor agrees to the split bound too
    dwe = torch.empty(N, Kp, device=DEV)
    ops.conv_wgrad(dsegs, taps, B, Fo, T, N, dyd, ops.OutMap(Fo * T * N, T * N, N), dwe, None,
                   stride_f=sf)
    assert _rel(_np(got), _np(dwe[:, :len(taps) * Cin].reshape(N, len(taps), Cin))) < 2e-5


@pytest.mark.parametrize("H,wave", [(16, 1), (32, 1), (32, 0), (128, 1)])
def test_lstm_bwd_against_torch(H, wave):
    """BPTT kernel: gate gradients for given dh, pre-activations rebuilt from the h history.
    H = 16 / 32 run the single-wave kernel (wave 1, default; T = 57 ends mid register ring) or
    the 4-wave one (CLSKD_LSTM_BWD_WAVE=0)."""
    from clskd import _lib, ops
    prev = _lib.set_knob("CLSKD_LSTM_BWD_WAVE", wave)
    try:
        _lstm_bwd_case(H)
    finally:
        _lib.set_knob("CLSKD_LSTM_BWD_WAVE", prev)


def _lstm_bwd_case(H):
    from clskd import ops
    g = torch.Generator().manual_seed(2)
    nseq, T = 3, 57
    lstm = torch.nn.LSTM(16, H)
    for p in lstm.parameters():
        torch.nn.init.uniform_(p, -0.3, 0.3, generator=g)
    x = torch.randn(T, nseq, 16, generator=g)
    out, _ = lstm(x)
    dh = torch.randn(out.shape, generator=g)
    whh_t = lstm.weight_hh_l0.detach()
    gx = (x @ lstm.weight_ih_l0.t() + lstm.bias_ih_l0 + lstm.bias_hh_l0).detach().requires_grad_()
    # full BPTT reference: d loss / d gx == d loss / d (gate pre-activations)
    h = torch.zeros(nseq, H)
    c = torch.zeros(nseq, H)
    hs, pres = [], []
    for t in range(T):
        pre_t = gx[t] + h @ whh_t.t()
        pres.append(pre_t.detach())
        gi, gf, gg, go = pre_t.chunk(4, 1)
        c = torch.sigmoid(gf) * c + torch.sigmoid(gi) * torch.tanh(gg)
        h = torch.sigmoid(go) * torch.tanh(c)
        hs.append(h)
    (torch.stack(hs) * dh).sum().backward()
    pre = torch.stack(pres)  # [T, nseq, 4H]
    # HIP: layouts [ws=1][seq][T][4H]
    pre_d = pre.permute(1, 0, 2).contiguous().to(DEV)
    dh_d = dh.permute(1, 0, 2).contiguous().to(DEV)
    whh = lstm.weight_hh_l0.detach().contiguous().to(DEV)
    dg = torch.empty_like(pre_d)
    st = (0, T * 4 * H, 4 * H)
    ops.lstm_bwd(pre_d, st, dh_d, (0, T * H, H), whh, 1, nseq, T, H, dg, st)
    ref = gx.grad.permute(1, 0, 2).numpy()
    assert _rel(_np(dg), ref) < 1e-4


def test_adam_kernel_matches_torch():
    from clskd import ops
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(1000, generator=g)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=6e-4, weight_decay=0.01)
    p = p0.clone().to(DEV)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step in range(1, 4):
        grad = torch.randn(1000, generator=g)
        ref.grad = grad.clone()
        opt.step()
        ops.adam_step(p, grad.to(DEV), m, v, 6e-4, 0.9, 0.999, 1e-8, 0.01, step)
    np.testing.assert_allclose(_np(p), ref.detach().numpy(), rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------------------------------------
# the whole CLSKD step against the oracle's autograd
# ------------------------------------------------------------------------------------------
def _kd(precision="fp32"):
    from clskd.distill import KnowledgeDistillation
    from clskd.model import DCCRN
    t = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    s = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    kd = KnowledgeDistillation(t.train(), s.train(), abf_reinit="once",
                               precision=precision).to(DEV)
    apply_recipe(kd.review_encoder, ABF_SEED, "encoder.")
    apply_recipe(kd.review_decoder, ABF_SEED, "decoder.")
    return kd


def _oracle_grads(noisy, clean):
    from oracle import ref_cpu as R
    from clskd.weights import recipe_state_dict
    pt = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.TEACHER), TEACHER_SEED))
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    shapes = {**cfg.review_param_shapes("encoder"), **cfg.review_param_shapes("decoder")}
    pa = R.to_torch_params(recipe_state_dict(shapes, ABF_SEED))
    for k, v in ps.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
            v.requires_grad_()
    # the oracle's explicit LSTM restatement (R.lstm) is differentiable w.r.t. the weight dict
    ref = R.clskd_step(pt, ps, pa, torch.from_numpy(noisy), torch.from_numpy(clean), lstm_fn=R.lstm)
    taps = ref["s_taps"]
    for t in list(taps["encoder"]) + list(taps["decoder"]) + [ref["student_wav"]]:
        t.retain_grad()
    ref["total"].backward()
    return ps, ref


def _compare(kd, ps, grads, tol):
    """Relative L2 error per parameter.  Conv biases feeding a train-mode BatchNorm have an
    analytically zero gradient (BN removes the per-channel mean); both sides then hold rounding
    noise, so those are checked as ~0 against the layer's weight-gradient norm instead."""
    bad, rows = [], []
    for name, p in kd.student.named_parameters():
        if name not in ps or ps[name].grad is None:
            continue
        got, ref = _np(grads[p]), ps[name].grad.numpy()
        pre_bn = name.endswith("_conv.bias") and not name.startswith("decoder.5.")
        if pre_bn:
            wref = np.linalg.norm(ps[name.replace(".bias", ".weight")].grad.numpy())
            e = max(np.linalg.norm(got), np.linalg.norm(ref)) / wref
            rows.append(f"{name:40s} {e:.2e} (|g| / |dW|, analytically 0)")
            ok = e <= 1e-3
        else:
            e = _rel(got, ref)
            rows.append(f"{name:40s} {e:.2e}")
            ok = e <= tol
        if not ok:
            bad.append(name)
    return bad, "\n".join(rows)


def test_clskd_backward_against_oracle():
    """Every student parameter gradient of the CLSKD loss (MRSTFT base + 14 SPKD terms through
    both ReviewKD fusions), plus the tap / waveform gradients, against the oracle's autograd."""
    from clskd.data import synthetic_pairs
    noisy, clean = synthetic_pairs(2, 8000, seed=21)
    ps, ref = _oracle_grads(noisy, clean)
    kd = _kd()
    out = kd.forward_with_tape(torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV))
    assert abs(out["loss"].item() - ref["total"].item()) <= 1e-4 * abs(ref["total"].item())
    grads = {p: torch.empty_like(p) for p in kd.student.parameters()}
    from clskd.backward import clskd_backward
    g = clskd_backward(out, kd.student, kd.review_encoder, kd.review_decoder, grads)
    torch.cuda.synchronize()
    taps = ref["s_taps"]
    errs = {"wav": _rel(_np(g["wav"]), ref["student_wav"].grad.numpy())}
    for i, t in enumerate(taps["encoder"]):
        errs[f"enc{i}"] = _rel(_np(g["enc"][i].permute(0, 3, 1, 2)), t.grad.numpy())
    for k in range(5):
        errs[f"dec{k}"] = _rel(_np(g["dec"][k].permute(0, 3, 1, 2)), taps["decoder"][k + 1].grad.numpy())
    bad, table = _compare(kd, ps, grads, 2e-3)
    msg = "\n".join(f"{k:8s} {v:.2e}" for k, v in errs.items()) + "\n" + table
    print(msg)
    assert all(v <= 2e-3 for v in errs.values()), msg
    assert not bad, f"parameters over tolerance: {bad}\n{msg}"


def test_autograd_dropin_and_train_step():
    """loss.backward() through KnowledgeDistillation.training_step gives the explicit backward's
    gradients; FlatParams + FlatAdam step matches torch.optim.Adam on those gradients; the HIP
    backward is bitwise repeatable."""
    from clskd.data import synthetic_pairs
    from clskd.train import FlatAdam, FlatParams
    noisy, clean = synthetic_pairs(2, 8000, seed=22)
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    kd = _kd()
    loss = kd.training_step((X, y), 0)
    assert loss.requires_grad
    loss.backward()
    g_auto = {n: p.grad.clone() for n, p in kd.student.named_parameters()}
    grads = {p: torch.empty_like(p) for p in kd.student.parameters()}
    kd.backward_into(kd.forward_with_tape(X, y), grads)
    grads2 = {p: torch.empty_like(p) for p in kd.student.parameters()}
    kd.backward_into(kd.forward_with_tape(X, y), grads2)
    for n, p in kd.student.named_parameters():
        assert torch.equal(grads[p], grads2[p]), n
        assert torch.equal(g_auto[n], grads[p]), n
    # one Adam step through the flat buffers vs torch.optim.Adam on the same gradients
    ref_params = {n: p.detach().clone().requires_grad_() for n, p in kd.student.named_parameters()}
    for n, p in kd.student.named_parameters():
        ref_params[n].grad = grads[p].clone()
    torch.optim.Adam(list(ref_params.values()), lr=cfg.learning_rate).step()
    kd.student.zero_grad(set_to_none=True)
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=cfg.learning_rate)
    for p in flat.params:
        flat.gviews[p].copy_(grads[p])
    opt.step()
    for n, p in kd.student.named_parameters():
        np.testing.assert_allclose(_np(p), _np(ref_params[n]), rtol=1e-6, atol=1e-7, err_msg=n)
    # the packed-weight caches see the update: the next forward uses the new weights
    l2 = kd.training_step((X, y), 0, return_parts=True)["loss"].item()
    assert l2 != loss.item()


def test_backward_refuses_redrawn_abf_weights():
    """abf_reinit='step' re-draws the ABF weights in place at every forward: the backward of an
    older tape must refuse (autograd's saved-tensor version check), the newest tape still runs."""
    from clskd.data import synthetic_pairs
    from clskd.distill import KnowledgeDistillation
    from clskd.model import DCCRN
    noisy, clean = synthetic_pairs(2, 8000, seed=24)
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    t = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    s = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    kd = KnowledgeDistillation(t.train(), s.train()).to(DEV)
    assert kd.abf_reinit == "step"  # the reference's semantics are the default
    old = kd.forward_with_tape(X, y)
    new = kd.forward_with_tape(X, y)
    grads = {p: torch.empty_like(p) for p in kd.student.parameters()}
    with pytest.raises(RuntimeError, match="modified in place"):
        kd.backward_into(old, grads)
    kd.backward_into(new, grads)
    torch.cuda.synchronize()
    assert all(torch.isfinite(g).all() for g in grads.values())


def test_clskd_backward_mixed_precision_close_to_fp32():
    """precision='mixed' (teacher + ReviewKD activations in bf16, the bench default): the
    student's gradients stay close to the all-fp32 step's (the ReviewKD backward reads bf16
    saved activations; gradients themselves are fp32 unless CLSKD_RKD_GRAD_BF16=1)."""
    from clskd.data import synthetic_pairs
    noisy, clean = synthetic_pairs(2, 8000, seed=23)
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    res = {}
    for prec in ("fp32", "mixed"):
        kd = _kd(prec)
        grads = {n: torch.empty_like(p) for n, p in kd.student.named_parameters()}
        pg = {p: grads[n] for n, p in kd.student.named_parameters()}
        kd.backward_into(kd.forward_with_tape(X, y), pg)
        res[prec] = grads
    worst = []
    for n in res["fp32"]:
        if n.endswith("_conv.bias") and not n.startswith("decoder.5."):
            continue  # analytically zero (conv bias before train-mode BN)
        worst.append((_rel(_np(res["mixed"][n]), _np(res["fp32"][n])), n))
    worst.sort(reverse=True)
    print(worst[:5])
    assert worst[0][0] < 5e-2, worst[:5]


def test_reviewkd_backward_bf16_gradient_storage():
    """The ReviewKD backward's bf16 gradient maps (precision='mixed'): abf_fuse_bwd with bf16
    dout / dnext / dx / dyup computes in fp32 exactly as the fp32-storage path fed the same
    (bf16-representable) gradients, so its outputs are that path's outputs rounded once —
    bitwise; nearest_down_sum of a bf16 map equals the fp32 sum of its upcast, bitwise; the
    conv1-BN backward from the bf16 path's partials stays within bf16 rounding of fp32's."""
    from clskd import ops
    bf = torch.bfloat16
    g = torch.Generator(device=DEV).manual_seed(5)
    B, F, T, Fr, Tr, F2, T2, C = 3, 16, 20, 8, 10, 32, 40, 64
    rn = lambda *s: torch.randn(*s, device=DEV, generator=g)
    x1 = rn(B, F, T, C).to(bf)
    res = rn(B, Fr, Tr, C).to(bf)
    w = (rn(2, 2 * C) * 0.2).contiguous()
    b = rn(2) * 0.1
    coef = torch.cat([rn(C).abs() + 0.5, rn(C) * 0.1]).contiguous()
    mv1 = torch.stack([rn(C) * 0.1, rn(C).abs() + 0.5]).contiguous()
    dout = rn(B, F, T, C).to(bf)
    dnext = rn(B, F2, T2, C).to(bf)
    outs = {}
    for gdt in (torch.float32, bf):
        dx = torch.empty(B, F, T, C, device=DEV, dtype=gdt)
        dyup = torch.empty_like(dx)
        part, nblk = ops.abf_fuse_bwd(x1, res, w, b, coef, dout.to(gdt), dx, dyup,
                                      dnext=dnext.to(gdt), mv1=mv1)
        d_x1 = torch.empty(B, F, T, C, device=DEV)
        ops.bn_bwd_from_partials(x1, dx, coef[:C], coef[C:], mv1[0], mv1[1], 1e-5,
                                 torch.ones(C, device=DEV), part, nblk, d_x1)
        down = torch.empty(B, Fr, Tr, C, device=DEV)
        ops.nearest_down_sum(dyup, down)
        outs[gdt] = (dx, dyup, d_x1, down)
    torch.cuda.synchronize()
    f, h = outs[torch.float32], outs[bf]
    assert torch.equal(h[0], f[0].to(bf))
    assert torch.equal(h[1], f[1].to(bf))
    ref_down = torch.empty_like(f[3])
    ops.nearest_down_sum(h[1].float().contiguous(), ref_down)
    torch.cuda.synchronize()
    assert torch.equal(h[3], ref_down)
    assert _rel(_np(h[2]), _np(f[2])) < 8e-3


@pytest.mark.parametrize("B,dt", [(16, torch.bfloat16), (16, torch.float32), (5, torch.bfloat16),
                                  (20, torch.bfloat16)])
def test_spkd_bn_bwd_against_fp64(B, dt):
    """clskd_spkd_bn_bwd (the SPKD gradient dz_b = sum_k M[b][k] z_k of the deferred-BN Gram
    input, fused into that BatchNorm's backward) against fp64 torch on the same rounded z: the
    exact-batch instance (B = 16), the guarded ones (B = 5, B = 20 on the 32-sample kernel), bf16
    and fp32 maps; dgamma / dbeta too; bitwise repeatable."""
    from clskd import ops
    g = torch.Generator().manual_seed(B)
    F, T, C, eps = 6, 37, 64, 1e-5
    raw = (torch.randn(B, F, T, C, generator=g) * 1.3 + 0.2).to(dt)
    xr = raw.double()
    mean = xr.mean((0, 1, 2))
    var = xr.var((0, 1, 2), unbiased=False)
    gamma = torch.rand(C, generator=g) + 0.5
    sc = torch.rand(C, generator=g) + 0.5
    sh = torch.randn(C, generator=g) * 0.1
    M = torch.randn(B, B, generator=g) * 0.01
    # the Gram's (rounded) input: fmaf(raw, sc, sh) rounded once to fp32, then to the map's type
    z = (raw.double() * sc.double() + sh.double()).float().to(dt).double()
    dz = torch.einsum("bk,kftc->bftc", M.double(), z)
    rs = 1.0 / torch.sqrt(var + eps)
    xhat = (xr - mean) * rs
    n = B * F * T
    db = dz.sum((0, 1, 2))
    dgm = (dz * xhat).sum((0, 1, 2))
    ref = gamma.double() * rs * (dz - db / n - xhat * dgm / n)
    coef = torch.cat([sc, sh]).to(DEV)
    outs = []
    for _ in range(2):
        draw = torch.empty(B, F, T, C, device=DEV)
        dgam = torch.empty(C, device=DEV)
        dbet = torch.empty(C, device=DEV)
        ops.spkd_bn_bwd(raw.to(DEV), coef, M.to(DEV), mean.float().to(DEV), var.float().to(DEV), eps,
                        gamma.to(DEV), draw, dgam, dbet)
        outs.append((draw, dgam, dbet))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    draw, dgam, dbet = outs[0]
    assert _rel(_np(draw), ref.numpy()) < 2e-5
    assert _rel(_np(dgam), dgm.numpy()) < 2e-5
    assert _rel(_np(dbet), db.numpy()) < 2e-5


# ------------------------------------------------------------------------------------------
# streaming inference (config C5)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("graph", [False, True])
def test_streaming_matches_offline_eval_forward(graph):
    """Hop-by-hop enhancement (6.25 ms hops, 9-hop latency, decoder look-ahead drained at the
    end) equals the offline eval-mode forward on the same clip (max |diff| <= 1e-5); the
    hipGraph-replayed hop equals the eager hop."""
    from clskd.data import synthetic_pairs
    from clskd.model import DCCRN
    from clskd.streaming import StreamingDCCRN
    noisy, _ = synthetic_pairs(2, 16000, seed=31)
    x = torch.from_numpy(noisy).to(DEV)
    m = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED).to(DEV)
    m.train()
    m(x)  # one train-mode pass: non-trivial running statistics for eval-mode BN
    m.eval()
    ref = m(x, is_feat=True)
    out = StreamingDCCRN(m, 2, graph=graph).process(x)
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    err = (out - ref).abs().max().item()
    assert err <= 1e-5, err


@pytest.mark.parametrize("prelu", [True, False])
def test_bn_bwd_against_torch(prelu):
    """BatchNorm2d(train) [+ PReLU] backward (clskd_bn_bwd: reduce partials, finalize, apply)
    against fp64 torch autograd: dx, dgamma, dbeta, dalpha; bitwise repeatable."""
    from clskd import ops
    g = torch.Generator().manual_seed(11)
    rows, C, eps = 16 * 64 * 37, 32, 1e-5
    x = torch.randn(rows, C, generator=g) * 1.5 + 0.3
    dy = torch.randn(rows, C, generator=g)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    a = torch.tensor([0.25])
    xd = x.double().requires_grad_()
    gd, bd, ad = gamma.double().requires_grad_(), beta.double().requires_grad_(), a.double().requires_grad_()
    mean = xd.mean(0)
    var = xd.var(0, unbiased=False)
    y = (xd - mean) / torch.sqrt(var + eps) * gd + bd
    z = torch.nn.functional.prelu(y, ad) if prelu else y
    (z * dy.double()).sum().backward()
    m, v = mean.detach().float(), var.detach().float()
    scale = (gamma / torch.sqrt(v + eps)).contiguous()
    shift = (beta - m * scale).contiguous()
    outs = []
    for _ in range(2):
        dx = torch.empty(rows, C, device=DEV)
        dg = torch.empty(C, device=DEV)
        db = torch.empty(C, device=DEV)
        da = torch.empty(1, device=DEV)
        ops.bn_bwd(x.to(DEV), dy.to(DEV), scale.to(DEV), shift.to(DEV), m.to(DEV), v.to(DEV), eps,
                   gamma.to(DEV), a.to(DEV) if prelu else None, dx, dg, db, da if prelu else None)
        outs.append((dx, dg, db, da))
    for t0, t1 in list(zip(outs[0], outs[1]))[:4 if prelu else 3]:  # (da unwritten without PReLU)
        assert torch.equal(t0, t1)
    dx, dg, db, da = outs[0]
    assert _rel(_np(dx), xd.grad.numpy()) < 1e-5
    assert _rel(_np(dg), gd.grad.numpy()) < 1e-5
    assert _rel(_np(db), bd.grad.numpy()) < 1e-5
    if prelu:
        assert _rel(_np(da), ad.grad.numpy()) < 1e-5


@pytest.mark.parametrize("C,N", [(64, 64), (32, 64), (64, 32)])
def test_split_plane_data_gradient_matches_fp32(C, N):
    """A data-gradient conv on bf16 hi / lo planes with the tripled weight [W_hi | W_hi | W_lo]
    (bf16 LDS-DMA engine, accumulate epilogue) against the exact fp32 engine on the same taps:
    the split product's error (<= ~3 * 2^-18 per product) and the read-add-write."""
    from clskd import backward as bw
    from clskd import ops
    from clskd.ops import OutMap, Seg, SegGeom
    g = torch.Generator(device=DEV).manual_seed(C + N)
    B, F, T = 2, 12, 45
    draw = torch.randn(B, F, T, C, device=DEV, generator=g)
    geom = SegGeom(C, F * T * C, T * C, C, F, T)
    taps = [(dF, dT) for dF in (-1, 0, 1) for dT in (0, 1)]
    wt = ops.pack_weight(torch.randn(N, len(taps), C, device=DEV, generator=g), len(taps) * C)
    ref = torch.empty(B, F, T, N, device=DEV)
    ops.conv([Seg(draw, 0, geom)], taps, B, F, T, N, wt, None, ref, OutMap(F * T * N, T * N, N))
    base = torch.randn(B, F, T, N, device=DEV, generator=g)
    out = base.clone()
    prev = bw._DGRAD_PLANES
    bw._DGRAD_PLANES = True
    try:
        planes, segs = bw._planes_of(draw, geom)
        w3 = bw._split3_weight(wt, len(taps), C)
        ops.conv(segs, taps, B, F, T, N, w3, None, out, OutMap(F * T * N, T * N, N), accumulate=True)
    finally:
        bw._DGRAD_PLANES = prev
    torch.cuda.synchronize()
    hi = draw.to(torch.bfloat16)
    assert torch.equal(planes[..., :C], hi)
    assert torch.equal(planes[..., C:], (draw - hi.float()).to(torch.bfloat16))
    assert _rel(_np(out - base), _np(ref)) < 2e-5


@pytest.mark.parametrize("N", [8, 16, 32, 64])
@pytest.mark.parametrize("dts", [(torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
                                 (torch.float32, torch.float32)])
def test_bn_bwd_conv1x1_against_fp64(N, dts):
    """clskd_bn_bwd_conv1x1 (ABF conv1 BatchNorm backward applied inside conv1's data gradient)
    against fp64 torch: coefficients from the partials path and from the reduce path, overwrite
    and accumulate; bitwise repeatable."""
    from clskd import ops
    xdt, gdt = dts
    g = torch.Generator().manual_seed(N)
    rows, C, eps = 4 * 9 * 37, 64, 1e-5
    x = (torch.randn(rows, C, generator=g) * 1.2 + 0.1).to(xdt)
    dy = torch.randn(rows, C, generator=g).to(gdt)
    w = torch.randn(C, N, generator=g) * 0.1
    gamma = torch.rand(C, generator=g) + 0.5
    xd = x.double()
    mean, var = xd.mean(0), xd.var(0, unbiased=False)
    rs = 1.0 / torch.sqrt(var + eps)
    xh = (xd - mean) * rs
    dd = dy.double()
    dx = gamma.double() * rs * (dd - dd.mean(0) - xh * (dd * xh).mean(0))
    base = torch.randn(rows, N, generator=g)
    ref = dx @ w.double()
    scale = (gamma / torch.sqrt(var.float() + eps)).contiguous()
    shift = (-mean.float() * scale).contiguous()
    X, DY = x.to(DEV).contiguous(), dy.to(DEV).contiguous()
    args = (X, DY, scale.to(DEV), shift.to(DEV), mean.float().to(DEV), var.float().to(DEV), eps,
            gamma.to(DEV))
    outs = []
    for rep in range(2):
        if gdt == torch.float32:
            k = ops.bn_bwd_coeffs(*args)
        else:  # partials of the fused producer's layout: {sum dy, sum dy*xhat, 0} per block
            part = torch.zeros(1, C, 3, dtype=torch.float64)
            part[0, :, 0] = dd.sum(0)
            part[0, :, 1] = (dd * xh).sum(0)
            k = ops.bn_bwd_coeffs(*args, partial=part.reshape(-1).to(DEV), nblk=1)
        o1 = torch.empty(rows, N, device=DEV)
        ops.bn_bwd_conv1x1(X, DY, k, w.to(DEV), o1)
        o2 = base.to(DEV).clone()
        ops.bn_bwd_conv1x1(X, DY, k, w.to(DEV), o2, accumulate=True)
        outs.append((o1, o2))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert _rel(_np(outs[0][0]), ref.numpy()) < 2e-5
    assert _rel(_np(outs[0][1]), (ref + base.double()).numpy()) < 2e-5


@pytest.mark.parametrize("N,Kp", [(2, 32), (8, 96), (16, 160), (12, 48)])
def test_direct_weight_gather_matches_layout(N, Kp):
    """ops.direct_weight's fp32 repack (one index gather) equals the k-major zero-padded layout
    of the direct kernel (wd[k][n] = w[n][k], n < N; zeros beyond), bitwise."""
    from clskd import ops
    w = torch.randn(N, Kp, device=DEV)
    wd = ops.direct_weight(w)
    NP = ops.direct_np(N)
    ref = torch.zeros(Kp, NP, device=DEV)
    ref[:, :N] = w.t()
    torch.cuda.synchronize()
    assert wd.shape == ref.shape and torch.equal(wd, ref)


def test_index_gather_jobs_matches_single_gathers():
    """clskd_index_gather_jobs (the backward's batched packed-gradient -> parameter scatters)
    equals one clskd_index_gather per job, bitwise, including more jobs than one launch takes."""
    from clskd import _lib, ops
    g = torch.Generator().manual_seed(3)
    jobs, refs = [], []
    for k in range(_lib.GATHER_JOBS_MAX + 7):
        src = torch.randn(500 + 13 * k, generator=g).to(DEV)
        n, J = 37 + 29 * k, 1 + k % 3
        idx = torch.randint(-1, src.numel(), (n, J), generator=g, dtype=torch.int32).to(DEV)
        sgn = (torch.randint(0, 2, (n, J), generator=g).float() * 2 - 1).to(DEV)
        out = torch.full((n,), float("nan"), device=DEV)
        ref = torch.empty(n, device=DEV)
        ops.index_gather(src, idx, sgn, ref)
        jobs.append((src, idx, sgn, out))
        refs.append(ref)
    ops.index_gather_jobs(jobs)
    for (_, _, _, out), ref in zip(jobs, refs):
        assert torch.equal(out, ref)


def test_lstm_recurrent_pre_writes_gate_preactivations():
    """clskd_lstm_recurrent_pre (the taped forward of the student's H = 32 layers): h identical
    to clskd_lstm_recurrent bit for bit, and gx overwritten with the gate pre-activations
    gx + W_hh h_{t-1} (h_{-1} = 0) of every step — against fp64 torch from the returned h
    history, 1e-5 relative (what the backward otherwise recomputed with a GEMM)."""
    from clskd import ops
    H, B, T = 32, 3, 37
    if not ops.lstm_pre_capable(H):
        pytest.skip("pre-activation output disabled (CLSKD_LSTM_PRE=0)")
    g = torch.Generator().manual_seed(5)
    gx = torch.randn(2, 2 * B, T, 4 * H, generator=g).to(DEV)
    whh = (torch.randn(2, 4 * H, H, generator=g) * 0.3).to(DEV)
    st = (2 * B * T * 4 * H, T * 4 * H, 4 * H)
    hs1 = torch.empty(2, 2 * B, T, H, device=DEV)
    hs2 = torch.empty_like(hs1)
    gx2 = gx.clone()
    ops.lstm_recurrent(gx, *st, whh, 2, 2 * B, T, H, hs1, 2 * B * T * H, T * H, H)
    ops.lstm_recurrent_pre(gx2, *st, whh, 2, 2 * B, T, H, hs2, 2 * B * T * H, T * H, H)
    torch.cuda.synchronize()
    assert torch.equal(hs1, hs2)
    h = hs1.double().cpu()
    hprev = torch.cat([torch.zeros(2, 2 * B, 1, H, dtype=torch.float64), h[:, :, :-1]], 2)
    exp = gx.double().cpu() + torch.einsum("wstk,wgk->wstg", hprev, whh.double().cpu())
    np.testing.assert_allclose(gx2.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=1e-5)


def test_lstm_forward_cell_states_feed_the_backward():
    """Round 6: clskd_lstm_recurrent_pre with a cell-state buffer stores c_t of every step, and
    clskd_lstm_bwd with c_ready = 1 (no cell-state scan of its own) gives the gate gradients of
    the scanning backward: c_t within 1e-6 relative of the backward's own scan (the same gate
    functions; only the compiler's FMA contraction of c = f c + i g may differ), dgates within
    1e-5 relative."""
    from clskd import ops
    H, B, T = 32, 3, 41
    if not ops.lstm_pre_capable(H):
        pytest.skip("pre-activation output disabled (CLSKD_LSTM_PRE=0)")
    g = torch.Generator().manual_seed(7)
    gx = torch.randn(2, 2 * B, T, 4 * H, generator=g).to(DEV)
    whh = (torch.randn(2, 4 * H, H, generator=g) * 0.3).to(DEV)
    dh = torch.randn(2, 2 * B, T, H, generator=g).to(DEV)
    st = (2 * B * T * 4 * H, T * 4 * H, 4 * H)
    hs = torch.empty(2, 2 * B, T, H, device=DEV)
    cells = torch.full((2 * 2 * B * T * H,), float("nan"), device=DEV)
    ops.lstm_recurrent_pre(gx, *st, whh, 2, 2 * B, T, H, hs, 2 * B * T * H, T * H, H, cbuf=cells)
    dg_scan = torch.empty(2, 2 * B, T, 4 * H, device=DEV)
    dg_fwd = torch.empty_like(dg_scan)
    ds = (2 * B * T * H, T * H, H)
    ops.lstm_bwd(gx, st, dh, ds, whh, 2, 2 * B, T, H, dg_scan, st)  # its own cell-state scan
    ops.lstm_bwd(gx, st, dh, ds, whh, 2, 2 * B, T, H, dg_fwd, st, cells=cells)
    torch.cuda.synchronize()
    assert torch.isfinite(cells).all()
    # c_t from the pre-activations in fp64
    pre = gx.double().cpu()
    c = torch.zeros(2, 2 * B, H, dtype=torch.float64)
    ref = []
    for t in range(T):
        q = pre[:, :, t]
        ig, fg = torch.sigmoid(q[..., :H]), torch.sigmoid(q[..., H:2 * H])
        gg = torch.tanh(q[..., 2 * H:3 * H])
        c = fg * c + ig * gg
        ref.append(c.clone())
    ref = torch.stack(ref, 2).reshape(-1)
    np.testing.assert_allclose(cells.double().cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dg_fwd.cpu().numpy(), dg_scan.cpu().numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,T,extra", [(3, 37, 2), (2, 16, 0), (1, 1, 0)])
def test_mask_e_tiles_against_fp64(B, T, extra):
    """Masking mode 'E' (DCCRN.py:207-226) forward and backward, the LDS-tiled kernels (16 frames
    per block): ragged last tile, mask columns past T (zero gradient), against fp64 autograd of
    the same formula."""
    from clskd import ops
    g = torch.Generator().manual_seed(B * 100 + T)
    Tm = T + 1 + extra
    spec = torch.randn(B, T, 520, generator=g, dtype=torch.float64)
    mask = torch.randn(B, 256, Tm, 2, generator=g, dtype=torch.float64)
    dest = torch.randn(B, T, 600, generator=g, dtype=torch.float64)
    # fp64 reference of the forward (bins 1..256 masked with the mask at frame t + 1)
    mr_ = mask[:, :, 1:T + 1, 0].transpose(1, 2).clone().requires_grad_(True)
    mi_ = mask[:, :, 1:T + 1, 1].transpose(1, 2).clone().requires_grad_(True)
    re, im = spec[..., :257], spec[..., 257:514]
    mags = torch.sqrt(re * re + im * im + 1e-8)
    phase = torch.atan2(im, re)
    z = torch.zeros(B, T, 1, dtype=torch.float64)
    mr = torch.cat([z, mr_], -1)
    mi = torch.cat([z, mi_], -1)
    mm = torch.sqrt(mr * mr + mi * mi)
    mphase = torch.atan2(mi / (mm + 1e-8), mr / (mm + 1e-8))
    em = torch.tanh(mm) * mags
    e_re, e_im = em * torch.cos(phase + mphase), em * torch.sin(phase + mphase)
    (e_re * dest[..., :257] + e_im * dest[..., 257:514]).sum().backward()
    f32 = lambda t: t.to(DEV, torch.float32).contiguous()
    est = torch.full((B, T, 600), 7.0, device=DEV)
    ops.mask_e(f32(spec), f32(mask), T, est)
    dmask = torch.full((B, 256, Tm, 2), 7.0, device=DEV)
    ops.mask_e_bwd(f32(spec), f32(mask), T, f32(dest), dmask)
    torch.cuda.synchronize()
    est, dmask = est.cpu().double(), dmask.cpu().double()
    assert _rel(est[..., :257], e_re.detach()) < 1e-5
    assert _rel(est[..., 257:514], e_im.detach()) < 1e-5
    assert torch.all(est[..., 514:600] == 0)
    assert _rel(dmask[:, :, 1:T + 1, 0], mr_.grad.transpose(1, 2)) < 1e-4
    assert _rel(dmask[:, :, 1:T + 1, 1], mi_.grad.transpose(1, 2)) < 1e-4
    assert torch.all(dmask[:, :, 0] == 0) and torch.all(dmask[:, :, T + 1:] == 0)


@pytest.mark.parametrize("H", [16, 32])
def test_lstm_bwd_pinned_reads_are_bitwise_identical(H):
    """CLSKD_LSTM_BWD_PIN only changes when the single-wave BPTT kernel issues its LDS reads (all
    of a step's gate-gradient reads together): dgates bitwise equal to the unpinned schedule."""
    from clskd import _lib, ops
    B, T = 3, 37
    g = torch.Generator().manual_seed(H)
    pre = (torch.randn(2, 2 * B, T, 4 * H, generator=g) * 0.5).to(DEV)
    dh = torch.randn(2, 2 * B, T, H, generator=g).to(DEV)
    whh = (torch.randn(2, 4 * H, H, generator=g) * 0.05).to(DEV)
    st = (2 * B * T * 4 * H, T * 4 * H, 4 * H)
    outs = []
    for pin in (0, 1):
        prev = _lib.set_knob("CLSKD_LSTM_BWD_PIN", pin)
        try:
            dg = torch.empty_like(pre)
            ops.lstm_bwd(pre, st, dh, (2 * B * T * H, T * H, H), whh, 2, 2 * B, T, H, dg, st)
            torch.cuda.synchronize()
            outs.append(dg)
        finally:
            _lib.set_knob("CLSKD_LSTM_BWD_PIN", prev)
    assert torch.equal(outs[0], outs[1])
