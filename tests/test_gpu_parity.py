"""GPU parity: the HIP path (through libclskd_hip.so) against the CPU oracle and the reference's
golden fixtures.  fp32 everywhere; tolerances are stated per test.

Parity bar (BASELINE.json north_star): waveform RMS diff <= 1e-4, SI-SNR within 0.01 dB.
"""
import os

import re

import numpy as np
import pytest
import torch

from conftest import check_summary, golden
from clskd import config as cfg
from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, apply_recipe

pytestmark = pytest.mark.gpu

DEV = "cuda"
torch.set_num_threads(min(16, os.cpu_count() or 1))


def _models(kind):
    from clskd.model import DCCRN
    spec = cfg.TEACHER if kind == "teacher" else cfg.STUDENT
    seed = TEACHER_SEED if kind == "teacher" else STUDENT_SEED
    m = DCCRN(masking_mode="E", use_clstm=True, **spec)
    apply_recipe(m, seed)
    return m.to(DEV)


def _oracle_params(kind):
    from oracle import ref_cpu as R
    from clskd.weights import recipe_state_dict
    if kind == "abf":
        shapes = {**cfg.review_param_shapes("encoder"), **cfg.review_param_shapes("decoder")}
        return R.to_torch_params(recipe_state_dict(shapes, ABF_SEED))
    spec = cfg.TEACHER if kind == "teacher" else cfg.STUDENT
    seed = TEACHER_SEED if kind == "teacher" else STUDENT_SEED
    return R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**spec), seed))


def _np(t):
    return t.detach().float().cpu().numpy()


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


# ------------------------------------------------------------------------------------------
# primitives
# ------------------------------------------------------------------------------------------
def test_conv_engine_against_torch():
    """Generic implicit GEMM: 3x3 conv with 2 segments, odd sizes, N not a tile multiple."""
    from clskd import ops
    g = torch.Generator().manual_seed(0)
    B, F, T, C1, C2, N = 3, 7, 37, 8, 12, 45
    a = torch.randn(B, F, T, C1, generator=g)
    b = torch.randn(B, F, T, C2, generator=g)
    w = torch.randn(N, C1 + C2, 3, 3, generator=g) * 0.1
    bias = torch.randn(N, generator=g)
    ref = torch.nn.functional.conv2d(torch.cat([a, b], 3).permute(0, 3, 1, 2), w, bias, padding=1)
    ad, bd = a.to(DEV), b.to(DEV)
    wp = ops.pack_weight(w.permute(0, 2, 3, 1).reshape(N, 9, C1 + C2).to(DEV), 9 * (C1 + C2))
    out = torch.empty(B, F, T, N, device=DEV)
    taps = [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)]
    ops.conv([ops.seg_bftc(ad), ops.seg_bftc(bd)], taps, B, F, T, N, wp, bias.to(DEV), out,
             ops.OutMap(F * T * N, T * N, N))
    np.testing.assert_allclose(_np(out.permute(0, 3, 1, 2)), ref.numpy(), rtol=1e-5, atol=1e-5)
    # scalar (non-vec4) path: channel counts not multiple of 4
    a3 = torch.randn(B, F, T, 3, generator=g)
    w3 = torch.randn(N, 3, 3, 3, generator=g) * 0.1
    ref3 = torch.nn.functional.conv2d(a3.permute(0, 3, 1, 2), w3, None, padding=1)
    wp3 = ops.pack_weight(w3.permute(0, 2, 3, 1).reshape(N, 9, 3).to(DEV), 27)
    out3 = torch.empty(B, F, T, N, device=DEV)
    ops.conv([ops.seg_bftc(a3.to(DEV))], taps, B, F, T, N, wp3, None, out3,
             ops.OutMap(F * T * N, T * N, N))
    np.testing.assert_allclose(_np(out3.permute(0, 3, 1, 2)), ref3.numpy(), rtol=1e-5, atol=1e-5)



_DIRECT_SHAPES = [(2, 0, 8), (2, 0, 16), (8, 8, 2), (16, 16, 2), (6, 0, 4), (6, 2, 3), (3, 0, 1),
                  (1, 0, 16), (2, 0, 32), (3, 0, 32)]


# 16-bit segments need channel runs of 8 (the kernel's 16-B loads): only those shapes run in
# bf16 / fp16, every shape in fp32
@pytest.mark.parametrize("dt,C1,C2,N", [("f32",) + s for s in _DIRECT_SHAPES] +
                         [(d,) + s for d in ("bf16", "fp16") for s in _DIRECT_SHAPES
                          if s[0] % 8 == 0 and s[1] % 8 == 0])
def test_conv_direct_against_torch_and_engine(dt, C1, C2, N):
    """Direct-convolution kernel (narrow N / short K): 2-segment 5x2 stride-(2,1) conv with fused
    BN statistics against torch (fp64 on the same bf16-rounded operands for bf16) and against the
    MFMA engines on the same descriptor (CLSKD_WLAYOUT_NK).  Tolerance: 1e-5 relative (fp32
    accumulation orders differ)."""
    _direct_case(dt, C1, C2, N)


@pytest.mark.parametrize("C1,C2,N,omap", [(2, 0, 8, "plain"), (2, 0, 8, "poly"), (8, 0, 16, "plain"),
                                            (4, 4, 2, "plain"), (2, 0, 3, "plain"), (4, 4, 8, "poly")])
def test_conv_direct_accumulate_against_torch(C1, C2, N, omap):
    """accumulate=True on the direct kernel (out += conv, fp32): the data-gradient sums of the
    narrow decoder / encoder layers (backward.py's stride-2 mask-gradient gather, N = 8 / 16, K up
    to 128).  Output maps: contiguous rows (the LDS-staged store), a polyphase parity (of_mul 2:
    the per-row vector store) and N not a power of two (the scalar store).  Against fp64 torch
    plus the prior contents; 1e-5 relative."""
    from clskd import ops
    g = torch.Generator().manual_seed(C1 * 100 + C2 * 10 + N)
    B, F, T = 3, 33, 29
    segs_h = [torch.randn(B, F, T, C1, generator=g)]
    if C2:
        segs_h.append(torch.randn(B, F, T, C2, generator=g))
    Cin = C1 + C2
    w = torch.randn(N, Cin, 5, 2, generator=g) * 0.2
    taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
    Fo = (F + 4 - 5) // 2 + 1
    wp = ops.pack_weight(w.permute(0, 2, 3, 1).reshape(N, 10, Cin).to(DEV), 10 * Cin)
    assert ops.direct_ok(N, wp.shape[1])
    xin = torch.cat([x.double() for x in segs_h], 3).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(xin, (1, 0, 2, 2)), w.double(),
                                     stride=(2, 1))[..., :T].permute(0, 2, 3, 1)
    segs = [ops.seg_bftc(x.to(DEV)) for x in segs_h]
    if omap == "poly":  # rows 2*fo + 1 of a [B][2*Fo][T][N] buffer
        out = torch.randn(B, 2 * Fo, T, N, generator=g).to(DEV)
        om = ops.OutMap(2 * Fo * T * N, T * N, N, of_mul=2, of_add=1)
    else:
        out = torch.randn(B, Fo, T, N, generator=g).to(DEV)
        om = ops.OutMap(Fo * T * N, T * N, N)
    prior = out.double().cpu()
    ops.conv(segs, taps, B, Fo, T, N, wp, None, out, om, stride_f=2, accumulate=True)
    assert ops.conv_kernel_of_last_launch().startswith("conv_direct_kernel")
    exp = prior.clone()
    if omap == "poly":
        exp[:, 1::2] += ref
    else:
        exp += ref
    np.testing.assert_allclose(out.double().cpu().numpy(), exp.numpy(), rtol=1e-5, atol=1e-5)


def _direct_case(dt, C1, C2, N):
    from clskd import ops
    g = torch.Generator().manual_seed(C1 * 100 + C2 * 10 + N)
    B, F, T = 3, 33, 29
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(dt, torch.float32)
    segs_h = [torch.randn(B, F, T, C1, generator=g).to(tdt)]
    if C2:
        segs_h.append(torch.randn(B, F, T, C2, generator=g).to(tdt))
    Cin = C1 + C2
    w = (torch.randn(N, Cin, 5, 2, generator=g) * 0.2)
    bias = torch.randn(N, generator=g)
    taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
    Fo = (F + 4 - 5) // 2 + 1
    To = T
    wk = w.permute(0, 2, 3, 1).reshape(N, 10, Cin)
    wp = ops.pack_weight(wk.to(DEV), 10 * Cin, dt if dt != "f32" else "fp32")
    wq = wp[:, :10 * Cin].float().cpu().reshape(N, 5, 2, Cin).permute(0, 3, 1, 2).double()
    xin = torch.cat([x.double() for x in segs_h], 3).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(xin, (1, 0, 2, 2)), wq, bias.double(),
                                     stride=(2, 1))[..., :To]
    segs = [ops.seg_bftc(x.to(DEV)) for x in segs_h]
    res = {}
    for route in ("direct", "engine"):
        ops._NO_DIRECT = route == "engine"
        try:
            assert ops.direct_ok(N, wp.shape[1]) == (route == "direct")
            out = torch.empty(B, Fo, To, N, device=DEV, dtype=torch.float32)
            nblk = ops.conv_mblocks(B, Fo, To)
            st = torch.empty(nblk * N * 2, device=DEV, dtype=torch.float64)
            ops.conv(segs, taps, B, Fo, To, N, wp, bias.to(DEV), out, ops.OutMap(Fo * To * N, To * N, N),
                     stride_f=2, stats=st)
            if route == "direct":
                kn = ops.conv_kernel_of_last_launch()
                assert kn.startswith("conv_direct_kernel"), kn
            res[route] = (out.permute(0, 3, 1, 2).double().cpu(), st.view(nblk, N, 2).sum(0).cpu())
        finally:
            ops._NO_DIRECT = False
    for route, (o, st) in res.items():
        np.testing.assert_allclose(o.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5, err_msg=route)
        np.testing.assert_allclose(st[:, 0].numpy(), ref.sum((0, 2, 3)).numpy(), rtol=1e-5, atol=1e-3)
        np.testing.assert_allclose(st[:, 1].numpy(), (ref ** 2).sum((0, 2, 3)).numpy(), rtol=1e-5)
    np.testing.assert_allclose(res["direct"][0].numpy(), res["engine"][0].numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("N", [45, 64, 96, 100, 136, 256, 300])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_conv_bf16_engine_against_torch(N, out_bf16):
    """bf16 LDS-DMA MFMA engine (every tile configuration the dispatcher picks for these N):
    2-segment 5x2 stride-(2,1) conv with fused BN statistics, M not a tile multiple, vs torch in
    fp64 on the same bf16 operands.  Tolerance: outputs 1e-4 relative (fp32 accumulation;
    bf16 output storage adds its own rounding: 8e-3), statistics 1e-5 relative."""
    from clskd import ops
    g = torch.Generator().manual_seed(N)
    B, F, T, C1, C2 = 3, 34, 61, 64, 32
    segs_h = [torch.randn(B, F, T, C1, generator=g).to(torch.bfloat16),
              torch.randn(B, F, T, C2, generator=g).to(torch.bfloat16)]
    Cin = C1 + C2
    w = torch.randn(N, Cin, 5, 2, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
    Fo, To = (F + 4 - 5) // 2 + 1, T
    wp = ops.pack_weight(w.permute(0, 2, 3, 1).reshape(N, 10, Cin).to(DEV), 10 * Cin, "bf16")
    assert not ops.direct_ok(N, wp.shape[1])
    wq = wp[:, :10 * Cin].float().cpu().reshape(N, 5, 2, Cin).permute(0, 3, 1, 2).double()
    xin = torch.cat([x.double() for x in segs_h], 3).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(xin, (1, 0, 2, 2)), wq, bias.double(),
                                     stride=(2, 1))[..., :To]
    out = torch.empty(B, Fo, To, N, device=DEV, dtype=torch.bfloat16 if out_bf16 else torch.float32)
    nblk = ops.conv_mblocks(B, Fo, To)
    st = torch.full((nblk * N * 2,), float("nan"), device=DEV, dtype=torch.float64)
    ops.conv([ops.seg_bftc(x.to(DEV)) for x in segs_h], taps, B, Fo, To, N, wp, bias.to(DEV), out,
             ops.OutMap(Fo * To * N, To * N, N), stride_f=2, stats=st)
    o = out.permute(0, 3, 1, 2).double().cpu()
    tol = 8e-3 if out_bf16 else 1e-4
    np.testing.assert_allclose(o.numpy(), ref.numpy(), rtol=tol, atol=tol)
    stc = st.view(nblk, N, 2).cpu()
    assert torch.isfinite(stc).all(), "every 128-row partial must be written"
    np.testing.assert_allclose(stc[:, :, 0].sum(0).numpy(), ref.sum((0, 2, 3)).numpy(), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(stc[:, :, 1].sum(0).numpy(), (ref ** 2).sum((0, 2, 3)).numpy(), rtol=1e-5)


HALO_CASES = {
    # name: (segment channels, N, taps, stride_f, Fi, Fo, of_mul, of_add, out_bf16)
    "abf3x3_n32": ((64,), 32, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 24, 24, 1, 0, True),
    "abf3x3_n64": ((64,), 64, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 24, 24, 1, 0, True),
    "enc5x2_s2": ((32,), 64, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 48, 24, 1, 0, True),
    "dec_parity1": ((32, 32), 32, [(dF, -kt) for dF in (1, 0) for kt in (0, 1)], 1, 24, 24, 2, 1, False),
    # [64][1536] weights exceed LDS beside the halo buffers: two 32-column launches
    "dec_parity0_n64_split": ((128, 128), 64, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1,
                              24, 24, 2, 0, True),
}


_LP = {"bf16": torch.bfloat16, "fp16": torch.float16}
_LP_TOL = {"bf16": 8e-3, "fp16": 2e-3}  # 16-bit output rounding (unit roundoff 2^-9 / 2^-12)


@pytest.mark.parametrize("lp", ["bf16", "fp16"])
@pytest.mark.parametrize("case", sorted(HALO_CASES))
def test_conv_halo_kernel_against_torch(case, lp):
    """Halo-tiled narrow bf16 conv (weights resident in LDS, input halo reused across taps):
    shapes the dispatcher routes there (N <= 64, channel runs of 32) incl. two segments, stride-2
    F and an interleaved (polyphase) output map, fused BN statistics; vs torch fp64 on the same
    bf16 operands.  Tolerance 1e-4 relative (fp32 out) / 8e-3 (bf16 out); stats 1e-5."""
    from clskd import ops
    segc, N, taps, sf, Fi, Fo, of_mul, of_add, out_bf16 = HALO_CASES[case]
    g = torch.Generator().manual_seed(len(case) * 7 + N)
    B, T = 3, 100
    segs_h = [torch.randn(B, Fi, T, c, generator=g).to(_LP[lp]) for c in segc]
    Cin = sum(segc)
    K = len(taps) * Cin
    w = torch.randn(N, len(taps), Cin, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.to(DEV), K, lp)
    assert not ops.direct_ok(N, wp.shape[1])
    wq = wp[:, :K].float().cpu().double().view(N, len(taps), Cin)
    x = torch.cat([s.double() for s in segs_h], 3)  # [B, Fi, T, Cin]
    ref = bias.double().view(1, 1, 1, N).expand(B, Fo, T, N).clone()
    for ti, (dF, dT) in enumerate(taps):
        fi = torch.arange(Fo) * sf + dF
        tt = torch.arange(T) + dT
        vf = (fi >= 0) & (fi < Fi)
        vt = (tt >= 0) & (tt < T)
        sub = torch.zeros(B, Fo, T, Cin, dtype=torch.float64)
        sub[:, vf.nonzero()[:, 0][:, None], vt.nonzero()[:, 0][None, :]] = \
            x[:, fi[vf][:, None], tt[vt][None, :]]
        ref += torch.einsum("bftc,nc->bftn", sub, wq[:, ti])
    Fout = Fo * of_mul
    out = torch.zeros(B, Fout, T, N, device=DEV, dtype=_LP[lp] if out_bf16 else torch.float32)
    nblk = ops.conv_mblocks(B, Fo, T)
    st = torch.full((nblk * N * 2,), float("nan"), device=DEV, dtype=torch.float64)
    ops.conv([ops.seg_bftc(s.to(DEV)) for s in segs_h], taps, B, Fo, T, N, wp, bias.to(DEV), out,
             ops.OutMap(Fout * T * N, T * N, N, of_mul=of_mul, of_add=of_add), stride_f=sf, stats=st)
    kname = ops.conv_kernel_of_last_launch()
    assert kname.startswith("conv_halo_kernel") and (kname.endswith(",f16>") == (lp == "fp16")), kname
    o = out.double().cpu()[:, of_add::of_mul]
    tol = _LP_TOL[lp] if out_bf16 else 1e-4
    np.testing.assert_allclose(o.numpy(), ref.numpy(), rtol=tol, atol=tol)
    if of_mul > 1:  # the other parity's rows are untouched
        assert torch.all(out.double().cpu()[:, (of_add + 1) % of_mul::of_mul] == 0)
    stc = st.view(nblk, N, 2).cpu()
    assert torch.isfinite(stc).all(), "every statistics slot must be written"
    np.testing.assert_allclose(stc[:, :, 0].sum(0).numpy(), ref.sum((0, 1, 2)).numpy(), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(stc[:, :, 1].sum(0).numpy(), (ref ** 2).sum((0, 1, 2)).numpy(), rtol=1e-5)


HALO32_CASES = {
    # name: (segment channels, N, taps, stride_f, Fi, Fo, of_mul, of_add) — the student's layers
    # (B = 3, T = 101: >= 32 tiles of 8 F-rows x 32 steps, the kernel's eligibility floor)
    "enc_c16_n32": ((16,), 32, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 38, 19, 1, 0),
    "enc_c32_n64": ((32,), 64, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 48, 24, 1, 0),
    # [64][640] weights exceed LDS beside the halo buffers: two 32-column launches
    "enc_c64_n64_split": ((64,), 64, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 40, 20, 1, 0),
    "enc_c24_n48": ((8, 16), 48, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 37, 19, 1, 0),
    "dec_parity0_n64_split": ((64, 64), 64, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1,
                              20, 20, 2, 0),
    "dec_parity1_n32": ((32, 32), 32, [(dF, -kt) for dF in (1, 0) for kt in (0, 1)], 1, 20, 20, 2, 1),
    # 8/16-wide decoder layers (CLSKD_HALO32_MIN_N=8: the 32-column block with zero columns)
    "dec_parity0_n8": ((16, 16), 8, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1, 20, 20, 2, 0),
    "dec_parity0_n16": ((32, 32), 16, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1, 20, 20, 2, 0),
    "dec_parity1_n16": ((32, 32), 16, [(dF, -kt) for dF in (1, 0) for kt in (0, 1)], 1, 20, 20, 2, 1),
    "abf3x3_n64_split": ((64,), 64, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 17, 17,
                         1, 0),
}


@pytest.mark.parametrize("case", sorted(HALO32_CASES))
def test_conv_halo_f32_against_torch(case):
    """Halo-tiled exact-fp32 conv (csrc/conv_halo32.hip: weights resident in LDS in k-quad order,
    8-channel input halo chunks reused across taps, v_mfma_f32_32x32x2_f32): the student's layer
    shapes (stride-2 encoder, two-segment polyphase decoder with interleaved output rows, 3x3),
    N = 32 / 48 / 64, column-split launches (CLSKD_HALO32_SPLIT=1: the dispatcher leaves those to
    the engine by default), ragged F and T tiles, fused BN statistics; vs torch fp64 and vs the
    fp32 engine on the same descriptor.  Tolerance 1e-5 relative (fp32 accumulation orders
    differ); stats 1e-5."""
    from clskd import _lib, ops
    segc, N, taps, sf, Fi, Fo, of_mul, of_add = HALO32_CASES[case]
    g = torch.Generator().manual_seed(len(case) * 11 + N)
    B, T = 3, 101
    segs_h = [torch.randn(B, Fi, T, c, generator=g) for c in segc]
    Cin = sum(segc)
    K = len(taps) * Cin
    w = torch.randn(N, len(taps), Cin, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.to(DEV), K)
    assert not ops.direct_ok(N, wp.shape[1])
    wq = w.double()
    x = torch.cat([s.double() for s in segs_h], 3)  # [B, Fi, T, Cin]
    ref = bias.double().view(1, 1, 1, N).expand(B, Fo, T, N).clone()
    for ti, (dF, dT) in enumerate(taps):
        fi = torch.arange(Fo) * sf + dF
        tt = torch.arange(T) + dT
        vf = (fi >= 0) & (fi < Fi)
        vt = (tt >= 0) & (tt < T)
        sub = torch.zeros(B, Fo, T, Cin, dtype=torch.float64)
        sub[:, vf.nonzero()[:, 0][:, None], vt.nonzero()[:, 0][None, :]] = \
            x[:, fi[vf][:, None], tt[vt][None, :]]
        ref += torch.einsum("bftc,nc->bftn", sub, wq[:, ti])
    Fout = Fo * of_mul
    res = {}
    for route in ("halo", "engine"):
        prev = _lib.set_knob("CLSKD_NO_HALO32", int(route == "engine"))
        prev_split = _lib.set_knob("CLSKD_HALO32_SPLIT", 1)
        prev_min = _lib.set_knob("CLSKD_HALO32_MIN_N", 8)
        try:
            out = torch.zeros(B, Fout, T, N, device=DEV)
            nblk = ops.conv_mblocks(B, Fo, T)
            st = torch.full((nblk * N * 2,), float("nan"), device=DEV, dtype=torch.float64)
            ops.conv([ops.seg_bftc(s.to(DEV)) for s in segs_h], taps, B, Fo, T, N, wp, bias.to(DEV),
                     out, ops.OutMap(Fout * T * N, T * N, N, of_mul=of_mul, of_add=of_add),
                     stride_f=sf, stats=st)
            kname = ops.conv_kernel_of_last_launch()
        finally:
            _lib.set_knob("CLSKD_NO_HALO32", prev)
            _lib.set_knob("CLSKD_HALO32_SPLIT", prev_split)
            _lib.set_knob("CLSKD_HALO32_MIN_N", prev_min)
        assert kname.startswith("conv_halo_f32_kernel") == (route == "halo"), (route, kname)
        res[route] = out.double().cpu()
        o = res[route][:, of_add::of_mul]
        np.testing.assert_allclose(o.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5, err_msg=route)
        if of_mul > 1:  # the other parity's rows are untouched
            assert torch.all(res[route][:, (of_add + 1) % of_mul::of_mul] == 0)
        stc = st.view(nblk, N, 2).cpu()
        assert torch.isfinite(stc).all(), "every statistics slot must be written"
        np.testing.assert_allclose(stc[:, :, 0].sum(0).numpy(), ref.sum((0, 1, 2)).numpy(), rtol=1e-5,
                                   atol=1e-3)
        np.testing.assert_allclose(stc[:, :, 1].sum(0).numpy(), (ref ** 2).sum((0, 1, 2)).numpy(), rtol=1e-5)
    np.testing.assert_allclose(res["halo"].numpy(), res["engine"].numpy(), rtol=1e-5, atol=1e-5)


def _abf_torch(x, y, shape, abf):
    """framework.py:204-222 in torch fp64 (train-mode BatchNorm): returns (out, x_fused, mean1,
    var1) from NCHW inputs."""
    import torch.nn.functional as Fn
    d = lambda t: t.detach().double().cpu()  # noqa: E731
    x1 = Fn.conv2d(x, d(abf.conv1[0].weight))
    m1, v1 = x1.mean((0, 2, 3)), x1.var((0, 2, 3), unbiased=False)
    xb = Fn.batch_norm(x1, None, None, d(abf.conv1[1].weight), d(abf.conv1[1].bias), True, 0.1, 1e-5)
    if abf.att_conv is not None:
        yu = Fn.interpolate(y, (shape, x.shape[-1]), mode="nearest")
        z = torch.sigmoid(Fn.conv2d(torch.cat([xb, yu], 1), d(abf.att_conv[0].weight),
                                    d(abf.att_conv[0].bias)))
        xb = xb * z[:, 0:1] + yu * z[:, 1:2]
    o = Fn.conv2d(xb, d(abf.conv2[0].weight), padding=1)
    o = Fn.batch_norm(o, None, None, d(abf.conv2[1].weight), d(abf.conv2[1].bias), True, 0.1, 1e-5)
    return o, xb, m1, v1


@pytest.mark.parametrize("cin", [8, 16, 32, 64])
@pytest.mark.parametrize("fuse", [False, True])
@pytest.mark.parametrize("compute", ["fp32", "bf16"])
def test_abf_folded_level_against_torch(cin, fuse, compute):
    """ABF level with conv1 folded (clskd_abf_moments / _bn1_finalize / _conv1_fuse): conv1's
    BatchNorm statistics from the tap's moments, conv1 recomputed in the fused kernel.  Against
    torch fp64 (framework.py:204-222) on a strided tap (a channel sub-range view), plus the BN1
    running statistics and the tape's raw conv1 output / batch mean-var.  Tolerances: fp32
    storage 2e-5 (fused map) / 1e-4 (output); bf16 storage 2e-2 / 5e-2 (relative to max)."""
    from clskd.framework import ABF
    g = torch.Generator().manual_seed(cin * 10 + fuse)
    B, F, T = 3, 16, 37
    base = torch.randn(B, F, T, cin + 4, generator=g).abs()  # PReLU-like, non-zero mean
    x = base.to(DEV)[..., 4:]                                  # strided view: channels 4..cin+3
    abf = ABF(cin, 64, 32, fuse).to(DEV).train()
    abf.compute = compute
    with torch.no_grad():
        for bn in (abf.conv1[1], abf.conv2[1]):
            bn.weight.uniform_(0.5, 1.5, generator=None)
            bn.bias.uniform_(-0.2, 0.2)
    y = torch.randn(B, F // 2, T, 64, generator=g).to(DEV).to(abf.act_dtype) if fuse else None
    rm0, rv0 = abf.conv1[1].running_mean.clone(), abf.conv1[1].running_var.clone()
    tape = {}
    out, xf = abf.forward_bftc(x, y, F if fuse else None, F, tape=tape)
    torch.cuda.synchronize()
    xn = x.permute(0, 3, 1, 2).double().cpu()
    yn = y.permute(0, 3, 1, 2).double().cpu() if fuse else None
    o_ref, xf_ref, m1, v1 = _abf_torch(xn, yn, F, abf)
    tol_f, tol_o = (2e-5, 1e-4) if compute == "fp32" else (2e-2, 5e-2)
    got_xf = xf.permute(0, 3, 1, 2).double().cpu()
    got_o = out.permute(0, 3, 1, 2).double().cpu()
    assert float((got_xf - xf_ref).abs().max()) <= tol_f * float(xf_ref.abs().max())
    assert float((got_o - o_ref).abs().max()) <= tol_o * float(o_ref.abs().max())
    np.testing.assert_allclose(_np(tape["mv1"][0]), m1.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_np(tape["mv1"][1]), v1.numpy(), rtol=1e-4, atol=1e-6)
    n = B * F * T
    np.testing.assert_allclose(_np(abf.conv1[1].running_mean), 0.9 * _np(rm0) + 0.1 * m1.numpy(),
                               rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_np(abf.conv1[1].running_var),
                               0.9 * _np(rv0) + 0.1 * v1.numpy() * n / (n - 1), rtol=1e-4)
    x1_ref = torch.einsum("bcft,nc->bnft", xn, abf.conv1[0].weight.detach().double().cpu().reshape(64, cin))
    got_x1 = tape["x1"].permute(0, 3, 1, 2).double().cpu()
    tol_x1 = 1e-5 if compute == "fp32" else 1e-2
    assert float((got_x1 - x1_ref).abs().max()) <= tol_x1 * float(x1_ref.abs().max())
    # the materialising path (pointwise conv + BN + fuse) agrees with the folded one
    w1p, _, att = abf._weights(x.dtype)
    x1_old = abf._level_conv1(x.contiguous(), y, F if fuse else None, w1p, att, True, None,
                              __import__("clskd.ops", fromlist=["ops"]).conv_mblocks(B, F, T))
    torch.cuda.synchronize()
    diff = float((x1_old.double() - xf.double()).abs().max())
    assert diff <= (1e-5 if compute == "fp32" else 3e-2) * float(xf.double().abs().max()), diff


def test_stft_istft_golden():
    st = golden("stft.npz")
    m = _models("student")
    x = torch.from_numpy(st["x"]).to(DEV)
    spec = m.spectrum(x)  # [B][T][514]
    np.testing.assert_allclose(_np(spec.permute(0, 2, 1)), st["spec"], rtol=1e-5, atol=2e-5)


def test_sisnr_known_answers_and_examples():
    from clskd.tools_for_loss import si_snr
    k = golden("kat_sisnr.npz")
    ref = torch.from_numpy(k["reference"]).float().to(DEV)
    for name in ("flip", "ref_plus_flip", "ref_plus_half", "two_ref_plus_one"):
        est = torch.from_numpy(k[f"est/{name}"]).float().to(DEV)
        v = si_snr(est, ref).item()
        assert abs(v - float(k[f"si_snr32/{name}"])) < 1e-3, name
        assert abs(v - float(k[f"doc/si_sdr/{name}"])) < 1e-3, name
    v = si_snr(torch.from_numpy(k["rand/s1"]).to(DEV), torch.from_numpy(k["rand/s2"]).to(DEV)).item()
    assert abs(v - float(k["rand/si_snr"])) < 1e-4
    ex = golden("examples.npz")
    for e in ["606", "1038", "1132", "1431", "2158"]:
        s0 = torch.from_numpy(ex[f"{e}/s0"] / 32768.0).float().to(DEV)
        est = torch.from_numpy(ex[f"{e}/est"] / 32768.0).float().to(DEV)
        assert abs(si_snr(est, s0).item() - float(ex[f"{e}/si_snr"])) < 1e-3, e  # << 0.01 dB


def test_losses_golden():
    from clskd.framework import MultiResolutionSTFTLoss, SPKDLoss
    ls = golden("losses.npz")
    x = torch.from_numpy(ls["mr/x"]).to(DEV)
    y = torch.from_numpy(ls["mr/y"]).to(DEV)
    sc, mag = MultiResolutionSTFTLoss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100]).to(DEV)(x, y)
    assert abs(sc.item() - float(ls["mr/sc"])) < 2e-6
    assert abs(mag.item() - float(ls["mr/mag"])) < 2e-5
    sc3, mag3 = MultiResolutionSTFTLoss().to(DEV)(x, y)
    assert abs(sc3.item() - float(ls["mr3/sc"])) < 2e-6
    assert abs(mag3.item() - float(ls["mr3/mag"])) < 2e-5
    for n in range(3):
        a = torch.from_numpy(ls[f"spkd{n}/s"]).to(DEV)
        b = torch.from_numpy(ls[f"spkd{n}/t"]).to(DEV)
        v = SPKDLoss(a, b, "batchmean")().item()
        assert abs(v - float(ls[f"spkd{n}/batchmean"])) <= 1e-4 * abs(float(ls[f"spkd{n}/batchmean"])) + 1e-8
        v = SPKDLoss(a, b, "sum")().item()
        assert abs(v - float(ls[f"spkd{n}/sum"])) <= 1e-4 * abs(float(ls[f"spkd{n}/sum"])) + 1e-7


def test_gram_batch32_and_determinism():
    """B in (16, 32] uses the 2x2-block MFMA path; results are bitwise repeatable."""
    from clskd import ops
    from oracle import ref_cpu as R
    g = torch.Generator().manual_seed(1)
    a = torch.randn(29, 3, 50, 12, generator=g)
    b = torch.randn(29, 5, 50, 12, generator=g) + 0.3
    ad, bd = a.to(DEV), b.to(DEV)
    l1, gs, gt = ops.spkd_losses([(ops.gram_view(ad), ops.gram_view(bd))], 29, True, True)
    l2 = ops.spkd_losses([(ops.gram_view(ad), ops.gram_view(bd))], 29, True)
    assert torch.equal(l1, l2)
    np.testing.assert_allclose(_np(gs[0]), R.spkd_gram(a).numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(_np(gt[0]), R.spkd_gram(b).numpy(), rtol=1e-4, atol=1e-6)
    assert abs(l1.item() - R.spkd_loss(a, b).item()) <= 1e-4 * R.spkd_loss(a, b).item()


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("B", [16, 29])
def test_bn_apply_gram_fused_matches_separate_passes(dtype, B):
    """ops.bn_apply_gram (the teacher taps' BatchNorm + PReLU apply fused with their SPKD Gram
    partials, in place) against the two passes it replaces: the applied tensor is bitwise
    clskd_bn_apply's, the Gram slabs are bitwise those of a Gram over that tensor (same slab
    split), and the normalised Gram matches fp64 torch."""
    from clskd import _lib, ops
    from oracle import ref_cpu as R
    g = torch.Generator().manual_seed(B)
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    F, T, C = 6, 37, 64
    x = (torch.randn(B, F, T, C, generator=g) * 2 + 0.5).to(tdt).to(DEV)
    coef = torch.cat([torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g)]).to(DEV)
    alpha = torch.tensor([0.25], device=DEV)
    # separate passes: clskd_bn_apply, then a Gram with the slab split bn_apply_gram picks
    y = torch.empty_like(x)
    sc = coef.data_ptr()
    ops.check(ops.lib().clskd_bn_apply(x.data_ptr(), y.data_ptr(), B * F * T, C, sc, sc + 4 * C,
                                       alpha.data_ptr(), ops._dt(x), ops._stream()), "bn_apply")
    per_row = F * T * C
    ce = max(C, min(16384, -(-(-(-per_row // ops._APPLY_GRAM_SLABS)) // C) * C))
    ref = ops.GramSlabs([ops.gram_view(y)], B, chunk_elems=ce)
    xf = x.clone()
    fused = ops.bn_apply_gram(xf, coef, alpha, B)
    torch.cuda.synchronize()
    assert torch.equal(xf, y), "fused apply differs from clskd_bn_apply"
    assert fused.slabs.numel() == ref.slabs.numel()
    assert torch.equal(fused.slabs, ref.slabs), "fused Gram partials differ"
    loss, gs, gt = ops.spkd_finalize(fused.refs, ref.refs, B, return_grams=True, device=x.device)
    torch.cuda.synchronize()
    assert loss.item() == 0.0
    np.testing.assert_allclose(_np(gs[0]), R.spkd_gram(y.permute(0, 3, 1, 2).double().cpu()).numpy(),
                               rtol=1e-4, atol=1e-6)


# ------------------------------------------------------------------------------------------
# model forwards
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["student", "teacher"])
def test_forward_train_golden(kind):
    fx = golden(f"{kind}_fwd_train.npz")
    m = _models(kind).train()
    res = m.run(torch.from_numpy(fx["x"]).to(DEV), train=True, bn_updates=0)
    for k, v in enumerate(res["enc_nchw"]):
        check_summary(f"enc{k}", _np(v), fx, rtol=2e-4, atol=2e-5)
    for k, v in enumerate(res["dec_nchw"]):
        check_summary(f"dec{k}", _np(v), fx, rtol=2e-4, atol=2e-5)
    r, i = m.clstm_from_dec_in(res["dec_in"])
    check_summary("clstm_real", _np(r.transpose(0, 1)), fx, rtol=2e-4, atol=2e-5)
    check_summary("clstm_img", _np(i.transpose(0, 1)), fx, rtol=2e-4, atol=2e-5)
    for name in ("mask_real", "mask_imag", "real", "imag"):
        check_summary(name, _np(res[name]), fx, rtol=2e-4, atol=2e-5)
    wav = _np(res["out_wav"])
    assert rms(wav, fx["out_wav"]) <= 1e-5
    np.testing.assert_allclose(wav, fx["out_wav"], atol=1e-4)


def test_bn_running_stats_two_updates():
    """distill.py:85+:100 train forwards update BN running stats twice."""
    fx = golden("student_fwd_train.npz")
    m = _models("student").train()
    m.run(torch.from_numpy(fx["x"]).to(DEV), train=True, bn_updates=2)
    sd = m.state_dict()
    for k in fx.files:
        if k.startswith("bn2/"):
            np.testing.assert_allclose(_np(sd[k[4:]]), fx[k], rtol=1e-4, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("pfold", [0, 3])
@pytest.mark.parametrize("nblk,C", [(3, 8), (256, 64), (2048, 16), (3000, 128), (12000, 8),
                                    (1500, 100), (2100, 200)])
def test_bn_finalize_reads_all_partials(nblk, C, pfold):
    """clskd_bn_finalize alone (no level-2 compaction launch) on up to 12,000 {sum, sumsq}
    partials, read directly (CLSKD_BN_PFOLD 0) or after the in-place fold to 512 rows (above
    1,024 rows; 2C elements per row from 16 to 400: one and two element chunks per workgroup):
    scale / shift / batch mean / var and one running-stat update vs fp64 numpy."""
    from clskd import ops, _lib
    _lib.set_knob("CLSKD_BN_PFOLD", pfold)
    try:
        _bn_finalize_case(ops, nblk, C)
    finally:
        _lib.set_knob("CLSKD_BN_PFOLD", 1)


@pytest.mark.parametrize("nblk,C", [(16384, 64), (2000, 8), (700, 16)])
def test_bn_bwd_from_partials_fold_matches_direct(nblk, C):
    """clskd_bn_bwd_from_partials with its [nblk][C][3] partials folded in place first
    (CLSKD_BN_PFOLD bit 1, above 1,024 rows) against the direct read: dx within fp64-sum
    reassociation (1e-6 relative), and bitwise repeatable across calls."""
    from clskd import ops, _lib
    g = torch.Generator().manual_seed(nblk + C)
    rows = 64 * nblk
    x = torch.randn(rows, C, generator=g).to(DEV)
    dy = torch.randn(rows, C, generator=g).to(DEV)
    scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
    shift = torch.randn(C, generator=g).to(DEV)
    mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
    var = (torch.rand(C, generator=g) + 0.5).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    part0 = (torch.randn(nblk, C, 3, generator=g, dtype=torch.float64) * 10.0).to(DEV).reshape(-1)
    outs = []
    try:
        for pf in (0, 1, 1):
            _lib.set_knob("CLSKD_BN_PFOLD", pf)
            dx = torch.empty_like(x)
            ops.bn_bwd_from_partials(x, dy, scale, shift, mean, var, 1e-5, gamma, part0.clone(),
                                     nblk, dx)
            outs.append(dx)
    finally:
        _lib.set_knob("CLSKD_BN_PFOLD", 1)
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(outs[1]), _np(outs[0]), rtol=1e-6, atol=1e-6)
    assert torch.equal(outs[1], outs[2])


def _bn_finalize_case(ops, nblk, C):
    g = torch.Generator().manual_seed(nblk + C)
    rows = 1000 * nblk
    x = torch.randn(nblk, C, 2, generator=g, dtype=torch.float64)
    x[..., 0] *= 50.0
    x[..., 1] = x[..., 1].abs() * 1000.0 + 2000.0
    part = x.to(DEV)
    gamma = torch.rand(C, generator=g).to(DEV)
    beta = torch.randn(C, generator=g).to(DEV)
    rm = torch.randn(C, generator=g).to(DEV)
    rv = torch.rand(C, generator=g).to(DEV) + 0.5
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
        bn.running_mean.copy_(rm)
        bn.running_var.copy_(rv)
    coef = torch.empty(2 * C, device=DEV)
    mean_o = torch.empty(C, device=DEV)
    var_o = torch.empty(C, device=DEV)
    ops.bn_coef_from_partials(part.reshape(-1), nblk, rows, C, bn, coef, (mean_o, var_o))
    torch.cuda.synchronize()
    S, Q = x[..., 0].sum(0).numpy(), x[..., 1].sum(0).numpy()
    mean = S / rows
    var = np.maximum(Q / rows - mean * mean, 0.0)
    sc = gamma.double().cpu().numpy() / np.sqrt(var + bn.eps)
    np.testing.assert_allclose(_np(mean_o), mean, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(_np(var_o), var, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(_np(coef[:C]), sc, rtol=1e-6)
    np.testing.assert_allclose(_np(coef[C:]), beta.double().cpu().numpy() - mean * sc, rtol=1e-5, atol=1e-5)
    unb = var * rows / (rows - 1)
    np.testing.assert_allclose(_np(bn.running_mean), 0.9 * rm.double().cpu().numpy() + 0.1 * mean, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_np(bn.running_var), 0.9 * rv.double().cpu().numpy() + 0.1 * unb, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kind,B,L", [("student", 1, 16037), ("student", 3, 401), ("student", 2, 250),
                                      ("teacher", 1, 12345), ("student", 5, 8000)])
@pytest.mark.parametrize("train", [True, False])
def test_forward_ragged_lengths_against_oracle(kind, B, L, train):
    """Edge cases of DCCRN.forward (DCCRN.py:149-240) against the oracle: a batch of one, odd
    batch sizes, lengths that are not a whole number of hops (the ConvSTFT floor, T = (L+200)//100
    + 1) and clips shorter than one 400-sample window (T = 3 or 5 frames) — train-mode BN (batch
    statistics over whatever rows exist) and eval-mode BN (running statistics).  Output length,
    waveform RMS <= 1e-5 and max |diff| <= 1e-4, masks within 2e-4 relative."""
    from clskd.data import synthetic_pairs
    from oracle import ref_cpu as R
    noisy, _ = synthetic_pairs(B, L, seed=B * 1000 + L)
    m = _models(kind).train(train)
    p = {k: v.detach().cpu() for k, v in m.state_dict().items() if not k.startswith(("stft.", "istft."))}
    x = torch.from_numpy(noisy).to(DEV)
    with torch.no_grad():
        out = m(x)
        ref = R.dccrn_forward(p, torch.from_numpy(noisy), train=train)
    wav = _np(out[4])
    rw = ref["out_wav"].numpy()
    assert wav.shape == rw.shape, (wav.shape, rw.shape)
    assert rms(wav, rw) <= 1e-5
    assert np.abs(wav - rw).max() <= 1e-4
    for i, name in ((0, "mask_real"), (1, "mask_imag")):
        np.testing.assert_allclose(_np(out[i]), ref[name].numpy(), rtol=2e-4, atol=2e-5)


def test_forward_eval_golden():
    fx = golden("student_fwd_eval.npz")
    m = _models("student").eval()
    out = m(torch.from_numpy(fx["x"]).to(DEV))
    assert rms(_np(out[4]), fx["out_wav"]) <= 1e-5
    check_summary("mask_real", _np(out[0]), fx, rtol=2e-4, atol=2e-5)


def test_feature_extraction_api():
    from clskd import feature_extraction
    fx = golden("student_fwd_train.npz")
    m = _models("student").train()
    ext = feature_extraction.DCCRN(m)
    fm = ext.extract_feature_maps(torch.from_numpy(fx["x"]).to(DEV))
    ext.remove_hook()
    assert len(fm["encoder"]) == 6 and len(fm["decoder"]) == 6 and len(fm["clstm"]) == 1
    assert tuple(fm["encoder"][0].shape) == tuple(fx["enc0/shape"])
    assert tuple(fm["decoder"][2].shape) == tuple(fx["dec2/shape"])
    r, i = fm["clstm"][0]
    check_summary("clstm_real", _np(r.transpose(0, 1)), fx, rtol=2e-4, atol=2e-5)
    assert m._tap_sinks == []


# ------------------------------------------------------------------------------------------
# the CLSKD step
# ------------------------------------------------------------------------------------------
def _kd(abf_seed=ABF_SEED):
    from clskd.distill import KnowledgeDistillation
    kd = KnowledgeDistillation(_models("teacher").train(), _models("student").train(),
                               abf_reinit="once").to(DEV)
    apply_recipe(kd.review_encoder, abf_seed, "encoder.")
    apply_recipe(kd.review_decoder, abf_seed, "decoder.")
    return kd


def test_step_g8_grid_cap_is_bitwise_neutral():
    """clskd_step caps conv_gemm8's persistent grid at 7/8 of the CUs inside the concurrent
    step (distill._STEP_G8_GRID_FRAC): only the deal of tiles to workgroups changes, so every
    loss slot, the student waveform and the BatchNorm running statistics are bitwise those of
    the full-grid step.  Checked on the data-parallel deal (CLSKD_G8_SK=0): with stream-K the
    grid also sets where split tiles' K sums are cut (deterministic per grid, rounding-level
    across grids: test_conv_gemm8_stream_k)."""
    from clskd import _lib, distill
    from clskd.data import synthetic_pairs
    n, c = synthetic_pairs(4, 32000, seed=41)
    X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
    outs = []
    prev = distill._STEP_G8_GRID_FRAC
    prev_sk = _lib.set_knob("CLSKD_G8_SK", 0)
    try:
        for frac in (0.0, 0.875, 0.5):
            distill._STEP_G8_GRID_FRAC = frac
            kd = _kd().set_precision("mixed")
            o = kd.training_step((X, y), 0, return_parts=True)
            torch.cuda.synchronize()
            outs.append((torch.cat([o["loss"].reshape(1), o["spkd"], o["base"].reshape(1)]),
                         o["student_wav"].clone(),
                         [b.clone() for nme, b in kd.named_buffers() if "running" in nme]))
    finally:
        distill._STEP_G8_GRID_FRAC = prev
        _lib.set_knob("CLSKD_G8_SK", prev_sk)
    for loss, wav, bufs in outs[1:]:
        assert torch.equal(loss, outs[0][0])
        assert torch.equal(wav, outs[0][1])
        assert all(torch.equal(a, b) for a, b in zip(bufs, outs[0][2]))


@pytest.mark.parametrize("precision", ["fp32", "mixed"])
def test_teacher_ahead_matches_serial_schedule(precision):
    """clskd_step(teacher_ahead=True): the teacher chain of step i+1 overlapping step i's tail
    gives bitwise the same per-step losses (all 16 loss slots) as the step-by-step schedule over
    five back-to-back steps on distinct resident batches (the overlap changes when kernels run,
    not what they compute: deterministic reductions, no atomics)."""
    from clskd.data import synthetic_pairs
    kd = _kd()
    kd.set_precision(precision)
    batches = []
    for k in range(5):
        n, c = synthetic_pairs(4, 16000, seed=70 + k)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))
    torch.cuda.synchronize()

    def run(ahead):
        kd.teacher_ahead = ahead
        outs = []
        with torch.no_grad():
            for b in batches:
                o = kd.training_step(b, 0, return_parts=True)
                outs.append(torch.cat([o["loss"].reshape(1), o["sc"].reshape(1), o["base"].reshape(1),
                                       o["spkd"].reshape(-1)]).clone())
        torch.cuda.synchronize()
        kd.teacher_ahead = False
        return torch.stack(outs).cpu()

    ref = run(False)
    got = run(True)
    assert torch.equal(ref, got), (ref - got).abs().max()


@pytest.mark.parametrize("precision", ["fp32", "mixed"])
def test_ahead_executor_matches_serial_schedule(precision):
    """clskd.graph.AheadStepExecutor: two captures in the teacher_ahead layout replayed
    alternately by the C++ executor, each one's teacher stream waiting for the end of its own
    previous replay instead of the fork (clskd_exec_launch_ahead) — bitwise the per-step losses
    (all 16 slots) and the student waveforms of the eager step-by-step schedule over five
    back-to-back steps on distinct resident batches, and the same BatchNorm running statistics
    afterwards (teacher and student, one update per step each)."""
    from clskd.data import synthetic_pairs
    from clskd.graph import AheadStepExecutor
    batches = []
    for k in range(5):
        n, c = synthetic_pairs(4, 16000, seed=170 + k)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))

    def slots(o):
        return torch.cat([o["loss"].reshape(1), o["sc"].reshape(1), o["base"].reshape(1),
                          o["spkd"].reshape(-1)]).clone()

    kd_e, kd_x = _kd().set_precision(precision), _kd().set_precision(precision)
    ref, ref_w = [], []
    with torch.no_grad():
        for b in batches:
            o = kd_e.training_step(b, 0, return_parts=True)
            ref.append(slots(o))
            ref_w.append(o["student_wav"].clone())
    ex = AheadStepExecutor(kd_x, *batches[0])
    got, got_w = [], []
    for b in batches:
        ex(*b)
        got.append(slots(ex.out))
        got_w.append(ex.out["student_wav"].clone())
    torch.cuda.synchronize()
    assert torch.equal(torch.stack(ref), torch.stack(got)), (torch.stack(ref) - torch.stack(got)).abs().max()
    assert all(torch.equal(a, b) for a, b in zip(ref_w, got_w))
    for (k, a), b in zip(kd_e.state_dict().items(), kd_x.state_dict().values()):
        if "running" in k or "num_batches" in k:
            assert torch.equal(a, b), k


def test_teacher_ahead_toggled_between_steps():
    """switching teacher_ahead on and off between back-to-back steps with no
    synchronize in between.  A step after a non-ahead step must not run its teacher ahead (the
    earlier step's tensors were not held), and the losses stay those of the serial schedule."""
    from clskd.data import synthetic_pairs
    kd = _kd()
    kd.set_precision("mixed")
    batches = []
    for k in range(7):
        n, c = synthetic_pairs(4, 16000, seed=90 + k)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))
    torch.cuda.synchronize()

    def run(pattern):
        outs = []
        with torch.no_grad():
            for b, ahead in zip(batches, pattern):
                kd.teacher_ahead = ahead
                o = kd.training_step(b, 0, return_parts=True)
                outs.append(torch.cat([o["loss"].reshape(1), o["spkd"].reshape(-1)]).clone())
        torch.cuda.synchronize()
        kd.teacher_ahead = False
        return torch.stack(outs).cpu()

    ref = run([False] * 7)
    got = run([False, True, True, False, True, True, True])
    assert torch.equal(ref, got), (ref - got).abs().max()
    # a non-fp32 input cannot run ahead (its conversion would be queued on the caller's stream)
    kd.teacher_ahead = True
    with torch.no_grad():
        for b in batches[:3]:
            kd.training_step(b, 0)
        with pytest.raises(ValueError):
            kd.training_step((batches[0][0].double(), batches[0][1]), 0)
    torch.cuda.synchronize()
    kd.teacher_ahead = False


def test_clskd_step_golden():
    fx = golden("clskd_step.npz")
    kd = _kd()
    X = torch.from_numpy(fx["x"]).to(DEV)
    y = torch.from_numpy(fx["y"]).to(DEV)
    out = kd.training_step((X, y), 0, return_parts=True)
    assert abs(out["base"].item() - float(fx["loss/base"])) < 2e-5
    np.testing.assert_allclose(_np(out["enc"]), fx["loss/enc"], rtol=2e-3, atol=1e-6)
    np.testing.assert_allclose(_np(out["dec"]), fx["loss/dec"], rtol=2e-3, atol=1e-6)
    assert abs(out["clstm_real"].item() - float(fx["loss/clstm_real"])) < 1e-5
    assert abs(out["clstm_img"].item() - float(fx["loss/clstm_img"])) < 1e-5
    assert abs(out["loss"].item() - float(fx["loss/total"])) < 5e-5
    for k, v in enumerate(out["s_enc"]):
        check_summary(f"s_enc{k}", _np(v.permute(0, 3, 1, 2)), fx, rtol=5e-4, atol=5e-5)
    for k, v in enumerate(out["s_dec"]):
        check_summary(f"s_dec{k}", _np(v.permute(0, 3, 1, 2)), fx, rtol=5e-4, atol=5e-5)
    assert rms(_np(out["student_wav"]), fx["student_wav"]) <= 1e-5


def test_spkd_output_step_golden():
    from clskd.distill import SPKDDistillation
    fx = golden("spkd_output_step.npz")
    kd = SPKDDistillation(_models("teacher").train(), _models("student").train()).to(DEV)
    out = kd.training_step((torch.from_numpy(fx["x"]).to(DEV), torch.from_numpy(fx["y"]).to(DEV)),
                           0, return_parts=True)
    assert abs(out["base"].item() - float(fx["loss/base"])) < 2e-5
    assert abs(out["spkd"].item() - float(fx["loss/spkd"])) <= 1e-3 * float(fx["loss/spkd"]) + 1e-8
    assert abs(out["loss"].item() - float(fx["loss/total"])) < 5e-5


def test_spkd_output_step_mixed_precision():
    """C4 as bench.py --spkd runs it: the teacher on bf16 MFMA operands (fp32 accumulate), the
    student fp32.  The base loss depends on the student only, so it stays at the fp32 golden;
    the SPKD term (teacher waveform Gram) within 2 % of the golden (bf16 operand rounding)."""
    from clskd.distill import SPKDDistillation
    fx = golden("spkd_output_step.npz")
    kd = SPKDDistillation(_models("teacher").train(), _models("student").train(),
                          precision="mixed").to(DEV)
    assert kd.teacher.compute == "bf16" and kd.student.compute == "fp32"
    out = kd.training_step((torch.from_numpy(fx["x"]).to(DEV), torch.from_numpy(fx["y"]).to(DEV)),
                           0, return_parts=True)
    assert abs(out["base"].item() - float(fx["loss/base"])) < 2e-5
    assert abs(out["spkd"].item() - float(fx["loss/spkd"])) <= 2e-2 * float(fx["loss/spkd"]) + 1e-6
    assert torch.isfinite(out["teacher_wav"]).all()


def test_clskd_step_4s_against_oracle():
    """Configuration-C2 clip length (4 s @ 16 kHz, T=643) at B=4: every loss term and the
    student waveform against the CPU oracle; SI-SNR of the enhanced waveform within 0.01 dB.
    The oracle's SPKD Grams are evaluated in fp64 here: at K ~ 2.6M the reference's own fp32
    matmul is ~1e-3 relative off the exact loss, while the HIP Gram (fp32 MFMA chains + fp64 slab
    sums) lands within ~1e-6 of it (tests/diag_spkd_precision.py)."""
    from clskd.data import synthetic_pairs
    from clskd.tools_for_loss import si_snr
    from oracle import ref_cpu as R
    noisy, clean = synthetic_pairs(4, 64000, seed=5)
    kd = _kd()
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    out = kd.training_step((X, y), 0, return_parts=True)
    with torch.no_grad():
        ref = R.clskd_step(_oracle_params("teacher"), _oracle_params("student"),
                           _oracle_params("abf"), torch.from_numpy(noisy), torch.from_numpy(clean),
                           gram_dtype=torch.float64)
    wav = _np(out["student_wav"])
    assert rms(wav, ref["student_wav"].numpy()) <= 1e-4
    s_hip = si_snr(out["student_wav"], y).item()
    s_ref = R.si_snr(ref["student_wav"], torch.from_numpy(clean)).item()
    assert abs(s_hip - s_ref) <= 0.01
    assert abs(out["base"].item() - ref["base"].item()) <= 1e-4 * abs(ref["base"].item())
    np.testing.assert_allclose(_np(out["enc"]), [v.item() for v in ref["enc"]], rtol=5e-5, atol=1e-8)
    np.testing.assert_allclose(_np(out["dec"]), [v.item() for v in ref["dec"]], rtol=5e-5, atol=1e-8)
    assert abs(out["clstm_real"].item() - ref["clstm_real"].item()) <= 5e-5 * ref["clstm_real"].item()
    assert abs(out["clstm_img"].item() - ref["clstm_img"].item()) <= 5e-5 * ref["clstm_img"].item()
    assert abs(out["loss"].item() - ref["total"].item()) <= 2e-5 * abs(ref["total"].item())


@pytest.mark.parametrize("B,L", [(3, 12345), (5, 4321)])
def test_clskd_step_ragged_against_oracle(B, L):
    """The CLSKD step (distill.py:72-148) at odd batch sizes and lengths that are not a whole
    number of hops, against the oracle with fp64 Grams: student waveform RMS <= 1e-4, base loss
    within 1e-4 relative, the 14 SPKD terms within 5e-5 relative (or 1e-8 absolute), the total
    within 2e-5.  (Batch 1 is not a reference case: distill.py:100-101 squeezes the batch axis
    away before the MRSTFT's torch.stft, which then raises on the transpose; the oracle follows.)"""
    from clskd.data import synthetic_pairs
    from oracle import ref_cpu as R
    noisy, clean = synthetic_pairs(B, L, seed=B * 7 + L)
    kd = _kd()
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    out = kd.training_step((X, y), 0, return_parts=True)
    with torch.no_grad():
        ref = R.clskd_step(_oracle_params("teacher"), _oracle_params("student"),
                           _oracle_params("abf"), torch.from_numpy(noisy), torch.from_numpy(clean),
                           gram_dtype=torch.float64)
    wav = _np(out["student_wav"])
    assert wav.shape == tuple(ref["student_wav"].shape)
    assert rms(wav, ref["student_wav"].numpy()) <= 1e-4
    assert abs(out["base"].item() - ref["base"].item()) <= 1e-4 * abs(ref["base"].item())
    np.testing.assert_allclose(_np(out["enc"]), [v.item() for v in ref["enc"]], rtol=5e-5, atol=1e-8)
    np.testing.assert_allclose(_np(out["dec"]), [v.item() for v in ref["dec"]], rtol=5e-5, atol=1e-8)
    assert abs(out["loss"].item() - ref["total"].item()) <= 2e-5 * abs(ref["total"].item())


def test_clskd_step_full_batch_properties():
    """B=16 x 4 s (the bench workload): finite loss, SPKD terms in [0, 4], bitwise-repeatable step,
    per-sample independence of the student waveform (a sample's output does not depend on the
    others except through BN batch statistics -> compare against a permuted batch)."""
    from clskd.data import synthetic_pairs
    noisy, clean = synthetic_pairs(16, 64000, seed=6)
    kd = _kd()
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    sd_t = {k: v.clone() for k, v in kd.teacher.state_dict().items()}
    sd_s = {k: v.clone() for k, v in kd.student.state_dict().items()}
    o1 = kd.training_step((X, y), 0, return_parts=True)
    l1, w1, s1 = o1["loss"].item(), o1["student_wav"].clone(), o1["spkd"].clone()
    kd.teacher.load_state_dict(sd_t)
    kd.student.load_state_dict(sd_s)
    o2 = kd.training_step((X, y), 0, return_parts=True)
    assert o2["loss"].item() == l1
    assert torch.equal(o2["student_wav"], w1)
    assert np.isfinite(l1) and torch.all(s1 >= 0) and torch.all(s1 <= 4)
    perm = torch.randperm(16, generator=torch.Generator().manual_seed(0)).to(DEV)
    kd.teacher.load_state_dict(sd_t)
    kd.student.load_state_dict(sd_s)
    o3 = kd.training_step((X[perm], y[perm]), 0, return_parts=True)
    # BN batch statistics are permutation invariant up to summation order
    assert rms(_np(o3["student_wav"]), _np(w1[perm])) <= 1e-5
    # SPKD Grams are permutation-equivariant -> loss invariant
    assert abs(o3["loss"].item() - l1) <= 1e-4 * abs(l1)


def test_clskd_step_mixed_precision():
    """precision='mixed' (bf16 MFMA operands for the teacher and ReviewKD GEMMs, the student's
    fp32 convs on 3 x bf16 split products): the student waveform within RMS 1e-5 and SI-SNR
    1e-3 dB of the exact fp32 step, the base loss within 1e-5 relative; with the student held on
    the exact engines (compute 'fp32') it is untouched bitwise; SPKD terms within 2 % of the
    fp32 step."""
    from clskd.tools_for_loss import si_snr
    from clskd.data import synthetic_pairs
    noisy, clean = synthetic_pairs(4, 64000, seed=5)
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    kd = _kd()
    sd_t = {k: v.clone() for k, v in kd.teacher.state_dict().items()}
    sd_s = {k: v.clone() for k, v in kd.student.state_dict().items()}
    ref = kd.training_step((X, y), 0, return_parts=True)
    r_spkd, r_wav, r_base = _np(ref["spkd"]), ref["student_wav"].clone(), ref["base"].item()
    kd.teacher.load_state_dict(sd_t)
    kd.student.load_state_dict(sd_s)
    kd.set_precision("mixed")
    assert kd.student.compute == "f32x3"
    out = kd.training_step((X, y), 0, return_parts=True)
    wr = rms(_np(out["student_wav"]), _np(r_wav))
    ds = abs(si_snr(out["student_wav"], y).item() - si_snr(r_wav, y).item())
    print(f"split-product student: waveform RMS {wr:.2e}, SI-SNR delta {ds:.2e} dB")
    assert wr <= 1e-5 and ds <= 1e-3
    assert abs(out["base"].item() - r_base) <= 1e-5 * abs(r_base)
    kd.teacher.load_state_dict(sd_t)
    kd.student.load_state_dict(sd_s)
    kd.student.compute = "fp32"  # the exact engines: the student is untouched bitwise
    exact = kd.training_step((X, y), 0, return_parts=True)
    assert torch.equal(exact["student_wav"], r_wav)
    assert exact["base"].item() == r_base
    rel = np.abs(_np(out["spkd"]) - r_spkd) / r_spkd
    print("mixed-precision SPKD relative deviation per term:",
          " ".join(f"{v:.1e}" for v in rel), "total", out["loss"].item(), ref["loss"].item())
    assert rel.max() <= 2e-2, rel
    assert abs(out["loss"].item() - ref["loss"].item()) <= 2e-3 * ref["loss"].item()


@pytest.mark.parametrize("launch", ["graph", "exec"])
def test_step_graph_matches_eager(launch):
    """clskd.graph.StepGraph (hipGraph capture of the whole step, four streams; replayed by
    hipGraphLaunch) and clskd.graph.StepExecutor (the same capture replayed by the library's C++
    multi-stream executor, clskd_exec_launch) reproduce bitwise what the eager step computes:
    loss, SPKD terms, student waveform and BN running statistics, over two different batches; a
    changed student parameter triggers a re-capture."""
    from clskd.data import synthetic_pairs
    from clskd.graph import StepExecutor, StepGraph
    batches = []
    for seed in (11, 12, 13):
        n, c = synthetic_pairs(4, 32000, seed=seed)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))
    kd_e, kd_g = _kd().set_precision("mixed"), _kd().set_precision("mixed")
    ref = []
    for X, y in batches[:2]:
        o = kd_e.training_step((X, y), 0, return_parts=True)
        ref.append((o["loss"].item(), o["spkd"].clone(), o["student_wav"].clone()))
    g = (StepGraph if launch == "graph" else StepExecutor)(kd_g, *batches[0])
    if launch == "exec":
        print("executor:", g.info)
        assert g.info["kernels"] > 100 and sum(g.info["per_stream"]) == g.info["nodes"] - g.info["empty"]
        assert min(g.info["per_stream"]) > 0  # the branches run on all four streams
    for (X, y), (l, sp, wav) in zip(batches[:2], ref):
        assert g(X, y).item() == l
        assert torch.equal(g.out["spkd"], sp)
        assert torch.equal(g.out["student_wav"], wav)
    for (k, a), b in zip(kd_e.state_dict().items(), kd_g.state_dict().values()):
        assert torch.equal(a, b), k
    with torch.no_grad():
        for kd in (kd_e, kd_g):
            kd.student.encoder[0][0].real_conv.weight.mul_(1.01)
    X, y = batches[2]
    # return_parts: the no-tape step the graph captured (without it, grad mode routes through
    # autograd's taped step, whose student runs the exact engines, not the split products)
    l3 = kd_e.training_step((X, y), 0, return_parts=True)["loss"].item()
    assert g(X, y).item() == l3 and g.captures == 2


@pytest.mark.parametrize("launch", ["graph", "exec"])
def test_step_graph_redraws_abf_each_replay(launch):
    """abf_reinit='step': the ABF re-initialisation (kaiming_uniform, framework.py:194-195) is
    recorded into the graph and re-drawn on every replay (graph-safe Philox offsets): SPKD
    ReviewKD terms change between replays of the same batch while the student waveform and the
    clstm terms (no ABF on their path) do not."""
    from clskd.data import synthetic_pairs
    from clskd.distill import KnowledgeDistillation
    from clskd.graph import StepExecutor, StepGraph
    n, c = synthetic_pairs(4, 32000, seed=21)
    X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
    kd = KnowledgeDistillation(_models("teacher").train(), _models("student").train(),
                               abf_reinit="step", precision="mixed").to(DEV)
    g = (StepGraph if launch == "graph" else StepExecutor)(kd, X, y)
    outs = []
    for _ in range(2):
        g(X, y)
        outs.append({k: g.out[k].clone() for k in ("spkd", "student_wav", "loss")})
    assert torch.isfinite(outs[0]["loss"]) and torch.isfinite(outs[1]["loss"])
    assert torch.equal(outs[0]["student_wav"], outs[1]["student_wav"])
    assert torch.equal(outs[0]["spkd"][12:], outs[1]["spkd"][12:])  # clstm real / imag
    assert not torch.equal(outs[0]["spkd"][:12], outs[1]["spkd"][:12])


def test_abf_redraw_kernel():
    """clskd_uniform_redraw (the per-step ABF rebuild, framework.py:179-195): every ABF weight
    lies in its kaiming-uniform bound and is spread like U(-b, b); the packed MFMA operands hold
    exactly the drawn parameters (bf16 RNE / fp32) so no repack is needed; two draws differ;
    the draw counter advances in device memory (one launch per ReviewKD module)."""
    import math
    from clskd import ops
    from clskd.distill import KnowledgeDistillation
    from clskd.data import synthetic_pairs
    n, c = synthetic_pairs(2, 16000, seed=5)
    X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
    kd = KnowledgeDistillation(_models("teacher").train(), _models("student").train(),
                               abf_reinit="step", precision="mixed").to(DEV)
    kd.training_step((X, y))  # builds the packed operands; the next draws target them
    kd._reinit_abf(None)
    torch.cuda.synchronize()
    snap = {}
    for name, rk in (("encoder", kd.review_encoder), ("decoder", kd.review_decoder)):
        assert int(kd._draw_state[(name, X.device)][0]) == 2
        for i, abf in enumerate(rk.abfs):
            for j, (w, wp, cin, ntap, bound) in enumerate(abf.redraw_jobs()):
                v = w.detach().float().reshape(-1)
                assert float(v.abs().max()) <= bound * (1 + 1e-6)
                if v.numel() >= 4096:  # uniform: mean ~ 0, var ~ b^2 / 3
                    assert abs(float(v.mean())) < 0.05 * bound
                    assert abs(float(v.var()) / (bound * bound / 3) - 1) < 0.05
                if wp is not None:
                    ref = ops.pack_weight(w.detach().reshape(w.shape[0], w.shape[1], ntap)
                                          .permute(0, 2, 1), cin * ntap,
                                          "bf16" if wp.dtype == torch.bfloat16 else "fp32")
                    assert torch.equal(ref, wp), (name, i, j)
                snap[(name, i, j)] = v.clone()
    # the caches see the draw as current: a forward uses the drawn weights without repacking
    w1p_before = kd.review_decoder.abfs[0]._wcache["w"][1][0]
    kd.training_step((X, y))
    assert kd.review_decoder.abfs[0]._wcache["w"][1][0] is w1p_before
    for name, rk in (("encoder", kd.review_encoder), ("decoder", kd.review_decoder)):
        for i, abf in enumerate(rk.abfs):
            for j, (w, *_r) in enumerate(abf.redraw_jobs()):
                assert not torch.equal(snap[(name, i, j)], w.detach().float().reshape(-1))
    assert math.isfinite(float(kd.last["loss"]))


G8_CASES = {
    # name: (segment channels, N, taps, stride_f, Fi, Fo, of_mul, of_add, out_bf16)
    "enc5x2_n256": ((128,), 256, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 40, 20, 1, 0, True),
    "dec_parity0_n256": ((256, 256), 256, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1, 10, 10, 2, 0, True),
    "dec_parity1_n128": ((128, 128), 128, [(dF, -kt) for dF in (1, 0) for kt in (0, 1)], 1, 12, 12, 2, 1, False),
    "abf3x3_n128": ((64,), 128, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 16, 16, 1, 0, True),
    "pw_k64_nk1_n256": ((64,), 200, [(0, 0)], 1, 9, 9, 1, 0, False),
    "pw_k128_nk2_n128": ((128,), 128, [(0, 0)], 1, 9, 9, 1, 0, True),
    "pw_k192_nk3_n256": ((192,), 256, [(0, 0)], 1, 9, 9, 1, 0, True),
    "enc5x2_fo4_n256": ((128,), 256, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 8, 4, 1, 0, True),
    "abf3x3_n200": ((64,), 200, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 16, 16, 1, 0, False),
    # K-tiles straddle taps (96 channels per tap): the per-chunk gather, never tap-addressed
    "enc5x2_c96_n256": ((96,), 256, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 40, 20, 1, 0, True),
}


@pytest.mark.parametrize("engine", ["gemm8", "gemm8-noTA", "halow"])
@pytest.mark.parametrize("lp", ["bf16", "fp16"])
@pytest.mark.parametrize("case", sorted(G8_CASES))
def test_conv_gemm8_against_torch(case, lp, engine, loop="phased"):
    """The wide-layer bf16 engines (N > 64), each forced in turn (CLSKD_HALOW):
    engine="gemm8": the phase-interleaved 8-wave implicit GEMM (conv_gemm8.hip) — im2col 5x2
    stride-2, two-segment polyphase decoder layers with an interleaved output map, ABF 3x3, and
    pointwise layers with 1-3 K-tiles (pipeline prologue/drain edge cases);
    engine="halow" (experiments library only, CLSKD_LIB=exp: measured slower):
    the halo-tiled kernel with streamed weight slabs (conv_halow.hip) on every
    tap-structured case (8x32 tiles, 4x64 tiles at Fo = 4, N not a multiple of 32);
    fused BN statistics, M not a tile multiple; vs torch fp64 on the same bf16 operands.
    Tolerance 1e-4 relative (fp32 out) / 8e-3 (bf16 out); statistics 1e-5.  loop="pingpong"
    (CLSKD_G8_PP=1, bf16 operands): the ping-pong K loop of the experiments build (CLSKD_LIB=exp;
    not in the product library)."""
    from clskd import _lib, ops
    if loop == "pingpong" and lp == "fp16":
        pytest.skip("the ping-pong K loop is built for bf16 operands")
    segc, N, taps, sf, Fi, Fo, of_mul, of_add, out_bf16 = G8_CASES[case]
    if engine == "halow" and not _lib.experiments():
        pytest.skip("conv_halow is in the experiments library only (CLSKD_LIB=exp)")
    if engine == "halow" and (len(taps) < 3 or loop == "pingpong"):
        pytest.skip("conv_halow takes tap-structured layers (>= 3 taps)")
    if engine == "halow" and not out_bf16:
        pytest.skip("conv_halow stages 32x32 output tiles in a halo buffer: fp32 outputs need "
                    "a 32 KB halo (these cases' halos are smaller; they stay on conv_gemm8)")
    g = torch.Generator().manual_seed(len(case) * 13 + N)
    B, T = 3, 97
    segs_h = [torch.randn(B, Fi, T, c, generator=g).to(_LP[lp]) for c in segc]
    Cin = sum(segc)
    K = len(taps) * Cin
    w = torch.randn(N, len(taps), Cin, generator=g) * (0.5 / K ** 0.5)
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.to(DEV), K, lp)
    wq = wp[:, :K].float().cpu().double().view(N, len(taps), Cin)
    x = torch.cat([s.double() for s in segs_h], 3)
    ref = bias.double().view(1, 1, 1, N).expand(B, Fo, T, N).clone()
    for ti, (dF, dT) in enumerate(taps):
        fi = torch.arange(Fo) * sf + dF
        tt = torch.arange(T) + dT
        vf = (fi >= 0) & (fi < Fi)
        vt = (tt >= 0) & (tt < T)
        sub = torch.zeros(B, Fo, T, Cin, dtype=torch.float64)
        sub[:, vf.nonzero()[:, 0][:, None], vt.nonzero()[:, 0][None, :]] = \
            x[:, fi[vf][:, None], tt[vt][None, :]]
        ref += torch.einsum("bftc,nc->bftn", sub, wq[:, ti])
    Fout = Fo * of_mul
    out = torch.zeros(B, Fout, T, N, device=DEV, dtype=_LP[lp] if out_bf16 else torch.float32)
    nblk = ops.conv_mblocks(B, Fo, T)
    st = torch.full((nblk * N * 2,), float("nan"), device=DEV, dtype=torch.float64)
    prev = _lib.set_knob("CLSKD_G8_PP", int(loop == "pingpong"))
    prev_hw = _lib.set_knob("CLSKD_HALOW", int(engine == "halow")) if _lib.experiments() else 0
    prev_ta = _lib.set_knob("CLSKD_G8_TA", int(engine != "gemm8-noTA"))
    try:
        ops.conv([ops.seg_bftc(s.to(DEV)) for s in segs_h], taps, B, Fo, T, N, wp, bias.to(DEV),
                 out, ops.OutMap(Fout * T * N, T * N, N, of_mul=of_mul, of_add=of_add),
                 stride_f=sf, stats=st)
        kname = ops.conv_kernel_of_last_launch()
    finally:
        _lib.set_knob("CLSKD_G8_PP", prev)
        if _lib.experiments():
            _lib.set_knob("CLSKD_HALOW", prev_hw)
        _lib.set_knob("CLSKD_G8_TA", prev_ta)
    prefix = "conv_halow" if engine == "halow" else "conv_gemm8"
    assert kname.startswith(prefix) and ((",f16" in kname) == (lp == "fp16")), kname
    assert (",pp" in kname) == (loop == "pingpong"), kname
    # tap-addressed pieces: every 64-deep K-tile inside one tap and segment
    ta = (engine == "gemm8" and loop != "pingpong" and sum(segc) % 64 == 0
          and all(c % 64 == 0 for c in segc[:-1]))
    if engine != "halow":  # TA instances carry every template argument: ...,InT,PP,TA>
        assert bool(re.search(r",(bf16|f16),0,[13]>$", kname)) == ta, kname
    o = out.double().cpu()[:, of_add::of_mul]
    tol = _LP_TOL[lp] if out_bf16 else 1e-4
    np.testing.assert_allclose(o.numpy(), ref.numpy(), rtol=tol, atol=tol)
    if of_mul > 1:
        assert torch.all(out.double().cpu()[:, (of_add + 1) % of_mul::of_mul] == 0)
    stc = st.view(nblk, N, 2).cpu()
    assert torch.isfinite(stc).all(), "every statistics slot must be written"
    np.testing.assert_allclose(stc[:, :, 0].sum(0).numpy(), ref.sum((0, 1, 2)).numpy(), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(stc[:, :, 1].sum(0).numpy(), (ref ** 2).sum((0, 1, 2)).numpy(), rtol=1e-5)



@pytest.mark.parametrize("prio", [0, 1])
@pytest.mark.parametrize("variant", ["1", "8", "h128"])
def test_lstm_recurrence_against_torch(variant, prio):
    """Complex-LSTM recurrence (tools_for_model.py:159-174, nn.LSTM gates i, f, g, o, zero
    state) at the student's H = 32 — the single-wave kernel (CLSKD_LSTM_NKS32=1, default) and the
    8-slice multi-wave kernel — and the teacher's H = 128, each with and without the issue
    priority (CLSKD_LSTM_PRIO), vs a torch fp64 recurrence on the same gate inputs.  Tolerance
    2e-5 (v_exp / v_rcp gate activations, fp32 state)."""
    from clskd import _lib
    prev = _lib.set_knob("CLSKD_LSTM_NKS32", 1 if variant == "h128" else int(variant))
    prev_p = _lib.set_knob("CLSKD_LSTM_PRIO", prio)
    try:
        _lstm_recurrence_check(128 if variant == "h128" else 32)
    finally:
        _lib.set_knob("CLSKD_LSTM_NKS32", prev)
        _lib.set_knob("CLSKD_LSTM_PRIO", prev_p)


def _lstm_recurrence_check(H=32):
    from clskd import ops
    g = torch.Generator().manual_seed(3)
    nws, nseq, T = 2, 5, 37
    gx = torch.randn(nseq, T, nws * 4 * H, generator=g)
    whh = torch.randn(nws, 4 * H, H, generator=g) * (0.2 * (32 / H) ** 0.5)
    out = torch.empty(nws, nseq, T, H, device=DEV)
    ops.lstm_recurrent(gx.to(DEV), 4 * H, T * nws * 4 * H, nws * 4 * H, whh.to(DEV), nws, nseq, T, H,
                       out, nseq * T * H, T * H, H)
    ref = torch.empty(nws, nseq, T, H, dtype=torch.float64)
    for ws in range(nws):
        W = whh[ws].double()
        h = torch.zeros(nseq, H, dtype=torch.float64)
        c = torch.zeros(nseq, H, dtype=torch.float64)
        for t in range(T):
            z = gx[:, t, ws * 4 * H:(ws + 1) * 4 * H].double() + h @ W.t()
            i, f, gg, o = z.split(H, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
            ref[ws, :, t] = h
    np.testing.assert_allclose(out.double().cpu().numpy(), ref.numpy(), rtol=2e-5, atol=2e-5)


def _sk_expected(ntiles, nk, grid, force=False):
    """conv_gemm8's stream-K rule (launch_g8): a partial last round and a gain of more than the
    hand-off cost (12 K-tiles); CLSKD_G8_SK=2 forces it wherever the deal splits."""
    return (grid >= 8 and grid % 8 == 0 and ntiles >= grid and ntiles % grid != 0
            and (force or -(-ntiles * nk // grid) + 12 < -(-ntiles // grid) * nk))


@pytest.mark.parametrize("grid", [40, 64])
@pytest.mark.parametrize("lp", ["bf16", "fp16"])
@pytest.mark.parametrize("case", ["enc5x2_n256", "dec_parity1_n128", "abf3x3_n200"])
def test_conv_gemm8_stream_k(case, lp, grid):
    """Stream-K deal of conv_gemm8 (round 5): the K-tile units of all tiles split evenly over a
    persistent grid (capped here with CLSKD_G8_GRID so a small layer has a partial last round),
    a tile shared by two workgroups finished by the later arrival with the earlier one's fp32
    partial.  Against torch fp64 (outputs and fused statistics, the G8 tolerances), against the
    data-parallel deal (CLSKD_G8_SK=0: the K sums only regroup, fp32 rounding), and bitwise
    repeatable (a commutative add: arrival order does not matter)."""
    from clskd import _lib, ops
    segc, N, taps, sf, Fi, Fo, of_mul, of_add, out_bf16 = G8_CASES[case]
    g = torch.Generator().manual_seed(7 + grid)
    B, T = 4, 301
    segs_h = [torch.randn(B, Fi, T, c, generator=g).to(_LP[lp]) for c in segc]
    Cin = sum(segc)
    K = len(taps) * Cin
    w = torch.randn(N, len(taps), Cin, generator=g) * (0.5 / K ** 0.5)
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.to(DEV), K, lp)
    wq = wp[:, :K].float().cpu().double().view(N, len(taps), Cin)
    x = torch.cat([s.double() for s in segs_h], 3)
    ref = bias.double().view(1, 1, 1, N).expand(B, Fo, T, N).clone()
    for ti, (dF, dT) in enumerate(taps):
        fi = torch.arange(Fo) * sf + dF
        tt = torch.arange(T) + dT
        vf = (fi >= 0) & (fi < Fi)
        vt = (tt >= 0) & (tt < T)
        sub = torch.zeros(B, Fo, T, Cin, dtype=torch.float64)
        sub[:, vf.nonzero()[:, 0][:, None], vt.nonzero()[:, 0][None, :]] = \
            x[:, fi[vf][:, None], tt[vt][None, :]]
        ref += torch.einsum("bftc,nc->bftn", sub, wq[:, ti])
    Fout = Fo * of_mul
    segs = [ops.seg_bftc(s.to(DEV)) for s in segs_h]
    nblk = ops.conv_mblocks(B, Fo, T)
    bn = 256 if N > 128 else 128
    ntiles = -(-(B * Fo * T) // 256) * -(-N // bn)
    expect_sk = _sk_expected(ntiles, K // 64, grid, force=True)

    def run(sk):
        out = torch.zeros(B, Fout, T, N, device=DEV, dtype=_LP[lp] if out_bf16 else torch.float32)
        st = torch.full((nblk * N * 2,), float("nan"), device=DEV, dtype=torch.float64)
        prev_sk = _lib.set_knob("CLSKD_G8_SK", 2 if sk else 0)  # 2: split even where not paying
        prev_g = _lib.set_g8_grid(grid)
        try:
            ops.conv(segs, taps, B, Fo, T, N, wp, bias.to(DEV), out,
                     ops.OutMap(Fout * T * N, T * N, N, of_mul=of_mul, of_add=of_add),
                     stride_f=sf, stats=st)
            used = ops.conv_last_stream_k()
        finally:
            _lib.set_knob("CLSKD_G8_SK", prev_sk)
            _lib.set_g8_grid(prev_g)
        torch.cuda.synchronize()
        return out, st, used

    o1, s1, used = run(True)
    assert used == expect_sk, (ntiles, K // 64, grid)
    o2, s2, _ = run(True)
    assert torch.equal(o1, o2) and torch.equal(s1, s2), "stream-K must be bitwise repeatable"
    o0, s0, used0 = run(False)
    assert not used0
    o = o1.double().cpu()[:, of_add::of_mul]
    tol = _LP_TOL[lp] if out_bf16 else 1e-4
    np.testing.assert_allclose(o.numpy(), ref.numpy(), rtol=tol, atol=tol)
    if not out_bf16:  # fp32 outputs: only the K-sum grouping differs from the data-parallel deal
        np.testing.assert_allclose(o1.cpu().numpy(), o0.cpu().numpy(), rtol=1e-5, atol=1e-5)
    stc = s1.view(nblk, N, 2).cpu()
    assert torch.isfinite(stc).all(), "every statistics slot must be written"
    np.testing.assert_allclose(stc[:, :, 0].sum(0).numpy(), ref.sum((0, 1, 2)).numpy(), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(stc[:, :, 1].sum(0).numpy(), (ref ** 2).sum((0, 1, 2)).numpy(), rtol=1e-5)
