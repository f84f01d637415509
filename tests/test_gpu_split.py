"""fp32 layers on the bf16 MFMA pipe with 3 x bf16 split products (csrc/conv_split.hip,
CLSKD_F32_SPLIT=1): per-launch parity against torch fp64 with an error bound derived from the
split, the fused statistics and the folded BatchNorm finalize, and the student's fp32 goldens
(the reference-generated fixtures, at the exact path's bars) with the split on.

Error model (per product x*w, operands split hi = bf16(x), lo = bf16(x - hi)): the dropped
lo*wlo term and the residuals beyond the 16 kept mantissa bits are <= ~3 * 2^-18 |x w|, the
fp32 accumulation adds <= K * 2^-24 relative to sum |x w|.  Bound used: |out - ref| <=
2e-5 * (sum_k |x_k w_k| + |bias|) + 1e-7 per output element."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def split_on():
    from clskd import _lib
    prev = _lib.set_knob("CLSKD_F32_SPLIT", 1)
    yield
    _lib.set_knob("CLSKD_F32_SPLIT", prev)


def _ref(segs, taps, sf, Fo, T, wq, bias):
    """fp64 implicit GEMM over BFTC segments (same tap / padding semantics as clskd_conv2d_fwd)."""
    x = torch.cat([s.double() for s in segs], 3)
    B, Fi, _, Cin = x.shape
    N = wq.shape[0]
    out = bias.double().view(1, 1, 1, N).expand(B, Fo, T, N).clone()
    for ti, (dF, dT) in enumerate(taps):
        fi = torch.arange(Fo) * sf + dF
        tt = torch.arange(T) + dT
        vf = (fi >= 0) & (fi < Fi)
        vt = (tt >= 0) & (tt < T)
        sub = torch.zeros(B, Fo, T, Cin, dtype=torch.float64)
        sub[:, vf.nonzero()[:, 0][:, None], vt.nonzero()[:, 0][None, :]] = \
            x[:, fi[vf][:, None], tt[vt][None, :]]
        out += torch.einsum("bftc,nc->bftn", sub, wq[:, ti])
    return out


SPLIT_CASES = {
    # name: (segment channels, N, taps, stride_f, Fi, Fo, of_mul, of_add)
    "enc5x2_n32": ((16,), 32, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 33, 17, 1, 0),
    "enc5x2_n64": ((64,), 64, [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)], 2, 16, 8, 1, 0),
    "dec_parity1_n16": ((32, 32), 16, [(dF, -kt) for dF in (1, 0) for kt in (0, 1)], 1, 9, 9, 2, 1),
    "dec_parity0_n8": ((16, 16), 8, [(dF, -kt) for dF in (1, 0, -1) for kt in (0, 1)], 1, 9, 9, 2, 0),
    "framing_n514_k400": ((400,), 514, [(0, 0)], 1, 1, 1, 1, 0),
    "proj_n256_k32": ((32,), 256, [(0, 0)], 1, 1, 1, 1, 0),
    "abf3x3_n64": ((8,), 64, [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)], 1, 12, 12, 1, 0),
}


@pytest.mark.parametrize("bk", [0, 32, 16])
@pytest.mark.parametrize("case", sorted(SPLIT_CASES))
def test_split_conv_against_torch(case, bk, split_on):
    """Every K-tile depth the dispatch can pick (CLSKD_SPLIT_BK caps it: 0 = deepest K allows),
    routed by the global A/B knob CLSKD_F32_SPLIT=1."""
    from clskd import _lib
    prev_bk = _lib.set_knob("CLSKD_SPLIT_BK", bk)
    try:
        _split_case(case)
    finally:
        _lib.set_knob("CLSKD_SPLIT_BK", prev_bk)


@pytest.mark.parametrize("pd,grid,occ", [(1, 0, 0), (2, 0, 0), (2, 1, 0), (1, 1, 0), (2, 0, 1), (1, 1, 1)])
@pytest.mark.parametrize("case", sorted(SPLIT_CASES))
def test_split_conv_prefetch_depth(case, pd, grid, occ, split_on):
    """Gather prefetch depth (CLSKD_SPLIT_PD: 1 K-tile ahead — the default — or 2 wherever the
    K-tile count allows) with the grid capped to one CU (CLSKD_SPLIT_GRID=1): every workgroup walks
    many tiles, so the prefetch of K-tiles k + 1 / k + 2 crosses tile boundaries.  CLSKD_SPLIT_OCC
    1 (default) / 0: the grid of register-resident workgroups / of the LDS bound."""
    from clskd import _lib
    prev = {k: _lib.set_knob(k, v) for k, v in
            (("CLSKD_SPLIT_PD", pd), ("CLSKD_SPLIT_GRID", grid), ("CLSKD_SPLIT_OCC", occ))}
    try:
        _split_case(case)
    finally:
        for k, v in prev.items():
            _lib.set_knob(k, v)


@pytest.mark.parametrize("ns2,grid", [(0, 0), (1, 0), (1, 1), (2, 0)])
@pytest.mark.parametrize("case", sorted(SPLIT_CASES))
def test_split_conv_lds_stages(case, ns2, grid, split_on):
    """64-deep K-tiles on one LDS stage (CLSKD_SPLIT_NS2=0) or two (1, the default for the
    instances of one resident workgroup per CU), also with many tiles per workgroup."""
    from clskd import _lib
    prev = {k: _lib.set_knob(k, v) for k, v in (("CLSKD_SPLIT_NS2", ns2), ("CLSKD_SPLIT_GRID", grid))}
    try:
        _split_case(case)
    finally:
        for k, v in prev.items():
            _lib.set_knob(k, v)


@pytest.mark.parametrize("case", sorted(SPLIT_CASES))
def test_split_descriptor_against_torch(case):
    """The same layers asked for per descriptor (compute CLSKD_F32X3, ops.split_products: how the
    student of precision 'mixed' runs), the global knob off."""
    from clskd import ops
    with ops.split_products(True):
        _split_case(case)


def _split_case(case, accumulate=False):
    from clskd import ops
    segc, N, taps, sf, Fi, Fo, of_mul, of_add = SPLIT_CASES[case]
    g = torch.Generator().manual_seed(len(case) * 7 + N)
    B, T = (3, 701) if Fi == 1 else (3, 61)
    segs = [torch.randn(B, Fi, T, c, generator=g) * 1.7 + 0.2 for c in segc]
    Cin = sum(segc)
    K = len(taps) * Cin
    w = torch.randn(N, len(taps), Cin, generator=g) * (0.7 / K ** 0.5)
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.to(DEV), K)
    wq = wp[:, :K].cpu().double().view(N, len(taps), Cin)
    ref = _ref(segs, taps, sf, Fo, T, wq, bias)
    mag = _ref([s.abs() for s in segs], taps, sf, Fo, T, wq.abs(), bias.abs())
    Fout = Fo * of_mul
    prior = (torch.randn(B, Fout, T, N, generator=g) if accumulate else torch.zeros(B, Fout, T, N)).to(DEV)
    out = prior.clone()
    stats_on = N <= 128 and not accumulate
    nblk = ops.conv_mblocks(B, Fo, T)
    st = torch.full((nblk * N * 2,), float("nan"), device=DEV, dtype=torch.float64) if stats_on else None
    ops.conv([ops.seg_bftc(s.to(DEV)) for s in segs], taps, B, Fo, T, N, wp, bias.to(DEV), out,
             ops.OutMap(Fout * T * N, T * N, N, of_mul=of_mul, of_add=of_add), stride_f=sf, stats=st,
             accumulate=accumulate)
    kname = ops.conv_kernel_of_last_launch()
    if kname.startswith("conv_direct") or kname.startswith("conv_pointwise"):
        pytest.skip(f"{case}: dispatched to {kname} (not an MFMA layer)")
    assert kname.startswith("conv_split3_kernel"), kname
    o = (out.double() - prior.double()).cpu()[:, of_add::of_mul]
    err = (o - ref).abs()
    bound = 2e-5 * mag + 1e-7
    worst = float((err / bound).max())
    print(f"{case}: max err {float(err.max()):.2e}, worst err/bound {worst:.3f}, "
          f"median rel {float((err / mag.clamp_min(1e-30)).median()):.2e}")
    assert worst <= 1.0
    if of_mul > 1:
        other = slice((of_add + 1) % of_mul, None, of_mul)
        assert torch.equal(out.cpu()[:, other], prior.cpu()[:, other])
    if stats_on:
        stc = st.view(nblk, N, 2).cpu()
        assert torch.isfinite(stc).all(), "every statistics slot must be written"
        S, Q = stc[..., 0].sum(0), stc[..., 1].sum(0)
        np.testing.assert_allclose(S.numpy(), ref.sum((0, 1, 2)).numpy(), rtol=1e-5,
                                   atol=1e-5 * float(mag.sum((0, 1, 2)).max()))
        np.testing.assert_allclose(Q.numpy(), (ref * ref).sum((0, 1, 2)).numpy(), rtol=5e-5)


@pytest.mark.parametrize("case", sorted(SPLIT_CASES))
def test_split_conv_accumulate_against_torch(case):
    """accumulate=True (out += conv: the data-gradient sums of a split-product backward, config C3
    in precision 'mixed') on the split engine, asked for per descriptor: the increment against
    fp64 at the split bound, the other polyphase parity rows untouched."""
    from clskd import ops
    with ops.split_products(True):
        _split_case(case, accumulate=True)


def test_split_bn_fold_against_torch(split_on):
    """Folded finalize on the split kernel: batch mean / variance and coefficients vs fp64."""
    from clskd import ops
    g = torch.Generator().manual_seed(11)
    B, F, T, Cin, N = 4, 64, 128, 16, 32
    taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
    x = torch.randn(B, F, T, Cin, generator=g) + 0.3
    w = torch.randn(N, 10, Cin, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.to(DEV), 10 * Cin)
    Fo = (F - 1) // 2 + 1
    ref = _ref([x], taps, 2, Fo, T, wp.cpu().double().view(N, 10, Cin), bias)
    bn = torch.nn.BatchNorm2d(N).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(N, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(N, generator=g))
    mv = torch.empty(2, N, device=DEV)
    out = torch.empty(B, Fo, T, N, device=DEV)
    stt = ops.BnStats(bn, N, B * Fo * T, 1, DEV, stats_out=(mv[0], mv[1]))
    ops.conv([ops.seg_bftc(x.to(DEV))], taps, B, Fo, T, N, wp, bias.to(DEV), out,
             ops.OutMap(Fo * T * N, T * N, N), stride_f=2, bn_stats=(stt, True))
    coef = stt.coefficients().clone()
    torch.cuda.synchronize()
    assert stt.mode == "fold"
    assert ops.conv_kernel_of_last_launch().startswith("conv_split3_kernel")
    mean = ref.mean((0, 1, 2))
    var = ref.var((0, 1, 2), unbiased=False)
    np.testing.assert_allclose(mv[0].cpu().numpy(), mean.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(mv[1].cpu().numpy(), var.numpy(), rtol=1e-4, atol=1e-6)
    scale = bn.weight.detach().cpu().double() / torch.sqrt(var + bn.eps)
    np.testing.assert_allclose(coef[:N].cpu().numpy(), scale.numpy(), rtol=1e-4)
    acc, ticket = ops.bn_fold_state(bn, N, torch.device(DEV))
    assert int(acc.abs().sum()) == 0 and int(ticket.abs().sum()) == 0


# the student's fp32 goldens (reference-generated fixtures) at the exact path's own bars
def test_split_student_train_golden(split_on):
    import test_gpu_parity as P
    P.test_forward_train_golden("student")


def test_split_student_eval_golden_and_stft(split_on):
    """Eval forward golden at the exact path's bars; the ConvSTFT spectrum against the golden
    within the split's per-element bound (2e-5 * sum |x||w| + 1e-7: the spectrum's raw values
    reach ~1e2, so the exact path's fixed atol 2e-5 is below one split rounding of them)."""
    import test_gpu_parity as P
    from conftest import golden
    P.test_forward_eval_golden()
    st = golden("stft.npz")
    m = P._models("student")
    x = torch.from_numpy(st["x"]).to(DEV)
    spec = m.spectrum(x).permute(0, 2, 1).double().cpu()
    ref = torch.from_numpy(st["spec"]).double()
    w = m.stft.weight.detach().double().cpu().abs()  # [514, 1, 400]
    xp = torch.nn.functional.pad(torch.from_numpy(st["x"]).double().abs()[:, None], (300, 300))
    mag = torch.nn.functional.conv1d(xp, w, stride=100)[..., :ref.shape[-1]]
    assert mag.shape == ref.shape, (mag.shape, ref.shape)
    worst = float(((spec - ref).abs() / (2e-5 * mag + 1e-7)).max())
    print(f"stft: max |diff| {float((spec - ref).abs().max()):.2e}, worst diff/bound {worst:.3f}")
    assert worst <= 1.0


@pytest.mark.parametrize("B,L", [(1, 16037), (3, 401)])
def test_split_student_ragged_against_oracle(B, L, split_on):
    import test_gpu_parity as P
    P.test_forward_ragged_lengths_against_oracle("student", B, L, True)
