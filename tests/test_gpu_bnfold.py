"""Folded BatchNorm finalize (clskd_bn_fold, round 4): a conv launch whose kernel is one of the
persistent engines (conv_gemm8, conv_halo, conv_halo_f32) turns its output's train-mode batch
statistics into the BatchNorm coefficients itself — fixed-point limb accumulators, a last-arriver
ticket — instead of writing per-block partials for a clskd_bn_finalize launch.

Checked against fp64 torch on the same operands: the batch mean / biased variance, the
coefficients scale = gamma / sqrt(var + eps) and shift = beta - mean * scale, and the running
statistics after two updates (nn.BatchNorm2d train forward, momentum 0.1, unbiased variance);
bitwise repeatability; the device state returned to zero; and the layer spread over two launches
(the decoder's polyphase parities) with only the last one finalizing."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _conv_case(kind, N, dt, g):
    """(segments, taps, geometry, packed weight, bias, torch fp64 reference [B, N, Fo, To])."""
    from clskd import ops
    # sizes the persistent kernels take (conv_halo needs >= 32 tiles of 8 x 32 outputs)
    B, T = 4, 128
    if kind == "enc":  # 5x2 stride-(2,1), the encoder blocks (fp32: the student's enc2 / enc3)
        if dt == "bf16":
            F, Cin = (128, 32) if N == 64 else (34, 64)  # teacher enc1 (halo) / gemm8 shapes
        else:
            F, Cin = (64, 16) if N == 32 else (32, 32)
        taps = [(kf - 2, kt - 1) for kf in range(5) for kt in range(2)]
        Fo, sf = (F + 4 - 5) // 2 + 1, 2
    else:  # 3x3, the ABF conv2
        F, Cin = 40, 64
        taps = [(kf - 1, kt - 1) for kf in range(3) for kt in range(3)]
        Fo, sf = F, 1
    tdt = torch.bfloat16 if dt == "bf16" else torch.float32
    x = (torch.randn(B, F, T, Cin, generator=g) + 0.3).to(tdt)
    kh = 5 if kind == "enc" else 3
    kw = 2 if kind == "enc" else 3
    w = torch.randn(N, Cin, kh, kw, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    wp = ops.pack_weight(w.permute(0, 2, 3, 1).reshape(N, kh * kw, Cin).to(DEV), kh * kw * Cin,
                         dt)
    wq = wp[:, :kh * kw * Cin].float().cpu().reshape(N, kh, kw, Cin).permute(0, 3, 1, 2).double()
    xin = x.double().permute(0, 3, 1, 2)
    if kind == "enc":
        ref = torch.nn.functional.conv2d(torch.nn.functional.pad(xin, (1, 0, 2, 2)), wq,
                                         bias.double(), stride=(2, 1))[..., :T]
    else:
        ref = torch.nn.functional.conv2d(xin, wq, bias.double(), padding=1)
    return x, taps, (B, Fo, T, sf), wp, bias, ref


def _bn(N, g):
    bn = torch.nn.BatchNorm2d(N)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(N, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(N, generator=g))
        bn.running_mean.copy_(torch.randn(N, generator=g) * 0.1)
        bn.running_var.copy_(torch.rand(N, generator=g) + 0.5)
    return bn


@pytest.mark.parametrize("kind,N,dt,grid", [("enc", 64, "bf16", 0), ("enc", 128, "bf16", 0),
                                            ("enc", 256, "bf16", 0), ("abf", 32, "bf16", 0),
                                            ("enc", 64, "f32", 0), ("enc", 32, "f32", 0),
                                            ("enc", 256, "bf16", 16), ("enc", 128, "bf16", 24)])
def test_bn_fold_against_torch(kind, N, dt, grid):
    """grid > 0: conv_gemm8 on a capped persistent grid, where its stream-K deal splits tiles
    between workgroups (the finishing workgroup folds the tile's statistics)."""
    from clskd import _lib
    prev_g = _lib.set_g8_grid(grid)
    prev_sk = _lib.set_knob("CLSKD_G8_SK", 2 if grid else 1)  # 2: split even where not paying
    try:
        _bn_fold_check(kind, N, dt, grid)
    finally:
        _lib.set_g8_grid(prev_g)
        _lib.set_knob("CLSKD_G8_SK", prev_sk)


def _bn_fold_check(kind, N, dt, grid):
    from clskd import ops
    g = torch.Generator().manual_seed(N + (7 if dt == "f32" else 0) + (3 if kind == "abf" else 0))
    x, taps, (B, Fo, T, sf), wp, bias, ref = _conv_case(kind, N, dt, g)
    bn = _bn(N, g)
    rm0, rv0 = bn.running_mean.clone().double(), bn.running_var.clone().double()
    bnd = bn.to(DEV)
    out = torch.empty(B, Fo, T, N, device=DEV, dtype=x.dtype)
    mv = torch.empty(2, N, device=DEV)
    res = []
    for rep in range(2):
        with torch.no_grad():
            bnd.running_mean.copy_(rm0.float())
            bnd.running_var.copy_(rv0.float())
        st = ops.BnStats(bnd, N, B * Fo * T, 2, DEV, stats_out=(mv[0], mv[1]))
        ops.conv([ops.seg_bftc(x.to(DEV))], taps, B, Fo, T, N, wp, bias.to(DEV), out,
                 ops.OutMap(Fo * T * N, T * N, N), stride_f=sf, bn_stats=(st, True))
        assert ops.conv_last_stream_k() == (grid > 0), "stream-K expected on the capped grid"
        coef = st.coefficients().clone()
        torch.cuda.synchronize()
        assert st.mode == "fold", f"{kind} N={N} {dt} did not dispatch to a folding engine"
        res.append((coef.cpu(), mv.clone().cpu(), bnd.running_mean.clone().cpu(),
                    bnd.running_var.clone().cpu()))
    assert all(torch.equal(a, b) for a, b in zip(res[0], res[1])), "not bitwise repeatable"
    acc, ticket = ops.bn_fold_state(bnd, N, torch.device(DEV))
    assert int(acc.abs().sum()) == 0 and int(ticket.abs().sum()) == 0, "state not back at zero"
    coef, mvh, rm, rv = res[0]
    n = B * Fo * T
    mean = ref.mean((0, 2, 3))
    var = ref.var((0, 2, 3), unbiased=False)
    np.testing.assert_allclose(mvh[0].numpy(), mean.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(mvh[1].numpy(), var.numpy(), rtol=1e-4, atol=1e-6)
    gam, bet = bn.weight.detach().cpu().double(), bn.bias.detach().cpu().double()
    scale = gam / torch.sqrt(var + bn.eps)
    np.testing.assert_allclose(coef[:N].numpy(), scale.numpy(), rtol=1e-4)
    np.testing.assert_allclose(coef[N:].numpy(), (bet - mean * scale).numpy(), rtol=1e-4, atol=1e-4)
    erm, erv = rm0, rv0
    for _ in range(2):
        erm = 0.9 * erm + 0.1 * mean
        erv = 0.9 * erv + 0.1 * var * n / (n - 1)
    np.testing.assert_allclose(rm.numpy(), erm.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(rv.numpy(), erv.numpy(), rtol=1e-4, atol=1e-6)


def test_bn_fold_two_launch_layer_matches_model_decoder():
    """A DCCRN decoder block (two polyphase launches, one BatchNorm) with the fold against the
    same block run through partials + clskd_bn_finalize (the fp32 student's N = 64 layer on the
    halo kernel vs the engine path that cannot fold, CLSKD_NO_HALO32=1): coefficients and
    running statistics agree to fp32 rounding."""
    from clskd import _lib
    from clskd import config as cfg
    from clskd.data import synthetic_pairs
    from clskd.model import DCCRN
    from clskd.weights import STUDENT_SEED, apply_recipe
    noisy, _ = synthetic_pairs(2, 16000, seed=3)
    x = torch.from_numpy(noisy).to(DEV)
    outs = []
    for no_halo in (0, 1):
        m = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED).to(DEV)
        prev = _lib.set_knob("CLSKD_NO_HALO32", no_halo)
        try:
            res = m.run(x, train=True, bn_updates=2)
            torch.cuda.synchronize()
        finally:
            _lib.set_knob("CLSKD_NO_HALO32", prev)
        outs.append((res["out_wav"].cpu(), {k: v.cpu() for k, v in m.state_dict().items()
                                            if "running" in k}))
    (w0, s0), (w1, s1) = outs
    assert float((w0 - w1).abs().max()) <= 1e-5
    for k in s0:
        np.testing.assert_allclose(s0[k].numpy(), s1[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
