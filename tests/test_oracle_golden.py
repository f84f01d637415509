"""Pins the CPU oracle (oracle/ref_cpu.py) against fixtures produced by the reference itself.

Runs on CPU (no GPU marker).  Tolerances: fp32 re-expression of the same ops, so agreement is at
fp32 rounding level (1e-5 relative on outputs; 1e-6 absolute on losses).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, check_summary, golden
from oracle import ref_cpu as R
from clskd import config as cfg
from clskd.weights import (ABF_SEED, STUDENT_SEED, TEACHER_SEED, recipe_state_dict)

torch.set_num_threads(min(8, os.cpu_count() or 1))


def params(kind):
    if kind == "teacher":
        shapes = cfg.dccrn_param_shapes(**cfg.TEACHER)
        return R.to_torch_params(recipe_state_dict(shapes, TEACHER_SEED))
    if kind == "student":
        shapes = cfg.dccrn_param_shapes(**cfg.STUDENT)
        return R.to_torch_params(recipe_state_dict(shapes, STUDENT_SEED))
    shapes = {**cfg.review_param_shapes("encoder"), **cfg.review_param_shapes("decoder")}
    return R.to_torch_params(recipe_state_dict(shapes, ABF_SEED))


def test_param_keys_match_reference():
    keys = json.load(open(os.path.join(GOLDEN, "param_keys.json")))
    for kind, spec in (("teacher", cfg.TEACHER), ("student", cfg.STUDENT)):
        ref = {k: tuple(v) for k, v in keys[kind].items() if not k.startswith(("stft.", "istft."))}
        ours = {k: tuple(v) for k, v in cfg.dccrn_param_shapes(**spec).items()}
        assert ours == ref
        assert list(ours) == list(ref)  # same order as the reference state_dict
    for ft in ("encoder", "decoder"):
        ref = {k: tuple(v) for k, v in keys[f"review_{ft}"].items()}
        assert dict(cfg.review_param_shapes(ft)) == ref


def test_sisnr_known_answers():
    k = golden("kat_sisnr.npz")
    ref = torch.from_numpy(k["reference"])
    for name in ("flip", "ref_plus_flip", "ref_plus_half", "two_ref_plus_one"):
        est = torch.from_numpy(k[f"est/{name}"])
        assert abs(R.si_snr(est, ref).item() - float(k[f"si_snr/{name}"])) < 1e-9
        # tools_for_loss.py:60-77 docstring values, to the eps-induced 3e-5 dB
        assert abs(R.si_snr(est, ref).item() - float(k[f"doc/si_sdr/{name}"])) < 5e-5
    v = R.si_snr(torch.from_numpy(k["rand/s1"]), torch.from_numpy(k["rand/s2"])).item()
    assert abs(v - float(k["rand/si_snr"])) < 1e-5


def test_sisnr_shipped_examples():
    ex = golden("examples.npz")
    for e in ["606", "1038", "1132", "1431", "2158"]:
        s0 = torch.from_numpy(ex[f"{e}/s0"] / 32768.0).float()
        est = torch.from_numpy(ex[f"{e}/est"] / 32768.0).float()
        assert abs(R.si_snr(est, s0).item() - float(ex[f"{e}/si_snr"])) < 1e-5


def test_stft_istft():
    st = golden("stft.npz")
    x = torch.from_numpy(st["x"])
    spec = R.conv_stft(x)
    np.testing.assert_allclose(spec.numpy(), st["spec"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(R.conv_istft(spec).numpy(), st["istft"], rtol=1e-5, atol=1e-5)
    fwd, inv, _ = R._kernels()
    np.testing.assert_allclose(fwd.numpy()[::37, 0, ::13], st["kernel_sample"], atol=1e-6)
    np.testing.assert_allclose(inv.numpy()[::37, 0, ::13], st["inv_kernel_sample"], atol=1e-6)


@pytest.mark.parametrize("kind", ["student", "teacher"])
def test_forward_train(kind):
    fx = golden(f"{kind}_fwd_train.npz")
    p = params(kind)
    x = torch.from_numpy(fx["x"])
    with torch.no_grad():
        out = R.dccrn_forward(p, x, train=True)
    for k, v in enumerate(out["enc"]):
        check_summary(f"enc{k}", v.numpy(), fx)
    for k, v in enumerate(out["dec"]):
        check_summary(f"dec{k}", v.numpy(), fx)
    check_summary("clstm_real", out["clstm"][0].transpose(0, 1).numpy(), fx)
    check_summary("clstm_img", out["clstm"][1].transpose(0, 1).numpy(), fx)
    for name in ("mask_real", "mask_imag", "real", "imag"):
        check_summary(name, out[name].numpy(), fx)
    np.testing.assert_allclose(out["out_wav"].numpy(), fx["out_wav"], rtol=1e-4, atol=1e-5)


def test_forward_eval_student():
    fx = golden("student_fwd_eval.npz")
    p = params("student")
    with torch.no_grad():
        out = R.dccrn_forward(p, torch.from_numpy(fx["x"]), train=False)
    np.testing.assert_allclose(out["out_wav"].numpy(), fx["out_wav"], rtol=1e-4, atol=1e-5)
    check_summary("mask_real", out["mask_real"].numpy(), fx)


def test_explicit_lstm_matches_torch_lstm():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(37, 3, 24, generator=g)
    w = [torch.randn(4 * 8, 24, generator=g) * 0.3, torch.randn(4 * 8, 8, generator=g) * 0.3,
         torch.randn(32, generator=g) * 0.1, torch.randn(32, generator=g) * 0.1]
    with torch.no_grad():
        np.testing.assert_allclose(R.lstm(x, *w).numpy(), R.lstm_torch(x, *w).numpy(), atol=2e-6)


def test_losses():
    ls = golden("losses.npz")
    x, y = torch.from_numpy(ls["mr/x"]), torch.from_numpy(ls["mr/y"])
    sc, mag = R.mrstft_loss(x, y)
    assert abs(sc.item() - float(ls["mr/sc"])) < 1e-6
    assert abs(mag.item() - float(ls["mr/mag"])) < 1e-6
    sc3, mag3 = R.mrstft_loss(x, y, (1024, 2048, 512), (120, 240, 50), (600, 1200, 240))
    assert abs(sc3.item() - float(ls["mr3/sc"])) < 1e-6
    assert abs(mag3.item() - float(ls["mr3/mag"])) < 1e-6
    for n in range(3):
        a, b = torch.from_numpy(ls[f"spkd{n}/s"]), torch.from_numpy(ls[f"spkd{n}/t"])
        assert abs(R.spkd_loss(a, b).item() - float(ls[f"spkd{n}/batchmean"])) < 1e-7
        assert abs(R.spkd_loss(a, b, "sum").item() - float(ls[f"spkd{n}/sum"])) < 1e-5


def test_clskd_step():
    fx = golden("clskd_step.npz")
    pt, ps, pabf = params("teacher"), params("student"), params("abf")
    with torch.no_grad():
        out = R.clskd_step(pt, ps, pabf, torch.from_numpy(fx["x"]), torch.from_numpy(fx["y"]))
    assert abs(out["base"].item() - float(fx["loss/base"])) < 1e-6
    np.testing.assert_allclose([v.item() for v in out["enc"]], fx["loss/enc"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose([v.item() for v in out["dec"]], fx["loss/dec"], rtol=1e-4, atol=1e-7)
    assert abs(out["clstm_real"].item() - float(fx["loss/clstm_real"])) < 1e-7
    assert abs(out["clstm_img"].item() - float(fx["loss/clstm_img"])) < 1e-7
    assert abs(out["total"].item() - float(fx["loss/total"])) < 1e-5
    for k, v in enumerate(out["s_enc"]):
        check_summary(f"s_enc{k}", v.numpy(), fx)
    for k, v in enumerate(out["s_dec"]):
        check_summary(f"s_dec{k}", v.numpy(), fx)
    np.testing.assert_allclose(out["student_wav"].numpy(), fx["student_wav"], rtol=1e-4, atol=1e-5)


def test_spkd_output_step():
    fx = golden("spkd_output_step.npz")
    pt, ps = params("teacher"), params("student")
    with torch.no_grad():
        out = R.spkd_output_step(pt, ps, torch.from_numpy(fx["x"]), torch.from_numpy(fx["y"]))
    assert abs(out["total"].item() - float(fx["loss/total"])) < 1e-6
    assert abs(out["spkd"].item() - float(fx["loss/spkd"])) < 1e-7
