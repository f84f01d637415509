"""GPU: the validation metrics (clskd.metrics: clskd_sisdr_f64, clskd_stoi) and
KnowledgeDistillation.validation_step (distill.py:149-199) against the CPU oracle
(oracle/metrics_cpu.py: pb_bss si_sdr, pystoi 0.3.3 stoi restated with numpy/scipy).

Pinning: SI-SDR by the tools_for_loss.py:60-77 doctest values; STOI is "parity unpinned" (pystoi
is absent and no reference file holds the STOI of a clip we have) — the HIP STOI is checked
against the restatement only.  Tolerances: SI-SDR 1e-9 dB on the doctests / 1e-6 dB elsewhere
(both fp64); STOI 1e-7 absolute (fp64 on both sides: a direct DFT against pocketfft and
different summation orders); validation_step within 1e-4 (the HIP student waveform differs
from the oracle's fp32 CPU forward at the 1e-6 level).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import metrics_cpu as MC

pytestmark = pytest.mark.gpu
DEV = "cuda"
IDS = ["606", "1038", "1132", "1431", "2158"]


def _t(a):
    return torch.from_numpy(np.asarray(a, np.float32)).to(DEV)


def test_sisdr_doctests_and_examples():
    from clskd import metrics
    r = np.random.RandomState(0).randn(100)
    cases = [(r, np.flip(r), -25.127672346460717), (r, r + np.flip(r), 0.481070445785553),
             (r, r + 0.5, 6.3704606032577304), (r, r * 2 + 1, 6.3704606032577304)]
    for ref, est, want in cases:
        # the doctests run in float64; the device API takes fp32 rows: compare with the oracle
        # on the same fp32-rounded rows, and the oracle itself with the doctest values
        assert abs(MC.si_sdr(ref, est) - want) < 1e-9
        got = float(metrics.si_sdr(_t(ref), _t(est)).cpu())
        o = float(MC.si_sdr(np.float32(ref), np.float32(est)))
        assert abs(got - o) < 1e-9, (got, o)
    ex = golden("examples.npz")
    for k in IDS:
        s0 = ex[k + "/s0"].astype(np.float32) / 32768
        est = ex[k + "/est"].astype(np.float32) / 32768
        got = float(metrics.si_sdr(_t(s0), _t(est)).cpu())
        assert abs(got - MC.si_sdr(s0, est)) < 1e-6
        assert abs(got - float(ex[k + "/si_snr"])) < 2e-3  # the eps'd fp32 si_snr of a14


def test_stoi_examples_against_oracle():
    """Single utterances of different lengths (4.3-11.6 s), identity (= 1) and a mixture."""
    from clskd import metrics
    ex = golden("examples.npz")
    for k in IDS:
        s0 = ex[k + "/s0"].astype(np.float32) / 32768
        est = ex[k + "/est"].astype(np.float32) / 32768
        got = float(metrics.stoi(_t(s0), _t(est), 16000).cpu())
        want = MC.stoi(s0, est, 16000)
        assert abs(got - want) < 1e-7, (k, got, want)
    s0 = ex["606/s0"].astype(np.float32)[:64000] / 32768
    mix = ex["606/mixture64k"].astype(np.float32) / 32768
    assert abs(float(metrics.stoi(_t(s0), _t(s0), 16000).cpu()) - 1.0) < 1e-9
    got = float(metrics.stoi(_t(s0), _t(mix), 16000).cpu())
    assert abs(got - MC.stoi(s0, mix, 16000)) < 1e-7


def test_stoi_batched_rates_and_edges():
    """A batch of rows with different kept-frame counts (a silent gap in one), the 10 kHz path
    (no resampling), 8 kHz (another rational ratio) and a clip too short for one segment
    (pystoi returns 1e-5)."""
    from clskd import metrics
    ex = golden("examples.npz")
    rows_c, rows_e = [], []
    for k in IDS:
        rows_c.append(ex[k + "/s0"].astype(np.float32)[:64000] / 32768)
        rows_e.append(ex[k + "/est"].astype(np.float32)[:64000] / 32768)
    rows_c[2] = rows_c[2].copy()
    rows_c[2][20000:40000] *= 1e-4  # long quiet stretch: frames dropped mid-utterance
    c, e = np.stack(rows_c), np.stack(rows_e)
    got = metrics.stoi(_t(c), _t(e), 16000).cpu().numpy()
    want = np.array([MC.stoi(c[i], e[i], 16000) for i in range(len(IDS))])
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-7)
    for fs in (10000, 8000):
        got = metrics.stoi(_t(c[:2]), _t(e[:2]), fs).cpu().numpy()
        want = np.array([MC.stoi(c[i], e[i], fs) for i in range(2)])
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-7)
    short = c[:1, :4000]  # 0.25 s: fewer than 30 STFT frames
    assert float(metrics.stoi(_t(short), _t(short * 0.5), 16000).cpu()) == 1e-5
    assert MC.stoi(short[0], short[0] * 0.5, 16000) == 1e-5


def test_validation_step_against_oracle():
    """distill.py:149-199 end to end: eval-mode student estimate, si_sdr / stoi of estimate and
    mixture, batch means and improvements."""
    from clskd import config as cfg
    from clskd.data import synthetic_pairs
    from clskd.distill import KnowledgeDistillation
    from clskd.model import DCCRN
    from clskd.weights import STUDENT_SEED, TEACHER_SEED, apply_recipe, recipe_state_dict
    from oracle import ref_cpu as R
    teacher = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    student = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    kd = KnowledgeDistillation(teacher, student).to(DEV).train()
    noisy, clean = synthetic_pairs(3, 16000, seed=5)
    res = kd.validation_step((torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)), 0)
    assert kd.student.training, "validation_step restores the training mode"
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    with torch.no_grad():
        est = R.dccrn_forward(ps, torch.from_numpy(noisy), train=False)["out_wav"].numpy()
    utt = [MC.get_metrics(noisy[i], clean[i], est[i]) for i in range(3)]
    for m in ("si_sdr", "stoi"):
        want = np.mean([u[m] for u in utt])
        imp = np.mean([u[m] - u["input_" + m] for u in utt])
        assert abs(res[m] - want) < 1e-4, (m, res[m], want)
        assert abs(res[m + "_imp"] - imp) < 1e-4, (m, res[m + "_imp"], imp)
