"""Configuration C4 as BASELINE.json states it: distill_SPKD.py's step (distill_SPKD.py:69-87) at
batch 32 x 4 s with the frozen teacher in fp16, against the CPU oracle.

The step: student forward (fp32, train-mode BN), teacher forward (no_grad, distill_SPKD.py:75-76)
on IEEE-half MFMA operands with fp16 feature storage and fp32 accumulation, the MRSTFT base loss
on the student waveform, and ONE SPKD term over the two output waveforms [B, 1, L]
(framework.py:150-172).  Oracle: oracle/ref_cpu.dccrn_forward (fp32) for both models, the SPKD
term with fp64 Grams (the exact term of the oracle's waveforms).

Bars: student waveform RMS <= 1e-4 and SI-SNR within 0.01 dB (fp32 student), base loss within
1e-4 relative, the fp16 teacher waveform within RHO_MAX_F16 row-wise relative error, the SPKD
term within the rigorous perturbation bound of tests/spkd_bound.py at the measured errors and
within REL_SPKD of the exact term.
"""
import os

import numpy as np
import pytest
import torch

from spkd_bound import _gram, row_rel_err, spkd_bound, spkd_term

pytestmark = pytest.mark.gpu

DEV = "cuda"
torch.set_num_threads(min(16, os.cpu_count() or 1))

# fp16 carries 3 more mantissa bits than bf16 (unit roundoff 2^-12 vs 2^-9); the teacher's
# waveform row error is the fp16 feature error carried through mask 'E' and the iSTFT.
RHO_MAX_F16 = 5e-3
REL_SPKD = 2e-3


@pytest.mark.timeout(900)
@pytest.mark.parametrize("precision", ["fp16"])
def test_c4_spkd_output_step_b32_against_oracle(precision):
    from clskd import config as cfg
    from clskd.data import synthetic_pairs
    from clskd.distill import SPKDDistillation
    from clskd.model import DCCRN
    from clskd.tools_for_loss import si_snr
    from clskd.weights import STUDENT_SEED, TEACHER_SEED, apply_recipe, recipe_state_dict
    from oracle import ref_cpu as R

    B, L = 32, 64000
    noisy, clean = synthetic_pairs(B, L, seed=12)
    teacher = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    student = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    kd = SPKDDistillation(teacher, student, precision=precision).to(DEV).train()
    assert kd.teacher.compute == "fp16" and kd.teacher.act_dtype == torch.float16
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    out = kd.training_step((X, y), 0, return_parts=True)
    torch.cuda.synchronize()

    pt = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.TEACHER), TEACHER_SEED))
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    Xc, yc = torch.from_numpy(noisy), torch.from_numpy(clean)
    with torch.no_grad():
        s_ref = R.dccrn_forward(ps, Xc, train=True)["out_wav"]
        t_ref = R.dccrn_forward(pt, Xc, train=True)["out_wav"]
        base_ref = R.mrstft_loss(s_ref.squeeze(), yc.squeeze())[1].item()

    s_hip = out["student_wav"].double().cpu().numpy()
    wav_rms = float(np.sqrt(np.mean((s_hip - s_ref.double().numpy()) ** 2)))
    d_snr = abs(si_snr(out["student_wav"], y).item() - R.si_snr(s_ref, yc).item())
    print(f"C4 {precision}: student RMS {wav_rms:.2e}, SI-SNR delta {d_snr:.2e} dB, base "
          f"{out['base'].item():.6f} vs {base_ref:.6f}")
    assert wav_rms <= 1e-4 and d_snr <= 0.01
    assert abs(out["base"].item() - base_ref) <= 1e-4 * abs(base_ref)

    t_hip = out["teacher_wav"].float().cpu().numpy().reshape(B, -1)
    rs, rt = s_ref.numpy().reshape(B, -1), t_ref.numpy().reshape(B, -1)
    rho_s = row_rel_err(s_hip.reshape(B, -1), rs)
    rho_t = row_rel_err(t_hip, rt)
    Gs, Gt = _gram(rs), _gram(rt)
    L_exact = spkd_term(Gs, Gt)
    bnd = spkd_bound(Gs, Gt, rho_s, rho_t)
    got = out["spkd"].item()
    dev = abs(got - L_exact)
    print(f"C4 {precision}: spkd exact {L_exact:.6e} hip {got:.6e} rel {dev / L_exact:.2e} | "
          f"rho_t max {rho_t.max():.2e} rho_s max {rho_s.max():.2e} | bound {bnd:.2e}")
    assert rho_t.max() <= RHO_MAX_F16
    assert dev <= bnd
    assert dev <= REL_SPKD * L_exact
