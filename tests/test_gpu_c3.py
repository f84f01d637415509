"""Configuration C3 (the CLSKD training step, BASELINE.json configs[2]) on the GPU:

  * the benched workload's gradients — precision='mixed', B=16 x 64000 samples, the step
    `bench.py --train` times — against the CPU oracle's autograd (oracle/ref_cpu.clskd_step with
    fp64 SPKD Grams, /root/reference distill.py:72-148 + the Adam of :202-204), per student
    parameter (missing #2);
  * data parallelism through the HIP training step: two ranks (processes) on the one GPU of the
    box over gloo, each running KnowledgeDistillation.train_step on its own shard through
    clskd.train.allreduce_grads + FlatAdam — the code path `bench.py --train --gpus N` runs over
    RCCL (missing #1).

Tolerance of the full-size gradient check (derived like DESIGN.md §4.1).  The student is fp32 end
to end, so the MRSTFT part of every gradient carries fp32 rounding only.  The SPKD part reaches
the student through the bf16 ReviewKD fusions: every ReviewKD activation is stored bf16 in the
forward and the raw-output gradient of each level is stored bf16 in the backward, and the teacher
features that set the SPKD coefficient matrices M = dG + dG^T are bf16 (row error rho <= 1.5e-2,
tests/test_gpu_c2_mixed.py).  One bf16 rounding has unit roundoff u = 2^-9 (RMS u/sqrt(3) = 1.1e-3
per element); a student parameter's SPKD gradient crosses at most 2 x 6 such roundings per
ReviewKD chain (forward activation + backward gradient per level), so its relative L2 error is
of order u * sqrt(12) = 6.8e-3 from the ReviewKD chain, plus the relative change of M.  M is
linear in the row-normalised Gram difference, whose relative error the loss-term check bounds
at 5e-3.  That estimate (~1.2e-2 for the worst parameter) is an upper scale: measured on the
MI355X (round 5, profiles/r5_c3_grad_parity.txt, every parameter listed) the worst relative L2
error is 3.2e-3 (decoder.1.2.weight, a BatchNorm gain), the LSTM / projection parameters
0.9-1.3e-3, the convolution weights <= 1e-3, and the loss 1.9e-5 relative.  The gates sit at
about 2x the measured worst: REL_GRAD = 7e-3 (still below the u * sqrt(12) = 6.8e-3 + 5e-3
derivation), REL_LOSS = 1e-4 (5x; the loss is a sum of 14 SPKD terms with independent bf16
errors and the fp32 base loss).  Set CLSKD_GRAD_PARITY_OUT=<file> to record the table.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from clskd import config as cfg
from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, apply_recipe

pytestmark = pytest.mark.gpu

DEV = "cuda"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch.set_num_threads(min(16, os.cpu_count() or 1))

REL_GRAD = 7e-3  # measured worst 3.2e-3 (profiles/r5_c3_grad_parity.txt)
REL_LOSS = 1e-4  # measured 1.9e-5; base (fp32 path) + 14 SPKD terms (each <= 5e-3, test_gpu_c2_mixed)


def _rel(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _kd(precision, abf_reinit="once"):
    from clskd.distill import KnowledgeDistillation
    from clskd.model import DCCRN
    t = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    s = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    kd = KnowledgeDistillation(t.train(), s.train(), abf_reinit=abf_reinit,
                               precision=precision).to(DEV)
    apply_recipe(kd.review_encoder, ABF_SEED, "encoder.")
    apply_recipe(kd.review_decoder, ABF_SEED, "decoder.")
    return kd


@pytest.mark.timeout(900)
def test_c3_mixed_full_batch_gradients_against_oracle():
    from clskd.data import synthetic_pairs
    from clskd.weights import recipe_state_dict
    from oracle import ref_cpu as R

    B, L = 16, 64000
    noisy, clean = synthetic_pairs(B, L, seed=8)
    kd = _kd("mixed")
    X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
    out = kd.forward_with_tape(X, y)
    grads = {n: torch.empty_like(p) for n, p in kd.student.named_parameters()}
    kd.backward_into(out, {p: grads[n] for n, p in kd.student.named_parameters()})
    torch.cuda.synchronize()
    loss = out["loss"].item()
    got = {n: g.double().cpu().numpy() for n, g in grads.items()}
    del out, grads
    torch.cuda.empty_cache()

    pt = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.TEACHER), TEACHER_SEED))
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    pa = R.to_torch_params(recipe_state_dict(
        {**cfg.review_param_shapes("encoder"), **cfg.review_param_shapes("decoder")}, ABF_SEED))
    for k, v in ps.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var")):
            v.requires_grad_()
    ref = R.clskd_step(pt, ps, pa, torch.from_numpy(noisy), torch.from_numpy(clean),
                       lstm_fn=R.lstm, gram_dtype=torch.float64)
    ref["total"].backward()
    rloss = ref["total"].item()
    print(f"loss hip-mixed {loss:.7f} oracle (fp64 Grams) {rloss:.7f} rel {abs(loss - rloss) / rloss:.2e}")
    assert abs(loss - rloss) <= REL_LOSS * abs(rloss)

    rows, bad, worst = [], [], 0.0
    for name, g in got.items():
        if name not in ps or ps[name].grad is None:
            continue
        r = ps[name].grad.double().numpy()
        if name.endswith("_conv.bias") and not name.startswith("decoder.5."):
            # conv bias before a train-mode BatchNorm: analytically zero gradient
            wref = np.linalg.norm(ps[name.replace(".bias", ".weight")].grad.double().numpy())
            e = max(np.linalg.norm(g), np.linalg.norm(r)) / wref
            rows.append(f"{name:42s} {e:.2e}  (|g|/|dW|, analytically 0)")
            if e > 1e-3:
                bad.append(name)
            continue
        e = _rel(g, r)
        worst = max(worst, e)
        rows.append(f"{name:42s} {e:.2e}")
        if e > REL_GRAD:
            bad.append(name)
    print("\n".join(rows))
    print(f"worst relative L2 gradient error {worst:.2e} (tolerance {REL_GRAD})")
    rec = os.environ.get("CLSKD_GRAD_PARITY_OUT")
    if rec:  # the measured margins behind REL_GRAD (profiles/r5_c3_grad_parity.txt)
        with open(rec, "w") as f:
            f.write(f"loss hip-mixed {loss:.7f} oracle (fp64 Grams) {rloss:.7f} "
                    f"rel {abs(loss - rloss) / rloss:.3e} (tolerance {REL_LOSS})\n")
            f.write("\n".join(rows) + "\n")
            f.write(f"worst relative L2 gradient error {worst:.3e} (tolerance {REL_GRAD})\n")
    assert len(rows) > 40
    assert not bad, bad


# ------------------------------------------------------------------------------------------
# data parallelism: two ranks on one GPU over gloo, through the HIP training step
# ------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        from clskd import dist as cdist
        from clskd.data import synthetic_pairs
        from clskd.train import FlatAdam, FlatParams, allreduce_grads
        cdist.init("gloo")
        kd = _kd("mixed")
        flat = FlatParams(kd.student)
        opt = FlatAdam(flat, lr=cfg.learning_rate)
        p0 = flat.data.clone()
        noisy, clean = synthetic_pairs(2, 8000, seed=cdist.shard_seed(40, rank))
        X, y = torch.from_numpy(noisy).to(DEV), torch.from_numpy(clean).to(DEV)
        # step 1, spelled out (KnowledgeDistillation.train_step) so the rank-local gradient is seen
        out = kd.forward_with_tape(X, y)
        kd.backward_into(out, flat.grad_dict())  # writes (does not accumulate into) the views
        torch.cuda.synchronize()
        local = flat.grad.clone()
        scale = allreduce_grads(flat)
        summed = flat.grad.clone()
        opt.step(grad_scale=scale)
        p1 = flat.data.clone()
        # step 2 through the API the bench times
        kd.train_step((X, y), flat, opt)
        torch.cuda.synchronize()
        q.put((rank, scale, p0.cpu().numpy(), local.cpu().numpy(), summed.cpu().numpy(),
               p1.cpu().numpy(), flat.data.cpu().numpy(), None))
        torch.distributed.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, None, None, None, None, traceback.format_exc()))
        raise


@pytest.mark.timeout(600)
def test_ddp_world2_train_step_on_gpu():
    """Two ranks, one process each, both on cuda:0, gloo for the gradient all-reduce: after the
    all-reduce both ranks hold the bitwise sum of the two rank-local gradients, and after Adam
    (1/world folded into the launch) bitwise-identical parameters equal to torch.optim.Adam on
    the mean gradient; a second train_step keeps the ranks identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=500) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    errs = [r[7] for r in res if r[7]]
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs)
    (_, s0, p00, g0, sum0, p10, p20, _), (_, s1, p01, g1, sum1, p11, p21, _) = res
    assert s0 == s1 == 0.5
    np.testing.assert_array_equal(p00, p01)  # same initial weights (recipe)
    assert not np.array_equal(g0, g1)  # different shards -> different local gradients
    np.testing.assert_array_equal(sum0, sum1)
    np.testing.assert_array_equal(sum0, g0 + g1)  # fp32 a + b: exact and commutative
    np.testing.assert_array_equal(p10, p11)  # identical parameters after Adam
    np.testing.assert_array_equal(p20, p21)  # and after a second train_step
    # Adam on the mean gradient (torch.optim.Adam semantics, first step)
    ref = torch.from_numpy(p00.copy()).requires_grad_()
    ref.grad = torch.from_numpy((g0 + g1) * np.float32(0.5))
    torch.optim.Adam([ref], lr=cfg.learning_rate).step()
    np.testing.assert_allclose(p10, ref.detach().numpy(), rtol=1e-6, atol=1e-7)
    assert not np.array_equal(p10, p00) and not np.array_equal(p20, p10)
