"""Configuration C3 as a captured step (clskd.graph.TrainStepExecutor / TrainStepGraph): the
training step — fwd+loss with the tape, HIP backward, Adam — recorded once and replayed by the C++
step executor or hipGraphLaunch must
be the same computation as eager ``train_step`` calls: loss, every parameter, Adam's moments and
step count bitwise equal after each of three steps on different batches (same kernels, same
arguments, deterministic reductions).  Plus the device-step Adam kernel against the host-step
one and torch.optim.Adam (distill.py:202-204)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
torch.set_num_threads(min(16, os.cpu_count() or 1))


def test_adam_device_step_matches_host_step_and_torch():
    from clskd import ops
    g = torch.Generator().manual_seed(5)
    p0 = torch.randn(5000, generator=g)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=6e-4, weight_decay=0.01)
    p_h, p_d = p0.clone().to(DEV), p0.clone().to(DEV)
    m_h, v_h = torch.zeros_like(p_h), torch.zeros_like(p_h)
    m_d, v_d = torch.zeros_like(p_d), torch.zeros_like(p_d)
    t = torch.zeros(1, dtype=torch.int32, device=DEV)
    for step in range(1, 5):
        grad = torch.randn(5000, generator=g)
        ref.grad = grad.clone()
        opt.step()
        ops.adam_step(p_h, grad.to(DEV), m_h, v_h, 6e-4, 0.9, 0.999, 1e-8, 0.01, step)
        ops.adam_step_dev(p_d, grad.to(DEV), m_d, v_d, 6e-4, 0.9, 0.999, 1e-8, 0.01, t)
    assert int(t.item()) == 4
    # bias corrections: powf on the device vs on the host (a few ulp at most)
    np.testing.assert_allclose(p_d.cpu().numpy(), p_h.cpu().numpy(), rtol=2e-7, atol=1e-9)
    np.testing.assert_allclose(p_d.cpu().numpy(), ref.detach().numpy(), rtol=1e-6, atol=1e-7)
    assert torch.equal(m_d, m_h) and torch.equal(v_d, v_h)


@pytest.mark.parametrize("launch", ["exec", "graph"])
@pytest.mark.parametrize("precision", ["mixed", "fp32"])
def test_train_graph_matches_eager_train_steps(precision, launch):
    """TrainStepExecutor (the C++ step executor) / TrainStepGraph (hipGraphLaunch) replays of the
    captured training step vs eager."""
    from clskd.data import synthetic_pairs
    from clskd.graph import TrainStepExecutor, TrainStepGraph
    from clskd.train import FlatAdam, FlatParams
    from test_gpu_parity import _kd
    batches = []
    for seed in (31, 32, 33):
        n, c = synthetic_pairs(4, 16000, seed=seed)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))
    kd_e, kd_g = _kd().set_precision(precision), _kd().set_precision(precision)
    runs = []
    for kd in (kd_e, kd_g):
        flat = FlatParams(kd.student)
        runs.append((flat, FlatAdam(flat, lr=6e-4, device_step=True)))
    (fe, oe), (fg, og) = runs
    assert torch.equal(fe.data, fg.data)
    ex = (TrainStepExecutor if launch == "exec" else TrainStepGraph)(kd_g, fg, og, *batches[0])
    assert og.step_count == 0 and torch.equal(fe.data, fg.data)  # warm-up state restored
    if launch == "exec":
        # (a whole captured step: ~480 kernels once the packing gathers are batched)
        assert ex.info["memcpys"] == 0 and ex.info["kernels"] > 400, ex.info
    for i, (X, y) in enumerate(batches):
        le = kd_e.train_step((X, y), fe, oe)
        lg = ex(X, y)
        torch.cuda.synchronize()
        assert lg.item() == le.item(), (i, lg.item(), le.item())
        assert torch.equal(fg.grad, fe.grad), i
        assert torch.equal(fg.data, fe.data), i
    assert oe.step_count == og.step_count == 3
    assert torch.equal(oe.m, og.m) and torch.equal(oe.v, og.v)
    assert ex.captures == 1
    # BatchNorm running statistics of the student (updated inside the replayed forward)
    for (k, a), b in zip(kd_e.student.state_dict().items(), kd_g.student.state_dict().values()):
        assert torch.equal(a, b), k


@pytest.mark.parametrize("launch", ["exec", "graph"])
def test_eager_train_step_right_after_capture(launch):
    """An eager training step between the capture and the first replay (bench.py's census step)
    must not read the packed weights the capture built (they hold nothing until a replay): the
    capture advances the parameters' versions.  Eager, replay, eager — bitwise the all-eager
    sequence on a second model."""
    from clskd.data import synthetic_pairs
    from clskd.graph import TrainStepExecutor, TrainStepGraph
    from clskd.train import FlatAdam, FlatParams
    from test_gpu_parity import _kd
    batches = []
    for seed in (51, 52, 53):
        n, c = synthetic_pairs(4, 16000, seed=seed)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))
    kd_e, kd_g = _kd().set_precision("mixed"), _kd().set_precision("mixed")
    (fe, oe), (fg, og) = [(f, FlatAdam(f, lr=6e-4, device_step=True))
                          for f in (FlatParams(kd_e.student), FlatParams(kd_g.student))]
    ex = (TrainStepExecutor if launch == "exec" else TrainStepGraph)(kd_g, fg, og, *batches[0])
    for i, (X, y) in enumerate(batches):
        le = kd_e.train_step((X, y), fe, oe)
        lg = ex(X, y) if i == 1 else kd_g.train_step((X, y), fg, og)
        torch.cuda.synchronize()
        assert lg.item() == le.item(), (i, lg.item(), le.item())
        assert torch.equal(fg.data, fe.data), i


@pytest.mark.parametrize("launch", ["exec", "graph"])
def test_train_graph_replays_interleaved_with_eager_forwards(launch):
    """Replay, eager eval forward, replay, eager eval forward: every eager forward of the trained
    student must use the parameters the replays' Adam wrote (the packed-weight cache is keyed on
    the parameters' version counters, which a replay bumps) — checked against a fresh copy of
    the student (no caches) holding the same parameters."""
    from clskd import config as cfg
    from clskd.data import synthetic_pairs
    from clskd.graph import TrainStepExecutor, TrainStepGraph
    from clskd.model import DCCRN
    from clskd.train import FlatAdam, FlatParams
    from test_gpu_parity import _kd
    n, c = synthetic_pairs(4, 16000, seed=41)
    X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
    xe = torch.from_numpy(synthetic_pairs(2, 16000, seed=42)[0]).to(DEV)
    kd = _kd().set_precision("mixed")
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=6e-4, device_step=True)
    ex = (TrainStepExecutor if launch == "exec" else TrainStepGraph)(kd, flat, opt, X, y)
    outs = []
    for _ in range(2):
        ex(X, y)
        kd.student.eval()
        with torch.no_grad():
            got = kd.student(xe, is_feat=True).clone()
            # a new student holding the same parameters and statistics: no packed-weight caches
            fresh = DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT).to(DEV)
            fresh.load_state_dict(kd.student.state_dict())
            fresh.compute = kd.student.compute
            ref = fresh.eval()(xe, is_feat=True)
        kd.student.train()
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
        outs.append(got)
    assert not torch.equal(outs[0], outs[1])  # the second replay changed the parameters


def test_pack_maps_match_builds():
    """The trained student's parameter groups are re-packed by one index_gather from the flat
    parameter buffer (model._pack_group, maps probed on the first build): after Adam steps every
    mapped group's outputs equal the torch packing of a fresh student holding the same
    parameters, bitwise."""
    from clskd import config as cfg
    from clskd.data import synthetic_pairs
    from clskd.model import DCCRN
    from clskd.train import FlatAdam, FlatParams
    from test_gpu_parity import _kd
    n, c = synthetic_pairs(4, 16000, seed=43)
    X, y = torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)
    kd = _kd().set_precision("mixed")
    flat = FlatParams(kd.student)
    opt = FlatAdam(flat, lr=6e-4)
    for _ in range(3):
        kd.train_step((X, y), flat, opt)
    s = kd.student
    mapped = [k for k, v in s._pmaps.items() if v]
    assert len(mapped) >= 8, sorted(s._pmaps)
    fresh = DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT).to(DEV)
    fresh.load_state_dict(s.state_dict())
    flat.bump_versions()  # force the re-packs through the maps
    calls = {"enc": "_enc_w", "dec": "_dec_w", "lstm": "_lstm_w"}
    for key in mapped:
        fn = calls[key[0]]
        got = getattr(s, fn)(*key[1:])
        ref = getattr(fresh, fn)(*key[1:])
        got = [got] if isinstance(got, torch.Tensor) else list(got)
        ref = [ref] if isinstance(ref, torch.Tensor) else list(ref)
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            assert a.shape == b.shape and torch.equal(a, b), key
