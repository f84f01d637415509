"""Host-side logic of the Python drop-in layer that needs no GPU: caches and bookkeeping."""
import gc
import os

import torch


class _FakeWeight:
    """Stands in for a device tensor: same storage address and version for two distinct objects
    (what the allocator can hand a new model after an old one is freed)."""

    def __init__(self, ptr, version=0):
        self._ptr, self._version = ptr, version

    def data_ptr(self):
        return self._ptr


def test_tw_cache_rebuilds_for_a_new_source_identity():
    """backward._tw (transposed-weight cache): a source with the same data_ptr and _version but a
    new object identity must rebuild (the round-2 stale-entry flake), an in-place update
    (version bump) must rebuild, the same object must hit; dead sources are swept and the cache
    is bounded."""
    from clskd import backward as bw
    bw._TW.clear()
    calls = []

    def build(tag):
        def f():
            calls.append(tag)
            return torch.full((2,), float(len(calls)))
        return f

    key = ("abf", 1234, "conv2")
    a = _FakeWeight(0x1000)
    w1 = bw._tw(key, a, build("a"))
    assert bw._tw(key, a, build("a-again")) is w1 and calls == ["a"]
    b = _FakeWeight(0x1000)  # same address and version, different object
    w2 = bw._tw(key, b, build("b"))
    assert calls == ["a", "b"] and w2 is not w1
    b._version += 1  # in-place update of the source
    bw._tw(key, b, build("b-v1"))
    assert calls[-1] == "b-v1"
    # dead sources are swept on insert
    c = _FakeWeight(0x2000)
    bw._tw(("other", 1), c, build("c"))
    del c
    gc.collect()
    d = _FakeWeight(0x3000)
    bw._tw(("third", 1), d, build("d"))
    assert ("other", 1) not in bw._TW
    # bounded
    keep = [_FakeWeight(0x4000 + i) for i in range(bw._TW_MAX + 10)]
    for i, src in enumerate(keep):
        bw._tw(("many", i), src, lambda: torch.zeros(1))
    assert len(bw._TW) <= bw._TW_MAX
    bw._TW.clear()


def test_spkd_perturbation_bound_holds():
    """tests/spkd_bound.py: the bound on an SPKD term's change under row-wise relative feature
    errors rho holds for random and for aligned (worst-direction) perturbations.  (It is a
    worst-case bound: for random error directions the observed change is ~sqrt(K) smaller.)"""
    import numpy as np
    from spkd_bound import _gram, row_rel_err, spkd_bound, spkd_term
    rng = np.random.default_rng(0)
    B, K = 16, 4000
    for trial in range(20):
        base = rng.standard_normal(K)
        zt = np.maximum(0.6 * base + rng.standard_normal((B, K)), 0) + 0.05 * rng.standard_normal((B, K))
        zs = np.maximum(0.5 * base + rng.standard_normal((B, K)), 0)
        rho_t = 10 ** rng.uniform(-4, -1.5, B)
        rho_s = 10 ** rng.uniform(-5, -2, B)
        L0 = spkd_term(_gram(zs), _gram(zt))
        for aligned in (False, True):
            et = rng.standard_normal((B, K)) if not aligned else zt * np.sign(rng.standard_normal((B, 1)))
            es = rng.standard_normal((B, K)) if not aligned else -zs
            et *= (rho_t * np.linalg.norm(zt, axis=1) / np.linalg.norm(et, axis=1))[:, None]
            es *= (rho_s * np.linalg.norm(zs, axis=1) / np.linalg.norm(es, axis=1))[:, None]
            np.testing.assert_allclose(row_rel_err(zt + et, zt), rho_t, rtol=1e-9)
            L1 = spkd_term(_gram(zs + es), _gram(zt + et))
            bnd = spkd_bound(_gram(zs), _gram(zt), rho_s, rho_t)
            assert abs(L1 - L0) <= bnd, (trial, aligned, abs(L1 - L0), bnd)


def test_train_graph_requires_device_step_optimizer():
    """TrainStepGraph replays the optimizer: a host-side step count would be frozen into the
    capture, so it refuses FlatAdam(device_step=False) before touching the model."""
    import pytest
    import torch
    from clskd.graph import TrainStepGraph
    from clskd.train import FlatAdam, FlatParams
    m = torch.nn.Linear(4, 3)
    flat = FlatParams(m)
    with pytest.raises(ValueError, match="device_step"):
        TrainStepGraph(None, flat, FlatAdam(flat), torch.zeros(1, 8), torch.zeros(1, 8))
    opt = FlatAdam(flat, device_step=True)
    assert opt.step_count == 0 and len(opt.state()) == 4


def test_bench_standalone_multi_gpu_launch_command():
    """`bench.py --gpus N` outside a launcher starts N ranks itself (torch.distributed.run as a
    child, rendezvous on 127.0.0.1) with the same arguments."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cmd = bench.spawn_cmd(8, ["--gpus", "8", "--steps", "5"], 29512)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29512"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")


def test_pack_provenance_follows_the_current_cache_entry():
    """model.pack_provenance / pack_output (backward.tw_prebuild's source lookup): an output is
    traced to (model, group, slot) only while it is the object the registry recorded, and
    pack_output returns the model's current entry's slot (a re-pack replaces it)."""
    from clskd import model as M

    class Holder:
        def __init__(self):
            self._wcache = {}

    h = Holder()
    a, b = torch.zeros(3), torch.ones(2)
    h._wcache["g"] = ((), (a, b), None, None)
    M._note_pack_outputs(h, "g", (a, b))
    assert M.pack_provenance(b) == (h, "g", 1)
    assert M.pack_provenance(torch.zeros(2)) is None
    assert M.pack_output(h, "g", 1, None) is b
    a2, b2 = torch.zeros(3), torch.full((2,), 2.0)  # the next step's re-pack
    h._wcache["g"] = ((), (a2, b2), None, None)
    M._note_pack_outputs(h, "g", (a2, b2))
    assert M.pack_output(h, "g", 1, None) is b2
    assert M.pack_provenance(b2) == (h, "g", 1)
    t = torch.zeros(4)
    h._wcache["t"] = ((), t, None, None)
    M._note_pack_outputs(h, "t", t)
    assert M.pack_provenance(t) == (h, "t", None) and M.pack_output(h, "t", None, None) is t
    tok = object()  # an entry built inside a capture serves only that capture
    h._wcache["c"] = ((), t, tok, tok)
    assert M.pack_output(h, "c", None, None) is None and M.pack_output(h, "c", None, tok) is t
