"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/clskd.h declares; host-side plumbing (K tables, packing, module trees) is consistent.
No GPU compute is called here."""
import ctypes
import os

import numpy as np
import pytest
import torch

from clskd import _lib, config as cfg


def test_library_exports_every_header_symbol():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    lib = _lib.load(require_gpu=False)
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # every bound signature is a header symbol and vice versa
    assert set(_lib.SIGNATURES) == set(syms)
    assert lib.clskd_version() == 1
    assert isinstance(lib.clskd_last_error(), bytes)


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors have the C compiler's layout of include/clskd.h (sizeof and the
    offset of each struct's last field, from a probe compiled with gcc)."""
    import subprocess
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    probe = tmp_path / "probe.c"
    probe.write_text("""
#include <stdio.h>
#include <stddef.h>
#include "clskd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(clskd_seg),
         sizeof(clskd_ktab_entry), sizeof(clskd_gram_job), offsetof(clskd_gram_job, shift),
         sizeof(clskd_draw_job), offsetof(clskd_draw_job, stream_id), sizeof(clskd_conv_desc),
         offsetof(clskd_conv_desc, tap_dt), offsetof(clskd_conv_desc, accumulate),
         sizeof(clskd_gram_bwd_job), offsetof(clskd_gram_bwd_job, accumulate),
         sizeof(clskd_stream_hop_args), offsetof(clskd_stream_hop_args, dec_co),
         offsetof(clskd_stream_hop_args, off_frames), offsetof(clskd_conv_desc, bn_fold),
         sizeof(clskd_bn_fold), offsetof(clskd_bn_fold, count), offsetof(clskd_bn_fold, eps),
         offsetof(clskd_bn_fold, var_out), offsetof(clskd_gram_job, out));
  return 0;
}
""")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", inc, str(probe), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [ctypes.sizeof(_lib.Seg), ctypes.sizeof(_lib.KtabEntry), ctypes.sizeof(_lib.GramJob),
            _lib.GramJob.shift.offset, ctypes.sizeof(_lib.DrawJob), _lib.DrawJob.stream_id.offset,
            ctypes.sizeof(_lib.ConvDesc), _lib.ConvDesc.tap_dt.offset,
            _lib.ConvDesc.accumulate.offset, ctypes.sizeof(_lib.GramBwdJob),
            _lib.GramBwdJob.accumulate.offset, ctypes.sizeof(_lib.StreamHopArgs),
            _lib.StreamHopArgs.dec_co.offset, _lib.StreamHopArgs.off_frames.offset,
            _lib.ConvDesc.bn_fold.offset, ctypes.sizeof(_lib.BnFold), _lib.BnFold.count.offset,
            _lib.BnFold.eps.offset, _lib.BnFold.var_out.offset, _lib.GramJob.out.offset]
    assert got == want


def test_error_path_reports_without_gpu():
    lib = _lib.load(require_gpu=False)
    rc = lib.clskd_conv2d_fwd(None, None)
    assert rc == -4
    assert b"null descriptor" in lib.clskd_last_error()
    rc = lib.clskd_lstm_recurrent(None, 0, 0, 0, None, 1, 1, 1, 32, None, 0, 0, 0, None)
    assert rc < 0


def test_ktab_construction():
    from clskd import ops
    g1 = ops.SegGeom(8, 1000, 100, 8, 5, 12)
    g2 = ops.SegGeom(4, 500, 40, 4, 5, 12)
    entries = []
    taps = [(-1, 0), (0, -1)]
    for dF, dT in taps:
        for s, g in enumerate((g1, g2)):
            for c in range(g.C):
                entries.append((c + dF * g.sF + dT * g.sT, dF, dT, s))
    assert len(entries) == 24  # padded to 32 in the device table
    # K order is (tap, segment, channel): the packer must follow it
    w = torch.arange(3 * 2 * 12, dtype=torch.float32).reshape(3, 2, 12)
    wp = ops.pack_weight(w, 24)
    assert wp.shape == (3, 32) and torch.all(wp[:, 24:] == 0)
    assert torch.equal(wp[:, :24], w.reshape(3, 24))


def test_module_tree_matches_reference_state_dict():
    from clskd.model import DCCRN
    for spec in (cfg.STUDENT, cfg.TEACHER):
        m = DCCRN(masking_mode="E", use_clstm=True, **spec)
        keys = [k for k in m.state_dict() if not k.startswith(("stft.", "istft."))]
        assert keys == list(cfg.dccrn_param_shapes(**spec))
    with pytest.raises(NotImplementedError):
        DCCRN(masking_mode="C", use_clstm=True, **cfg.STUDENT)


def test_stft_kernels_match_oracle():
    from clskd.model import ConvSTFT, ConviSTFT
    from oracle import ref_cpu
    fwd, inv, win = ref_cpu._kernels()
    assert torch.equal(ConvSTFT(400, 100, 512, "hamming", "complex").weight, fwd)
    i = ConviSTFT(400, 100, 512, "hamming", "complex")
    assert torch.equal(i.weight, inv) and torch.equal(i.window, win)


def test_synthetic_data_recipe():
    from clskd.data import synthetic_pairs
    a, b = synthetic_pairs(2, 16000, seed=3)
    a2, _ = synthetic_pairs(2, 16000, seed=3)
    assert a.shape == (2, 16000) and np.array_equal(a, a2)
    assert np.abs(a).max() <= 1.0 and np.abs(b).max() < 1.0


def test_gram_job_validation_without_gpu():
    """clskd_gram_partial / clskd_spkd_finalize take HOST job arrays (kernel arguments) and
    validate them before any launch: bad geometry, non-contiguous slab ranges and pair indices
    are reported, not executed."""
    lib = _lib.load(require_gpu=False)
    J = _lib.GramJob
    fake = 1 << 20  # never dereferenced: validation fails first
    good = J(fake, 64, 100, 8, 0, 8, 10, 0, 10, _lib.F32, 0)
    bad_gap = (J * 2)(good, J(fake, 64, 100, 8, 0, 8, 10, 11, 10, _lib.F32, 0))
    assert lib.clskd_gram_partial(bad_gap, 2, 4, fake, None) == -1
    assert b"not contiguous" in lib.clskd_last_error()
    bad_cs = (J * 1)(J(fake, 64, 100, 6, 0, 6, 10, 0, 10, _lib.F32, 0))
    assert lib.clskd_gram_partial(bad_cs, 1, 4, fake, None) == -1
    assert lib.clskd_gram_partial((J * 1)(good), 1, 33, fake, None) == -1  # B > 32
    pairs = (ctypes.c_int32 * 2)(0, 5)
    assert lib.clskd_spkd_finalize((J * 1)(good), 1, pairs, 1, 4, 1, fake, None, None, fake,
                                   None) == -1
    assert b"outside" in lib.clskd_last_error()


def test_gram_chunk_and_bn_bwd_alignment_validation_without_gpu():
    """Validation added with the division-free Gram loads and the vectorised backward BN apply:
    a slab whose chunk * Cs^2 reaches 2^32 (the 32-bit multiply-high split would be inexact) and
    a misaligned bn_bwd workspace are reported before any launch."""
    lib = _lib.load(require_gpu=False)
    J = _lib.GramJob
    fake = 1 << 20
    big = (J * 1)(J(fake, 1024 * 100, 100, 1024, 0, 1024, 8192, 0, 1, _lib.F32, 0))
    assert lib.clskd_gram_partial(big, 1, 4, fake, None) == -1
    assert b"2^32" in lib.clskd_last_error()
    ok = (J * 1)(J(fake, 1024 * 100, 100, 1024, 0, 1024, 16, 0, 7, _lib.F32, 0))
    assert lib.clskd_gram_partial(ok, 1, 4, 0, None) < 0  # passes the chunk check, then null slabs
    assert b"null slab" in lib.clskd_last_error()
    f = fake
    rc = lib.clskd_bn_bwd(f, f, 1024, 64, f, f, f, f, 1e-5, None, None, f + 8, 16, None, None,
                          None, f, 0, 0, _lib.F32, None)
    assert rc < 0 and b"16-byte aligned" in lib.clskd_last_error()


def test_dispatch_knobs_and_experiment_guard_without_gpu():
    """Dispatch knobs are read once and switched through clskd_set_knob; unknown names are
    rejected.  The product library has no timing-only modes: selecting one makes the affected
    entry point fail with CLSKD_E_ARG before any launch instead of computing a wrong result
    (CLSKD_LSTM*_TDIV / CLSKD_G8 >= 10 / CLSKD_BF16_DEBUG_MODE)."""
    lib = _lib.load(require_gpu=False)
    assert lib.clskd_experiments_build() == 0
    v = ctypes.c_int32(-1)
    assert lib.clskd_get_knob(b"CLSKD_LSTM_NKS32", ctypes.byref(v)) == 0 and v.value == 1
    assert lib.clskd_set_knob(b"CLSKD_NO_SUCH_KNOB", 1) == -4
    assert b"unknown knob" in lib.clskd_last_error()
    prev = _lib.set_knob("CLSKD_LSTM_NKS32", 8)
    assert prev == 1 and lib.clskd_get_knob(b"CLSKD_LSTM_NKS32", ctypes.byref(v)) == 0 and v.value == 8
    _lib.set_knob("CLSKD_LSTM_NKS32", prev)
    # experiment knobs (timing-only modes, A/B dispatch switches, grid caps): a product library
    # holds them at their defaults and refuses any other value (every remaining
    # knob is parity-tested or gone from the product)
    for name in ("CLSKD_LSTM128_TDIV", "CLSKD_LSTM32_TDIV", "CLSKD_G8", "CLSKD_HALO_GRID",
                 "CLSKD_NO_HALO", "CLSKD_BF16_DEBUG_MODE", "CLSKD_G8_KORDER", "CLSKD_EXEC_GATE"):
        assert lib.clskd_get_knob(name.encode(), ctypes.byref(v)) == 0
        dflt = v.value
        assert lib.clskd_set_knob(name.encode(), dflt) == 0  # its default stays settable
        assert lib.clskd_set_knob(name.encode(), dflt + 2) == -4, name
        assert b"CLSKD_EXPERIMENTS" in lib.clskd_last_error(), name
        assert lib.clskd_get_knob(name.encode(), ctypes.byref(v)) == 0 and v.value == dflt
    # CLSKD_G8_GRID is a product knob since round 4 (clskd_step's concurrent-step grid cap,
    # tests/test_gpu_parity.py::test_step_g8_grid_cap_is_bitwise_neutral)
    assert _lib.set_g8_grid(224) == 0 and _lib.set_g8_grid(0) == 224
    # the removed knobs are unknown
    for name in (b"CLSKD_DIRECT_COOP", b"CLSKD_EXEC_PRIO", b"CLSKD_EXEC_PACE_NS"):
        assert lib.clskd_set_knob(name, 1) == -4 and b"unknown knob" in lib.clskd_last_error()
