"""CPU: the validation-metric oracle (oracle/metrics_cpu.py) — SI-SDR pinned by the
tools_for_loss.py:60-77 doctests; STOI (pystoi 0.3.3 restated, parity unpinned: pystoi absent)
checked for its defining properties on the shipped example WAVs."""
import numpy as np

from conftest import golden
from oracle import metrics_cpu as MC


def test_sisdr_doctests():
    r = np.random.RandomState(0).randn(100)
    assert np.isinf(MC.si_sdr(r, r)) and np.isinf(MC.si_sdr(r, r * 2))
    assert abs(MC.si_sdr(r, np.flip(r)) - -25.127672346460717) < 1e-12
    assert abs(MC.si_sdr(r, r + np.flip(r)) - 0.481070445785553) < 1e-12
    assert abs(MC.si_sdr(r, r + 0.5) - 6.3704606032577304) < 1e-12
    assert abs(MC.si_sdr(r, r * 2 + 1) - 6.3704606032577304) < 1e-12
    np.testing.assert_allclose(MC.si_sdr([r, r], [r * 2 + 1, r * 1 + 0.5]), [6.3704606] * 2,
                               rtol=1e-7)


def test_stoi_properties():
    """Identity -> 1; more noise -> lower; scale invariance of the processed signal; the
    octave-band bins of pystoi's thirdoct at 10 kHz / 512."""
    ex = golden("examples.npz")
    s0 = ex["606/s0"].astype(np.float64) / 32768
    assert abs(MC.stoi(s0, s0, 16000) - 1.0) < 1e-12
    g = np.random.default_rng(0)
    noise = g.standard_normal(s0.shape) * np.std(s0)
    vals = [MC.stoi(s0, s0 + a * noise, 16000) for a in (0.1, 0.5, 2.0)]
    assert vals[0] > vals[1] > vals[2] > 0.2, vals
    assert abs(MC.stoi(s0, 3.0 * (s0 + 0.5 * noise), 16000) - vals[1]) < 1e-12
    assert MC.BANDS[0] == (7, 9) and MC.BANDS[-1] == (174, 219)
    h = MC._resample_window_oct(10000, 16000)
    assert h.size == 581  # 60 dB Octave filter for 5/8
