"""CPU oracle for the validation metrics of distill.py:149-199: SI-SDR and STOI (numpy / scipy).

TEST INFRASTRUCTURE ONLY (same contract as ``oracle/ref_cpu.py``): only ``tests/`` may import it,
as the checker of the HIP metrics in ``clskd.metrics``.

The reference computes its validation metrics through third-party code that is NOT in
``/root/reference`` and not importable here:

* ``asteroid.metrics.get_metrics`` (asteroid 0.6.1dev fork, un-vendored), which delegates to
  ``pb_bss_eval.InputMetrics`` / ``OutputMetrics``:
  - ``si_sdr`` = ``pb_bss_eval.evaluation.si_sdr(reference, estimation)`` — the same formula
    (and the same docstring doctests) as the reference's own ``tools_for_loss.si_sdr``
    (tools_for_loss.py:50-92) without its eps terms; float64, no mean removal.
  - ``stoi`` = ``pystoi.stoi(clean, estimate, fs, extended=False)`` (pystoi 0.3.3 — the
    version whose ``resample_oct`` / ``remove_silent_frames`` are restated below; the
    reference's own ``tools_for_model.cal_stoi`` calls the same function, tools_for_model.py:
    595-600).

Parity of STOI is therefore UNPINNED in this container: no pystoi, no golden STOI value of a
clip we hold (the notebook value test_eval.ipynb ``stoi 0.8652`` is over LibriMix dev audio that
is absent).  SI-SDR is pinned by the tools_for_loss.py:60-77 doctest values.
"""
import numpy as np
from scipy.signal import resample_poly

FS = 10000          # pystoi.stoi: internal sample rate
N_FRAME = 256       # window length
NFFT = 512
NUMBAND = 15
MINFREQ = 150
N = 30              # frames per intermediate-intelligibility segment
BETA = -15.0        # lower SDR bound
DYN_RANGE = 40      # silent-frame threshold (dB below the loudest clean frame)
EPS = np.finfo("float").eps


# ------------------------------------------------------------------------------------------
# SI-SDR (pb_bss_eval.evaluation.si_sdr = tools_for_loss.py:50-92 without eps)
# ------------------------------------------------------------------------------------------
def si_sdr(reference, estimation):
    reference = np.asarray(reference, np.float64)
    estimation = np.asarray(estimation, np.float64)
    estimation, reference = np.broadcast_arrays(estimation, reference)
    reference_energy = np.sum(reference ** 2, axis=-1, keepdims=True)
    optimal_scaling = np.sum(reference * estimation, axis=-1, keepdims=True) / reference_energy
    projection = optimal_scaling * reference
    noise = estimation - projection
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = np.sum(projection ** 2, axis=-1) / np.sum(noise ** 2, axis=-1)
        return 10 * np.log10(ratio)


# ------------------------------------------------------------------------------------------
# STOI (pystoi 0.3.3: stoi.py, utils.py)
# ------------------------------------------------------------------------------------------
def thirdoct(fs, nfft, num_bands, min_freq):
    """1/3-octave band matrix [num_bands][nfft/2+1] (0/1) and centre frequencies."""
    f = np.linspace(0, fs, nfft + 1)
    f = f[:int(nfft / 2) + 1]
    k = np.array(range(num_bands)).astype(float)
    cf = np.power(2. ** (1. / 3), k) * min_freq
    freq_low = min_freq * np.power(2., (2 * k - 1) / 6)
    freq_high = min_freq * np.power(2., (2 * k + 1) / 6)
    obm = np.zeros((num_bands, len(f)))
    bands = []
    for i in range(len(cf)):
        l_ind = int(np.argmin(np.square(f - freq_low[i])))
        h_ind = int(np.argmin(np.square(f - freq_high[i])))
        obm[i, l_ind:h_ind] = 1
        bands.append((l_ind, h_ind))
    return obm, cf, bands


def _resample_window_oct(p, q):
    """Octave resample()'s anti-aliasing filter (pystoi.utils._resample_window_oct)."""
    gcd = np.gcd(p, q)
    if gcd > 1:
        p /= gcd
        q /= gcd
    log10_rejection = -3.0
    stopband_cutoff_f = 1. / (2 * max(p, q))
    roll_off_width = stopband_cutoff_f / 10
    rejection_db = -20 * log10_rejection
    L = np.ceil((rejection_db - 8) / (28.714 * roll_off_width))
    t = np.arange(-L, L + 1)
    ideal_filter = 2 * p * stopband_cutoff_f * np.sinc(2 * stopband_cutoff_f * t)
    if 21 <= rejection_db <= 50:
        beta = 0.5842 * (rejection_db - 21) ** 0.4 + 0.07886 * (rejection_db - 21)
    elif rejection_db > 50:
        beta = 0.1102 * (rejection_db - 8.7)
    else:
        beta = 0.0
    return np.kaiser(2 * L + 1, beta) * ideal_filter


def resample_oct(x, p, q):
    h = _resample_window_oct(p, q)
    window = h / np.sum(h)
    return resample_poly(x, p, q, window=window)


def _hanning(n):
    return np.hanning(n + 2)[1:-1]  # MATLAB hanning


def stft(x, win_size, fft_size, overlap=4):
    hop = int(win_size / overlap)
    w = _hanning(win_size)
    return np.array([np.fft.rfft(w * x[i:i + win_size], n=fft_size)
                     for i in range(0, len(x) - win_size, hop)])


def remove_silent_frames(x, y, dyn_range, framelen, hop):
    w = _hanning(framelen)
    x_frames = np.array([w * x[i:i + framelen] for i in range(0, len(x) - framelen, hop)])
    y_frames = np.array([w * y[i:i + framelen] for i in range(0, len(x) - framelen, hop)])
    x_energies = 20 * np.log10(np.linalg.norm(x_frames, axis=1) + EPS)
    mask = (np.max(x_energies) - dyn_range - x_energies) < 0
    x_frames = x_frames[mask]
    y_frames = y_frames[mask]
    n_sil = (len(x_frames) - 1) * hop + framelen
    x_sil = np.zeros(n_sil)
    y_sil = np.zeros(n_sil)
    for i in range(x_frames.shape[0]):
        x_sil[i * hop:i * hop + framelen] += x_frames[i, :]
        y_sil[i * hop:i * hop + framelen] += y_frames[i, :]
    return x_sil, y_sil


OBM, CF, BANDS = thirdoct(FS, NFFT, NUMBAND, MINFREQ)


def stoi(x, y, fs_sig, extended=False):
    """pystoi.stoi(clean x, processed y, fs_sig) — classic STOI (extended=False)."""
    if extended:
        raise NotImplementedError("extended STOI is not on the reference's path")
    x = np.asarray(x)
    y = np.asarray(y)
    if x.shape != y.shape:
        raise Exception("x and y should have the same length")
    if fs_sig != FS:
        x = resample_oct(x, FS, fs_sig)
        y = resample_oct(y, FS, fs_sig)
    x, y = remove_silent_frames(x, y, DYN_RANGE, N_FRAME, int(N_FRAME / 2))
    x_spec = stft(x, N_FRAME, NFFT, overlap=2).transpose()
    y_spec = stft(y, N_FRAME, NFFT, overlap=2).transpose()
    if x_spec.shape[-1] < N:
        return 1e-5
    x_tob = np.sqrt(np.matmul(OBM, np.square(np.abs(x_spec))))
    y_tob = np.sqrt(np.matmul(OBM, np.square(np.abs(y_spec))))
    x_segments = np.array([x_tob[:, m - N:m] for m in range(N, x_tob.shape[1] + 1)])
    y_segments = np.array([y_tob[:, m - N:m] for m in range(N, x_tob.shape[1] + 1)])
    normalization_consts = (np.linalg.norm(x_segments, axis=2, keepdims=True)
                            / (np.linalg.norm(y_segments, axis=2, keepdims=True) + EPS))
    y_segments_normalized = y_segments * normalization_consts
    clip_value = 10 ** (-BETA / 20)
    y_primes = np.minimum(y_segments_normalized, x_segments * (1 + clip_value))
    y_primes = y_primes - np.mean(y_primes, axis=2, keepdims=True)
    x_segments = x_segments - np.mean(x_segments, axis=2, keepdims=True)
    y_primes /= (np.linalg.norm(y_primes, axis=2, keepdims=True) + EPS)
    x_segments /= (np.linalg.norm(x_segments, axis=2, keepdims=True) + EPS)
    correlations_components = y_primes * x_segments
    J = x_segments.shape[0]
    M = x_segments.shape[1]
    return np.sum(correlations_components) / (J * M)


def get_metrics(mix, clean, estimate, sample_rate=16000, metrics_list=("si_sdr", "stoi")):
    """asteroid.metrics.get_metrics for one utterance, one source: {input_<m>, <m>}."""
    out = {}
    for m in metrics_list:
        if m == "si_sdr":
            out["input_si_sdr"] = float(si_sdr(clean, mix))
            out["si_sdr"] = float(si_sdr(clean, estimate))
        elif m == "stoi":
            out["input_stoi"] = float(stoi(clean, mix, sample_rate))
            out["stoi"] = float(stoi(clean, estimate, sample_rate))
        else:
            raise NotImplementedError(m)
    return out
