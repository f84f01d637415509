"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Run in the survey/build container only (needs /root/reference):
    python tests/golden/gen_golden.py

The reference is imported through ``_ref_shims`` (SURVEY.md §8 c).  Weights come from the
deterministic recipe ``clskd.weights.recipe_state_dict`` (no weight files are committed).
Only the resulting ``.npz``/``.json`` data files are committed; nothing of the reference's source
is copied.  ``KnowledgeDistillation.training_step`` (distill.py:72-148) cannot be imported
(pytorch_lightning absent, script trains at import), so ``ref_training_step`` below re-drives it
from the reference's own modules: feature_extraction.DCCRN hooks, framework.build_review_kd,
framework.SPKDLoss and framework.MultiResolutionSTFTLoss.

Large tensors are stored as checksums (float64 sum, |sum|, square-sum) plus a fixed strided
sample of 1024 elements; small ones are stored whole.
"""
import json
import os
import sys
import wave

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "speech-enhancement-clskd_amd"))
sys.path.insert(0, HERE)

import _ref_shims  # noqa: E402

_ref_shims.install()

import torch  # noqa: E402

torch.set_num_threads(8)
torch.manual_seed(0)

import DCCRN as ref_dccrn  # noqa: E402  (reference module)
import feature_extraction as ref_fe  # noqa: E402
import framework as ref_fw  # noqa: E402
import tools_for_loss as ref_loss  # noqa: E402
import tools_for_model as ref_tm  # noqa: E402

from clskd import config as ccfg  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from clskd.weights import (ABF_SEED, STUDENT_SEED, TEACHER_SEED,  # noqa: E402
                           recipe_state_dict)

SAMPLE_N = 1024


def summ(prefix, x, out):
    x = np.asarray(x.detach().cpu().numpy() if torch.is_tensor(x) else x, np.float64)
    flat = x.ravel()
    n = flat.size
    idx = np.linspace(0, n - 1, min(n, SAMPLE_N)).astype(np.int64)
    out[prefix + "/shape"] = np.array(x.shape, np.int64)
    out[prefix + "/sum"] = flat.sum()
    out[prefix + "/abssum"] = np.abs(flat).sum()
    out[prefix + "/sqsum"] = (flat ** 2).sum()
    out[prefix + "/idx"] = idx
    out[prefix + "/sample"] = flat[idx].astype(np.float32)


def full(prefix, x, out):
    out[prefix] = (x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)).astype(np.float32)


def make_model(kind):
    if kind == "teacher":
        m = ref_dccrn.DCCRN(rnn_units=ccfg.rnn_units, masking_mode="E", use_clstm=True,
                            kernel_num=ccfg.kernel_num)
        seed = TEACHER_SEED
    else:
        m = ref_dccrn.DCCRN(rnn_units=ccfg.rnn_units_student, masking_mode="E", use_clstm=True,
                            kernel_num=ccfg.kernel_num_student)
        seed = STUDENT_SEED
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = recipe_state_dict(shapes, seed)
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()},
                                            strict=False)
    assert not unexpected and all(k.startswith(("stft.", "istft.")) for k in missing), missing
    return m, shapes


def inject_review(model, ft_type):
    shapes = {f"{ft_type}." + k: tuple(v.shape) for k, v in model.state_dict().items()}
    sd = recipe_state_dict(shapes, ABF_SEED)
    model.load_state_dict({k[len(ft_type) + 1:]: torch.from_numpy(v) for k, v in sd.items()})
    return shapes


def local_taps(model, X):
    """feature_extraction.DCCRN hooks (feature_extraction.py:3-50) + the asteroid-equivalent
    tap contract."""
    ext = ref_fe.DCCRN(model)
    fm = ext.extract_feature_maps(X)
    ext.remove_hook()
    r, i = fm["clstm"][0]
    L, B, P = r.shape
    C = 2 * (P // 4)
    lstm_out = torch.cat([r.reshape(L, B, C // 2, 4), i.reshape(L, B, C // 2, 4)], 2).permute(1, 2, 3, 0)
    return dict(encoder=list(fm["encoder"]), decoder=[lstm_out] + list(fm["decoder"][:5]),
                clstm_real=r.transpose(0, 1), clstm_img=i.transpose(0, 1),
                dec_all=list(fm["decoder"]))


def ref_training_step(teacher, student, X, y, out):
    """distill.py:72-148 driven through the reference's own modules (local DCCRN)."""
    t = local_taps(teacher, X)
    s = local_taps(student, X)
    model_encoder = ref_fw.build_review_kd(s["encoder"], "encoder")
    inject_review(model_encoder, "encoder")
    s_enc = model_encoder(X)
    model_decoder = ref_fw.build_review_kd(s["decoder"], "decoder")
    inject_review(model_decoder, "decoder")
    s_dec = model_decoder(X)
    student_preds = student(X, is_feat=True)
    stft_loss = ref_fw.MultiResolutionSTFTLoss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100])
    base = stft_loss(student_preds.squeeze(), y.squeeze())[1]
    enc_terms = [ref_fw.SPKDLoss(sf, tf, "batchmean")() for sf, tf in zip(s_enc, t["encoder"])]
    dec_terms = [ref_fw.SPKDLoss(sf, tf, "batchmean")() for sf, tf in zip(s_dec, t["decoder"])]
    cr = ref_fw.SPKDLoss(s["clstm_real"], t["clstm_real"], reduction="batchmean")()
    ci = ref_fw.SPKDLoss(s["clstm_img"], t["clstm_img"], reduction="batchmean")()
    total = base + sum(enc_terms) + sum(dec_terms) + cr + ci
    out["loss/total"] = total.item()
    out["loss/base"] = base.item()
    out["loss/enc"] = np.array([v.item() for v in enc_terms])
    out["loss/dec"] = np.array([v.item() for v in dec_terms])
    out["loss/clstm_real"] = cr.item()
    out["loss/clstm_img"] = ci.item()
    for k, v in enumerate(s_enc):
        summ(f"s_enc{k}", v, out)
    for k, v in enumerate(s_dec):
        summ(f"s_dec{k}", v, out)
    for k, v in enumerate(t["encoder"]):
        summ(f"t_enc{k}", v, out)
    for k, v in enumerate(t["decoder"]):
        summ(f"t_dec{k}", v, out)
    # normalised Grams of every pair (small: B x B)
    for name, a, b in ([(f"enc{k}", s_enc[k], t["encoder"][k]) for k in range(6)]
                       + [(f"dec{k}", s_dec[k], t["decoder"][k]) for k in range(6)]
                       + [("clstm_real", s["clstm_real"], t["clstm_real"]),
                          ("clstm_img", s["clstm_img"], t["clstm_img"])]):
        kd = ref_fw.SPKDLoss(a, b, "batchmean")
        full(f"gram_s/{name}", kd.matmul_and_normalize(a), out)
        full(f"gram_t/{name}", kd.matmul_and_normalize(b), out)
    full("student_wav", student_preds, out)


def read_wav(path):
    with wave.open(path) as w:
        return np.frombuffer(w.readframes(w.getnframes()), np.int16).copy()


def main():
    out_dir = HERE
    keys = {}

    # ---- 1. SI-SNR / SI-SDR known-answer tests (tools_for_loss.py:37-108 docstring) ----------
    kat = {}
    np.random.seed(0)
    ref = np.random.randn(100)
    cases = {"flip": np.flip(ref).copy(), "ref_plus_flip": ref + np.flip(ref), "ref_plus_half": ref + 0.5,
             "two_ref_plus_one": ref * 2 + 1}
    kat["reference"] = ref
    for name, est in cases.items():
        kat[f"est/{name}"] = est
        r = torch.from_numpy(ref)
        e = torch.from_numpy(est)
        kat[f"si_sdr/{name}"] = ref_loss.si_sdr(r, e).item()
        kat[f"si_snr/{name}"] = ref_loss.si_snr(e, r).item()
        kat[f"si_snr32/{name}"] = ref_loss.si_snr(e.float(), r.float()).item()
    kat["doc/si_sdr/flip"] = -25.127672346460717
    kat["doc/si_sdr/ref_plus_flip"] = 0.481070445785553
    kat["doc/si_sdr/ref_plus_half"] = 6.3704606032577304
    kat["doc/si_sdr/two_ref_plus_one"] = 6.3704606032577304
    g = np.random.default_rng(5)
    s1 = g.standard_normal((6, 3001)).astype(np.float32)
    s2 = (0.7 * s1 + 0.3 * g.standard_normal((6, 3001))).astype(np.float32)
    kat["rand/s1"] = s1
    kat["rand/s2"] = s2
    kat["rand/si_snr"] = ref_loss.si_snr(torch.from_numpy(s1), torch.from_numpy(s2)).item()
    np.savez_compressed(os.path.join(out_dir, "kat_sisnr.npz"), **kat)

    # ---- 2. the five shipped examples (example_CLSKD/*) ---------------------------------------
    ex = {}
    for e in ["606", "1038", "1132", "1431", "2158"]:
        d = os.path.join(_ref_shims.REFERENCE, "example_CLSKD", f"ex_{e}")
        mix, s0, est = (read_wav(os.path.join(d, n + ".wav")) for n in ("mixture", "s0", "s0_estimate"))
        ex[f"{e}/s0"] = s0
        ex[f"{e}/est"] = est
        ex[f"{e}/mixture64k"] = mix[:64000]
        ex[f"{e}/si_snr"] = ref_loss.si_snr(torch.from_numpy(est / 32768.0).float(),
                                            torch.from_numpy(s0 / 32768.0).float()).item()
    np.savez_compressed(os.path.join(out_dir, "examples.npz"), **ex)

    # ---- 3. ConvSTFT / ConviSTFT (tools_for_model.py:35-109) ----------------------------------
    st = {}
    x = torch.from_numpy(np.random.default_rng(3).uniform(-1, 1, (2, 4000)).astype(np.float32))
    stft = ref_tm.ConvSTFT(400, 100, 512, "hamming", "complex")
    istft = ref_tm.ConviSTFT(400, 100, 512, "hamming", "complex")
    spec = stft(x)
    st["x"] = x.numpy()
    st["spec"] = spec.numpy()
    st["istft"] = istft(spec).numpy()
    st["kernel_sample"] = stft.weight.numpy()[::37, 0, ::13]
    st["inv_kernel_sample"] = istft.weight.numpy()[::37, 0, ::13]
    np.savez_compressed(os.path.join(out_dir, "stft.npz"), **st)

    # ---- 4. model forwards -------------------------------------------------------------------
    teacher, tshapes = make_model("teacher")
    student, sshapes = make_model("student")
    keys["teacher"] = {k: list(v) for k, v in tshapes.items()}
    keys["student"] = {k: list(v) for k, v in sshapes.items()}
    noisy, clean = synthetic_pairs(2, 8000, seed=11)
    X = torch.from_numpy(noisy)
    Y = torch.from_numpy(clean)

    for kind, model in (("student", student), ("teacher", teacher)):
        fw = {"x": noisy}
        model.train()
        m0 = {k: v.clone() for k, v in model.state_dict().items() if "running" in k}
        taps = local_taps(model, X)
        outs = model(X)
        for k, v in enumerate(taps["encoder"]):
            summ(f"enc{k}", v, fw)
        for k, v in enumerate(taps["dec_all"]):
            summ(f"dec{k}", v, fw)
        summ("clstm_real", taps["clstm_real"], fw)
        summ("clstm_img", taps["clstm_img"], fw)
        for name, v in zip(("mask_real", "mask_imag", "real", "imag"), outs[:4]):
            summ(name, v, fw)
        full("out_wav", outs[4], fw)
        # BN running stats after two train forwards (hooks pass + plain pass), from the recipe
        for k, v in model.state_dict().items():
            if "running" in k:
                full(f"bn2/{k}", v, fw)
        model.load_state_dict({**model.state_dict(), **m0})
        np.savez_compressed(os.path.join(out_dir, f"{kind}_fwd_train.npz"), **fw)

    # eval-mode student forward (C1: BN running stats), 1 s @16 kHz, batch 1
    ev = {}
    xe, _ = synthetic_pairs(1, 16000, seed=12)
    student.eval()
    with torch.no_grad():
        outs = student(torch.from_numpy(xe))
    ev["x"] = xe
    full("out_wav", outs[4], ev)
    summ("mask_real", outs[0], ev)
    summ("real", outs[2], ev)
    student.train()
    np.savez_compressed(os.path.join(out_dir, "student_fwd_eval.npz"), **ev)

    # ---- 5. the CLSKD step (distill.py:72-148) ------------------------------------------------
    cs = {"x": noisy, "y": clean}
    sd_t = {k: v.clone() for k, v in teacher.state_dict().items()}
    sd_s = {k: v.clone() for k, v in student.state_dict().items()}
    ref_training_step(teacher, student, X, Y, cs)
    teacher.load_state_dict(sd_t)
    student.load_state_dict(sd_s)
    for ft in ("encoder", "decoder"):
        rk = ref_fw.build_review_kd([None] * 6, ft)
        keys[f"review_{ft}"] = {f"{ft}." + k: list(v.shape) for k, v in rk.state_dict().items()}
    np.savez_compressed(os.path.join(out_dir, "clskd_step.npz"), **cs)

    # ---- 6. distill_SPKD.py:69-87 (SPKD on the output waveforms) ------------------------------
    sp = {"x": noisy, "y": clean}
    s_wav = student(X, is_feat=True)
    with torch.no_grad():
        t_wav = teacher(X, is_feat=True)
    stft_loss = ref_fw.MultiResolutionSTFTLoss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100])
    base = stft_loss(s_wav.squeeze(), Y.squeeze())[1]
    spk = ref_fw.SPKDLoss(s_wav, t_wav, reduction="batchmean")()
    sp["loss/base"] = base.item()
    sp["loss/spkd"] = spk.item()
    sp["loss/total"] = (base + spk).item()
    teacher.load_state_dict(sd_t)
    student.load_state_dict(sd_s)
    np.savez_compressed(os.path.join(out_dir, "spkd_output_step.npz"), **sp)

    # ---- 7. loss kernels in isolation ---------------------------------------------------------
    ls = {}
    g = np.random.default_rng(9)
    xa = g.uniform(-0.5, 0.5, (3, 8000)).astype(np.float32)
    ya = (0.6 * xa + 0.2 * g.standard_normal((3, 8000))).astype(np.float32)
    mr = ref_fw.MultiResolutionSTFTLoss(fft_sizes=[512], win_lengths=[400], hop_sizes=[100])
    sc, mag = mr(torch.from_numpy(xa), torch.from_numpy(ya))
    ls["mr/x"], ls["mr/y"], ls["mr/sc"], ls["mr/mag"] = xa, ya, sc.item(), mag.item()
    mr3 = ref_fw.MultiResolutionSTFTLoss()  # the class defaults: 3 resolutions
    sc3, mag3 = mr3(torch.from_numpy(xa), torch.from_numpy(ya))
    ls["mr3/sc"], ls["mr3/mag"] = sc3.item(), mag3.item()
    for n, (shape_s, shape_t) in enumerate([((4, 8, 16, 23), (4, 32, 16, 23)),
                                            ((16, 16, 4, 20), (16, 48, 4, 20)),
                                            ((5, 37, 128), (5, 37, 512))]):
        a = g.standard_normal(shape_s).astype(np.float32)
        b = g.standard_normal(shape_t).astype(np.float32) + 0.5
        ls[f"spkd{n}/s"], ls[f"spkd{n}/t"] = a, b
        ls[f"spkd{n}/batchmean"] = ref_fw.SPKDLoss(torch.from_numpy(a), torch.from_numpy(b), "batchmean")().item()
        ls[f"spkd{n}/sum"] = ref_fw.SPKDLoss(torch.from_numpy(a), torch.from_numpy(b), "sum")().item()
    np.savez_compressed(os.path.join(out_dir, "losses.npz"), **ls)

    with open(os.path.join(out_dir, "param_keys.json"), "w") as f:
        json.dump(keys, f, indent=0)
    print("fixtures written to", out_dir)
    for fn in sorted(os.listdir(out_dir)):
        if fn.endswith((".npz", ".json")):
            print(f"  {fn:28s} {os.path.getsize(os.path.join(out_dir, fn)) / 1024:8.1f} KiB")


if __name__ == "__main__":
    main()
