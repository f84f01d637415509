"""Characterise the mixed-precision backward flake (DESIGN.md §8 "Known flake"): run the C3
student backward N times per mode on one process and report the worst relative gradient error
of each run against the first fp32 run.  Modes: fp32 and mixed on the normal multi-stream
schedule, and mixed under distill.serialized_streams (every side stream = the caller's).
    python tools/flake_probe.py [--runs 6]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from clskd import config as cfg  # noqa: E402
from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, apply_recipe  # noqa: E402


def _kd(precision):
    from clskd.distill import KnowledgeDistillation
    from clskd.model import DCCRN
    t = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    s = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    kd = KnowledgeDistillation(t.train(), s.train(), abf_reinit="once",
                               precision=precision).to("cuda")
    apply_recipe(kd.review_encoder, ABF_SEED, "encoder.")
    apply_recipe(kd.review_decoder, ABF_SEED, "decoder.")
    return kd


def grads_of(kd, X, y):
    grads = {n: torch.empty_like(p) for n, p in kd.student.named_parameters()}
    pg = {p: grads[n] for n, p in kd.student.named_parameters()}
    kd.backward_into(kd.forward_with_tape(X, y), pg)
    torch.cuda.synchronize()
    return {n: g.double().cpu().numpy() for n, g in grads.items()}


def worst(a, ref):
    out = []
    for n in ref:
        if n.endswith("_conv.bias") and not n.startswith("decoder.5."):
            continue
        d = np.linalg.norm(a[n] - ref[n]) / max(np.linalg.norm(ref[n]), 1e-30)
        out.append((d, n))
    return max(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    args = ap.parse_args()
    from clskd.data import synthetic_pairs
    from clskd.distill import serialized_streams
    noisy, clean = synthetic_pairs(2, 8000, seed=23)
    X, y = torch.from_numpy(noisy).cuda(), torch.from_numpy(clean).cuda()
    ref = grads_of(_kd("fp32"), X, y)
    for mode in ("fp32", "mixed", "mixed-serial", "mixed-fresh"):
        kd = None if mode == "mixed-fresh" else _kd(mode.split("-")[0])
        for r in range(args.runs):
            k = _kd("mixed") if kd is None else kd
            if mode == "mixed-serial":
                with serialized_streams():
                    gr = grads_of(k, X, y)
            else:
                gr = grads_of(k, X, y)
            w = worst(gr, ref)
            print(f"{mode:13s} run {r}: worst rel {w[0]:.3e} ({w[1]})", flush=True)


if __name__ == "__main__":
    main()
