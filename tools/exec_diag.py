"""Diagnose executor-replay mismatches (tests/test_gpu_parity.py::test_step_graph_*[exec]):
eager vs StepExecutor replay on the same batches, per output (loss, the 16 loss slots, student
waveform), for 4-stream and 1-stream (serial) replays, with and without the folded BatchNorm
finalize, abf_reinit 'once' and 'step', and after a re-capture.

    python tools/exec_diag.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "speech-enhancement-clskd_amd"))

import torch  # noqa: E402

DEV = "cuda"


def main():
    from clskd import _lib, ops
    from clskd.data import synthetic_pairs
    from clskd.graph import StepExecutor, StepGraph
    import test_gpu_parity as P
    batches = []
    for seed in (11, 12):
        n, c = synthetic_pairs(4, 32000, seed=seed)
        batches.append((torch.from_numpy(n).to(DEV), torch.from_numpy(c).to(DEV)))

    def report(tag, kd_e, g):
        for i, (X, y) in enumerate(batches):
            o = kd_e.training_step((X, y), 0, return_parts=True)
            le, sp, wav = o["loss"].item(), o["spkd"].clone(), o["student_wav"].clone()
            lg = g(X, y).item()
            torch.cuda.synchronize()
            spd = (g.out["spkd"] - sp).abs().max().item()
            wd = (g.out["student_wav"] - wav).abs().max().item()
            bad = [k for k in range(sp.numel()) if not torch.equal(g.out["spkd"][k], sp[k])]
            print(f"{tag} batch {i}: loss eager {le:.7f} replay {lg:.7f} | spkd max diff {spd:.3e} "
                  f"slots differing {bad} | wav max diff {wd:.3e} finite {bool(torch.isfinite(g.out['spkd']).all())}",
                  flush=True)

    for fold in (True, False):
        ops._BN_FOLD = fold
        _lib.KNOB_EPOCH += 1  # re-ask every plan whether it folds
        for nst in (4, 1):
            for kind in ("exec", "graph"):
                if kind == "graph" and nst == 1:
                    continue
                kd_e, kd_g = P._kd().set_precision("mixed"), P._kd().set_precision("mixed")
                g = StepExecutor(kd_g, *batches[0], nstreams=nst) if kind == "exec" else \
                    StepGraph(kd_g, *batches[0])
                report(f"fold={int(fold)} {kind} streams={nst}", kd_e, g)
                with torch.no_grad():
                    for kd in (kd_e, kd_g):
                        kd.student.encoder[0][0].real_conv.weight.mul_(1.01)
                report(f"fold={int(fold)} {kind} streams={nst} recaptured", kd_e, g)
                del g
                torch.cuda.synchronize()
    # abf_reinit='step' (the redraw kernel inside the capture): finiteness per loss slot
    from clskd.distill import KnowledgeDistillation
    for fold in (True, False):
        ops._BN_FOLD = fold
        _lib.KNOB_EPOCH += 1  # re-ask every plan whether it folds
        for nst in (4, 1):
            kd = KnowledgeDistillation(P._models("teacher").train(), P._models("student").train(),
                                       abf_reinit="step", precision="mixed").to(DEV)
            g = StepExecutor(kd, *batches[0], nstreams=nst)
            for r in range(2):
                g(*batches[0])
                torch.cuda.synchronize()
                sp = g.out["spkd"]
                print(f"redraw fold={int(fold)} streams={nst} replay {r}: loss {g.out['loss'].item():.6f} "
                      f"non-finite slots {[k for k in range(sp.numel()) if not torch.isfinite(sp[k])]} "
                      f"wav finite {bool(torch.isfinite(g.out['student_wav']).all())}", flush=True)
            del g
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
