"""Diagnostic (not collected by pytest): where does the CLSKD loss gap vs the oracle come from?
Compares, per SPKD pair, (a) the HIP kernel loss, (b) the fp64 loss of the HIP taps, (c) the
oracle fp32 loss, (d) the fp64 loss of the oracle taps."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conftest  # noqa: F401,E402
from test_gpu_parity import _kd, _oracle_params  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402


def loss64(s, t):
    s = s.reshape(s.shape[0], -1).double()
    t = t.reshape(t.shape[0], -1).double()
    gs = torch.nn.functional.normalize(s @ s.t(), p=1, dim=1)
    gt = torch.nn.functional.normalize(t @ t.t(), p=1, dim=1)
    return (torch.norm(gt - gs) ** 2 / s.shape[0] ** 2).item()


def main():
    torch.set_num_threads(16)
    noisy, clean = synthetic_pairs(4, 64000, seed=5)
    kd = _kd()
    X, y = torch.from_numpy(noisy).cuda(), torch.from_numpy(clean).cuda()
    out = kd.training_step((X, y), 0, return_parts=True)
    tf, sf = out["t"], out["s"]
    with torch.no_grad():
        ref = R.clskd_step(_oracle_params("teacher"), _oracle_params("student"),
                           _oracle_params("abf"), torch.from_numpy(noisy), torch.from_numpy(clean))
    hip_pairs = [(a, b) for a, b in zip(out["s_enc"], tf["enc"])]
    hip_pairs += [(a, b) for a, b in zip(out["s_dec"], [tf["dec_in"]] + tf["dec"][:5])]
    ref_pairs = [(a, b) for a, b in zip(ref["s_enc"], ref["t_taps"]["encoder"])]
    ref_pairs += [(a, b) for a, b in zip(ref["s_dec"], ref["t_taps"]["decoder"])]
    names = [f"enc{k}" for k in range(6)] + [f"dec{k}" for k in range(6)]
    hip_k = out["spkd"].cpu().numpy()
    ref_k = [v.item() for v in ref["enc"]] + [v.item() for v in ref["dec"]]
    print(f"{'pair':8s} {'hip_kernel':>12s} {'hip_taps64':>12s} {'oracle32':>12s} {'oracle64':>12s}"
          f" {'kern_err':>9s} {'orc_err':>9s} {'tap_gap':>9s}")
    for i, n in enumerate(names):
        a, b = hip_pairs[i]
        h64 = loss64(a.cpu(), b.cpu())
        r64 = loss64(*ref_pairs[i])
        print(f"{n:8s} {hip_k[i]:12.8f} {h64:12.8f} {ref_k[i]:12.8f} {r64:12.8f} "
              f"{(hip_k[i]-h64)/h64:9.1e} {(ref_k[i]-r64)/r64:9.1e} {(h64-r64)/r64:9.1e}")
    print("clstm_real hip", out["clstm_real"].item(), "oracle", ref["clstm_real"].item())
    print("clstm_img  hip", out["clstm_img"].item(), "oracle", ref["clstm_img"].item())
    print("base hip", out["base"].item(), "oracle", ref["base"].item())
    print("total hip", out["loss"].item(), "oracle", ref["total"].item())
    # tap agreement
    for k in range(6):
        a = tf["enc"][k].permute(0, 3, 1, 2).cpu().double()
        b = ref["t_taps"]["encoder"][k].double()
        print(f"t_enc{k} rel-rms {(torch.norm(a-b)/torch.norm(b)).item():.2e}")
    for k in range(6):
        a = out["s_enc"][k].permute(0, 3, 1, 2).cpu().double()
        b = ref["s_enc"][k].double()
        print(f"s_enc{k} rel-rms {(torch.norm(a-b)/torch.norm(b)).item():.2e}")


if __name__ == "__main__":
    main()
