"""Fixture for the asteroid DCCRNet_mini path (SURVEY.md §8 f rank 2): the reference's trained
CLSKD student checkpoint and the full-length example mixtures its eval script enhanced.

Run in the build container only (needs /root/reference):
    python tests/golden/gen_asteroid.py

Sources (data files of the reference, nothing executable):
  * checkpoint/the_best_model.pth — asteroid ``serialize()`` dict of ``DCCRNet_mini``
    ('DCCRN-CL-test'); loaded with ``torch.load(weights_only=True)`` (TorchVersion allow-listed
    for the ``infos`` entry).  Every ``state_dict`` tensor is stored as a float32 array under its
    key; ``decoder.filterbank.*`` equal ``encoder.filterbank.*`` bit for bit and are stored once.
  * example_CLSKD/ex_<id>/mixture.wav — the int16 mixtures eval.py:57-96 enhanced and wrote
    (s0_estimate.wav is already in examples.npz as ``<id>/est``).
Writes tests/golden/asteroid_mini.npz.
"""
import json
import os
import wave

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
IDS = ["606", "1038", "1132", "1431", "2158"]


def read_wav(path):
    with wave.open(path) as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1 and w.getframerate() == 16000
        return np.frombuffer(w.readframes(w.getnframes()), np.int16).copy()


def main():
    torch.serialization.add_safe_globals([torch.torch_version.TorchVersion])
    ck = torch.load(os.path.join(REF, "checkpoint", "the_best_model.pth"), map_location="cpu",
                    weights_only=True)
    sd = ck["state_dict"]
    for k in ("_filters", "torch_window"):
        assert torch.equal(sd["encoder.filterbank." + k], sd["decoder.filterbank." + k])
    out = {}
    for k, v in sd.items():
        if k.startswith("decoder.filterbank."):
            continue
        out["w/" + k] = v.numpy().astype(np.float32 if v.is_floating_point() else np.int64)
    out["model_name"] = np.array(ck["model_name"])
    out["model_args"] = np.array(json.dumps(ck["model_args"]))
    for i in IDS:
        out[f"{i}/mixture"] = read_wav(os.path.join(REF, "example_CLSKD", f"ex_{i}", "mixture.wav"))
    np.savez_compressed(os.path.join(HERE, "asteroid_mini.npz"), **out)
    print("wrote asteroid_mini.npz:", len(sd), "state_dict keys,", len(IDS), "mixtures")


if __name__ == "__main__":
    main()
