"""CPU: the asteroid DCCRNet_mini oracle (oracle/asteroid_cpu.py) against the reference's own
outputs — the five example_CLSKD/*/s0_estimate.wav its eval script (eval.py:57-96) wrote from
checkpoint/the_best_model.pth (SURVEY.md §8 f rank 2).  Pinned: int16 estimates within 2 LSB,
>= 99 % of samples bit-exact; the STFTFB filter formula equals the checkpoint's filters."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import asteroid_cpu as A

IDS = ["606", "1038", "1132", "1431", "2158"]


def test_stftfb_formula_matches_checkpoint():
    sd = A.state_dict_from_fixture(golden("asteroid_mini.npz"))
    f = A.stftfb_filters()
    assert float((f - sd["encoder.filterbank._filters"]).abs().max()) < 1e-8


@pytest.mark.parametrize("ex", IDS)
def test_oracle_reproduces_shipped_estimates(ex):
    fx = golden("asteroid_mini.npz")
    est_ref = golden("examples.npz")[ex + "/est"].astype(np.int64)
    sd = A.state_dict_from_fixture(fx)
    mix = A.mixture_from_wav(fx[ex + "/mixture"])
    torch.set_num_threads(4)
    with torch.no_grad():
        y = A.forward(sd, torch.from_numpy(mix)[None], train=True)[0].numpy()
    q = A.to_pcm16(A.normalize_estimates(y, mix))
    d = np.abs(q - est_ref)
    assert d.max() <= 2, d.max()
    assert np.mean(d == 0) >= 0.99, np.mean(d == 0)


def test_dropin_state_dict_keys_and_load():
    """clskd.asteroid.DCCRNet_mini has the checkpoint's 182 keys / shapes and loads it via the
    asteroid API (from_pretrained on a serialize() dict); its STFTFB init equals the checkpoint."""
    from clskd.asteroid import DCCRNet_mini, load_conf
    conf = load_conf(golden("asteroid_mini.npz"))
    m = DCCRNet_mini(**conf["model_args"])
    ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    theirs = {k: tuple(v.shape) for k, v in conf["state_dict"].items()}
    assert ours == theirs
    assert float((m.encoder.filterbank._filters - conf["state_dict"]["encoder.filterbank._filters"]).abs().max()) < 1e-8
    m2 = DCCRNet_mini.from_pretrained(conf)
    assert torch.equal(m2.masker.output_layer[0].re_module.bias,
                       conf["state_dict"]["masker.output_layer.0.re_module.bias"])
