"""GPU: the asteroid DCCRNet_mini drop-in (clskd.asteroid, SURVEY.md §8 f rank 2) on the
reference's trained checkpoint against (a) the reference's own outputs — the five shipped int16
estimates example_CLSKD/*/s0_estimate.wav written by eval.py:57-96 — and (b) the fp32 CPU oracle
(oracle/asteroid_cpu.py).  Tolerances: int16 estimates within 2 LSB with >= 99 % bit-exact
samples (the oracle's own bar against the WAVs); float estimate vs oracle max |diff| <= 1e-4 of
the peak (fp32 on both sides, different summation orders)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import asteroid_cpu as A

pytestmark = pytest.mark.gpu
DEV = "cuda"
IDS = ["606", "1038", "1132", "1431", "2158"]


def _model():
    from clskd.asteroid import DCCRNet_mini, load_conf
    return DCCRNet_mini.from_pretrained(load_conf(golden("asteroid_mini.npz"))).to(DEV)


def test_shipped_estimates_reproduced():
    from clskd.asteroid import enhance
    fx = golden("asteroid_mini.npz")
    ex = golden("examples.npz")
    model = _model()  # train mode, as eval.py leaves it
    mixes = [torch.from_numpy(A.mixture_from_wav(fx[i + "/mixture"])).to(DEV) for i in IDS]
    outs = enhance(model, mixes)
    sd = A.state_dict_from_fixture(fx)
    for i, mix, est in zip(IDS, mixes, outs):
        q = A.to_pcm16(est.cpu().numpy())
        d = np.abs(q - ex[i + "/est"].astype(np.int64))
        assert d.max() <= 2 and np.mean(d == 0) >= 0.99, (i, d.max(), np.mean(d == 0))
        if i == "606":  # float output vs the oracle on one utterance
            with torch.no_grad():
                ref = A.forward(sd, mix.cpu()[None], train=True)[0].numpy()
            got = model(mix[None])[0, 0].detach().cpu().numpy()
            assert np.abs(got - ref).max() <= 1e-4 * np.abs(ref).max()


def test_eval_mode_and_batching():
    """model.eval(): running statistics, so a batch equals its rows run one by one; against the
    oracle's eval-mode forward."""
    fx = golden("asteroid_mini.npz")
    model = _model().eval()
    rows = np.stack([A.mixture_from_wav(fx[i + "/mixture"])[:48000] for i in IDS[:3]])
    x = torch.from_numpy(rows).to(DEV)
    with torch.no_grad():
        yb = model(x)[:, 0].cpu().numpy()
        y1 = np.stack([model(x[j:j + 1])[0, 0].cpu().numpy() for j in range(3)])
        ref = A.forward(A.state_dict_from_fixture(fx), torch.from_numpy(rows), train=False).numpy()
    np.testing.assert_allclose(yb, y1, rtol=0, atol=1e-6 * np.abs(y1).max())
    assert np.abs(yb - ref).max() <= 1e-4 * np.abs(ref).max()
