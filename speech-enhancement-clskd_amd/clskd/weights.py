"""Deterministic parameter recipe for DCCRN teacher/student and the ReviewKD ABF modules.

Parity needs the reference model, the CPU oracle and the HIP path to run on identical weights
without committing multi-MB weight files.  Every parameter is drawn from its own numpy stream
``default_rng([seed, crc32(name)])`` so a value depends only on (seed, key, shape), never on
iteration order.  Keys are the reference's own ``state_dict`` keys (``DCCRN.py:63-147``,
``tools_for_model.py:138-330``; ReviewKD keys ``framework.py:226-238`` prefixed with
``"encoder."``/``"decoder."``), so one dict loads into the reference module (fixture generator),
the CPU oracle and ``clskd.DCCRN`` alike.

Distributions (chosen to exercise every term; the reference's own init is zero-bias / unit BN,
which would hide bias and BN-affine bugs):
  * complex conv / convT weights  N(0, 0.05)   (the reference's init std, tools_for_model.py:231,260)
  * conv biases                   N(0, 0.02)
  * BN weight 1+0.1N, bias 0.1N, running_mean 0.1N, running_var 1+0.2U
  * PReLU alpha 0.25 + 0.05N      (nn.PReLU init is 0.25)
  * LSTM / Linear                 U(-1/sqrt(fan), 1/sqrt(fan))   (torch defaults)
  * ABF conv1/conv2               U(-sqrt(3/fan_in), +)  == kaiming_uniform_(a=1) (framework.py:194-195)
  * ABF att conv weight and bias  U(-1/sqrt(fan_in), +)  (nn.Conv2d default bound)
"""
import zlib

import numpy as np


def _rng(seed, name):
    return np.random.default_rng([int(seed), zlib.crc32(name.encode())])


def _f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


def _abf_value(g, name, shape, shapes):
    leaf = name.split(".")[-1]
    if len(shape) == 4:  # conv weight [out, in, kh, kw]
        fan_in = shape[1] * shape[2] * shape[3]
        k = 1.0 / np.sqrt(fan_in) if ".att_conv." in name else np.sqrt(3.0 / fan_in)
        return _f32(g.uniform(-k, k, shape))
    if ".att_conv." in name and leaf == "bias":
        w = shapes[name.rsplit(".", 1)[0] + ".weight"]
        k = 1.0 / np.sqrt(int(w[1]) * int(w[2]) * int(w[3]))
        return _f32(g.uniform(-k, k, shape))
    if leaf == "weight":  # BatchNorm affine
        return _f32(1.0 + 0.1 * g.standard_normal(shape))
    if leaf == "bias":
        return _f32(0.1 * g.standard_normal(shape))
    raise KeyError(f"no ABF recipe for {name} {shape}")


def _value(seed, name, shape, shapes):
    g = _rng(seed, name)
    leaf = name.split(".")[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, np.int64)
    if leaf == "running_mean":
        return _f32(0.1 * g.standard_normal(shape))
    if leaf == "running_var":
        return _f32(1.0 + 0.2 * g.random(shape))
    if ".abfs." in name:
        return _abf_value(g, name, shape, shapes)
    if "_lstm." in name:  # nn.LSTM: U(-1/sqrt(H), 1/sqrt(H)), H = rows/4
        k = 1.0 / np.sqrt(shape[0] // 4)
        return _f32(g.uniform(-k, k, shape))
    if "_trans." in name:  # nn.Linear: bound 1/sqrt(in_features) for weight and bias
        w = shapes[name.rsplit(".", 1)[0] + ".weight"]
        k = 1.0 / np.sqrt(int(w[1]))
        return _f32(g.uniform(-k, k, shape))
    if "_conv.weight" in name:
        return _f32(0.05 * g.standard_normal(shape))
    if "_conv.bias" in name:
        return _f32(0.02 * g.standard_normal(shape))
    if leaf == "weight" and shape == (1,):  # PReLU single alpha (DCCRN.py:82,126)
        return _f32(0.25 + 0.05 * g.standard_normal(shape))
    if leaf == "weight" and len(shape) == 1:  # BatchNorm affine
        return _f32(1.0 + 0.1 * g.standard_normal(shape))
    if leaf == "bias" and len(shape) == 1:
        return _f32(0.1 * g.standard_normal(shape))
    raise KeyError(f"no recipe for parameter {name} {shape}")


def recipe_state_dict(shapes, seed):
    """shapes: mapping key -> shape (e.g. ``{k: v.shape for k, v in module.state_dict().items()}``).

    Returns {key: np.ndarray}.  The fixed STFT buffers (``stft.*``, ``istft.*``) are skipped:
    both sides derive them from the window definition (tools_for_model.py:15-32).
    """
    shapes = {k: tuple(int(s) for s in v) for k, v in shapes.items()}
    out = {}
    for name, shape in shapes.items():
        if name.startswith("stft.") or name.startswith("istft."):
            continue
        out[name] = _value(seed, name, shape, shapes)
    return out


# Seeds used across fixtures, tests and bench (SURVEY.md §8 d).
TEACHER_SEED = 1001
STUDENT_SEED = 2002
ABF_SEED = 7
DATA_SEED = 20231015


def apply_recipe(module, seed, prefix=""):
    """Load the recipe into a torch module whose state_dict keys (optionally prefixed, e.g.
    ``"encoder."`` for a ReviewKD) are reference keys.  Returns the module."""
    import torch

    shapes = {prefix + k: tuple(v.shape) for k, v in module.state_dict().items()}
    sd = recipe_state_dict(shapes, seed)
    dev = next(iter(module.state_dict().values())).device
    missing, unexpected = module.load_state_dict(
        {k[len(prefix):]: torch.from_numpy(v).to(dev) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith(("stft.", "istft.")) for k in missing), missing
    return module
