"""hipGraph capture of one CLSKD fwd+loss step (the launch-bound host side of distill.py:72-148).

A step is ~200 kernel launches on two streams (teacher on the caller's stream, student on the
side stream, joined before the ReviewKD / Gram / MRSTFT tail).  Eagerly, the Python host spends
~40 us per conv launch building descriptors, so the GPU idles while the student forward is
being enqueued.  ``StepGraph`` records the whole step — ABF re-initialisation (torch's
graph-safe Philox RNG), weight repacking of re-drawn ABF modules, both forwards with their
BN running-stat updates, the batched Gram, SPKD finalize and MRSTFT — once, and replays it with
one ``hipGraphLaunch`` per step.  Every replay recomputes the step from the static input
buffers; nothing is cached between replays except the packed weights of modules whose
parameters did not change (checked on every call: a changed teacher / student / ABF parameter
triggers a re-capture).

Usage::

    step = StepGraph(kd, X, y)          # warm-up (BN running stats restored) + capture
    loss = step(X_next, y_next)         # copy into the static inputs, replay
    parts = step.out                    # static output dict (overwritten by the next replay)
"""
import torch

from .distill import KnowledgeDistillation


def _bn_buffers(kd):
    # teacher, student and ABF BatchNorms
    return [b for n, b in kd.named_buffers()
            if n.endswith(("running_mean", "running_var", "num_batches_tracked"))]


class StepGraph:
    def __init__(self, kd, X, y, warmup=1):
        if not isinstance(kd, KnowledgeDistillation):
            raise TypeError("StepGraph captures a clskd.distill.KnowledgeDistillation step")
        if not X.is_cuda:
            raise RuntimeError("StepGraph needs device-resident inputs")
        self.kd = kd
        self.X = X.detach().clone()
        self.y = y.detach().clone()
        self.warmup = warmup
        self.graph = None
        self.out = None
        self.captures = 0
        self._capture()

    # parameters whose packed forms are baked into the graph (ABF modules re-drawn inside the
    # graph each step are excluded: their re-init and repack are recorded)
    def _baked(self):
        mods = [self.kd.teacher, self.kd.student]
        if self.kd.abf_reinit != "step":
            mods += [self.kd.review_encoder, self.kd.review_decoder]
        return [p for m in mods for p in m.parameters()]

    def _sig(self):
        return tuple((p.data_ptr(), p._version) for p in self._baked())

    def _capture(self):
        dev = self.X.device
        cur = torch.cuda.current_stream(dev)
        # warm-up populates K tables and packed weights outside the graph; BN running statistics
        # are restored afterwards so capture leaves the model state as it found it
        saved = [b.clone() for b in _bn_buffers(self.kd)]
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s), torch.no_grad():
            for _ in range(self.warmup):
                self.kd.training_step((self.X, self.y))
        cur.wait_stream(s)
        torch.cuda.synchronize(dev)
        with torch.no_grad():
            for b, v in zip(_bn_buffers(self.kd), saved):
                b.copy_(v)
        self.graph = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.out = self.kd.training_step((self.X, self.y), return_parts=True)
        self.graph = g
        self.sig = self._sig()
        self.captures += 1

    def __call__(self, X=None, y=None):
        if self._sig() != self.sig:
            self._capture()
        if X is not None:
            if X.shape != self.X.shape:
                raise ValueError(f"StepGraph captured inputs of shape {tuple(self.X.shape)}, "
                                 f"got {tuple(X.shape)}")
            self.X.copy_(X)
        if y is not None:
            self.y.copy_(y.reshape(self.y.shape))
        self.graph.replay()
        return self.out["loss"]
