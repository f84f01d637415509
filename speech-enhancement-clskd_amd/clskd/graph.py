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
import os

import torch

from . import ops
from .distill import KnowledgeDistillation


def _bn_buffers(kd):
    # teacher, student and ABF BatchNorms
    return [b for n, b in kd.named_buffers()
            if n.endswith(("running_mean", "running_var", "num_batches_tracked"))]


class StepGraph:
    # capture in clskd_step's teacher_ahead layout (the spectrum on the teacher stream; replays
    # by AheadStepExecutor)
    ahead_layout = False

    def __init__(self, kd, X, y, warmup=1):
        from .distill import SPKDDistillation
        if not isinstance(kd, (KnowledgeDistillation, SPKDDistillation)):
            raise TypeError("StepGraph captures a clskd.distill.KnowledgeDistillation (C2) or "
                            "SPKDDistillation (C4) step")
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
        if getattr(self.kd, "abf_reinit", "step") != "step":  # C4 (SPKD) has no ReviewKD modules
            mods += [self.kd.review_encoder, self.kd.review_decoder]
        return [p for m in mods for p in m.parameters()]

    def _sig(self):
        # the baked parameter list is fixed per capture (module trees do not change): resolved
        # once, so a replay's check is one pass over the tensors (no module traversal)
        ps = getattr(self, "_baked_ps", None)
        if ps is None or getattr(self, "_baked_for", None) != self.captures:
            ps = self._baked_ps = tuple(self._baked())
            self._baked_for = self.captures
        return tuple([(p.data_ptr(), p._version) for p in ps])

    keep_graph = False

    def _capture(self):
        self._release()
        dev = self.X.device
        # the step's side streams exist before any helper stream: HIP hands a process's few
        # hardware queues (GPU_MAX_HW_QUEUES = 4) to streams in creation order, and the eager
        # schedule's four streams must not share one (measured: a shared queue serialises two
        # of the replayed branches, 6.5 vs 5.6 ms per C2 step)
        from .distill import _side_stream
        for w in (0, 1, 2):
            _side_stream(dev, w)
        cur = torch.cuda.current_stream(dev)
        # warm-up populates K tables and packed weights outside the graph; BN running statistics
        # are restored afterwards so capture leaves the model state as it found it
        saved = [b.clone() for b in _bn_buffers(self.kd)]
        s = ops.capture_stream(dev)  # prepared: warm-up and capture take the same conv paths
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
        g = torch.cuda.CUDAGraph(keep_graph=True) if self.keep_graph else torch.cuda.CUDAGraph()
        scope = self._new_scope(s)
        self._tagging(True)
        prev_ahead = getattr(self.kd, "teacher_ahead", False)
        self.kd.teacher_ahead = self.ahead_layout
        try:
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                self.out = self.kd.training_step((self.X, self.y), return_parts=True)
        finally:
            scope.end()
            self._tagging(False)
            self.kd.teacher_ahead = prev_ahead
        self.graph = g
        self.sig = self._sig()
        self.captures += 1
        self._after_capture()

    def _after_capture(self):
        pass

    def _new_scope(self, s):
        """The stream-K workspaces of the capture about to start (ops.CaptureScope): one per stream
        the step launches on; the previous capture's (its graph is being replaced) are freed."""
        from .distill import _side_stream
        old = getattr(self, "_scope", None)
        if old is not None:
            old.free()
        dev = self.X.device
        self._scope = ops.CaptureScope([s] + [_side_stream(dev, w) for w in (0, 1, 2)])
        return self._scope

    def _tagging(self, on):
        pass

    def _release(self):
        pass

    def _replay(self):
        self.graph.replay()

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
        self._replay()
        return self.out["loss"]


class StepExecutor(StepGraph):
    """StepGraph replayed by the library's C++ step executor (clskd_exec_launch, include/clskd.h)
    instead of hipGraphLaunch: the captured nodes are re-launched with their captured arguments
    on `nstreams` HIP streams along the graph's dependency edges, so the step keeps the eager
    schedule's concurrency (ROCm's graph executor runs the branches one after another: 7.3 vs
    5.6 ms per C2 step) while the host issues a step in about a millisecond instead of the
    4-5 ms of the Python launch path.  Bitwise equal to eager launch (same kernels, arguments and
    dependency order; tests/test_gpu_parity.py)."""

    keep_graph = True

    def __init__(self, kd, X, y, warmup=1, nstreams=None, ahead_layout=False):
        if nstreams is None:  # diagnostic override: CLSKD_EXEC_STREAMS (1 = serial replay)
            nstreams = int(os.environ.get("CLSKD_EXEC_STREAMS", "4"))
        self.nstreams = nstreams
        self.ahead_layout = ahead_layout
        self._ex = None
        super().__init__(kd, X, y, warmup)

    def _tagging(self, on):
        """While capturing: after every library call report its stream (index 0 = the capture
        stream, 1/2/3 = the step's student / ReviewKD-encoder / teacher streams) so the
        executor replays each node on the stream the schedule put it on."""
        from . import _lib
        from .distill import _side_stream
        lib = _lib.load()
        if not on:
            _lib.TAG_HOOK = None
            return
        lib.clskd_exec_tag_reset()
        dev = self.X.device
        idx = {_side_stream(dev, w).cuda_stream: i + 1 for i, w in enumerate((0, 1, 2))}
        raw = _lib.stream_ptr

        def hook():
            s = raw()
            lib.clskd_exec_tag(s, idx.get(s, 0))

        _lib.TAG_HOOK = hook

    def _after_capture(self):
        import ctypes as C
        from . import _lib
        from .distill import _side_stream
        lib = _lib.load()
        h = C.c_void_p()
        # the step's own side streams (student, ReviewKD-encoder, teacher): same hardware queues
        dev = self.X.device
        side = (C.c_void_p * 3)(*[_side_stream(dev, w).cuda_stream for w in (0, 1, 2)])
        own = os.environ.get("CLSKD_EXEC_OWN_STREAMS") == "1"  # A/B: the executor's own streams
        tags = os.environ.get("CLSKD_EXEC_TAGS", "1") == "1"  # A/B: capture-time stream tags
        _lib.check(lib.clskd_exec_create(C.c_void_p(self.graph.raw_cuda_graph()), self.nstreams,
                                         side if (self.nstreams == 4 and not own) else None,
                                         1 if tags else 0, C.byref(h)),
                   "exec_create")
        self._ex = h
        info = (C.c_int32 * 16)()
        _lib.check(lib.clskd_exec_info(h, info, 16), "exec_info")
        self.info = dict(nodes=info[0], kernels=info[1], memsets=info[2], memcpys=info[3],
                         empty=info[4], waits=info[5], records=info[6], program=info[7],
                         per_stream=list(info[8:8 + self.nstreams]))

    def _release(self):
        if getattr(self, "_ex", None) is not None:
            from . import _lib
            torch.cuda.synchronize()  # no launch of this executor may still be queued
            _lib.load().clskd_exec_destroy(self._ex)
            self._ex = None

    # Replays in flight on the device at most (CLSKD_EXEC_INFLIGHT, 0 = unbounded): before a
    # launch the host waits for the end of the replay `inflight` launches back.  The executor
    # enqueues a step in ~1 ms; unthrottled the host runs many steps ahead until a hardware
    # queue's ring is full, and then blocks inside a launch in program order while the other
    # streams' queues drain (head-of-line blocking); bounded, it waits at a step boundary.
    inflight = int(os.environ.get("CLSKD_EXEC_INFLIGHT", "2"))

    def _throttle(self):
        import collections
        import time
        q = self.__dict__.setdefault("_done_q", collections.deque())
        t0 = time.perf_counter()
        while self.inflight > 0 and len(q) >= self.inflight:
            q.popleft().synchronize()
        # host time spent waiting here (not enqueue work): bench subtracts it
        self.throttle_s = getattr(self, "throttle_s", 0.0) + time.perf_counter() - t0

    def _mark_done(self):
        if self.inflight > 0:
            ev = torch.cuda.Event()
            ev.record()
            self._done_q.append(ev)

    def _replay(self):
        from . import _lib
        self._throttle()
        _lib.check(_lib.load().clskd_exec_launch(self._ex, _lib.stream_ptr()), "exec_launch")
        self._mark_done()

    def census(self):
        """One replay of the captured step in program order on the current stream with every
        kernel node event-timed (clskd_exec_census): {host function: [launches, total ms]} — the
        isolated per-kernel view of a serialised step, over ALL kernels (library and torch).
        A real step; synchronises."""
        return exec_census(self._ex, self.info["kernels"])

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass


def exec_census(handle, nkernels):
    import ctypes as C
    from . import _lib
    fns = (C.c_void_p * nkernels)()
    ms = (C.c_float * nkernels)()
    n = C.c_int32(0)
    _lib.check(_lib.load().clskd_exec_census(handle, _lib.stream_ptr(), nkernels, fns, ms,
                                             C.byref(n)), "exec_census")
    out = {}
    for i in range(n.value):
        a = out.setdefault(fns[i], [0, 0.0])
        a[0] += 1
        a[1] += float(ms[i])
    return out


def kernel_name(fn):
    """Demangled name of a kernel host function (clskd_kernel_name)."""
    import ctypes as C
    from . import _lib
    buf = C.create_string_buffer(4096)
    n = _lib.load().clskd_kernel_name(C.c_void_p(fn), buf, 4096)
    return buf.value.decode() if n >= 0 else hex(fn or 0)


class AheadStepExecutor:
    """The C2 step replayed by the C++ executor with clskd_step's teacher_ahead overlap: step
    i + 1's frozen-teacher chain runs while step i's ReviewKD / Gram / loss tail finishes.  Two
    StepExecutors, each captured in the ahead layout with static buffers of its own, alternate;
    an executor's teacher stream does not wait for the fork (the caller's stream, behind the
    previous step's join) but for the end of its OWN previous replay — the last reader of its
    buffers — and then takes the new batch on that stream (clskd_exec_launch_ahead).  Every
    other branch forks from the caller's stream as before, so BatchNorm running statistics, ABF
    re-draws and the loss stay step-ordered: the results are those of back-to-back eager steps
    (tests/test_gpu_parity.py).  Host enqueue: one C-ABI call per step instead of ~140 Python
    launches.

        step = AheadStepExecutor(kd, X0, y0)
        loss = step(X, y)      # inputs resident on the device; loss: that replay's output slot
    """

    def __init__(self, kd, X, y, warmup=1):
        self.ex = [StepExecutor(kd, X, y, warmup, ahead_layout=True) for _ in range(2)]
        if self.ex[0].nstreams != 4:
            raise ValueError("AheadStepExecutor needs the four-stream replay")
        if os.environ.get("CLSKD_EXEC_OWN_STREAMS") == "1":
            # the batch copy below is ordered only with the step's own teacher stream (executor
            # stream 3 when the executor replays on the step's streams)
            raise ValueError("AheadStepExecutor replays on the step's own streams "
                             "(unset CLSKD_EXEC_OWN_STREAMS)")
        self.done = [torch.cuda.Event(), torch.cuda.Event()]
        self.i = 0
        self.last = self.ex[0]
        self.info = self.ex[0].info

    @property
    def out(self):
        return self.last.out

    def __call__(self, X=None, y=None):
        from . import _lib
        from .distill import _side_stream
        e = self.ex[self.i]
        if e._sig() != e.sig:
            raise RuntimeError("AheadStepExecutor: a baked parameter changed; re-create it")
        if X is not None and X.shape != e.X.shape:
            raise ValueError(f"AheadStepExecutor captured inputs of shape {tuple(e.X.shape)}, "
                             f"got {tuple(X.shape)}")
        if y is not None and y.numel() != e.y.numel():
            raise ValueError(f"AheadStepExecutor captured targets of {e.y.numel()} elements, "
                             f"got {tuple(y.shape)}")
        infl = StepExecutor.inflight
        if infl > 0:  # bounded run-ahead (StepExecutor.inflight)
            import time
            self._q = getattr(self, "_q", [])
            t0 = time.perf_counter()
            while len(self._q) >= infl:
                self._q.pop(0).synchronize()
            self.throttle_s = getattr(self, "throttle_s", 0.0) + time.perf_counter() - t0
        dev = e.X.device
        main = torch.cuda.current_stream(dev)
        t = _side_stream(dev, 2)  # the teacher stream: executor stream 3 (capture tag)
        t.wait_event(self.done[self.i])
        if X is not None:
            with torch.cuda.stream(t):
                e.X.copy_(X)
                # the caller's resident batch is read on the teacher stream
                X.record_stream(t)
        if y is not None:
            e.y.copy_(y.reshape(e.y.shape))
        _lib.check(_lib.load().clskd_exec_launch_ahead(e._ex, _lib.stream_ptr(), 1 << 3, None),
                   "exec_launch_ahead")
        self.done[self.i].record(main)
        if infl > 0:
            ev = torch.cuda.Event()
            ev.record(main)
            self._q.append(ev)
        self.last = e
        self.i ^= 1
        return e.out["loss"]

    def census(self, X=None, y=None):
        """StepExecutor.census of the capture the next call would replay (after the batch is
        copied into its static inputs); the alternation is unchanged."""
        torch.cuda.synchronize()
        e = self.ex[self.i]
        if X is not None:
            e.X.copy_(X)
        if y is not None:
            e.y.copy_(y.reshape(e.y.shape))
        return e.census()


class TrainStepGraph(StepGraph):
    """Configuration C3 as one captured step: ``kd.train_step`` — fwd+loss with the autograd
    tape, the HIP backward into the flat gradient buffer, Adam over the flat parameters
    (distill.py:72-148, 202-204) — recorded once and replayed with hipGraphLaunch.  Every replay packs the student's weights from the parameters the
    previous replay's Adam wrote (DCCRN.repack_in_capture) and advances the optimizer's device
    step count (FlatAdam(device_step=True)), so N replays are N training steps, bitwise equal to
    N eager ``train_step`` calls with the same optimizer (tests/test_gpu_train_graph.py).  The
    eager path spends ~16 ms of host time per step issuing ~1,000 launches; a replay is one
    hipGraphLaunch.

    Multi-rank (round 6): the gradient all-reduce is not captured.  With a process group of more
    than one rank (or ``collective=True``) the capture holds fwd+loss and the backward only; every
    replay is followed by the one flat-gradient all-reduce (clskd.train.allreduce_grads: RCCL,
    gloo in tests) and the Adam launch, issued on the caller's stream — the eager step's order, so
    a replayed step is bitwise the eager ``train_step`` (tests/test_gpu_bench_ddp.py).  Captures
    use torch's thread-local capture mode, so the process group's watchdog thread may query its
    own streams while the step is being recorded.

        flat = FlatParams(kd.student); opt = FlatAdam(flat, lr=..., device_step=True)
        step = TrainStepGraph(kd, flat, opt, X, y)      # hipGraphLaunch replay
        loss = step(X_next, y_next)        # one training step on the new batch

    TrainStepExecutor replays the same capture with the C++ step executor.  The capture holds
    no memcpy nodes (ops.pack_weight copies with a kernel): ROCm 7.2's
    hipGraphMemcpyNodeGetParams does not return the parameters of the one-dimensional memcpy
    nodes torch's D2D copies record (null destination, garbage extent), and clskd_exec_create
    refuses graphs that hold one.
    """

    def __init__(self, kd, flat, opt, X, y, warmup=1, collective=None, **kw):
        import torch.distributed as dist
        if not getattr(opt, "device_step", False):
            raise ValueError("TrainStepGraph needs FlatAdam(device_step=True): the step count "
                             "must live on the device to be replayed")
        if collective is None:
            collective = dist.is_initialized() and dist.get_world_size() > 1
        self.collective = bool(collective)
        self.flat, self.opt = flat, opt
        super().__init__(kd, X, y, warmup, **kw)

    def _baked(self):
        # the trainable student parameters are the step's state, not baked constants
        trainable = {id(p) for p in self.flat.params}
        return [p for p in super()._baked() if id(p) not in trainable]

    def _run(self):
        if self.collective:  # the captured part: fwd+loss with the tape and the backward
            out = self.kd.forward_with_tape(self.X, self.y)
            self.kd.backward_into(out, self.flat.grad_dict())
            return out["loss"]
        return self.kd.train_step((self.X, self.y), self.flat, self.opt)

    def _finish(self):
        """The uncaptured tail of a multi-rank step (kd.train_step's): all-reduce + Adam."""
        from .train import allreduce_grads
        scale = allreduce_grads(self.flat)
        self.opt.step(grad_scale=scale)

    def _replay(self):
        super()._replay()
        if self.collective:
            self._finish()
        # the replay's Adam rewrote the parameters on the device: advance their version counters
        # (as FlatAdam.step does eagerly) so caches keyed on (data_ptr, _version) — the student's
        # packed weights, DCCRN._packed — rebuild on the next eager forward instead of serving
        # weights packed before this replay
        self.flat.bump_versions()

    def census(self):
        """StepExecutor.census of the training step (TrainStepExecutor); the replayed Adam (one
        rank) rewrote the parameters: their versions advance as after any replay."""
        out = super().census()
        self.flat.bump_versions()
        return out

    def _capture(self):
        self._release()
        dev = self.X.device
        from .distill import _side_stream
        for w in (0, 1, 2):
            _side_stream(dev, w)
        cur = torch.cuda.current_stream(dev)
        # warm-up (tables, index maps, caches) restores every piece of state a step changes:
        # BatchNorm running statistics, the parameters, Adam's moments and step count
        state = _bn_buffers(self.kd) + self.opt.state()
        saved = [t.clone() for t in state]
        s = ops.capture_stream(dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self._run()
                if self.collective:
                    self._finish()
        cur.wait_stream(s)
        torch.cuda.synchronize(dev)
        with torch.no_grad():
            for t, v in zip(state, saved):
                t.copy_(v)
        self.graph = None
        g = torch.cuda.CUDAGraph(keep_graph=True) if self.keep_graph else torch.cuda.CUDAGraph()
        student = self.kd.student
        student.repack_in_capture = True
        scope = self._new_scope(s)
        self._tagging(True)
        try:
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                self.out = dict(loss=self._run())
        finally:
            scope.end()
            self._tagging(False)
            student.repack_in_capture = False
        self.graph = g
        self.sig = self._sig()
        self.captures += 1
        self._after_capture()


class TrainStepExecutor(TrainStepGraph, StepExecutor):
    """TrainStepGraph replayed by the C++ step executor (clskd_exec_launch) on the step's four
    streams instead of hipGraphLaunch (whose host cost grows with the node count: ~20 us per node
    on ROCm 7.2, ~1,000 nodes here).

    One replay in flight (CLSKD_EXEC_INFLIGHT, default 1 here): the host enqueues step i + 1 once
    step i has finished.  Letting two training steps overlap measured slower — their memory-bound
    backward kernels contend (19.8-20.0 vs 17.8-18.0 ms per step, profiles/r5_train_split_ab.txt)."""

    inflight = int(os.environ.get("CLSKD_EXEC_INFLIGHT", "1"))


class CapturedCall:
    """Any stream-ordered device computation ``fn(*inputs)`` captured once and replayed by the
    step executor (clskd_exec_launch) — e.g. the B=1 eval forward of configuration C1, whose
    ~70 small launches a Python host cannot issue as fast as the device runs them.

        cc = CapturedCall(lambda x: student(x, is_feat=True), x_static)
        y = cc(x_new)          # copies into the static input, replays; y is a static output

    The output (any tensor / tuple / dict of tensors returned by fn) is overwritten by the next
    replay.  Parameters baked into the capture must not change (re-create the object if they do).
    """

    def __init__(self, fn, *inputs, warmup=1, nstreams=1):
        import ctypes as C
        from . import _lib
        self.inputs = [t.detach().clone() for t in inputs]
        dev = self.inputs[0].device
        cur = torch.cuda.current_stream(dev)
        s = ops.capture_stream(dev)
        s.wait_stream(cur)
        with torch.cuda.stream(s), torch.no_grad():
            for _ in range(warmup):
                fn(*self.inputs)
        cur.wait_stream(s)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        self._scope = ops.CaptureScope([s])
        try:
            with torch.cuda.graph(self.graph, stream=s, capture_error_mode="thread_local"), \
                    torch.no_grad():
                self.out = fn(*self.inputs)
        finally:
            self._scope.end()
        lib = _lib.load()
        h = C.c_void_p()
        _lib.check(lib.clskd_exec_create(C.c_void_p(self.graph.raw_cuda_graph()), nstreams, None,
                                         0, C.byref(h)), "exec_create")
        self._ex = h
        info = (C.c_int32 * 16)()
        _lib.check(lib.clskd_exec_info(h, info, 16), "exec_info")
        self.info = dict(nodes=info[0], kernels=info[1], waits=info[5])

    def __call__(self, *inputs):
        from . import _lib
        for dst, src in zip(self.inputs, inputs):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src.reshape(dst.shape))
        _lib.check(_lib.load().clskd_exec_launch(self._ex, _lib.stream_ptr()), "exec_launch")
        return self.out

    def __del__(self):
        try:
            if getattr(self, "_ex", None) is not None:
                from . import _lib
                torch.cuda.synchronize()
                _lib.load().clskd_exec_destroy(self._ex)
                self._ex = None
        except Exception:
            pass
