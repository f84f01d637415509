"""Benchmark: DCCRN-CLSKD fwd+loss step (configuration C2 of BASELINE.json) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N)

A step = one KnowledgeDistillation.training_step (distill.py:72-148) over B=16 synthetic 16 kHz
4 s noisy/clean pairs per GPU: teacher + student DCCRN forwards (train-mode BN), ReviewKD
fusions, 14 SPKD Gram losses and the MRSTFT base loss; frames = B * T with T = L/100 + 3 = 643.
Each rank processes its own batch shard (weak scaling; forward+loss has no exchange step).
The step runs on four HIP streams (caller | teacher | student -> ReviewKD-decoder | ReviewKD-encoder ->
MRSTFT), launched eagerly (the host enqueues ahead of the device); --graph replays a captured
hipGraph of the same step instead (clskd.graph.StepGraph: every replay recomputes the step from
the batch copied into its static inputs).
Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from clskd import config as cfg  # noqa: E402

METRIC = "frames/sec/GPU DCCRN-CLSKD fwd+loss @16k 4s; SI-SNR parity ±0.01 dB"
METRIC_TRAIN = "frames/sec/GPU DCCRN-CLSKD training step (fwd+loss+bwd+Adam) @16k 4s"
METRIC_SPKD = "frames/sec/GPU DCCRN SPKD-output fwd+loss (distill_SPKD.py) @16k 4s"
B_SPKD = 32  # config C4: batch 32 x 4 s
PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix peak (f32-in MFMA), dense
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (no sparsity)
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
B_PER_GPU = 16
NBATCH = 4
# per-kernel HBM traffic of the PMC passes (tools/pmc_traffic.py): the C2 leg's, and the C3 leg's
# own passes (round 6: a C3 line never borrows the C2 file's same-named, different-shape launches)
TRAFFIC_FILE = "r6_pmc_traffic.json"
TRAFFIC_FILE_TRAIN = "r6_train_pmc_traffic.json"
L = 64000


def _range_push(name):
    torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds of torch


def _range_pop():
    torch.cuda.nvtx.range_pop()


def dispatch_span_us(dev, n=64):
    """Event overhead of one event-timed launch: what an event pair around a launch measures
    beyond the kernel's own duration (command-processor packet processing and wave launch;
    rocprofv3's kernel-trace duration excludes it).  The SMALLEST span of n back-to-back
    1-element fills (after one warm-up): overhead plus a near-empty kernel.  Traced runs of this
    round put the census spans 5.4-5.6 us above rocprof's durations of the same launches and a
    fill's span 5.7 us above its own duration (profiles/README.md); a calibration against
    dispatch-attached events (hipExtLaunchKernel) was tried and dropped: those events add packets
    of their own and read 0-10 us depending on the tracer."""
    from clskd import ops
    t = torch.empty(1, device=dev)
    ops.fill(t, 0.0)
    evs = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.fill(t, 0.0)
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize(dev)
    return float(np.min([a.elapsed_time(b) for a, b in evs])) * 1e3


def launches_per_step(kd, X, y):
    """Kernel launches of one step: the step captured once (clskd.graph.StepExecutor, after the
    timed region) and its kernel nodes counted — library and torch kernels alike."""
    from clskd.graph import StepExecutor
    ex = StepExecutor(kd, X, y)
    n = dict(kernels=ex.info["kernels"], memsets=ex.info["memsets"], memcpys=ex.info["memcpys"])
    ex._release()
    del ex
    return n


def build_kd(dev, abf_reinit, precision="fp32", spkd=False):
    from clskd.distill import KnowledgeDistillation, SPKDDistillation
    from clskd.model import DCCRN
    from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, apply_recipe
    teacher = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.TEACHER), TEACHER_SEED)
    student = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED)
    if spkd:
        return SPKDDistillation(teacher, student, precision=precision).to(dev).train()
    kd = KnowledgeDistillation(teacher, student, abf_reinit=abf_reinit,
                               precision=precision).to(dev).train()
    apply_recipe(kd.review_encoder, ABF_SEED, "encoder.")
    apply_recipe(kd.review_decoder, ABF_SEED, "decoder.")
    return kd


def host_cpu_info():
    """Host CPU model, the machine's logical CPU count, and the CPUs this process may use
    (affinity mask, capped by the cgroup CPU quota: on the GPU box nproc shows the whole
    machine while the job's share is smaller)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            usable = max(1, min(usable, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return model, total, usable


def cpu_baseline(n_timed=10, n_warm=3, spkd=False):
    """The CPU oracle (fp32 PyTorch-CPU restatement of the reference, oracle/ref_cpu.py) timed on
    this host following BASELINE.md §2: every usable host core, the same seeded B=16 x 4 s
    workload as the GPU leg, 3 warm-up steps and the median of 10 timed steps — all full B=16
    steps (round 5 warmed up at B=4, which left the first timed B=16 step cold: 9.5 vs 7.5 s).
    spkd: configuration C4's step (oracle/ref_cpu.spkd_output_step, B=32 x 4 s) instead."""
    from oracle import ref_cpu as R
    from clskd.data import synthetic_pairs
    from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, recipe_state_dict
    model, total, usable = host_cpu_info()
    threads = usable
    torch.set_num_threads(threads)
    pt = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.TEACHER), TEACHER_SEED))
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    pa = R.to_torch_params(recipe_state_dict(
        {**cfg.review_param_shapes("encoder"), **cfg.review_param_shapes("decoder")}, ABF_SEED))
    Bc = B_SPKD if spkd else B_PER_GPU
    noisy, clean = synthetic_pairs(Bc, L, seed=99)
    X, Y = torch.from_numpy(noisy), torch.from_numpy(clean)
    fn = (lambda: R.spkd_output_step(pt, ps, X, Y)) if spkd else (lambda: R.clskd_step(pt, ps, pa, X, Y))
    times = []
    with torch.no_grad():
        for _ in range(n_warm):
            fn()
        for _ in range(n_timed):
            t0 = time.perf_counter()
            fn()
            times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    frames = Bc * cfg.n_frames(L)
    return dict(value=round(frames / med, 2), unit="frames/s", cores=threads, kind="port",
                batch=Bc, host_cpus=total, cpu_model=model,
                step_s=[round(t, 3) for t in times],
                sample=f"oracle/ref_cpu.{'spkd_output_step' if spkd else 'clskd_step'} on the "
                       f"bench workload (B={Bc} x 4 s @16 kHz, "
                       f"same step as the GPU leg): {n_warm} warm-up steps (B={Bc}), median of "
                       f"{n_timed} timed B={Bc} steps, fp32, torch CPU {threads} threads = every "
                       f"CPU this job may use ({total} logical CPUs on the host), {model}")


METRIC_C1 = "frames/sec DCCRN student eval forward, batch 1 (framework.py eval path, no KD)"


def run_c1(args, dev):
    """Configuration C1 (BASELINE.json configs[0]): the student's eval-mode forward (BatchNorm
    running statistics, DCCRN.py:149-240) on one clip, 16000 samples (1 s @16 kHz) and 8000
    samples ("8 kHz 1 s" restated as 8000 samples), as a latency: each
    forward is synchronised.  GPU legs: the Python eager launch path and the same forward
    captured once and replayed by the C++ step executor (clskd.graph.CapturedCall).  CPU leg:
    the oracle's eval forward (oracle/ref_cpu.dccrn_forward(train=False)) on every usable host
    core and on one thread, 3 warm-ups + median of 10."""
    from oracle import ref_cpu as R
    from clskd.data import synthetic_pairs
    from clskd.graph import CapturedCall
    from clskd.model import DCCRN
    from clskd.weights import STUDENT_SEED, apply_recipe, recipe_state_dict
    student = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT),
                           STUDENT_SEED).to(dev).eval()
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    model, total, usable = host_cpu_info()
    legs = {}
    K = max(args.steps, 10)
    for n in (16000, 8000):
        noisy, _ = synthetic_pairs(1, n, seed=5)
        x = torch.from_numpy(noisy).to(dev)
        frames = cfg.n_frames(n)
        fwd = (lambda t: student(t, is_feat=True))
        with torch.no_grad():
            for _ in range(args.warmup):
                fwd(x)
            torch.cuda.synchronize()
            eager = []
            for _ in range(K):
                t0 = time.perf_counter()
                fwd(x)
                torch.cuda.synchronize()
                eager.append(time.perf_counter() - t0)
            ref_out = fwd(x).clone()
        cc = CapturedCall(fwd, x)
        for _ in range(args.warmup):
            cc(x)
        torch.cuda.synchronize()
        ex = []
        for _ in range(K):
            t0 = time.perf_counter()
            cc(x)
            torch.cuda.synchronize()
            ex.append(time.perf_counter() - t0)
        assert torch.equal(cc.out, ref_out), "executor replay differs from the eager forward"
        xc = torch.from_numpy(noisy)
        cpu = {}
        for threads in (usable, 1):
            torch.set_num_threads(threads)
            with torch.no_grad():
                for _ in range(3):
                    R.dccrn_forward(ps, xc, train=False)
                ts = []
                for _ in range(10):
                    t0 = time.perf_counter()
                    o = R.dccrn_forward(ps, xc, train=False)
                    ts.append(time.perf_counter() - t0)
            cpu[threads] = float(np.median(ts))
        rms = float((o["out_wav"].reshape(-1) - ref_out.cpu().reshape(-1)).pow(2).mean().sqrt())
        lat = float(np.median(ex))
        legs[n] = dict(frames=frames, gpu_exec_ms=round(lat * 1e3, 4),
                       gpu_eager_ms=round(float(np.median(eager)) * 1e3, 4),
                       gpu_frames_per_s=round(frames / lat, 1),
                       cpu_ms=round(cpu[usable] * 1e3, 3), cpu_1thread_ms=round(cpu[1] * 1e3, 3),
                       cpu_frames_per_s=round(frames / min(cpu.values()), 1),
                       gpu_over_cpu=round(min(cpu.values()) / lat, 1),
                       kernels=cc.info["kernels"], wav_rms_vs_oracle=rms)
    main_leg = legs[16000]
    best_cpu_ms, best_threads = min((main_leg["cpu_ms"], usable), (main_leg["cpu_1thread_ms"], 1))
    mflop = 7.6e6 * main_leg["frames"]  # SURVEY.md §8 d: 3.79 MMAC/frame
    out = {
        "metric": METRIC_C1, "value": main_leg["gpu_frames_per_s"], "unit": "frames/s",
        "n_gpus": 1, "steps": K, "warmup": args.warmup,
        "ms_per_step": main_leg["gpu_exec_ms"], "higher_is_better": True, "scaling": "none",
        "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (seeded 16 kHz enveloped-sinusoid clean + noise); recipe weights",
        "config": {"workload": "C1: student DCCRN eval forward (running-stat BN), batch 1, "
                               "16000 samples (value) and 8000 samples; latency per forward",
                   "legs": {str(k): v for k, v in legs.items()}},
        "roofline": {"bound": "latency", "achieved": round(mflop / (main_leg["gpu_exec_ms"] * 1e-3) / 1e12, 4),
                     "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(mflop / (main_leg["gpu_exec_ms"] * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 6),
                     "traffic": None,
                     "note": "one 1 s clip is ~70 dependent small launches: the forward is bound by "
                             "launch latency and the 163-step LSTM recurrence, not by MFMA or HBM"},
        "cpu_baseline": {"value": round(main_leg["frames"] / (best_cpu_ms * 1e-3), 1),
                         "unit": "frames/s", "cores": best_threads,
                         "kind": "port", "cpu_model": model, "host_cpus": total,
                         "sample": "oracle/ref_cpu.dccrn_forward(train=False), B=1 x 16000 samples, "
                                   f"3 warm-ups + median of 10, fp32; {usable} threads "
                                   f"{main_leg['cpu_ms']} ms, 1 thread {main_leg['cpu_1thread_ms']} ms "
                                   "(the faster one is the value: a 1 s clip is too small to "
                                   "spread over many cores)"},
    }
    print(json.dumps(out))


METRIC_C5 = "frames/sec streaming DCCRN student inference (6.25 ms hops, 30 s @16 kHz per stream)"


def run_c5(args, dev):
    """Configuration C5 (BASELINE.json configs[4]): streaming inference of the student (eval BN)
    over 30 s @ 16 kHz per stream, 100-sample (6.25 ms) hops, one clskd_stream_hop launch per hop
    for every stream at once (clskd.streaming.FusedStreamingDCCRN; pinned to the oracle's offline
    eval forward by tests/test_gpu_streaming.py).  A step = one hop of all `--streams` streams over
    input already resident in HBM; value = frames (hops x streams) per second over the timed
    hops; the hop kernel's duration is HIP-event-timed on the launching stream.  Also measured:
    one stream's hop (the latency view) and the per-layer hipGraph hop.  CPU leg: the oracle's
    OFFLINE eval forward on one 30 s clip (the reference has no streaming path; the same MACs
    per frame), 1 warm-up + median of 3."""
    from oracle import ref_cpu as R
    from clskd.data import synthetic_pairs
    from clskd.model import DCCRN
    from clskd.streaming import HOP, FusedStreamingDCCRN, StreamingDCCRN
    from clskd.weights import STUDENT_SEED, apply_recipe, recipe_state_dict
    student = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT),
                           STUDENT_SEED).to(dev).eval()
    S = args.streams
    L = 480000
    nh = L // HOP
    K = min(max(args.steps, 200), nh - args.warmup)  # hops timed (a step = one hop of every stream)
    noisy, _ = synthetic_pairs(S, L, seed=3)
    x = torch.from_numpy(noisy).to(dev)
    legs = {}

    def timed(s, n_streams):
        for t in range(args.warmup):
            s.step(x[:n_streams, t * HOP:(t + 1) * HOP])
        torch.cuda.synchronize()
        evs = []
        t0 = time.perf_counter()
        for t in range(args.warmup, args.warmup + K):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.x_in.copy_(x[:n_streams, t * HOP:(t + 1) * HOP])
            e0.record()
            s._hop()
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        return el / K, kern_ms

    fs = FusedStreamingDCCRN(student, S)
    per_hop, kern_ms = timed(fs, S)
    legs["fused_all"] = dict(streams=S, ms_per_hop=round(per_hop * 1e3, 4), kernel_ms=round(kern_ms, 4),
                             frames_per_s=round(S / per_hop, 1),
                             real_time_factor=round(per_hop / (HOP / 16000.0), 5))
    f1 = FusedStreamingDCCRN(student, 1)
    p1, k1 = timed(f1, 1)
    legs["fused_1"] = dict(streams=1, ms_per_hop=round(p1 * 1e3, 4), kernel_ms=round(k1, 4),
                           real_time_factor=round(p1 / (HOP / 16000.0), 5))
    g1 = StreamingDCCRN(student, 1, graph=True)
    for t in range(4):
        g1.step(x[:1, t * HOP:(t + 1) * HOP])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(4, 4 + K):
        g1.step(x[:1, t * HOP:(t + 1) * HOP])
    torch.cuda.synchronize()
    pg = (time.perf_counter() - t0) / K
    legs["graph_1"] = dict(streams=1, ms_per_hop=round(pg * 1e3, 4),
                           real_time_factor=round(pg / (HOP / 16000.0), 5))
    # CPU: the oracle's offline eval forward over one 30 s clip
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    model, total, usable = host_cpu_info()
    torch.set_num_threads(usable)
    xc = torch.from_numpy(noisy[:1])
    with torch.no_grad():
        R.dccrn_forward(ps, xc, train=False)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            R.dccrn_forward(ps, xc, train=False)
            ts.append(time.perf_counter() - t0)
    cpu_s = float(np.median(ts))
    frames_clip = cfg.n_frames(L)
    value = S / per_hop
    # roofline of the hop kernel: per stream and hop 3.8 MMAC (SURVEY.md §8 d, 7.6 MFLOP) on fp32
    # v_pk_fma_f32, one 512-thread workgroup per stream.  The hop is bound by VALU instruction
    # issue, not by FLOPs: profiles/r3_stream_c5_sq_counters.json counts 137.3 k VALU wave-
    # instructions per hop (8 waves), i.e. 34.3 k per SIMD; a wave64 VALU instruction holds its
    # SIMD 4 cycles (16 lanes), so one hop cannot take less than 137 k cycles = 57 us at 2.4 GHz
    # whatever its FLOP count.  Priced as achieved VALU issue rate per SIMD (instructions per
    # cycle) against that 0.25 ceiling; the FLOP rate against the fp32 vector peak is the note.
    fl = 7.6e6 * S / (kern_ms * 1e-3) / 1e12
    valu_per_hop, clk = 137344.0, 2.4e9
    cus = min(S, 256)
    issue = valu_per_hop * S / (kern_ms * 1e-3 * clk * 4 * cus)
    out = {
        "metric": METRIC_C5, "value": round(value, 1), "unit": "frames/s", "n_gpus": 1,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(per_hop * 1e3, 4),
        "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (seeded 16 kHz enveloped-sinusoid clean + noise); recipe weights",
        "config": {"workload": f"C5: {S} concurrent streams x 30 s @16 kHz, student eval BN, one "
                               "clskd_stream_hop launch per 6.25 ms hop (algorithmic latency 9 hops "
                               "= 56.25 ms)", "legs": legs},
        "roofline": {"bound": "valu_issue", "kernel": "stream_hop_kernel", "achieved": round(issue, 4),
                     "peak": 0.25, "unit": "VALU wave-instructions / cycle / SIMD",
                     "frac": round(issue / 0.25, 4), "traffic": None,
                     "note": "137.3 k VALU wave-instructions per hop and stream "
                             "(profiles/r3_stream_c5_sq_counters.json) on the stream's CU at 2.4 GHz; "
                             "a wave64 VALU op holds a SIMD 4 cycles (ceiling 0.25/cycle); the rest "
                             "of the hop is load latency (SQ_WAIT_ANY 53 % of wave cycles). FLOP view: "
                             f"{round(fl, 3)} TF/s = {round(fl / PEAK_F32_MFMA_TFLOPS, 4)} of the fp32 "
                             f"vector peak; weights from L2 {round(3.2e6 * S / (kern_ms * 1e-3) / 1e12, 2)} TB/s"},
        "cpu_baseline": {"value": round(frames_clip / cpu_s, 1), "unit": "frames/s",
                         "cores": usable, "kind": "port", "cpu_model": model, "host_cpus": total,
                         "sample": "oracle/ref_cpu.dccrn_forward(train=False) offline over one 30 s "
                                   f"clip ({frames_clip} frames), 1 warm-up + median of 3, "
                                   f"{usable} threads: {round(cpu_s * 1e3, 1)} ms"},
    }
    print(json.dumps(out))


def spawn_cmd(n, argv, port):
    """The launcher command of a standalone multi-GPU run: torch.distributed.run, one rank per
    GPU of this node, rendezvous on 127.0.0.1, each rank running this file with the same args."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def spawn_ranks(n, argv):
    """Start the ranks as a child process group (no exec: nothing here has initialised the GPU,
    but a child keeps the launcher's exit code ours to return).  Returns the worst exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    return subprocess.run(spawn_cmd(n, argv, port), env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-steps", type=int, default=None,
                    help="timed CPU-oracle steps (median; BASELINE.md §2: 10 for C2; C4 default 3 "
                         "timed after 1 warm-up: a bounded sample of its B=32 step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--abf-reinit", default="step", choices=["step", "once"])
    ap.add_argument("--launch", default=None, choices=["exec", "eager", "graph"],
                    help="default: exec for C2 (one rank), eager for C3 / C4 / multi-rank.  "
                         "C3 (--train) also takes exec / graph (the captured training step, "
                         "clskd.graph.TrainStepExecutor / TrainStepGraph).  eager: launch the "
                         "four-stream schedule from Python every step (host enqueue ~3.9 ms under "
                         "a ~5.3 ms device step); exec: capture the step once and replay it with "
                         "the library's C++ multi-stream executor — with the teacher_ahead "
                         "overlap (two alternating captures, clskd.graph.AheadStepExecutor; "
                         "--no-ahead: one capture, clskd.graph.StepExecutor): ~1.7 ms host "
                         "enqueue, the eager device time; graph: hipGraphLaunch of the capture "
                         "(ROCm's graph executor runs the branches one after another)")
    ap.add_argument("--graph", action="store_true", help="same as --launch graph")
    ap.add_argument("--no-ahead", dest="ahead", action="store_false",
                    help="C2 (eager and exec): start each step's teacher chain after the previous "
                         "step's join.  Default: the teacher chain of step i+1 overlaps step i's tail "
                         "(clskd_step teacher_ahead, bitwise the serial schedule's results; "
                         "measured 0.6-1 %% faster: 5.35/5.37 vs 5.40/5.40 ms, 5.70 vs 5.76 ms)")
    ap.add_argument("--train", action="store_true",
                    help="config C3: the full training step — fwd+loss, HIP backward into the flat "
                         "student gradient, one RCCL all-reduce (N > 1), one Adam launch "
                         "(KnowledgeDistillation.train_step); reported under its own metric")
    ap.add_argument("--spkd", action="store_true",
                    help="config C4: distill_SPKD.py's step (student + teacher full forwards, MRSTFT "
                         "base, one SPKD Gram over the output waveforms) at B=32 x 4 s per GPU; "
                         "reported under its own metric")
    ap.add_argument("--c5", action="store_true",
                    help="config C5: streaming inference, --streams streams x 30 s, one fused "
                         "clskd_stream_hop launch per hop (see run_c5)")
    ap.add_argument("--streams", type=int, default=256, help="C5: concurrent streams")
    ap.add_argument("--c1", action="store_true",
                    help="config C1: the student's eval forward at batch 1 (16000 and 8000 "
                         "samples) as a latency, GPU (eager and executor) beside the CPU oracle")
    ap.add_argument("--precision", default=None, choices=["mixed", "fp16", "fp32"],
                    help="mixed (C2/C3 default): teacher + ReviewKD GEMMs on bf16 MFMA operands (fp32 "
                         "accumulate), student fp32 (C2: its fp32 convs as 3 x bf16 split products); fp16 (C4 default, --spkd only): the teacher on "
                         "IEEE-half operands and fp16 storage; fp32: every GEMM on exact-f32 MFMA")
    args = ap.parse_args()
    if args.precision is None:
        args.precision = "fp16" if args.spkd else "mixed"
    if args.precision == "fp16" and not args.spkd:
        raise SystemExit("--precision fp16 is the C4 (--spkd) teacher mode")

    from clskd import dist as cdist
    rank, world, local_rank = cdist.env_rank()
    if args.gpus > 1 and world == 1:
        # standalone `bench.py --gpus N`: start the N ranks (one process per GPU) before anything
        # here touches the GPU, relay their output (rank 0 prints the JSON line), exit with the
        # launcher's code (non-zero when any rank failed)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    # test-only overrides (tests/test_gpu_bench_ddp.py runs two ranks on the one GPU of a box):
    # CLSKD_DIST_BACKEND=gloo, CLSKD_BENCH_DEVICE=<index> for every rank
    dev_index = int(os.environ.get("CLSKD_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    cdist.init(os.environ.get("CLSKD_DIST_BACKEND", "nccl"), dev)

    from clskd import ops
    from clskd.data import synthetic_pairs
    if args.c1:
        return run_c1(args, dev)
    if args.c5:
        return run_c5(args, dev)
    if args.graph:
        args.launch = "graph"
    if args.spkd and args.train:
        raise SystemExit("--spkd is its own leg (no --train)")
    if args.launch is None:
        # C2: the step captured once and replayed by the C++ executor with the teacher_ahead
        # overlap (clskd.graph.AheadStepExecutor): the eager device schedule at ~0.6 ms of host
        # time per step instead of ~3.9 ms of Python launches (same-box A/B,
        # profiles/r5_exec_ab.txt: 5.28 vs 5.28 ms per step).  C3: the captured training step
        # replayed by the executor, one replay in flight (TrainStepExecutor): 17.8-18.0 ms at
        # ~2.5 ms of host time against 18.15 ms eager with 14 ms of Python launches
        # (profiles/r5_train_split_ab.txt).  Every rank count runs the same launch path (round
        # 6): with N > 1 ranks the C2 step has no exchange, and the C3 replay (fwd+loss +
        # backward) is followed by the flat-gradient all-reduce and the Adam launch
        # (clskd.graph.TrainStepGraph, collective mode)
        args.launch = "exec"
    args.graph = args.launch == "graph"
    bsz = B_SPKD if args.spkd else B_PER_GPU
    kd = build_kd(dev, args.abf_reinit, args.precision, spkd=args.spkd)
    # --ahead: C2 eager steps over resident batches with the teacher chain of step i+1 overlapping
    # step i's tail (clskd_step teacher_ahead; identical results, tests/test_gpu_parity.py)
    kd.teacher_ahead = not args.spkd and not args.train and args.launch == "eager" and args.ahead
    # NBATCH distinct batches resident in HBM; step i consumes batch i % NBATCH
    Xs, Ys = [], []
    for k in range(NBATCH):
        noisy, clean = synthetic_pairs(bsz, L, seed=cdist.shard_seed(1000 + k, rank))
        Xs.append(torch.from_numpy(noisy).to(dev))
        Ys.append(torch.from_numpy(clean).to(dev))
    T = cfg.n_frames(L)

    def _gc_setting():
        # The step's Python launch path allocates short-lived objects only; the long-lived ones
        # (modules, launch plans, descriptors, resident batches, a captured executor) exist by
        # now.  Moving them to Python's permanent GC generation (gc.freeze, the usual setting for
        # a long-running service) keeps the cyclic collector from re-traversing them on every
        # collection.  CLSKD_BENCH_GC=on: plain collector; off: collector disabled (A/B).
        import gc
        mode = os.environ.get("CLSKD_BENCH_GC", "freeze")
        if mode in ("freeze", "off"):
            gc.collect()
            gc.freeze()
        if mode == "off":
            gc.disable()

    executor = None
    if args.train:
        from clskd.train import FlatAdam, FlatParams
        flat = FlatParams(kd.student)
        # the step count on the device for every launch path (a captured step replays it), so
        # eager and replayed steps run the same Adam kernel (bitwise comparable)
        opt = FlatAdam(flat, lr=cfg.learning_rate, device_step=True)

        def eager_step(i):
            return kd.train_step((Xs[i % NBATCH], Ys[i % NBATCH]), flat, opt)
        if args.launch in ("exec", "graph"):
            # the captured training step, replayed by the C++ executor (exec) or hipGraphLaunch
            from clskd.graph import TrainStepExecutor, TrainStepGraph
            if args.launch == "exec":
                executor = captured = TrainStepExecutor(kd, flat, opt, Xs[0], Ys[0])
            else:
                graph = captured = TrainStepGraph(kd, flat, opt, Xs[0], Ys[0])

            def step(i):
                return captured(Xs[i % NBATCH], Ys[i % NBATCH])
        else:
            step = eager_step
    elif args.launch == "eager":
        def step(i):
            # fwd+loss only: no autograd tape (the C3 leg above records and consumes one)
            with torch.no_grad():
                return kd.training_step((Xs[i % NBATCH], Ys[i % NBATCH]), i)
    elif args.launch == "exec":
        from clskd.graph import StepExecutor
        if executor is None:
            if args.spkd:  # C4: the captured two-stream step (round 6), one capture
                executor = StepExecutor(kd, Xs[0], Ys[0])
            elif args.ahead:  # the teacher_ahead overlap, replayed (two alternating captures)
                from clskd.graph import AheadStepExecutor
                executor = AheadStepExecutor(kd, Xs[0], Ys[0])
            else:
                executor = StepExecutor(kd, Xs[0], Ys[0])

        def step(i):
            return executor(Xs[i % NBATCH], Ys[i % NBATCH])

        def eager_step(i):
            with torch.no_grad():
                return kd.training_step((Xs[i % NBATCH], Ys[i % NBATCH]), i)
    else:
        from clskd.graph import StepGraph
        graph = StepGraph(kd, Xs[0], Ys[0])

        def step(i):
            return graph(Xs[i % NBATCH], Ys[i % NBATCH])

    # the last warm-up step times every conv launch (census: which kernel instance dominates,
    # per-kernel table); the timed region then brackets only the dominant instance's launches
    # with HIP events, so the live roofline costs two event records per launch of that kernel
    # The census step runs the same work on ONE stream (distill.serialized_streams), so its
    # per-kernel durations are isolated ones — the view rocprofv3's kernel trace has — and the
    # dominant kernel (largest total isolated time) is the same instance in every run.
    from clskd.distill import serialized_streams
    census = None
    serial_ms = None
    disp_us = dispatch_span_us(dev)
    for i in range(args.warmup):
        last = i == args.warmup - 1 and not args.graph
        if last:
            torch.cuda.synchronize()
            _range_push("clskd_census")
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ops.KernelTimer.start()
            c0.record()
            with serialized_streams():
                (eager_step if args.launch == "exec" else step)(i)
            c1.record()
            census = ops.KernelTimer.stop()
            serial_ms = c0.elapsed_time(c1)
            _range_pop()
        else:
            step(i)
    torch.cuda.synchronize()
    dominant = max(census.items(), key=lambda kv: kv[1][1])[0] if census else None
    census_all, dom_fn = None, None
    if args.launch == "exec":
        # one more untimed step: the captured step replayed in program order on ONE stream with
        # every kernel node event-timed (clskd_exec_census) — the isolated duration of EVERY
        # kernel, library and torch alike; the dominant instance is the one with the largest
        # total, whatever kernel family it is (round 6: the C3 line no longer picks among conv
        # launches only)
        from clskd.graph import kernel_name
        _range_push("clskd_exec_census")
        kc = args.warmup % NBATCH
        census_all = (executor.census(Xs[kc], Ys[kc]) if hasattr(executor, "ex")
                      else executor.census())
        _range_pop()
        conv_of_fn = {fn: nm for nm, fn in ops.KernelTimer.fns.items()}
        dom_fn = max(census_all, key=lambda f: census_all[f][1])
        dominant = conv_of_fn.get(dom_fn) or ops.canonical_kernel_name(kernel_name(dom_fn))
        # live HIP-event timing of the dominant instance inside the executor's launches
        n_dom = census_all[dom_fn][0]
        for e in getattr(executor, "ex", [executor]):
            ops.check(ops.lib().clskd_exec_profile(e._ex, dom_fn, n_dom * args.steps), "exec_profile")

    _gc_setting()
    # ---- timed region: exactly K steps, barrier + sync on both sides --------------------
    cdist.barrier(dev)
    # roctx range (rocprofv3 --marker-trace): tools/region_stats.py splits the kernel trace at it,
    # so the profile's per-kernel averages are those of exactly the timed steps
    _range_push("clskd_timed")
    if args.launch == "eager":
        ops.KernelTimer.start(only=dominant)
    waited0 = getattr(executor, "throttle_s", 0.0) if executor is not None else 0.0
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    host_el = time.perf_counter() - t0  # host enqueue of K steps (no sync inside the loop)
    # an executor bounds its run-ahead (clskd.graph.StepExecutor.inflight): the host time it
    # spent waiting for the device at step boundaries is not enqueue work
    host_wait = (getattr(executor, "throttle_s", 0.0) - waited0) if executor is not None else 0.0
    host_el -= host_wait
    cdist.barrier(dev)
    el = time.perf_counter() - t0
    _range_pop()
    if args.launch == "exec":
        import ctypes
        tot, cnt = ctypes.c_double(0), ctypes.c_int32(0)
        for e in getattr(executor, "ex", [executor]):
            t1, c1 = ctypes.c_double(0), ctypes.c_int32(0)
            ops.check(ops.lib().clskd_exec_profile_read(e._ex, ctypes.byref(t1), ctypes.byref(c1)),
                      "exec_profile_read")
            tot.value += t1.value
            cnt.value += c1.value
        if dominant in census:  # a conv instance: FLOPs from the eager census step
            fl = census[dominant][2] / census[dominant][0]
        else:  # another kernel family: the algorithmic work its wrapper noted (census step)
            w = ops.KernelTimer.work.get(dominant)
            fl = w[2] / w[0] if w else 0.0
        ktimes = {dominant: [cnt.value, tot.value, fl * cnt.value]}
        timing = ("HIP events around every launch of the dominant kernel inside the timed "
                  "region, recorded by the step executor on the kernel's own stream (concurrent "
                  "streams: a launch's event span includes time it shares the CUs); dominant = "
                  "largest total isolated time over EVERY kernel node of one executor census "
                  "replay (clskd_exec_census: the captured step on one stream, each node "
                  "event-timed: all_kernels_isolated)")
        census_steps = 1
    elif (not args.graph):
        ktimes = ops.KernelTimer.stop()
        timing = ("HIP events around every launch of the dominant conv kernel inside the timed "
                  "region (4 concurrent streams: a launch's event span includes time it shares the "
                  "CUs); dominant = largest total isolated time in the census step (the last "
                  "warm-up step run on one stream, every conv launch timed: conv_all_kernels)")
        if census is None:
            census = ktimes
            timing = "HIP events around every conv launch inside the timed region"
        census_steps = 1 if dominant else args.steps
    else:
        # graph nodes carry no timing events: the conv launches are timed with HIP events in an
        # eager pass over the same K batches right after the timed replays (same kernels, shapes)
        ops.KernelTimer.start()
        for i in range(args.steps):
            with torch.no_grad():
                kd.training_step((Xs[i % NBATCH], Ys[i % NBATCH]), i)
        ktimes = ops.KernelTimer.stop()
        timing = ("HIP events around every conv-engine launch of an eager pass over the K timed "
                  "batches (the timed region replays the captured hipGraph)")
        census, census_steps = ktimes, args.steps
    el = cdist.max_over_ranks(el, dev)
    loss_v = float(loss.item())
    param_hashes = None
    if args.train:
        # data-parallel consistency of the benched training step: every rank's student
        # parameters after the last Adam step, hashed (identical on every rank when the gradient
        # all-reduce and the optimizer agree)
        import hashlib
        h = hashlib.sha256(flat.data.detach().cpu().numpy().tobytes()).hexdigest()[:16]
        param_hashes = [h]
        if world > 1:
            param_hashes = [None] * world
            torch.distributed.all_gather_object(param_hashes, h)
    quality = None
    if not args.train and not args.spkd and args.precision == "mixed":
        # quality gate of the metric ("SI-SNR parity ±0.01 dB"): the timed step's student
        # waveform vs the all-fp32 step on the same batch (after the timed region)
        from clskd.tools_for_loss import si_snr
        last = (args.steps - 1) % NBATCH
        src = executor.out if args.launch == "exec" else (graph.out if args.graph else kd.last)
        wav_m = src["student_wav"].clone()
        from clskd import _lib
        with torch.no_grad():
            # the reference leg is the EXACT fp32 path: fp32 MFMA engines even where the benched
            # step runs its fp32 layers as 3 x bf16 split products (CLSKD_F32_SPLIT)
            split = _lib.set_knob("CLSKD_F32_SPLIT", 0)
            s_compute = getattr(kd.student, "compute", None)
            kd.set_precision("fp32")
            o32 = kd.training_step((Xs[last], Ys[last]), 0, return_parts=True)
            kd.set_precision(args.precision)
            _lib.set_knob("CLSKD_F32_SPLIT", split)
            s_m = si_snr(wav_m, Ys[last]).item()
            s_32 = si_snr(o32["student_wav"], Ys[last]).item()
            wav_rms = float((wav_m - o32["student_wav"]).pow(2).mean().sqrt())
        quality = dict(si_snr_db=round(s_m, 6), si_snr_fp32_step_db=round(s_32, 6),
                       si_snr_delta_db=abs(s_m - s_32), student_wav_rms_vs_fp32_step=wav_rms,
                       loss=round(loss_v, 6), loss_fp32_step=round(float(o32["loss"].item()), 6),
                       f32_split_knob=bool(split), student_compute=s_compute,
                       note="timed batch (last step) vs the exact all-fp32 step on the same batch "
                            "(fp32 MFMA engines, no split products); the oracle-pinned full-size "
                            "check is tests/test_gpu_c2_mixed.py")

    step_counts = None
    if world == 1 and not args.train and not args.spkd and not args.graph:
        # after the timed region: one capture of the step, its kernel nodes counted
        step_counts = launches_per_step(kd, Xs[0], Ys[0])
    elif args.train and args.launch == "exec" and executor is not None:
        # the captured training step the executor replays: its kernel nodes
        step_counts = dict(kernels=int(executor.info["kernels"]),
                           memsets=int(executor.info.get("memsets", 0)),
                           memcpys=int(executor.info.get("memcpys", 0)))

    if rank == 0:
        frames = world * bsz * T * args.steps
        # dominant kernel = conv kernel instance with the largest total time
        name, (n_l, ms, flops) = max(ktimes.items(), key=lambda kv: kv[1][1])
        conv_total_ms = sum(v[1] for v in census.values())
        conv_total_fl = sum(v[2] for v in census.values())
        avg_ms = ms / n_l
        achieved = flops / n_l / (avg_ms * 1e-3) / 1e12
        def _peak(kname):
            # 16-bit MFMA engines (bf16 / f16 operands, fp32 or 16-bit outputs)
            lowp = kname.startswith(("conv_igemm_bf16", "conv_halo_kernel", "conv_gemm8"))
            return PEAK_BF16_MFMA_TFLOPS if lowp else PEAK_F32_MFMA_TFLOPS

        def _bytes(kname):  # compulsory bytes per launch (census: input + weights + output once)
            nb = ops.KernelTimer.nbytes.get(kname)
            if nb:
                return nb[1] / nb[0]
            w = ops.KernelTimer.work.get(kname)  # non-conv kernels: their wrappers' note_work
            return w[1] / w[0] if w and w[1] > 0 else None

        peak = _peak(name)
        byt = _bytes(name)
        # roofline: MFMA-bound when the launch's arithmetic intensity (FLOP per compulsory byte)
        # is above the ridge peak_flops / HBM peak, HBM-bound below it
        intensity = flops / n_l / byt if byt else None
        ridge = peak * 1e12 / (PEAK_HBM_GBPS * 1e9)
        hbm_bound = intensity is not None and intensity < ridge
        traffic, traffic_src = None, None
        tfile = TRAFFIC_FILE_TRAIN if args.train else TRAFFIC_FILE
        tpath = os.path.join(REPO, "profiles", tfile)
        if os.path.exists(tpath) and not args.spkd:  # PMC passes of this leg's own bench command
            kern = json.load(open(tpath))["kernels"]
            tk = kern.get(name)
            if tk is None:  # match in one canonical spelling (rocprof vs demangled vs census)
                cn = ops.canonical_kernel_name(name)
                same = [k for k in kern if ops.canonical_kernel_name(k) == cn]
                if not same:  # rocprof names carry template arguments the census name omits
                    same = [k for k in kern if ops.canonical_kernel_name(k).startswith(cn[:-1] + ",")]
                    best = [k for k in same if k.count(",") == name.count(",") + 1]
                    same = best if best else same
                tk = kern[same[0]] if len(same) == 1 else None
            if tk is not None:
                traffic = round(tk["hbm_bytes_per_launch"])
                traffic_src = f"profiles/{tfile} (PMC FETCH_SIZE x2 + WRITE_SIZE, per launch)"
        # achieved / frac: the ISOLATED rate — the dominant instance's average duration in the
        # census step (its launches one at a time on one stream: the view a rocprofv3 kernel
        # trace of the census range reproduces, tools/region_stats.py); the live rate inside the
        # concurrent step (a launch's event span includes the time it shares the CUs with the
        # other streams) is reported beside it as achieved_live / frac_live
        if census_all is not None and dom_fn in census_all:  # the executor census (every kernel)
            iso_span_ms = census_all[dom_fn][1] / census_all[dom_fn][0]
            iso_fl = flops / n_l
        else:
            iso_span_ms = census[name][1] / census[name][0] if name in census else avg_ms
            iso_fl = census[name][2] / census[name][0] if name in census else flops / n_l
        # the census times each launch with an event pair, which also spans the launch's dispatch
        # (disp_us, measured above on an empty launch): the kernel's own duration — what a
        # rocprofv3 kernel trace of the census range reports — is the span minus that
        iso_ms = max(iso_span_ms - disp_us * 1e-3, 0.5 * iso_span_ms)
        ach_iso = iso_fl / (iso_ms * 1e-3) / 1e12
        # the live spans carry the same dispatch span: live_kernel_us is the kernel's own duration
        # inside the concurrent step (rocprofv3's timed-range average of the instance)
        live_ms = max(avg_ms - disp_us * 1e-3, 0.5 * avg_ms)
        achieved = flops / n_l / (live_ms * 1e-3) / 1e12
        if hbm_bound or (byt and not flops):
            hbm_bound = True
            ach_bw = byt / (iso_ms * 1e-3) / 1e9
            live_bw = byt / (live_ms * 1e-3) / 1e9
            roof = dict(bound="hbm", kernel=name, achieved=round(ach_bw, 1), peak=PEAK_HBM_GBPS,
                        unit="GB/s", frac=round(ach_bw / PEAK_HBM_GBPS, 4),
                        achieved_tflops=round(ach_iso, 2), achieved_live=round(live_bw, 1),
                        frac_live=round(live_bw / PEAK_HBM_GBPS, 4))
        else:
            roof = dict(bound="mfma", kernel=name, achieved=round(ach_iso, 2), peak=peak,
                        unit="TFLOP/s", frac=round(ach_iso / peak, 4),
                        achieved_live=round(achieved, 2), frac_live=round(achieved / peak, 4))
        roof.update(traffic=traffic, traffic_source=traffic_src,
                    algorithmic_bytes_per_launch=round(byt) if byt else None,
                    arithmetic_intensity_flop_per_byte=round(intensity, 1) if intensity else None,
                    ridge_flop_per_byte=round(ridge, 1),
                    launches_per_step=n_l // args.steps, timing=timing,
                    frac_basis=("isolated: census-step average kernel duration (one stream, the "
                                "timed steps' kernel instances): isolated_kernel_us = the HIP-event "
                                "span isolated_avg_launch_us minus dispatch_span_us (the span of an "
                                "empty launch); live_kernel_us / achieved_live / frac_live: the same "
                                "instance inside the timed concurrent steps, its event span "
                                "avg_launch_us minus dispatch_span_us"),
                    avg_launch_us=round(avg_ms * 1e3, 2),
                    live_kernel_us=round(live_ms * 1e3, 2),
                    algorithmic_gflop_per_launch=round(flops / n_l / 1e9, 3),
                    isolated_avg_launch_us=round(iso_span_ms * 1e3, 2),
                    isolated_kernel_us=round(iso_ms * 1e3, 2),
                    dispatch_span_us=round(disp_us, 2),
                    # the isolated rate WITHOUT the dispatch-span correction (the basis of
                    # rounds 1-4's frac): the event span of the launch, dispatch included
                    achieved_isolated=round(iso_fl / (iso_span_ms * 1e-3) / 1e12, 2),
                    frac_isolated_span=round(iso_fl / (iso_span_ms * 1e-3) / 1e12 / peak, 4)
                    if not hbm_bound else round(byt / (iso_span_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                    all_kernels_isolated=(dict(
                        note="executor census replay (clskd_exec_census): every kernel node of the "
                             "captured step on one stream, event-timed; top 25 by total",
                        ms_per_step=round(sum(v[1] for v in census_all.values()), 3),
                        per_kernel={
                            (conv_of_fn.get(f) or ops.canonical_kernel_name(kernel_name(f))):
                                dict(launches=v[0], avg_us=round(v[1] / v[0] * 1e3, 1),
                                     total_ms=round(v[1], 3))
                            for f, v in sorted(census_all.items(), key=lambda kv: -kv[1][1])[:25]})
                        if census_all else None),
                    conv_all_kernels=dict(
                        steps=census_steps,
                        note=("census step on one stream: isolated kernel durations"
                              if not args.graph else "eager pass over the timed batches"),
                        ms_per_step=round(conv_total_ms / census_steps, 3),
                        tflops=round(conv_total_fl / (conv_total_ms * 1e-3) / 1e12, 2),
                        per_kernel={k: dict(launches_per_step=v[0] // census_steps,
                                            avg_us=round(v[1] / v[0] * 1e3, 1),
                                            tflops=round(v[2] / (v[1] * 1e-3) / 1e12, 1),
                                            compulsory_gbps=(round(_bytes(k) * v[0] / (v[1] * 1e-3) / 1e9, 1)
                                                             if _bytes(k) else None),
                                            bound=("hbm" if _bytes(k) and v[2] / v[0] / _bytes(k) <
                                                   _peak(k) * 1e12 / (PEAK_HBM_GBPS * 1e9) else "mfma"))
                                    for k, v in sorted(census.items(), key=lambda kv: -kv[1][1])}))
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not args.train:
            if args.spkd:
                cpu = cpu_baseline(args.cpu_steps or 3, n_warm=1, spkd=True)
            else:
                cpu = cpu_baseline(args.cpu_steps or 10)
            # GPU / CPU-oracle ratio on the same workload.  `vs_baseline` stays null: it is
            # reserved for a published number for this metric, and BASELINE.md has none
            cpu["gpu_over_cpu"] = round(frames / el / cpu["value"], 1)
        workload = ("C2: DCCRN-CLSKD fwd+loss (teacher 3.67M + student 0.23M params, ReviewKD "
                    "enc+dec, 14 SPKD Grams, MRSTFT)")
        if args.train:
            workload = ("C3: DCCRN-CLSKD training step = C2 fwd+loss + HIP backward to the 231,565 "
                        "student parameters + flat-bucket RCCL all-reduce (N > 1) + Adam(lr 6e-4)")
        if args.spkd:
            workload = ("C4: distill_SPKD.py fwd+loss (student + full teacher forward incl. mask "
                        "and iSTFT, MRSTFT base, SPKD Gram over the 32 output waveforms)")
        out = {
            "metric": METRIC_TRAIN if args.train else (METRIC_SPKD if args.spkd else METRIC),
            "value": round(frames / el, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "host_enqueue_ms_per_step": round(host_el / args.steps * 1e3, 3),
            "host_wait_ms_per_step": round(host_wait / args.steps * 1e3, 3),
            "launches_per_step": step_counts["kernels"] if step_counts else None,
            "launch_count_detail": (dict(step_counts, how="kernel nodes of one captured step "
                                         "(library + torch kernels)") if step_counts else None),
            "serialized_kernel_ms_per_step": round(serial_ms, 3) if serial_ms else None,
            "serialized_note": ("census step: the same step with all four streams folded onto one "
                                "(distill.serialized_streams), HIP-event timed end to end — the sum "
                                "of the step's isolated kernel times plus launch gaps")
                               if serial_ms else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"mixed": "bf16", "fp16": "fp16"}.get(args.precision, "fp32"),
            "data": "synthetic (seeded 16 kHz enveloped-sinusoid clean + noise at 0-10 dB SNR; "
                    "recipe weights, SURVEY.md §8 d)",
            "config": {"workload": workload,
                       "global_batch": world * bsz, "per_gpu_batch": bsz,
                       "clip_samples": L, "frames_per_clip": T, "parallelism": f"dp{world}",
                       "abf_reinit": args.abf_reinit, "loss": round(loss_v, 6),
                       "launch": (("eager, 2 HIP streams (caller: teacher; side: student + "
                                   "MRSTFT)" if args.spkd else
                                   "eager, 4 HIP streams (caller, teacher, student, ReviewKD-"
                                   "encoder/MRSTFT)" + ("; teacher chain of step i+1 overlaps step "
                                                        "i's ReviewKD/Gram/loss tail (teacher_ahead)"
                                                        if kd.teacher_ahead else ""))
                                  if args.launch == "eager" else
                                  "C++ step executor (clskd_exec_launch" +
                                  ("_ahead: two captures alternating, each step's teacher chain "
                                   "overlapping the previous step's tail"
                                   if args.ahead and not args.train and not args.spkd else "") +
                                  "): the captured step replayed on 4 HIP streams along its "
                                  "dependency edges "
                                  f"({executor.info['kernels']} kernels, "
                                  f"{executor.info['waits']} cross-stream waits per step)"
                                  if args.launch == "exec"
                                  else f"hipGraph replay (clskd.graph.{type(graph).__name__})"),
                       "precision": ("teacher GEMMs bf16 MFMA operands / fp32 accumulate; "
                                     "student, STFT/iSTFT, LSTM recurrence, BN, losses fp32")
                       if (args.spkd and args.precision == "mixed") else
                                    ("teacher GEMMs fp16 MFMA operands (v_mfma_f32_32x32x16_f16) / "
                                     "fp32 accumulate, fp16 teacher features; student, STFT/iSTFT, "
                                     "LSTM recurrence, BN, losses fp32")
                       if args.precision == "fp16" else
                                    ("teacher+ReviewKD GEMMs bf16 MFMA operands / fp32 accumulate; "
                                     "student fp32 storage/accumulation with its fp32 convs as "
                                     "3 x bf16 split-product MFMA (CLSKD_F32X3, <= ~3*2^-18 per "
                                     "product; the reference trains with TF32 matmuls); "
                                     "STFT, LSTM recurrence, BN, losses fp32" +
                                     ({0: "; training step exact fp32",
                                       1: "; weight gradients on split products",
                                       3: "; taped forward, data and weight gradients on split "
                                          "products"}.get(getattr(kd.student, "train_split", 0), "")
                                      if args.train else "")
                                     if kd.student.compute == "f32x3" else
                                     "teacher+ReviewKD GEMMs bf16 MFMA operands / fp32 accumulate; "
                                     "student, STFT/iSTFT, LSTM recurrence, BN, losses fp32")
                       if args.precision == "mixed" else "fp32 MFMA everywhere"},
            "roofline": roof,
            "quality": quality,
            "param_hash_per_rank": param_hashes,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        cdist.barrier(dev)
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
