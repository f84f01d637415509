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
B_PER_GPU = 16
NBATCH = 4
TRAFFIC_FILE = "r2_pmc_traffic.json"  # written by tools/pmc_traffic.py
L = 64000


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


def cpu_baseline(seconds):
    """The CPU oracle (fp32 PyTorch-CPU restatement of the reference, oracle/ref_cpu.py) timed on
    this host on a bounded sample of the same workload: the same B=16 x 4 s step as the GPU leg
    (one warm-up step at B=2), repeated until `seconds` of CPU work (at least one step)."""
    from oracle import ref_cpu as R
    from clskd.data import synthetic_pairs
    from clskd.weights import ABF_SEED, STUDENT_SEED, TEACHER_SEED, recipe_state_dict
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    pt = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.TEACHER), TEACHER_SEED))
    ps = R.to_torch_params(recipe_state_dict(cfg.dccrn_param_shapes(**cfg.STUDENT), STUDENT_SEED))
    pa = R.to_torch_params(recipe_state_dict(
        {**cfg.review_param_shapes("encoder"), **cfg.review_param_shapes("decoder")}, ABF_SEED))
    Bc = B_PER_GPU
    noisy, clean = synthetic_pairs(Bc, L, seed=99)
    X, Y = torch.from_numpy(noisy), torch.from_numpy(clean)
    with torch.no_grad():
        R.clskd_step(pt, ps, pa, X[:2], Y[:2])  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            R.clskd_step(pt, ps, pa, X, Y)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    frames = n * Bc * cfg.n_frames(L)
    return dict(value=round(frames / el, 2), unit="frames/s", cores=threads, kind="port",
                batch=Bc,
                sample=f"oracle/ref_cpu.clskd_step on the bench workload (B={Bc} x 4 s @16 kHz, "
                       f"same step as the GPU leg), {n} step(s) in {el:.1f} s, fp32, torch CPU "
                       f"{threads} threads")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--abf-reinit", default="step", choices=["step", "once"])
    ap.add_argument("--graph", action="store_true",
                    help="replay the captured hipGraph of the step (clskd.graph.StepGraph) instead "
                         "of launching the three-stream schedule eagerly; ROCm's graph executor "
                         "does not keep the three streams concurrent, so eager is faster here")
    ap.add_argument("--train", action="store_true",
                    help="config C3: the full training step — fwd+loss, HIP backward into the flat "
                         "student gradient, one RCCL all-reduce (N > 1), one Adam launch "
                         "(KnowledgeDistillation.train_step); reported under its own metric")
    ap.add_argument("--spkd", action="store_true",
                    help="config C4: distill_SPKD.py's step (student + teacher full forwards, MRSTFT "
                         "base, one SPKD Gram over the output waveforms) at B=32 x 4 s per GPU; "
                         "reported under its own metric")
    ap.add_argument("--precision", default="mixed", choices=["mixed", "fp32"],
                    help="mixed: teacher + ReviewKD GEMMs on bf16 MFMA operands (fp32 accumulate), "
                         "student fp32; fp32: every GEMM on exact-f32 MFMA")
    args = ap.parse_args()

    from clskd import dist as cdist
    rank, world, local_rank = cdist.env_rank()
    if args.gpus > 1 and world == 1:
        raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    cdist.init("nccl", dev)

    from clskd import ops
    from clskd.data import synthetic_pairs
    if args.spkd and (args.train or args.graph):
        raise SystemExit("--spkd is its own eager leg (no --train / --graph)")
    bsz = B_SPKD if args.spkd else B_PER_GPU
    kd = build_kd(dev, args.abf_reinit, args.precision, spkd=args.spkd)
    # NBATCH distinct batches resident in HBM; step i consumes batch i % NBATCH
    Xs, Ys = [], []
    for k in range(NBATCH):
        noisy, clean = synthetic_pairs(bsz, L, seed=cdist.shard_seed(1000 + k, rank))
        Xs.append(torch.from_numpy(noisy).to(dev))
        Ys.append(torch.from_numpy(clean).to(dev))
    T = cfg.n_frames(L)

    if args.train:
        from clskd.train import FlatAdam, FlatParams
        flat = FlatParams(kd.student)
        opt = FlatAdam(flat, lr=cfg.learning_rate)

        def step(i):
            return kd.train_step((Xs[i % NBATCH], Ys[i % NBATCH]), flat, opt)
    elif (not args.graph):
        def step(i):
            # fwd+loss only: no autograd tape (the C3 leg above records and consumes one)
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
    for i in range(args.warmup):
        last = i == args.warmup - 1 and not args.graph
        if last:
            ops.KernelTimer.start()
            with serialized_streams():
                step(i)
            census = ops.KernelTimer.stop()
        else:
            step(i)
    torch.cuda.synchronize()
    dominant = max(census.items(), key=lambda kv: kv[1][1])[0] if census else None

    # ---- timed region: exactly K steps, barrier + sync on both sides --------------------
    cdist.barrier(dev)
    if (not args.graph):
        ops.KernelTimer.start(only=dominant)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    host_el = time.perf_counter() - t0  # host enqueue of K steps (no sync inside the loop)
    cdist.barrier(dev)
    el = time.perf_counter() - t0
    if (not args.graph):
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

    if rank == 0:
        frames = world * bsz * T * args.steps
        # dominant kernel = conv kernel instance with the largest total time
        name, (n_l, ms, flops) = max(ktimes.items(), key=lambda kv: kv[1][1])
        conv_total_ms = sum(v[1] for v in census.values())
        conv_total_fl = sum(v[2] for v in census.values())
        avg_ms = ms / n_l
        achieved = flops / n_l / (avg_ms * 1e-3) / 1e12
        bf16_ops = name.startswith(("conv_igemm_bf16", "conv_halo_kernel", "conv_gemm8"))
        peak = PEAK_BF16_MFMA_TFLOPS if bf16_ops else PEAK_F32_MFMA_TFLOPS
        traffic, traffic_src = None, None
        tpath = os.path.join(REPO, "profiles", TRAFFIC_FILE)
        if os.path.exists(tpath) and not args.spkd:  # the PMC passes profile the C2 leg
            tk = json.load(open(tpath))["kernels"].get(name)
            if tk is not None:
                traffic = round(tk["hbm_bytes_per_launch"])
                traffic_src = f"profiles/{TRAFFIC_FILE} (PMC FETCH_SIZE x2 + WRITE_SIZE, per launch)"
        roof = dict(bound="mfma", kernel=name, achieved=round(achieved, 2),
                    peak=peak, unit="TFLOP/s",
                    frac=round(achieved / peak, 4), traffic=traffic, traffic_source=traffic_src,
                    launches_per_step=n_l // args.steps, timing=timing,
                    avg_launch_us=round(avg_ms * 1e3, 2),
                    algorithmic_gflop_per_launch=round(flops / n_l / 1e9, 3),
                    isolated_avg_launch_us=(round(census[name][1] / census[name][0] * 1e3, 2)
                                            if name in census else None),
                    achieved_isolated=(round(census[name][2] / (census[name][1] * 1e-3) / 1e12, 2)
                                       if name in census else None),
                    conv_all_kernels=dict(
                        steps=census_steps,
                        note=("census step on one stream: isolated kernel durations"
                              if not args.graph else "eager pass over the timed batches"),
                        ms_per_step=round(conv_total_ms / census_steps, 3),
                        tflops=round(conv_total_fl / (conv_total_ms * 1e-3) / 1e12, 2),
                        per_kernel={k: dict(launches_per_step=v[0] // census_steps,
                                            avg_us=round(v[1] / v[0] * 1e3, 1),
                                            tflops=round(v[2] / (v[1] * 1e-3) / 1e12, 1))
                                    for k, v in sorted(census.items(), key=lambda kv: -kv[1][1])}))
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not args.train and not args.spkd:
            cpu = cpu_baseline(args.cpu_seconds)
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
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if args.precision == "mixed" else "fp32",
            "data": "synthetic (seeded 16 kHz enveloped-sinusoid clean + noise at 0-10 dB SNR; "
                    "recipe weights, SURVEY.md §8 d)",
            "config": {"workload": workload,
                       "global_batch": world * bsz, "per_gpu_batch": bsz,
                       "clip_samples": L, "frames_per_clip": T, "parallelism": f"dp{world}",
                       "abf_reinit": args.abf_reinit, "loss": round(loss_v, 6),
                       "launch": ("eager, 2 HIP streams (caller: teacher; side: student + "
                                  "MRSTFT)" if args.spkd else
                                  "eager, 4 HIP streams (caller, teacher, student, ReviewKD-"
                                  "encoder/MRSTFT)" if (not args.graph)
                                  else "hipGraph replay (clskd.graph.StepGraph)"),
                       "precision": ("teacher GEMMs bf16 MFMA operands / fp32 accumulate; "
                                     "student, STFT/iSTFT, LSTM recurrence, BN, losses fp32")
                       if (args.spkd and args.precision == "mixed") else
                                    ("teacher+ReviewKD GEMMs bf16 MFMA operands / fp32 accumulate; "
                                     "student, STFT/iSTFT, LSTM recurrence, BN, losses fp32")
                       if args.precision == "mixed" else "fp32 MFMA everywhere"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        cdist.barrier(dev)
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
