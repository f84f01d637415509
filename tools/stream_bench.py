"""Config C5 throughput: streaming DCCRN (student, eval BN) over 30 s @ 16 kHz per stream,
6.25 ms hops replayed as one hipGraph each; reports per-hop latency and the real-time factor.
    python tools/stream_bench.py [--streams B] [--seconds S] [--no-graph]
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from clskd import config as cfg  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402
from clskd.model import DCCRN  # noqa: E402
from clskd.streaming import HOP, LATENCY_HOPS, FusedStreamingDCCRN, StreamingDCCRN  # noqa: E402
from clskd.weights import STUDENT_SEED, apply_recipe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--engine", default="fused", choices=["fused", "graph", "eager"],
                    help="fused: the whole hop as one launch (clskd_stream_hop); graph: the "
                         "per-layer hop replayed as a hipGraph; eager: per-layer launches")
    a = ap.parse_args()
    if a.no_graph:
        a.engine = "eager"
    dev = torch.device("cuda", 0)
    m = apply_recipe(DCCRN(masking_mode="E", use_clstm=True, **cfg.STUDENT), STUDENT_SEED).to(dev).eval()
    L = int(a.seconds * 16000) // HOP * HOP
    noisy, _ = synthetic_pairs(a.streams, L, seed=3)
    x = torch.from_numpy(noisy).to(dev)
    s = (FusedStreamingDCCRN(m, a.streams) if a.engine == "fused"
         else StreamingDCCRN(m, a.streams, graph=a.engine == "graph"))
    nh = L // HOP
    for t in range(4):  # warm-up: plans, then capture
        s.step(x[:, t * HOP:(t + 1) * HOP])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(4, nh):
        s.step(x[:, t * HOP:(t + 1) * HOP])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    hops = nh - 4
    per_hop = el / hops
    # latency of one hop on its own (synchronised each hop): input copy + hop + output copy
    lat = []
    for t in range(4, min(nh, 204)):
        t1 = time.perf_counter()
        s.step(x[:, t * HOP:(t + 1) * HOP])
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    lat.sort()
    print(json.dumps({
        "config": "C5 streaming DCCRN student (eval BN), 16 kHz, win 400 / hop 100",
        "streams": a.streams, "audio_seconds_per_stream": a.seconds,
        "launch": {"fused": "one clskd_stream_hop launch per hop (one workgroup per stream)",
                   "graph": "hipGraph per hop (~70 per-layer nodes)",
                   "eager": "per-layer launches"}[a.engine],
        "ms_per_hop": round(per_hop * 1e3, 4), "hop_ms_audio": HOP / 16.0,
        "hop_latency_ms_median_synced": round(lat[len(lat) // 2] * 1e3, 4),
        "real_time_factor": round(per_hop / (HOP / 16000.0), 5),
        "stream_seconds_per_second": round(a.streams * (HOP / 16000.0) / per_hop, 2),
        "frames_per_second": round(a.streams / per_hop, 1),
        "latency_ms_algorithmic": LATENCY_HOPS * HOP / 16.0}))


if __name__ == "__main__":
    main()
