"""World-size-2 data-parallel plumbing on CPU (gloo, 127.0.0.1): batch shards are disjoint and
reproducible, timing is the max over ranks, and the flat-bucket gradient all-reduce averages."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "speech-enhancement-clskd_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from clskd import dist as cdist
    from clskd.data import synthetic_pairs
    r, w = cdist.init("gloo")
    noisy, _ = synthetic_pairs(2, 1600, seed=cdist.shard_seed(7, r))
    t_max = cdist.max_over_ranks(0.5 + r)
    grads = [torch.full((3, 4), float(r + 1)), torch.arange(5, dtype=torch.float32) * (r + 1)]
    cdist.allreduce_mean_flat(grads)
    cdist.barrier()
    q.put((r, w, float(noisy.sum()), t_max, grads[0].numpy().copy(), grads[1].numpy().copy()))
    torch.distributed.destroy_process_group()


def test_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, s0, t0, g0a, g0b), (r1, w1, s1, t1, g1a, g1b) = res
    assert (r0, r1, w0, w1) == (0, 1, 2, 2)
    assert s0 != s1  # disjoint shards
    assert t0 == t1 == 1.5  # max over ranks
    np.testing.assert_allclose(g0a, np.full((3, 4), 1.5))
    np.testing.assert_allclose(g1b, np.arange(5) * 1.5)
    np.testing.assert_array_equal(g0b, g1b)
