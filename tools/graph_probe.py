"""Census of a captured C2 step graph: node types, kernel count, edges (diagnostic).

    python tools/graph_probe.py
"""
import collections
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "speech-enhancement-clskd_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

sys.argv += []
import bench  # noqa: E402
from clskd.data import synthetic_pairs  # noqa: E402

dev = torch.device("cuda", 0)
kd = bench.build_kd(dev, "step", "mixed")
noisy, clean = synthetic_pairs(16, 64000, seed=1)
X = torch.from_numpy(noisy).to(dev)
Y = torch.from_numpy(clean).to(dev)
with torch.no_grad():
    kd.training_step((X, Y))
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph(keep_graph=True)
with torch.cuda.graph(g):
    out = kd.training_step((X, Y), return_parts=True)
hg = C.c_void_p(g.raw_cuda_graph())
hip = C.CDLL("libamdhip64.so")
n = C.c_size_t(0)
assert hip.hipGraphGetNodes(hg, None, C.byref(n)) == 0
nodes = (C.c_void_p * n.value)()
assert hip.hipGraphGetNodes(hg, nodes, C.byref(n)) == 0
types = collections.Counter()
for i in range(n.value):
    t = C.c_int(-1)
    hip.hipGraphNodeGetType(C.c_void_p(nodes[i]), C.byref(t))
    types[t.value] += 1
ne = C.c_size_t(0)
hip.hipGraphGetEdges(hg, None, None, C.byref(ne))
print("nodes", n.value, "edges", ne.value, "types", dict(types))
