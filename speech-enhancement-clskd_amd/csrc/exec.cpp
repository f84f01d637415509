// Step executor: replays a captured hipGraph of one training / fwd+loss step from C++ on several
// HIP streams.
//
// Why: the C2 step is ~400 launches on four streams.  Launched from Python the host needs 4-5 ms
// per step for them (descriptor building, allocator calls, ctypes), about the device time, so the
// step turns host-bound and run-to-run spread follows the host.  hipGraphLaunch of the captured
// step costs 0.8 ms of host time, but ROCm's graph executor runs the branches one after another
// (7.3 ms per step against 5.6 ms eager on four streams, measured on MI355X with and without
// packet capture and forced graph queues).  This executor keeps both: the graph's nodes are
// re-launched with their captured arguments (hipLaunchKernel: no Python, no descriptor work),
// distributed over `nstreams` streams along the graph's dependency edges, with one event
// record / wait per cross-stream edge that is not already implied by an earlier wait (vector
// clocks, resolved once at creation).  Stream 0 is the caller's stream at launch time: the
// other streams fork from it at the start and are joined back into it at the end, so a launch
// is stream-ordered like any other library call.
//
// The graph is borrowed: the kernels' captured arguments live in its nodes, and the buffers they
// point to in the capture's memory pool, so the caller keeps both alive while the executor is
// used (clskd.graph.StepExecutor owns the torch CUDAGraph for this).
#include <cxxabi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <mutex>
#include <queue>
#include <unordered_map>
#include <string>
#include <vector>

#include "common.h"

namespace {

enum OpKind : uint8_t { OP_KERNEL, OP_MEMSET, OP_MEMCPY, OP_WAIT, OP_RECORD };

struct Op {
  OpKind kind;
  uint8_t stream;
  int32_t idx;  // kernel / memset / memcpy slot, or event slot
};

struct KNode {
  const void* func;
  dim3 grid, block;
  void** args;
  unsigned shmem;
};

}  // namespace

struct clskd_exec {
  hipGraph_t graph = nullptr;
  int nstreams = 0;
  std::vector<hipStream_t> own;  // streams 1..nstreams-1 (stream 0 = caller's)
  bool owns_streams = true;      // false: borrowed from the caller (clskd_exec_create)
  std::vector<hipEvent_t> events;
  std::vector<KNode> kernels;
  std::vector<hipMemsetParams> memsets;
  std::vector<hipMemcpy3DParms> memcpys;
  // a memcpy node that is one contiguous range between linear allocations (torch's clone /
  // copy_ under capture) replays as a flat hipMemcpyAsync: {dst, src, bytes}, bytes = 0 -> 3D
  struct Flat {
    void* dst;
    const void* src;
    size_t bytes;
    hipMemcpyKind kind;
  };
  std::vector<Flat> flat;
  std::vector<Op> program;
  size_t join_at = 0;  // program[join_at..]: every used side stream's join into stream 0
  int ev_fork = -1;    // event slot of the fork (recorded on stream 0 first)
  int32_t n_nodes = 0, n_waits = 0, n_records = 0, n_empty = 0;
  int32_t per_stream[8] = {0};
  // optional live timing of one kernel (bench: the dominant instance): an event pair around
  // each of its launches, on its stream
  std::vector<char> timed;  // per kernel slot
  std::vector<hipEvent_t> tev;
  int32_t t_used = 0;
  // optional per-stream milestones: a timing event before the fork and at every stream's tail,
  // per launch in a ring of MK launches (diagnostic: which branch ends when)
  static constexpr int MK = 64;
  std::vector<hipEvent_t> mk;  // [MK][1 + nstreams]
  int32_t mk_n = 0;
};

using namespace clskd;

static int hip_fail(const char* what, hipError_t e) {
  set_error("exec: %s: %s", what, hipGetErrorString(e));
  return CLSKD_E_HIP;
}

// Capture-time stream tags: after each library call during a capture, the host reports which
// of its streams the call ran on; the capture's current dependency set of that stream is then
// exactly the node(s) just added, which get the tag.  exec_create places tagged nodes on the
// stream of that index, so the replay keeps the eager schedule's chains (one node per stream
// position) instead of a reconstructed chain cover.
static std::mutex g_tag_mu;
static std::unordered_map<hipGraphNode_t, int> g_tags;

extern "C" void clskd_exec_tag_reset(void) {
  std::lock_guard<std::mutex> lk(g_tag_mu);
  g_tags.clear();
}

extern "C" int clskd_exec_tag(void* stream, int32_t tag) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  const hipError_t e = hipStreamGetCaptureInfo_v2(as_stream(stream), &st, nullptr, nullptr, &deps, &nd);
  if (e != hipSuccess) return hip_fail("hipStreamGetCaptureInfo_v2", e);
  if (st != hipStreamCaptureStatusActive) return CLSKD_OK;
  std::lock_guard<std::mutex> lk(g_tag_mu);
  for (size_t i = 0; i < nd; ++i) g_tags.emplace(deps[i], tag);  // first report wins
  return CLSKD_OK;
}

extern "C" int clskd_exec_create(void* hip_graph, int32_t nstreams, void* const* side_streams,
                                 int32_t use_tags, clskd_exec** out) {
  CLSKD_CHECK_ARG(hip_graph && out, "exec_create: null graph or output");
  CLSKD_CHECK_ARG(nstreams >= 1 && nstreams <= 8, "exec_create: nstreams %d outside [1, 8]", nstreams);
  *out = nullptr;
  hipGraph_t g = reinterpret_cast<hipGraph_t>(hip_graph);
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  if (e != hipSuccess) return hip_fail("hipGraphGetNodes", e);
  std::vector<hipGraphNode_t> nodes(n);
  if (n) {
    e = hipGraphGetNodes(g, nodes.data(), &n);
    if (e != hipSuccess) return hip_fail("hipGraphGetNodes", e);
  }
  std::unordered_map<hipGraphNode_t, int> index;
  index.reserve(n * 2);
  for (size_t i = 0; i < n; ++i) index[nodes[i]] = (int)i;
  size_t ne = 0;
  e = hipGraphGetEdges(g, nullptr, nullptr, &ne);
  if (e != hipSuccess) return hip_fail("hipGraphGetEdges", e);
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne) {
    e = hipGraphGetEdges(g, from.data(), to.data(), &ne);
    if (e != hipSuccess) return hip_fail("hipGraphGetEdges", e);
  }
  std::vector<std::vector<int>> preds(n), succs(n);
  std::vector<int> indeg(n, 0);
  for (size_t k = 0; k < ne; ++k) {
    const int a = index.at(from[k]), b = index.at(to[k]);
    preds[b].push_back(a);
    succs[a].push_back(b);
    ++indeg[b];
  }
  // topological order, ties broken by node order (the capture order, i.e. the host's enqueue
  // order, which the schedule was tuned for)
  std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
  for (size_t i = 0; i < n; ++i)
    if (!indeg[i]) ready.push((int)i);
  std::vector<int> topo;
  topo.reserve(n);
  while (!ready.empty()) {
    const int v = ready.top();
    ready.pop();
    topo.push_back(v);
    for (int s : succs[v])
      if (--indeg[s] == 0) ready.push(s);
  }
  CLSKD_CHECK_ARG(topo.size() == n, "exec_create: graph has a cycle");

  auto* ex = new clskd_exec();
  ex->graph = g;
  ex->nstreams = nstreams;
  ex->n_nodes = (int32_t)n;
  std::vector<int> type(n, -1), slot(n, -1);
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    e = hipGraphNodeGetType(nodes[i], &t);
    if (e != hipSuccess) {
      delete ex;
      return hip_fail("hipGraphNodeGetType", e);
    }
    type[i] = (int)t;
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams p{};
      e = hipGraphKernelNodeGetParams(nodes[i], &p);
      if (e != hipSuccess) {
        delete ex;
        return hip_fail("hipGraphKernelNodeGetParams", e);
      }
      if (!p.func || (p.extra && !p.kernelParams)) {
        delete ex;
        set_error("exec_create: kernel node %zu has no host function or uses 'extra' arguments", i);
        return CLSKD_E_ARG;
      }
      // replayed with hipLaunchKernel: p.func must be a registered host stub, not a
      // hipFunction_t captured from a module launch (rejected here instead of failing mid-step)
      hipFuncAttributes fa{};
      if (hipFuncGetAttributes(&fa, p.func) != hipSuccess) {
        (void)hipGetLastError();
        delete ex;
        set_error("exec_create: kernel node %zu is not a host-stub launch (module kernel?)", i);
        return CLSKD_E_ARG;
      }
      slot[i] = (int)ex->kernels.size();
      ex->kernels.push_back(KNode{p.func, p.gridDim, p.blockDim, p.kernelParams, p.sharedMemBytes});
    } else if (t == hipGraphNodeTypeMemset) {
      hipMemsetParams p{};
      e = hipGraphMemsetNodeGetParams(nodes[i], &p);
      if (e != hipSuccess) {
        delete ex;
        return hip_fail("hipGraphMemsetNodeGetParams", e);
      }
      if (!(p.elementSize == 1 || p.elementSize == 2 || p.elementSize == 4) ||
          (p.height > 1 && p.elementSize != 1)) {
        delete ex;
        set_error("exec_create: memset node %zu: element size %u, height %zu not supported", i,
                  p.elementSize, p.height);
        return CLSKD_E_ARG;
      }
      slot[i] = (int)ex->memsets.size();
      ex->memsets.push_back(p);
    } else if (t == hipGraphNodeTypeMemcpy) {
      hipMemcpy3DParms p{};
      e = hipGraphMemcpyNodeGetParams(nodes[i], &p);
      if (e != hipSuccess) {
        delete ex;
        return hip_fail("hipGraphMemcpyNodeGetParams", e);
      }
      // ROCm 7.2 returns unusable parameters for one-dimensional memcpy nodes (the kind torch's
      // copies record under capture: null destination, garbage extent); such a graph cannot be
      // replayed node by node — refuse it (hipGraphLaunch replays it)
      if (!p.dstArray && !p.dstPtr.ptr) {
        delete ex;
        set_error("exec_create: memcpy node %zu has unreadable parameters (a 1-D copy node); "
                  "replay this graph with hipGraphLaunch", i);
        return CLSKD_E_ARG;
      }
      slot[i] = (int)ex->memcpys.size();
      ex->memcpys.push_back(p);
      clskd_exec::Flat f{nullptr, nullptr, 0, p.kind};
      if (!p.srcArray && !p.dstArray && p.extent.height <= 1 && p.extent.depth <= 1 &&
          p.srcPos.y == 0 && p.srcPos.z == 0 && p.dstPos.y == 0 && p.dstPos.z == 0 &&
          p.srcPtr.ptr && p.dstPtr.ptr) {
        f.dst = static_cast<char*>(p.dstPtr.ptr) + p.dstPos.x;
        f.src = static_cast<const char*>(p.srcPtr.ptr) + p.srcPos.x;
        f.bytes = p.extent.width;
      }
      ex->flat.push_back(f);
    } else if (t == hipGraphNodeTypeEmpty) {
      ++ex->n_empty;
    } else {
      delete ex;
      set_error("exec_create: node %zu has type %d (only kernel, memset, memcpy and empty nodes "
                "are replayed)", i, (int)t);
      return CLSKD_E_ARG;
    }
  }

  // real dependencies: an empty node passes its own dependencies through
  std::vector<std::vector<int>> deps(n);
  for (int v : topo) {
    std::vector<int> d;
    for (int u : preds[v]) {
      if (type[u] == hipGraphNodeTypeEmpty)
        d.insert(d.end(), deps[u].begin(), deps[u].end());
      else
        d.push_back(u);
    }
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    deps[v] = std::move(d);
  }

  // capture-time stream tags (clskd_exec_tag); an untagged node (e.g. the first kernel of a
  // multi-launch call) inherits the tag of a tagged successor that depends on it directly
  std::vector<int> tag(n, -1);
  if (use_tags) {
    std::lock_guard<std::mutex> lk(g_tag_mu);
    for (size_t i = 0; i < n; ++i) {
      auto it = g_tags.find(nodes[i]);
      if (it != g_tags.end() && it->second >= 0 && it->second < nstreams) tag[i] = it->second;
    }
  }
  for (auto it = topo.rbegin(); it != topo.rend(); ++it) {
    const int u = *it;
    if (tag[u] >= 0) continue;
    for (int v : succs[u])
      if (tag[v] >= 0) {
        tag[u] = tag[v];
        break;
      }
  }
  // stream assignment + redundant-wait elimination (vector clocks over topological positions)
  const int S = nstreams;
  std::vector<int> pos(n, -1), stream_of(n, -1);
  for (size_t k = 0; k < topo.size(); ++k) pos[topo[k]] = (int)k;
  std::vector<int> tail(S, -1);                                  // last node on each stream
  std::vector<std::vector<int>> clock(S, std::vector<int>(S, -1));  // clock[s][t]: pos known done
  std::vector<std::vector<int>> nclock(n);
  std::vector<char> needs_event(n, 0);
  struct Pending {
    int v, s;
    std::vector<int> waits;  // nodes whose events stream s waits for before v
  };
  std::vector<Pending> plan;
  plan.reserve(n);
  for (int v : topo) {
    if (type[v] == hipGraphNodeTypeEmpty) continue;
    // dependency clock of v: per stream, the last position v depends on (directly or not)
    std::vector<int> dc(S, -1);
    for (int u : deps[v]) {
      const std::vector<int>& cu = nclock[u];
      for (int t = 0; t < S; ++t) dc[t] = std::max(dc[t], cu[t]);
    }
    // a stream is free for v when v already depends on all its work (no false serialisation);
    // among free streams prefer one whose tail is a direct dependency (continue that chain),
    // the most recent first; with none free, the stream whose work is oldest
    int bs = tag[v];  // the stream the eager schedule ran it on, when tagged at capture
    if (bs < 0) {
      int best = -2;
      for (int s = 0; s < S; ++s) {
        const int tp = tail[s] < 0 ? -1 : pos[tail[s]];
        if (tp > dc[s]) continue;
        const bool direct = tail[s] >= 0 && std::binary_search(deps[v].begin(), deps[v].end(), tail[s]);
        const int score = direct ? (1 << 20) + tp : tp;
        if (score > best) {
          best = score;
          bs = s;
        }
      }
    }
    if (bs < 0) {
      int oldest = 1 << 30;
      for (int s = 0; s < S; ++s) {
        const int p = tail[s] < 0 ? -1 : pos[tail[s]];
        if (p < oldest) {
          oldest = p;
          bs = s;
        }
      }
    }
    Pending pd{v, bs, {}};
    std::vector<int>& c = clock[bs];
    for (int u : deps[v]) {
      const int su = stream_of[u];
      if (su == bs || c[su] >= pos[u]) continue;
      pd.waits.push_back(u);
      needs_event[u] = 1;
      const std::vector<int>& cu = nclock[u];
      for (int t = 0; t < S; ++t) c[t] = std::max(c[t], cu[t]);
    }
    c[bs] = pos[v];
    nclock[v] = c;
    stream_of[v] = bs;
    tail[bs] = v;
    ex->per_stream[bs]++;
    plan.push_back(std::move(pd));
  }
  // scheduling gate (knob CLSKD_EXEC_GATE = s*100000 + g*10000 + k, A/B): stream s's first node
  // additionally waits for the k-th node of stream g — a head start for a critical chain that the
  // replay, which issues the whole step at once, does not otherwise give it
  if (const int gate = knob(KNOB_EXEC_GATE)) {
    const int gs = gate / 100000, gg = (gate / 10000) % 10, gk = gate % 10000;
    int first = -1, seen = 0, gu = -1;
    for (size_t i = 0; i < plan.size(); ++i) {
      if (plan[i].s == gg && gu < 0 && ++seen == gk) gu = plan[i].v;
      if (plan[i].s == gs && first < 0) first = (int)i;
    }
    if (gs < S && gg < S && gs != gg && first >= 0 && gu >= 0 && pos[gu] < pos[plan[first].v]) {
      plan[first].waits.push_back(gu);
      needs_event[gu] = 1;
    }
  }

  // events: one per node with a cross-stream consumer, plus fork and one join per side stream
  std::vector<int> ev_of(n, -1);
  int nev = 0;
  for (size_t i = 0; i < n; ++i)
    if (needs_event[i]) ev_of[i] = nev++;
  const int ev_fork = nev++;
  ex->ev_fork = ev_fork;
  const int ev_join0 = nev;
  nev += S - 1;
  ex->events.resize(nev, nullptr);
  for (int k = 0; k < nev; ++k) {
    e = hipEventCreateWithFlags(&ex->events[k], hipEventDisableTiming);
    if (e != hipSuccess) {
      for (int j = 0; j < k; ++j) (void)hipEventDestroy(ex->events[j]);
      delete ex;
      return hip_fail("hipEventCreateWithFlags", e);
    }
  }
  ex->own.resize(S > 1 ? S - 1 : 0, nullptr);
  ex->owns_streams = side_streams == nullptr;
  for (int s = 1; s < S; ++s) {
    if (side_streams) {  // the caller's streams: the same hardware-queue mapping as its eager path
      ex->own[s - 1] = as_stream(side_streams[s - 1]);
      continue;
    }
    e = hipStreamCreateWithFlags(&ex->own[s - 1], hipStreamNonBlocking);
    if (e != hipSuccess) {
      clskd_exec_destroy(ex);
      return hip_fail("hipStreamCreateWithFlags", e);
    }
  }
  // program: fork, the plan in topological order (waits, the node, its record), join
  std::vector<char> used(S, 0);
  for (const Pending& pd : plan) used[pd.s] = 1;
  if (S > 1) {
    ex->program.push_back(Op{OP_RECORD, 0, ev_fork});
    for (int s = 1; s < S; ++s)
      if (used[s]) ex->program.push_back(Op{OP_WAIT, (uint8_t)s, ev_fork});
  }
  for (const Pending& pd : plan) {
    for (int u : pd.waits) {
      ex->program.push_back(Op{OP_WAIT, (uint8_t)pd.s, ev_of[u]});
      ++ex->n_waits;
    }
    const int t = type[pd.v];
    const OpKind k = t == hipGraphNodeTypeKernel ? OP_KERNEL : t == hipGraphNodeTypeMemset ? OP_MEMSET : OP_MEMCPY;
    ex->program.push_back(Op{k, (uint8_t)pd.s, slot[pd.v]});
    if (needs_event[pd.v]) {
      ex->program.push_back(Op{OP_RECORD, (uint8_t)pd.s, ev_of[pd.v]});
      ++ex->n_records;
    }
  }
  ex->join_at = ex->program.size();
  for (int s = 1; s < S; ++s)
    if (used[s]) {
      ex->program.push_back(Op{OP_RECORD, (uint8_t)s, ev_join0 + s - 1});
      ex->program.push_back(Op{OP_WAIT, 0, ev_join0 + s - 1});
    }
  *out = ex;
  return CLSKD_OK;
}

extern "C" int clskd_exec_launch(clskd_exec* ex, void* stream) {
  return clskd_exec_launch_ahead(ex, stream, 0, nullptr);
}

extern "C" int clskd_exec_launch_ahead(clskd_exec* ex, void* stream, uint32_t ahead_mask, void* ahead_event) {
  CLSKD_CHECK_ARG(ex, "exec_launch: null executor");
  CLSKD_CHECK_ARG((ahead_mask & 1u) == 0, "exec_launch_ahead: stream 0 always follows the fork");
  hipStream_t st[8];
  st[0] = as_stream(stream);
  for (int s = 1; s < ex->nstreams; ++s) st[s] = ex->own[s - 1];
  const int S1 = ex->nstreams + 1;
  hipEvent_t* mk = ex->mk.empty() ? nullptr : &ex->mk[(size_t)(ex->mk_n % clskd_exec::MK) * S1];
  if (mk) (void)hipEventRecord(mk[0], st[0]);
  for (size_t i = 0; i < ex->program.size(); ++i) {
    const Op& op = ex->program[i];
    hipError_t e = hipSuccess;
    const hipStream_t s = st[op.stream];
    switch (op.kind) {
      case OP_KERNEL: {
        const KNode& k = ex->kernels[op.idx];
        const bool tm = !ex->timed.empty() && ex->timed[op.idx] && 2 * ex->t_used + 1 < (int)ex->tev.size();
        if (tm) (void)hipEventRecord(ex->tev[2 * ex->t_used], s);
        e = hipLaunchKernel(k.func, k.grid, k.block, k.args, k.shmem, s);
        if (tm) (void)hipEventRecord(ex->tev[2 * ex->t_used++ + 1], s);
        break;
      }
      case OP_MEMSET: {
        const hipMemsetParams& p = ex->memsets[op.idx];
        if (p.height > 1)
          e = hipMemset2DAsync(p.dst, p.pitch, (int)p.value, p.width, p.height, s);
        else if (p.elementSize == 4)
          e = hipMemsetD32Async((hipDeviceptr_t)p.dst, (int)p.value, p.width, s);
        else if (p.elementSize == 2)
          e = hipMemsetD16Async((hipDeviceptr_t)p.dst, (unsigned short)p.value, p.width, s);
        else
          e = hipMemsetD8Async((hipDeviceptr_t)p.dst, (unsigned char)p.value, p.width, s);
        break;
      }
      case OP_MEMCPY: {
        const clskd_exec::Flat& f = ex->flat[op.idx];
        e = f.bytes ? hipMemcpyAsync(f.dst, f.src, f.bytes, f.kind, s)
                    : hipMemcpy3DAsync(&ex->memcpys[op.idx], s);
        break;
      }
      case OP_WAIT:
        if (i < ex->join_at && op.idx == ex->ev_fork && ((ahead_mask >> op.stream) & 1u)) {
          // ahead stream: instead of the fork (the caller's stream, behind the previous launch's
          // join), wait for the caller's event — e.g. the end of this executor's own previous
          // launch, the last reader of its static buffers (none: the stream's own order only)
          if (ahead_event) e = hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(ahead_event), 0);
        } else {
          e = hipStreamWaitEvent(s, ex->events[op.idx], 0);
        }
        break;
      case OP_RECORD:
        e = hipEventRecord(ex->events[op.idx], s);
        break;
    }
    if (e != hipSuccess) {
      // still join every side stream back into the caller's, so later work on stream 0 stays
      // ordered after whatever part of the step was enqueued
      for (size_t j = ex->join_at; j < ex->program.size(); ++j) {
        const Op& jo = ex->program[j];
        if (jo.kind == OP_RECORD) (void)hipEventRecord(ex->events[jo.idx], st[jo.stream]);
        else (void)hipStreamWaitEvent(st[jo.stream], ex->events[jo.idx], 0);
      }
      static const char* kinds[] = {"kernel", "memset", "memcpy", "wait", "record"};
      char what[320];
      int w = snprintf(what, sizeof what, "launch (program op %zu: %s #%d, stream %d)", i,
                       op.kind < 5 ? kinds[op.kind] : "?", op.idx, op.stream);
      if (op.kind == OP_MEMCPY && w > 0 && w < (int)sizeof what) {
        const hipMemcpy3DParms& p = ex->memcpys[op.idx];
        snprintf(what + w, sizeof what - w,
                 " [src %p+%zu pitch %zu, dst %p+%zu pitch %zu, extent %zux%zux%zu, kind %d, "
                 "arrays %p/%p]", p.srcPtr.ptr, p.srcPos.x, p.srcPtr.pitch, p.dstPtr.ptr,
                 p.dstPos.x, p.dstPtr.pitch, p.extent.width, p.extent.height, p.extent.depth,
                 (int)p.kind, (void*)p.srcArray, (void*)p.dstArray);
      }
      return hip_fail(what, e);
    }
  }
  if (mk) {
    for (int s = ex->nstreams - 1; s >= 0; --s) (void)hipEventRecord(mk[1 + s], st[s]);
    ++ex->mk_n;
  }
  return CLSKD_OK;
}

extern "C" int clskd_exec_marks(clskd_exec* ex, int32_t on) {
  CLSKD_CHECK_ARG(ex, "exec_marks: null executor");
  for (hipEvent_t ev : ex->mk) (void)hipEventDestroy(ev);
  ex->mk.clear();
  ex->mk_n = 0;
  if (!on) return CLSKD_OK;
  ex->mk.resize((size_t)clskd_exec::MK * (ex->nstreams + 1), nullptr);
  for (auto& ev : ex->mk) {
    const hipError_t e = hipEventCreate(&ev);
    if (e != hipSuccess) return hip_fail("hipEventCreate", e);
  }
  return CLSKD_OK;
}

// out[s] = mean over the recorded launches (at most the last MK) of (tail of stream s - fork), ms
extern "C" int clskd_exec_marks_read(clskd_exec* ex, float* out, int32_t n) {
  CLSKD_CHECK_ARG(ex && out && n >= ex->nstreams && !ex->mk.empty(), "exec_marks_read: arguments");
  const int S1 = ex->nstreams + 1, cnt = ex->mk_n < clskd_exec::MK ? ex->mk_n : clskd_exec::MK;
  for (int s = 0; s < ex->nstreams; ++s) {
    double acc = 0;
    for (int i = 0; i < cnt; ++i) {
      float ms = 0.f;
      const hipError_t e = hipEventElapsedTime(&ms, ex->mk[(size_t)i * S1], ex->mk[(size_t)i * S1 + 1 + s]);
      if (e != hipSuccess) return hip_fail("hipEventElapsedTime", e);
      acc += ms;
    }
    out[s] = cnt ? (float)(acc / cnt) : 0.f;
  }
  return CLSKD_OK;
}

extern "C" int clskd_exec_info(const clskd_exec* ex, int32_t* info, int32_t n) {
  CLSKD_CHECK_ARG(ex && info && n >= 8, "exec_info: needs 8 output slots");
  info[0] = ex->n_nodes;
  info[1] = (int32_t)ex->kernels.size();
  info[2] = (int32_t)ex->memsets.size();
  info[3] = (int32_t)ex->memcpys.size();
  info[4] = ex->n_empty;
  info[5] = ex->n_waits;
  info[6] = ex->n_records;
  info[7] = (int32_t)ex->program.size();
  for (int s = 0; s < 8 && 8 + s < n; ++s) info[8 + s] = ex->per_stream[s];
  return CLSKD_OK;
}

extern "C" int64_t clskd_exec_dump(const clskd_exec* ex, char* buf, int64_t cap) {
  if (!ex) return -1;
  std::string out;
  char line[512];
  static const char* kinds[] = {"kernel", "memset", "memcpy", "wait", "record"};
  for (size_t i = 0; i < ex->program.size(); ++i) {
    const Op& op = ex->program[i];
    const char* name = "";
    if (op.kind == OP_KERNEL) {
      const KNode& k = ex->kernels[op.idx];
      name = hipKernelNameRefByPtr(k.func, nullptr);
      if (!name) name = "?";
      snprintf(line, sizeof line, "%zu %s s%d #%d grid %u block %u %s\n", i, kinds[op.kind],
               (int)op.stream, op.idx, k.grid.x * k.grid.y * k.grid.z, k.block.x, name);
    } else {
      snprintf(line, sizeof line, "%zu %s s%d #%d\n", i, kinds[op.kind], (int)op.stream, op.idx);
    }
    out += line;
  }
  if (buf && cap > 0) {
    const size_t n = out.size() < (size_t)cap - 1 ? out.size() : (size_t)cap - 1;
    memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return (int64_t)out.size();
}

static void drop_timing(clskd_exec* ex) {
  for (hipEvent_t ev : ex->tev) (void)hipEventDestroy(ev);
  ex->tev.clear();
  ex->timed.clear();
  ex->t_used = 0;
}

extern "C" int clskd_exec_profile(clskd_exec* ex, const void* fn, int32_t max_launches) {
  CLSKD_CHECK_ARG(ex, "exec_profile: null executor");
  drop_timing(ex);
  if (!fn || max_launches <= 0) return CLSKD_OK;
  ex->timed.assign(ex->kernels.size(), 0);
  int hits = 0;
  for (size_t i = 0; i < ex->kernels.size(); ++i)
    if (ex->kernels[i].func == fn) ex->timed[i] = 1, ++hits;
  if (!hits) {
    drop_timing(ex);
    set_error("exec_profile: no kernel node launches that function");
    return CLSKD_E_ARG;
  }
  ex->tev.resize(2 * (size_t)max_launches, nullptr);
  for (auto& ev : ex->tev) {
    const hipError_t e = hipEventCreate(&ev);
    if (e != hipSuccess) {
      ev = nullptr;
      drop_timing(ex);
      return hip_fail("hipEventCreate", e);
    }
  }
  return CLSKD_OK;
}

extern "C" int clskd_exec_profile_read(clskd_exec* ex, double* total_ms, int32_t* count) {
  CLSKD_CHECK_ARG(ex && total_ms && count, "exec_profile_read: null argument");
  double tot = 0;
  for (int i = 0; i < ex->t_used; ++i) {
    float ms = 0.f;
    const hipError_t e = hipEventElapsedTime(&ms, ex->tev[2 * i], ex->tev[2 * i + 1]);
    if (e != hipSuccess) return hip_fail("hipEventElapsedTime", e);
    tot += ms;
  }
  *total_ms = tot;
  *count = ex->t_used;
  return CLSKD_OK;
}

// Per-kernel census of one replay (round 6; bench.py picks the dominant kernel instance from it):
// the program's nodes in program order (a topological order) on ONE stream, the caller's, with an
// event pair around every kernel node — each kernel's isolated duration, the view a rocprofv3
// kernel trace of a serialised step has.  The replay is a real step of the captured computation.
// fns / ms receive one entry per kernel node in program order (*n = the node count; cap too small:
// CLSKD_E_ARG with *n set).  Synchronises the stream.
extern "C" int clskd_exec_census(clskd_exec* ex, void* stream, int32_t cap, const void** fns, float* ms,
                                 int32_t* n) {
  CLSKD_CHECK_ARG(ex && n, "exec_census: null argument");
  const int nk = (int)ex->kernels.size();
  *n = nk;
  CLSKD_CHECK_ARG(cap >= nk && fns && ms, "exec_census: %d kernel nodes, room for %d", nk, cap);
  const hipStream_t s = as_stream(stream);
  std::vector<hipEvent_t> ev(2 * (size_t)nk, nullptr);
  auto cleanup = [&]() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
  };
  for (auto& e : ev) {
    const hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) {
      e = nullptr;
      cleanup();
      return hip_fail("hipEventCreate", r);
    }
  }
  int k = 0;
  for (const Op& op : ex->program) {
    hipError_t e = hipSuccess;
    if (op.kind == OP_KERNEL) {
      const KNode& kn = ex->kernels[op.idx];
      (void)hipEventRecord(ev[2 * k], s);
      e = hipLaunchKernel(kn.func, kn.grid, kn.block, kn.args, kn.shmem, s);
      (void)hipEventRecord(ev[2 * k + 1], s);
      fns[k++] = kn.func;
    } else if (op.kind == OP_MEMSET) {
      const hipMemsetParams& p = ex->memsets[op.idx];
      if (p.height > 1)
        e = hipMemset2DAsync(p.dst, p.pitch, (int)p.value, p.width, p.height, s);
      else if (p.elementSize == 4)
        e = hipMemsetD32Async((hipDeviceptr_t)p.dst, (int)p.value, p.width, s);
      else if (p.elementSize == 2)
        e = hipMemsetD16Async((hipDeviceptr_t)p.dst, (unsigned short)p.value, p.width, s);
      else
        e = hipMemsetD8Async((hipDeviceptr_t)p.dst, (unsigned char)p.value, p.width, s);
    } else if (op.kind == OP_MEMCPY) {
      const clskd_exec::Flat& f = ex->flat[op.idx];
      e = f.bytes ? hipMemcpyAsync(f.dst, f.src, f.bytes, f.kind, s) : hipMemcpy3DAsync(&ex->memcpys[op.idx], s);
    }  // waits / records: one stream in program order needs none
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(s);
      cleanup();
      return hip_fail("exec_census launch", e);
    }
  }
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    cleanup();
    return hip_fail("hipStreamSynchronize", e);
  }
  for (int i = 0; i < k; ++i) {
    float t = 0.f;
    e = hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail("hipEventElapsedTime", e);
    }
    ms[i] = t;
  }
  cleanup();
  return CLSKD_OK;
}

// Demangled name of a kernel's host stub (the function pointers exec_census reports).  Returns
// the name's length (buf: NUL-terminated, truncated to cap), -1 when HIP does not know the
// function.
extern "C" int32_t clskd_kernel_name(const void* fn, char* buf, int32_t cap) {
  const char* m = fn ? hipKernelNameRefByPtr(fn, nullptr) : nullptr;
  if (!m) {
    (void)hipGetLastError();
    return -1;
  }
  int st = 0;
  char* dm = abi::__cxa_demangle(m, nullptr, nullptr, &st);
  const std::string out = (st == 0 && dm) ? std::string(dm) : std::string(m);
  free(dm);
  if (buf && cap > 0) {
    const size_t nb = out.size() < (size_t)cap - 1 ? out.size() : (size_t)cap - 1;
    memcpy(buf, out.data(), nb);
    buf[nb] = 0;
  }
  return (int32_t)out.size();
}

extern "C" void clskd_exec_destroy(clskd_exec* ex) {
  if (!ex) return;
  drop_timing(ex);
  for (hipEvent_t ev : ex->mk) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : ex->events)
    if (ev) (void)hipEventDestroy(ev);
  if (ex->owns_streams)
    for (hipStream_t s : ex->own)
      if (s) (void)hipStreamDestroy(s);
  delete ex;
}
