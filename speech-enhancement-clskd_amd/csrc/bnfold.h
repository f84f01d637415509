// Folded BatchNorm finalize (round 4): the conv launch that produces a BatchNorm's batch
// statistics also turns them into the normalisation coefficients — no bn_finalize launch.
//
// Every workgroup reduces its rows (all its tiles) to one fp64 {sum, sumsq} per channel, splits
// each value EXACTLY into three fixed-point int64 limbs (2^20, 2^-22 and 2^-64 units) and adds
// them with agent-scope int64 atomics into one of REPL accumulator replicas.  Integer addition is
// associative, so the totals — and the coefficients — do not depend on the order in which
// workgroups arrive: bitwise reproducible like the fixed-order partial reduction it replaces.
// The atomics execute at the memory side; a workgroup signals with one agent-scope ticket add
// after every wave's vmcnt(0) (the atomics are then performed), and the workgroup that draws the
// last ticket of the layer's finalizing launch reads the replicas back with exchange(0) atomics —
// which also return the accumulators to zero for the next use — and writes scale / shift, the
// batch mean / var and the running statistics (bn_channel_coeffs, the same arithmetic as
// clskd_bn_finalize).  The ticket is reset by that workgroup too: state is zero at rest, so
// replays (graphs, the step executor) need no memset.  MI355X_MICROARCH.md §visibility: "8-B
// agent atomics both sides" is a valid hand-off form.
#pragma once
#include "common.h"

namespace clskd {

constexpr int BNF_REPL = CLSKD_BN_FOLD_REPL;  // replicas: <= 32 adders per address at 256 workgroups

struct BnFoldArgs {
  long long* acc;     // [REPL][C][2][3] limbs (nullptr: no fold)
  unsigned* ticket;
  int32_t finalize;   // this launch's last workgroup finalizes
  int32_t C, c_off;   // channels of the BatchNorm; this launch's first channel
  int32_t n_updates;
  int64_t count;      // rows of the whole layer
  const float* gamma;
  const float* beta;
  float eps, momentum;
  float* running_mean;
  float* running_var;
  float* scale;
  float* shift;
  float* mean_out;
  float* var_out;
};

inline BnFoldArgs make_bnfold(const clskd_conv_desc& d) {
  BnFoldArgs f{};
  if (const clskd_bn_fold* b = d.bn_fold) {
    f.acc = reinterpret_cast<long long*>(b->acc);
    f.ticket = reinterpret_cast<unsigned*>(b->ticket);
    f.finalize = b->finalize;
    f.C = b->C;
    f.c_off = b->c_off;
    f.n_updates = b->n_updates;
    f.count = b->count;
    f.gamma = b->gamma;
    f.beta = b->beta;
    f.eps = b->eps;
    f.momentum = b->momentum;
    f.running_mean = b->running_mean;
    f.running_var = b->running_var;
    f.scale = b->scale;
    f.shift = b->shift;
    f.mean_out = b->mean_out;
    f.var_out = b->var_out;
  }
  return f;
}

// exact split of v (|v| < 2^61) into q2 * 2^20 + q1 * 2^-22 + q0 * 2^-64 (q0 rounded: below
// 2^-64 absolute nothing is kept); every q fits 42 bits, so 2^20 contributions cannot overflow
__device__ __forceinline__ void bnf_limbs(double v, long long& q2, long long& q1, long long& q0) {
  const double f2 = floor(v * 0x1p-20);
  const double r = v - f2 * 0x1p20;    // exact, in [0, 2^20)
  const double f1 = floor(r * 0x1p22);
  const double r1 = r - f1 * 0x1p-22;  // exact, in [0, 2^-22)
  q2 = (long long)f2;
  q1 = (long long)f1;
  q0 = (long long)rint(r1 * 0x1p64);
}

__device__ __forceinline__ double bnf_value(long long s2, long long s1, long long s0) {
  return ((double)s2 * 0x1p20 + (double)s1 * 0x1p-22) + (double)s0 * 0x1p-64;
}

// Called by EVERY thread of the workgroup (uniform control flow) after the workgroup's own
// statistics are final: S(n), Q(n) for the launch's channels n in [0, N) (channel c_off + n of
// the BatchNorm).  `flag` is one int of LDS the caller does not use concurrently (the last-
// arriver broadcast).  nthreads = blockDim.x; wg / nwg = this workgroup's index and the launch's
// workgroup count.
template <typename SQ>
__device__ __forceinline__ void bnfold_commit(const BnFoldArgs& f, int N, SQ sq, int* flag,
                                              int wg, int nwg) {
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  long long* rep = f.acc + (int64_t)(wg % BNF_REPL) * f.C * 6;
  for (int i = tid; i < 2 * N; i += nt) {
    const int n = i >> 1, w = i & 1;
    double S, Q;
    sq(n, S, Q);
    long long q2, q1, q0;
    bnf_limbs(w ? Q : S, q2, q1, q0);
    long long* p = rep + ((int64_t)(f.c_off + n) * 2 + w) * 3;
    __hip_atomic_fetch_add(p, q2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(p + 1, q1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(p + 2, q0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!f.finalize) return;  // uniform: an earlier launch of the layer only contributes
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics are performed
  __syncthreads();
  // Ordering without an agent release/acquire: every access to the replicas and to the ticket is
  // an 8-/4-B agent-scope atomic, performed at the memory side ("agent atomics both sides",
  // MI355X_MICROARCH.md §Workgroup dispatch, Valid forms), and a no-return atomic stays counted
  // in vmcnt until it is performed (§Global float atomics), so the vmcnt(0) + barrier above put
  // every limb add of this workgroup before its ticket add.  An acq_rel ticket would lower to
  // buffer_wbl2 sc1 + buffer_inv sc1 per workgroup — a write-back of the XCD L2 right after the
  // conv's output tiles were stored (redraw: a 4 % step regression measured for a
  // fence per workgroup) — and guard no non-atomic hand-off: the coefficients the last arriver
  // writes are read by later kernels only (kernel boundary).
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(f.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = t == (unsigned)(nwg - 1);
  }
  __syncthreads();
  if (!*flag) return;
  // the last workgroup: every contribution of every launch of the layer is in the replicas
  for (int c = tid; c < f.C; c += nt) {
    long long L[2][3] = {{0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int r = 0; r < BNF_REPL; ++r) {
      long long* p = f.acc + ((int64_t)r * f.C + c) * 6;
#pragma unroll
      for (int k = 0; k < 6; ++k)
        L[k / 3][k % 3] += __hip_atomic_exchange(p + k, 0ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    bn_channel_coeffs(c, bnf_value(L[0][0], L[0][1], L[0][2]), bnf_value(L[1][0], L[1][1], L[1][2]),
                      f.count, f.gamma, f.beta, f.eps, f.running_mean, f.running_var, f.momentum,
                      f.n_updates, f.scale, f.shift, f.mean_out, f.var_out);
  }
  if (tid == 0) __hip_atomic_store(f.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace clskd
