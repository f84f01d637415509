// conv_wgrad_x3: the weight gradient of a conv launch (grad.hip's contract, same descriptor, same
// [S][N][K] + [S][N] partial layout for wgrad_reduce_kernel) on the bf16 MFMA pipe with 3 x bf16
// split products, for descriptors of compute CLSKD_F32X3 (the student of precision 'mixed').
//
//     dW[n][k] = sum_rows dY(row, n) * A(row, k)     (A: the forward's K-table gather)
//
// Why a second engine: the exact one (conv_wgrad_f32) runs a 64 x 64 (n, k) tile of
// v_mfma_f32_32x32x2_f32 per 32 rows whatever N and K are — the student's outer layers have N of
// 2-16 and K of 20-384 over 0.3-1.3 M rows, so its MFMA time is mostly padding (1-15 TF/s there,
// 4.6 ms of the C3 step in 28 launches, tools/bwd_census.py).  Here:
//   * v_mfma_f32_16x16x32_bf16 with the ROW axis as the MFMA reduction (32 rows per MFMA): the
//     n side of the tile is 16, 32 or 64 wide (by N), k is 64; x * w ~ hi*hi + hi*lo + lo*hi as in
//     conv_split.hip (hi = bf16(x), lo = bf16(x - hi), fp32 accumulation; each dropped term
//     <= ~2^-16 relative, about 3 * 2^-18 per product);
//   * every wave owns whole 32-row chunks: it gathers its chunk into registers (8 consecutive rows
//     of one k-quad per lane, so the hi/lo planes are written transposed — rows contiguous per
//     column, the MFMA's operand order — as 16-byte runs), writes its own LDS region and reads
//     it back: no workgroup barrier in the row loop; the next chunk's gather is in flight under
//     the current chunk's MFMAs;
//   * the four waves' partial tiles (and the dbias column sums) are added in a fixed order in LDS
//     at the end, so results are bitwise repeatable (no float atomics).
#include <algorithm>

#include "common.h"

namespace clskd {

namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

constexpr int X3_TK = 64;  // k per tile
constexpr int X3_RB = 32;  // rows per wave chunk (the MFMA reduction depth)
constexpr int X3_CS = 40;  // LDS column stride in bf16 elements: 32 rows + 16 B pad (80 B)

struct WgradX3Args {
  clskd_conv_desc d;
  const float* dy;
  float* work;
  int rows_per_split;
  int S;
  int want_bias;
  int xcd;  // XCD-major work order (CLSKD_WGRAD_XCD): the k-tiles of a row chunk on one XCD
};

template <int R> struct RowVec;
template <> struct RowVec<8> { typedef s16x8 T; };
template <> struct RowVec<4> { typedef s16x4 T; };
template <> struct RowVec<2> { typedef s16x2 T; };

__device__ __forceinline__ short bf16_bits(float x) { return __builtin_bit_cast(short, (__bf16)x); }

// hi / lo bf16 split of R row values of one column, packed rows-contiguous
template <int R>
__device__ __forceinline__ void split_col(const float (&v)[R], typename RowVec<R>::T& hi,
                                          typename RowVec<R>::T& lo) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const __bf16 h = (__bf16)v[r];
    hi[r] = __builtin_bit_cast(short, h);
    lo[r] = bf16_bits(v[r] - (float)h);
  }
}

__device__ __forceinline__ f32x4 mfma1632(const s16x8& a, const s16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, a),
                                                  __builtin_bit_cast(bf16x8v, b), c, 0, 0, 0);
}

// (b, fo, to) of row m, and the step to row m + 1
struct RowPos {
  int b = 0, fo = 0, to = 0;
  __device__ __forceinline__ void set(unsigned m, unsigned FoTo, unsigned To) {
    b = (int)(m / FoTo);
    const unsigned r = m - (unsigned)b * FoTo;
    fo = (int)(r / To);
    to = (int)(r - (unsigned)fo * To);
  }
  __device__ __forceinline__ void next(int Fo, int To) {
    if (++to == To) {
      to = 0;
      if (++fo == Fo) {
        fo = 0;
        ++b;
      }
    }
  }
};

// DEPTH: 32-row chunks in flight per wave (1: the next chunk's gather under this chunk's MFMAs;
// 2: two register sets, the gathers of the next two chunks in flight)
template <int TN, bool VEC4, int DEPTH>
__global__ __launch_bounds__(256) void conv_wgrad_x3(const WgradX3Args a) {
  const clskd_conv_desc& d = a.d;
  constexpr int QN = TN / 4;             // dY side: column quads per row
  constexpr int RPL = TN / 8;            // dY side: rows per lane (QN * RPL * 16 = 32 rows * 64 lanes / ... )
  constexpr int LPG = 64 / QN;           // dY side: lanes per column quad (row groups)
  constexpr int PA = X3_TK * X3_CS;      // bf16 elements of one A plane
  constexpr int PD = TN * X3_CS;         // of one dY plane
  constexpr int WAVE_E = 2 * PA + 2 * PD;
  typedef typename RowVec<RPL>::T dvec;
  extern __shared__ __attribute__((aligned(16))) short lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  short* const wl = lds + wave * WAVE_E;  // this wave's planes: A hi, A lo, dY hi, dY lo
  // work item (row chunk, n-tile, k-tile).  The hardware deals workgroups round-robin over the
  // eight XCDs; with a.xcd each XCD instead walks one contiguous run of work items, k-tile
  // fastest, so the k-tiles re-reading one row chunk's dY and gathered rows share its L2
  int split = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
  if (a.xcd) {
    const int ny = gridDim.y, nz = gridDim.z;
    const int total = gridDim.x * ny * nz;
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + ny * blockIdx.z);
    const int v = xcd_tile(lin, total);
    split = v / (ny * nz);
    const int rem = v - split * (ny * nz);
    ty = rem / nz;
    tz = rem - ty * nz;
  }
  const int n0 = ty * TN;
  const int k0 = tz * X3_TK;
  const unsigned M = (unsigned)d.B * d.Fo * d.To;
  const unsigned FoTo = (unsigned)d.Fo * d.To;
  const unsigned r_begin = (unsigned)split * a.rows_per_split;
  const unsigned r_end = min(M, r_begin + (unsigned)a.rows_per_split);
  const bool ncontig = d.oNlo == 1 && d.nlo >= d.N;

  // A side: k-quad kq = lane & 15 (k = k0 + 4 kq .. + 3), rows 8 rg .. 8 rg + 7 of a chunk
  const int kq = lane & 15, rg = lane >> 4;
  clskd_ktab_entry ke[4];
  int kvalid[4];
  const float* kp[4];
  int64_t ksB[4], ksF[4], ksT[4];
  int kF[4], kT[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + kq * 4 + j;
    const int kc = min(k, d.K - 1);
    ke[j] = d.ktab[kc];
    const clskd_seg& g = d.seg[d.kseg[kc]];
    kp[j] = g.ptr;
    ksB[j] = g.sB;
    ksF[j] = g.sF;
    ksT[j] = g.sT;
    kF[j] = g.F;
    kT[j] = g.T;
    kvalid[j] = k < d.K;
  }
  // dY side: column quad nq (n = n0 + 4 nq .. + 3), rows RPL * (lane / QN) ..
  const int nq = lane % QN, dg = lane / QN;

  float av[8][4], dv[RPL][4], av2[8][4], dv2[RPL][4];  // av2 / dv2: the second set (DEPTH 2)
  f32x4 bsum = {0.f, 0.f, 0.f, 0.f};
  const bool bias_lane = a.want_bias && tz == 0;

  // loop-invariant parts of the addressing: the vec4 quad's base and row strides, the dY
  // column offsets of this lane's n-quad
  const float* const qbase = kp[0] + ke[0].off;
  const int64_t sFs = ksF[0] * d.stride_f, sTs = ksT[0] * d.stride_t;
  const int nl = n0 + 4 * nq;
  const bool dvec4 = ncontig && nl + 3 < d.N;
  int64_t coff[4];
  bool cval[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nl + j;
    cval[j] = n < d.N;
    coff[j] = cval[j] ? (int64_t)(n / d.nlo) * d.oNhi + (int64_t)(n % d.nlo) * d.oNlo : 0;
  }

  auto gather = [&](unsigned rc, float (&xa)[8][4], float (&xd)[RPL][4]) {  // chunk rows rc .. rc + 31
    {
      RowPos p;
      const unsigned m0 = rc + 8 * rg;
      if (m0 < r_end) p.set(m0, FoTo, d.To);
      // the lane's 8 rows share (b, fo) — all but ~1 % of row groups: one row base, a stride
      const bool fast = VEC4 && m0 + 7 < r_end && p.to + 7 < d.To;
      if (fast) {
        const int fi = p.fo * d.stride_f + ke[0].dF;
        const bool fok = kvalid[0] && fi >= 0 && fi < kF[0];
        const float* rp = qbase + p.b * ksB[0] + p.fo * sFs + p.to * sTs;
        const int ti0 = p.to * d.stride_t + ke[0].dT;
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const int ti = ti0 + rr * d.stride_t;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (fok && ti >= 0 && ti < kT[0]) v = *reinterpret_cast<const f32x4*>(rp + rr * sTs);
#pragma unroll
          for (int j = 0; j < 4; ++j) xa[rr][j] = v[j];
        }
      } else {
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const bool valid = m0 + rr < r_end;
          if constexpr (VEC4) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            const int64_t fi = (int64_t)p.fo * d.stride_f + ke[0].dF, ti = (int64_t)p.to * d.stride_t + ke[0].dT;
            if (valid && kvalid[0] && fi >= 0 && fi < kF[0] && ti >= 0 && ti < kT[0])
              v = *reinterpret_cast<const f32x4*>(qbase + p.b * ksB[0] + p.fo * sFs + p.to * sTs);
#pragma unroll
            for (int j = 0; j < 4; ++j) xa[rr][j] = v[j];
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int64_t fi = (int64_t)p.fo * d.stride_f + ke[j].dF, ti = (int64_t)p.to * d.stride_t + ke[j].dT;
              float v = 0.f;
              if (valid && kvalid[j] && fi >= 0 && fi < kF[j] && ti >= 0 && ti < kT[j])
                v = kp[j][p.b * ksB[j] + (int64_t)p.fo * d.stride_f * ksF[j] +
                          (int64_t)p.to * d.stride_t * ksT[j] + ke[j].off];
              xa[rr][j] = v;
            }
          }
          if (valid) p.next(d.Fo, d.To);
        }
      }
    }
    {
      RowPos p;
      const unsigned m0 = rc + RPL * dg;
      if (m0 < r_end) p.set(m0, FoTo, d.To);
      const bool fast = m0 + RPL - 1 < r_end && p.to + RPL - 1 < d.To;
      const int64_t orow0 = (int64_t)p.b * d.oB + (int64_t)(p.fo * d.of_mul + d.of_add) * d.oF +
                            (int64_t)p.to * d.oT;
#pragma unroll
      for (int rr = 0; rr < RPL; ++rr) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const bool valid = m0 + rr < r_end;
        if (valid) {
          const int64_t orow = fast ? orow0 + rr * d.oT
                                    : (int64_t)p.b * d.oB + (int64_t)(p.fo * d.of_mul + d.of_add) * d.oF +
                                          (int64_t)p.to * d.oT;
          if (dvec4 && ((orow + nl) & 3) == 0) {
            v = *reinterpret_cast<const f32x4*>(a.dy + orow + nl);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (cval[j]) v[j] = a.dy[orow + coff[j]];
          }
          if (!fast) p.next(d.Fo, d.To);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) xd[rr][j] = v[j];
        if (bias_lane) bsum += v;
      }
    }
  };

  // registers -> this wave's hi / lo planes, transposed (rows contiguous)
  auto stage = [&](const float (&xa)[8][4], const float (&xd)[RPL][4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float col[8];
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) col[rr] = xa[rr][c];
      s16x8 hi, lo;
      split_col<8>(col, hi, lo);
      const int off = (kq * 4 + c) * X3_CS + 8 * rg;
      *reinterpret_cast<s16x8*>(wl + off) = hi;
      *reinterpret_cast<s16x8*>(wl + PA + off) = lo;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float col[RPL];
#pragma unroll
      for (int rr = 0; rr < RPL; ++rr) col[rr] = xd[rr][c];
      dvec hi, lo;
      split_col<RPL>(col, hi, lo);
      const int off = (nq * 4 + c) * X3_CS + RPL * dg;
      *reinterpret_cast<dvec*>(wl + 2 * PA + off) = hi;
      *reinterpret_cast<dvec*>(wl + 2 * PA + PD + off) = lo;
    }
  };

  constexpr int NB = TN / 16, KB = X3_TK / 16;
  f32x4 acc[NB][KB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < KB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int l16 = lane & 15, lg = lane >> 4;
  auto compute = [&]() {  // this wave's planes -> 3 x (NB x KB) MFMAs
    s16x8 bh[KB], bl[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      const int off = (j * 16 + l16) * X3_CS + 8 * lg;
      bh[j] = *reinterpret_cast<const s16x8*>(wl + off);
      bl[j] = *reinterpret_cast<const s16x8*>(wl + PA + off);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int off = (i * 16 + l16) * X3_CS + 8 * lg;
      const s16x8 ah = *reinterpret_cast<const s16x8*>(wl + 2 * PA + off);
      const s16x8 al = *reinterpret_cast<const s16x8*>(wl + 2 * PA + PD + off);
#pragma unroll
      for (int j = 0; j < KB; ++j) acc[i][j] = mfma1632(ah, bh[j], acc[i][j]);
#pragma unroll
      for (int j = 0; j < KB; ++j) acc[i][j] = mfma1632(ah, bl[j], acc[i][j]);
#pragma unroll
      for (int j = 0; j < KB; ++j) acc[i][j] = mfma1632(al, bh[j], acc[i][j]);
    }
  };

  constexpr unsigned STEP = 4 * X3_RB;  // the workgroup's four waves take consecutive chunks
  unsigned rc = r_begin + (unsigned)wave * X3_RB;
  if (rc < r_end) gather(rc, av, dv);
  if (DEPTH == 2 && rc + STEP < r_end) gather(rc + STEP, av2, dv2);
  bool second = false;  // DEPTH 2: this chunk sits in the second set
  for (; rc < r_end; rc += STEP) {
    if (second)
      stage(av2, dv2);
    else
      stage(av, dv);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: planes written
    const unsigned nx = rc + DEPTH * STEP;  // refill the set just staged: in flight under the MFMAs
    if (nx < r_end) {
      if (second)
        gather(nx, av2, dv2);
      else
        gather(nx, av, dv);
    }
    compute();
    if (DEPTH == 2) second = !second;
  }

  // ---- the four waves' tiles added in LDS (fixed order), partial tile out: work[split][n][k] ----
  __syncthreads();  // every wave is done with its planes
  float* red = reinterpret_cast<float*>(lds);  // [4][TN][64]
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < KB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * TN + i * 16 + lg * 4 + r) * X3_TK + j * 16 + l16] = acc[i][j][r];
  f32x4* bred = reinterpret_cast<f32x4*>(red + 4 * TN * X3_TK);  // [4][64]
  if (bias_lane) bred[wave * 64 + lane] = bsum;
  __syncthreads();
  const int K = d.K;
  float* wp = a.work + (int64_t)split * d.N * K;
  for (int idx = tid; idx < TN * X3_TK; idx += 256) {
    const int n = n0 + idx / X3_TK, k = k0 + idx % X3_TK;
    const float s = ((red[idx] + red[TN * X3_TK + idx]) + red[2 * TN * X3_TK + idx]) + red[3 * TN * X3_TK + idx];
    if (n < d.N && k < K) wp[(int64_t)n * K + k] = s;
  }
  if (bias_lane && tid < TN && n0 + tid < d.N) {
    const int q = tid / 4, c = tid % 4;
    float s = 0.f;
    for (int w = 0; w < 4; ++w)
      for (int g = 0; g < LPG; ++g) s += bred[w * 64 + g * QN + q][c];
    a.work[(int64_t)a.S * d.N * K + (int64_t)split * d.N + n0 + tid] = s;
  }
}

inline int x3_tn(int N) { return N <= 16 ? 16 : N <= 32 ? 32 : 64; }

template <int TN, bool VEC4, int DEPTH>
void launch_x3(dim3 grid, hipStream_t st, const WgradX3Args& a) {
  constexpr size_t lds = (size_t)4 * (2 * X3_TK * X3_CS + 2 * TN * X3_CS) * 2;
  static_assert(lds >= (size_t)4 * TN * X3_TK * 4 + 4 * 64 * 16, "the reduction fits the planes");
  const void* k = (const void*)conv_wgrad_x3<TN, VEC4, DEPTH>;
  static const bool attr = lds <= 64 * 1024 ||
      hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  (void)attr;
  hipLaunchKernelGGL((conv_wgrad_x3<TN, VEC4, DEPTH>), grid, dim3(256), lds, st, a);
  note_kernel_fn(k);
}

}  // namespace

// rows per split (a multiple of the 128 rows one workgroup round covers): about 1024 workgroups
void wgrad_x3_plan(const clskd_conv_desc& d, int& S, int64_t& rps) {
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  const int tn = x3_tn(d.N);
  const int64_t tiles = cdiv(d.N, tn) * cdiv(d.K, X3_TK);
  int64_t s = cdiv(1024, tiles);
  s = std::max<int64_t>(1, std::min<int64_t>({s, (int64_t)1024, cdiv(M, 512)}));
  rps = cdiv(cdiv(M, s), 4 * X3_RB) * 4 * X3_RB;
  S = (int)cdiv(M, rps);
}

bool wgrad_x3_takes(const clskd_conv_desc& d) {
  const int64_t M = (int64_t)d.B * d.Fo * d.To;
  return d.compute == CLSKD_F32X3 && M < ((int64_t)1 << 31) - 1024;
}

void launch_wgrad_x3(const clskd_conv_desc& d, const float* dy, float* work, int S, int64_t rps,
                     int want_bias, hipStream_t st) {
  WgradX3Args a{d, dy, work, (int)rps, S, want_bias, knob(KNOB_WGRAD_XCD) != 0 ? 1 : 0};
  const int tn = x3_tn(d.N);
  // chunks in flight per wave (CLSKD_WGRAD_DEPTH 1 / 2; 0 = by instance): two for the vec4
  // gathers of the narrow tiles, where the second register set keeps the occupancy and the
  // gather latency is what a chunk waits on (n2-n32: -18..-22 %); one for TN = 64 (328 VGPRs at
  // two: one wave per SIMD, +40..50 %) and the scalar gathers (+70 %) (tools/wgrad_micro.py)
  const int dk = knob(KNOB_WGRAD_DEPTH);
  const int depth = dk == 1 || dk == 2 ? dk : (d.vec4 && tn <= 32 ? 2 : 1);
  dim3 grid(S, (unsigned)cdiv(d.N, tn), (unsigned)cdiv(d.K, X3_TK));
  const bool v = d.vec4 != 0;
  if (tn == 16) {
    if (v) depth == 2 ? launch_x3<16, true, 2>(grid, st, a) : launch_x3<16, true, 1>(grid, st, a);
    else depth == 2 ? launch_x3<16, false, 2>(grid, st, a) : launch_x3<16, false, 1>(grid, st, a);
  } else if (tn == 32) {
    if (v) depth == 2 ? launch_x3<32, true, 2>(grid, st, a) : launch_x3<32, true, 1>(grid, st, a);
    else depth == 2 ? launch_x3<32, false, 2>(grid, st, a) : launch_x3<32, false, 1>(grid, st, a);
  } else {
    if (v) depth == 2 ? launch_x3<64, true, 2>(grid, st, a) : launch_x3<64, true, 1>(grid, st, a);
    else depth == 2 ? launch_x3<64, false, 2>(grid, st, a) : launch_x3<64, false, 1>(grid, st, a);
  }
  note_kernel("conv_wgrad_x3<%d,%s,%d>", tn, v ? "true" : "false", depth);
}

}  // namespace clskd
