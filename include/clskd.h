/*
 * clskd.h — C ABI of libclskd_hip.so, the MI355X (gfx950) hot path of DCCRN + CLSKD.
 *
 * The reference has no FFI: its hot path sits behind PyTorch nn.Module calls
 * (SURVEY.md §8 b).  Each entry point below replaces one reference operator; the Python
 * package `clskd` (speech-enhancement-clskd_amd/clskd) binds them with ctypes and keeps the
 * reference's module/function names and signatures.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer owned by the caller (no allocations are kept across
 *     calls; no hidden host<->device copies or syncs, so every call is hipGraph-capturable).
 *   - Activations use the "BFTC" layout: [batch][freq][time][channel], channel fastest.  The
 *     reference's NCHW tensor x[b][c][f][t] is x_bftc[b][f][t][c].
 *   - Work is enqueued on `stream` (a hipStream_t; NULL = default stream).
 *   - Return 0 on success, a negative clskd_status otherwise; clskd_last_error() returns a
 *     thread-local message.  No exceptions or aborts cross the ABI.
 *   - Storage is fp32 or bf16 per tensor (dtype arguments); GEMM-shaped ops accumulate in fp32.
 */
#ifndef CLSKD_H
#define CLSKD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  CLSKD_OK = 0,
  CLSKD_E_SHAPE = -1,
  CLSKD_E_DTYPE = -2,
  CLSKD_E_HIP = -3,
  CLSKD_E_ARG = -4
} clskd_status;

/* storage / MFMA operand types.  CLSKD_F16 (IEEE half) is the operand type of configuration C4
 * (distill_SPKD.py at fp16): the conv engines, BN and STFT-side kernels of a DCCRN forward
 * take it wherever they take bf16.  CLSKD_F32X3 (conv descriptors only, fp32 storage): fp32
 * products formed from three bf16 MFMA products of split operands (hi = bf16(x), lo =
 * bf16(x - hi): hi*hi + hi*lo + lo*hi, fp32 accumulation; <= ~3 * 2^-18 relative per product)
 * where the split engine takes the layer, the exact fp32 engines elsewhere. */
typedef enum { CLSKD_F32 = 0, CLSKD_BF16 = 1, CLSKD_F16 = 2, CLSKD_F32X3 = 3 } clskd_compute;

const char* clskd_last_error(void);
int clskd_version(void);

/* Dispatch knobs (engine A/B switches, grid caps, LSTM k-slicing): each is read from the
 * environment variable of the same name once, at the library's first launch, and can be changed
 * afterwards only through clskd_set_knob (tests, tools) — never per launch from the environment.
 * Every knob selects between kernels that compute the same result.  The timing-only experiment
 * modes that do not (CLSKD_G8 >= 10, CLSKD_LSTM128_TDIV, CLSKD_LSTM32_TDIV,
 * CLSKD_BF16_DEBUG_MODE) exist only in a -DCLSKD_EXPERIMENTS build; in the product build a
 * non-zero value makes the affected launch return CLSKD_E_ARG instead of a wrong result.
 * clskd_set_knob / clskd_get_knob return CLSKD_E_ARG for an unknown name. */
int clskd_set_knob(const char* name, int32_t value);
int clskd_get_knob(const char* name, int32_t* value);
/* 1 when the library was built with -DCLSKD_EXPERIMENTS (timing-only modes present), else 0. */
int clskd_experiments_build(void);

/* ------------------------------------------------------------------------------------------
 * Implicit-GEMM convolution over BFTC activations.
 * Replaces: ComplexConv2d.forward (tools_for_model.py:236-262, packed [[Wr,-Wi],[Wi,Wr]]),
 *           ComplexConvTranspose2d.forward (tools_for_model.py:303-330, polyphase),
 *           ABF conv1/conv2/att 1x1 & 3x3 convs (framework.py:179-191),
 *           ConvSTFT / ConviSTFT framing GEMMs (tools_for_model.py:53-67, 90-109),
 *           nn.LSTM input projections and NavieComplexLSTM Linear projections
 *           (tools_for_model.py:164-173).
 *
 * out[b, fo, to, n] = bias[n] + sum_k A[(b,fo,to), k] * W[n, k]
 * A is gathered through a K table: for K index k with ktab[k] = {off, dF, dT}, s = kseg[k]:
 *   fi = fo*stride_f + dF,  ti = to*stride_t + dT
 *   A[(b,fo,to), k] = seg[s].ptr[b*sB + (fo*stride_f)*sF + (to*stride_t)*sT + off]
 *                     if 0 <= fi < seg[s].F and 0 <= ti < seg[s].T, else 0
 * where the host folds the displacement into off (off = cin + dF*sF + dT*sT).  K is padded to a
 * multiple of 16 with entries whose dF = -32768 (always out of bounds) and zero weights.
 * ConvTranspose2d(stride (2,1)) runs as two polyphase launches (output fo = 2*j + parity,
 * of_mul = 2, of_add = parity) with the parity's taps in the K table.
 * -------------------------------------------------------------------------------------- */
#define CLSKD_MAX_SEGS 4

typedef struct {
  const float* ptr; /* segment base (already offset to its first channel / time) */
  int64_t sB, sF, sT; /* element strides; channel stride is 1 inside a K-table entry */
  int32_t F, T;       /* bounds for the gathered freq / time index */
} clskd_seg;

typedef struct {
  int32_t off; /* element offset added after the row offset (cin*sC + dF*sF + dT*sT) */
  int16_t dF;  /* freq displacement (bounds check) */
  int16_t dT;  /* time displacement (bounds check) */
} clskd_ktab_entry; /* 8 bytes; seg index is stored in ktab_seg[k] */

typedef struct {
  /* geometry: output rows are (b, fo, to), fo in [0,Fo), to in [0,To) */
  int32_t B, Fo, To;
  int32_t N, K;         /* output channels, reduction length */
  int32_t stride_f;     /* fi = fo*stride_f + dF  (convT polyphase: fo=j, stride 1) */
  int32_t stride_t;     /* ti = to*stride_t + dT */
  int32_t nseg;
  clskd_seg seg[CLSKD_MAX_SEGS];
  const clskd_ktab_entry* ktab; /* device, K entries */
  const uint8_t* kseg;          /* device, K entries: segment index of each k */
  int32_t vec4;                 /* 1: every aligned group of 4 k's is 4 contiguous channels */
  const void* weight;  /* device [N][K] packed, fp32 (compute F32) or bf16 / f16 (compute BF16 / F16) */
  const float* bias;   /* device [N] or NULL */
  /* output address: out + b*oB + (fo*of_mul+of_add)*oF + to*oT + (n/nlo)*oNhi + (n%nlo)*oNlo */
  void* out;
  int64_t oB, oF, oT, oNhi, oNlo;
  int32_t nlo, of_mul, of_add;
  int32_t compute;   /* clskd_compute: MFMA operand type */
  int32_t in_dtype;  /* CLSKD_F32 / CLSKD_BF16 / CLSKD_F16 storage of every segment (= compute;
                        bf16 needs segment channel runs of 8 and strides % 8) */
  int32_t out_dtype; /* CLSKD_F32 / CLSKD_BF16 / CLSKD_F16 storage of `out` (16-bit outs match in_dtype) */
  double* stats;     /* optional fused BatchNorm statistics: per M-block (128 output rows) fp64
                        partials stats[blockIdx.x][N][2] = {sum, sumsq} of the biased outputs,
                        consumed by clskd_bn_finalize (nblk = number of M-blocks) */
  int32_t kvec;      /* channel-run granule of the K table: every aligned group of kvec k's is
                        kvec contiguous channels of one tap and segment (1, 2, 4 or 8; 0 = 8 for
                        bf16 segments, 4 if vec4, else 1).  Sets the direct-conv load width. */
  int32_t wlayout;   /* CLSKD_WLAYOUT_NK: weight [N][K] -> implicit-GEMM MFMA engines.
                        CLSKD_WLAYOUT_DIRECT: weight k-major [K][NP] fp32, or [K/2][NP][2] bf16
                        (pairs of consecutive k), NP = clskd_conv_direct_np(N), zero columns for
                        n >= N -> direct-convolution kernel (narrow GEMMs: N <= 16, or K <= 64
                        with N <= 64; see clskd_conv_direct_ok). */
  /* Optional K-table structure (ntaps = 0: not provided).  When given, K is ordered (tap,
     segment, channel) with ctot = sum(seg_c) channels per tap and tap t's displacement
     (tap_df[t], tap_dt[t]); this lets small-N bf16 launches run the halo-tiled kernel (input
     tile staged once per channel chunk and reused across taps, weights resident in LDS). */
  int32_t ntaps;
  int32_t ctot;
  int32_t seg_c[CLSKD_MAX_SEGS];
  int16_t tap_df[16];
  int16_t tap_dt[16];
  /* 1: out += result (read-modify-write, fp32 `out`, no statistics: the fp32 MFMA engines with
     wlayout NK, the direct kernel with wlayout DIRECT for narrow N / short K, or — bf16 compute —
     the bf16 LDS-DMA engine) — lets several data-gradient contributions of one tensor sum in
     place. */
  int32_t accumulate;
  int32_t reserved_;
  /* Optional folded BatchNorm finalize (HOST pointer, read at launch; NULL = none): the launch
     accumulates its output channels' batch statistics (fixed-point, order-independent) into
     bn_fold->acc and, when bn_fold->finalize, its last workgroup writes the coefficients — no
     clskd_bn_finalize launch.  Only for launches clskd_conv_fold_capable() accepts; `stats`
     must then be NULL. */
  const struct clskd_bn_fold_s* bn_fold;
} clskd_conv_desc;

/* ------------------------------------------------------------------------------------------
 * Folded BatchNorm finalize (round 4; replaces the clskd_bn_finalize launch after a conv with
 * fused statistics — the finalize of nn.BatchNorm2d.forward in train mode, tools_for_model.py
 * encoder/decoder blocks, framework.py:188-199 ABF BatchNorms).  A BatchNorm's launches all
 * point at the same acc/ticket state (device, zero at rest, returned to zero by the finalizing
 * workgroup); the LAST launch of the layer carries finalize = 1.  Coefficients: scale = gamma *
 * invstd, shift = beta - mean * scale; batch mean / var (biased) optionally; running statistics
 * updated n_updates times with the unbiased variance (as clskd_bn_finalize).
 * clskd_bn_fold_state_size(C): int64 elements of acc for C channels (CLSKD_BN_FOLD_REPL replicas).
 * clskd_conv_fold_capable(d): 1 if the kernel d dispatches to folds the finalize (the persistent
 *                     engines: conv_gemm8, conv_halo, conv_halo_f32), else 0 (use `stats` +
 *                     clskd_bn_finalize).
 * -------------------------------------------------------------------------------------- */
#define CLSKD_BN_FOLD_REPL 8
typedef struct clskd_bn_fold_s {
  int64_t* acc;            /* device [REPL][C][2][3] int64, zero at rest */
  uint32_t* ticket;        /* device, zero at rest */
  int32_t finalize;        /* 1 on the layer's last launch */
  int32_t C;               /* BatchNorm channels */
  int32_t c_off;           /* the launch's first channel (column-split / output-offset launches) */
  int32_t n_updates;       /* running-statistics updates (0: none) */
  int64_t count;           /* rows of the whole layer (all launches) */
  const float* gamma;      /* [C] or NULL (1) */
  const float* beta;       /* [C] or NULL (0) */
  float eps, momentum;
  float* running_mean;     /* [C] or NULL */
  float* running_var;
  float* scale;            /* out [C] */
  float* shift;            /* out [C] */
  float* mean_out;         /* out [C] or NULL */
  float* var_out;          /* out [C] or NULL */
} clskd_bn_fold;

int64_t clskd_bn_fold_state_size(int32_t C);
/* clskd_abf_bn1_partials with the finalize folded (fold->C = 64 conv1 channels, finalize = 1,
 * count = B*F*T): the ABF conv1 BatchNorm's coefficients straight from the tap's moments. */
int clskd_abf_bn1_fold(const float* s, int32_t B, int32_t F, int32_t T, int64_t sB, int64_t sF,
                       int64_t sT, int32_t cin, const float* w1, const clskd_bn_fold* fold,
                       int32_t nblk, void* stream);
int32_t clskd_conv_fold_capable(const clskd_conv_desc* d);

#define CLSKD_WLAYOUT_NK 0
#define CLSKD_WLAYOUT_DIRECT 1

int clskd_conv2d_fwd(const clskd_conv_desc* d, void* stream);
/* Instance name ("kernel<template args>", as rocprofv3 reports it) of the kernel the calling
 * thread's last successful clskd_conv2d_fwd launched — the dispatch policy (direct / halo /
 * 128- or 256-row bf16 engine / fp32 engine) is the library's, so hosts label timings with it. */
const char* clskd_conv_last_kernel(void);
/* Host function (kernel stub address) of that kernel: the key clskd_exec_profile times by. */
const void* clskd_conv_last_kernel_fn(void);
/* 1 if that launch was a conv_gemm8 stream-K launch (round 5): the K-tile units of all tiles split
 * evenly over the persistent grid, a tile shared by two workgroups finished by the later one
 * (per-tile ticket, fp32 partial handed over write-through).  Deterministic for a fixed grid;
 * CLSKD_G8_SK=0 keeps the data-parallel tile deal. */
int32_t clskd_conv_last_stream_k(void);
/* Allocate the stream-K workspace of `stream` (128 MiB partial slabs + tickets, zero at rest).
 * Done implicitly by the first conv on a stream outside graph capture; hosts call it for a stream
 * they are about to capture on, so captured and eager launches take the same path. */
int clskd_stream_prepare(void* stream);
/* Stream-K workspaces of one graph capture (round 6).  A launch made while its stream is being
 * captured never uses the stream's own workspace (the graph is replayed on other streams, and two
 * graphs captured on one stream may replay concurrently); it uses the workspace the capturing
 * thread's bound scope holds for that stream, or runs the data-parallel tile deal when there is
 * none.  begin (outside capture): allocate a zeroed workspace for each of `streams` and bind the
 * scope to the calling thread; end: unbind (after the capture); free: release it once no replay
 * of the graph is queued or will be launched again. */
int clskd_capture_scope_begin(void* const* streams, int32_t nstreams, void** scope);
int clskd_capture_scope_end(void* scope);
int clskd_capture_scope_free(void* scope);
/* Direct-path helpers: padded output width NP of the direct layout, and whether an (N, K)
 * GEMM is served by the direct kernel (returns 1) — hosts pack CLSKD_WLAYOUT_DIRECT weights
 * exactly when this is 1. */
int clskd_conv_direct_np(int32_t N);
int clskd_conv_direct_ok(int32_t N, int32_t K);

/* ------------------------------------------------------------------------------------------
 * BatchNorm2d (train or eval) + optional PReLU over a BFTC tensor of `rows` x C.
 * Replaces nn.BatchNorm2d / nn.PReLU inside the encoder/decoder Sequentials
 * (DCCRN.py:69-141) and the ABF BNs (framework.py:179-186).
 *   clskd_bn_stats_partial: per-block fp64 partial sums -> partial[nblk][C][2]
 *   clskd_bn_finalize: mean/var (biased) -> scale/shift; running stats update (momentum,
 *                      unbiased var) applied `n_updates` times when running_* != NULL
 *   clskd_bn_apply: y = x*scale[c] + shift[c]; if alpha: y = y>=0 ? y : alpha*y
 *   x / y storage is fp32 or bf16 (`dtype`, clskd_compute values); statistics are fp64/fp32.
 * -------------------------------------------------------------------------------------- */
int clskd_bn_stats_partial(const void* x, int64_t rows, int32_t C, double* partial,
                           int32_t nblk, int32_t dtype, void* stream);
/* clskd_bn_compact: level-2 reduction of [nblk][C][2] partials into [ceil(nblk/group)][C][2]
 * (fixed-order group sums).  Optional: clskd_bn_finalize reads any nblk directly (16-B loads,
 * eight in flight per lane; above 1,024 rows after an in-place fold, below). */
int clskd_bn_compact(const double* partial, int32_t nblk, int32_t C, int32_t group, double* out,
                     void* stream);
/* clskd_bn_finalize / clskd_bn_bwd_from_partials treat `partial` as scratch: above 1,024 rows
 * they fold it in place to 512 rows first (fixed order, CLSKD_BN_PFOLD bit 2 / bit 1), so its
 * contents are undefined after the call. */
int clskd_bn_finalize(double* partial, int32_t nblk, int64_t rows, int32_t C,
                      const float* gamma, const float* beta, float eps,
                      float* running_mean, float* running_var, float momentum,
                      int32_t n_updates, float* scale, float* shift, float* mean_out,
                      float* var_out, void* stream);
int clskd_bn_eval_coeffs(const float* running_mean, const float* running_var,
                         const float* gamma, const float* beta, float eps, int32_t C,
                         float* scale, float* shift, void* stream);
int clskd_bn_apply(const void* x, void* y, int64_t rows, int32_t C, const float* scale,
                   const float* shift, const float* alpha, int32_t dtype, void* stream);
/* clskd_bn_apply_reim: as clskd_bn_apply with asteroid's OnReIm(PReLU) (one slope per part):
 * alpha_re_im[0] for channels [0, C/2) (real), alpha_re_im[1] for [C/2, C) (imaginary). */
int clskd_bn_apply_reim(const void* x, void* y, int64_t rows, int32_t C, const float* scale,
                        const float* shift, const float* alpha_re_im, int32_t dtype,
                        void* stream);
int32_t clskd_bn_partial_blocks(int64_t rows, int32_t C);

/* ------------------------------------------------------------------------------------------
 * Complex LSTM recurrence (tools_for_model.py:159-174, nn.LSTM gates i,f,g,o, zero state).
 * gx:  [nws][nseq][T][4H]  precomputed x@W_ih^T + b_ih + b_hh (nws weight sets: real_lstm,
 *      imag_lstm), with element stride: gx + ws*gx_ws + s*gx_seq + t*gx_t + g
 * whh: [nws][4H][H];  out: h_t as out + ws*o_ws + s*o_seq + t*o_t + j
 * -------------------------------------------------------------------------------------- */
int clskd_lstm_recurrent(const float* gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
                         const float* whh, int32_t nws, int32_t nseq, int32_t T, int32_t H,
                         float* out, int64_t o_ws, int64_t o_seq, int64_t o_t, void* stream);
/* Taped forward (training): as clskd_lstm_recurrent, and gx is overwritten in place with the gate
 * pre-activations gx + W_hh h_{t-1} of every step — the `pre` input of clskd_lstm_bwd, so the
 * backward does not recompute them with a GEMM over the saved history.  Only where
 * clskd_lstm_pre_capable(H) (the single-wave H = 32 kernel; CLSKD_LSTM_PRE=0 turns it off). */
int clskd_lstm_pre_capable(int32_t H);
/* cbuf (optional, round 6): nws*nseq*T*H floats, [ws][seq][t][j] — the cell states c_t are stored
 * too, so clskd_lstm_bwd (c_ready = 1) skips its serial cell-state scan. */
int clskd_lstm_recurrent_pre(float* gx, int64_t gx_ws, int64_t gx_seq, int64_t gx_t,
                             const float* whh, int32_t nws, int32_t nseq, int32_t T, int32_t H,
                             float* out, int64_t o_ws, int64_t o_seq, int64_t o_t, float* cbuf,
                             void* stream);

/* One recurrence step with carried state (streaming inference, config C5): per (ws, seq),
 * gates = gx + W_hh h; c = f c + i g; h = o tanh(c) — h, c updated in place (strides s_ws,
 * s_seq), h also written to out.  Same gate functions as clskd_lstm_recurrent. */
int clskd_lstm_cell(const float* gx, int64_t gx_ws, int64_t gx_seq, const float* whh, int32_t nws,
                    int32_t nseq, int32_t H, float* h, float* c, int64_t s_ws, int64_t s_seq,
                    float* out, int64_t o_ws, int64_t o_seq, void* stream);

/* real = a - b, imag = c + d  (tools_for_model.py:168-169); all [n] contiguous */
int clskd_complex_combine(const float* rr, const float* ii, const float* ir, const float* ri,
                          float* real_out, float* imag_out, int64_t n, void* stream);
/* The same with real_out / imag_out stored as out_dtype (CLSKD_F32 | CLSKD_BF16 | CLSKD_F16,
 * round-to-nearest-even): the frozen teacher's LSTM outputs as the 16-bit operands of its next
 * GEMMs (precision 'mixed' / 'fp16'). */
int clskd_complex_combine_dt(const float* rr, const float* ii, const float* ir, const float* ri,
                             void* real_out, void* imag_out, int64_t n, int32_t out_dtype, void* stream);

/* ------------------------------------------------------------------------------------------
 * STFT helpers.
 * clskd_frame_pad: xp[b][j] = x[b][j - pad] with zero (mode 0) or reflect (mode 1) padding,
 *                  j in [0, Lp); x is [B][L] with row stride ldx.
 * clskd_spec_bftc: encoder input of DCCRN.py:165-170 (real = spec[:, 1:257], imag =
 *                  spec[:, 258:514] stacked as channels) in BFTC: out[b][f][t][0] =
 *                  spec[b][t][re0+f], out[b][f][t][1] = spec[b][t][im0+f], f < F.
 * clskd_mask_e:    DCCRN masking_mode 'E' (DCCRN.py:207-226) from spec [B][T][ldspec] (real
 *                  bins 0..256 at 0.., imag at 257..) and the last decoder output
 *                  mask[B][256][Tm][2] read at time t+1; writes est [B][T][ldest] (real at 0..,
 *                  imag at 257.., zero tail) and optionally mask_r/mask_i [B][T][257].
 *                  1 <= B <= 65535, T >= 1 (a block per utterance and 16 frames); the same
 *                  bounds hold for clskd_mask_e_bwd.
 * clskd_ola:       ConviSTFT overlap-add (tools_for_model.py:95-107): frames [B][T][400] ->
 *                  wav[b][n] = (sum frames) / (sum window^2 + 1e-8), trimmed, clamp(-1,1)
 *                  (DCCRN.py:235-237) when clamp != 0.  window == NULL: the plain sum
 *                  (asteroid's STFT Decoder, conv_transpose1d with the synthesis filters).
 * clskd_mask_bdt:  asteroid DCCRNet mask (complex_nn.BoundComplexMask('tanh') then
 *                  DCCRNet.apply_masks): est = tanh(|M|) e^{i angle M} * X on bins 0..255 of
 *                  spec rows [B][T][ldspec] (re 0.., im 257..), bin 256 = 0; mask BFTC
 *                  [B][256][Tm][2]; est rows [B][T][ldest] (zero tail columns 514..).
 * -------------------------------------------------------------------------------------- */
int clskd_frame_pad(const float* x, int64_t ldx, int32_t B, int32_t L, int32_t pad, int32_t Lp,
                    int32_t mode, float* xp, void* stream);
int clskd_spec_bftc(const float* spec, int32_t B, int32_t T, int32_t ld, int32_t re0, int32_t im0,
                    int32_t F, float* out, void* stream);
int clskd_mask_e(const float* spec, int32_t ldspec, const float* mask, int32_t Tm, int32_t B,
                 int32_t T, float* est, int32_t ldest, float* mask_r, float* mask_i,
                 void* stream);
int clskd_mask_bdt(const float* spec, int32_t ldspec, const float* mask, int32_t Tm, int32_t B,
                   int32_t T, float* est, int32_t ldest, void* stream);
int clskd_ola(const float* frames, const float* window, int32_t B, int32_t T, int32_t win,
              int32_t hop, int32_t out_len, int32_t trim, int32_t clamp, float* wav,
              void* stream);

/* ------------------------------------------------------------------------------------------
 * ReviewKD ABF attention fusion (framework.py:209-217), mid = 64 channels:
 *   y_up = nearest-interpolate(res [B][Fr][Tr][64] -> (F, T))
 *   z = sigmoid(W[2][128] . [x; y_up] + b);  out = x*z0 + y_up*z1
 * x_scale/x_shift (optional, 64 fp32 each, both or neither): x := x*x_scale + x_shift on load
 *   — the ABF's conv1 BatchNorm (framework.py:181) folded into the fuse, x = raw conv1 output.
 * -------------------------------------------------------------------------------------- */
int clskd_abf_fuse(const void* x, const void* res, int32_t B, int32_t F, int32_t T,
                   int32_t Fr, int32_t Tr, const float* w, const float* b,
                   const float* x_scale, const float* x_shift, void* out, int32_t dtype,
                   void* stream);

/* ------------------------------------------------------------------------------------------
 * ABF level with conv1 folded (framework.py:179-222, replaces ABF.conv1's nn.Conv2d(1x1) +
 * nn.BatchNorm2d and the fuse above): conv1's 64-channel output never reaches HBM.
 *   s:  student tap, fp32 BFTC rows [B][F][T][cin] at element strides (sB, sF, sT), channels
 *       contiguous, 16-B aligned rows; cin in {8, 16, 32, 64}; w1: conv1 weight [64][cin] fp32.
 * clskd_abf_bn1_partials: partial[nblk][64][2] (fp64) = {sum, sumsq} of x1 = W1 s over block
 *   `blk`'s rows, from that block's moments S1 = sum s, S2 = sum s s^T (sum_n = w_n.S1,
 *   sumsq_n = w_n^T S2 w_n): the fused-statistics contract of the conv engines, finalised by
 *   clskd_bn_compact / clskd_bn_finalize.  nblk = clskd_abf_moment_blocks(B*F*T, cin).
 * clskd_abf_conv1_fuse: out[r] = x(r) := (W1 s[r])*scale + shift, or with a residual
 *   res [B][Fr][Tr][64] the attention fusion of clskd_abf_fuse applied to x(r); x1_raw
 *   (optional) receives W1 s[r] (the training tape).  out / x1_raw / res storage: `dtype`.
 * -------------------------------------------------------------------------------------- */
int32_t clskd_abf_moment_blocks(int64_t rows, int32_t cin);
int clskd_abf_bn1_partials(const float* s, int32_t B, int32_t F, int32_t T, int64_t sB,
                           int64_t sF, int64_t sT, int32_t cin, const float* w1, double* partial,
                           int32_t nblk, void* stream);
int clskd_abf_conv1_fuse(const float* s, int32_t B, int32_t F, int32_t T, int64_t sB, int64_t sF,
                         int64_t sT, int32_t cin, const float* w1, const float* scale,
                         const float* shift, const void* res, int32_t Fr, int32_t Tr,
                         const float* w, const float* b, void* out, void* x1_raw, int32_t dtype,
                         void* stream);

/* ------------------------------------------------------------------------------------------
 * Validation metrics of KnowledgeDistillation.validation_step (distill.py:149-199,
 * COMPUTE_METRICS = ["si_sdr", "stoi"], distill.py:35), per utterance, float64 results.
 * clskd_sisdr_f64: asteroid get_metrics' si_sdr = pb_bss_eval.evaluation.si_sdr(ref, est)
 *   (the formula of tools_for_loss.py:50-92 without eps; no mean removal):
 *   out[r] = 10 log10(|a ref|^2 / |est - a ref|^2), a = <ref, est> / <ref, ref>.
 * clskd_stoi: pystoi.stoi(clean, est, fs, extended=False) (tools_for_model.py:595-600):
 *   resampling to 10 kHz (Octave resample filter, scipy resample_poly alignment), silent-frame
 *   removal (40 dB below the loudest clean frame), 512-point STFT of 256-sample Hanning frames,
 *   15 one-third-octave bands, 30-frame segments with -15 dB clipping, mean correlation.
 *   Rows of `clean` / `est` at strides ld_clean / ld_est (fp32); workspace: device memory of
 *   clskd_stoi_workspace(B, L, fs) bytes; at most 6144 energy frames (78 s) per utterance.
 * -------------------------------------------------------------------------------------- */
int clskd_sisdr_f64(const float* ref, const float* est, int32_t rows, int32_t L, int64_t ld_ref,
                    int64_t ld_est, double* out, void* stream);
int64_t clskd_stoi_workspace(int32_t B, int32_t L, int32_t fs);
int clskd_stoi(const float* clean, const float* est, int32_t B, int32_t L, int64_t ld_clean,
               int64_t ld_est, int32_t fs, void* workspace, int64_t ws_bytes, double* out,
               void* stream);

/* ------------------------------------------------------------------------------------------
 * Uniform weight re-draw (replaces the per-step ABF rebuild of framework.py:194-195 —
 * nn.init.kaiming_uniform_(w, a=1) on conv1/conv2 and Conv2d.reset_parameters on att_conv —
 * and the repacking of the drawn weights).  Job k draws numel values U(-bound, bound) into
 * param (contiguous fp32, layout [N][Cin][ntap]) and, when packed != NULL, the same values into
 * the packed conv operand packed[n][tap*Cin + c] (row pitch Kp, storage packed_dtype; padding
 * columns untouched).  Philox4x32-10 keyed by `seed`; the draw counter state[0] (device
 * uint64[2] = {counter, ticket}, zeroed once by the caller; one state per concurrently running
 * stream) is read by the kernel and advanced by its last workgroup, so graph replays re-draw.
 * Job arrays are host memory passed as kernel arguments.  Distribution matches the reference;
 * the random stream is this library's own (the reference draws from torch's generator).
 * -------------------------------------------------------------------------------------- */
#define CLSKD_DRAW_MAX_JOBS 32

typedef struct {
  float* param;
  void* packed;
  int64_t numel;
  int32_t Cin, ntap, Kp;
  int32_t packed_dtype;
  float bound;
  int32_t stream_id; /* distinct per job within a launch (decorrelates the Philox counters) */
} clskd_draw_job;

int clskd_uniform_redraw(const clskd_draw_job* jobs, int32_t njobs, uint64_t seed,
                         uint64_t* state, void* stream);

/* ------------------------------------------------------------------------------------------
 * SPKD / Gram (framework.py:150-172; replaces SPKDLoss.forward / get_similarity_matrix, the
 * per-tap torch.mm(z, z.t()) of framework.py:156-160, for every tap of a step at once).
 * A gram job views a tap as z_b = x[b][p][c0 .. c0+Cs) for p < P positions with position
 * stride Ctot and batch stride sB (elements).  Job arrays are HOST memory: the library passes
 * them to the kernels as kernel arguments (no device upload; launches are graph-capturable).
 * clskd_gram_partial: job k covers slabs [first_slab, first_slab + nslab), nslab = ceil(P/chunk),
 *                     jobs contiguous from slab 0; one 32x32 fp32 partial Gram per slab into
 *                     slabs[slab][32][32] (device, caller-owned).
 * clskd_spkd_finalize: per pair (student job pairs[2i], teacher job pairs[2i+1], host array):
 *                     sum the slabs in order (fp64), L1-normalise rows (normalize(G, p=1) — the
 *                     reference passes 1 as p), loss = ||Gt-Gs||_F^2 (/B^2 if batchmean);
 *                     writes losses[i] and, if non-null, grams_s/grams_t[i][B][B].
 * clskd_spkd_finalize_ranges: the same finalize over slab ranges given directly (pair i: the
 *                     s_nslab[i] slabs at s_slabs[i], device pointers into any slab buffers),
 *                     so a step can run its Gram launches on several streams — each as soon
 *                     as its features exist — and finalize once after joining them.
 * -------------------------------------------------------------------------------------- */
#define CLSKD_GRAM_MAX_JOBS 32   /* jobs per kernel launch (the library splits larger lists) */
#define CLSKD_SPKD_MAX_PAIRS 64  /* pairs per finalize launch (likewise) */

typedef struct {
  const void* ptr;
  int64_t sB;
  int64_t P;
  int32_t Ctot, c0, Cs;
  int32_t chunk;      /* positions per slab */
  int32_t first_slab; /* index of this job's first slab */
  int32_t nslab;
  int32_t dtype;      /* CLSKD_F32 (Cs % 4 == 0) or CLSKD_BF16 (Cs % 8 == 0) storage */
  int32_t reserved;
  /* optional per-channel affine applied to every loaded element before the product (NULL =
   * none): z = x*scale[ch] + shift[ch], ch in [0, Ctot), rounded to the storage type — a
   * BatchNorm whose apply pass is folded into the Gram (bitwise the same as clskd_bn_apply
   * followed by a plain gram).  Ctot <= 1024 when given. */
  const float* scale;
  const float* shift;
  /* optional, with scale/shift: PReLU slope alpha[0] applied after the affine (NULL = none) —
   * z = t >= 0 ? t : alpha[0]*t, t = x*scale + shift, then the storage rounding, exactly as
   * clskd_bn_apply computes it */
  const float* alpha;
  /* optional output (NULL = none): every element the job loads is ALSO written, transformed, to
   * out at the same element offset (out may equal ptr: an in-place BatchNorm+PReLU apply fused
   * with the tap's SPKD Gram partials — the tap is read once instead of twice).  The job must
   * then cover the channels it writes; 16-byte aligned, the job's storage type. */
  void* out;
} clskd_gram_job;

int clskd_gram_partial(const clskd_gram_job* jobs, int32_t njobs, int32_t B, float* slabs,
                       void* stream);
int clskd_spkd_finalize(const clskd_gram_job* jobs, int32_t njobs, const int32_t* pairs,
                        int32_t npairs, int32_t B, int32_t batchmean, const float* slabs,
                        float* grams_s, float* grams_t, float* losses, void* stream);
int clskd_spkd_finalize_ranges(const float* const* s_slabs, const int32_t* s_nslab,
                               const float* const* t_slabs, const int32_t* t_nslab,
                               int32_t npairs, int32_t B, int32_t batchmean, float* grams_s,
                               float* grams_t, float* losses, void* stream);

/* ------------------------------------------------------------------------------------------
 * Losses.
 * clskd_stft_mag_loss: one STFTLoss resolution (framework.py:16-101) from raw spectra
 *   X, Y [rows][ld] (real part of bin f at f, imaginary at nbins+f); magnitudes
 *   sqrt(max(re^2+im^2, 1e-7)).  Writes 256 per-block partials acc[256][3] (fp64) =
 *   {sum (Y-X)^2, sum Y^2, sum |log Y - log X|}.
 * clskd_stft_loss_finalize: out2[0] = factor_sc*||Y-X||_F/||Y||_F (SpectralConvergenge),
 *   out2[1] = factor_mag*mean|log Y - log X| (LogSTFTMagnitude) over `count` elements.
 * clskd_sisnr_rows: tools_for_loss.py:37-47 per row -> out[rows] (dB); two passes, fp64 sums.
 * clskd_sum_f32: out[0] = scale * sum of a[0..n) (fixed order, fp64).
 * clskd_stft_loss_finalize with accumulate != 0 adds into out2 (multi-resolution sum).
 * -------------------------------------------------------------------------------------- */
int clskd_stft_mag_loss(const float* X, const float* Y, int64_t rows, int32_t ld,
                        int32_t nbins, double* acc, void* stream);
int clskd_stft_loss_finalize(const double* acc, int64_t count, float factor_sc,
                             float factor_mag, int32_t accumulate, float* out2, void* stream);
int clskd_sisnr_rows(const float* s1, const float* s2, int32_t rows, int32_t L, int64_t ld1,
                     int64_t ld2, float eps, float* out, void* stream);
int clskd_sum_f32(const float* a, int32_t n, float scale, float* out, void* stream);

/* small utilities */
int clskd_zero_f64(double* p, int64_t n, void* stream);

/* ==========================================================================================
 * Backward pass of the CLSKD training step (config C3; SURVEY.md §8 f rank 1 — the student's
 * gradients for distill.py's automatic optimisation: loss.backward() + Adam, distill.py:202-204).
 * Gradients are fp32.  Every reduction has a fixed order (no float atomics): bitwise repeatable.
 * ======================================================================================== */

/* Weight gradient of a clskd_conv2d_fwd launch, through the SAME descriptor (segments = the
 * forward's inputs, fp32 storage): dw[n][k] (+)= sum_rows dY(row, n) * A(row, k) over the
 * padded K of the packed weight, dbias[n] (+)= sum_rows dY(row, n) (dbias may be NULL).  dY is
 * read through the descriptor's output map (d->out is ignored; dy replaces it).  Replaces the
 * autograd weight gradients of ComplexConv2d / ComplexConvTranspose2d (tools_for_model.py:
 * 236-330), nn.LSTM W_ih / W_hh (with a time-shifted segment over the hidden history) and the
 * NavieComplexLSTM Linear projections (tools_for_model.py:164-173).
 * accumulate: bit 0 -> dw (+)=, bit 1 -> dbias (+)= (e.g. polyphase halves sharing one bias).
 * `work` holds clskd_conv2d_wgrad_workspace(d) floats (split-M partials). */
int64_t clskd_conv2d_wgrad_workspace(const clskd_conv_desc* d);
int clskd_conv2d_wgrad(const clskd_conv_desc* d, const float* dy, float* dw, float* dbias,
                       float* work, int64_t work_elems, int32_t accumulate, void* stream);

/* out[i] (+)= sum_{j<J} sgn[i*J+j] * src[idx[i*J+j]] (idx < 0 skipped): maps packed-operand
 * gradients back onto module parameters (complex [[Wr,-Wi],[Wi,Wr]] blocks, polyphase taps). */
int clskd_index_gather(const float* src, const int32_t* idx, const float* sgn, int32_t J,
                       int64_t n, float* out, int32_t accumulate, void* stream);
/* Several index gathers in one launch: job i computes out_i[e] (+)= sum_j sgn_i[e*J+j] *
 * src_i[idx_i[e*J+j]] exactly as clskd_index_gather.  `jobs` is HOST memory (read at enqueue,
 * n_jobs <= CLSKD_GATHER_JOBS_MAX); jobs must write disjoint outputs.  Used to apply a backward
 * pass's packed-gradient -> parameter maps in one launch (clskd.backward). */
#define CLSKD_GATHER_JOBS_MAX 48
typedef struct {
  const float* src;
  const int32_t* idx;
  const float* sgn;
  float* out;
  int64_t n;
  int32_t J;
  int32_t accumulate;
} clskd_gather_job;
int clskd_index_gather_jobs(const clskd_gather_job* jobs, int32_t n_jobs, void* stream);

/* torch.optim.Adam step (distill.py:202-204) over a flat parameter buffer: g *= grad_scale
 * (e.g. 1/world for a summed all-reduce), L2 weight decay, bias corrections for `step` (1-based). */
int clskd_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                    float beta1, float beta2, float eps, float weight_decay, int32_t step,
                    float grad_scale, void* stream);
/* The same step with the step count in device memory (for a captured, replayed training step):
 * applies step *step + 1, then stores *step + 1 (stream-ordered, two launches). */
int clskd_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                        float beta1, float beta2, float eps, float weight_decay, int32_t* step,
                        float grad_scale, void* stream);
int clskd_fill_f32(float* p, int64_t n, float value, void* stream);
int clskd_axpy_f32(const float* x, float* y, int64_t n, float alpha, int32_t accumulate,
                   void* stream);

/* BatchNorm2d(train) + optional PReLU backward over a BFTC tensor x[rows][C] (the RAW conv
 * output, storage `dtype`), given dy = dL/d(output).  scale/shift: the forward's coefficients
 * (y_bn = x*scale + shift), mean/var: its batch statistics (biased var), gamma: BN weight.
 * Writes dgamma/dbeta/dalpha (accumulate_params) and dx (accumulate_dx), fp32.
 * `work`: clskd_bn_bwd_workspace(nblk, C) doubles, nblk = clskd_bn_bwd_blocks(rows, C). */
int32_t clskd_bn_bwd_blocks(int64_t rows, int32_t C);
int64_t clskd_bn_bwd_workspace(int32_t nblk, int32_t C);
int clskd_bn_bwd(const void* x, const float* dy, int64_t rows, int32_t C, const float* scale,
                 const float* shift, const float* mean, const float* var, float eps,
                 const float* gamma, const float* alpha, double* work, int32_t nblk,
                 float* dgamma, float* dbeta, float* dalpha, float* dx, int32_t accumulate_dx,
                 int32_t accumulate_params, int32_t dtype, void* stream);

/* ABF fusion backward (framework.py:209-219): from dout = dL/d(fused x), dx = dL/d(conv1 BN
 * output) and dyup = dL/d(upsampled residual) ([B][F][T][64]); operands as clskd_abf_fuse.
 * grad_dtype (CLSKD_F32 or CLSKD_BF16) is the storage type of all four gradient maps (dout,
 * dnext, dx, dyup); arithmetic is fp32 either way.  With bf16 storage the bn_partial sums are
 * taken over the stored (rounded) dx, so clskd_bn_bwd_from_partials reading that dx back
 * (dy_dtype CLSKD_BF16) applies statistics consistent with its input.
 * clskd_nearest_down_sum folds a gradient of a nearest upsampling (F.interpolate 'nearest',
 * framework.py:213-222) back onto the source grid: out[b][fr][tr][c] (+)= sum of g over the
 * destination pixels whose nearest source is (fr, tr).
 * Fusions in clskd_abf_fuse_bwd: dnext (optional, fp32 [B][F2][T2][64]) = the NEXT ReviewKD
 * level's dyup, folded onto this level's grid and added to dout on load (the residual path of
 * framework.py:213-215 without a separate down-sum pass); bn_partial (optional, fp64
 * [clskd_abf_fuse_bwd_blocks(B,F,T)][64][3]) receives the conv1-BatchNorm backward statistics of
 * dx (mean1/var1: that BN's batch statistics) for clskd_bn_bwd_from_partials.  dyup may be NULL
 * (the first level has no residual input). */
int32_t clskd_abf_fuse_bwd_blocks(int32_t B, int32_t F, int32_t T);
int clskd_abf_fuse_bwd(const void* x1, const void* res, int32_t B, int32_t F, int32_t T,
                       int32_t Fr, int32_t Tr, const float* w, const float* b,
                       const float* x_scale, const float* x_shift, const void* dout, void* dx,
                       void* dyup, const void* dnext, int32_t F2, int32_t T2,
                       const float* mean1, const float* var1, float eps, double* bn_partial,
                       int32_t dtype, int32_t grad_dtype, void* stream);
/* BatchNorm backward whose statistics partials [nblk][C][3] were produced by a fused producer
 * (clskd_abf_fuse_bwd): finalize + apply of clskd_bn_bwd (no PReLU).  kbuf: 3*C floats. */
int clskd_bn_bwd_from_partials(const void* x, const void* dy, int64_t rows, int32_t C,
                               const float* scale, const float* shift, const float* mean,
                               const float* var, float eps, const float* gamma,
                               double* partial, int32_t nblk, float* kbuf, float* dgamma,
                               float* dbeta, float* dx, int32_t accumulate_dx, int32_t dtype,
                               int32_t dy_dtype, void* stream);
/* dx == NULL (clskd_bn_bwd_from_partials, clskd_bn_bwd): coefficients only — kbuf (resp. the
 * floats at work + nblk*C*3 doubles) receives k [3][C] with d = k0*dy + k1*x + k2, for a consumer
 * that applies them itself (clskd_bn_bwd_conv1x1). */
/* BatchNorm-backward apply fused with a 1x1 conv's data gradient (the ReviewKD ABF conv1,
 * framework.py:179-182, no bias): per row, d[c] = k0[c]*dy[c] + k1[c]*x[c] + k2[c] (C = 64), then
 * out[row][n] (+)= sum_c w[c][n] d[c] (ascending c, fp32), N in {8, 16, 32, 64}.  x: the BN input
 * (dtype), dy: the BN output gradient (dy_dtype), both [rows][64] contiguous; w [64][N] fp32
 * (conv1's weight [64][N][1][1]); out [rows][N] fp32; x, dy, k, out 16-byte aligned. */
int clskd_bn_bwd_conv1x1(const void* x, int32_t dtype, const void* dy, int32_t dy_dtype,
                         int64_t rows, int32_t C, const float* k, const float* w, int32_t N,
                         float* out, int32_t accumulate, void* stream);
/* Split-product data gradients on the bf16 engines (round 6): clskd_split_planes writes an fp32
 * map [rows][C] as bf16 planes [rows][2C] (hi = bf16(x) in channels [0, C), lo = bf16(x - hi) in
 * [C, 2C)); clskd_pack_split3 turns a packed fp32 weight [N][ntaps*C] (K order tap, channel) into
 * the bf16 weight [N][Kp] (Kp = ntaps*3C padded to 64) of the two-segment K table (tap, [planes
 * 2C | planes' hi C], channel): per tap [W_hi | W_hi | W_lo], so one bf16 implicit GEMM sums
 * hi*W_hi + lo*W_hi + hi*W_lo — the CLSKD_F32X3 split product as three K segments. */
int clskd_split_planes(const float* src, int64_t rows, int32_t C, void* dst, void* stream);
int clskd_pack_split3(const float* w, int32_t N, int32_t ldw, int32_t ntaps, int32_t C, int32_t Kp,
                      void* out, void* stream);
/* g_dtype: storage type of g (CLSKD_F32 or CLSKD_BF16); out is fp32. */
int clskd_nearest_down_sum(const void* g, int32_t B, int32_t F, int32_t T, int32_t Fr,
                           int32_t Tr, int32_t C, float* out, int32_t accumulate, int32_t g_dtype,
                           void* stream);

/* Masking mode 'E' backward (DCCRN.py:207-226): d est [B][T][ldest] -> d mask [B][256][Tm][2]
 * (time 0 of the decoder output gets zero).  ConviSTFT OLA + clamp backward (tools_for_model.py:
 * 95-107, DCCRN.py:237): dwav -> dframes [B][T][win] (pre-clamp samples recomputed from frames).
 * Framing pad backward (zero / reflect, as clskd_frame_pad): dxp [B][Lp] -> dx [B][L] (row ldx).
 * STFT log-magnitude L1 backward (framework.py:58-68): dX = d(scale * sum|log|Y| - log|X||)/dX
 * for raw spectra X, Y [rows][ld] (re at f, im at nbins+f), written with row pitch ldd (columns
 * >= 2*nbins zero: a pitch padded to a multiple of 4 keeps the framing dgrad's gather vec4).
 * Complex-LSTM combine backward (tools_for_model.py:168-169): dh[2][2B][n] from dreal/dimag. */
int clskd_mask_e_bwd(const float* spec, int32_t ldspec, const float* mask, int32_t Tm, int32_t B,
                     int32_t T, const float* dest, int32_t ldest, float* dmask, void* stream);
int clskd_ola_bwd(const float* frames, const float* window, const float* dwav, int32_t B,
                  int32_t T, int32_t win, int32_t hop, int32_t out_len, int32_t trim,
                  int32_t clamp, float* dframes, void* stream);
int clskd_frame_pad_bwd(const float* dxp, int32_t B, int32_t L, int32_t pad, int32_t Lp,
                        int32_t mode, float* dx, int64_t ldx, int32_t accumulate, void* stream);
int clskd_stft_mag_loss_bwd(const float* X, const float* Y, int64_t rows, int32_t ld,
                            int32_t nbins, float scale, float* dX, int32_t ldd, void* stream);
int clskd_complex_combine_bwd(const float* dreal, const float* dimag, int32_t B, int64_t n,
                              float* dh, void* stream);

/* LSTM backward through time (nn.LSTM, tools_for_model.py:159-174).  pre: the forward's gate
 * pre-activations [nws][nseq][T][4H] (strided like gx; rebuild them as gx + h_{t-1} W_hh^T with
 * one accumulate conv over the saved h history), dh: dL/dh_t, whh [nws][4H][H].  Writes the
 * gate pre-activation gradients dgates (strided like gx) — whose conv-engine wgrad / dgrad give
 * dW_ih, db, dx and (over the shifted h history) dW_hh.  cbuf: nws*nseq*T*H floats (cell states):
 * c_ready = 1 when clskd_lstm_recurrent_pre stored them there (the single-wave H = 16 / 32 kernel
 * then skips its cell-state scan), 0: scratch the kernel fills itself. */
int clskd_lstm_bwd(const float* pre, int64_t p_ws, int64_t p_seq, int64_t p_t, const float* dh,
                   int64_t d_ws, int64_t d_seq, int64_t d_t, const float* whh, int32_t nws,
                   int32_t nseq, int32_t T, int32_t H, float* cbuf, int32_t c_ready, float* dgates,
                   int64_t g_ws, int64_t g_seq, int64_t g_t, void* stream);

/* SPKD backward (framework.py:150-172).  clskd_spkd_grad_ranges: per pair (slab ranges as in
 * clskd_spkd_finalize_ranges) M = dG + dG^T [pair][B][B] where dG = d(scale * loss)/d(z z^T)
 * through the row L1 normalisation.  clskd_gram_bwd: dz = M z for every job (student taps;
 * optional folded BatchNorm affine as in the Gram), written fp32 with its own strides. */
typedef struct {
  const void* ptr;    /* z: as clskd_gram_job (element (b, p, c) at b*sB + p*Ctot + c0 + c) */
  int64_t sB;
  int64_t P;
  int32_t Ctot, c0, Cs;
  int32_t dtype;
  const float* scale; /* optional affine on load (NULL = none), indexed by channel < Ctot */
  const float* shift;
  const float* coef;  /* device M [B][B] of this job's pair */
  float* out;         /* dz (b, p, c) at out + b*o_sB + p*o_Ctot + o_c0 + c */
  int64_t o_sB;
  int32_t o_Ctot, o_c0;
  int32_t accumulate;
  int32_t reserved;
} clskd_gram_bwd_job;

int clskd_spkd_grad_ranges(const float* const* s_slabs, const int32_t* s_nslab,
                           const float* const* t_slabs, const int32_t* t_nslab, int32_t npairs,
                           int32_t B, int32_t batchmean, float scale, float* coef, void* stream);
int clskd_gram_bwd(const clskd_gram_bwd_job* jobs, int32_t njobs, int32_t B, void* stream);

/* SPKD gradient fused into the train-mode BatchNorm backward of a Gram'd map whose BN apply was
 * folded into the Gram (ReviewKD outputs, framework.py:183-186 + 150-172): for raw[b][p][c]
 * (batch stride sB elements, P positions x C channels, storage dtype), z = round(raw*scale +
 * shift), dz = M z (coef = M [B][B] of clskd_spkd_grad_ranges); writes d raw (storage
 * draw_dtype) and dgamma / dbeta without materialising dz.  work: clskd_bn_bwd_workspace(nblk,
 * C) doubles, nblk = clskd_bn_bwd_blocks(B*P, C). */
int clskd_spkd_bn_bwd(const void* raw, int32_t dtype, int64_t sB, int64_t P, int32_t C, int32_t B,
                      const float* scale, const float* shift, const float* coef, const float* mean,
                      const float* var, float eps, const float* gamma, double* work, int32_t nblk,
                      float* dgamma, float* dbeta, void* draw, int32_t draw_dtype, void* stream);

/* ------------------------------------------------------------------------------------------
 * Step executor.
 * Replaces: the host side of KnowledgeDistillation.training_step (distill.py:72-148) — the
 * ~400 per-step launches a Python host issues one by one.  Takes a hipGraph captured from one
 * step (stream capture of the library's own calls, e.g. torch.cuda.CUDAGraph(keep_graph=True)
 * + raw_cuda_graph()) and replays its kernel / memset / memcpy nodes with their captured
 * arguments on `nstreams` HIP streams along the graph's dependency edges (one event record /
 * wait per cross-stream edge not already implied; resolved once here).  Unlike hipGraphLaunch
 * the independent branches run concurrently.  Stream 0 is the launch stream: the others fork
 * from it and join back into it, so a launch is stream-ordered like any other call.
 * side_streams (nstreams - 1 hipStream_t, or NULL: the executor creates its own): streams the
 * caller already uses, so the replay keeps the eager path's hardware-queue mapping (a process has
 * few hardware queues; streams created later can share one with a busy stream).  The graph is
 * BORROWED: the caller keeps it (its nodes hold the kernels' arguments) and the memory its
 * nodes address alive while the executor exists.
 * info[0..7] = nodes, kernel nodes, memset nodes, memcpy nodes, empty nodes, cross-stream
 * waits, event records, program length; info[8..8+nstreams) = nodes per stream (n >= 8). */
typedef struct clskd_exec clskd_exec;
int clskd_exec_create(void* hip_graph, int32_t nstreams, void* const* side_streams,
                      int32_t use_tags, clskd_exec** out);
/* Capture-time stream tags: during the capture, after each library call the host calls
 * clskd_exec_tag(stream, index) with the stream the call was issued on; the node(s) that call
 * added are placed on stream `index` by a later clskd_exec_create(..., use_tags = 1), so the
 * replay keeps the host's own chains.  clskd_exec_tag_reset clears the tags. */
int clskd_exec_tag(void* stream, int32_t tag);
void clskd_exec_tag_reset(void);
int clskd_exec_launch(clskd_exec* ex, void* stream);
/* clskd_exec_launch with the side streams in ahead_mask (bit s = stream s >= 1) not waiting for
 * the fork on `stream`: each waits for ahead_event instead (a hipEvent_t; NULL = no wait, the
 * stream's own order only).  The teacher_ahead schedule of clskd_step (distill.py step i + 1's
 * frozen-teacher chain overlapping step i's tail) for captured steps: two executors with their
 * own static buffers alternate, each one's teacher stream waiting for the end of its own
 * previous launch (clskd.graph.AheadStepExecutor). */
int clskd_exec_launch_ahead(clskd_exec* ex, void* stream, uint32_t ahead_mask, void* ahead_event);
int clskd_exec_info(const clskd_exec* ex, int32_t* info, int32_t n);
/* Text listing of the replay program (one op per line: index, kind, stream, slot, and for kernel
 * ops the grid size, block size and kernel name) into buf (NUL-terminated, truncated at cap);
 * returns the full length, or -1 for a null executor.  Diagnostic. */
int64_t clskd_exec_dump(const clskd_exec* ex, char* buf, int64_t cap);
void clskd_exec_destroy(clskd_exec* ex);
/* Live timing of one kernel under the executor: every launch of host function `fn` (e.g.
 * clskd_conv_last_kernel_fn() after a conv call) gets a HIP event pair around it on its stream,
 * for up to max_launches launches (fn NULL disables).  clskd_exec_profile_read (after a
 * synchronize) returns the summed event spans and the number of timed launches. */
int clskd_exec_profile(clskd_exec* ex, const void* fn, int32_t max_launches);
int clskd_exec_profile_read(clskd_exec* ex, double* total_ms, int32_t* count);
/* Per-kernel census of one replay (round 6): the captured step run once in program order on ONE
 * stream (the caller's), an event pair around every kernel node; fns[i] / ms[i] = host function
 * and duration of the i-th kernel node (cap >= the node count, exec_info slot 1; *n = the count).
 * The isolated per-kernel view of a rocprofv3 trace of a serialised step — bench.py picks the
 * dominant kernel instance over ALL kernels from it.  A real step; synchronises the stream. */
int clskd_exec_census(clskd_exec* ex, void* stream, int32_t cap, const void** fns, float* ms, int32_t* n);
/* Demangled name of a kernel host function into buf (NUL-terminated, truncated at cap); returns
 * the full length, -1 if HIP does not know the function. */
int32_t clskd_kernel_name(const void* fn, char* buf, int32_t cap);
/* Per-stream milestones (diagnostic): with marks on, every launch records a timing event before
 * the fork and at each stream's tail; clskd_exec_marks_read (after a synchronize) returns per
 * stream the mean tail time after the fork in ms over the last <= 64 launches (n >= nstreams). */
int clskd_exec_marks(clskd_exec* ex, int32_t on);
int clskd_exec_marks_read(clskd_exec* ex, float* out, int32_t n);

/* ------------------------------------------------------------------------------------------
 * Streaming hop (configuration C5): one 6.25 ms hop of the DCCRN eval forward for B streams as
 * ONE launch (one workgroup per stream).
 * Replaces: the per-hop launch sequence of the streaming driver — ConvSTFT row
 * (tools_for_model.py:53-67), encoder (DCCRN.py:171-176), complex LSTMs with carried state
 * (tools_for_model.py:159-174), decoder with its one-frame look-ahead per layer (DCCRN.py:201-206),
 * mask 'E' (DCCRN.py:207-226), ConviSTFT row + overlap-add (tools_for_model.py:90-109).
 * Weights are fp32 copies of the packed operands in k-quad layout [K/4][N][4] (element (k, n) at
 * ((k/4)*N + n)*4 + k%4, so a lane per output reads four k at once and a wavefront reads one
 * contiguous run): encoder K order (kf*2+kt, ci) with encoder 0's two input channels padded to
 * four; decoder per parity (tap, [input | skip] channels); LSTM input [K][8H] of both weight sets;
 * W_hh as [H][2*4H] (n = ws*4H + gate row); projections [H][P]; STFT [400][514]; iSTFT
 * [516][400].  BatchNorm as eval [scale | shift] + PReLU slope.
 * `state` holds per-stream rings (stride state_stride floats, zero at the start of a stream):
 * off_* are float offsets inside one stream's state (xwin 400; spectrum [7][514]; encoder output
 * i [7-i][128>>i][enc_cout[i]]; decoder input [2][D4][C6]; decoder output d [2][2*(D4<<d)][dec_co[d]];
 * h, c [2 layers][2 ws][2 halves][H]; iSTFT frames [4][400]).  Hop t consumes x_in[b][100]
 * (live = 1) or zeros (live = 0, drain) and writes wav_out[b][100]: the samples the offline
 * forward outputs 9 hops earlier (6 decoder look-ahead frames + the 300-sample centring).
 * Decoder output frames >= zero_from (>= 0) are zeros (the offline decoder's out-of-range frames). */
typedef struct {
  const float* stft_w;      /* [100][514][4] */
  const float* istft_w;     /* [129][400][4] */
  const float* window;      /* [400] */
  const float* enc_w[6];
  const float* enc_b[6];
  const float* enc_coef[6]; /* [2*Co] scale | shift */
  const float* enc_alpha[6];
  const float* lstm_w[2];   /* [K/4][8H][4] */
  const float* lstm_b[2];   /* [8H] */
  const float* lstm_whh[2]; /* [H/4][8H][4] */
  const float* proj_w[2];   /* [H/4][P][4] per half */
  const float* proj_b[2];
  const float* dec_w[6][2]; /* per parity */
  const float* dec_b[6][2];
  const float* dec_coef[6]; /* d < 5 */
  const float* dec_alpha[6];
  float* state;
  int64_t state_stride;
  const float* x_in;        /* [B][100] */
  float* wav_out;           /* [B][100] */
  int32_t B, t, live, zero_from;
  int32_t H, D4;
  int32_t enc_cin[6], enc_cout[6];
  int32_t dec_ca[6], dec_cb[6], dec_co[6];
  int32_t off_xwin, off_spec, off_enc[6], off_decin, off_dout[5], off_h, off_c, off_frames;
} clskd_stream_hop_args;
int clskd_stream_hop(const clskd_stream_hop_args* a, void* stream);
/* Diagnostic (-DCLSKD_EXPERIMENTS builds only; else an error): wall-clock (100 MHz) timestamps
 * of stream 0's hop phases from the last launch — start, STFT, encoders 0-5, LSTMs 0-1,
 * projection, decoders 0-5, mask, iSTFT, end, then per encoder layer (staged, conv done) — n <= 40
 * values (after a synchronize). */
int clskd_stream_hop_marks(int64_t* out, int32_t n);
/* Diagnostic (-DCLSKD_EXPERIMENTS builds only; else an error): wall-clock (100 MHz) timeline of
 * workgroup 0 of the last halo-tiled fp32 conv launched with CLSKD_H32_DEBUG_MODE=5 — waves 0
 * and 4 (one SIMD) at [0, 64) and [64, 128): after each chunk barrier, after each chunk's MFMAs,
 * after each tile — n <= 128 values (after a synchronize). */
int clskd_h32_marks(int64_t* out, int32_t n);

#ifdef __cplusplus
}
#endif
#endif /* CLSKD_H */
