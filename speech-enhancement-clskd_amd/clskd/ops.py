"""Thin torch-facing wrappers over libclskd_hip.so.

torch is plumbing here (device memory, streams); every arithmetic op runs in a HIP kernel of
the library.  Tensors are BFTC ([batch][freq][time][channel]) unless noted.
"""
import ctypes as C
import os
import threading
from collections import OrderedDict
from dataclasses import dataclass
from functools import lru_cache

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr

BK = 16
ZERO_DF = -32768
_NO_DIRECT = os.environ.get("CLSKD_NO_DIRECT", "") == "1"  # host switch: MFMA engines only
# A/B switch (measurement only): CLSKD_BN_FOLD=0 keeps every BatchNorm on fused partials + one
# clskd_bn_finalize launch even where the dispatched kernel could fold the finalize
_BN_FOLD = os.environ.get("CLSKD_BN_FOLD", "1") == "1"


def lib():
    return _lib.load()


class KernelTimer:
    """Live per-launch timing of the conv engine with HIP events on the launching stream.
    Enabled by bench.py over its timed region; records (kernel variant, flops, start, end)."""
    active = False
    records = []
    only = None  # optional kernel-instance name: time just that kernel's launches
    fns = {}  # kernel-instance name -> host function (clskd_exec_profile key)
    nbytes = {}  # kernel-instance name -> [launches, summed compulsory bytes]
    # non-conv kernels (round 6): canonical instance name -> [launches, summed algorithmic bytes,
    # summed algorithmic FLOPs], noted by their wrappers while the timer is on (census step)
    work = {}

    @classmethod
    def note_work(cls, name, nbytes, flops=0.0):
        if cls.active and not torch.cuda.is_current_stream_capturing():
            w = cls.work.setdefault(name, [0, 0.0, 0.0])
            w[0] += 1
            w[1] += float(nbytes)
            w[2] += float(flops)

    @classmethod
    def start(cls, only=None):
        cls.active, cls.records, cls.only = True, [], only

    @classmethod
    def wants(cls, name):
        return cls.only is None or name == cls.only

    @classmethod
    def per_launch(cls):
        """Per-launch records (name, (M, N, K, in_dtype), us, TFLOP/s) — call after a sync."""
        return [(n, shp, e0.elapsed_time(e1) * 1e3, fl / (e0.elapsed_time(e1) * 1e-3) / 1e12)
                for n, fl, e0, e1, shp in cls.records]

    @classmethod
    def stop(cls):
        cls.active = False
        torch.cuda.synchronize()
        out = {}
        for name, flops, e0, e1, _shape in cls.records:
            ms = e0.elapsed_time(e1)
            agg = out.setdefault(name, [0, 0.0, 0.0])
            agg[0] += 1
            agg[1] += ms
            agg[2] += flops
        cls.records = []
        return out  # name -> [launches, total_ms, total_flops]


# accumulating launches on the direct kernel (A/B: CLSKD_DIRECT_ACC=0 keeps them on the engines)
_DIRECT_ACC = os.environ.get("CLSKD_DIRECT_ACC", "1") != "0"


@lru_cache(maxsize=4096)
def _direct_policy(N, K):
    return bool(_lib.load(require_gpu=False).clskd_conv_direct_ok(N, K))


def direct_ok(N, K):
    """Whether an (N, K) GEMM runs on the direct-convolution kernel (the library's policy,
    clskd_conv_direct_ok; CLSKD_NO_DIRECT=1 routes everything to the MFMA engines)."""
    return not _NO_DIRECT and _direct_policy(N, K)


def direct_np(N):
    return int(_lib.load(require_gpu=False).clskd_conv_direct_np(N))


_DIRECT_W = OrderedDict()
_DIRECT_MAPS = {}


def _direct_map(N, Kp, NP, dev):
    """index_gather map of the fp32 direct layout: wd[k][n] = w[n][k] for n < N, else 0."""
    key = (N, Kp, NP, str(dev))
    m = _DIRECT_MAPS.get(key)
    if m is None:
        k = torch.arange(Kp, dtype=torch.int64).view(Kp, 1)
        n = torch.arange(NP, dtype=torch.int64).view(1, NP)
        idx = torch.where(n < N, n * Kp + k, torch.full_like(n * k, -1)).to(torch.int32)
        m = (idx.reshape(-1, 1).to(dev), torch.ones(Kp * NP, 1, dtype=torch.float32, device=dev))
        _DIRECT_MAPS[key] = m
    return m


def direct_weight(wpacked):
    """[N][Kp] packed weight -> the direct kernel's k-major layout (CLSKD_WLAYOUT_DIRECT):
    fp32 [Kp][NP]; bf16 [Kp/2][NP][2].  Cached per packed tensor (pointer + version; the cache
    holds the source alive so a pointer is never reused while its entry exists)."""
    tok = capture_token()
    key = (wpacked.data_ptr(), wpacked._version, tuple(wpacked.shape), wpacked.dtype)
    ent = _DIRECT_W.get(key)
    # an entry built inside a capture holds its values only in that graph's replays
    if ent is not None and cache_entry_usable(ent[2], tok):
        _DIRECT_W.move_to_end(key)
        capture_keep(ent, tok)
        return ent[1]
    N, Kp = wpacked.shape
    NP = direct_np(N)
    if wpacked.dtype in (torch.bfloat16, torch.float16):
        wd = wpacked.new_zeros(Kp // 2, NP, 2)
        wd[:, :N, :] = wpacked.view(N, Kp // 2, 2).permute(1, 0, 2)
    elif wpacked.is_cuda and wpacked.is_contiguous() and (
            (N, Kp, NP, str(wpacked.device)) in _DIRECT_MAPS
            or not torch.cuda.is_current_stream_capturing()):  # (the map's H2D copy: eager)
        # fp32 (re-packed every training step): one index gather instead of a fill + strided copy
        idx, sgn = _direct_map(N, Kp, NP, wpacked.device)
        wd = torch.empty(Kp, NP, dtype=torch.float32, device=wpacked.device)
        index_gather(wpacked, idx, sgn, wd)
    else:
        wd = wpacked.new_zeros(Kp, NP)
        wd[:, :N] = wpacked.t()
    # cached under graph capture too: the caller passes wd's address to a kernel and drops the
    # tensor, and a block freed inside a capture is handed to the next allocation of the same
    # capture — the BN partials of the very launch that reads these weights (a race in every
    # replay; the eager path always hit this cache).  A capture-built entry keeps its graph-pool
    # block alive; the captured repack rewrites the same values on every replay.
    _DIRECT_W[key] = ent = (wpacked, wd, tok)
    capture_keep(ent, tok)
    while len(_DIRECT_W) > 512:
        _DIRECT_W.popitem(last=False)
    return wd


_stream = _lib.stream_ptr


def _addr(struct):
    return C.addressof(struct)


# ------------------------------------------------------------------------------------------
# implicit-GEMM convolution
# ------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class SegGeom:
    """Gather geometry of one channel segment (pointer supplied at call time)."""
    C: int      # channels in this segment (contiguous, stride 1)
    sB: int
    sF: int
    sT: int
    F: int
    T: int


@dataclass
class Seg:
    tensor: torch.Tensor  # storage owner
    offset: int           # element offset of the segment's (b=0, f=0, t=0, c=0)
    geom: SegGeom


def seg_bftc(t, c0=0, C=None, t0=0, T=None):
    """Segment over a contiguous BFTC tensor t[B][F][T][Ct], channels [c0, c0+C), time from t0."""
    B, F, Tt, Ct = t.shape
    assert t.is_contiguous()
    C = Ct - c0 if C is None else C
    T = Tt - t0 if T is None else T
    return Seg(t, c0 + t0 * Ct, SegGeom(C, F * Tt * Ct, Tt * Ct, Ct, F, T))


BK_BF16 = 64


@lru_cache(maxsize=1024)
def _ktab(geoms, taps, device_index, bk=BK):
    """K table for segments `geoms` and spatial taps [(dF, dT)], K order (tap, seg, cin),
    padded to a multiple of `bk` with always-out-of-bounds entries."""
    ent, kseg = [], []
    for dF, dT in taps:
        for s, g in enumerate(geoms):
            for c in range(g.C):
                ent.append((c + dF * g.sF + dT * g.sT, dF, dT))
                kseg.append(s)
    K = len(ent)
    Kp = -(-K // bk) * bk
    for _ in range(Kp - K):
        ent.append((0, ZERO_DF, 0))
        kseg.append(0)
    arr = np.zeros(Kp, dtype=[("off", "<i4"), ("dF", "<i2"), ("dT", "<i2")])
    offs = np.array([e[0] for e in ent], np.int64)
    assert np.all(np.abs(offs) < 2 ** 31), "K-table offset overflow"
    arr["off"] = offs
    arr["dF"] = [e[1] for e in ent]
    arr["dT"] = [e[2] for e in ent]
    dev = torch.device("cuda", device_index)
    kt = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
    ks = torch.tensor(kseg, dtype=torch.uint8, device=dev)
    vec4 = all(g.C % 4 == 0 and g.sB % 4 == 0 and g.sF % 4 == 0 and g.sT % 4 == 0 for g in geoms)
    return kt, ks, K, Kp, vec4


def pack_weight(w, K, compute="fp32"):
    """w: [N, ntaps, Cin] (K order tap-major, channel-minor) -> [N, Kp] contiguous, zero pad.
    fp32: Kp multiple of 16, float32; bf16 / fp16: Kp multiple of 64, bfloat16 / float16 (RNE)."""
    N = w.shape[0]
    w = w.reshape(N, -1).float()
    assert w.shape[1] == K, (w.shape, K)
    bk = BK_BF16 if compute in ("bf16", "fp16") else BK
    Kp = -(-K // bk) * bk
    if Kp != K:
        w = torch.cat([w, w.new_zeros(N, Kp - K)], 1)
    if compute == "bf16":
        return w.to(torch.bfloat16).contiguous()
    if compute == "fp16":
        return w.to(torch.float16).contiguous()
    # always a fresh, 16-B-aligned tensor: never a view aliasing the parameter storage (which
    # may sit at any offset of a flat parameter buffer, clskd.train.FlatParams).  On the device
    # the copy is a kernel (clskd_axpy_f32, alpha 1: exact), not torch's clone: a D2D clone is a
    # memcpy node in a captured step, which the step executor cannot replay (clskd.graph)
    w = w.contiguous()
    if not w.is_cuda or w.numel() == 0:
        return w.clone(memory_format=torch.contiguous_format)
    out = torch.empty(w.shape, dtype=torch.float32, device=w.device)
    check(lib().clskd_axpy_f32(ptr(w), ptr(out), w.numel(), 1.0, 0, _stream()), "pack_weight copy")
    return out


def _dt(t):
    """clskd storage-type code of a tensor (0 = fp32, 1 = bf16, 2 = fp16)."""
    if t.dtype == torch.float32:
        return _lib.F32
    if t.dtype == torch.bfloat16:
        return _lib.BF16
    if t.dtype == torch.float16:
        return _lib.F16
    raise TypeError(f"clskd kernels take float32, bfloat16 or float16 tensors, got {t.dtype}")


def seg_addr(s):
    return s.tensor.data_ptr() + s.tensor.element_size() * s.offset


@dataclass(frozen=True)
class OutMap:
    oB: int
    oF: int
    oT: int
    oNhi: int = 0
    oNlo: int = 1
    nlo: int = 1 << 30
    of_mul: int = 1
    of_add: int = 0


def out_bftc(t, c0=0, of_mul=1, of_add=0):
    """Output map for a contiguous BFTC tensor (channels from c0)."""
    B, F, T, Ct = t.shape
    return OutMap(F * T * Ct, T * Ct, Ct, 0, 1, 1 << 30, of_mul, of_add), c0


def conv_mblocks(B, Fo, To):
    """Number of 128-row M-blocks of a conv launch (= fused-statistics partial count)."""
    return -(-(B * Fo * To) // 128)


class _ConvPlan:
    """Launch descriptor of one conv signature, built once; per call only the pointers change."""
    __slots__ = ("desc", "segs", "nseg", "direct", "name", "fn", "flops", "bytes", "shape", "nstats",
                 "osize", "fold")


_CONV_PLANS = {}


def _conv_plan(key, segs, geoms, taps, B, Fo, To, N, wpacked, bias, out, omap, stride_f, stride_t,
               stats, accumulate=False, mfma_only=False, split=False):
    in_dt = {_dt(s.tensor) for s in segs}
    assert len(in_dt) == 1, "all segments of one conv share a storage type"
    in_dt = in_dt.pop()
    bf16 = in_dt in (_lib.BF16, _lib.F16)  # 16-bit MFMA operands (bf16, or fp16 for C4)
    kt, ks, K, Kp, vec4 = _ktab(geoms, taps, out.device.index or 0, BK_BF16 if bf16 else BK)
    assert wpacked.shape == (N, Kp) and wpacked.is_contiguous(), (wpacked.shape, N, Kp)
    assert wpacked.dtype == {_lib.BF16: torch.bfloat16, _lib.F16: torch.float16}.get(
        in_dt, torch.float32), wpacked.dtype
    for s in segs:
        if seg_addr(s) % 16 != 0:
            vec4 = False
    # channel-run granule of the K table (direct-conv load width): 8 bf16 / 4 / 2 / 1 fp32
    if bf16:
        kvec = 8
    elif vec4:
        kvec = 4
    elif all(g.C % 2 == 0 and g.sB % 2 == 0 and g.sF % 2 == 0 and g.sT % 2 == 0 for g in geoms) \
            and all(seg_addr(s) % 8 == 0 for s in segs):
        kvec = 2
    else:
        kvec = 1
    if bf16 and not all(g.C % 8 == 0 and g.sB % 8 == 0 and g.sF % 8 == 0 and g.sT % 8 == 0
                        for g in geoms):
        raise RuntimeError("bf16 conv segments need channel runs of 8 and strides % 8")
    d = _lib.ConvDesc()
    d.B, d.Fo, d.To, d.N, d.K = B, Fo, To, N, Kp
    d.stride_f, d.stride_t = stride_f, stride_t
    d.nseg = len(segs)
    for i, g in enumerate(geoms):
        d.seg[i] = _lib.Seg(0, g.sB, g.sF, g.sT, g.F, g.T)
    for i in range(len(segs), _lib.MAX_SEGS):
        d.seg[i] = d.seg[0]
    d.ktab, d.kseg, d.vec4 = kt.data_ptr(), ks.data_ptr(), int(vec4)
    d.oB, d.oF, d.oT, d.oNhi, d.oNlo = omap.oB, omap.oF, omap.oT, omap.oNhi, omap.oNlo
    d.nlo = min(omap.nlo, 1 << 30)
    d.of_mul, d.of_add = omap.of_mul, omap.of_add
    # split products: fp32 layers launched inside split_products(True) (the accumulating
    # data-gradient sums of a split-product backward too)
    d.compute = _lib.F32X3 if (split and in_dt == _lib.F32) else in_dt
    d.in_dtype = in_dt
    d.out_dtype = _dt(out)
    d.kvec = kvec
    if len(taps) <= 16:  # K-table structure (tap, segment, channel) for the halo-tiled kernel
        d.ntaps = len(taps)
        d.ctot = sum(g.C for g in geoms)
        for i, g in enumerate(geoms):
            d.seg_c[i] = g.C
        for i, (dF, dT) in enumerate(taps):
            d.tap_df[i], d.tap_dt[i] = dF, dT
    # accumulate (data-gradient sums): the direct kernel takes it for fp32 outputs too
    direct = direct_ok(N, Kp) and not mfma_only and not (
        accumulate and (out.dtype != torch.float32 or in_dt != _lib.F32 or not _DIRECT_ACC))
    d.accumulate = int(bool(accumulate))
    d.wlayout = _lib.WLAYOUT_DIRECT if direct else _lib.WLAYOUT_NK
    pl = _ConvPlan()
    pl.desc, pl.nseg, pl.direct = d, len(segs), direct
    pl.segs = [d.seg[i] for i in range(_lib.MAX_SEGS)]  # views into d (patched per call)
    pl.name = None  # kernel instance the library dispatches to (read after the first launch)
    pl.fn = None  # its host function (the executor times launches by it)
    pl.flops = 2.0 * B * Fo * To * N * K
    # compulsory (algorithmic) bytes of one launch: every input element once, the weights once,
    # every output element once — the HBM roofline's traffic floor
    esz = {_lib.BF16: 2, _lib.F16: 2}.get(in_dt, 4)
    pl.bytes = float(sum(B * g.F * g.T * g.C for g in geoms) * esz + N * K * esz
                     + B * Fo * To * N * out.element_size())
    pl.shape = (B * Fo * To, N, K, {_lib.BF16: "bf16", _lib.F16: "f16"}.get(in_dt, "f32"))
    pl.nstats = conv_mblocks(B, Fo, To) * N * 2
    pl.osize = out.element_size()
    pl.fold = None  # the dispatched kernel folds a BatchNorm finalize (asked at the first launch)
    _CONV_PLANS[key] = pl
    return pl


_PROBE_FOLD = _lib.BnFold()  # zero fold record: clskd_conv_fold_capable inspects only presence

# fp32 convs launched inside split_products(True) ask for 3 x bf16 split products (CLSKD_F32X3:
# the student's layers in precision 'mixed'); a thread-local flag, so a model can switch its
# whole forward (DCCRN.run) without threading an argument through every call site
_SPLIT = threading.local()


class split_products:
    """Context manager: fp32 conv launches of this thread ask for split-product MFMA; weight
    gradients (conv_wgrad) likewise when `wgrad` (default: the same as `on`)."""

    def __init__(self, on, wgrad=None):
        self.on = bool(on)
        self.wgrad = self.on if wgrad is None else bool(wgrad)

    def __enter__(self):
        self.prev = (getattr(_SPLIT, "on", False), getattr(_SPLIT, "wgrad", False))
        _SPLIT.on, _SPLIT.wgrad = self.on, self.wgrad
        return self

    def __exit__(self, *exc):
        _SPLIT.on, _SPLIT.wgrad = self.prev
        return False


def conv_folds(segs, taps, B, Fo, To, N, wpacked, bias, out, omap, stride_f=1, stride_t=1):
    """Whether a conv(..., bn_stats=...) launch with these arguments dispatches to a kernel that
    folds the BatchNorm finalize (nothing launched).  A layer produced by several launches (the
    decoder's polyphase parities) folds only if all of them can: BnStats.partials_only()."""
    return conv(segs, taps, B, Fo, To, N, wpacked, bias, out, omap, stride_f=stride_f,
                stride_t=stride_t, bn_stats=(None, False), _query=True)


def conv(segs, taps, B, Fo, To, N, wpacked, bias, out, omap, out_offset=0, stride_f=1,
         stride_t=1, stats=None, stats_offset=0, accumulate=False, mfma_only=False, bn_stats=None,
         _query=False):
    """out[b, fo*of_mul+of_add, to, n] = bias[n] + sum_k A[(b,fo,to),k] W[n,k].
    bf16 segments run the LDS-DMA bf16-MFMA engine (weights packed bf16, K % 64); fp32 segments
    the fp32-MFMA engine (weights fp32, K % 16).  `out` may be fp32 or bf16 storage.
    The descriptor of each launch signature (geometry, taps, output map, dtypes, pointer
    alignment class) is built once (_conv_plan); a call patches only the pointers.
    accumulate=True adds into `out` (fp32 engines or the direct kernel, fp32 out; data-gradient
    sums); mfma_only skips the direct-convolution kernel.
    bn_stats=(BnStats, is_last): the launch produces (part of) a train-mode BatchNorm's batch
    statistics — folded into the launch when the dispatched kernel can (clskd_bn_fold), else as
    fused partials for BnStats.coefficients()."""
    addrs = [s.tensor.data_ptr() + s.tensor.element_size() * s.offset for s in segs]
    taps = tuple(taps)
    geoms = tuple(s.geom for s in segs)
    if bn_stats is not None and stats is not None:
        raise ValueError("conv: stats and bn_stats are exclusive")
    split = getattr(_SPLIT, "on", False)
    key = (geoms, taps, B, Fo, To, N, wpacked.shape, wpacked.dtype, omap, stride_f, stride_t,
           out.dtype, out.device.index, "bn" if bn_stats is not None else stats is None,
           bias is None,
           tuple(a % 16 for a in addrs), tuple(s.tensor.dtype for s in segs), accumulate, mfma_only,
           split)
    pl = _CONV_PLANS.get(key)
    if pl is None:
        pl = _conv_plan(key, segs, geoms, taps, B, Fo, To, N, wpacked, bias, out, omap, stride_f,
                        stride_t, stats, accumulate, mfma_only, split)
    if not wpacked.is_contiguous():
        raise RuntimeError("conv: packed weight must be contiguous")
    d = pl.desc
    sg = pl.segs
    for i, a in enumerate(addrs):
        sg[i].ptr = a
    for i in range(pl.nseg, _lib.MAX_SEGS):
        sg[i].ptr = addrs[0]
    d.weight = direct_weight(wpacked).data_ptr() if pl.direct else wpacked.data_ptr()
    d.bias = bias.data_ptr() if bias is not None else None
    d.out = out.data_ptr() + pl.osize * out_offset
    L = lib()
    fold = None
    d.bn_fold = None
    if bn_stats is not None:
        st, last = bn_stats
        if pl.fold is None or pl.fold[0] != _lib.KNOB_EPOCH:
            # which kernel the library dispatches this signature to (re-asked after a knob change)
            # — asked with a fold attached: eligibility can depend on it (epilogue scratch)
            d.bn_fold = C.addressof(_PROBE_FOLD)
            pl.fold = (_lib.KNOB_EPOCH, bool(L.clskd_conv_fold_capable(C.byref(d))) and _BN_FOLD)
            d.bn_fold = None
        if _query:
            return pl.fold[1]
        if out_offset or N != st.C:
            raise ValueError("conv: bn_stats needs the launch to produce all the BatchNorm's channels")
        if pl.fold[1] and not st.no_fold:
            fold = st.fold_struct(bool(last), 0)
            d.bn_fold = C.addressof(fold)
        else:
            stats, stats_offset = st.partials(conv_mblocks(B, Fo, To))
        st.launched(d.bn_fold is not None)
    if stats is not None:
        if stats.dtype != torch.float64 or stats.numel() < stats_offset + pl.nstats:
            raise RuntimeError("conv: fused statistics buffer must be float64 with room for "
                               "2 x N x mblocks partials")
        d.stats = stats.data_ptr() + 8 * stats_offset
    else:
        d.stats = None
    if fold is not None:
        try:
            _launch_conv(L, d, pl)
        except Exception:
            # an earlier launch of this BatchNorm may already have added into the fold state:
            # return it to zero so later steps do not inherit a dirty accumulator
            bn_stats[0].abort()
            raise
    else:
        _launch_conv(L, d, pl)
    return out


def _launch_conv(L, d, pl):
    if KernelTimer.active and not torch.cuda.is_current_stream_capturing() \
            and KernelTimer.wants(pl.name):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        check(L.clskd_conv2d_fwd(d, _stream()), "conv2d")
        e1.record()
        if pl.name is None:
            pl.name = L.clskd_conv_last_kernel().decode()
            pl.fn = L.clskd_conv_last_kernel_fn()
        KernelTimer.records.append((pl.name, pl.flops, e0, e1, pl.shape))
        KernelTimer.fns[pl.name] = pl.fn
        nb = KernelTimer.nbytes.setdefault(pl.name, [0, 0.0])
        nb[0] += 1
        nb[1] += pl.bytes
    else:
        check(L.clskd_conv2d_fwd(d, _stream()), "conv2d")
        if pl.name is None:
            pl.name = L.clskd_conv_last_kernel().decode()
            pl.fn = L.clskd_conv_last_kernel_fn()


def prepare_stream(stream):
    """Allocate the library's per-stream state (the conv_gemm8 stream-K workspace) for a torch
    stream before a graph is captured on it: captured launches then take the same path as eager
    ones (a stream without a workspace runs the data-parallel tile deal)."""
    check(lib().clskd_stream_prepare(stream.cuda_stream), "stream_prepare")
    return stream


def probe_values_are_indices(v, numel):
    """Whether the output of a packing build evaluated on (flat index + 1)-valued parameters can be
    read as a ±(index + 1) selection map of a `numel`-element source: every value an exact
    integer of magnitude <= numel (0 = no source element).  The probes (model._probe_pack_map,
    backward._tw_probe) check this before launching an index_gather built from the values."""
    if v.numel() == 0:
        return True
    if not bool(torch.isfinite(v).all()):
        return False
    a = v.abs()
    # float32 holds every integer up to 2^24 exactly: larger sources cannot be probed this way
    return numel < (1 << 24) and bool((v == v.round()).all()) and float(a.max()) <= numel


# ---- caches under graph capture ------------------------------------------------------------
# Weight-layout caches (DCCRN._packed, ABF._weights, backward._tw, direct_weight) hold device
# tensors keyed on their sources' (pointer, version).  Two hazards come with graph capture:
#  (1) an entry BUILT while a graph is being captured holds nothing until that graph replays —
#      served to an eager launch (e.g. bench.py's census step right after the capture, or any
#      eager step before the first replay) it is garbage;
#  (2) an entry a capture READS must outlive the graph, even when an eager rebuild later replaces
#      it in the cache.
# So every entry records the capture it was built in (capture_token(): None = eager), a lookup
# reuses an entry only from its own capture or from eager code, and every value a capture reads
# is appended to that capture's keep-alive list (CaptureScope.keep, owned with the graph).
_CAPTURE_TOKEN = None  # the CaptureScope being recorded on this process's capturing thread
_ANON_CAPTURE = object()  # a capture without a CaptureScope (nothing kept alive for it)


_MANGLED_TYPES = {"f": "float", "d": "double", "i": "int", "j": "unsigned", "b": "bool",
                  "l": "long", "m": "unsigned long", "DF16b": "bf16", "bf16": "bf16", "DF16_": "f16",
                  "Dh": "f16", "h": "unsigned char", "s": "short", "t": "unsigned short"}


def _demangle_simple(m):
    """'_ZN5clskd19abf_fuse_bwd_kernelIbf16EEvPKT_...' -> 'clskd::abf_fuse_bwd_kernel<bf16>':
    nested name + template arguments of the forms kernel instances use (types, L<type><n>E
    literals); anything else is returned unchanged."""
    try:
        i = 2
        if m[i] != "N":
            return m
        i += 1
        parts = []
        while m[i].isdigit():
            j = i
            while m[j].isdigit():
                j += 1
            n = int(m[i:j])
            parts.append(m[j:j + n])
            i = j + n
        args = []
        if m[i] == "I":
            i += 1
            while m[i] != "E":
                if m[i] == "L":  # literal: L <type> <value> E
                    j = m.index("E", i)
                    lit = m[i + 1:j]
                    for t in ("i", "j", "l", "m", "b"):
                        if lit.startswith(t) and (lit[1:].lstrip("n").isdigit()):
                            v = lit[1:].replace("n", "-", 1)
                            args.append(("true" if v == "1" else "false") if t == "b" else v)
                            break
                    else:
                        return m
                    i = j + 1
                    continue
                for code in sorted(_MANGLED_TYPES, key=len, reverse=True):
                    if m.startswith(code, i):
                        args.append(_MANGLED_TYPES[code])
                        i += len(code)
                        break
                else:
                    return m
        return "::".join(parts) + ("<" + ",".join(args) + ">" if args else "")
    except (IndexError, ValueError):
        return m


def canonical_kernel_name(name):
    """Kernel instance name in one canonical form, for matching demangled names
    (clskd_kernel_name), rocprofv3's kernel names and the conv engines' note_kernel names: return
    type, namespaces and the argument list dropped, 16-bit float types spelled bf16 / f16, no
    spaces ('void clskd::abf_fuse_bwd_kernel<__bf16>(__bf16 const*, ...)' ->
    'abf_fuse_bwd_kernel<bf16>')."""
    s = name.strip()
    if s.startswith("_Z"):  # a mangled name the demangler refused (HIP spells __bf16 "bf16")
        s = _demangle_simple(s)
    if s.startswith("void "):
        s = s[5:]
    s = s.replace("(anonymous namespace)::", "")
    depth, cut = 0, len(s)
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    s = s[:cut]
    depth, start = 0, 0
    for i, ch in enumerate(s):  # namespace qualifiers of the name (not inside template args)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == ":" and depth == 0 and i + 1 < len(s) and s[i + 1] == ":":
            start = i + 2
    s = s[start:]
    for a, b in (("std::bfloat16_t", "bf16"), ("__bf16", "bf16"), ("DF16b", "bf16"),
                 ("std::float16_t", "f16"), ("_Float16", "f16"), ("clskd::", ""), (" ", "")):
        s = s.replace(a, b)
    return s


def capture_token():
    """None outside graph capture; else the identity of the capture being recorded."""
    if not (torch.cuda.is_initialized() and torch.cuda.is_current_stream_capturing()):
        return None
    return _CAPTURE_TOKEN if _CAPTURE_TOKEN is not None else _ANON_CAPTURE


def cache_entry_usable(built_token, token):
    """Whether a cache entry built under `built_token` may serve a lookup under `token`."""
    return built_token is None or built_token is token


def capture_keep(obj, token):
    """Keep `obj` alive as long as the graph being captured under `token`."""
    if token is not None and token is not _ANON_CAPTURE:
        token.keep.append(obj)


class CaptureScope:
    """One graph capture's library state: the conv_gemm8 stream-K workspaces
    (clskd_capture_scope_begin, include/clskd.h) — created just before ``torch.cuda.graph(...)``
    with every stream the capture launches on, ended right after it, freed together with the
    graph (without a scope a captured launch runs the data-parallel tile deal, and its replays
    would differ in the last bits from the eager launches of a prepared stream, which split
    tiles) — and the cache token / keep-alive list above."""

    def __init__(self, streams):
        import ctypes as C
        global _CAPTURE_TOKEN
        if _CAPTURE_TOKEN is not None:
            raise RuntimeError("CaptureScope: another capture is being recorded")
        self._lib = lib()
        ptrs = (C.c_void_p * len(streams))(*[s.cuda_stream for s in streams])
        h = C.c_void_p()
        check(self._lib.clskd_capture_scope_begin(ptrs, len(streams), C.byref(h)), "capture_scope_begin")
        self.h, self.bound = h, True
        self.keep = []
        _CAPTURE_TOKEN = self

    def end(self):
        global _CAPTURE_TOKEN
        if self.bound:
            self.bound = False
            if _CAPTURE_TOKEN is self:
                _CAPTURE_TOKEN = None
            check(self._lib.clskd_capture_scope_end(self.h), "capture_scope_end")

    def free(self):
        """Release the workspaces and kept tensors: the graph captured under this scope must not
        run again."""
        self.end()
        if self.h is not None and self.h.value:
            torch.cuda.synchronize()  # no replay using them may still be queued
            check(self._lib.clskd_capture_scope_free(self.h), "capture_scope_free")
        self.h = None
        self.keep = []

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


_CAPTURE_STREAMS = {}


def capture_stream(device):
    """One prepared stream per device for graph capture (torch.cuda.graph(..., stream=)) and the
    capture's warm-up."""
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    s = _CAPTURE_STREAMS.get(idx)
    if s is None:
        s = _CAPTURE_STREAMS[idx] = prepare_stream(torch.cuda.Stream(device=idx))
    return s


def conv_last_stream_k():
    """Whether this thread's last conv launch ran conv_gemm8's stream-K deal."""
    return bool(lib().clskd_conv_last_stream_k())


def conv_kernel_of_last_launch():
    """Kernel instance (rocprof name, 'base<args>') of this thread's last conv launch."""
    return lib().clskd_conv_last_kernel().decode()


# ------------------------------------------------------------------------------------------
# BatchNorm (+ PReLU)
# ------------------------------------------------------------------------------------------
def batch_norm_bftc(x, y, gamma, beta, running_mean, running_var, train, momentum=0.1,
                    eps=1e-5, n_updates=1, alpha=None, stats_out=None, partial=None,
                    return_coef=False):
    """nn.BatchNorm2d over a BFTC tensor (channels last), then optional PReLU (single alpha).
    train: batch statistics (biased var), running stats updated n_updates times (if given).
    partial=(tensor, nblk): statistics already produced by the conv epilogue (fused).
    y=None: compute the coefficients only and return the [scale | shift] fp32 tensor (for a
    consumer kernel that applies them on load).  return_coef: return (y, coef) (the backward
    pass needs the forward's coefficients with stats_out's batch mean / var)."""
    L = lib()
    Cn = x.shape[-1]
    if Cn > 4096:
        raise RuntimeError("batch_norm_bftc: more than 4096 channels")
    rows = x.numel() // Cn
    dev = x.device
    coef = torch.empty(2 * Cn, device=dev, dtype=torch.float32)  # [scale | shift]
    scale = coef.data_ptr()
    shift = scale + 4 * Cn
    st = _stream()
    if train:
        if partial is not None:
            part, nblk = partial
        else:
            nblk = L.clskd_bn_partial_blocks(rows, Cn)
            part = torch.empty(nblk * Cn * 2, device=dev, dtype=torch.float64)
            check(L.clskd_bn_stats_partial(ptr(x), rows, Cn, ptr(part), nblk, _dt(x), st), "bn_stats")
        mean_o = var_o = None
        if stats_out is not None:
            mean_o, var_o = stats_out
        upd = running_mean is not None and running_var is not None and n_updates > 0
        check(L.clskd_bn_finalize(ptr(part), nblk, rows, Cn, ptr(gamma), ptr(beta), eps,
                                  ptr(running_mean) if upd else None,
                                  ptr(running_var) if upd else None, momentum, n_updates,
                                  scale, shift, ptr(mean_o), ptr(var_o), st),
              "bn_finalize")
    else:
        check(L.clskd_bn_eval_coeffs(ptr(running_mean), ptr(running_var), ptr(gamma), ptr(beta),
                                     eps, Cn, scale, shift, st), "bn_eval")
    if y is None:
        return coef
    assert x.dtype == y.dtype
    check(L.clskd_bn_apply(ptr(x), ptr(y), rows, Cn, scale, shift, ptr(alpha), _dt(x), st),
          "bn_apply")
    return (y, coef) if return_coef else y


def bn_fold_state(bn, Cn, device):
    """Device state of a BatchNorm's folded finalize (clskd_bn_fold): int64 limb accumulators
    and the last-arriver ticket, zero at rest (the finalizing workgroup returns them to zero), so
    one allocation per module and device serves every step, graph replay included."""
    states = bn.__dict__.setdefault("_clskd_fold", {})
    key = (torch.device(device).index, Cn)
    st = states.get(key)
    if st is None:
        n = int(lib().clskd_bn_fold_state_size(Cn))
        st = (torch.zeros(n, dtype=torch.int64, device=device),
              torch.zeros(2, dtype=torch.int32, device=device))
        states[key] = st
    return st


class BnStats:
    """Train-mode batch statistics of one BatchNorm over the conv launches that produce its input
    (the decoder's two polyphase parities are two launches of one layer).  Each launch passes
    bn_stats=(this, is_last) to conv(); the library either folds the finalize into the launch
    (the persistent engines: no clskd_bn_finalize launch, coefficients written by the last
    workgroup) or writes fused per-128-row partials that coefficients() finalizes with one
    clskd_bn_finalize launch.  coefficients() returns the [scale | shift] fp32 tensor; the
    running statistics are updated n_updates times (nn.BatchNorm2d train forward) and the batch
    mean / biased var written to stats_out if given."""

    def __init__(self, bn, Cn, rows, n_updates, device, stats_out=None, gamma=None, beta=None):
        self.bn, self.C, self.rows, self.dev = bn, Cn, int(rows), device
        self.gamma = bn.weight if gamma is None else gamma
        self.beta = bn.bias if beta is None else beta
        upd = bn.running_mean is not None and bn.running_var is not None and n_updates > 0
        self.rm = bn.running_mean if upd else None
        self.rv = bn.running_var if upd else None
        self.n_updates = n_updates if upd else 0
        self.coef = torch.empty(2 * Cn, device=device, dtype=torch.float32)
        self.stats_out = stats_out
        self.mode = None  # "fold" | "part", set by the first launch
        self.no_fold = False  # partials_only(): some launch of the layer cannot fold
        self.part, self.used, self.nblk = None, 0, 0
        self._keep = []

    def partials_only(self):
        """Every launch of this BatchNorm writes partials (one of them cannot fold)."""
        self.no_fold = True
        return self

    def fold_struct(self, last, c_off):
        acc, ticket = bn_fold_state(self.bn, self.C, self.dev)
        sc = self.coef.data_ptr()
        mo, vo = self.stats_out if self.stats_out is not None else (None, None)
        f = _lib.BnFold(acc.data_ptr(), ticket.data_ptr(), int(last), self.C, int(c_off),
                        self.n_updates, self.rows, ptr(self.gamma), ptr(self.beta), self.bn.eps,
                        self.bn.momentum, ptr(self.rm), ptr(self.rv), sc, sc + 4 * self.C,
                        ptr(mo), ptr(vo))
        self._keep.append(f)
        return f

    def partials(self, nblk):
        """(buffer, element offset) for the next non-folding launch's partials."""
        if self.part is None:  # sized for the largest layer this object can describe
            self.nblk = -(-self.rows // 128) + 64
            self.part = torch.empty(self.nblk * self.C * 2, device=self.dev, dtype=torch.float64)
        off = self.used * self.C * 2
        self.used += nblk
        assert self.used <= self.nblk, "BnStats: more partial blocks than rows / 128"
        return self.part, off

    def abort(self):
        """A launch of this BatchNorm failed: zero its fold accumulators and ticket (stream-
        ordered), which only the finalizing launch would otherwise return to zero."""
        states = self.bn.__dict__.get("_clskd_fold", {})
        st = states.get((torch.device(self.dev).index, self.C))
        if st is not None:
            st[0].zero_()
            st[1].zero_()

    def launched(self, fold):
        mode = "fold" if fold else "part"
        if self.mode is None:
            self.mode = mode
        elif self.mode != mode:
            raise RuntimeError("BnStats: the launches of one BatchNorm dispatch to folding and "
                               "non-folding kernels")

    def coefficients(self):
        if self.mode == "part":
            L = lib()
            sc = self.coef.data_ptr()
            mo, vo = self.stats_out if self.stats_out is not None else (None, None)
            check(L.clskd_bn_finalize(ptr(self.part), self.used, self.rows, self.C,
                                      ptr(self.gamma), ptr(self.beta), self.bn.eps, ptr(self.rm),
                                      ptr(self.rv), self.bn.momentum, self.n_updates, sc,
                                      sc + 4 * self.C, ptr(mo), ptr(vo), _stream()),
                  "bn_finalize")
            self.mode = "done"
        elif self.mode not in ("fold", "done"):
            raise RuntimeError("BnStats: no launch produced these statistics")
        self._keep = []
        return self.coef


def bn_apply(x, y, coef, alpha=None):
    """y = x * scale + shift per channel (BFTC, channels last) [then PReLU(alpha)] with the
    [scale | shift] coefficients coef; y may be x."""
    Cn = x.shape[-1]
    sc = coef.data_ptr()
    assert x.dtype == y.dtype and coef.numel() == 2 * Cn
    check(lib().clskd_bn_apply(ptr(x), ptr(y), x.numel() // Cn, Cn, sc, sc + 4 * Cn, ptr(alpha),
                               _dt(x), _stream()), "bn_apply")
    return y


# ------------------------------------------------------------------------------------------
# LSTM, STFT helpers, ABF fuse
# ------------------------------------------------------------------------------------------
def lstm_recurrent(gx, gx_ws, gx_seq, gx_t, whh, nws, nseq, T, H, out, o_ws, o_seq, o_t):
    check(lib().clskd_lstm_recurrent(ptr(gx), gx_ws, gx_seq, gx_t, ptr(whh), nws, nseq, T, H,
                                     ptr(out), o_ws, o_seq, o_t, _stream()), "lstm")
    return out


def lstm_pre_capable(H):
    """Whether lstm_recurrent_pre runs for hidden size H (else: lstm_recurrent + the backward's
    pre-activation recompute)."""
    return bool(lib().clskd_lstm_pre_capable(H))


def lstm_recurrent_pre(gx, gx_ws, gx_seq, gx_t, whh, nws, nseq, T, H, out, o_ws, o_seq, o_t,
                       cbuf=None):
    """lstm_recurrent that also overwrites gx with the gate pre-activations (taped forward) and,
    given cbuf (nws*nseq*T*H fp32), stores the cell states there for lstm_bwd."""
    assert cbuf is None or (cbuf.dtype == torch.float32 and cbuf.numel() == nws * nseq * T * H)
    check(lib().clskd_lstm_recurrent_pre(ptr(gx), gx_ws, gx_seq, gx_t, ptr(whh), nws, nseq, T, H,
                                         ptr(out), o_ws, o_seq, o_t, ptr(cbuf), _stream()),
          "lstm_pre")
    return out


def lstm_cell(gx, gx_ws, gx_seq, whh, nws, nseq, H, h, c, s_ws, s_seq, out, o_ws, o_seq):
    """One LSTM step with carried (h, c), updated in place (clskd_lstm_cell)."""
    check(lib().clskd_lstm_cell(ptr(gx), gx_ws, gx_seq, ptr(whh), nws, nseq, H, ptr(h), ptr(c),
                                s_ws, s_seq, ptr(out), o_ws, o_seq, _stream()), "lstm_cell")


def complex_combine(rr, ii, ir, ri, ro, io):
    """ro = rr - ii, io = ir + ri (fp32 inputs); ro / io may be fp32, bf16 or fp16 storage."""
    if ro.dtype == torch.float32 and io.dtype == torch.float32:
        check(lib().clskd_complex_combine(ptr(rr), ptr(ii), ptr(ir), ptr(ri), ptr(ro), ptr(io),
                                          ro.numel(), _stream()), "complex_combine")
        return
    assert ro.dtype == io.dtype
    check(lib().clskd_complex_combine_dt(ptr(rr), ptr(ii), ptr(ir), ptr(ri), ptr(ro), ptr(io),
                                         ro.numel(), _dt(ro), _stream()), "complex_combine_dt")


def frame_pad(x, pad, Lp, mode, out):
    B, L = x.shape
    check(lib().clskd_frame_pad(ptr(x), x.stride(0), B, L, pad, Lp, mode, ptr(out), _stream()),
          "frame_pad")
    return out


def spec_bftc(spec, re0, im0, F, out):
    """Frame-major spectrum [B][T][ld] -> BFTC [B][F][T][2] (re at re0+f, im at im0+f)."""
    B, T, ld = spec.shape
    check(lib().clskd_spec_bftc(ptr(spec), B, T, ld, re0, im0, F, ptr(out), _stream()), "spec_bftc")
    return out


def mask_e(spec, mask, T, est, mask_r=None, mask_i=None):
    B = spec.shape[0]
    Tm = mask.shape[2]
    check(lib().clskd_mask_e(ptr(spec), spec.shape[-1], ptr(mask), Tm, B, T, ptr(est),
                             est.shape[-1], ptr(mask_r), ptr(mask_i), _stream()), "mask_e")


def ola_hop(frames, window, hop, out_len, trim, clamp, wav):
    B, T, win = frames.shape
    check(lib().clskd_ola(ptr(frames), ptr(window), B, T, win, hop, out_len, trim, int(clamp),
                          ptr(wav), _stream()), "ola")


def abf_fuse(x, res, w, b, out, x_coef=None):
    """x_coef: optional [scale | shift] (64 + 64 fp32) applied to x on load — the conv1
    BatchNorm of the ABF folded into the fuse (x is then the raw conv1 output)."""
    B, F, T, Cm = x.shape
    _, Fr, Tr, Cr = res.shape
    assert Cm == 64 and Cr == 64, "ABF fuse is built for mid_channel = 64 (framework.py:235)"
    assert x.dtype == res.dtype == out.dtype
    sc = sh = None
    if x_coef is not None:
        assert x_coef.dtype == torch.float32 and x_coef.numel() == 2 * Cm
        sc = x_coef.data_ptr()
        sh = sc + 4 * Cm
    check(lib().clskd_abf_fuse(ptr(x), ptr(res), B, F, T, Fr, Tr, ptr(w), ptr(b), sc, sh,
                               ptr(out), _dt(x), _stream()), "abf_fuse")
    return out


ABF_CIN = (8, 16, 32, 64)


def abf_tap_ok(x):
    """Can the folded-conv1 ABF kernels read this student tap in place?  (fp32 BFTC rows,
    channels contiguous, 16-B aligned rows, cin in ABF_CIN, 32-bit element offsets)."""
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[-1] not in ABF_CIN or x.stride(3) != 1:
        return False
    B, F, T, C = x.shape
    sB, sF, sT, _ = x.stride()
    if x.data_ptr() % 16 or sB % 4 or sF % 4 or sT % 4:
        return False
    return B * F * T < 2 ** 31 and (B - 1) * sB + (F - 1) * sF + (T - 1) * sT + C < 2 ** 31


def abf_bn1_coef(x, w1, bn, train, stats_out=None):
    """conv1 BatchNorm of an ABF level from the tap's moments (clskd_abf_bn1_partials, then the
    common finalize; eval: running statistics).  Returns [scale | shift] (64 + 64 fp32) and
    updates the running statistics like every other train-mode BatchNorm."""
    L = lib()
    B, F, T, C = x.shape
    rows = B * F * T
    dev = x.device
    mid = w1.shape[0]
    coef = torch.empty(2 * mid, device=dev, dtype=torch.float32)
    scale = coef.data_ptr()
    shift = scale + 4 * mid
    st = _stream()
    if not train:
        check(L.clskd_bn_eval_coeffs(ptr(bn.running_mean), ptr(bn.running_var), ptr(bn.weight),
                                     ptr(bn.bias), bn.eps, mid, scale, shift, st), "bn_eval")
        return coef
    nblk = int(L.clskd_abf_moment_blocks(rows, C))
    sB, sF, sT, _ = x.stride()
    if _BN_FOLD:  # the moments kernel's last block writes the coefficients (clskd_bn_fold)
        bst = BnStats(bn, mid, rows, 1, dev, stats_out=stats_out)
        f = bst.fold_struct(True, 0)
        check(L.clskd_abf_bn1_fold(ptr(x), B, F, T, sB, sF, sT, C, ptr(w1.reshape(mid, C)),
                                   _addr(f), nblk, st), "abf_bn1_fold")
        bst.launched(True)
        return bst.coefficients()
    part = torch.empty(nblk * mid * 2, device=dev, dtype=torch.float64)
    check(L.clskd_abf_bn1_partials(ptr(x), B, F, T, sB, sF, sT, C, ptr(w1.reshape(mid, C)),
                                   ptr(part), nblk, st), "abf_bn1_partials")
    return bn_coef_from_partials(part, nblk, rows, mid, bn, coef, stats_out)


def bn_coef_from_partials(part, nblk, rows, C, bn, coef, stats_out=None):
    """Train-mode BatchNorm coefficients [scale | shift] into `coef` from fused {sum, sumsq}
    partials [nblk][C][2] (one clskd_bn_finalize launch reads them all); updates bn's running
    statistics once."""
    L = lib()
    st = _stream()
    mean_o = var_o = None
    if stats_out is not None:
        mean_o, var_o = stats_out
    scale = coef.data_ptr()
    check(L.clskd_bn_finalize(ptr(part), nblk, rows, C, ptr(bn.weight), ptr(bn.bias), bn.eps,
                              ptr(bn.running_mean), ptr(bn.running_var), bn.momentum, 1, scale,
                              scale + 4 * C, ptr(mean_o), ptr(var_o), st), "bn_finalize")
    return coef


def abf_conv1_fuse(x, w1, coef, res, att, out, x1_raw=None):
    """out = ABF level map: BN1(W1 x) [attention-fused with the nearest-upsampled residual res]
    (clskd_abf_conv1_fuse); x1_raw (optional) receives W1 x."""
    B, F, T, C = x.shape
    mid = w1.shape[0]
    assert mid == 64 and out.shape == (B, F, T, 64) and out.is_contiguous()
    sB, sF, sT, _ = x.stride()
    Fr = Tr = 1
    aw = ab = None
    if res is not None:
        assert res.dtype == out.dtype and res.is_contiguous() and res.shape[-1] == 64
        _, Fr, Tr, _ = res.shape
        aw, ab = att
    if x1_raw is not None:
        assert x1_raw.dtype == out.dtype and x1_raw.shape == out.shape and x1_raw.is_contiguous()
    sc = coef.data_ptr()
    check(lib().clskd_abf_conv1_fuse(ptr(x), B, F, T, sB, sF, sT, C, ptr(w1.reshape(mid, C)), sc,
                                     sc + 4 * mid, ptr(res), Fr, Tr, ptr(aw), ptr(ab), ptr(out),
                                     ptr(x1_raw), _dt(out), _stream()), "abf_conv1_fuse")
    return out


# ------------------------------------------------------------------------------------------
# Gram / SPKD
# ------------------------------------------------------------------------------------------
@dataclass
class GramView:
    tensor: torch.Tensor
    offset: int
    sB: int
    P: int
    Ctot: int
    c0: int
    Cs: int
    affine: torch.Tensor = None  # optional [scale | shift] (2 x Ctot fp32) applied on load
    alpha: torch.Tensor = None   # optional PReLU slope (with affine), applied after it
    out: torch.Tensor = None     # optional: the transformed elements are also written here
                                 # (same layout as the view's tensor; may be the tensor itself)


class DeferredBN:
    """A BFTC conv output whose BatchNorm apply is deferred: raw tensor + [scale | shift]
    coefficients.  A Gram over it folds the affine into its loads (GramView.affine);
    materialize() runs clskd_bn_apply once (on the current stream) for anyone who wants the
    normalised tensor itself."""

    def __init__(self, raw, coef):
        self.raw, self.coef = raw, coef
        self._y = None

    @property
    def shape(self):
        return self.raw.shape

    def materialize(self):
        if self._y is None:
            x = self.raw
            Cn = x.shape[-1]
            y = torch.empty_like(x)
            sc = self.coef.data_ptr()
            check(lib().clskd_bn_apply(ptr(x), ptr(y), x.numel() // Cn, Cn, sc, sc + 4 * Cn, None,
                                       _dt(x), _stream()), "bn_apply")
            self._y = y
        return self._y


class MaterializingList(list):
    """List of tensors / DeferredBN entries that hands out materialised tensors."""

    def __getitem__(self, i):
        v = super().__getitem__(i)
        if isinstance(i, slice):
            return [x.materialize() if isinstance(x, DeferredBN) else x for x in v]
        return v.materialize() if isinstance(v, DeferredBN) else v

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


def gram_view(t):
    """View of a tensor as z_b (any tensor whose per-sample block is contiguous)."""
    B = t.shape[0]
    if t.dtype not in (torch.float32, torch.bfloat16):
        t = t.float()
    g = 8 if t.dtype == torch.bfloat16 else 4
    if t.is_contiguous():
        n = t.numel() // B
        if n % g == 0:
            return GramView(t, 0, n, n // g, g, 0, g)
    # BFTC buffer exposed as an NCHW permuted view: underlying storage contiguous
    if t.dim() == 4 and t.stride(1) == 1:
        Bn, Cn, Fn, Tn = t.shape
        if t.stride() == (Fn * Tn * Cn, 1, Tn * Cn, Cn) and (Fn * Tn * Cn) % g == 0:
            n = Fn * Tn * Cn
            return GramView(t, 0, n, n // g, g, 0, g)
    tc = t.contiguous()
    n = tc.numel() // B
    if n % g != 0:  # zero padding adds nothing to z z^T
        tc = torch.cat([tc.reshape(B, n), tc.new_zeros(B, g - n % g)], 1)
        n = tc.shape[1]
    return GramView(tc, 0, n, n // g, g, 0, g)


# Elements per row per slab (one workgroup each).  Smaller slabs mean more workgroups in flight
# and more partials for the finalize; tools/gram_micro.py on MI355X (one view, isolated):
# bf16 8192 -> 5.4-5.9 TB/s (16384: 3.5-5.9), fp32 2048 -> 4.0-4.9 TB/s (16384: 1.0-1.9, about
# 100 workgroups).  A/B knobs CLSKD_GRAM_CHUNK_BF16 / CLSKD_GRAM_CHUNK_F32.
_GRAM_CHUNK_BF16 = int(os.environ.get("CLSKD_GRAM_CHUNK_BF16", "16384"))
_GRAM_CHUNK_F32 = int(os.environ.get("CLSKD_GRAM_CHUNK_F32", "16384"))


class GramSlabs:
    """Gram partials of some views, launched on the current stream into a slab buffer of their
    own (clskd_gram_partial).  `refs[i]` = (device address of view i's first slab, slab count)
    for clskd_spkd_finalize_ranges; the object owns the buffer (keep it until the finalize ran)."""

    def __init__(self, views, B, chunk_elems=None):
        dev = views[0].tensor.device
        jobs = (_lib.GramJob * len(views))()
        first = 0
        spans = []
        for j, v in enumerate(views):
            dt = _dt(v.tensor)
            ce = chunk_elems or (_GRAM_CHUNK_BF16 if dt == _lib.BF16 else _GRAM_CHUNK_F32)
            chunk = max(1, ce // v.Cs)
            ns = -(-v.P // chunk)
            assert v.Cs % (8 if dt == _lib.BF16 else 4) == 0
            sc = sh = al = out = None
            if v.affine is not None:
                assert v.affine.dtype == torch.float32 and v.affine.numel() == 2 * v.Ctot
                sc = v.affine.data_ptr()
                sh = sc + 4 * v.Ctot
            if v.alpha is not None:
                assert v.affine is not None and v.alpha.dtype == torch.float32
                al = v.alpha.data_ptr()
            if v.out is not None:
                assert v.affine is not None and v.out.dtype == v.tensor.dtype
                assert v.out.numel() == v.tensor.numel() and v.out.is_contiguous()
                out = v.out.data_ptr() + v.out.element_size() * v.offset
            jobs[j] = _lib.GramJob(v.tensor.data_ptr() + v.tensor.element_size() * v.offset, v.sB,
                                   v.P, v.Ctot, v.c0, v.Cs, chunk, first, ns, dt, 0, sc, sh, al, out)
            spans.append((first, ns))
            first += ns
        self.slabs = torch.empty(first * 1024, dtype=torch.float32, device=dev)
        base = self.slabs.data_ptr()
        self.refs = [(base + 4096 * f, n) for f, n in spans]
        # job table is a host array passed as kernel arguments (no upload, capturable)
        check(lib().clskd_gram_partial(jobs, len(views), B, base, _stream()), "gram_partial")
        if KernelTimer.active:  # algorithmic bytes: every tap once (+ the fused apply's write)
            nb = self.slabs.numel() * 4
            fl = 0.0
            for v in views:
                n = B * v.P * v.Cs * v.tensor.element_size()
                nb += n * (2 if v.out is not None else 1)
                fl += 2.0 * B * B * v.P * v.Cs
            KernelTimer.note_work(f"gram_partial_kernel<{1 if B <= 16 else 2}>", nb, fl)


# fused BatchNorm-apply + Gram (bn_apply_gram): slabs per tap.  The launch sits on the producing
# chain (it replaces the bn_apply pass), so it gets enough workgroups to stream the tap at the
# HBM rate; the SPKD finalize sums every slab, so not many more.
_APPLY_GRAM_SLABS = 512


def bn_apply_gram(x, coef, alpha, B, out=None):
    """In-place BatchNorm (+ PReLU alpha) apply of the BFTC tensor x with the [scale | shift]
    coefficients `coef`, fused with the SPKD Gram partials of the applied tensor (one pass over
    the tap instead of an apply pass and a Gram pass; bitwise the same tensor as clskd_bn_apply
    and the same partials as a Gram over it).  Returns the GramSlabs (keep it until the finalize
    ran)."""
    Bn, F, T, C = x.shape
    assert x.is_contiguous() and Bn == B
    per_row = F * T * C
    ce = -(-per_row // _APPLY_GRAM_SLABS)
    ce = max(C, min(16384, -(-ce // C) * C))
    view = GramView(x, 0, per_row, F * T, C, 0, C, coef, alpha, x if out is None else out)
    return GramSlabs([view], B, chunk_elems=ce)


def spkd_finalize(s_refs, t_refs, B, batchmean=True, out=None, return_grams=False, device=None):
    """Per pair i: Gs from the slabs s_refs[i], Gt from t_refs[i] (GramSlabs.refs entries, any
    streams — the caller orders them before this launch); row-L1-normalise, ||Gt - Gs||^2."""
    n = len(s_refs)
    assert len(t_refs) == n and n >= 1
    losses = out if out is not None else torch.empty(n, dtype=torch.float32, device=device)
    assert losses.is_contiguous() and losses.numel() == n
    gs = gt = None
    if return_grams:
        gs = torch.empty(n, B, B, dtype=torch.float32, device=losses.device)
        gt = torch.empty_like(gs)
    sp = (C.c_void_p * n)(*[r[0] for r in s_refs])
    tp = (C.c_void_p * n)(*[r[0] for r in t_refs])
    sn = (C.c_int32 * n)(*[r[1] for r in s_refs])
    tn = (C.c_int32 * n)(*[r[1] for r in t_refs])
    check(lib().clskd_spkd_finalize_ranges(sp, sn, tp, tn, n, B, int(batchmean), ptr(gs), ptr(gt),
                                           ptr(losses), _stream()), "spkd_finalize")
    if return_grams:
        return losses, gs, gt
    return losses


def spkd_losses(pairs_views, B, batchmean=True, return_grams=False, chunk_elems=None, out=None):
    """pairs_views: list of (student GramView, teacher GramView).  One gram launch for every
    view, one finalize launch for every pair.  Returns losses [npairs] (and grams)."""
    views = [v for pr in pairs_views for v in pr]
    g = GramSlabs(views, B, chunk_elems)
    r = spkd_finalize(g.refs[0::2], g.refs[1::2], B, batchmean, out, return_grams,
                      device=views[0].tensor.device)
    del g  # slab buffer returns to the allocator after both launches are enqueued (same stream)
    return r


# ------------------------------------------------------------------------------------------
# losses
# ------------------------------------------------------------------------------------------
def stft_mag_loss(X, Y, nbins, factor_sc=0.1, factor_mag=0.1, out2=None, accumulate=False):
    """X, Y: raw spectra [..., 2*nbins] (re | im).  Returns out2 = [sc, mag] (device);
    accumulate=True adds into out2 (multi-resolution sums)."""
    rows = X.numel() // X.shape[-1]
    dev = X.device
    acc = torch.empty(256 * 3, dtype=torch.float64, device=dev)
    if out2 is None:
        out2 = torch.empty(2, dtype=torch.float32, device=dev)
    L = lib()
    st = _stream()
    check(L.clskd_stft_mag_loss(ptr(X), ptr(Y), rows, X.shape[-1], nbins, ptr(acc), st), "stft_mag_loss")
    check(L.clskd_stft_loss_finalize(ptr(acc), rows * nbins, factor_sc, factor_mag,
                                     int(accumulate), ptr(out2), st),
          "stft_loss_finalize")
    return out2


def sisnr_rows(s1, s2, eps=1e-8):
    """Per-row SI-SNR (tools_for_loss.py:37-47) of [rows, L] tensors -> [rows] (device)."""
    s1 = s1.reshape(-1, s1.shape[-1])
    s2 = s2.reshape(-1, s2.shape[-1])
    if s1.stride(-1) != 1:
        s1 = s1.contiguous()
    if s2.stride(-1) != 1:
        s2 = s2.contiguous()
    out = torch.empty(s1.shape[0], dtype=torch.float32, device=s1.device)
    check(lib().clskd_sisnr_rows(ptr(s1), ptr(s2), s1.shape[0], s1.shape[1], s1.stride(0),
                                 s2.stride(0), eps, ptr(out), _stream()), "sisnr")
    return out


def sum_f32(a, out, scale=1.0):
    """out[0] = scale * sum(a) for a contiguous (or 1-D strided-1) tensor a."""
    check(lib().clskd_sum_f32(ptr(a), a.numel(), scale, ptr(out), _stream()), "sum_f32")
    return out


# ------------------------------------------------------------------------------------------
# backward (training step): weight gradients, data-gradient helpers, optimizer
# ------------------------------------------------------------------------------------------
_WGRAD_PLANS = {}


def conv_wgrad(segs, taps, B, Fo, To, N, dy, omap, dw, dbias=None, dy_offset=0, stride_f=1,
               stride_t=1, accumulate=False, accumulate_bias=None):
    """Weight gradient of the conv launch conv(segs, taps, B, Fo, To, N, ..., omap): fp32
    segments (the forward inputs), dy read through the forward's output map at dy + dy_offset.
    dw: [N][Kp] fp32 (the packed-weight layout, Kp = K padded to 16); dbias: [N] or None.
    accumulate adds into dw (and dbias, unless accumulate_bias says otherwise).
    Inside split_products(..., wgrad=True) the descriptor asks for 3 x bf16 split products
    (CLSKD_F32X3: csrc/wgrad_x3.hip), else the exact fp32 engine runs."""
    addrs = [seg_addr(sg) for sg in segs]
    taps = tuple(taps)
    geoms = tuple(sg.geom for sg in segs)
    split = getattr(_SPLIT, "wgrad", False)
    key = (geoms, taps, B, Fo, To, N, omap, stride_f, stride_t, dy.device.index,
           tuple(a % 16 for a in addrs), split)
    pl = _WGRAD_PLANS.get(key)
    if pl is None:
        assert all(sg.tensor.dtype == torch.float32 for sg in segs), "wgrad: fp32 segments"
        kt, ks, K, Kp, vec4 = _ktab(geoms, taps, dy.device.index or 0, BK)
        if any(a % 16 for a in addrs):
            vec4 = False
        d = _lib.ConvDesc()
        d.B, d.Fo, d.To, d.N, d.K = B, Fo, To, N, Kp
        d.stride_f, d.stride_t = stride_f, stride_t
        d.nseg = len(segs)
        for i, g in enumerate(geoms):
            d.seg[i] = _lib.Seg(0, g.sB, g.sF, g.sT, g.F, g.T)
        for i in range(len(segs), _lib.MAX_SEGS):
            d.seg[i] = d.seg[0]
        d.ktab, d.kseg, d.vec4 = kt.data_ptr(), ks.data_ptr(), int(vec4)
        d.oB, d.oF, d.oT, d.oNhi, d.oNlo = omap.oB, omap.oF, omap.oT, omap.oNhi, omap.oNlo
        d.nlo = min(omap.nlo, 1 << 30)
        d.of_mul, d.of_add = omap.of_mul, omap.of_add
        d.in_dtype = d.out_dtype = _lib.F32
        d.compute = _lib.F32X3 if split else _lib.F32
        ws = int(lib().clskd_conv2d_wgrad_workspace(d))
        pl = (d, Kp, ws)
        _WGRAD_PLANS[key] = pl
    d, Kp, ws = pl
    assert dw.shape == (N, Kp) and dw.dtype == torch.float32 and dw.is_contiguous(), (dw.shape, N, Kp)
    for i, a in enumerate(addrs):
        d.seg[i].ptr = a
    for i in range(len(segs), _lib.MAX_SEGS):
        d.seg[i].ptr = addrs[0]
    work = torch.empty(ws, dtype=torch.float32, device=dy.device)
    acc_b = accumulate if accumulate_bias is None else accumulate_bias
    check(lib().clskd_conv2d_wgrad(d, dy.data_ptr() + 4 * dy_offset, ptr(dw), ptr(dbias), ptr(work),
                                   ws, int(bool(accumulate)) | (int(bool(acc_b)) << 1), _stream()),
          "conv2d_wgrad")
    if KernelTimer.active and split:  # the split engine names its instance (conv_wgrad_x3<...>)
        name = lib().clskd_conv_last_kernel().decode()
        if name.startswith("conv_wgrad_x3"):
            K = sum(len(taps) * g.C for g in geoms)
            # algorithmic work: the GEMM's fp32-equivalent FLOPs; bytes: every operand once
            KernelTimer.note_work(name, 4 * (sum(B * g.F * g.T * g.C for g in geoms)
                                             + B * Fo * To * N + N * Kp),
                                  2.0 * B * Fo * To * N * K)
    return dw


def bn_bwd(x, dy, scale, shift, mean, var, eps, gamma, alpha, dx, dgamma=None, dbeta=None,
           dalpha=None, accumulate_dx=False, accumulate_params=False):
    """BatchNorm2d(train) [+ PReLU] backward over BFTC x (raw conv output, fp32 or bf16)."""
    L = lib()
    Cn = x.shape[-1]
    rows = x.numel() // Cn
    nblk = int(L.clskd_bn_bwd_blocks(rows, Cn))
    work = torch.empty(int(L.clskd_bn_bwd_workspace(nblk, Cn)), dtype=torch.float64, device=x.device)
    check(L.clskd_bn_bwd(ptr(x), ptr(dy), rows, Cn, ptr(scale), ptr(shift), ptr(mean), ptr(var), eps,
                         ptr(gamma), ptr(alpha), ptr(work), nblk, ptr(dgamma), ptr(dbeta),
                         ptr(dalpha), ptr(dx), int(accumulate_dx), int(accumulate_params), _dt(x),
                         _stream()), "bn_bwd")
    return dx


def abf_fuse_bwd(x1, res, w, b, x_coef, dout, dx, dyup, dnext=None, mv1=None, eps=1e-5):
    """ABF fusion backward.  dnext: the next level's dyup, folded onto this grid and added to
    dout on load.  mv1 = conv1 BN [mean; var]: also returns (partials, nblk) of that BN's
    backward statistics for bn_bwd_from_partials.  The gradient maps (dout, dnext, dx, dyup)
    share one storage type, fp32 or bf16 (dout's)."""
    L = lib()
    gdt = dout.dtype
    assert gdt in (torch.float32, torch.bfloat16), gdt
    for t in (dx, dyup, dnext):
        assert t is None or t.dtype == gdt, (t.dtype, gdt)
    B, F, T, Cm = x1.shape
    _, Fr, Tr, _ = res.shape
    sc = sh = None
    if x_coef is not None:
        sc = x_coef.data_ptr()
        sh = sc + 4 * Cm
    F2 = T2 = 0
    if dnext is not None:
        _, F2, T2, _ = dnext.shape
    part, nblk = None, 0
    if mv1 is not None:
        nblk = int(L.clskd_abf_fuse_bwd_blocks(B, F, T))
        part = torch.empty(nblk * Cm * 3, dtype=torch.float64, device=x1.device)
    check(L.clskd_abf_fuse_bwd(ptr(x1), ptr(res), B, F, T, Fr, Tr, ptr(w), ptr(b), sc, sh,
                               ptr(dout), ptr(dx), ptr(dyup), ptr(dnext), F2, T2,
                               ptr(mv1[0]) if mv1 is not None else None,
                               ptr(mv1[1]) if mv1 is not None else None, eps, ptr(part),
                               _dt(x1), _dt(dout), _stream()), "abf_fuse_bwd")
    if KernelTimer.active:  # algorithmic bytes: every operand once
        es, gs, npix = x1.element_size(), dout.element_size(), B * F * T
        nb = (npix * Cm * es + B * Fr * Tr * Cm * es + npix * Cm * gs * (2 + (dyup is not None))
              + (B * F2 * T2 * Cm * gs if dnext is not None else 0) + nblk * Cm * 3 * 8)
        tn = lambda e: "bf16" if e == 2 else "float"
        KernelTimer.note_work(f"abf_fuse_bwd_kernel<{tn(es)},{tn(gs)}>", nb)
    return part, nblk


def bn_bwd_from_partials(x, dy, scale, shift, mean, var, eps, gamma, partial, nblk, dx,
                         accumulate_dx=False):
    Cn = x.shape[-1]
    kbuf = torch.empty(3 * Cn, dtype=torch.float32, device=x.device)
    check(lib().clskd_bn_bwd_from_partials(ptr(x), ptr(dy), x.numel() // Cn, Cn, ptr(scale),
                                           ptr(shift), ptr(mean), ptr(var), eps, ptr(gamma),
                                           ptr(partial), nblk, ptr(kbuf), None, None, ptr(dx),
                                           int(accumulate_dx), _dt(x), _dt(dy), _stream()),
          "bn_bwd_from_partials")
    return dx


def bn_bwd_coeffs(x, dy, scale, shift, mean, var, eps, gamma, partial=None, nblk=0):
    """The BatchNorm-backward coefficients k [3][C] (d = k0*dy + k1*x + k2) without the apply
    pass: from a fused producer's partials (clskd_bn_bwd_from_partials with dx NULL), else by
    the reduce + finalize of clskd_bn_bwd (dx NULL)."""
    L = lib()
    Cn = x.shape[-1]
    rows = x.numel() // Cn
    if partial is not None:
        kbuf = torch.empty(3 * Cn, dtype=torch.float32, device=x.device)
        check(L.clskd_bn_bwd_from_partials(ptr(x), ptr(dy), rows, Cn, ptr(scale), ptr(shift),
                                           ptr(mean), ptr(var), eps, ptr(gamma), ptr(partial),
                                           nblk, ptr(kbuf), None, None, None, 0, _dt(x), _dt(dy),
                                           _stream()), "bn_bwd_coeffs")
        return kbuf
    assert dy.dtype == torch.float32, dy.dtype
    nb = int(L.clskd_bn_bwd_blocks(rows, Cn))
    work = torch.empty(int(L.clskd_bn_bwd_workspace(nb, Cn)), dtype=torch.float64, device=x.device)
    check(L.clskd_bn_bwd(ptr(x), ptr(dy), rows, Cn, ptr(scale), ptr(shift), ptr(mean), ptr(var), eps,
                         ptr(gamma), None, ptr(work), nb, None, None, None, None, 0, 0, _dt(x),
                         _stream()), "bn_bwd_coeffs")
    return work.view(torch.float32)[nb * Cn * 6:nb * Cn * 6 + 3 * Cn]


def bn_bwd_conv1x1_ok(x, dy, w, out):
    C = x.shape[-1]
    N = w.shape[1]
    return (C == 64 and N in (8, 16, 32, 64) and x.is_contiguous() and dy.is_contiguous()
            and w.is_contiguous() and w.dtype == torch.float32 and out.dtype == torch.float32
            and out.is_contiguous() and out.numel() == x.numel() // C * N
            and all(t.data_ptr() % 16 == 0 for t in (x, dy, out)))


def bn_bwd_conv1x1(x, dy, k, w, out, accumulate=False):
    """out [rows][N] (+)= (k0*dy + k1*x + k2) @ w [64][N]: a BatchNorm-backward apply fused with
    the 1x1 conv's data gradient (clskd_bn_bwd_conv1x1)."""
    C = x.shape[-1]
    rows = x.numel() // C
    assert k.data_ptr() % 16 == 0 and k.numel() >= 3 * C
    check(lib().clskd_bn_bwd_conv1x1(ptr(x), _dt(x), ptr(dy), _dt(dy), rows, C, ptr(k), ptr(w),
                                     w.shape[1], ptr(out), int(bool(accumulate)), _stream()),
          "bn_bwd_conv1x1")
    if KernelTimer.active:  # algorithmic bytes: x, dy, out (read + write when accumulating)
        n = w.shape[1]
        tn = lambda e: "bf16" if e == 2 else "float"
        KernelTimer.note_work(f"bn_bwd_conv1x1_kernel<{tn(x.element_size())},"
                              f"{tn(dy.element_size())},{n}>",
                              rows * (C * (x.element_size() + dy.element_size())
                                      + n * 4 * (2 if accumulate else 1)))
    return out


def split_planes(x, planes):
    """fp32 [..][C] -> bf16 planes [..][2C]: hi = bf16(x) | lo = bf16(x - hi) (clskd_split_planes)."""
    C = x.shape[-1]
    assert planes.shape[-1] == 2 * C and planes.dtype == torch.bfloat16 and x.is_contiguous()
    check(lib().clskd_split_planes(ptr(x), x.numel() // C, C, ptr(planes), _stream()),
          "split_planes")


def pack_split3(w, ntaps, C, out):
    """fp32 [N][ldw] (K order tap, channel) -> bf16 [N][Kp]: per tap [W_hi | W_hi | W_lo]."""
    N, ldw = w.shape
    assert w.dtype == torch.float32 and w.is_contiguous() and out.dtype == torch.bfloat16
    check(lib().clskd_pack_split3(ptr(w), N, ldw, ntaps, C, out.shape[1], ptr(out), _stream()),
          "pack_split3")


def nearest_down_sum(g, out, accumulate=False):
    B, F, T, Cn = g.shape
    _, Fr, Tr, _ = out.shape
    assert out.dtype == torch.float32, out.dtype
    check(lib().clskd_nearest_down_sum(ptr(g), B, F, T, Fr, Tr, Cn, ptr(out), int(accumulate),
                                       _dt(g), _stream()), "nearest_down_sum")


def mask_e_bwd(spec, mask, T, dest, dmask):
    B = spec.shape[0]
    check(lib().clskd_mask_e_bwd(ptr(spec), spec.shape[-1], ptr(mask), mask.shape[2], B, T,
                                 ptr(dest), dest.shape[-1], ptr(dmask), _stream()), "mask_e_bwd")


def ola_bwd(frames, window, dwav, hop, out_len, trim, clamp, dframes):
    B, T, win = frames.shape
    check(lib().clskd_ola_bwd(ptr(frames), ptr(window), ptr(dwav), B, T, win, hop, out_len, trim,
                              int(clamp), ptr(dframes), _stream()), "ola_bwd")


def frame_pad_bwd(dxp, L, pad, mode, dx, accumulate=False):
    B, Lp = dxp.shape
    check(lib().clskd_frame_pad_bwd(ptr(dxp), B, L, pad, Lp, mode, ptr(dx), dx.stride(0),
                                    int(accumulate), _stream()), "frame_pad_bwd")


def stft_mag_loss_bwd(X, Y, nbins, scale, dX):
    rows = X.numel() // X.shape[-1]
    check(lib().clskd_stft_mag_loss_bwd(ptr(X), ptr(Y), rows, X.shape[-1], nbins, scale, ptr(dX),
                                        dX.shape[-1], _stream()), "stft_mag_loss_bwd")


def complex_combine_bwd(dre, dim, dh):
    B = dre.shape[0]
    check(lib().clskd_complex_combine_bwd(ptr(dre), ptr(dim), B, dre.numel() // B, ptr(dh),
                                          _stream()), "complex_combine_bwd")


def lstm_bwd(pre, p_strides, dh, d_strides, whh, nws, nseq, T, H, dgates, g_strides, cells=None):
    """cells: the forward's cell states (lstm_recurrent_pre's cbuf), else recomputed here."""
    c_ready = cells is not None
    cbuf = cells if c_ready else torch.empty(nws * nseq * T * H, dtype=torch.float32, device=pre.device)
    assert cbuf.numel() == nws * nseq * T * H
    check(lib().clskd_lstm_bwd(ptr(pre), *p_strides, ptr(dh), *d_strides, ptr(whh), nws, nseq, T, H,
                               ptr(cbuf), int(c_ready), ptr(dgates), *g_strides, _stream()),
          "lstm_bwd")


def spkd_grad(s_refs, t_refs, B, batchmean=True, scale=1.0, out=None, device=None):
    """M = dG + dG^T per pair (clskd_spkd_grad_ranges) -> [npairs][B][B] fp32."""
    n = len(s_refs)
    coef = out if out is not None else torch.empty(n, B, B, dtype=torch.float32, device=device)
    sp = (C.c_void_p * n)(*[r[0] for r in s_refs])
    tp = (C.c_void_p * n)(*[r[0] for r in t_refs])
    sn = (C.c_int32 * n)(*[r[1] for r in s_refs])
    tn = (C.c_int32 * n)(*[r[1] for r in t_refs])
    check(lib().clskd_spkd_grad_ranges(sp, sn, tp, tn, n, B, int(batchmean), scale, ptr(coef),
                                       _stream()), "spkd_grad")
    return coef


def gram_bwd(items, B):
    """items: list of (GramView z, coef [B][B] tensor, out tensor, o_sB, o_Ctot, o_c0,
    accumulate): dz = M z written fp32 into out."""
    jobs = (_lib.GramBwdJob * len(items))()
    for i, (v, coef, out, o_sB, o_Ctot, o_c0, acc) in enumerate(items):
        sc = sh = None
        if v.affine is not None:
            sc = v.affine.data_ptr()
            sh = sc + 4 * v.Ctot
        assert out.dtype == torch.float32 and coef.dtype == torch.float32
        jobs[i] = _lib.GramBwdJob(v.tensor.data_ptr() + v.tensor.element_size() * v.offset, v.sB,
                                  v.P, v.Ctot, v.c0, v.Cs, _dt(v.tensor), sc, sh, coef.data_ptr(),
                                  out.data_ptr(), o_sB, o_Ctot, o_c0, int(acc), 0)
    check(lib().clskd_gram_bwd(jobs, len(items), B, _stream()), "gram_bwd")


def spkd_bn_bwd(raw, coef_bn, coef_m, mean, var, eps, gamma, draw, dgamma=None, dbeta=None):
    """SPKD gradient (dz = M z, z = the deferred-BN Gram input) fused into the BN backward of a
    BFTC map raw [B][F][T][C] (clskd_spkd_bn_bwd); writes draw (fp32 or bf16)."""
    L = lib()
    B = raw.shape[0]
    Cn = raw.shape[-1]
    P = raw.numel() // (B * Cn)
    # a reduce thread covers one (position, 4 channels) over all B samples: size the grid by
    # positions x channel quads, not by B*P rows
    nblk = int(L.clskd_bn_bwd_blocks(P * Cn // 2, Cn))
    work = torch.empty(int(L.clskd_bn_bwd_workspace(nblk, Cn)), dtype=torch.float64,
                       device=raw.device)
    sc = coef_bn.data_ptr()
    check(L.clskd_spkd_bn_bwd(ptr(raw), _dt(raw), P * Cn, P, Cn, B, sc, sc + 4 * Cn, ptr(coef_m),
                              ptr(mean), ptr(var), eps, ptr(gamma), ptr(work), nblk, ptr(dgamma),
                              ptr(dbeta), ptr(draw), _dt(draw), _stream()), "spkd_bn_bwd")
    if KernelTimer.active:  # algorithmic bytes: the reduce reads raw once, the apply raw + draw
        t = {2: "bf16", 4: "float"}
        bm = 32 if B > 16 else 16
        ex = "true" if B == bm else "false"  # the exact-batch instance (no sample guards)
        n = raw.numel()
        KernelTimer.note_work(f"spkd_bn_bwd_reduce_kernel<{t[raw.element_size()]},{bm},{ex}>",
                              n * raw.element_size() + nblk * Cn * 3 * 8)
        KernelTimer.note_work(f"spkd_bn_bwd_apply_kernel<{t[raw.element_size()]},"
                              f"{t[draw.element_size()]},{bm},{ex}>",
                              n * (raw.element_size() + draw.element_size()))
    return draw


def index_gather(src, idx, sgn, out, accumulate=False):
    """out[i] (+)= sum_j sgn[i, j] * src.flat[idx[i, j]] (idx < 0 skipped)."""
    n, J = idx.shape
    assert out.numel() == n and out.is_contiguous()
    check(lib().clskd_index_gather(ptr(src), ptr(idx), ptr(sgn), J, n, ptr(out), int(accumulate),
                                   _stream()), "index_gather")


def index_gather_jobs(jobs):
    """Several index gathers [(src, idx, sgn, out), ...] (no accumulation, disjoint outputs) in
    clskd_index_gather_jobs launches of up to GATHER_JOBS_MAX jobs each, on the current stream."""
    L = lib()
    for i in range(0, len(jobs), _lib.GATHER_JOBS_MAX):
        chunk = jobs[i:i + _lib.GATHER_JOBS_MAX]
        arr = (_lib.GatherJob * len(chunk))()
        for k, (src, idx, sgn, out) in enumerate(chunk):
            assert out.numel() == idx.shape[0] and out.is_contiguous()
            arr[k] = _lib.GatherJob(ptr(src), ptr(idx), ptr(sgn), ptr(out), idx.shape[0],
                                    idx.shape[1], 0)
        check(L.clskd_index_gather_jobs(arr, len(chunk), _stream()), "index_gather_jobs")


def adam_step(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    check(lib().clskd_adam_step(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, beta1, beta2, eps,
                                weight_decay, step, grad_scale, _stream()), "adam")


def adam_step_dev(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    """adam_step with the step count in `step` (int32 device tensor, advanced by the call)."""
    if step.dtype != torch.int32 or step.device != p.device:
        raise ValueError("adam_step_dev: step must be an int32 tensor on the parameters' device")
    check(lib().clskd_adam_step_dev(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, beta1, beta2,
                                    eps, weight_decay, ptr(step), grad_scale, _stream()), "adam_dev")


def fill(t, value=0.0):
    check(lib().clskd_fill_f32(ptr(t), t.numel(), value, _stream()), "fill")
    return t
