"""ctypes binding of libclskd_hip.so (include/clskd.h).

The product path has no CPU fallback: importing the ops on a machine without the built library
or without a HIP device raises immediately.
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# CLSKD_LIB=exp selects the timing-experiments build (clskd.build: never the product library)
# (or a .so file next to this one: a saved earlier build for a same-box A/B, tools/ only)
_LIB_ENV = os.environ.get("CLSKD_LIB", "")
LIB_PATH = os.path.join(_HERE, "libclskd_hip_exp.so" if _LIB_ENV == "exp"
                        else (os.path.basename(_LIB_ENV) if _LIB_ENV.endswith(".so")
                              else "libclskd_hip.so"))

MAX_SEGS = 4
F32, BF16, F16 = 0, 1, 2
F32X3 = 3  # conv compute: fp32 storage, 3 x bf16 split-product MFMA (include/clskd.h)
WLAYOUT_NK, WLAYOUT_DIRECT = 0, 1


class Seg(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("sB", C.c_int64), ("sF", C.c_int64), ("sT", C.c_int64),
                ("F", C.c_int32), ("T", C.c_int32)]


class KtabEntry(C.Structure):
    _fields_ = [("off", C.c_int32), ("dF", C.c_int16), ("dT", C.c_int16)]


class ConvDesc(C.Structure):
    _fields_ = [("B", C.c_int32), ("Fo", C.c_int32), ("To", C.c_int32), ("N", C.c_int32),
                ("K", C.c_int32), ("stride_f", C.c_int32), ("stride_t", C.c_int32),
                ("nseg", C.c_int32), ("seg", Seg * MAX_SEGS), ("ktab", C.c_void_p),
                ("kseg", C.c_void_p), ("vec4", C.c_int32), ("weight", C.c_void_p),
                ("bias", C.c_void_p), ("out", C.c_void_p), ("oB", C.c_int64), ("oF", C.c_int64),
                ("oT", C.c_int64), ("oNhi", C.c_int64), ("oNlo", C.c_int64), ("nlo", C.c_int32),
                ("of_mul", C.c_int32), ("of_add", C.c_int32), ("compute", C.c_int32),
                ("in_dtype", C.c_int32), ("out_dtype", C.c_int32), ("stats", C.c_void_p),
                ("kvec", C.c_int32), ("wlayout", C.c_int32), ("ntaps", C.c_int32),
                ("ctot", C.c_int32), ("seg_c", C.c_int32 * MAX_SEGS), ("tap_df", C.c_int16 * 16),
                ("tap_dt", C.c_int16 * 16), ("accumulate", C.c_int32), ("reserved_", C.c_int32),
                ("bn_fold", C.c_void_p)]


BN_FOLD_REPL = 8


class BnFold(C.Structure):
    """clskd_bn_fold (include/clskd.h): the folded BatchNorm finalize of a conv launch."""
    _fields_ = [("acc", C.c_void_p), ("ticket", C.c_void_p), ("finalize", C.c_int32),
                ("C", C.c_int32), ("c_off", C.c_int32), ("n_updates", C.c_int32),
                ("count", C.c_int64), ("gamma", C.c_void_p), ("beta", C.c_void_p),
                ("eps", C.c_float), ("momentum", C.c_float), ("running_mean", C.c_void_p),
                ("running_var", C.c_void_p), ("scale", C.c_void_p), ("shift", C.c_void_p),
                ("mean_out", C.c_void_p), ("var_out", C.c_void_p)]


class GramJob(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("sB", C.c_int64), ("P", C.c_int64), ("Ctot", C.c_int32),
                ("c0", C.c_int32), ("Cs", C.c_int32), ("chunk", C.c_int32),
                ("first_slab", C.c_int32), ("nslab", C.c_int32), ("dtype", C.c_int32),
                ("reserved", C.c_int32), ("scale", C.c_void_p), ("shift", C.c_void_p),
                ("alpha", C.c_void_p), ("out", C.c_void_p)]


class DrawJob(C.Structure):
    _fields_ = [("param", C.c_void_p), ("packed", C.c_void_p), ("numel", C.c_int64),
                ("Cin", C.c_int32), ("ntap", C.c_int32), ("Kp", C.c_int32),
                ("packed_dtype", C.c_int32), ("bound", C.c_float), ("stream_id", C.c_int32)]


class GramBwdJob(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("sB", C.c_int64), ("P", C.c_int64), ("Ctot", C.c_int32),
                ("c0", C.c_int32), ("Cs", C.c_int32), ("dtype", C.c_int32), ("scale", C.c_void_p),
                ("shift", C.c_void_p), ("coef", C.c_void_p), ("out", C.c_void_p),
                ("o_sB", C.c_int64), ("o_Ctot", C.c_int32), ("o_c0", C.c_int32),
                ("accumulate", C.c_int32), ("reserved", C.c_int32)]


class StreamHopArgs(C.Structure):
    _fields_ = [("stft_w", C.c_void_p), ("istft_w", C.c_void_p), ("window", C.c_void_p),
                ("enc_w", C.c_void_p * 6), ("enc_b", C.c_void_p * 6), ("enc_coef", C.c_void_p * 6),
                ("enc_alpha", C.c_void_p * 6), ("lstm_w", C.c_void_p * 2), ("lstm_b", C.c_void_p * 2),
                ("lstm_whh", C.c_void_p * 2), ("proj_w", C.c_void_p * 2), ("proj_b", C.c_void_p * 2),
                ("dec_w", (C.c_void_p * 2) * 6), ("dec_b", (C.c_void_p * 2) * 6),
                ("dec_coef", C.c_void_p * 6), ("dec_alpha", C.c_void_p * 6),
                ("state", C.c_void_p), ("state_stride", C.c_int64), ("x_in", C.c_void_p),
                ("wav_out", C.c_void_p), ("B", C.c_int32), ("t", C.c_int32), ("live", C.c_int32),
                ("zero_from", C.c_int32), ("H", C.c_int32), ("D4", C.c_int32),
                ("enc_cin", C.c_int32 * 6), ("enc_cout", C.c_int32 * 6), ("dec_ca", C.c_int32 * 6),
                ("dec_cb", C.c_int32 * 6), ("dec_co", C.c_int32 * 6), ("off_xwin", C.c_int32),
                ("off_spec", C.c_int32), ("off_enc", C.c_int32 * 6), ("off_decin", C.c_int32),
                ("off_dout", C.c_int32 * 5), ("off_h", C.c_int32), ("off_c", C.c_int32),
                ("off_frames", C.c_int32)]


assert C.sizeof(KtabEntry) == 8
assert C.sizeof(DrawJob) == 48
assert C.sizeof(GramJob) == 88

_p, _i32, _i64, _f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float

GATHER_JOBS_MAX = 48  # include/clskd.h CLSKD_GATHER_JOBS_MAX


class GatherJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("idx", C.c_void_p), ("sgn", C.c_void_p), ("out", C.c_void_p),
                ("n", C.c_int64), ("J", C.c_int32), ("accumulate", C.c_int32)]

SIGNATURES = {
    "clskd_last_error": (C.c_char_p, []),
    "clskd_conv_last_kernel": (C.c_char_p, []),
    "clskd_conv_last_kernel_fn": (_p, []),
    "clskd_conv_last_stream_k": (_i32, []),
    "clskd_exec_launch_ahead": (_i32, [_p, _p, C.c_uint32, _p]),
    "clskd_stream_prepare": (_i32, [_p]),
    "clskd_capture_scope_begin": (_i32, [_p, _i32, _p]),
    "clskd_exec_census": (_i32, [_p, _p, _i32, _p, _p, _p]),
    "clskd_kernel_name": (_i32, [_p, _p, _i32]),
    "clskd_capture_scope_end": (_i32, [_p]),
    "clskd_capture_scope_free": (_i32, [_p]),
    "clskd_version": (_i32, []),
    "clskd_set_knob": (_i32, [C.c_char_p, _i32]),
    "clskd_get_knob": (_i32, [C.c_char_p, C.POINTER(C.c_int32)]),
    "clskd_experiments_build": (_i32, []),
    "clskd_conv2d_fwd": (_i32, [C.POINTER(ConvDesc), _p]),
    "clskd_conv_fold_capable": (_i32, [C.POINTER(ConvDesc)]),
    "clskd_bn_fold_state_size": (_i64, [_i32]),
    "clskd_abf_bn1_fold": (_i32, [_p, _i32, _i32, _i32, _i64, _i64, _i64, _i32, _p, _p, _i32, _p]),
    "clskd_conv_direct_np": (_i32, [_i32]),
    "clskd_conv_direct_ok": (_i32, [_i32, _i32]),
    "clskd_bn_partial_blocks": (_i32, [_i64, _i32]),
    "clskd_bn_stats_partial": (_i32, [_p, _i64, _i32, _p, _i32, _i32, _p]),
    "clskd_bn_compact": (_i32, [_p, _i32, _i32, _i32, _p, _p]),
    "clskd_bn_finalize": (_i32, [_p, _i32, _i64, _i32, _p, _p, _f32, _p, _p, _f32, _i32, _p, _p,
                                 _p, _p, _p]),
    "clskd_bn_eval_coeffs": (_i32, [_p, _p, _p, _p, _f32, _i32, _p, _p, _p]),
    "clskd_bn_apply": (_i32, [_p, _p, _i64, _i32, _p, _p, _p, _i32, _p]),
    "clskd_bn_apply_reim": (_i32, [_p, _p, _i64, _i32, _p, _p, _p, _i32, _p]),
    "clskd_mask_bdt": (_i32, [_p, _i32, _p, _i32, _i32, _i32, _p, _i32, _p]),
    "clskd_lstm_recurrent": (_i32, [_p, _i64, _i64, _i64, _p, _i32, _i32, _i32, _i32, _p, _i64,
                                    _i64, _i64, _p]),
    "clskd_lstm_recurrent_pre": (_i32, [_p, _i64, _i64, _i64, _p, _i32, _i32, _i32, _i32, _p, _i64,
                                        _i64, _i64, _p, _p]),
    "clskd_lstm_pre_capable": (_i32, [_i32]),
    "clskd_complex_combine": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _p]),
    "clskd_complex_combine_dt": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i32, _p]),
    "clskd_lstm_cell": (_i32, [_p, _i64, _i64, _p, _i32, _i32, _i32, _p, _p, _i64, _i64, _p, _i64,
                               _i64, _p]),
    "clskd_frame_pad": (_i32, [_p, _i64, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "clskd_spec_bftc": (_i32, [_p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "clskd_mask_e": (_i32, [_p, _i32, _p, _i32, _i32, _i32, _p, _i32, _p, _p, _p]),
    "clskd_ola": (_i32, [_p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "clskd_abf_fuse": (_i32, [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _p, _i32,
                              _p]),
    "clskd_abf_moment_blocks": (_i32, [_i64, _i32]),
    "clskd_abf_bn1_partials": (_i32, [_p, _i32, _i32, _i32, _i64, _i64, _i64, _i32, _p, _p, _i32,
                                      _p]),
    "clskd_abf_conv1_fuse": (_i32, [_p, _i32, _i32, _i32, _i64, _i64, _i64, _i32, _p, _p, _p, _p,
                                    _i32, _i32, _p, _p, _p, _p, _i32, _p]),
    "clskd_sisdr_f64": (_i32, [_p, _p, _i32, _i32, _i64, _i64, _p, _p]),
    "clskd_stoi_workspace": (_i64, [_i32, _i32, _i32]),
    "clskd_stoi": (_i32, [_p, _p, _i32, _i32, _i64, _i64, _i32, _p, _i64, _p, _p]),
    "clskd_gram_partial": (_i32, [_p, _i32, _i32, _p, _p]),
    "clskd_spkd_finalize": (_i32, [_p, _i32, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p]),
    "clskd_uniform_redraw": (_i32, [_p, _i32, C.c_uint64, _p, _p]),
    "clskd_spkd_finalize_ranges": (_i32, [C.POINTER(C.c_void_p), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_int32), _i32, _i32,
                                          _i32, _p, _p, _p, _p]),
    "clskd_stft_mag_loss": (_i32, [_p, _p, _i64, _i32, _i32, _p, _p]),
    "clskd_stft_loss_finalize": (_i32, [_p, _i64, _f32, _f32, _i32, _p, _p]),
    "clskd_sisnr_rows": (_i32, [_p, _p, _i32, _i32, _i64, _i64, _f32, _p, _p]),
    "clskd_sum_f32": (_i32, [_p, _i32, _f32, _p, _p]),
    "clskd_zero_f64": (_i32, [_p, _i64, _p]),
    # backward (training step)
    "clskd_conv2d_wgrad_workspace": (_i64, [C.POINTER(ConvDesc)]),
    "clskd_conv2d_wgrad": (_i32, [C.POINTER(ConvDesc), _p, _p, _p, _p, _i64, _i32, _p]),
    "clskd_index_gather": (_i32, [_p, _p, _p, _i32, _i64, _p, _i32, _p]),
    "clskd_index_gather_jobs": (_i32, [_p, _i32, _p]),
    "clskd_adam_step": (_i32, [_p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _i32, _f32, _p]),
    "clskd_adam_step_dev": (_i32, [_p, _p, _p, _p, _i64, _f32, _f32, _f32, _f32, _f32, _p, _f32, _p]),
    "clskd_fill_f32": (_i32, [_p, _i64, _f32, _p]),
    "clskd_axpy_f32": (_i32, [_p, _p, _i64, _f32, _i32, _p]),
    "clskd_bn_bwd_blocks": (_i32, [_i64, _i32]),
    "clskd_bn_bwd_workspace": (_i64, [_i32, _i32]),
    "clskd_bn_bwd": (_i32, [_p, _p, _i64, _i32, _p, _p, _p, _p, _f32, _p, _p, _p, _i32, _p, _p,
                            _p, _p, _i32, _i32, _i32, _p]),
    "clskd_abf_fuse_bwd_blocks": (_i32, [_i32, _i32, _i32]),
    "clskd_abf_fuse_bwd": (_i32, [_p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p,
                                  _p, _p, _i32, _i32, _p, _p, _f32, _p, _i32, _i32, _p]),
    "clskd_bn_bwd_from_partials": (_i32, [_p, _p, _i64, _i32, _p, _p, _p, _p, _f32, _p, _p, _i32,
                                          _p, _p, _p, _p, _i32, _i32, _i32, _p]),
    "clskd_nearest_down_sum": (_i32, [_p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32,
                                      _p]),
    "clskd_bn_bwd_conv1x1": (_i32, [_p, _i32, _p, _i32, _i64, _i32, _p, _p, _i32, _p, _i32, _p]),
    "clskd_split_planes": (_i32, [_p, _i64, _i32, _p, _p]),
    "clskd_pack_split3": (_i32, [_p, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "clskd_mask_e_bwd": (_i32, [_p, _i32, _p, _i32, _i32, _i32, _p, _i32, _p, _p]),
    "clskd_ola_bwd": (_i32, [_p, _p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p]),
    "clskd_frame_pad_bwd": (_i32, [_p, _i32, _i32, _i32, _i32, _i32, _p, _i64, _i32, _p]),
    "clskd_stft_mag_loss_bwd": (_i32, [_p, _p, _i64, _i32, _i32, _f32, _p, _i32, _p]),
    "clskd_complex_combine_bwd": (_i32, [_p, _p, _i32, _i64, _p, _p]),
    "clskd_lstm_bwd": (_i32, [_p, _i64, _i64, _i64, _p, _i64, _i64, _i64, _p, _i32, _i32, _i32,
                              _i32, _p, _i32, _p, _i64, _i64, _i64, _p]),
    "clskd_spkd_grad_ranges": (_i32, [C.POINTER(C.c_void_p), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_int32), _i32, _i32,
                                      _i32, _f32, _p, _p]),
    "clskd_gram_bwd": (_i32, [_p, _i32, _i32, _p]),
    "clskd_exec_create": (_i32, [_p, _i32, C.POINTER(C.c_void_p), _i32, C.POINTER(C.c_void_p)]),
    "clskd_exec_tag": (_i32, [_p, _i32]),
    "clskd_exec_tag_reset": (None, []),
    "clskd_exec_launch": (_i32, [_p, _p]),
    "clskd_exec_info": (_i32, [_p, C.POINTER(C.c_int32), _i32]),
    "clskd_exec_dump": (_i64, [_p, C.c_char_p, _i64]),
    "clskd_exec_destroy": (None, [_p]),
    "clskd_exec_profile": (_i32, [_p, _p, _i32]),
    "clskd_exec_profile_read": (_i32, [_p, C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
    "clskd_exec_marks": (_i32, [_p, _i32]),
    "clskd_exec_marks_read": (_i32, [_p, C.POINTER(C.c_float), _i32]),
    "clskd_stream_hop": (_i32, [C.POINTER(StreamHopArgs), _p]),
    "clskd_stream_hop_marks": (_i32, [C.POINTER(C.c_int64), _i32]),
    "clskd_h32_marks": (_i32, [C.POINTER(C.c_int64), _i32]),
    "clskd_spkd_bn_bwd": (_i32, [_p, _i32, _i64, _i64, _i32, _i32, _p, _p, _p, _p, _p, _f32, _p, _p,
                                 _i32, _p, _p, _p, _i32, _p]),
}


def header_symbols():
    """Function names declared in include/clskd.h (parsed, for the export test)."""
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "clskd.h")
    src = open(hdr).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(clskd_[a-z0-9_]+)\s*\(", src)))


_LIB = None
_GPU_OK = False


def load(require_gpu=True):
    """Load the shared library.  Raises (never falls back) when missing."""
    global _LIB, _GPU_OK
    if _GPU_OK:  # launch fast path: library loaded and a HIP device already verified
        return _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libclskd_hip.so not built at {LIB_PATH}; run __graft_entry__.build()")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    if require_gpu:
        if not torch.cuda.is_available():
            raise RuntimeError("clskd: no HIP device visible; the MI355X path has no CPU fallback")
        _GPU_OK = True
    return _LIB


KNOB_EPOCH = 0


def experiments():
    """Whether the loaded library is the timing-experiments build (CLSKD_LIB=exp)."""
    return bool(load(require_gpu=False).clskd_experiments_build())


def set_knob(name, value):
    """Switch a dispatch knob of the loaded library (include/clskd.h: read from the environment
    once, then only through this call).  Returns the previous value."""
    lib = load(require_gpu=False)
    prev = C.c_int32(0)
    check(lib.clskd_get_knob(name.encode(), C.byref(prev)), f"get_knob {name}")
    check(lib.clskd_set_knob(name.encode(), int(value)), f"set_knob {name}")
    global KNOB_EPOCH
    KNOB_EPOCH += 1  # dispatch decisions cached per launch signature are re-asked
    return prev.value


_GRID_KNOB = b"CLSKD_G8_GRID"


def set_g8_grid(value):
    """conv_gemm8's persistent-grid cap (CLSKD_G8_GRID; 0 = every CU).  It changes how tiles are
    dealt to workgroups at launch, never which kernel runs or what it computes, so unlike
    set_knob it leaves the cached dispatch decisions valid.  Returns the previous value."""
    lib = load(require_gpu=False)
    prev = C.c_int32(0)
    check(lib.clskd_get_knob(_GRID_KNOB, C.byref(prev)), "get_knob CLSKD_G8_GRID")
    if prev.value != value:
        check(lib.clskd_set_knob(_GRID_KNOB, int(value)), "set_knob CLSKD_G8_GRID")
    return prev.value


# capture-time stream tagging (clskd.graph.StepExecutor): a callable run after every library
# call while a step is being captured
TAG_HOOK = None


def check(rc, what=""):
    if TAG_HOOK is not None:
        TAG_HOOK()
    if rc != 0:
        msg = _LIB.clskd_last_error().decode() if _LIB is not None else ""
        raise RuntimeError(f"clskd {what} failed ({rc}): {msg}")


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_dev = torch._C._cuda_getDevice


def stream_ptr():
    """hipStream_t (as an int) of torch's current stream on the current device."""
    return _raw_stream(_cur_dev())


def ptr(t):
    """Device address of a tensor for a c_void_p argument (None -> NULL)."""
    return t.data_ptr() if t is not None else None
