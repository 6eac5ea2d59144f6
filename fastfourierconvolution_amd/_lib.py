"""ctypes binding of the C ABI in include/ffc_amd.h (libffc_amd.so, built in-tree for gfx950).

There is deliberately no fallback: if the library is missing or no HIP device is
present, every op raises.  The product path never computes on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libffc_amd.so")

c_int, c_float, c_void_p, c_longlong, c_size_t, c_double = (
    ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_size_t, ctypes.c_double)

MAX_SEG = 3
MAX_PHASE = 16
CONVP_EXACT_F32 = 8   # include/ffc_amd.h FFC_CONVP_EXACT_F32 (ffc_convp_forward cfg flag)

ACT = {"Identity": 0, "ReLU": 1, "LeakyReLU": 2, "Tanh": 3, "Sigmoid": 4, "GELU": 5}


class ConvSeg(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("gate", c_void_p), ("C", c_int), ("IH", c_int), ("IW", c_int),
                ("mult_y", c_int), ("mult_x", c_int), ("pool", c_int), ("pad_", c_int)]


class ConvPhase(ctypes.Structure):
    _fields_ = [("py", c_int), ("px", c_int), ("PH", c_int), ("PW", c_int), ("K", c_int), ("Kpad", c_int),
                ("a_off", c_longlong), ("kt_off", c_int), ("pad_", c_int)]


class ConvJob(ctypes.Structure):
    _fields_ = [("seg", ConvSeg * MAX_SEG), ("ph", ConvPhase * MAX_PHASE),
                ("A", c_void_p), ("ktab", c_void_p), ("out", c_void_p), ("bias", c_void_p),
                ("addend", c_void_p), ("stats", c_void_p),
                ("nseg", c_int), ("nphase", c_int), ("B", c_int), ("M", c_int), ("Mpad", c_int),
                ("OH", c_int), ("OW", c_int), ("Sy", c_int), ("Sx", c_int),
                ("act", c_int), ("act_param", c_float), ("pad_", c_int)]


class ConvPSeg(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("gate", c_void_p), ("C", c_int), ("Cpad", c_int), ("IH", c_int), ("IW", c_int),
                ("mult_y", c_int), ("mult_x", c_int), ("org_y", c_int), ("org_x", c_int), ("PR", c_int),
                ("PC", c_int), ("pool", c_int), ("vec4", c_int), ("cc", c_int), ("direct", c_int),
                ("qrow", c_int), ("qsample", c_int)]


class ConvPPhase(ctypes.Structure):
    _fields_ = [("py", c_int), ("px", c_int), ("PH", c_int), ("PW", c_int), ("Kpad", c_int),
                ("T", c_int * MAX_SEG), ("kseg", c_int * MAX_SEG), ("tap", (c_int * 8) * MAX_SEG),
                ("tap_h", c_int * MAX_SEG),
                ("a_off", c_longlong)]


class ConvPJob(ctypes.Structure):
    _fields_ = [("seg", ConvPSeg * MAX_SEG), ("ph", ConvPPhase * 4),
                ("A", c_void_p), ("out", c_void_p), ("bias", c_void_p),
                ("addend", c_void_p), ("stats", c_void_p),
                ("nseg", c_int), ("nphase", c_int), ("B", c_int), ("M", c_int), ("Mpad", c_int),
                ("OH", c_int), ("OW", c_int), ("Sy", c_int), ("Sx", c_int),
                ("NS", c_int), ("TR", c_int), ("TC", c_int), ("nrb", c_int), ("ncb", c_int),
                ("act", c_int), ("act_param", c_float), ("A3", c_void_p), ("a3_stride", ctypes.c_longlong)]


class BnFold(ctypes.Structure):
    """ffc_bn_fold: a train-mode BatchNorm finalized inside its consumer kernel"""
    _fields_ = [("slab", c_void_p), ("nrows", c_int), ("C", c_int), ("gamma", c_void_p), ("beta", c_void_p),
                ("running_mean", c_void_p), ("running_var", c_void_p), ("num_batches_tracked", c_void_p),
                ("update_running", c_int), ("momentum", c_float), ("eps", c_float), ("count_mult", c_float),
                ("scale_out", c_void_p), ("shift_out", c_void_p), ("moments", c_void_p)]


class InTf(ctypes.Structure):
    """ffc_in_tf: a producer's BN + activation (+ NoiseInjection) applied by the consuming conv"""
    _fields_ = [("scale", c_void_p), ("shift", c_void_p), ("act", c_int), ("act_param", c_float),
                ("noise_w", c_void_p), ("noise", c_void_p)]


class BnRfItem(ctypes.Structure):
    """ffc_bn_rf_item: one BN of ffc_bn_reduce_finalize_batch"""
    _fields_ = [("slab", c_void_p), ("nrows", c_int), ("C", c_int), ("moments", c_void_p), ("gamma", c_void_p),
                ("beta", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p),
                ("num_batches_tracked", c_void_p), ("update_running", c_int), ("momentum", c_float), ("eps", c_float),
                ("count_mult", c_float), ("scale", c_void_p), ("shift", c_void_p)]


class BnApplyItem(ctypes.Structure):
    """ffc_bn_apply_item: one tensor of ffc_bn_act_apply_batch"""
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("B", c_int), ("C", c_int), ("HW", c_int), ("scale", c_void_p),
                ("shift", c_void_p), ("act", c_int), ("act_param", c_float), ("noise_w", c_void_p), ("noise", c_void_p),
                ("plane_sum", c_void_p)]


# (name, restype, argtypes) for every entry point declared in include/ffc_amd.h
SIGNATURES = [
    ("ffc_last_error", ctypes.c_char_p, []),
    ("ffc_abi_version", c_int, []),
    ("ffc_struct_sizes", c_int, [ctypes.POINTER(c_int), c_int]),
    ("ffc_conv_forward", c_int, [ctypes.POINTER(ConvJob), c_int, c_void_p, c_int, c_int, c_void_p]),
    ("ffc_conv_stat_rows_per_tile", c_int, [c_int]),
    ("ffc_convp_forward", c_int, [ctypes.POINTER(ConvPJob), c_int, c_void_p, c_int, c_int, c_void_p]),
    ("ffc_convq_config", c_int, [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    ("ffc_convq_pack_a3", c_int, [ctypes.POINTER(ConvPJob), c_void_p, c_void_p, c_void_p]),
    ("ffc_convq_forward", c_int, [ctypes.POINTER(ConvPJob), c_int, c_void_p, c_int, c_int, c_void_p]),
    ("ffc_convq_split_floats", ctypes.c_longlong, [c_int, c_int, c_int]),
    ("ffc_convq_forward_split", c_int, [ctypes.POINTER(ConvPJob), c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                                        c_int, c_void_p, c_void_p]),
    ("ffc_split_bf16", c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_void_p]),
    ("ffc_pw_forward", c_int, [ctypes.POINTER(ConvJob), c_int, c_void_p]),
    ("ffc_pw_tiles", c_int, [c_int, c_int, c_int, c_int]),
    ("ffc_conv_pack", c_int, [ctypes.POINTER(ConvJob), ctypes.POINTER(c_void_p), ctypes.POINTER(c_int),
                              ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_void_p),
                              c_void_p, c_void_p, c_void_p]),
    ("ffc_bn_reduce_ws_doubles", c_size_t, [c_int, c_int]),
    ("ffc_bn_reduce_finalize_batch", c_int, [ctypes.POINTER(BnRfItem), c_int, c_void_p]),
    ("ffc_bn_act_apply_batch", c_int, [ctypes.POINTER(BnApplyItem), c_int, c_void_p]),
    ("ffc_plane_chunks", c_int, [c_int]),
    ("ffc_se_gate_sums", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_bn_reduce", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("ffc_bn_finalize", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                c_float, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    ("ffc_bn_reduce_finalize", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    ("ffc_bn_act_apply", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_float,
                                 c_void_p]),
    ("ffc_bn_act_noise_apply", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_float,
                                       c_void_p, c_void_p, c_void_p]),
    ("ffc_se_gate", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                            c_void_p]),
    ("ffc_fu_forward", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                               c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_fu_forward_ex", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                  c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, ctypes.POINTER(BnFold),
                                  ctypes.POINTER(BnFold), c_void_p, c_void_p]),
    ("ffc_fu_forward_ex3", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                   c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                   ctypes.POINTER(BnFold), ctypes.POINTER(BnFold), c_void_p, c_void_p]),
    ("ffc_fu_forward_ex4", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                   c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                   ctypes.POINTER(BnFold), ctypes.POINTER(BnFold), c_void_p, c_int, c_void_p]),
    ("ffc_fu_kgroups", c_int, [c_int, c_int, c_int, c_int]),
    ("ffc_fu_slab_rows", c_int, [c_int, c_int, c_int, c_int, c_int]),
    ("ffc_fu_mix3_elems", c_size_t, [c_int]),
    ("ffc_fu_pack_mix3", c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_fu_pack_mix", c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_pack_transpose", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("ffc_fu_lds_bytes", c_size_t, [c_int, c_int, c_int]),
    ("ffc_st_prologue_lds_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    ("ffc_st_prologue", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ffc_st_prologue_split", c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    ("ffc_st_prologue_ex", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                   c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ffc_st_pack_a3_elems", c_size_t, [c_int, c_int]),
    ("ffc_st_pack_a3", c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("ffc_st_prologue_ex3", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                    c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ffc_fu2d_supported", c_int, [c_int, c_int, c_int, c_int]),
    ("ffc_fu2d_slab_rows", c_int, [c_int, c_int, c_int, c_int]),
    ("ffc_fu2d_r2c", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_fu2d_mix", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p]),
    ("ffc_fu_pack_mix_f16", c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_fu2d_mix_f16", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p]),
    ("ffc_fu2d_cols_supported", c_int, [c_int, c_int, c_int, c_int, c_int]),
    ("ffc_fu2d_mix_cols", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
    ("ffc_fu2d_c2r_rows", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                  c_int, c_void_p, c_void_p]),
    ("ffc_fu2d_c2r", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                             c_int, c_void_p, c_void_p]),
    ("ffc_fu2d_c2r_bn", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ffc_fu2d_r2c_ex", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                ctypes.POINTER(BnFold), c_void_p, c_void_p]),
    ("ffc_fu2d_c2r_fold", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                  c_int, ctypes.POINTER(BnFold), c_void_p, c_void_p]),
    ("ffc_fu2d_r2c_mix_supported", c_int, [c_int, c_int, c_int, c_int]),
    ("ffc_fu2d_r2c_mix", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                 ctypes.POINTER(BnFold), c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ffc_noise_inject", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    ("ffc_noise_wgrad", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("ffc_quantize_u8", c_int, [c_void_p, c_void_p, c_longlong, c_void_p]),
    ("ffc_conv3x3_smallm", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                                   c_int, c_int, c_void_p, c_int, c_float, c_void_p]),
    ("ffc_conv3x3_smallm_tf", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                                      c_int, c_int, c_void_p, c_int, c_float, ctypes.POINTER(InTf),
                                      ctypes.POINTER(InTf), c_void_p]),
    ("ffc_pw_gate_blocks", c_int, [c_int]),
    ("ffc_pw_gate_lds_bytes", c_size_t, [c_int, c_int]),
    ("ffc_pw_gate_conv", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p]),
    ("ffc_dense_forward", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                  c_int, c_float, c_void_p]),
    ("ffc_convt_smallm_pack_floats", c_size_t, [c_int, c_int]),
    ("ffc_convt_smallm_pack", c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    ("ffc_convt_k4s2_smallm", c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                                      c_int, c_int, c_void_p, c_int, c_float, c_void_p]),
    ("ffc_act_bwd", c_int, [c_void_p, c_void_p, c_void_p, c_longlong, c_int, c_float, c_void_p]),
    ("ffc_reduce_splits", c_int, [c_int, c_int, c_int]),
    ("ffc_channel_moments", c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_bn_bwd_sums", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_float,
                                c_void_p, c_int, c_void_p, c_void_p]),
    ("ffc_bn_bwd_coeff", c_int, [c_void_p, c_int, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p]),
    ("ffc_bn_bwd_apply", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_float,
                                 c_void_p, c_void_p, c_void_p]),
    ("ffc_bn_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_float, c_void_p,
                           c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p]),
    ("ffc_conv_wgrad_tile", c_int, [c_int, c_int]),
    ("ffc_conv_wgrad", c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    ("ffc_rfft2_planes", c_int, [c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p]),
    ("ffc_irfft2_planes", c_int, [c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p]),
    ("ffc_se_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("ffc_conv_full_smallm", c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int,
                                     c_void_p, c_int, c_float, c_void_p]),
    ("ffc_pool2", c_int, [c_void_p, c_longlong, c_int, c_int, c_float, c_void_p, c_void_p]),
    ("ffc_up2", c_int, [c_void_p, c_longlong, c_int, c_int, c_float, c_void_p, c_void_p]),
]

_lock = threading.Lock()
_lib = None


class FFCError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libffc_amd.so (no GPU needed).  Raises if it is missing.  FFC_LIB_PATH overrides the
    in-tree library (A/B benchmarking of kernel variants)."""
    global _lib
    path = path or os.environ.get("FFC_LIB_PATH") or LIB_PATH
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise FFCError(f"{path} not found: build it with `python -m fastfourierconvolution_amd.build` "
                           "(the HIP path has no CPU fallback)")
        lib = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        sizes = (c_int * 10)()
        lib.ffc_struct_sizes(sizes, 10)
        want = (ctypes.sizeof(ConvSeg), ctypes.sizeof(ConvPhase), ctypes.sizeof(ConvJob),
                ctypes.sizeof(ConvPSeg), ctypes.sizeof(ConvPPhase), ctypes.sizeof(ConvPJob), ctypes.sizeof(BnFold),
                ctypes.sizeof(InTf), ctypes.sizeof(BnRfItem), ctypes.sizeof(BnApplyItem))
        if tuple(sizes) != want:
            raise FFCError(f"ABI struct layout mismatch: library {tuple(sizes)} vs binding {want}")
        _lib = lib
        return lib


def check(status: int, what: str = ""):
    if status != 0:
        msg = load().ffc_last_error().decode(errors="replace")
        raise FFCError(f"{what or 'ffc'} failed ({status}): {msg}")


def ptr(t) -> int | None:
    """device pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()
