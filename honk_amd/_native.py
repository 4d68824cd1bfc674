"""ctypes binding of libhonk_hip.so (include/honk_hip.h).

The shared library is the product's compute path for GPU tensors.  It is loaded
lazily; if it is missing or fails to load, every native call raises
``RuntimeError`` -- there is no silent fallback for device tensors.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhonk_hip.so")

c_f32p = ctypes.c_void_p


class ResDesc(ctypes.Structure):
    """honk_res_desc -- mirrors the SpeechResModel config keys (utils/model.py:85-92)."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_labels", "n_maps", "n_layers", "use_dilation", "pool_h", "pool_w", "height", "width", "precision")]


PRECISIONS = {"f32": 0, "bf16": 1, "bf16x3": 2, "f16x2": 3}
PREC_AUTO = 4  # HONK_PREC_AUTO: honk_res_select_precision's "fastest mode holding 1e-4"
PRECISION_NAMES = {v: k for k, v in PRECISIONS.items()}
NUM_COUNT = 8  # HONK_NUM_COUNT
NUM_FIELDS = ("scale", "range", "w0sum", "rho", "f16_overflow", "rho_layer", "valid", "out_scale")  # HONK_NUM_*
NUM_KW = 64  # HONK_NUM_KW: the per-layer f16x2 weight exponents follow the header


class CnnDesc(ctypes.Structure):
    """honk_cnn_desc -- mirrors the SpeechModel config keys (utils/model.py:126-180)."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "height", "width", "n_labels",
        "c1_out", "c1_kh", "c1_kw", "c1_sh", "c1_sw", "p1_h", "p1_w",
        "has_conv2", "c2_out", "c2_kh", "c2_kw", "c2_sh", "c2_sw", "p2_h", "p2_w",
        "has_lin", "dnn1", "dnn2", "dnn1_relu", "precision")]


# name -> (restype, argtypes)
_PROTOS = {
    "honk_res_packed_floats": (ctypes.c_size_t, [ctypes.POINTER(ResDesc)]),
    "honk_res_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(ResDesc), ctypes.c_int64]),
    "honk_res_launch_plan": (ctypes.c_int, [ctypes.POINTER(ResDesc), ctypes.c_int64, ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    "honk_res_pack": (ctypes.c_int, [ctypes.POINTER(ResDesc), ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32,
                                     c_f32p, ctypes.c_void_p]),
    "honk_res_numerics": (ctypes.c_int, [ctypes.POINTER(ResDesc), c_f32p, ctypes.POINTER(ctypes.c_float),
                                         ctypes.c_int32, ctypes.c_void_p]),
    "honk_res_select_precision": (ctypes.c_int, [ctypes.POINTER(ResDesc), ctypes.POINTER(ctypes.c_float),
                                                 ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]),
    "honk_res_forward": (ctypes.c_int, [ctypes.POINTER(ResDesc), c_f32p, c_f32p, c_f32p, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_res_rerun_count": (ctypes.c_int64, []),
    "honk_cnn_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(CnnDesc), ctypes.c_int64]),
    "honk_cnn_forward": (ctypes.c_int, [ctypes.POINTER(CnnDesc), ctypes.POINTER(ctypes.c_void_p), c_f32p, c_f32p,
                                        ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv2d_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, c_f32p, ctypes.c_int64] + [ctypes.c_int32] * 9
                        + [ctypes.c_void_p]),
    "honk_maxpool2d_f32": (ctypes.c_int, [c_f32p, c_f32p, ctypes.c_int64] + [ctypes.c_int32] * 5
                           + [ctypes.c_void_p]),
    "honk_linear_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, c_f32p, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "honk_maxpool2d_bwd_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, ctypes.c_int64] + [ctypes.c_int32] * 5
                               + [ctypes.c_void_p]),
    "honk_conv2d_wgrad_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64] + [ctypes.c_int32] * 8),
    "honk_conv2d_wgrad_f32": (ctypes.c_int, [c_f32p] * 5 + [ctypes.c_int64] + [ctypes.c_int32] * 8
                              + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv2d_dgrad_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64] + [ctypes.c_int32] * 6),
    "honk_conv2d_dgrad_f32": (ctypes.c_int, [c_f32p] * 4 + [ctypes.c_int64] + [ctypes.c_int32] * 6
                              + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv_same_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64] + [ctypes.c_int32] * 4),
    "honk_conv_same_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_int64] + [ctypes.c_int32] * 5
                           + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv_same_wgrad_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_int64] + [ctypes.c_int32] * 4
                                 + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_sgd_step_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, ctypes.c_int64, ctypes.c_float, ctypes.c_float,
                                         ctypes.c_float, ctypes.c_float, ctypes.c_int32, ctypes.c_void_p]),
    "honk_conv3x3_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, ctypes.c_int64] + [ctypes.c_int32] * 5
                         + [ctypes.c_void_p]),
    "honk_conv3x3_check": (ctypes.c_int, [ctypes.c_int32] * 4),
    "honk_conv3x3_wgrad_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64] + [ctypes.c_int32] * 4),
    "honk_conv3x3_wgrad_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, ctypes.c_int64] + [ctypes.c_int32] * 4
                               + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_bn_train_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64]),
    "honk_bn_train_fwd_f32": (ctypes.c_int, [c_f32p] * 6 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                             ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p]),
    "honk_bn_train_bwd_f32": (ctypes.c_int, [c_f32p] * 4 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_res_tail_fwd_f32": (ctypes.c_int, [c_f32p] * 8 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                             ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p]),
    "honk_res_tail_bwd_f32": (ctypes.c_int, [c_f32p] * 7 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                             ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_bn_count_scale": (ctypes.c_int, [ctypes.c_double]),
    "honk_bn_partials_f32": (ctypes.c_int, [c_f32p, c_f32p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int64,
                                            ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p]),
    "honk_conv3x3_stats_bytes": (ctypes.c_size_t, [ctypes.c_int64] + [ctypes.c_int32] * 4),
    "honk_conv3x3_stats_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_int64] + [ctypes.c_int32] * 6
                               + [c_f32p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv3x3_tail_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_int32] * 4
                              + [c_f32p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_res_tail_fwd_s_f32": (ctypes.c_int, [c_f32p] * 6 + [ctypes.c_void_p, ctypes.c_int64]
                                + [ctypes.c_int32] * 4 + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]),
    "honk_res_tail_bwd_mask_f32": (ctypes.c_int, [c_f32p] * 4 + [ctypes.c_void_p] + [c_f32p] * 2
                                   + [ctypes.c_int64] + [ctypes.c_int32] * 4
                                   + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv3x3_bn_fold_check": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_int32] * 4),
    "honk_conv3x3_tail_bn_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_int32] * 4
                                 + [c_f32p] * 3 + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv3x3_stats_bn_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_int64] + [ctypes.c_int32] * 6
                                  + [c_f32p] * 3 + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_conv3x3_wgrad_bn_f32": (ctypes.c_int, [c_f32p, c_f32p, c_f32p, ctypes.c_int64] + [ctypes.c_int32] * 4
                                  + [c_f32p] * 2 + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_res_tail_bwd_mask_bn_f32": (ctypes.c_int, [c_f32p] * 5 + [ctypes.c_void_p] + [c_f32p] * 2
                                      + [ctypes.c_int64] + [ctypes.c_int32] * 4
                                      + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_res_tail_fwd_part_f32": (ctypes.c_int, [c_f32p] * 8 + [ctypes.c_void_p, ctypes.c_int64]
                                   + [ctypes.c_int32] * 4 + [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]),
    "honk_res_tail_bwd_part_f32": (ctypes.c_int, [c_f32p] * 7 + [ctypes.c_void_p, ctypes.c_int64]
                                   + [ctypes.c_int32] * 4 + [ctypes.c_void_p]),
    "honk_res_stem_fwd_f32": (ctypes.c_int, [c_f32p] * 3 + [ctypes.c_int64] + [ctypes.c_int32] * 5
                              + [ctypes.c_void_p]),
    "honk_res_stem_wgrad_workspace_bytes": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int32]),
    "honk_res_stem_wgrad_f32": (ctypes.c_int, [c_f32p] * 4 + [ctypes.c_int64] + [ctypes.c_int32] * 5
                                + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "honk_mfcc_f32": (ctypes.c_int, [c_f32p, ctypes.c_int64, ctypes.c_int32, c_f32p, ctypes.c_int32, ctypes.c_int32,
                                     c_f32p, ctypes.c_int32, c_f32p, ctypes.c_int32, c_f32p, ctypes.c_void_p]),
    "honk_spatial_mean_f32": (ctypes.c_int, [c_f32p, c_f32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]),
    "honk_spatial_mean_bwd_f32": (ctypes.c_int, [c_f32p, c_f32p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]),
    "honk_cross_entropy_f32": (ctypes.c_int, [c_f32p, ctypes.c_void_p, c_f32p, ctypes.c_int64, ctypes.c_int32,
                                              ctypes.c_void_p]),
    "honk_cross_entropy_bwd_f32": (ctypes.c_int, [c_f32p, ctypes.c_void_p, c_f32p, c_f32p, ctypes.c_int64,
                                                  ctypes.c_int32, ctypes.c_void_p]),
    "honk_augment_f32": (ctypes.c_int, [c_f32p, c_f32p] + [ctypes.c_void_p] * 2 + [c_f32p, ctypes.c_void_p, c_f32p,
                                                                                    ctypes.c_int64, ctypes.c_int32,
                                                                                    ctypes.c_int64, ctypes.c_void_p]),
    "honk_last_error": (ctypes.c_char_p, []),
    "honk_version": (ctypes.c_char_p, []),
    "honk_timing_enable": (ctypes.c_int, [ctypes.c_int32]),
    "honk_timing_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.POINTER(ctypes.c_double)]),
}

EXPORTS = tuple(_PROTOS)

_lib = None
_lock = threading.Lock()


def load(path: str = None):
    """Load (once) and return the ctypes library; raise RuntimeError if unavailable.
    ``HONK_LIB`` names an alternative build of the library (experiment builds)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("HONK_LIB") or LIB_PATH
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"honk_amd: HIP extension not built ({path} missing); run `python -m honk_amd.build`")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on ROCm install
            raise RuntimeError(f"honk_amd: cannot load {path}: {e}") from e
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().honk_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def version() -> str:
    return load().honk_version().decode()


def ptr(t) -> int:
    return t.data_ptr() if t is not None else 0


def ptr_array(tensors):
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = ptr(t) if t is not None else None
    return arr


def stream_handle(device) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def timing_enable(on: bool):
    check(load().honk_timing_enable(1 if on else 0), "honk_timing_enable")


def timing_read():
    ms = ctypes.c_double()
    n = ctypes.c_int64()
    fl = ctypes.c_double()
    check(load().honk_timing_read(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)), "honk_timing_read")
    return ms.value, n.value, fl.value


# HONK_KERNEL_* of include/honk_hip.h
KERNEL_NAMES = {1: "block_kernel", 2: "block16r_kernel", 3: "block16w_kernel", 4: "block16p_kernel",
                5: "block16l_kernel", 6: "block16n_kernel", 7: "block16k_kernel"}


def res_launch_plan(desc, batch: int, n_cus: int = 0):
    """The block-layer launches honk_res_forward makes per batch chunk, as kernel
    names (HONK_KERNEL_* codes mapped through KERNEL_NAMES).  Host-only."""
    lib = load()
    kinds = (ctypes.c_int32 * 256)()
    n = lib.honk_res_launch_plan(ctypes.byref(desc), int(batch), int(n_cus), kinds, 256)
    if n < 0:
        check(n, "honk_res_launch_plan")
    return [KERNEL_NAMES[kinds[i]] for i in range(min(n, 256))]


def res_numerics(desc, packed, device):
    """The pack-time numerics record of a packed res model (HONK_NUM_*) as a dict;
    synchronises the device's current stream (once per pack)."""
    n = NUM_KW + desc.n_layers
    rec = (ctypes.c_float * n)()
    check(load().honk_res_numerics(ctypes.byref(desc), packed.data_ptr(), rec, n, stream_handle(device)),
          "honk_res_numerics")
    out = {k: float(rec[i]) for i, k in enumerate(NUM_FIELDS)}
    out["kw"] = [int(rec[NUM_KW + i]) for i in range(desc.n_layers)]
    return out, rec


def res_select_precision(desc, rec, requested: str):
    """honk_res_select_precision: (precision name to run, note on why the request was
    not taken or "")."""
    note = ctypes.create_string_buffer(512)
    req = PREC_AUTO if requested == "auto" else PRECISIONS[requested]
    p = load().honk_res_select_precision(ctypes.byref(desc), rec, req, note, len(note))
    if p < 0:
        check(p, "honk_res_select_precision")
    return PRECISION_NAMES[p], note.value.decode(errors="replace")
