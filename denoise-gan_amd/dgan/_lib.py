"""ctypes binding of libdgan.so (the C ABI declared in include/dgan.h).

The product path is this library: every op in dgan.ops goes through it and
there is no CPU fallback.  Loading fails loudly when the library is missing.
"""
import ctypes
import os

from .build import LIB_PATH

_lib = None

c_int = ctypes.c_int
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
c_int64 = ctypes.c_int64
c_uint32 = ctypes.c_uint32
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p

_P = c_void_p  # device pointer
_SIGS = {
    "dg_last_error_string": (c_char_p, []),
    "dg_version": (c_int, []),
    "dg_max_slot_floats": (c_int, []),
    "dg_build_info": (c_char_p, []),
    "dg_conv_desc_create": (c_int, [ctypes.POINTER(c_void_p)] + [c_int] * 14),
    "dg_conv_desc_destroy": (c_int, [c_void_p]),
    "dg_conv_out_shape": (c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "dg_conv_workspace_size": (c_int, [c_void_p, c_int, ctypes.POINTER(c_size_t)]),
    "dg_conv_set_math": (c_int, [c_void_p, c_int]),
    "dg_conv_get_math": (c_int, [c_void_p, ctypes.POINTER(c_int)]),
    "dg_conv_fwd": (c_int, [c_void_p, _P, c_int, _P, _P, _P, c_int, c_float, c_int, c_float, _P, c_size_t, _P]),
    "dg_conv_bwd_data": (c_int, [c_void_p, _P, c_int, _P, _P, c_int, c_float, _P, c_size_t, _P]),
    "dg_conv_bwd_filter": (c_int, [c_void_p, _P, c_int, _P, c_int, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_bn_workspace_size": (c_int, [c_int, c_int, ctypes.POINTER(c_size_t)]),
    "dg_bn_fwd_train": (c_int, [c_int, c_int, _P, c_int, _P, _P, _P, _P, _P, _P, c_float, c_float, _P, c_int, c_int,
                                c_float, c_float, c_uint32, _P, _P, c_size_t, _P]),
    "dg_bn_fwd_train_pl": (c_int, [c_int, c_int, _P, c_int, _P, _P, _P, _P, _P, _P, c_float, c_float, _P, c_int,
                                   c_int, c_float, c_float, c_uint32, _P, _P, c_int, c_int, _P, c_int, c_int, _P,
                                   c_size_t, _P]),
    "dg_bn_workspace_size_seg": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_size_t)]),
    "dg_bn_fwd_train_seg": (c_int, [c_int, c_int, c_int, _P, c_int, _P, _P, _P, _P, _P, _P, c_float, c_float, _P,
                                    c_int, c_int, c_float, c_float, c_uint32, c_uint32, _P, _P, c_int, c_int, _P,
                                    c_int, c_int, _P, c_size_t, _P]),
    "dg_bn_bwd_seg": (c_int, [c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, _P, c_int, c_float,
                              c_float, _P, c_int, _P, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_bn_fwd_infer": (c_int, [c_int, c_int, _P, c_int, _P, _P, _P, _P, c_float, _P, c_int, c_int, c_float, _P]),
    "dg_bn_bwd": (c_int, [c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, _P, c_int, c_float, c_float, _P,
                          c_int, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_bn_bwd_pl": (c_int, [c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, _P, c_int, c_float, c_float, _P,
                             c_int, _P, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_act_bwd": (c_int, [c_int, c_int, _P, c_int, _P, c_int, c_int, c_float, _P, c_int, _P]),
    "dg_p2p_loss_workspace_size": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_size_t)]),
    "dg_p2p_loss": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, c_int,
                            ctypes.POINTER(c_float), _P, _P, _P, c_int, _P, c_int, _P, _P, _P, _P, c_size_t, _P]),
    "dg_adam": (c_int, [_P, _P, _P, _P, c_int64, c_float, c_float, c_float, c_float, c_float, _P, _P]),
    "dg_counter_add": (c_int, [_P, ctypes.c_int32, _P]),
    "dg_scale_by": (c_int, [c_int64, _P, _P, _P]),
    "dg_check_finite": (c_int, [c_int64, _P, _P, _P]),
    "dg_adam_ls": (c_int, [_P, _P, _P, _P, c_int64, c_float, c_int64, c_float, c_int, c_float, c_float, c_float,
                           c_float, _P, _P, _P]),
    "dg_counter_add_ls": (c_int, [_P, ctypes.c_int32, _P, _P]),
    "dg_loss_scale_update": (c_int, [_P, c_int, c_float, _P]),
    "dg_channel_concat": (c_int, [c_int64, _P, c_int, c_int, _P, c_int, c_int, _P, c_int, _P]),
    "dg_fill": (c_int, [_P, c_int64, c_float, _P]),
    "dg_to_f16": (c_int, [c_int64, _P, _P, _P]),
    "dg_strided_copy": (c_int, [c_int64, c_int, _P, c_int, _P, c_int, _P]),
    "dg_stage_pair": (c_int, [c_int64, c_int, _P, _P, _P, c_int, _P, c_int, _P, _P, _P]),
    "dg_adam_sched": (c_int, [_P, _P, _P, _P, c_int64, c_float, c_int64, c_float, c_int, c_float, c_float, c_float,
                              c_float, _P, _P]),
    "dg_prelu_workspace_size": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_size_t)]),
    "dg_prelu_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, _P, c_int, _P, _P, c_int, _P]),
    "dg_prelu_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, _P, c_int, _P, _P, c_int, _P, c_int, c_float, _P,
                             c_float, _P, c_size_t, _P]),
    "dg_add": (c_int, [c_int64, c_int, _P, c_int, _P, c_int, _P, c_int, _P]),
    "dg_add_h": (c_int, [c_int64, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P]),
    "dg_prelu_fwd_h": (c_int, [c_int, c_int, c_int, c_int, c_int, _P, c_int, _P, _P, c_int, _P, _P]),
    "dg_prelu_bwd_h": (c_int, [c_int, c_int, c_int, c_int, c_int, _P, c_int, _P, _P, c_int, _P, c_int, _P, c_float,
                               _P, c_float, _P, c_size_t, _P]),
    "dg_bn_fwd_train_seg_h": (c_int, [c_int, c_int, c_int, _P, c_int, _P, _P, _P, _P, _P, _P, c_float, c_float, _P,
                                      c_int, c_int, c_float, c_float, c_uint32, c_uint32, _P, _P, c_int, c_int, _P,
                                      c_int, c_int, _P, c_int, _P, _P, c_size_t, _P]),
    "dg_bn_fwd_train_seg_x": (c_int, [c_int, c_int, c_int, _P, c_int, _P, _P, _P, _P, _P, _P, c_float, c_float, _P,
                                      c_int, c_int, c_float, c_float, c_uint32, c_uint32, _P, _P, c_int, c_int, _P,
                                      c_int, c_int, _P, _P, c_int, c_int, c_int, _P, _P, c_int, _P, _P, c_size_t,
                                      _P]),
    "dg_bn_bwd_seg_h": (c_int, [c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, _P, c_int, c_float,
                                c_float, _P, c_int, _P, _P, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_conv_op_arith": (c_int, [_P, c_int, _P]),
    "dg_bn_bwd_seg_x": (c_int, [c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, _P, c_int, c_float,
                                c_float, _P, c_int, _P, c_int, _P, _P, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_bn_bwd_seg_r": (c_int, [c_int, c_int, c_int, _P, c_int, _P, c_int, _P, _P, _P, _P, c_int, c_float,
                                _P, c_int, _P, c_int, _P, _P, _P, _P, c_float, _P, c_size_t, _P]),
    "dg_accumulate": (c_int, [c_int64, c_int, _P, c_int, _P, c_int, c_float, _P]),
    "dg_act_fwd": (c_int, [c_int64, c_int, _P, c_int, c_int, c_float, _P, c_int, _P]),
    "dg_maxpool2_fwd": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P]),
    "dg_maxpool2_bwd": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, c_float, c_int, c_float,
                                _P]),
    "dg_conv_bwd_data_masked": (c_int, [c_void_p, _P, c_int, _P, _P, c_int, c_float, _P, c_int, c_int, c_float, _P,
                                        c_size_t, _P]),
    "dg_maxpool2_fwd_pl": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, _P]),
    "dg_maxpool2_fwd_plf": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P]),
    "dg_maxpool2_fwd_x3": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, _P, _P, _P, _P]),
    "dg_maxpool2_bwd_pl": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, c_float, c_int,
                                   c_float, _P, _P]),
    "dg_conv_planes_size": (c_int, [c_void_p, c_int, ctypes.POINTER(c_size_t)]),
    "dg_conv_planes_format": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int)]),
    "dg_mark": (c_int, [c_int, _P]),
    "dg_conv_op_planes": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int)]),
    "dg_conv_fwd_pl": (c_int, [c_void_p, _P, c_int, _P, _P, _P, c_int, c_float, c_int, c_float, _P, _P, c_size_t,
                               _P]),
    "dg_conv_bwd_data_pl": (c_int, [c_void_p, _P, c_int, _P, _P, c_int, c_float, _P, c_int, c_int, c_float, _P, _P,
                                    c_size_t, _P]),
    "dg_conv_bwd_filter_pl": (c_int, [c_void_p, _P, c_int, _P, c_int, _P, _P, c_float, _P, _P, c_size_t, _P]),
    "dg_conv_fwd_pool_ok": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int)]),
    "dg_conv_bwd_data_xmask": (c_int, [c_void_p, _P, c_int, _P, _P, c_int, c_float, c_int, c_float, _P, _P, c_size_t,
                                       _P]),
    "dg_conv_bwd_data_masked_sum": (c_int, [c_void_p, _P, c_int, _P, _P, c_int, c_float, _P, c_int, c_int, c_float,
                                            _P, _P, c_size_t, _P]),
    "dg_conv_fwd_pool": (c_int, [c_void_p, _P, c_int, _P, _P, c_int, c_float, _P, c_int, _P, _P, _P, c_size_t, _P]),
    "dg_maxpool2_bwd_idx": (c_int, [c_int, c_int, c_int, c_int, _P, _P, c_int, _P, c_int, c_float, c_int, c_float, _P,
                                    _P]),
    "dg_maxpool2_bwd_idx_x3": (c_int, [c_int, c_int, c_int, c_int, _P, _P, c_int, _P, c_int, c_float, c_int, c_float,
                                       _P, _P, _P, _P]),
    "dg_conv_set_grad_scale": (c_int, [c_void_p, _P, _P, _P, _P, _P]),
    "dg_absmax": (c_int, [_P, ctypes.c_int64, c_int, c_int, _P, _P]),
    "dg_absmax_set": (c_int, [_P, ctypes.c_int64, c_int, c_int, _P, _P]),
    "dg_weight_bound": (c_int, [_P, ctypes.c_int64, c_int, _P, _P, _P, _P, _P]),
    "dg_weight_bound_in": (c_int, [_P, c_int, c_int, c_int, _P, _P]),
    "dg_conv_set_act_scale": (c_int, [c_void_p, _P, _P, _P, _P, _P, _P, _P]),
    "dg_upsample2_relu_fwd": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P]),
    "dg_upsample2_relu_bwd": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, c_int, c_float, _P]),
    "dg_dwconv3_workspace_size": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_size_t)]),
    "dg_dwconv3_fwd": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, _P, _P, c_int, _P]),
    "dg_dwconv3_bwd_data": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, _P, c_int, c_float, _P]),
    "dg_dwconv3_bwd_filter": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, _P, c_float, _P,
                                      c_size_t, _P]),
    "dg_vgg_preprocess_fwd": (c_int, [c_int64, _P, c_int, _P, c_int, _P]),
    "dg_vgg_preprocess_bwd": (c_int, [c_int64, _P, c_int, _P, c_int, c_float, _P]),
    "dg_mse_workspace_size": (c_int, [ctypes.POINTER(c_size_t)]),
    "dg_mse": (c_int, [c_int64, c_int, _P, c_int, _P, c_int, c_float, _P, _P, c_int, c_float, _P, c_size_t, _P]),
    "dg_gan_loss_workspace_size": (c_int, [ctypes.POINTER(c_size_t)]),
    "dg_gan_loss": (c_int, [c_int, c_int, c_int, c_int, _P, c_int, _P, c_int, _P, _P, c_int, ctypes.POINTER(c_float),
                            _P, _P, _P, c_int, _P, _P, _P, _P, c_size_t, _P]),
}

EXPORTED = tuple(_SIGS)


class DGError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DGError(f"libdgan.so not found at {LIB_PATH}: run `python __graft_entry__.py` (build) first")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().dg_last_error_string().decode()
        raise DGError(f"{what} failed (rc={rc}): {msg}")


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


def build_info():
    """dg_build_info() of the loaded library as a dict (source_sha, arch, hip)."""
    raw = lib().dg_build_info().decode()
    return dict(kv.split("=", 1) for kv in raw.split(";") if "=" in kv)
