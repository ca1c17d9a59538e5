"""ctypes binding of libnsm.so (the C ABI declared in include/nsm.h).

This is the ONLY way the host reaches the GPU kernels. There is no fallback:
if the shared library is missing or fails to load, importing this module
raises, and every op raises on a non-ROCm device.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NSM_LIB", os.path.join(_HERE, "libnsm.so"))

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_int64
F = ctypes.c_float
Z = ctypes.c_size_t
D = ctypes.c_double
U64 = ctypes.c_uint64

# name -> (restype, argtypes)
_SIGS = {
    "nsm_version": (I, []),
    "nsm_get_last_error": (I, [ctypes.c_char_p, Z]),
    "nsm_pack_conv_weight": (I, [P, I, I, I, I, I, I, P, P]),
    "nsm_pad_vec": (I, [P, I, I, P, P]),
    "nsm_conv_fwd": (I, [P, I, I, I, I, I, P, P, I, I, P, I, P, P, P, F, P]),
    "nsm_conv_stat_rows": (I, [I, I, I, I]),
    "nsm_conv_fwd_stats": (I, [P, I, I, I, I, I, P, P, I, I, P, I, P, P, P, F, P, P, P, P]),
    "nsm_wino_ws": (Z, [I, I, I, I, I, I]),
    "nsm_wino_weight": (I, [P, I, I, I, I, I, I, P, P]),
    "nsm_conv3x3_wino": (I, [P, I, I, I, I, I, P, P, I, I, I, P, I, P, Z, P]),
    "nsm_wino_input": (I, [P, I, I, I, I, I, I, I, P, P]),
    "nsm_wino_gemm": (I, [P, P, I, I, I, I, I, I, P, P]),
    "nsm_wino_gemm_s": (I, [P, P, I, I, I, I, I, I, P, P, P, P]),
    "nsm_absmax": (I, [P, L, P, P]),
    "nsm_zero_u32": (I, [P, L, P]),
    "nsm_absmax_bf16": (I, [P, L, P, P]),
    "nsm_pmc_calib": (I, [I, P, P, L, P]),
    "nsm_to_h2": (I, [P, L, I, P, F, P, P]),
    "nsm_wino_gemm_h2": (I, [P, P, I, I, I, I, I, I, P, P, F, P, F, P]),
    "nsm_wino_beta": (F, [I, I]),
    "nsm_wino_input_h2": (I, [P, I, I, I, I, I, I, I, I, P, P, P]),
    "nsm_wino_dual_input_h2": (I, [P, I, I, I, I, I, I, P, P, P, P]),
    "nsm_wino_dual_input_bn_h2": (I, [P, I, P, I, I, I, I, I, I, P, P, F, P, P, P, P, P, P, P]),
    "nsm_wino_input_f16": (I, [P, I, I, I, I, I, I, P, P, P]),
    "nsm_wino_input_f16_resize": (I, [P, I, I, I, I, I, I, I, I, P, P, P]),
    "nsm_wino_gemm_f16": (I, [P, P, I, I, I, I, I, I, P, P, F, P, F, P]),
    "nsm_wino_output_bf16": (I, [P, I, I, I, I, I, P, P, I, P, I, P]),
    "nsm_wino_gemm_f16m": (I, [P, P, I, I, I, I, I, I, P, P, P, F, P, F, P]),
    "nsm_wino_output_bf16m": (I, [P, P, I, I, I, I, I, I, P, F, P, F, P, P, I, P, I, P]),
    "nsm_wino_output_bf16m_act": (I, [P, P, I, I, I, I, I, I, P, F, P, F, P, P, I, P, P, F, P]),
    "nsm_wino_dout_f16": (I, [P, I, I, I, I, I, I, P, P, P]),
    "nsm_wino_dual_f16": (I, [P, I, I, I, I, I, I, P, P, P, P]),
    "nsm_wino_dual_bn_f16": (I, [P, I, P, I, I, I, I, I, I, P, P, F, P, P, P, P, P, P, P]),
    "nsm_wino_wgrad_f16_ws": (Z, [I, I, I, I, I, I]),
    "nsm_conv3x3_wgrad_wino_f16": (I, [P, P, I, I, I, I, I, I, I, I, P, P, Z, P, P, P]),
    "nsm_wino_wgrad_h2_ws": (Z, [I, I, I, I, I, I]),
    "nsm_conv3x3_wgrad_wino_h2": (I, [P, P, I, I, I, I, I, I, I, I, P, P, Z, P, P, P]),
    "nsm_set_f32_split": (I, [I]),
    "nsm_wino_output": (I, [P, I, I, I, I, I, P, P, I, P]),
    "nsm_wino_wgrad_ws": (Z, [I, I, I, I, I, I]),
    "nsm_conv3x3_wgrad_wino": (I, [P, I, P, I, I, I, I, I, I, I, I, P, P, Z, P]),
    "nsm_conv_wgrad_ws": (Z, [I, I, I, I, I, I]),
    "nsm_conv_wgrad": (I, [P, I, P, I, I, I, I, I, I, I, P, P, P, F, P, Z, I, I, P, P, P, P]),
    "nsm_reduce_chunks": (I, [I, I]),
    "nsm_reduce_rows": (I, [I, I]),
    "nsm_bn_stats": (I, [P, I, I, I, P, I, I, P]),
    "nsm_bn_finalize_train": (I, [P, I, I, I, I, I, P, P, P, P, P, F, F, I, P, P, P, P, P, F, P]),
    "nsm_bn_act_h2": (I, [P, I, I, I, P, P, F, P, I, P, P, P]),
    "nsm_conv1x1_h2_rows": (I, [I, I, I, I]),
    "nsm_conv1x1_h2": (I, [P, I, I, P, P, I, P, I, P, P, P, P]),
    "nsm_conv1x1_dgrad_bnbwd_h2": (I, [P, I, I, P, I, P, I, P, P, P, P, P, I, F, I, P, P, P, I, P,
                                       P, P, P, P]),
    "nsm_conv3x3_h2_rows": (I, [I, I]),
    "nsm_conv3x3_h2": (I, [P, I, I, I, I, P, P, I, P, I, P, P, P, P]),
    "nsm_conv3x3_wgrad_h2_ws": (Z, [I, I, I, I, I]),
    "nsm_conv3x3_wgrad_h2": (I, [P, P, I, I, I, I, I, I, I, P, P, Z, P, P, P]),
    "nsm_input_prep_h2": (I, [P, I, I, I, I, P, I, P, P]),
    "nsm_conv1x1_wgrad_h2_ws": (Z, [I, I, I]),
    "nsm_conv1x1_wgrad_h2": (I, [P, P, I, I, I, I, I, P, P, Z, P, P, P]),
    "nsm_bn_partials_merge": (I, [P, I, I, I, I, I, P, P]),
    "nsm_bn_finalize_eval": (I, [P, P, P, P, I, I, F, P, P, P, P, P]),
    "nsm_bn_act": (I, [P, I, I, I, P, P, F, P, I, P, I, P, I, I, P, P]),
    "nsm_bn_bwd_reduce": (I, [P, I, P, I, I, I, I, P, P, F, P, P, P, P, I, I, P, P]),
    "nsm_bn_bwd_finalize": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, P]),
    "nsm_bn_bwd_apply_h2": (I, [P, I, P, I, I, I, I, P, P, F, P, P, P, P, P, P]),
    "nsm_bn_bwd_apply": (I, [P, I, P, I, I, I, I, P, P, F, P, P, P, P, I, I, P, P]),
    "nsm_sum_rows": (I, [P, I, I, I, P, P]),
    "nsm_resize_fwd_act": (I, [P, I, I, I, I, P, I, I, P, P, F, P, I, P]),
    "nsm_up2_resize_fwd_act": (I, [P, I, I, I, I, P, I, I, P, P, F, P, I, P]),
    "nsm_bn_act_pool": (I, [P, I, I, I, I, P, P, F, P, P, I, P, P]),
    "nsm_wino_dual_input": (I, [P, I, I, I, I, I, I, P, P, P, P, P]),
    "nsm_wino_dual_input_bn": (I, [P, I, P, I, I, I, I, I, I, P, P, F, P, P, P, P, P, P, P, P]),
    "nsm_conv3x3_wgrad_wino_dm": (I, [P, P, I, I, I, I, I, I, I, I, P, P, Z, P, P, P]),
    "nsm_conv_fwd_act": (I, [P, I, I, I, I, I, P, P, I, I, P, I, P, P, F, P, I, I, P]),
    "nsm_wino_output_act": (I, [P, I, I, I, I, I, P, P, I, P, P, F, P, I, P]),
    "nsm_bnred_chunks": (I, [I, I, I, I, I]),
    "nsm_avgpool2_bwd_add_bnred": (I, [P, I, I, I, I, P, P, I, P, P, P, P, P, F, P, P, P]),
    "nsm_resize_bwd_bnred": (I, [P, I, I, I, I, P, I, I, I, P, P, P, P, P, F, P, P, P]),
    "nsm_up2_resize_bwd_bnred": (I, [P, I, I, I, I, P, I, I, I, P, P, P, P, P, F, P, P, P]),
    "nsm_wino_input_resize": (I, [P, I, I, I, I, I, I, I, I, I, P, P, P]),
    "nsm_wino_output_stats": (I, [P, I, I, I, I, I, P, P, I, P, I, P]),
    "nsm_wino_stat_slots": (I, [I, I, I, I, I]),
    "nsm_wino_stat_step": (I, [I, I]),
    "nsm_conv1x1_bnbwd_chunks": (I, [I, I, I, I, I, I]),
    "nsm_conv1x1_dgrad_bnbwd": (I, [P, I, I, I, I, I, P, I, P, I, P, P, P, P, P, F, I, P, P, P, I,
                                    I, P, P, P, P]),
    "nsm_avgpool2_fwd": (I, [P, I, I, I, I, P, I, P]),
    "nsm_avgpool2_bwd_add": (I, [P, I, I, I, I, P, P, I, P]),
    "nsm_resize_fwd": (I, [P, I, I, I, I, P, I, I, I, P]),
    "nsm_resize_bwd": (I, [P, I, I, I, I, P, I, I, I, P]),
    "nsm_up2_resize_fwd": (I, [P, I, I, I, I, P, I, I, I, P]),
    "nsm_up2_resize_bwd": (I, [P, I, I, I, I, P, I, I, I, P]),
    "nsm_input_prep": (I, [P, I, I, I, I, P, I, I, P, P]),
    "nsm_input_grad": (I, [P, I, I, I, I, I, P, I, P]),
    "nsm_head_fwd": (I, [P, I, I, I, I, P, P, P, I, P]),
    "nsm_head_bwd_blocks": (I, [I, I, I]),
    "nsm_head_bwd": (I, [P, P, P, I, I, I, I, P, P, P, P, P, I, P]),
    "nsm_loss_blocks": (I, [L]),
    "nsm_l1_loss_fwd": (I, [P, P, L, F, P, P, P]),
    "nsm_expdiff_mean": (I, [P, P, L, F, P, P, P]),
    "nsm_l1_loss_bwd": (I, [P, P, L, F, P, P, I, P]),
    "nsm_channel_std": (I, [P, I, I, I, I, P, P, P]),
    "nsm_perturb": (I, [P, P, P, I, I, I, I, F, P, P]),
    "nsm_sumsq": (I, [P, L, P, P, P]),
    "nsm_clip_coef": (I, [P, F, F, P, P]),
    "nsm_adamw_step": (I, [P, P, P, P, L, F, F, F, F, F, I, P, P]),
    "nsm_vgg_prep": (I, [P, P, I, I, I, F, F, P, P]),
    "nsm_npy_info": (I, [ctypes.c_char_p, P, I, P, P, P]),
    "nsm_loader_create": (P, [ctypes.c_char_p, ctypes.c_char_p, I, I, I, I, I]),
    "nsm_loader_batches": (L, [P]),
    "nsm_loader_frame_dims": (I, [P, P, P, P]),
    "nsm_loader_next": (I, [P, P, P, P]),
    "nsm_loader_destroy": (None, [P]),
    "nsm_normalize_frames": (I, [P, I, I, L, P, P, F, P]),
    "nsm_pack_conv_weight_bf16": (I, [P, I, I, I, I, I, I, P, P]),
    "nsm_conv_fwd_bf16": (I, [P, I, I, I, I, I, P, P, I, I, P, I, P, P, P, F, P, P]),
    "nsm_conv_wgrad_bf16_ws": (Z, [I, I, I, I, I, I]),
    "nsm_conv_stat_rows_bf16": (I, [I, I, I, I]),
    "nsm_conv_wgrad_bf16": (I, [P, I, P, I, I, I, I, I, I, I, P, P, P, F, P, Z, I, I, P, P]),
    # the fp16-autocast mode: the same entries on IEEE-half storage
    "nsm_pack_conv_weight_f16": (I, [P, I, I, I, I, I, I, P, P]),
    "nsm_conv_fwd_f16": (I, [P, I, I, I, I, I, P, P, I, I, P, I, P, P, P, F, P, P]),
    "nsm_conv_wgrad_f16": (I, [P, I, P, I, I, I, I, I, I, I, P, P, P, F, P, Z, I, I, P, P]),
    "nsm_maxpool2_fwd": (I, [P, I, I, I, I, P, P]),
    "nsm_tail_chunk": (L, []),
    "nsm_tail_plan": (I, [P, I, P, P, P, P, I]),
    "nsm_tail_ws_bytes": (Z, [I, I]),
    "nsm_grad_tail": (I, [P, I, P, P, P, P, P, I, F, F, F, P, U64, P, Z, P, P, P, P, P]),
    "nsm_adamw_tail": (I, [P, P, P, P, P, P, P, I, P, P, P, D, D, D, D, D, P]),
    "nsm_nchw_to_nhwc": (I, [P, I, I, I, I, P, I, I, I, P]),
    "nsm_nhwc_to_nchw": (I, [P, I, I, I, I, I, P, I, P]),
    "nsm_range_flag": (I, [P, L, F, F, P, P]),
    "nsm_dropout_masks": (I, [P, I, I, U64, P, P]),
    "nsm_dropout_masks_dev": (I, [P, I, I, P, P, P]),
    "nsm_stage_mark": (I, [I, P]),
    "nsm_prep_items": (L, [P]),
    "nsm_prep_weights": (I, [P, I, L, I, P, P, L, P, L, P]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libnsm.so not found at {LIB_PATH}: build it with `make -C pcss-unet_amd/csrc` "
            "(or __graft_entry__.build()). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class NsmError(RuntimeError):
    pass


def last_error():
    buf = ctypes.create_string_buffer(512)
    lib.nsm_get_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def call(name, *args):
    """Invoke a C-ABI entry point; raise NsmError with the library's message."""
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise NsmError(f"{name} failed (code {rc}): {last_error()}")
    return rc


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def require_gpu(t, what="tensor"):
    if not t.is_cuda:
        raise NsmError(f"{what} must be on a ROCm GPU device (got {t.device}); "
                       "the nsm_amd path has no CPU implementation")
    return t


def symbols():
    return list(_SIGS)
