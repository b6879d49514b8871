"""ctypes binding of libcfm.so — the C ABI declared in include/cfm.h.

The library is the product: if it is missing, or no GPU is visible, every op raises.  There
is no CPU / PyTorch fallback anywhere on the hot path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch  # noqa: F401  (load torch's libamdhip64 first: libcfm resolves to the same runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CFM_LIB") or os.path.join(_HERE, "libcfm.so")   # CFM_LIB: A/B builds only
CSRC = os.path.join(_HERE, "csrc")

F32, BF16, FP8 = 0, 1, 2
ACT_NONE, ACT_SILU = 0, 1

c_void_p, c_int, c_long, c_float, c_size_t = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_size_t
c_u64 = ctypes.c_uint64


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", c_int), ("N", c_int), ("K", c_int), ("batch", c_int),
        ("dtype_ab", c_int),
        ("A", c_void_p), ("lda", c_long), ("stride_a", c_long), ("a_kmajor", c_int),
        ("B", c_void_p), ("ldb", c_long), ("stride_b", c_long), ("b_kmajor", c_int),
        ("C", c_void_p), ("ldc", c_long), ("stride_c", c_long), ("dtype_c", c_int),
        ("alpha", c_float),
        ("bias", c_void_p),
        ("act", c_int),
        ("act_grad", c_int),
        ("pre", c_void_p), ("dtype_pre", c_int),
        ("drop_p", c_float), ("drop_seed", c_u64), ("drop_offset", c_u64),
        ("out_scale", c_float),
        ("residual", c_void_p), ("ldr", c_long), ("dtype_r", c_int),
        ("split_k", c_int),
        ("workspace", c_void_p),
        ("probe", c_void_p),
        ("a_colsum", c_void_p),
        ("rowdot_with", c_void_p), ("rowdot_out", c_void_p), ("rowdot_T", c_int),
        ("alpha_a_dev", c_void_p), ("alpha_b_dev", c_void_p),
        ("allow_overlap", c_int),
        ("mx_a", c_void_p), ("mx_b", c_void_p),
        ("mx_out", c_void_p), ("mx_out_scales", c_void_p),
    ]


class FfoldGeo(ctypes.Structure):
    """cfm_ffold_geo (include/cfm.h): the folded front-end geometry; cfm_ffold_geometry fills the derived fields."""
    _fields_ = [(n, c_int) for n in ("B", "F", "T", "C1", "C2", "D", "k1", "s1", "k2", "s2", "dtype", "hilo",
                                     "F2", "T2", "Ke", "Se", "Fp", "Cx", "Kp", "lda", "T2p", "Tslot")] + [
        ("xt_elems", c_long), ("ws_floats", c_long)]


# name -> (restype, argtypes)
_SIGS = {
    "cfm_version": (c_int, []),
    "cfm_get_last_error": (ctypes.c_char_p, []),
    "cfm_rng_bind": (c_int, [c_void_p]),
    "cfm_probe_slot": (c_int, [c_void_p, c_int, c_void_p]),
    "cfm_wallclock_khz": (c_int, []),
    "cfm_cast": (c_int, [c_void_p, c_int, c_void_p, c_int, c_long, c_void_p]),
    "cfm_cast_batch": (c_int, [c_void_p, c_int, c_long, c_int, c_int, c_void_p]),
    "cfm_cast_transpose_batch": (c_int, [c_void_p, c_int, c_long, c_int, c_int, c_void_p]),
    "cfm_specaug_apply": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_float, c_void_p]),
    "cfm_logmel_ws_bytes": (c_size_t, [c_int, c_int]),
    "cfm_logmel_fwd": (c_int, [c_void_p, c_long, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "cfm_gemm": (c_int, [ctypes.POINTER(GemmDesc), c_void_p]),
    "cfm_gemm_set_mode": (c_int, [c_int]),
    "cfm_quant_fp8": (c_int, [c_void_p, c_int, c_long, c_void_p, c_void_p, c_void_p, c_void_p]),
    "cfm_quant_fp8_ws_bytes": (c_size_t, []),
    "cfm_quant_fp8_batch_blocks": (c_long, [c_long]),
    "cfm_quant_fp8_batch": (c_int, [c_void_p, c_int, c_long, c_int, c_void_p, c_void_p]),
    "cfm_dequant_fp8": (c_int, [c_void_p, c_long, c_void_p, c_void_p, c_void_p]),
    "cfm_layernorm_fwd_mx": (c_int, [c_void_p] * 8 + [c_long, c_int, c_float, c_void_p]),
    "cfm_layernorm_fwd_mx_ex": (c_int, [c_void_p, c_int] + [c_void_p] * 7 + [c_long, c_int, c_float, c_void_p]),
    "cfm_layernorm_fwd_res": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int, c_float, c_void_p]),
    "cfm_quant_mx": (c_int, [c_void_p, c_int, c_long, c_int, c_long, c_void_p, c_void_p, c_void_p]),
    "cfm_quant_mx_batch_blocks": (c_long, [c_long, c_int]),
    "cfm_quant_mx_batch": (c_int, [c_void_p, c_int, c_long, c_int, c_void_p]),
    "cfm_dequant_mx": (c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    "cfm_wgrad_group_task_bytes": (c_size_t, []),
    "cfm_wgrad_group_tiles": (c_long, [c_int, c_int]),
    "cfm_wgrad_group_fill": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                     c_long]),
    "cfm_wgrad_group": (c_int, [c_void_p, c_int, c_long, c_void_p]),
    "cfm_wgrad_group_probed": (c_int, [c_void_p, c_int, c_long, c_void_p, c_void_p]),
    "cfm_wgrad_group_plan": (c_long, [c_void_p, c_int, c_int, c_int, c_void_p, c_long, c_void_p]),
    "cfm_wgrad_group_ws_floats": (c_long, [c_int, c_int, c_int]),
    "cfm_wgrad_group_red_blocks": (c_long, [c_int, c_int, c_int]),
    "cfm_wgrad_group_fill_split": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                           c_int, c_int, c_void_p, c_long]),
    "cfm_wgrad_group_sched": (c_int, [c_void_p, c_int, c_void_p, c_long, c_long, c_void_p, c_void_p]),
    "cfm_colreduce_group_task_bytes": (c_size_t, []),
    "cfm_colreduce_group_blocks": (c_long, [c_long]),
    "cfm_colreduce_group_fill": (c_int, [c_void_p, c_int, c_void_p, c_int, c_long, c_long, c_void_p, c_void_p, c_int,
                                         c_int, c_int, c_long]),
    "cfm_colreduce_group": (c_int, [c_void_p, c_int, c_long, c_void_p]),
    "cfm_attn_set_mode": (c_int, [c_int]),
    "cfm_colreduce": (c_int, [c_void_p, c_int, c_long, c_long, c_void_p, c_int, c_void_p]),
    "cfm_colsum": (c_int, [c_void_p, c_int, c_long, c_int, c_long, c_void_p, c_int, c_void_p, c_void_p]),
    "cfm_layernorm_fwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                  c_long, c_int, c_float, c_void_p]),
    "cfm_layernorm_ws_bytes": (c_size_t, [c_long, c_int]),
    "cfm_layernorm_bwd": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p]),
    "cfm_layernorm_bwd_drop": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p,
                                       c_float, c_float, c_u64, c_void_p]),
    "cfm_scale_dropout": (c_int, [c_void_p, c_int, c_void_p, c_int, c_long, c_float, c_float, c_u64, c_u64,
                                  c_void_p]),
    "cfm_convmod_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "cfm_convmod_nparts": (c_long, [c_int, c_int]),
    "cfm_glu_dwconv_fwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                   c_void_p, c_void_p]),
    "cfm_bn_silu_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_int,
                                c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "cfm_bn_silu_bwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p]),
    "cfm_bn_silu_fwd_sums": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "cfm_bn_silu_fwd_apply": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p,
                                      c_long, c_void_p, c_void_p, c_void_p, c_int, c_long, c_int, c_void_p]),
    "cfm_bn_silu_bwd_sums": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int,
                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "cfm_bn_silu_bwd_apply": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_long, c_void_p, c_long, c_int, c_void_p]),
    "cfm_adafactor_table_bytes": (c_size_t, [c_int]),
    "cfm_adafactor_fill_table": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long,
                                         c_int, c_int, c_int, c_long, c_long, c_long, c_long, c_long, c_long,
                                         c_long]),
    "cfm_adafactor_colpart_tasks": (c_long, [c_int, c_int, c_int]),
    "cfm_adafactor_part_floats": (c_long, [c_int, c_int, c_int]),
    "cfm_adafactor_blocks": (c_int, [c_long]),
    "cfm_adafactor_row_tasks": (c_long, [c_int, c_int, c_int]),
    "cfm_adafactor_rowmean_tasks": (c_long, [c_int, c_int]),
    "cfm_adafactor_step": (c_int, [c_void_p, c_int, c_long, c_long, c_long, c_long, c_long, c_void_p, c_void_p,
                                   c_void_p, c_float, c_float, c_float, c_float, c_float, c_void_p]),
    "cfm_silu_bwd": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_long, c_void_p]),
    "cfm_bn_ws_bytes": (c_size_t, [c_int]),
    "cfm_bn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_int, c_void_p,
                           c_void_p, c_void_p, c_int, c_long, c_int, c_int, c_void_p, c_void_p]),
    "cfm_bn_bwd": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                           c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p]),
    "cfm_glu_dwconv_bwd_bn": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_float, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                      c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "cfm_glu_dwconv_bwd_wgrad": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "cfm_glu_dwconv_bwd": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                   c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "cfm_attn_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                             c_int, c_int, c_int, c_float, c_u64, c_void_p]),
    "cfm_attn_bwd_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "cfm_attn_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_float,
                             c_u64, c_void_p, c_void_p]),
    "cfm_attn_bwd_with_d": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_float,
                             c_u64, c_void_p, c_void_p]),
    "cfm_attn_bwd_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                c_float, c_u64, c_int, c_void_p, c_void_p]),
    "cfm_conv1_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "cfm_conv2_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_void_p]),
    "cfm_conv2_bwd_data": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                   c_void_p]),
    "cfm_conv2_bwd_data_ws_bytes": (c_size_t, [c_int, c_int]),
    "cfm_conv2_bwd_data_ws": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_void_p, c_void_p]),
    "cfm_conv2_bwd_weight": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                     c_void_p]),
    "cfm_conv2_bwd_weight_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "cfm_conv2_bwd_weight_ws": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                        c_void_p, c_void_p]),
    "cfm_ctc_ws_bytes": (c_size_t, [c_int, c_int, c_int]),
    "cfm_ctc_mean": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "cfm_ctc_bind_abort_counter": (c_int, [c_void_p]),
    "cfm_ctc_set_debug": (c_int, [c_int]),
    "cfm_ctc_loss_fwd": (c_int, [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                 c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "cfm_ctc_loss_bwd": (c_int, [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                 c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_long,
                                 c_long, c_void_p]),
    "cfm_ctc_greedy_decode": (c_int, [c_void_p, c_long, c_long, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "cfm_lstm_ws_bytes": (c_size_t, [c_int, c_int]),   # (H, ndir)
    "cfm_lstm_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                             c_void_p]),
    "cfm_lstm_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                             c_void_p]),
    "cfm_ffold_geometry": (c_int, [c_void_p]),
    "cfm_ffold_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "cfm_ffold_compose": (c_int, [c_void_p] * 11),
    "cfm_ffold_bwd_weights": (c_int, [c_void_p] * 14),
    "cfm_conv1_bwd_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "cfm_conv1_bwd_weight": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                     c_void_p, c_void_p]),
}

EXPORTED = sorted(k for k in _SIGS)

_lib = None
MISSING = []


class CfmError(RuntimeError):
    pass


def build(verbose=False):
    """Compile libcfm.so in-tree with hipcc for gfx950 (make -C csrc)."""
    jobs = str(min(16, os.cpu_count() or 4))
    r = subprocess.run(["make", "-C", CSRC, "-j", jobs], capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise CfmError("libcfm build failed:\n" + (r.stdout or "") + (r.stderr or ""))
    return LIB_PATH


def load():
    """Load libcfm.so (no GPU work); raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CfmError(f"{LIB_PATH} not found: run `python -c 'import __graft_entry__ as g; g.build()'` "
                       "(hipcc, gfx950). There is no fallback path.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            MISSING.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


# True while a device dropout step counter is bound (cfm_rng_bind with a non-NULL pointer): the compiled
# encoder route (Conformer._forward_tokens_ops) needs it for fresh masks per step
RNG_BOUND = False


def call(name, *args):
    global RNG_BOUND
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.cfm_get_last_error().decode(errors="replace")
        raise CfmError(f"{name} failed ({rc}): {msg}")
    if name == "cfm_rng_bind":
        RNG_BOUND = bool(args and args[0])
    return rc


def size_call(name, *args):
    return int(getattr(load(), name)(*args))


def ptr(t):
    """Device pointer of a tensor (or None -> NULL). Tensors must live on the GPU."""
    if t is None:
        return None
    if not t.is_cuda:
        raise CfmError("cfm ops need GPU tensors (the HIP path has no CPU fallback)")
    return t.data_ptr()


def dt(t):
    if t is None:
        return F32
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype in (torch.uint8, torch.float8_e4m3fn):
        return FP8
    raise CfmError(f"unsupported dtype {t.dtype}")


def stream():
    return torch.cuda.current_stream().cuda_stream
