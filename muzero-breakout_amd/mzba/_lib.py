"""ctypes binding of the C-ABI library `libmzba.so` (include/mzba.h).

The library is the only compute path: if it is missing or a GPU is absent, the
product raises — there is no CPU fallback. torch is imported first so that the
process's HIP runtime (torch's libamdhip64.so.7) is the one the library binds to;
every launch goes to torch's current HIP stream (graph-capturable).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MZBA_LIB", os.path.join(_HERE, "libmzba.so"))

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
U64 = ctypes.c_uint64
F = ctypes.c_float
D = ctypes.c_double

# name -> argtypes (all return int: 0 ok, <0 bad argument, >0 hipError_t)
SIGNATURES = {
    "mzba_env_reset_planes": [P, P, P, I, I, I, I, I, U64, I, I, P, P],
    "mzba_env_step_planes": [P, P, P, P, P, P, P, P, I, I, I, I, P, P, P],
    "mzba_grayscale_planes": [P, P, I, I, I, P],
    "mzba_env_reset_compact": [P, P, P, P, P, P, P, I, P, P, P, P, P, I, I, I, I, I, I, U64, I, I, P, I, P],
    "mzba_env_step_compact": [P, P, P, P, P, P, P, I, P, P, P, P, P, P, P, P, I, P, P, P, P, I, I, I, I, I, I, P, P, I, P],
    "mzba_compact_to_planes": [P, P, P, P, P, I, P, I, I, I, I, I, P],
    "mzba_build_rep_input": [P, P, P, P, P, I, P, I, I, I, I, P],
    "mzba_env_current_frame": [P, P, P, P, I, P, I, I, P],
    "mzba_env_set_block_envs": [I],
    "mzba_conv2d": [I, P, LL, P, LL, P, P, P, P, I, P, P, I, I, I, I, I, I, I, P],
    "mzba_conv2d_set_variant": [I],
    "mzba_conv_halo_supported": [I, I, I, I, I],
    "mzba_conv_halo": [P, P, P, P, P, I, I, I, I, I, I, P],
    "mzba_conv_halo_ex_supported": [I, I, I, I, I, I],
    "mzba_conv_halo_ex": [P, LL, P, LL, P, P, P, P, I, P, P, I, I, I, I, I, I, P],
    "mzba_conv_x6_supported": [I, I, I, I, I],
    "mzba_conv_x6": [P, P, P, P, P, I, I, I, I, I, I, P],
    "mzba_conv_x6_ex_supported": [I, I, I, I, I, I],
    "mzba_conv_x6_ex": [P, LL, P, LL, P, P, P, P, I, P, P, I, I, I, I, I, I, I, P],
    "mzba_conv_x3_supported": [I, I, I, I, I, I],
    "mzba_conv_x3_ex": [P, LL, P, LL, P, P, P, P, P, I, P, P, I, I, I, I, I, I, I, P],
    "mzba_conv_x3_set_pipe": [I],
    "mzba_conv_x6_set_variant": [I],
    "mzba_conv_x6_set_waves": [I],
    "mzba_conv_lat_supported": [I, I, I, I, I],
    "mzba_conv_lat_set_variant": [I],
    "mzba_conv_lat_get_variant": [],
    "mzba_conv_lat": [P, LL, P, LL, P, P, P, P, I, P, P, I, I, I, I, I, I, I, P],
    "mzba_tower": [P, LL, P, LL, P, P, P, I, I, P, LL, P],
    "mzba_towerp": [P, LL, P, LL, P, P, P, I, I, P],
    "mzba_towerp_fused": [P, LL, P, LL, P, P, P, I, I, P, P],
    "mzba_tower_plan": [I],
    "mzba_tower_ws_bytes": [I],
    "mzba_tower_fused": [P, LL, P, LL, P, P, P, I, I, P, P],
    "mzba_rep_tail": [P, P, P, LL, P, P, I, I, P],
    "mzba_rep_blocks": [P, P, P, P, I, I, P],
    "mzba_rep_trunk": [P, P, P, P, I, I, I, P],
    "mzba_conv_band_supported": [I, I, I, I, I],
    "mzba_conv_band_set_xt": [I],
    "mzba_replay_plan": [P, P, P, P, P, P, P, I, I, I, I, I, P, P, P, P],
    "mzba_replay_write": [P, P, P, P, P, P, P, I, I, I, P, P, P, I, P, P, P, P, P, P, P, P, I, I, I, I, P, P],
    "mzba_replay_states": [P, P, I, P, P, I, I, P],
    "mzba_conv_band": [P, P, P, P, P, I, I, I, I, I, I, P],
    "mzba_conv_band_res_supported": [I, I, I],
    "mzba_conv_band_res": [P, P, P, P, P, P, I, I, I, I, P],
    "mzba_tower_set_variant": [I],
    "mzba_avgpool2": [I, P, P, I, I, I, I, P],
    "mzba_scale_state": [I, P, P, P, LL, P, I, LL, I, I, P],
    "mzba_heads": [I, I, P, P, P, I, I, I, P, P, P, P, P, I, I, I, P, P, F, F, I, P],
    "mzba_support_decode": [P, P, I, I, F, F, P],
    "mzba_heads_set_variant": [I],
    "mzba_heads_bf16": [I, P, P, P, I, I, I, P, P, P, P, P, I, I, I, P, P, F, F, I, P],
    "mzba_mcts_node_bytes": [],
    "mzba_mcts_root": [P, P, P, P, P, P, P, P, P, I, I, I, I, U64, P, P, P, P, P, F, F, P, F, P],
    "mzba_mcts_select": [P, P, P, P, P, P, P, P, P, I, I, I, I, U64, P, I, P],
    "mzba_mcts_backup": [P, P, P, P, P, P, P, P, P, I, I, I, I, U64, P, I, P, P, P, F, P],
    "mzba_mcts_results": [P, P, P, P, P, P, P, P, P, I, I, I, I, U64, P, P, P, P],
    "mzba_sample_actions": [P, P, P, I, D, P, I, I, I, I, I, U64, P, P],
    "mzba_torch_pow": [P, P, LL, D, LL, LL, I, I, P],
    "mzba_record_results": [P, P, P, P, I, I, P, P],
    "mzba_ctx_advance": [P, P],
    # learner (learn.hip)
    "mzba_bn_stats": [I, P, I, I, F, F, P, P, P, P, P, P, LL, P],
    "mzba_bn_apply": [I, P, P, P, I, P, I, I, P],
    "mzba_bn_backward": [I, P, P, P, P, I, I, P, P, P, P, LL, P],
    "mzba_bn_stats_final": [P, I, I, I, I, F, F, P, P, P, P, P, P],
    "mzba_bn_backward_final": [I, P, P, P, P, I, I, I, P, P, P, P, LL, P],
    "mzba_conv_lat_bn_chunks": [I, I, I, I, I, I, P, P],
    "mzba_conv_lat_bn": [P, P, P, P, P, I, I, I, I, I, I, I, P, P, P, P, P, P, I, P, P, P],
    "mzba_conv_lat_bn_fin": [P, P, P, P, P, I, I, I, I, I, I, I, P, P, P, P, P, P, I, P, P, P, F, F, P, P, P, P, P, P,
                             P, P, P],
    "mzba_bn_backward_coef": [P, I, I, I, P, P, P, P, P],
    "mzba_bn_backward_apply": [I, P, P, P, P, P, I, I, P],
    "mzba_conv_wpack": [I, P, P, I, I, I, I, I, P],
    "mzba_conv_wgrad_ws_bytes": [I, I, I, I, I, I],
    "mzba_conv_pack_bf16": [P, P, I, I, I, I, I, I, I, LL, P],
    "mzba_conv_pack_bf16_multi": [P, P, P, I, P],
    "mzba_conv_halo_set_waves": [I],
    "mzba_conv_halo_set_form": [I],
    "mzba_conv_wgrad_set_variant": [I],
    "mzba_conv_wgrad_set_form": [I],
    "mzba_conv_wgrad": [I, P, P, I, I, I, I, I, I, P, P, P, LL, P],
    "mzba_conv_wgrad_segs": [I, P, P, I, I, I, I, I, I, I, P, P, P, LL, P],
    "mzba_avgpool2_backward": [I, P, P, I, I, I, I, P],
    "mzba_axpy": [I, P, P, LL, P],
    "mzba_scale_forward": [I, P, P, P, P, I, I, I, P],
    "mzba_scale_backward": [I, P, P, P, P, P, I, I, I, P],
    "mzba_linear_forward": [I, P, P, P, P, I, I, I, P],
    "mzba_linear_ws_bytes": [I, I, I],
    "mzba_linear_backward": [I, P, P, P, P, I, P, P, I, I, I, P, LL, P],
    "mzba_learner_loss": [P, P, P, P, P, P, P, I, I, I, I, F, F, P, P, P, P, P],
    "mzba_learner_loss_ws_bytes": [I, I],
    "mzba_learner_loss_ws": [P, P, P, P, P, P, P, I, I, I, I, F, F, P, P, P, P, P, LL, P],
    "mzba_adam": [P, P, P, P, LL, F, F, F, F, F, F, F, P],
    "mzba_adam_dev": [P, P, P, P, LL, P, P],
    "mzba_learner_input": [I, P, P, P, P, P, I, I, I, I, P],
    "mzba_dyn_input": [I, P, P, P, I, I, P, I, I, I, I, I, P],
}

_lib = None


class TreeStep(ctypes.Structure):
    """include/mzba.h mzba_tree_step (backup + next select inside the fused prediction step)."""
    _fields_ = [("nodes", P), ("root_sum", P), ("calls", P), ("leaf_parent", P), ("leaf_action", P), ("depth", P),
                ("path", P), ("sqrt_tab", P), ("c_tab", P), ("B", I), ("S", I), ("env_offset", I),
                ("search_id", I), ("seed", U64), ("ctx", P), ("sim", I), ("gamma", F), ("r", P)]


class TowerExt(ctypes.Structure):
    """include/mzba.h mzba_tower_ext (fused dynamics / prediction step around the tower)."""
    _fields_ = [("w0", P), ("b0", P), ("act_bias", P), ("act", P), ("A", I),
                ("epilogue", I),
                ("we3", P), ("be3", P), ("we1", P), ("be1", P),
                ("lw", P * 2), ("lb", P * 2), ("lO", I * 2),
                ("logits", P * 2), ("dec", P * 2),
                ("pool", P), ("pool_env_stride", LL), ("pool_slot", I),
                ("smin", F), ("smax", F), ("tree", ctypes.POINTER(TreeStep)), ("elem", I), ("plan", I)]


# entry points that return something other than a status code
RESTYPES = {"mzba_tower_ws_bytes": LL, "mzba_tower_plan": I, "mzba_conv_lat_get_variant": I, "mzba_conv_wgrad_ws_bytes": LL,
            "mzba_linear_ws_bytes": LL, "mzba_learner_loss_ws_bytes": LL}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"mzba: HIP library not built ({LIB_PATH}); run __graft_entry__.build() / make -C csrc")
        L = ctypes.CDLL(LIB_PATH)
        # A/B tooling only (an older build that predates an entry point): MZBA_LIB_PARTIAL=1 skips
        # symbols the library does not export; the product binds every declared symbol or fails
        partial = os.environ.get("MZBA_LIB_PARTIAL") == "1"
        for name, argt in SIGNATURES.items():
            if partial and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = RESTYPES.get(name, ctypes.c_int)
        _lib = L
    return _lib


OPS_PATH = os.path.join(_HERE, "libmzba_torch.so")
_ops = None


def ops():
    """torch.ops.mz: the TORCH_LIBRARY(mz) custom ops of csrc/torch_ops.cpp (libmzba_torch.so,
    linked to libmzba.so) — the drop-in classes dispatch through these."""
    global _ops
    if _ops is None:
        lib()
        if not os.path.exists(OPS_PATH):
            raise RuntimeError(f"mzba: torch op library not built ({OPS_PATH}); run __graft_entry__.build()")
        torch.ops.load_library(OPS_PATH)
        _ops = torch.ops.mz
    return _ops


TORCH_OPS = ["env_reset_", "env_step", "grayscale", "mcts_root_", "mcts_select_", "mcts_backup_", "mcts_results_",
             "sample_actions", "support_decode",
             # the nets (csrc/net_ops.cpp): reference surface + NHWC acting forms + fused tree step
             "representation", "dynamics", "prediction", "representation_", "dynamics_", "prediction_",
             "prediction_tree_"]


def exported_symbols():
    return list(SIGNATURES)


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("mzba: no HIP device visible; the MI355X path has no CPU fallback")


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")
    return rc
