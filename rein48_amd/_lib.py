"""ctypes binding of librein48.so (C-ABI in include/rein48.h).

The library is the product: gfx950 HIP kernels behind an extern "C" boundary. There is
no CPU fallback. If the shared object is missing or cannot be loaded, importing any
compute entry point raises Rein48LibraryError with the build command.

torch is imported first on purpose: the torch ROCm wheel ships its own
libamdhip64.so.7, and loading it before librein48.so makes the library bind to that same
HIP runtime (one runtime per process, so torch streams and pointers are valid here).
"""
import ctypes as C
import os
import threading

import torch  # noqa: F401  (see module docstring: HIP runtime load order)

# R48_LIB: an alternative build of the same library (experiments in tools/ only)
LIB_PATH = os.environ.get("R48_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "librein48.so")

R48_OK, R48_EINVAL, R48_EHIP, R48_ENOMEM = 0, -1, -2, -3
AUTO_RESET, RANDOM_POLICY, MERGE_REWARD = 1, 2, 4
FEAT_VALUES, FEAT_EXPONENTS = 0, 1
F32, BF16 = 0, 1
REPLAY_RING, REPLAY_FILL_DRAIN = 0, 1
DRAW_CONTRACT = 3          # R48_DRAW_CONTRACT (include/rein48.h); test_abi checks the two agree

# name -> (restype, argtypes); mirrors include/rein48.h one to one
_P, _I32, _I64, _U32, _U64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64


class BnFinishArgs(C.Structure):
    """r48_bn_finish_args (include/rein48.h): the BN finish a conv does in its last workgroup."""
    _fields_ = [("gamma", _P), ("beta", _P), ("running_mean", _P), ("running_var", _P), ("save", _P), ("coef", _P),
                ("dgamma", _P), ("dbeta", _P), ("rows", _I64), ("momentum", C.c_float), ("eps", C.c_float)]


_FIN = C.POINTER(BnFinishArgs)
SIGNATURES = {
    "r48_cnn_train_grad": (C.c_int, [_P, _I64, _I64, _P, _P, _P, _P, _P, C.c_float, _I32, _P, _P, _P, _P, _P]),
    "r48_cnn_train_grad_seg": (C.c_int, [_P, _I64, _I64, _P, _P, _P, _P, C.c_float, _I32, _P, _P, _P, _P, _P]),
    "r48_cnn_train_workspace_floats": (_I64, []),
    "r48_cnn_train_grad_floats": (_I64, []),
    "r48_resnet_q_forward": (C.c_int, [_P, _I64, _P, _P, _P, C.c_float, _U64, _I64, _U32, _P]),
    "r48_resnet_q_blob_bytes": (_I64, []),
    "r48_resnet_pack": (C.c_int, [_P, C.c_float, _P, _P]),
    "r48_struct_conv_weight": (C.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    "r48_struct_conv_weight_grad": (C.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    "r48_bn_workspace_floats": (_I64, [_I64, _I32]),
    "r48_bn_forward": (C.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _P, C.c_float, C.c_float, _I32, _P, _P, _P, _P,
                                 _P]),
    "r48_bn_forward_stats": (C.c_int, [_P, _I32, _P, _P, _I64, _I32, _P, _P, _P, _P, C.c_float, C.c_float, _I32, _P,
                                       _P, _P, _P, _P]),
    "r48_bn_backward_part": (C.c_int, [_P, _I32, _P, _P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "r48_conv3x3_bn_grad": (C.c_int, [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _FIN, _P]),
    "r48_conv3x3_stats_finish": (C.c_int, [_P, _I64, _I32, _P, _P, _P, _P, _FIN, _P]),
    "r48_bn_apply": (C.c_int, [_P, _P, _I64, _I32, _P, _I32, _P, _P, _P]),
    "r48_bn_backward_apply": (C.c_int, [_P, _P, _P, _I64, _I32, _P, _P, _P]),
    "r48_bn_backward": (C.c_int, [_P, _P, _P, _P, _I64, _I32, _P, _P, _I32, _P, _P, _P, _P, _P, _P]),
    "r48_board_onehot": (C.c_int, [_P, _I64, _I32, _P, _P]),
    "r48_board_onehot32": (C.c_int, [_P, _I64, _P, _P]),
    "r48_conv3x3": (C.c_int, [_P, _I64, _I32, _P, _P, _P, _P, _P, _P]),
    "r48_conv_stats_floats": (_I64, []),
    "r48_conv_wgrad_workspace_floats": (_I64, [_I32]),
    "r48_conv3x3_wgrad": (C.c_int, [_P, _P, _I64, _I32, _P, _P, _P]),
    "r48_q_head_forward": (C.c_int, [_P, _I64, _P, _P, _P, _P]),
    "r48_conv_pack_resnet": (C.c_int, [_P, _P, _P, _P]),
    "r48_huber_grad": (C.c_int, [_P, _P, _P, _I64, _P, _P, _P, _P]),
    "r48_adam": (C.c_int, [_P, _P, _P, _P, _I64, C.c_float, C.c_float, C.c_float, C.c_float, _I64, _P]),
    "r48_q_head_workspace_floats": (_I64, []),
    "r48_q_head_backward": (C.c_int, [_P, _P, _I64, _P, _P, _P, _P, _P]),
    "r48_egreedy_actions": (C.c_int, [_P, _I64, C.c_float, _U64, _I64, _U32, _P, _P]),
    "r48_td_target": (C.c_int, [_P, _P, _P, _P, _I64, C.c_float, _I32, _P, _P]),
    "r48_replay_create": (C.c_int, [C.POINTER(_P), C.c_int, _I64, _U32, _U64]),
    "r48_replay_destroy": (C.c_int, [_P]),
    "r48_replay_capacity": (_I64, [_P]),
    "r48_replay_get_counters": (C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_U32)]),
    "r48_replay_set_counters": (C.c_int, [_P, _I64, _I64, _U32]),
    "r48_replay_planes": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.POINTER(_P),
                                    C.POINTER(_P)]),
    "r48_replay_clear": (C.c_int, [_P]),
    "r48_replay_store": (C.c_int, [_P, _P, _P, _P, _P, _P, _I64, C.POINTER(_I64), _P]),
    "r48_replay_sample": (C.c_int, [_P, _I64, _P, _P, _P, _P, _P, _P, C.POINTER(_I64), _P]),
    "r48_replay_gather": (C.c_int, [_P, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "r48_replay_error_count": (C.c_int, [_P, C.POINTER(_U64)]),
    "r48_env_create": (C.c_int, [C.POINTER(_P), C.c_int, _I64, _U64, _I64]),
    "r48_env_destroy": (C.c_int, [_P]),
    "r48_env_bind_boards": (C.c_int, [_P, _P]),
    "r48_env_boards": (_P, [_P]),
    "r48_env_size": (_I64, [_P]),
    "r48_env_get_counters": (C.c_int, [_P, C.POINTER(_U32), C.POINTER(_U32)]),
    "r48_env_set_counters": (C.c_int, [_P, _U32, _U32]),
    "r48_env_reset": (C.c_int, [_P, _P, _P]),
    "r48_env_reset_with_draws": (C.c_int, [_P, _P, _P, _P, _P]),
    "r48_env_fill_random": (C.c_int, [_P, _U32, _P]),
    "r48_env_step": (C.c_int, [_P, _P, _U32, _P, _P, _P, _P, _P]),
    "r48_env_step_n": (C.c_int, [_P, _I32, _P, _U32, _P, _P, _P, _P, _P]),
    "r48_env_step_with_draws": (C.c_int, [_P, _P, _P, _P, _U32, _P, _P, _P, _P]),
    "r48_env_move": (C.c_int, [_P, _P, _U32, _P, _P, _P, _P]),
    "r48_env_spawn": (C.c_int, [_P, _P, _P, _P, _P, _P]),
    "r48_env_rollout": (C.c_int, [_P, _I32, _P, _P, _P]),
    "r48_env_score": (C.c_int, [_P, _P, _P]),
    "r48_env_error_count": (C.c_int, [_P, C.POINTER(_I64), _P]),
    "r48_env_clear_errors": (C.c_int, [_P, _P]),
    "r48_game_step1": (C.c_int, [_P, _I32, _P, _P]),
    "r48_game_step1_out_bytes": (C.c_int, []),
    "r48_host_alloc": (C.c_void_p, [_I64, C.POINTER(C.c_void_p)]),
    "r48_host_free": (C.c_int, [_P]),
    "r48_values_move": (C.c_int, [_P, _P, _I64, _P, _P, _P]),
    "r48_values_check": (C.c_int, [_P, _I64, _I32, _I32, _P, _P, _P]),
    "r48_values_move_grid": (C.c_int, [_P, _I64, _I32, _I32, _P, _P, _P]),
    "r48_values_check_grid": (C.c_int, [_P, _I64, _I32, _I32, _P, _P, _P]),
    "r48_board_features": (C.c_int, [_P, _I64, _I32, _I32, _P, _P]),
    "r48_sample_actions": (C.c_int, [_P, _I64, _U64, _I64, _U32, _P, _P, _P, _P]),
    "r48_discounted_returns": (C.c_int, [_P, _P, _P, _I32, _I64, C.c_float, _I32, _P, _P]),
    "r48_a3c_segment_stats": (C.c_int, [_P, _P, _P, _P, _I32, _I64, _P, _P, _P, _P]),
    "r48_a3c_row_weights": (C.c_int, [_P, _P, _P, _I32, _I64, _P, _P, _P]),
    "r48_a3c_segments": (C.c_int, [_P, _P, _P, _P, _P, _I32, _I64, C.c_float, _I32, _P, _P, _P, _P]),
    "r48_rmsprop_tf1": (C.c_int, [_P, _P, _P, _P, _I64, C.c_float, C.c_float, C.c_float, C.c_float, _P]),
    "r48_cnn_rollout": (C.c_int, [_P, _I64, _I32, _P, _P, _I32, _P, _P, _P, _P, _P, _P, _U64, _I64, _U32, _U64,
                                  _U32, _U32, _P]),
    "r48_cnn_policy_forward": (C.c_int, [_P, _I64, _P, _P, _I32, _P, _P, _P, _P, _U64, _I64, _U32, _P]),
    "r48_mlp_weight_floats": (_I32, []),
    "r48_mlp_policy_forward": (C.c_int, [_P, _I64, _P, _I32, _P, _P, _P, _U64, _I64, _U32, _P]),
    "r48_mlp_rollout": (C.c_int, [_P, _I64, _I32, _P, _I32, _P, _P, _P, _P, _P, _P, _U64, _I64, _U32, _U64, _U32,
                                  _U32, _P]),
    "r48_mlp_train_workspace_floats": (_I64, [_I64]),
    "r48_mlp_train_grad": (C.c_int, [_P, _I64, _I64, _P, _P, _P, _P, _P, C.c_float, _I32, _P, _P, _P, _P]),
    "r48_mlp_train_grad_seg": (C.c_int, [_P, _I64, _I64, _P, _P, _P, _P, C.c_float, _I32, _P, _P, _P, _P]),
    "r48_conv3x3_bn_in": (C.c_int, [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _FIN, _P]),
    "r48_bn_finish": (C.c_int, [_P, _I32, _I64, _I32, _P, _P, _P, _P, C.c_float, C.c_float, _P, _P, _P]),
    "r48_last_error": (C.c_char_p, []),
    "r48_version": (C.c_char_p, []),
}


class Rein48LibraryError(ImportError):
    """librein48.so (the HIP extension) is missing or failed to load."""


class Rein48Error(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, status, msg):
        super().__init__("rein48 error %d: %s" % (status, msg))
        self.status = status


_lib = None
_lock = threading.Lock()


def load():
    """Load librein48.so once; raise Rein48LibraryError loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise Rein48LibraryError(
                    "librein48.so not found at %s -- build it with `make` (hipcc --offload-arch=gfx950) "
                    "or `python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
            try:
                lib = C.CDLL(LIB_PATH)
            except OSError as e:
                raise Rein48LibraryError("cannot load %s: %s" % (LIB_PATH, e)) from e
            for name, (res, args) in SIGNATURES.items():
                f = getattr(lib, name)
                f.restype = res
                f.argtypes = args
            _lib = lib
    return _lib


def check(status):
    if status != R48_OK:
        raise Rein48Error(status, load().r48_last_error().decode())
    return status


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())
