"""Loader for libsplendor_amd.so (the HIP/gfx950 engine, C ABI in include/splendor_amd.h).

There is NO CPU fallback: if the shared library is missing or cannot be loaded, every
entry point raises NativeEngineMissing. Build it with `python __graft_entry__.py build`
(or `make -C alphazero-general-ori_amd`).
"""
import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SPLENDOR_AMD_LIB") or os.path.join(PKG_ROOT, "libsplendor_amd.so")

ABI_VERSION = 11
EINVAL, EDEVICE = -1, -2
BACKUP_DEFER_GC = 4                 # spl_mcts_backup_kind: SPL_BACKUP_DEFER_GC


class NativeEngineMissing(RuntimeError):
    pass


class EngineError(RuntimeError):
    pass


_lib = None

_vp, _i8p, _i16p, _i32p, _u64p, _fp, _dp = (C.c_void_p,) * 7
_SIGS = {
    "spl_abi_version": ([], C.c_int),
    "spl_ctx_create": ([C.c_int, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "spl_ctx_destroy": ([C.c_void_p], C.c_int),
    "spl_ctx_set_token_limit": ([C.c_void_p, C.c_int], C.c_int),
    "spl_symmetries": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_state_rows": ([C.c_void_p], C.c_int),
    "spl_state_bytes": ([C.c_void_p], C.c_int),
    "spl_init": ([C.c_void_p, C.c_int, _vp, _vp, _vp, C.c_int, C.c_uint64, C.c_uint32, C.c_uint32,
                  _vp], C.c_int),
    "spl_valid_moves": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "spl_step": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, C.c_int, _vp, C.c_int, C.c_uint64,
                  C.c_uint32, C.c_uint32, _vp, _vp], C.c_int),
    "spl_game_ended": ([C.c_void_p, C.c_int, _vp, _vp, _vp], C.c_int),
    "spl_canonical": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "spl_score": ([C.c_void_p, C.c_int, _vp, _vp, _vp], C.c_int),
    "spl_round": ([C.c_void_p, C.c_int, _vp, _vp, _vp], C.c_int),
    "spl_tree_step": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_rollout_step": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint64, C.c_uint32,
                          C.c_uint32, _vp], C.c_int),
    "spl_nn_packed_floats": ([C.c_int], C.c_int),
    "spl_nn_forward": ([C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_nn_forward_indexed": ([C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_rollout_run": ([C.c_void_p, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint64,
                         C.c_uint32, C.c_uint32, _vp], C.c_int),
    "spl_mcts_create": ([C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)], C.c_int),
    "spl_mcts_destroy": ([C.c_void_p], C.c_int),
    "spl_mcts_device_bytes": ([C.c_void_p], C.c_longlong),
    "spl_mcts_plan_bytes": ([_vp, C.c_int, _vp], C.c_longlong),
    "spl_mcts_counters": ([C.c_void_p, _vp, _vp], C.c_int),
    "spl_mcts_pool_state": ([C.c_void_p, _vp, _vp], C.c_int),
    "spl_mcts_pool_pages": ([C.c_void_p, _vp], C.c_int),
    "spl_mcts_set_roots": ([C.c_void_p, _vp, C.c_int, C.c_int, _vp], C.c_int),
    "spl_mcts_set_roots_active": ([C.c_void_p, _vp, _vp, C.c_int, C.c_int, _vp], C.c_int),
    "spl_mcts_pick_best": ([C.c_void_p, _vp, C.c_uint32, C.c_uint32, _vp, _vp], C.c_int),
    "spl_mcts_select": ([C.c_void_p, _vp, _vp, _vp, _vp], C.c_int),
    "spl_mcts_select_compact": ([C.c_void_p, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_mcts_backup": ([C.c_void_p, _vp, _vp, _vp, _vp], C.c_int),
    "spl_mcts_backup_kind": ([C.c_void_p, _vp, _vp, _vp, C.c_int, _vp], C.c_int),
    "spl_mcts_root_stats": ([C.c_void_p, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_mcts_root_priors": ([C.c_void_p, _vp, _vp], C.c_int),
    "spl_mcts_headers": ([C.c_void_p, _vp, _vp], C.c_int),
    "spl_mcts_tree_sizes": ([C.c_void_p, _vp, _vp], C.c_int),
    "spl_mcts_reset_games": ([C.c_void_p, _vp], C.c_int),
    "spl_mcts_restart_games": ([C.c_void_p, _vp, _vp], C.c_int),
    "spl_mcts_commit": ([C.c_void_p, _vp], C.c_int),
    "spl_mcts_drain_examples": ([C.c_void_p, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int, _vp, _vp], C.c_int),
    "spl_nn_input": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_hash_eval": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "spl_hash_eval_mode": ([C.c_void_p, C.c_int, _vp, _vp, _vp, _vp, C.c_int, _vp], C.c_int),
}


class MctsConfig(C.Structure):
    """spl_mcts_config (include/splendor_amd.h)"""
    _fields_ = [("num_sims", C.c_int), ("ratio_full", C.c_int), ("prob_full", C.c_double),
                ("cpuct", C.c_double), ("fpu", C.c_double), ("forced_playouts", C.c_int),
                ("dirichlet_alpha", C.c_double), ("dirichlet_temp", C.c_double),
                ("temp_threshold", C.c_int), ("node_cap", C.c_int), ("edge_cap", C.c_int),
                ("seed", C.c_uint64), ("board_base", C.c_uint32), ("selfplay", C.c_int),
                ("out_cap", C.c_int), ("node_boards", C.c_int), ("pool_nodes", C.c_longlong),
                ("pool_edges", C.c_longlong)]


def exported_symbols():
    return list(_SIGS)


def lib():
    """Load the engine once; raise loudly if it is not there."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeEngineMissing(
            f"{LIB_PATH} not found: the HIP engine must be built (no CPU fallback exists)")
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeEngineMissing(f"cannot load {LIB_PATH}: {e}") from e
    for name, (args, res) in _SIGS.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.spl_abi_version() != ABI_VERSION:
        raise NativeEngineMissing(f"ABI mismatch: library {L.spl_abi_version()} != {ABI_VERSION}")
    _lib = L
    return L


def check(rc, what):
    if rc != 0:
        kind = {EINVAL: "invalid argument", EDEVICE: "HIP device error"}.get(rc, f"rc={rc}")
        raise EngineError(f"{what}: {kind}")
