"""CPU checks of the drop-in boundary: the HIP library loads (no GPU needed to dlopen)
and exports exactly the entry points include/splendor_amd.h declares; the product fails
loudly when its native engine is missing (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "splendor_amd.h")
LIB = os.path.join(ROOT, "alphazero-general-ori_amd", "libsplendor_amd.so")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|long long)\s+(spl_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("spl_init", "spl_valid_moves", "spl_step", "spl_game_ended", "spl_canonical",
                 "spl_tree_step", "spl_rollout_step", "spl_rollout_run"):
        assert must in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsplendor_amd.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.spl_abi_version() == 11


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsplendor_amd.so not built")
def test_host_binding_covers_header():
    from splendor import _lib
    assert sorted(_lib.exported_symbols()) == declared()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsplendor_amd.so not built")
def test_context_argument_validation():
    lib = ctypes.CDLL(LIB)
    h = ctypes.c_void_p()
    assert lib.spl_ctx_create(5, 10, ctypes.byref(h)) == -1
    assert lib.spl_ctx_create(2, 10, ctypes.byref(h)) == 0
    lib.spl_state_bytes.argtypes = [ctypes.c_void_p]
    assert lib.spl_state_bytes(h) == 392
    lib.spl_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.spl_ctx_destroy(h)
    # B == 0 is a no-op that never touches the device
    h4 = ctypes.c_void_p()
    assert lib.spl_ctx_create(4, 10, ctypes.byref(h4)) == 0
    lib.spl_valid_moves.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4
    assert lib.spl_valid_moves(h4, 0, None, None, None, None) == 0
    assert lib.spl_valid_moves(h4, 5, None, None, None, None) == -1


def test_missing_engine_fails_loudly(monkeypatch):
    from splendor import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libsplendor_amd.so")
    with pytest.raises(_lib.NativeEngineMissing):
        _lib.lib()


def test_mcts_config_struct_layout(tmp_path):
    """ctypes MctsConfig must match the C layout of spl_mcts_config."""
    import subprocess
    from splendor import _lib
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "splendor_amd.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(spl_mcts_config),'
                   'offsetof(spl_mcts_config, seed), offsetof(spl_mcts_config, node_cap),'
                   'offsetof(spl_mcts_config, dirichlet_temp), offsetof(spl_mcts_config, out_cap),'
                   'offsetof(spl_mcts_config, node_boards), offsetof(spl_mcts_config, pool_nodes),'
                   'offsetof(spl_mcts_config, pool_edges));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    size, off_seed, off_cap, off_temp, off_out, off_nb, off_pn, off_pe = map(
        int, subprocess.check_output([str(exe)]).split())
    M = _lib.MctsConfig
    assert ctypes.sizeof(M) == size
    assert M.seed.offset == off_seed and M.node_cap.offset == off_cap and M.dirichlet_temp.offset == off_temp
    assert M.out_cap.offset == off_out and M.node_boards.offset == off_nb
    assert M.pool_nodes.offset == off_pn and M.pool_edges.offset == off_pe


def test_search_and_arena_entry_points_reject_bad_arguments():
    """Null handles / buffers and out-of-range streams are rejected before any launch
    (no device needed)."""
    lib = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    lib.spl_mcts_set_roots_active.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, vp]
    lib.spl_mcts_pick_best.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp]
    lib.spl_mcts_select.argtypes = [vp] * 5
    lib.spl_rollout_run.argtypes = [vp, ctypes.c_int, ctypes.c_int] + [vp] * 6 + [ctypes.c_uint64, ctypes.c_uint32,
                                                                               ctypes.c_uint32, vp]
    assert lib.spl_mcts_set_roots_active(None, None, None, 1, 1, None) == -1
    assert lib.spl_mcts_pick_best(None, None, 0, 0, None, None) == -1
    assert lib.spl_mcts_select(None, None, None, None, None) == -1
    h = ctypes.c_void_p()
    assert lib.spl_ctx_create(2, 10, ctypes.byref(h)) == 0
    # rollouts need the per-board game counters (they key the deals)
    dummy = ctypes.c_void_p(1)
    assert lib.spl_rollout_run(h, 4, 1, dummy, dummy, None, dummy, dummy, None, 0, 0, 0, None) == -1
    assert lib.spl_rollout_run(h, 0, 1, None, None, None, None, None, None, 0, 0, 0, None) == 0
    lib.spl_ctx_destroy.argtypes = [vp]
    lib.spl_ctx_destroy(h)
