"""Loader for the C-ABI library libcoup_mi355x.so (include/coup_mi355x.h).

The library is built in-tree by open_spiel_coup_amd.build (hipcc, gfx950).
There is no fallback: if the library is missing or cannot be loaded, every
entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# COUP_LIB_PATH: load another build of the same library (A/B timing of two
# builds, tools/ab_builds.sh); there is still no fallback
LIB_PATH = os.environ.get("COUP_LIB_PATH") or os.path.join(HERE, "libcoup_mi355x.so")
ABI_VERSION = 14
FLAG_AUTO_RESET, FLAG_HISTORY, FLAG_GENERIC, FLAG_UNCHECKED = 1, 2, 4, 8
MAX_PLAYERS = 6
HISTORY_BYTES = 96

COUP_OK, COUP_E_INVALID, COUP_E_HIP, COUP_E_LANES = 0, 1, 2, 3
BUILD_AB_VARIANTS = 1  # coup_build_flags: a measurement build with every A/B variant
BUILD_TRAJ_STAGE_SHIFT, BUILD_TRAJ_STAGE_MASK = 1, 0x7  # coup_build_flags: the rules trajectories' output staging
SWEEP_RESIDENT, SWEEP_INDEX_BITS = 1, 2  # coup_measure_store_sweep mode bits

# Every symbol declared in include/coup_mi355x.h
SYMBOLS = (
    "coup_abi_version", "coup_last_error", "coup_create", "coup_create_ex", "coup_destroy", "coup_reload_knobs",
    "coup_set_stream", "coup_batch", "coup_num_players", "coup_state_bytes", "coup_reset", "coup_step", "coup_rollout",
    "coup_step_trajectory", "coup_step_many", "coup_step_host", "coup_step_host_layout",
    "coup_new_initial_state", "coup_apply_action", "coup_query",
    "coup_export_state", "coup_import_state", "coup_export_history",
    "coup_import_history", "coup_error_count", "coup_slot_op", "coup_slot_ops", "coup_measure_step_traffic", "coup_measure_store_sweep", "coup_obs_split_variant",
    "coup_info_split_variant", "coup_build_flags", "coup_launch_log",
    "coup_server_create", "coup_server_destroy", "coup_attach_server", "coup_server_stats",
    "coup_host_state_init", "coup_host_state_apply", "coup_host_state_tensors", "coup_host_state_string",
    "coup_host_state_step",
    "coup_write_lane",
)

# coup_slot_op flags and result layout (coup_slot_result, 128 bytes)
SLOT_INIT, SLOT_OBS, SLOT_INFO, SLOT_NO_RESULT, SLOT_RESET, SLOT_DEAL, SLOT_UNCHECKED = 1, 2, 4, 8, 16, 32, 64
HOST_OBS, HOST_INFO, HOST_ACTIVE = 1, 2, 4  # coup_step_host
SLOT_RESULT_BYTES = 128


class StepOutputs(ctypes.Structure):
    _fields_ = [("actions", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("step_type", ctypes.c_void_p), ("legal_mask", ctypes.c_void_p),
                ("cur_player", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("info_state", ctypes.c_void_p), ("episodes", ctypes.c_void_p),
                ("return_sum", ctypes.c_void_p), ("episode_word", ctypes.c_void_p),
                ("episode_word_bytes", ctypes.c_int32)]


class QueryOutputs(ctypes.Structure):
    _fields_ = [("legal_mask", ctypes.c_void_p), ("cur_player", ctypes.c_void_p),
                ("terminal", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("returns", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("info_state", ctypes.c_void_p)]


class RolloutStats(ctypes.Structure):
    _fields_ = [("episodes", ctypes.c_void_p), ("return_sum", ctypes.c_void_p),
                ("length_sum", ctypes.c_void_p), ("episode_word", ctypes.c_void_p),
                ("episode_word_bytes", ctypes.c_int32)]


class SlotReq(ctypes.Structure):
    """coup_slot_req (24 bytes)."""
    _fields_ = [("lane", ctypes.c_int64), ("src_lane", ctypes.c_int64), ("action", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


class CoupError(RuntimeError):
    """Raised for a failing C-ABI call (mirrors pyspiel.SpielError)."""


_lib = None


def load():
    """Load libcoup_mi355x.so once.  torch is imported first so the process
    uses torch's HIP runtime (same soname) for both torch and our kernels."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (HIP runtime first)
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run `python -m open_spiel_coup_amd.build`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    sig = {
        "coup_abi_version": ([], i32),
        "coup_last_error": ([], ctypes.c_char_p),
        "coup_create": ([i64, ctypes.c_uint64, ctypes.c_uint32, i32, ctypes.POINTER(vp)], i32),
        "coup_create_ex": ([i64, ctypes.c_uint64, ctypes.c_uint32, i32, i32, ctypes.POINTER(vp)], i32),
        "coup_destroy": ([vp], i32),
        "coup_reload_knobs": ([vp], i32),
        "coup_set_stream": ([vp, vp], i32),
        "coup_batch": ([vp], i64),
        "coup_num_players": ([vp], i32),
        "coup_state_bytes": ([vp], i32),
        "coup_reset": ([vp, vp], i32),
        "coup_step": ([vp, vp, ctypes.POINTER(StepOutputs)], i32),
        "coup_rollout": ([vp, i64, ctypes.POINTER(RolloutStats)], i32),
        "coup_step_trajectory": ([vp, i64, ctypes.POINTER(StepOutputs)], i32),
        "coup_step_many": ([vp, i64, ctypes.POINTER(StepOutputs)], i32),
        "coup_step_host": ([vp, vp, i32, vp], i32),
        "coup_step_host_layout": ([i64, i32, i32, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_size_t),
        "coup_new_initial_state": ([vp, vp], i32),
        "coup_apply_action": ([vp, vp], i32),
        "coup_query": ([vp, ctypes.POINTER(QueryOutputs)], i32),
        "coup_export_state": ([vp, vp], i32),
        "coup_import_state": ([vp, vp], i32),
        "coup_export_history": ([vp, vp], i32),
        "coup_import_history": ([vp, vp], i32),
        "coup_error_count": ([vp, ctypes.POINTER(i64)], i32),
        "coup_slot_op": ([vp, i64, vp, i64, i32, i32, vp], i32),
        "coup_slot_ops": ([vp, i64, ctypes.POINTER(SlotReq), vp, i32, vp], i32),
        "coup_measure_step_traffic": ([i64, vp, ctypes.POINTER(StepOutputs), vp], i32),
        "coup_measure_store_sweep": ([vp, i64, i32, i32, i32, vp], i32),
        "coup_obs_split_variant": ([i64], i32),
        "coup_info_split_variant": ([i64], i32),
        "coup_build_flags": ([], i32),
        "coup_launch_log": ([ctypes.c_char_p, i32, i32], i32),
        "coup_server_create": ([i64, ctypes.POINTER(vp)], i32),
        "coup_server_destroy": ([vp], i32),
        "coup_attach_server": ([vp, vp], i32),
        "coup_server_stats": ([vp, ctypes.POINTER(ctypes.c_uint64)], i32),
        "coup_host_state_init": ([vp], i32),
        "coup_host_state_apply": ([ctypes.c_char_p, i32, i32, vp], i32),
        "coup_host_state_tensors": ([ctypes.c_char_p, vp, vp], i32),
        "coup_host_state_string": ([ctypes.c_char_p, i32, i32, vp, i64], i64),
        "coup_host_state_step": ([ctypes.c_char_p, i32, i32, ctypes.c_uint64, ctypes.c_uint32, vp], i32),
        "coup_write_lane": ([vp, i64, ctypes.c_char_p], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.coup_abi_version() != ABI_VERSION:
        raise ImportError(f"libcoup_mi355x ABI {L.coup_abi_version()} != {ABI_VERSION}")
    _lib = L
    return L


def launch_log(reset=True):
    """The kernels this thread's library calls launched since the last reset
    (coup_launch_log): "coup::k_a<...> + coup::k_b<...>"; clears it."""
    L = load()
    n = L.coup_launch_log(None, 0, 0)
    buf = ctypes.create_string_buffer(n + 1)
    L.coup_launch_log(buf, n + 1, 1 if reset else 0)
    return buf.value.decode()


def check(rc):
    if rc != COUP_OK:
        msg = load().coup_last_error().decode(errors="replace")
        raise CoupError(f"coup C-ABI error {rc}: {msg}")
