"""Loader for libpgx.so, the HIP/gfx950 implementation of the env step (C-ABI in include/pgx.h).

The product path has no CPU fallback: if the shared library is missing or does
not export the full ABI, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

from .abi import PGX_E_INVALID  # noqa: F401 (re-exported for the C-ABI tests)
from .abi import PgxConfig, PgxReplayBatch, PgxReplayConfig, PgxStateView, PgxStepOut, PgxTransition

LIB_PATH = os.environ.get("PGX_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpgx.so")

EXPORTS = [
    "pgx_version", "pgx_last_error", "pgx_obs_dim", "pgx_action_dim", "pgx_dev_model_bytes", "pgx_create", "pgx_destroy",
    "pgx_get_state", "pgx_reset", "pgx_step", "pgx_step_kernel", "pgx_sample_actions", "pgx_compute_reward",
    "pgx_state_bytes", "pgx_save_state", "pgx_restore_state", "pgx_snapshot", "pgx_restore", "pgx_release",
    "pgx_set_rng_streams", "pgx_get_rng_streams",
    "pgx_replay_create", "pgx_replay_destroy", "pgx_replay_add", "pgx_replay_size", "pgx_replay_sample",
    "pgx_replay_episode_arrays", "pgx_replay_row_dim", "pgx_replay_row_stride",
]


class PgxError(RuntimeError):
    """A libpgx call returned a negative status (message from pgx_last_error)."""


_libs = {}


def load(path: str = None):
    """Load libpgx.so (or another build of the same ABI, e.g. libpgx_rtmodel.so) once per path;
    raise loudly if it is absent (build with __graft_entry__.build())."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise PgxError(f"libpgx.so not found at {path}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    for name in EXPORTS:
        if not hasattr(lib, name):
            raise PgxError(f"libpgx.so does not export {name}")
    lib.pgx_version.restype = C.c_char_p
    lib.pgx_last_error.restype = C.c_char_p
    lib.pgx_obs_dim.argtypes = [C.POINTER(PgxConfig)]
    lib.pgx_action_dim.argtypes = [C.POINTER(PgxConfig)]
    lib.pgx_dev_model_bytes.argtypes = [C.POINTER(PgxConfig), C.c_void_p, C.c_int64]
    lib.pgx_create.argtypes = [C.POINTER(PgxConfig), C.c_int, C.POINTER(C.c_void_p)]
    lib.pgx_destroy.argtypes = [C.c_void_p]
    lib.pgx_destroy.restype = None
    lib.pgx_get_state.argtypes = [C.c_void_p, C.POINTER(PgxStateView)]
    lib.pgx_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(PgxStepOut), C.c_void_p]
    lib.pgx_step.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(PgxStepOut), C.c_void_p]
    if hasattr(lib, "pgx_step_kernel"):   # (A/B runs load older builds with EXPORTS filtered)
        lib.pgx_step_kernel.argtypes = [C.c_void_p]
        lib.pgx_step_kernel.restype = C.c_char_p
    lib.pgx_sample_actions.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    lib.pgx_compute_reward.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_double, C.c_void_p,
                                       C.c_void_p]
    lib.pgx_state_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    lib.pgx_save_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.pgx_restore_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.pgx_snapshot.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_void_p]
    lib.pgx_restore.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    lib.pgx_release.argtypes = [C.c_void_p, C.c_int32]
    lib.pgx_set_rng_streams.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.pgx_get_rng_streams.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.pgx_replay_create.argtypes = [C.POINTER(PgxReplayConfig), C.c_int, C.POINTER(C.c_void_p)]
    lib.pgx_replay_row_dim.argtypes = [C.POINTER(PgxReplayConfig)]
    lib.pgx_replay_row_stride.argtypes = [C.POINTER(PgxReplayConfig)]
    lib.pgx_replay_destroy.argtypes = [C.c_void_p]
    lib.pgx_replay_destroy.restype = None
    lib.pgx_replay_add.argtypes = [C.c_void_p, C.POINTER(PgxTransition), C.c_void_p]
    lib.pgx_replay_size.argtypes = [C.c_void_p]
    lib.pgx_replay_size.restype = C.c_int64
    lib.pgx_replay_sample.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.POINTER(PgxReplayBatch), C.c_void_p]
    lib.pgx_replay_episode_arrays.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                              C.POINTER(C.c_void_p)]
    _libs[path] = lib
    return lib


def check(rc: int, what: str, lib=None) -> None:
    if rc != 0:
        msg = (lib or load()).pgx_last_error().decode(errors="replace")
        raise PgxError(f"{what} failed ({rc}): {msg}")
