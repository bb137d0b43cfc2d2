"""Loader for the native library (gloo_amd/libgloo_amd.so) and its C ABI
(include/gloo_amd/glx.h).

The HIP extension is the product: if it is missing this module raises
ImportError -- there is no CPU fallback.
"""
import ctypes
import os

# Import torch first when available so that the process uses ONE HIP runtime
# (torch ships libamdhip64.so.7; our library resolves to the already-loaded
# object by SONAME).
try:  # pragma: no cover - torch is present in this image
    import torch  # noqa: F401
except Exception:  # noqa: BLE001
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgloo_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "gloo_amd: native library %s is missing -- build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
        "There is no CPU fallback." % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)

_vp, _sz, _i, _i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64
_pi = ctypes.POINTER(ctypes.c_int)

# (name, restype, argtypes) for every symbol declared in include/gloo_amd/glx.h
SIGNATURES = [
    ("glx_last_error", ctypes.c_char_p, []),
    ("glx_version", ctypes.c_char_p, []),
    ("glx_dtype_size", _sz, [_i]),
    ("glx_reduce", _i, [_i, _i, _vp, _vp, _vp, _sz, _vp]),
    ("glx_reduce_n", _i, [_i, _i, _vp, ctypes.POINTER(_vp), _i, _sz, _vp]),
    ("glx_peer_copy", _i, [_vp, _i, _vp, _i, _sz, _vp]),
    ("glx_host_reduce_n", _i, [_i, _i, _vp, ctypes.POINTER(_vp), _i, _sz]),
    ("glx_copy", _i, [_vp, _vp, _sz, _i, _vp]),
    ("glx_enable_peer", _i, [_i, _i]),
    ("glx_tune_reduce", _i, [_i, _i, _i]),
    ("glx_reduce_tuning", _i, [_pi, _pi, _pi]),
    ("glx_set_max_message_bytes", _i, [_i64]),
    ("glx_allreduce_host_fn", _i, [_vp, _i, _sz, _vp, _vp, ctypes.POINTER(_vp), _i,
                                   ctypes.POINTER(_vp), _i, _sz, ctypes.c_uint32, _sz, _i64]),
    ("glx_allreduce_create_host_fn", _vp, [_vp, _i, ctypes.POINTER(_vp), _i, _i, _sz, _vp,
                                           _vp]),
    ("glx_max_message_bytes", _i64, []),
    ("glx_set_pipeline_bytes", _i, [_i64]),
    ("glx_pipeline_bytes", _i64, []),
    ("glx_reduce_segment_bytes", _sz, []),
    ("glx_set_copy_split", _i, [_i]),
    ("glx_set_pinned_mirror_limit", _i, [_sz]),
    ("glx_device_count", _i, [ctypes.POINTER(_i)]),
    ("glx_hash_store_create", _vp, []),
    ("glx_file_store_create", _vp, [ctypes.c_char_p]),
    ("glx_prefix_store_create", _vp, [ctypes.c_char_p, _vp]),
    ("glx_callback_store_create", _vp, [_vp, _vp, _vp]),
    ("glx_store_destroy", None, [_vp]),
    ("glx_store_set", _i, [_vp, ctypes.c_char_p, _vp, _sz]),
    ("glx_store_get", _i, [_vp, ctypes.c_char_p, _vp, _sz, ctypes.POINTER(_sz), _i64]),
    ("glx_context_create", _vp, [_i, _i, _i]),
    ("glx_context_destroy", None, [_vp]),
    ("glx_context_connect_full_mesh", _i, [_vp, _vp]),
    ("glx_context_rank", _i, [_vp]),
    ("glx_context_size", _i, [_vp]),
    ("glx_context_device", _i, [_vp]),
    ("glx_context_set_timeout", _i, [_vp, _i64]),
    ("glx_context_set_base", _i, [_vp, _i]),
    ("glx_plan_bcube", _i64, [_i, _i, _i64, _i, ctypes.POINTER(_i64), _i64,
                              ctypes.POINTER(_i64)]),
    ("glx_context_get_timeout", _i64, [_vp]),
    ("glx_context_next_slot", _i, [_vp, _i]),
    ("glx_allreduce_ring_chunked_create", _vp,
     [_vp, ctypes.POINTER(_vp), _i, _i, _i, _i, ctypes.POINTER(_vp), _i]),
    ("glx_allreduce_halving_doubling_create", _vp,
     [_vp, ctypes.POINTER(_vp), _i, _i, _i, _i, ctypes.POINTER(_vp), _i]),
    ("glx_allreduce_create", _vp,
     [_vp, _i, ctypes.POINTER(_vp), _i, _i, _i, _i, ctypes.POINTER(_vp), _i]),
    ("glx_algorithm_run", _i, [_vp]),
    ("glx_algorithm_run_fed", _i, [_vp]),
    ("glx_algorithm_feed", _i, [_vp, _i64, _i64]),
    ("glx_algorithm_done_ranges", _i64, [_vp, ctypes.POINTER(_i64), _i64]),
    ("glx_algorithm_bytes_sent", _i64, [_vp]),
    ("glx_algorithm_engine", _i, [_vp]),
    ("glx_algorithm_fast_streams", _i, [_vp]),
    ("glx_algorithm_sync", _i, [_vp]),
    ("glx_set_device_sync", _i, [_i]),
    ("glx_algorithm_destroy", None, [_vp]),
    ("glx_algorithm_transport_stats", _i, [_vp, ctypes.POINTER(_i64), _i]),
    ("glx_algorithm_record", _i, [_vp, _vp]),
    ("glx_context_ipc_stats", _i, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    ("glx_context_peer_info", _i, [_vp, _i, ctypes.POINTER(_i)]),
    ("glx_link_probe_create", _vp, [_vp, _sz]),
    ("glx_link_probe_run", _i, [_vp, _i, _i, _i, _i, ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(_sz)]),
    ("glx_link_probe_destroy", None, [_vp]),
    ("glx_event_create", _i, [ctypes.POINTER(_vp)]),
    ("glx_event_destroy", _i, [_vp]),
    ("glx_event_record", _i, [_vp, _vp]),
    ("glx_event_query", _i, [_vp]),
    ("glx_event_wait", _i, [_vp, _vp]),
    ("glx_device_layout", _i64, [_i, _i, _i, _i64, _i, _i64, ctypes.POINTER(_i64), _i64]),
    ("glx_plan_sync", _i64, [_i, _i, _i, _i64, _i, _i64, _i64, _i, ctypes.POINTER(_i64),
                             _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                             ctypes.POINTER(_i64), _i64]),
    ("glx_plan", _i64, [_i, _i, _i, _i64, ctypes.POINTER(_i64), _i64,
                        ctypes.POINTER(_i64)]),
    ("glx_plan_fold", _i64, [_i, _i, _i, _i64, _i64, ctypes.POINTER(_i64), _i64]),
    ("glx_plan_ex", _i64, [_i, _i, _i, _i64, _i, _i64, _i64, ctypes.POINTER(_i64), _i64,
                           ctypes.POINTER(_i64)]),
    ("glx_plan_fold_ex", _i64, [_i, _i, _i, _i64, _i, _i64, _i64, _i64,
                                ctypes.POINTER(_i64), _i64]),
    ("glx_plan_stage", _i64, [_i, _i, _i, _i64, _i, _i64, ctypes.POINTER(_i64), _i64,
                              ctypes.POINTER(_i64), _i64, ctypes.POINTER(_i64)]),
    ("glx_set_copy_engine", _i, [_i, _i]),
    ("glx_set_mesh_engine", _i, [_i]),
    ("glx_set_device_engines", _i, [_i]),
    ("glx_get_device_engines", _i, []),
    ("glx_device_engines_rule", _i, [_i, _i, _i, _i, _i]),
    ("glx_set_steps_engine", _i, [_i]),
    ("glx_set_engine_streams", _i, [_i]),
    ("glx_allreduce", _i, [_vp, _i, _i, _i, ctypes.POINTER(_vp), _i, ctypes.POINTER(_vp), _i,
                           ctypes.c_size_t, ctypes.c_uint32, ctypes.c_size_t, _i64, _vp]),
]

for _name, _res, _args in SIGNATURES:
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

STORE_SET_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p,
                                ctypes.c_void_p, ctypes.c_size_t)
STORE_GET_FN = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p,
                                ctypes.c_void_p, ctypes.c_size_t)
# glx_reduce_fn: (user, c, a, b, n) -> 0, or nonzero when the function failed
REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_size_t)

# status codes (glx_status), and GLX_NOT_READY of glx_event_query
OK, ERR_INVALID, ERR_HIP, ERR_TIMEOUT, ERR_IO, ERR_ENFORCE, ERR_INTERNAL, NOT_READY = range(8)


def last_error():
    msg = lib.glx_last_error()
    return msg.decode(errors="replace") if msg else ""
