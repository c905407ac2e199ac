"""ctypes binding of libprocgen_mi355x.so (the C ABI declared in include/libenv.h and
include/procgen_mi355x.h).

This is the binding a reference-side maintainer would otherwise get from gym3's cffi
``CEnv`` (procgen/env.py:152-160); see INTEGRATION.md.  The library is loaded from the
package directory -- there is no CPU fallback: if it is missing, importing fails loudly.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PROCGEN_MI355X_LIB=prof selects the diagnostic build (per-phase cycle counters); any other
# name selects an experiment build libprocgen_mi355x_<name>.so (csrc/Makefile VARIANT=)
_variant = os.environ.get("PROCGEN_MI355X_LIB", "")
LIB_PATH = os.path.join(HERE, "libprocgen_mi355x_%s.so" % _variant if _variant else "libprocgen_mi355x.so")

LIBENV_MAX_NAME_LEN = 128
LIBENV_MAX_NDIM = 16
DTYPE_UINT8, DTYPE_INT32, DTYPE_FLOAT32 = 1, 2, 3
SPACE_OBSERVATION, SPACE_ACTION, SPACE_INFO = 1, 2, 3
NP_DTYPE = {DTYPE_UINT8: np.uint8, DTYPE_INT32: np.int32, DTYPE_FLOAT32: np.float32}


class libenv_value(ctypes.Union):
    _fields_ = [("uint8", ctypes.c_uint8), ("int32", ctypes.c_int32), ("float32", ctypes.c_float)]


class libenv_tensortype(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * LIBENV_MAX_NAME_LEN), ("scalar_type", ctypes.c_int),
                ("dtype", ctypes.c_int), ("shape", ctypes.c_int * LIBENV_MAX_NDIM), ("ndim", ctypes.c_int),
                ("low", libenv_value), ("high", libenv_value)]


class libenv_option(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * LIBENV_MAX_NAME_LEN), ("dtype", ctypes.c_int),
                ("count", ctypes.c_int), ("data", ctypes.c_void_p)]


class libenv_options(ctypes.Structure):
    _fields_ = [("items", ctypes.POINTER(libenv_option)), ("count", ctypes.c_int)]


class libenv_buffers(ctypes.Structure):
    _fields_ = [("ob", ctypes.POINTER(ctypes.c_void_p)), ("ac", ctypes.POINTER(ctypes.c_void_p)),
                ("info", ctypes.POINTER(ctypes.c_void_p)), ("rew", ctypes.c_void_p),
                ("first", ctypes.c_void_p)]


class pg_image(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint32), ("w", ctypes.c_int32), ("h", ctypes.c_int32), ("pad", ctypes.c_int32)]


class pg_device_buffers(ctypes.Structure):
    _fields_ = [("rgb", ctypes.c_void_p), ("rew", ctypes.c_void_p), ("first", ctypes.c_void_p),
                ("prev_level_seed", ctypes.c_void_p), ("prev_level_complete", ctypes.c_void_p),
                ("level_seed", ctypes.c_void_p), ("actions", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


# name -> (restype, argtypes)
SIGNATURES = {
    "libenv_version": (ctypes.c_int, []),
    "libenv_make": (ctypes.c_void_p, [ctypes.c_int, libenv_options]),
    "libenv_get_tensortypes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(libenv_tensortype)]),
    "libenv_set_buffers": (None, [ctypes.c_void_p, ctypes.POINTER(libenv_buffers)]),
    "libenv_observe": (None, [ctypes.c_void_p]),
    "libenv_act": (None, [ctypes.c_void_p]),
    "libenv_close": (None, [ctypes.c_void_p]),
    "get_state": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "set_state": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "procgen_upload_atlas": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_atlas_host": (ctypes.c_int64, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_read_envs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6),
    "procgen_read_outputs": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 6),
    "procgen_set_obs_buffer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_set_latent_state": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 6),
    "procgen_start": (ctypes.c_int, [ctypes.c_void_p]),
    "procgen_act_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_act_hashed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32]),
    "procgen_wait": (ctypes.c_int, [ctypes.c_void_p]),
    "procgen_device_buffers": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(pg_device_buffers)]),
    "procgen_last_error": (ctypes.c_int, [ctypes.c_void_p]),
    "procgen_error_string": (ctypes.c_char_p, [ctypes.c_void_p]),
    "procgen_kernel_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    "procgen_set_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "procgen_num_parts": (ctypes.c_int, [ctypes.c_void_p]),
    "procgen_shard_plan": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_debug_env": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
    "procgen_profile_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_profile_raw": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "procgen_selftest_libm": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_void_p]),
}

_LIB = None


def load(path=LIB_PATH):
    """Load the HIP library (raises if it was not built: no silent fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise ImportError("libprocgen_mi355x.so not found at %s -- run `python -c 'import __graft_entry__ as g; "
                          "g.build()'` (or make -C procgen-1_amd/csrc)" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


class OptionList:
    """Builds a ``struct libenv_options`` from a python dict (gym3 CEnv's encoding:
    bool -> uint8, int -> int32, str -> uint8 bytes)."""

    def __init__(self, options):
        self._keep = []
        items = (libenv_option * len(options))()
        for i, (k, val) in enumerate(options.items()):
            items[i].name = k.encode()
            if isinstance(val, (bool, np.bool_)):
                arr = np.array([int(val)], dtype=np.uint8)
                items[i].dtype = DTYPE_UINT8
            elif isinstance(val, (int, np.integer)):
                arr = np.array([val], dtype=np.int32)
                items[i].dtype = DTYPE_INT32
            elif isinstance(val, str):
                arr = np.frombuffer(val.encode(), dtype=np.uint8).copy()
                items[i].dtype = DTYPE_UINT8
            else:
                raise TypeError("unsupported option type for %s: %r" % (k, type(val)))
            items[i].count = arr.size
            items[i].data = arr.ctypes.data
            self._keep.append(arr)
        self._keep.append(items)
        self.struct = libenv_options(ctypes.cast(items, ctypes.POINTER(libenv_option)), len(options))
