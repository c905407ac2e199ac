"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every symbol the
headers declare, and rejects bad options the way the reference does (vecoptions.cpp:73-94,
game.cpp:62-95) -- without touching a GPU (option validation precedes any HIP call)."""
import ctypes
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("libenv.h", "procgen_mi355x.h")]


def declared_symbols():
    names = []
    for h in HEADERS:
        src = open(h).read()
        names += re.findall(r"LIBENV_API\s+[\w\s\*]+?\b(\w+)\s*\(", src)
    return sorted(set(names))


def test_headers_declare_the_libenv_surface():
    names = declared_symbols()
    for n in ["libenv_version", "libenv_make", "libenv_get_tensortypes", "libenv_set_buffers", "libenv_observe",
              "libenv_act", "libenv_close", "get_state", "set_state"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from procgen_amd import _lib
    lib = _lib.load()
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.libenv_version() == 1


def make(options, num=4):
    from procgen_amd import _lib
    lib = _lib.load()
    o = _lib.OptionList(options)
    h = lib.libenv_make(num, o.struct)
    msg = lib.procgen_error_string(None)
    return h, (msg.decode() if msg else "")


BASE = {"env_name": "coinrun", "num_levels": 0, "start_level": 0, "num_actions": 15, "rand_seed": 0}


def test_unknown_option_rejected():
    h, msg = make(dict(BASE, bogus_option=1))
    assert not h and "bogus_option" in msg


def test_wrong_dtype_rejected():
    h, msg = make(dict(BASE, center_agent=3))  # int where the reference consumes a bool
    assert not h and "center_agent" in msg


def test_missing_start_level_rejected():
    opts = dict(BASE)
    del opts["start_level"]
    h, msg = make(opts)
    assert not h and "start_level" in msg


def test_unsupported_game_rejected():
    h, msg = make(dict(BASE, env_name="notagame"))  # vecgame.cpp: unknown names fatal
    assert not h and "notagame" in msg


def test_invalid_distribution_mode_rejected():
    h, msg = make(dict(BASE, distribution_mode=2))  # extreme: not valid for coinrun (game.cpp:81-82)
    assert not h and "distribution_mode" in msg


def test_option_encoding_matches_gym3():
    from procgen_amd import _lib
    o = _lib.OptionList({"a": True, "b": 7, "c": "coinrun"})
    items = o.struct.items
    assert (items[0].dtype, items[0].count) == (_lib.DTYPE_UINT8, 1)
    assert (items[1].dtype, items[1].count) == (_lib.DTYPE_INT32, 1)
    assert (items[2].dtype, items[2].count) == (_lib.DTYPE_UINT8, 7)
    assert ctypes.string_at(items[2].data, 7) == b"coinrun"


def test_struct_sizes_match_header():
    from procgen_amd import _lib
    # struct libenv_tensortype: 128 + 4 + 4 + 16*4 + 4 + 4 + 4
    assert ctypes.sizeof(_lib.libenv_tensortype) == 212
    assert ctypes.sizeof(_lib.libenv_option) == 144
    assert ctypes.sizeof(_lib.pg_image) == 16


def test_mixed_batch_size_must_divide():
    h, msg = make(dict(BASE, env_name="coinrun,maze"), num=5)  # vecgame.cpp:345 num_envs % #games
    assert not h and "multiple" in msg


def test_memory_mode_only_for_memory_games():
    h, msg = make(dict(BASE, env_name="bigfish", distribution_mode=10))  # game.cpp:83-84
    assert not h and "distribution_mode" in msg


def test_gym3_sequence_uses_only_libenv_symbols():
    """gym3's CEnv sequence (tests/gym3_cenv.py) needs no extension call: the driver resolves only
    the libenv symbols, and libenv_make loads the atlas itself (no procgen_upload_atlas step).
    Without a GPU the make stops at the first HIP call, never at a missing atlas."""
    from procgen_amd import _lib
    from gym3_cenv import LIBENV_SYMBOLS, CEnv, RecordingLib
    from conftest import has_gpu
    lib = RecordingLib(_lib.LIB_PATH)
    opts = dict(BASE, num_levels=200, use_backgrounds=True, center_agent=True, distribution_mode=1)
    if has_gpu():
        env = CEnv(lib, 2, opts)
        env.observe()
        env.act([1, 2])
        env.observe()
        env.close()
    else:
        with pytest.raises(RuntimeError):
            CEnv(lib, 2, opts)
        msg = _lib.load().procgen_error_string(None).decode()
        assert "asset" not in msg and "atlas" not in msg, msg
    assert set(lib.looked_up) <= set(LIBENV_SYMBOLS), lib.looked_up


def test_env_offset_must_be_nonnegative():
    h, msg = make(dict(BASE, env_offset=-3))
    assert not h and "env_offset" in msg
