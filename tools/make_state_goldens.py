#!/usr/bin/env python3
"""Golden vectors for the RandGen text inside get_state (tests/test_state_cpu.py).

Runs the REFERENCE RandGen::serialize (randgen.cpp:100-106, compiled from /root/reference by
`make -C oracle ref` into oracle/_ref/libref.so; ref_randgen_text in oracle/ref_harness.cpp) for a
few (seed, draws) pairs and stores the bytes it writes -- the std::mt19937 text libstdc++'s
operator<< produces.  Build container only (the reference tree is not on the GPU box).
"""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(0, 0), (1, 1), (5489, 7), (123456789, 623), (-5, 624), (2 ** 31 - 1, 625), (42, 1500), (7, 3000)]


def main():
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref.so"))
    lib.ref_randgen_text.argtypes = [ctypes.c_int32, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    texts = []
    for seed, draws in CASES:
        buf = ctypes.create_string_buffer(1 << 14)
        n = lib.ref_randgen_text(seed, draws, buf, len(buf))
        texts.append(buf.raw[:n])
    width = max(len(t) for t in texts)
    arr = np.zeros((len(texts), width), np.uint8)
    for i, t in enumerate(texts):
        arr[i, :len(t)] = np.frombuffer(t, np.uint8)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "randgen_text.npz"),
                        seeds=np.array([c[0] for c in CASES], np.int32), draws=np.array([c[1] for c in CASES], np.int32),
                        text=arr, length=np.array([len(t) for t in texts], np.int32))


if __name__ == "__main__":
    main()
