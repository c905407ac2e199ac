#!/usr/bin/env python3
"""Print the per-phase cycle table of a phase_profile.py output (concatenated JSON objects)."""
import json
import sys

txt = open(sys.argv[1]).read()
dec = json.JSONDecoder()
i = 0
while True:
    rest = txt[i:].lstrip()
    if not rest:
        break
    o, n = dec.raw_decode(rest)
    i = len(txt) - len(rest) + n
    r = o["cycles_per_env_step"]["render"]
    s = o["cycles_per_env_step"]["step"]
    print(o["game"].ljust(10), "R", " ".join("%s=%d" % (k[:8], v) for k, v in r.items()))
    print(" " * 10, "S", " ".join("%s=%d" % (k[:8], v) for k, v in s.items()))
