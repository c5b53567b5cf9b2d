"""Count flat_* memory instructions per kernel in a hipcc -save-temps .s file.

A flat load/store that could have been global or LDS costs twice: it occupies both memory
counters, so every later s_waitcnt on either one also waits for it (and for stores issued
before it).  Usage: python tools/flat_ops.py <file.s>"""
import re
import sys

cur, counts = None, {}
for line in open(sys.argv[1]):
    m = re.match(r"^([_A-Za-z][\w.$]*):", line)
    if m and not m.group(1).startswith(".L"):
        cur = m.group(1)
    elif cur and re.match(r"\s+flat_", line):
        counts[cur] = counts.get(cur, 0) + 1
for k, v in sorted(counts.items(), key=lambda kv: -kv[1]):
    print(f"{v:5d}  {k[:120]}")
