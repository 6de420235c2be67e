"""Print the last N kernel dispatches and memory copies of a rocprofv3 sqlite trace
(relative start and duration in microseconds)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
ev = [(s, e, name[:64]) for name, s, e in db.execute("select name,start,end from kernels")]
try:
    for s, e, src, dst in db.execute("select start,end,src_agent_type,dst_agent_type from memory_copies"):
        ev.append((s, e, f"copy {src}->{dst}"))
except sqlite3.Error:
    pass
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
for s, e, name in ev:
    print("%-66s %10.1f %9.1f" % (name, (s - t0) / 1e3, (e - s) / 1e3))
