#!/usr/bin/env python
"""Print the kernel timeline (start offset us, duration us, stream, name) of the last few steps
of a rocprofv3 rocpd database, to see how gate / bump / collective kernels interleave."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
ks = list(c.execute("select start, end, stream, name from kernels order by start"))
marks = [i for i, k in enumerate(ks) if "sgd" in k[3].lower() or "multi_tensor" in k[3].lower()]
lo = marks[-4] if len(marks) >= 4 else 0
t0 = ks[lo][0]
for s, e, st, n in ks[lo:]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {st!s:>14} {n[:100]}")
