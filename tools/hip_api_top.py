#!/usr/bin/env python
"""Host-side HIP API time from a rocprofv3 --hip-trace rocpd database: per API call name, count,
total and max duration (which runtime call blocks the host)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables:", ", ".join(n for n in names if not n.startswith("sqlite")))
src = next((n for n in ("regions", "region", "hip_api", "api") if n in names), None)
if src is None:
    src = next((n for n in names if "region" in n.lower() or "api" in n.lower()), None)
cols = [r[1] for r in c.execute(f"pragma table_info({src})")]
print("source:", src, cols)
rows = list(c.execute(f"select name, count(*), sum(end - start), max(end - start) from {src} group by name "
                      "order by sum(end - start) desc limit 40"))
print("| api | calls | total ms | max us |\n|---|---:|---:|---:|")
for n, k, t, m in rows:
    print(f"| {n[:60]} | {k} | {t / 1e6:.2f} | {m / 1e3:.1f} |")
