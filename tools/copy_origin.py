#!/usr/bin/env python
"""Where do the runtime's blit kernels (`__amd_rocclr_copyBuffer` / fill) of a traced step sit?
For every such dispatch in a rocprofv3 results.db: its stream, and the kernels dispatched right
before and after it on the same stream -- maps "copies from below Python" to the op that issued
them.

    python tools/copy_origin.py gpurun_out/prof/run_results.db [--top 20]
"""
import argparse
import collections
import re
import sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return (n.split("(")[0] if "<" not in n.split("(")[0] else n.split("(")[0])[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, stream, start, end from kernels order by start"))
    by_stream = collections.defaultdict(list)
    for r in rows:
        by_stream[r[1]].append(r)
    ctx = collections.Counter()
    per_stream = collections.Counter()
    for st, ks in by_stream.items():
        for i, (n, _, s, e) in enumerate(ks):
            if "rocclr" not in n:
                continue
            per_stream[(st, short(n))] += 1
            prev = short(ks[i - 1][0]) if i else "-"
            nxt = short(ks[i + 1][0]) if i + 1 < len(ks) else "-"
            ctx[(short(n), prev, nxt)] += 1
    print("| stream | blit kernel | count |\n|---|---|---:|")
    for (st, n), k in per_stream.most_common():
        print(f"| {st} | `{n}` | {k} |")
    print("\n| blit | previous kernel (same stream) | next kernel | count |\n|---|---|---|---:|")
    for (n, p, x), k in ctx.most_common(a.top):
        print(f"| `{n}` | `{p}` | `{x}` | {k} |")


if __name__ == "__main__":
    main()
