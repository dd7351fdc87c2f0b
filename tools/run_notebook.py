#!/usr/bin/env python
"""Run a notebook's code cells in order in one namespace (no jupyter in the image):

    cd notebooks && NB_EPOCHS=1 python ../tools/run_notebook.py 1_pytorch_dist_native_cpu.ipynb
"""
import json
import sys


def run(path):
    cells = json.load(open(path))["cells"]
    ns = {"__name__": "__main__"}
    for i, c in enumerate(cells):
        if c["cell_type"] != "code":
            continue
        src = "".join(c["source"])
        print(f"--- cell {i}", flush=True)
        exec(compile(src, f"{path}:cell{i}", "exec"), ns)


if __name__ == "__main__":
    run(sys.argv[1])
