#!/usr/bin/env python
"""Run a notebook's code cells in order in one namespace (no jupyter in the image):

    cd notebooks && NB_EPOCHS=1 python ../tools/run_notebook.py 1_pytorch_dist_native_cpu.ipynb

Reference notebooks are run VERBATIM (no cell is edited) with ``--compat``: the repo and its
import-path compat packages (sagemaker, boto3, torchvision, smdistributed) are put on
``sys.path`` the way an installed SDK would be, and ``--workdir`` copies the notebook's
directory (its ``code/`` source_dir) to a scratch dir that becomes the cwd:

    python tools/run_notebook.py --compat --workdir /tmp/nb2 --report /tmp/nb2.json \\
        ref_fixture/notebooks/2_pytorch_dist_smddp_gpu.ipynb

``--keep-going`` runs every cell even after one fails and ``--report`` writes per-cell
status (ok / error with the exception line / seconds) as JSON; the exit status is non-zero
when any cell failed that is not listed in ``--expect-fail``.
"""
import argparse
import json
import os
import shutil
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(path, keep_going=False, expect_fail=()):
    cells = json.load(open(path))["cells"]
    ns = {"__name__": "__main__"}
    report = []
    for i, c in enumerate(cells):
        if c["cell_type"] != "code":
            continue
        src = "".join(c["source"])
        print(f"--- cell {i}", flush=True)
        t0 = time.time()
        try:
            exec(compile(src, f"{os.path.basename(path)}:cell{i}", "exec"), ns)
            report.append({"cell": i, "status": "ok", "seconds": round(time.time() - t0, 2)})
        except BaseException as e:  # noqa: BLE001 -- a notebook cell may raise anything, SystemExit included
            line = f"{type(e).__name__}: {e}".splitlines()[0][:300]
            traceback.print_exc()
            report.append({"cell": i, "status": "error", "error": line, "seconds": round(time.time() - t0, 2),
                           "expected": i in expect_fail})
            if not keep_going:
                break
    return report


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("notebook")
    ap.add_argument("--compat", action="store_true", help="put the repo + compat packages on sys.path")
    ap.add_argument("--workdir", help="copy the notebook's directory here and run with it as cwd")
    ap.add_argument("--keep-going", action="store_true")
    ap.add_argument("--expect-fail", default="", help="comma-separated cell indices documented to fail")
    ap.add_argument("--report", help="write per-cell JSON status here")
    a = ap.parse_args(argv)
    nb = os.path.abspath(a.notebook)
    if a.report:
        a.report = os.path.abspath(a.report)
    if a.compat:
        sys.path.insert(0, ROOT)
        sys.path.append(os.path.join(ROOT, "compat"))
        os.environ["PYTHONPATH"] = os.pathsep.join(
            p for p in (ROOT, os.environ.get("PYTHONPATH"), os.path.join(ROOT, "compat")) if p)
    if a.workdir:
        if os.path.exists(a.workdir):
            shutil.rmtree(a.workdir)
        shutil.copytree(os.path.dirname(nb), a.workdir,
                        ignore=shutil.ignore_patterns(".ipynb_checkpoints", "shadow_model_ckpt"))
        nb = os.path.join(a.workdir, os.path.basename(nb))
        os.chdir(a.workdir)
    expect = {int(x) for x in a.expect_fail.split(",") if x.strip()}
    t0 = time.time()
    report = run(nb, a.keep_going, expect)
    wall = time.time() - t0
    if a.report:
        with open(a.report, "w") as f:
            json.dump({"notebook": os.path.basename(nb), "wall_s": round(wall, 2), "cells": report}, f, indent=1)
    bad = [r for r in report if r["status"] != "ok" and not r.get("expected")]
    print(f"--- notebook done in {wall:.1f}s: {sum(r['status'] == 'ok' for r in report)} ok, "
          f"{len(report) - sum(r['status'] == 'ok' for r in report)} failed "
          f"({len(bad)} unexpected)", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
