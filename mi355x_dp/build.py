"""Build the in-tree native components for gfx950.

    python -m mi355x_dp.build            # kernels + comm backend + launcher
    python -m mi355x_dp.build kernels    # only libmi355x_kernels.so

Artefacts land in ``mi355x_dp/_native`` (git-ignored, but shipped to the GPU box
with the repo snapshot).  Every HIP source is compiled with
``hipcc --offload-arch=gfx950``; no JIT cache under ~/.cache is used.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
NATIVE = os.path.join(ROOT, "mi355x_dp", "_native")
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("MI355X_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed: " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _digest(paths, extra=""):
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def build_kernels(force=False, verbose=True, debug=False, variant=None, defines=()):
    """debug=True: libmi355x_kernels_debug.so with -DMI_DEBUG (device-side bounds asserts that
    printf the failing index and trap), selected at run time by MI355X_DP_DEBUG_KERNELS=1.
    variant="x", defines=("MI_FOO=1",): an A/B build libmi355x_kernels_x.so with extra -D flags,
    selected at run time by MI355X_DP_KERNEL_VARIANT=x (same process, same shapes, one knob)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    flags = HIP_FLAGS + (["-DMI_DEBUG", "-g"] if debug else []) + [f"-D{d}" for d in defines]
    tag = "debug" if debug else variant
    out = os.path.join(NATIVE, f"libmi355x_kernels_{tag}.so" if tag else "libmi355x_kernels.so")
    stamp = out + ".sha256"
    dig = _digest(srcs + hdrs, " ".join(flags))
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == dig:
        if verbose:
            print(f"[build] {os.path.relpath(out, ROOT)} up to date")
        return out
    os.makedirs(os.path.join(BUILD, "kernels"), exist_ok=True)
    os.makedirs(NATIVE, exist_ok=True)
    objs = []

    def one(src):
        obj = os.path.join(BUILD, "kernels", os.path.basename(src) + (f".{tag}.o" if tag else ".o"))
        _run([HIPCC, *flags, "-c", src, "-o", obj])
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(one, srcs))
    tmp = out + ".tmp"
    _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs])
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(dig)
    if verbose:
        print(f"[build] built {os.path.relpath(out, ROOT)} from {len(srcs)} HIP sources")
    return out


def build_launcher(force=False, verbose=True):
    src = os.path.join(CSRC, "launch", "launcher.cpp")
    if not os.path.exists(src):
        return None
    out = os.path.join(NATIVE, "mi355x_launch")
    stamp = out + ".sha256"
    dig = _digest([src])
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == dig:
        return out
    os.makedirs(NATIVE, exist_ok=True)
    _run(["g++", "-O2", "-std=c++17", "-Wall", "-o", out + ".tmp", src])
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(dig)
    if verbose:
        print(f"[build] built {os.path.relpath(out, ROOT)}")
    return out


def build_comm(force=False, verbose=True):
    src_dir = os.path.join(CSRC, "comm")
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp")) + glob.glob(os.path.join(src_dir, "*.hip")))
    if not srcs:
        return None
    from mi355x_dp.parallel import _smddp_build
    return _smddp_build.build(srcs, NATIVE, force=force, verbose=verbose)


def build_reducer(force=False, verbose=True):
    """csrc/ddp/reducer.cpp -> mi355x_dp/_native/_reducer_ext*.so (libtorch + c10d, HIP events for the
    GPU-side collective timeline)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "ddp", "*.cpp")))
    if not srcs:
        return None
    from mi355x_dp.parallel import _smddp_build
    return _smddp_build.build(srcs, NATIVE, force=force, verbose=verbose, name="_reducer_ext", hip=True)


REF_NOTEBOOKS = os.environ.get("MI355X_DP_REF_SRC", "/root/reference/notebooks")
FIXTURE = os.path.join(ROOT, "ref_fixture", "notebooks")


def stage_reference_fixture(src=REF_NOTEBOOKS, dst=FIXTURE, verbose=True):
    """Copy the reference workshop's notebooks and top-level scripts (no checkpoints) into the
    git-ignored ``ref_fixture/`` so a GPU box -- which has no reference checkout -- can run
    them unmodified (tests/test_gpu_integration.py, tools/run_notebook.py).  Never committed:
    the files are the reference's own, used as test inputs only."""
    if not os.path.isdir(src):
        return None
    os.makedirs(os.path.join(dst, "code"), exist_ok=True)
    names = [f for f in os.listdir(src) if f.endswith(".ipynb")]
    for f in names:
        shutil.copyfile(os.path.join(src, f), os.path.join(dst, f))
    code = os.path.join(src, "code")
    for f in sorted(os.listdir(code)):
        p = os.path.join(code, f)
        if os.path.isfile(p) and f.endswith((".py", ".txt")):
            shutil.copyfile(p, os.path.join(dst, "code", f))
    if verbose:
        print(f"[build] staged reference notebooks/scripts into {os.path.relpath(dst, ROOT)}")
    return dst


def build_all(force=False, verbose=True):
    # the -DMI_DEBUG library is rebuilt with the release one so the two never diverge in symbols
    outs = [build_kernels(force, verbose), build_kernels(force, verbose, debug=True), build_launcher(force, verbose)]
    try:
        outs.append(build_comm(force, verbose))
        outs.append(build_reducer(force, verbose))
    except ImportError:
        pass
    return [o for o in outs if o]


def main(argv=None):
    """`mi355x-build [all|kernels|launcher|comm|reducer] [--force] [--debug]`"""
    argv = sys.argv[1:] if argv is None else argv
    what = next((a for a in argv if not a.startswith("-")), "all")
    force = "--force" in argv
    if what == "kernels":
        build_kernels(force, debug="--debug" in argv)
    elif what == "launcher":
        build_launcher(force)
    elif what == "comm":
        build_comm(force)
    elif what == "reducer":
        build_reducer(force)
    else:
        build_all(force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
