"""python -m mi355x_dp.trace [--steps N] [--out DIR] -- <command...>

Runs the command under rocprofv3 (kernel trace + stats) and prints a markdown per-kernel
summary (ms per step, share, calls, average) -- the format of profiles/*.md."""
import argparse
import os
import subprocess
import sys

from . import rocprof_cmd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1, help="training steps covered by the command (for per-step)")
    ap.add_argument("--out", default="gpurun_out/trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    os.makedirs(a.out, exist_ok=True)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    rc = subprocess.run(rocprof_cmd(cmd, a.out), env=env).returncode
    if rc != 0:
        sys.exit(rc)
    here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    summ = os.path.join(here, "tools", "prof_summary.py")
    subprocess.run([sys.executable, summ, os.path.join(a.out, "run_kernel_stats.csv"), "--steps", str(a.steps),
                    "--top", str(a.top)])


if __name__ == "__main__":
    main()
