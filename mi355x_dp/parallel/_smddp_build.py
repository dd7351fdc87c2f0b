"""Build the native smddp backend extension in-tree (no JIT cache): one g++ invocation
against torch's headers/libraries and ROCm's RCCL, output ``mi355x_dp/_native/_smddp_native_ext*.so``."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sysconfig

EXT_NAME = "_smddp_native_ext"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def ext_path(native_dir, name=EXT_NAME):
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(native_dir, name + suffix)


def build(srcs, native_dir, force=False, verbose=True, name=EXT_NAME, hip=True):
    """g++ a torch extension in-tree.  ``hip``: link the ROCm runtime / RCCL (the smddp
    backend); the reducer only needs libtorch + c10d."""
    import torch
    from torch.utils import cpp_extension as ce

    out = ext_path(native_dir, name)
    h = hashlib.sha256()
    for s in srcs:
        h.update(open(s, "rb").read())
    h.update(torch.__version__.encode())
    dig = h.hexdigest()
    stamp = out + ".sha256"
    if not force and os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == dig:
        if verbose:
            print(f"[build] {os.path.basename(out)} up to date")
        return out
    cpp = [s for s in srcs if s.endswith(".cpp")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = ce.include_paths() + [sysconfig.get_paths()["include"], os.path.join(ROCM, "include")]
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           f"-DTORCH_EXTENSION_NAME={name}", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    cmd += [f"-I{d}" for d in inc]
    cmd += cpp
    cmd += [f"-L{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
    if hip:
        cmd += ["-lc10_hip", "-ltorch_hip", f"-L{os.path.join(ROCM, 'lib')}", "-lrccl", "-lamdhip64"]
    cmd += [f"-Wl,-rpath,{libdir}", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}", "-o", out + ".tmp"]
    os.makedirs(native_dir, exist_ok=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{name} build failed:\n" + r.stdout[-6000:])
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(dig)
    if verbose:
        print(f"[build] built {os.path.relpath(out)}")
    return out
