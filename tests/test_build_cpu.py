"""Build-quality gates that run without a GPU: every HIP source compiles for gfx950 and the hot
MFMA kernels neither spill to scratch nor exceed the VGPR budget of their launch bounds."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip"))))
def test_kernels_compile_without_scratch(src, tmp_path):
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o",
                        str(tmp_path / "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    names = re.findall(r"Function Name: (\S+)", r.stderr)
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", r.stderr)]
    vgprs = [int(x) for x in re.findall(r"\bVGPRs: (\d+)", r.stderr)]
    assert len(names) == len(scratch) == len(vgprs) and names
    for n, sc, vg in zip(names, scratch, vgprs):
        assert sc == 0, f"{n} spills {sc} B/lane to scratch"
        if "gemm256" in n:
            assert vg <= 256, f"{n} uses {vg} VGPRs (> 2 waves/SIMD budget)"
        elif "nt_kernel" in n or "tn_kernel" in n:
            assert vg <= 168, f"{n} uses {vg} VGPRs (> 3 waves/SIMD budget)"
