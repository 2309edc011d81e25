"""Compile-only check of the measured build alternates (no GPU needed: hipcc
cross-compiles gfx950 here). The product sources hold one path per kernel; the
alternates they were measured against — the backward's round-2
instruction cuts undone and its probe bits (ABL), the one-wave backward's variants,
the ring forward's LDS row broadcasts, cache hints and timing-only ablations, the
chain's Rodrigues-form / unpacked evaluations, the 2-link forward on the generic RK4
— live in tools/archive/ablation/restore_alternates.patch. This test applies the patch to a
copy of the current sources and compiles them with the alternates switched on, so
that record stays reproducible against the product tree."""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCH = os.path.join(ROOT, "tools", "archive", "ablation", "restore_alternates.patch")
HIPCC = "/opt/rocm/bin/hipcc"


def _hipcc():
    return HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")


@pytest.mark.skipif(_hipcc() is None or shutil.which("patch") is None, reason="no hipcc / patch")
def test_restore_alternates_patch_builds(tmp_path):
    os.makedirs(tmp_path / "ilqr.jl_amd")
    shutil.copytree(os.path.join(ROOT, "ilqr.jl_amd", "csrc"), tmp_path / "ilqr.jl_amd" / "csrc")
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "include")
    with open(PATCH) as f:
        r = subprocess.run(["patch", "-p1", "--fuzz=3", "--no-backup-if-mismatch", "-s"], stdin=f,
                           cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, "restore_alternates.patch no longer applies: " + r.stdout + r.stderr
    csrc = tmp_path / "ilqr.jl_amd" / "csrc"
    base = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c"]
    mf = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
    jobs = [
        # the backward with the round-2 instruction cuts undone, slot loads without nt
        mf + ["-DILQR_BW4_MU_IN_H=0", "-DILQR_BW4_SEL_FMA=0", "-DILQR_BW4_SLOW_MFMA=0",
              "-DILQR_BW4_MFMA_T=0", "-DILQR_FW_LD_NT=0", "ilqr_bw4.hip"],
        # the ring forward's LDS row broadcasts, one-wave workgroups, ablation bits
        ["-DILQR_FW_LDS_BCAST=1", "-DILQR_FW_WAVES=1", "-DILQR_FW_ABLATE=3", "ilqr_lq.hip"],
        # the 2-link forward on the generic RK4 with a 4-deep prefetch
        mf + ["-DILQR_TL_RK4_SHIFT=0", "-DILQR_FW_GROUP_PF=4", "ilqr_twolink.hip"],
        # the chain's Rodrigues-form central differences, unpacked ±h and fp32 step
        mf + ["-fno-slp-vectorize", "-DILQR_CHAIN_FD_ROT=0", "-DILQR_CHAIN_FD_PAIR=0",
              "-DILQR_CHAIN_F2_FAST=0", "ilqr_chain.hip"],
    ]

    def build(args):
        src = args[-1]
        cmd = base + args[:-1] + [str(csrc / src), "-o", str(tmp_path / (src + ".o"))]
        return src, subprocess.run(cmd, capture_output=True, text=True, timeout=900)

    with ThreadPoolExecutor(4) as ex:
        for src, r in ex.map(build, jobs):
            assert r.returncode == 0, (src, r.stderr[-2000:])
