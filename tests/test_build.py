"""Compile-only checks of the HIP sources' non-default build variants (no GPU needed:
hipcc cross-compiles gfx950 here). The product library is built with the defaults
(ilqr.jl_amd/csrc/Makefile); the alternates below are measured ablations kept for the
record, so they are compiled here to keep them from rotting unseen."""
import os
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ilqr.jl_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_chain_macro_alternates_compile(tmp_path):
    """ilqr_chain.hip with the Rodrigues-form central differences
    (ILQR_CHAIN_FD_ROT=0), the unpacked ±h evaluation (ILQR_CHAIN_FD_PAIR=0) and the
    unpacked fp32 closed-form step (ILQR_CHAIN_F2_FAST=0)."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
           "-fno-slp-vectorize", "-DILQR_CHAIN_FD_ROT=0", "-DILQR_CHAIN_FD_PAIR=0", "-DILQR_CHAIN_F2_FAST=0", "-c",
           os.path.join(CSRC, "ilqr_chain.hip"), "-o", str(tmp_path / "chain_alt.o")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_forward_ring_alternates_compile(tmp_path):
    """ilqr_lq.hip's ring forward with the LDS row broadcasts (ILQR_FW_LDS_BCAST=1,
    bit-identical, measured slower), one-wave workgroups (ILQR_FW_WAVES=1) and the
    ablation bits (ILQR_FW_ABLATE=3) that tools/fw_alt.sh builds."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DILQR_FW_LDS_BCAST=1",
           "-DILQR_FW_WAVES=1", "-DILQR_FW_ABLATE=3", "-c", os.path.join(CSRC, "ilqr_lq.hip"),
           "-o", str(tmp_path / "lq_alt.o")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_twolink_alternates_compile(tmp_path):
    """ilqr_twolink.hip without the branch-free shifted-sincos RK4 (ILQR_TL_RK4_SHIFT=0:
    the forward group's robust pass only) and with a 4-deep forward prefetch."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
           "-DILQR_TL_RK4_SHIFT=0", "-DILQR_FW_GROUP_PF=4", "-c", os.path.join(CSRC, "ilqr_twolink.hip"),
           "-o", str(tmp_path / "tl_alt.o")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_backward4_alternates_compile(tmp_path):
    """ilqr_bw4.hip with the round-2 instruction cuts undone — μ added in the
    factorisation (ILQR_BW4_MU_IN_H=0), select chains for the solve's per-lane operands
    (ILQR_BW4_SEL_FMA=0), lower S blocks by lane permutation (ILQR_BW4_SLOW_MFMA=0),
    transposes by permutation (ILQR_BW4_MFMA_T=0) — and the forward's slot loads without
    the non-temporal hint (ILQR_FW_LD_NT=0): the A/B baselines of tools/bw_alt.sh."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
           "-DILQR_BW4_MU_IN_H=0", "-DILQR_BW4_SEL_FMA=0", "-DILQR_BW4_SLOW_MFMA=0", "-DILQR_BW4_MFMA_T=0",
           "-DILQR_FW_LD_NT=0", "-c", os.path.join(CSRC, "ilqr_bw4.hip"), "-o", str(tmp_path / "bw4_alt.o")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
