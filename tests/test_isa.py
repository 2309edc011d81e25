"""ISA regression guards for the headline kernels (CPU only: hipcc cross-compiles
gfx950 here). Compiles ilqr_bw4.hip (the fused iteration, the backward) with the
product flags and -save-temps, then checks the generated gfx950 assembly for two
code-generation traps found by reading the ISA (late round 2):
  * waterfall loops — a buffer access whose resource or scalar offset the compiler
    cannot prove wave-uniform becomes a `v_readfirstlane` / `s_and_saveexec` /
    `s_cbranch_execnz` loop around every load or store (the ring forward's x̄/ū stores
    and the chain backward's gain stores were such loops);
  * scratch (private-memory spills) in the step loops."""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ilqr.jl_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _functions(asm):
    """{mangled kernel name: list of instruction lines}"""
    out, cur = {}, None
    for line in asm.split("\n"):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
        elif cur is not None:
            out[cur].append(re.sub(r"\s+", " ", line.strip()))
    return out


def _waterfalls(body):
    """loops that branch back on execnz around a readfirstlane and a memory access"""
    labels = {}
    for k, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = k
    found = []
    for k, l in enumerate(body):
        m = re.search(r"s_cbranch_execnz (\.LBB\w+)", l)
        if m and labels.get(m.group(1), 1 << 30) < k:
            seg = body[labels[m.group(1)]:k + 1]
            # the waterfall's signature: exec narrowed to the lanes matching the
            # readfirstlane'd value, the access, then `s_xor_b64 exec, exec, …` and the
            # branch back (a backward execnz branch of an ordinary if/else block layout
            # has no exec-destination xor)
            if (any("v_readfirstlane" in x for x in seg) and any(x.startswith(("buffer_", "global_")) for x in seg)
                    and any(x.startswith("s_xor_b64 exec, exec") for x in seg)):
                found.append(k)
    return found


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_headline_kernels_have_no_waterfall_loops_or_scratch(tmp_path):
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
           "-save-temps", "-c", os.path.join(CSRC, "ilqr_bw4.hip"), "-o", str(tmp_path / "bw4.o")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    asm_file = [f for f in os.listdir(tmp_path) if f.endswith("gfx950.s")]
    assert asm_file, os.listdir(tmp_path)
    funcs = _functions(open(tmp_path / asm_file[0]).read())
    # the default (row-form forward) fused iteration, the fit's backward leg and the
    # ilqr_backward kernel
    checked = [n for n in funcs if re.search(r"lq_iter_fused4_kernelILb0E|lq_iter_backward4_kernel|"
                                             r"lq_backward4_kernelE", n)]
    assert len(checked) == 3, sorted(funcs)
    for n in checked:
        body = funcs[n]
        assert not _waterfalls(body), f"{n}: waterfall loop(s) at {_waterfalls(body)}"
        assert not [x for x in body if x.startswith("scratch_")], f"{n}: scratch accesses"


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_tiles_kernels_have_no_scratch(tmp_path):
    """The tiles backward (row f3): the wide kernel (nx ≤ 16, nu ≤ 8, run-time shapes,
    256 VGPRs + AGPRs at one wave per SIMD) and every narrow instantiation keep their
    prefetched tiles, LDLᵀ factors and dynamically selected solution entries in
    registers — a dynamically indexed register array (the first draft's g vector) or a
    spill would be a scratch access per step.

    And the step-ahead tile loads stay in flight across the step: inside the step loop,
    no `s_waitcnt vmcnt` may sit between the loop header and the last prefetch load.
    Before the opaque load-or-zero (`ldz_async`, DESIGN "The prefetch that waited") the
    wide kernel's loads were exec-masked branches, each joined by a `vmcnt(0)`, so every
    step waited for its successor's tiles before its first MFMA — 2.06 ms instead of
    1.10 ms for 16 × 8 at B = 4096 (`profiles/r05/tiles_bench_async_r05.log`). Both load
    paths are checked: ldz_async (small batches) and raw buffer loads (large ones)."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
           "-save-temps", "-c", os.path.join(CSRC, "ilqr_tiles.hip"), "-o", str(tmp_path / "tiles.o")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    asm_file = [f for f in os.listdir(tmp_path) if f.endswith("gfx950.s")]
    funcs = _functions(open(tmp_path / asm_file[0]).read())
    kernels = [n for n in funcs if "tiles_backward" in n and "kernel" in n]
    assert any("wide" in n for n in kernels) and len(kernels) >= 49, len(kernels)
    for n in kernels:
        body = funcs[n]
        assert not [x for x in body if x.startswith("scratch_")], f"{n}: scratch accesses"
        headers = [i for i, x in enumerate(body) if "Loop Header" in x]
        assert len(headers) == 1, f"{n}: step loop headers at {headers}"
        h = headers[0]
        loads = [i for i, x in enumerate(body) if i > h and x.startswith(("global_load", "buffer_load"))]
        assert loads, f"{n}: no prefetch loads in the step loop"
        # a wait before the last prefetch load may only drain loads of earlier steps:
        # vmcnt(N) leaves the newest N in flight, so N must cover every load this step
        # has issued by then (vmcnt(0) mid-prefetch was the bug)
        bad = []
        for w in range(h, loads[-1]):
            m = re.search(r"vmcnt\((\d+)\)", body[w])
            if m and int(m.group(1)) < sum(1 for i in loads if h < i < w):
                bad.append(body[w])
        assert not bad, f"{n}: the step waits on its own prefetch before issuing it all: {bad[:4]}"


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_floating_kernels_have_no_scratch(tmp_path):
    """The floating-base family (ilqr_floating.hip): the dual-number linearisation keeps
    ~460 registers at one wave per SIMD, the three-wave forward ~290; the model's
    constants are re-read per RK4 stage instead of hoisted — hoisted, they had spilled
    to scratch (364 and 140 bytes per lane), and so did a two-wave forward whose second
    wave took both the mass and the solve (184 bytes)."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    cmd = [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=on", "-save-temps", "-c",
           os.path.join(CSRC, "ilqr_floating.hip"), "-o", str(tmp_path / "fl.o")]  # as the Makefile
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    asm_file = [f for f in os.listdir(tmp_path) if f.endswith("gfx950.s")]
    funcs = _functions(open(tmp_path / asm_file[0]).read())
    kernels = [n for n in funcs if re.search(r"fb_(dynamics|linearize|forward)_kernel", n)]
    assert len(kernels) == 5, sorted(funcs)  # the forward at 4, 16 and 64 lanes a trajectory
    for n in kernels:
        assert not [x for x in funcs[n] if x.startswith("scratch_")], f"{n}: scratch accesses"
        # the forward's LDS exchange as ds_ ops: a flat access waits on global loads too
        assert not [x for x in funcs[n] if x.startswith("flat_")], f"{n}: flat accesses"
