"""ISA checks of the readout and ordered-update kernels (CPU: hipcc cross-compiles gfx950 to assembly, no GPU).

readout_bf_kernel and readout_h16_kernel issue their W2-chunk LDS-DMA as inline asm that loads M0, a register the compiler
reserves (csrc/kernels_bf.hip): that is only sound while nothing else in the kernel uses M0.  The
DIN-32 selu instances must also stay free of register spills (their chunk loops run at 204-244 VGPRs)."""
import os
import re
import subprocess

import pytest

HIPCC = "/opt/rocm/bin/hipcc"
SRC = os.path.join(os.path.dirname(__file__), "..", "ignnition_amd", "csrc", "kernels_bf.hip")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "kernels_bf.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-amdgpu-mfma-vgpr-form",
                    "--cuda-device-only", "-S", "-I", os.path.dirname(SRC), SRC, "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    return out.read_text()


@pytest.fixture(scope="module")
def asm_resident(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    src = os.path.join(os.path.dirname(SRC), "resident.hip")
    out = tmp_path_factory.mktemp("isa") / "resident.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-amdgpu-mfma-vgpr-form",
                    "--cuda-device-only", "-S", "-I", os.path.dirname(SRC), src, "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    return out.read_text()


def _functions(asm, pattern):
    for name in re.findall(r"^(%s\w*):" % pattern, asm, re.M):
        i = asm.index("\n" + name + ":")
        j = asm.index(".Lfunc_end", i)
        yield name, asm[i:j], asm[j:j + 4000]


def test_readout_m0_only_feeds_the_lds_dma(asm):
    seen = 0
    for name, body, _ in _functions(asm, "_Z1[78]readout_(?:bf|h16)_kernel"):
        lines = [l.strip() for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((";", "."))]
        for k, l in enumerate(lines):
            if "m0" not in l:
                continue
            assert re.match(r"s_mov_b32 m0, s\d+$", l), (name, l)
            nxt = next(x for x in lines[k + 1:] if not x.startswith("s_nop"))
            assert nxt.startswith("global_load_lds_dwordx4"), (name, l, nxt)
            seen += 1
    assert seen > 0


def test_default_readout_has_no_spills(asm):
    found = False
    for name, body, meta in _functions(asm, r"_Z1(?:7readout_bf_kernelILi32ELi2ELi8ELi6ELi1ELb1ELi2ELb1E|8readout_h16_kernelILi32ELi2ELi8ELi2E)"):
        found = True
        scratch = re.search(r"ScratchSize: (\d+)", meta)
        assert scratch and int(scratch.group(1)) == 0, name
    assert found


def test_default_ordered_update_keeps_four_waves(asm):
    """seq_gru_h16<32, 3> (the default ordered update) at 4 waves per SIMD: at most 128 VGPRs and
    no scratch; 5-6 waves (fewer registers) and 3 waves (a register prefetch) both measured slower
    (DESIGN.md §3b')."""
    found = False
    for name, body, meta in _functions(asm, r"_Z18seq_gru_h16_kernelILi32ELi3E"):
        found = True
        vgpr = re.search(r"NumVgprs: (\d+)", meta)
        scratch = re.search(r"ScratchSize: (\d+)", meta)
        if "Lb0E" in name:   # the inference form; the state-saving training form (Lb1E) may use more
            assert vgpr and int(vgpr.group(1)) <= 128, (name, vgpr and vgpr.group(1))
        else:                # the training forward at H = 32 (138 VGPRs in round 3): keep its 3 waves per SIMD
            assert vgpr and int(vgpr.group(1)) <= 168, (name, vgpr and vgpr.group(1))
        assert scratch and int(scratch.group(1)) == 0, name
    assert found


def test_resident_forward_fits_its_workgroup(asm_resident):
    """resident_forward_kernel: 16 waves (one workgroup per graph) need <= 128 VGPRs; no scratch in
    any of its five instances -- three forms of the forward, two of the training forward's SAVE
    variant (the per-lane fragment addresses stay inside the loops)."""
    found = 0
    for name, body, meta in _functions(asm_resident, r"_Z23resident_forward_kernel"):
        found += 1
        vgpr = re.search(r"NumVgprs: (\d+)", meta)
        scratch = re.search(r"ScratchSize: (\d+)", meta)
        print(name, vgpr.group(1), scratch.group(1))
        assert vgpr and int(vgpr.group(1)) <= 128, name
        if name.endswith("ELb1EEv12ResidentArgs"):   # SAVE: a few 4-8 B reloads per tile, none per step
            assert scratch and int(scratch.group(1)) <= 96, name
            # phase A's step loop: from the loop header that precedes the first split-fp16 MFMA to
            # the last branch back to it
            m = body.index("v_mfma_f32_16x16x32_f16")
            h = body.rindex("Loop Header", 0, m)
            label = re.findall(r"^(\.LBB\w+):", body[:h], re.M)[-1]
            start, back = body.index(label + ":"), body.rindex(label, m)
            assert back > m and "scratch_" not in body[start:back], name
        else:
            assert scratch and int(scratch.group(1)) == 0, name
    assert found == 5
