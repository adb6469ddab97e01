"""Instruction mix of the graph-resident forward's ordered-update step (phase A), from the gfx950
assembly hipcc emits for csrc/resident.hip -- the input of bench.py's roofline.issue.

The step loop is the innermost loop whose blocks issue the 18 split-fp16 MFMAs of one tile-step
(v_mfma_f32_16x16x32_f16: 3 products x 3 gates x 2 column tiles).  Its instructions are classed as
the SIMD issues them (MI355X_MICROARCH.md, constants table, 'vector-instruction ISSUE cost'):
transcendental VALU (v_exp/v_log/v_rcp/v_rsq/v_sqrt/v_sin/v_cos: 8 cycles per wave64), packed f32 VALU
(v_pk_*_f32: 4), other VALU (2 on the SIMD-32 at throughput), MFMA 16x16x32 (16 cycles of the matrix
pipe, 8 of them holding the vector issue), LDS, vector memory, scalar.

    python tools/isa_mix.py [resident.s]     # prints the JSON; build.py writes ignnition_amd/isa_mix.json
"""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "ignnition_amd", "csrc")
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")
# issue cycles per wave64 instruction on one SIMD at throughput (VALU over the SIMD-32's 2 cycles;
# transcendentals at quarter rate; an MFMA holds the vector issue 8 of its 16 cycles)
CYC = {"valu": 2, "valu_pk": 4, "trans": 8, "mfma16_hold": 8, "mfma16_pipe": 16}


def assemble(src=os.path.join(CSRC, "resident.hip")) -> str:
    out = os.path.join(tempfile.mkdtemp(prefix="ign_isa_"), "resident.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm",
                    "-amdgpu-mfma-vgpr-form", "--cuda-device-only", "-S", "-I", CSRC, src, "-o", out],
                   check=True, capture_output=True, timeout=600)
    return open(out).read()


def _blocks(asm: str, kernel: str):
    i = asm.index("\n" + kernel + ":")
    j = asm.index(".Lfunc_end", i)
    blocks, cur = [], None
    for line in asm[i:j].splitlines():
        m = re.match(r"^\.LBB(\d+_\d+):(.*)", line)
        if m:
            hdr = re.search(r"Header=BB(\d+_\d+) Depth=(\d+)", m.group(2))
            own = re.search(r"Loop Header: Depth=(\d+)", m.group(2))
            cur = {"label": m.group(1), "loop": hdr.group(1) if hdr else (m.group(1) if own else None),
                   "depth": int(hdr.group(2)) if hdr else (int(own.group(1)) if own else 0), "ins": []}
            blocks.append(cur)
            continue
        t = line.strip()
        if cur is None or not t or t.startswith((";", ".")):
            continue
        cur["ins"].append(t.split()[0])
    return blocks


def classify(ins):
    c = {"valu": 0, "valu_pk": 0, "trans": 0, "mfma16": 0, "mfma_other": 0, "lds": 0, "vmem": 0, "salu": 0,
         "branch_wait": 0}
    for x in ins:
        if x.startswith("v_mfma_f32_16x16x32"):
            c["mfma16"] += 1
        elif x.startswith("v_mfma"):
            c["mfma_other"] += 1
        elif x.startswith(TRANS):
            c["trans"] += 1
        elif x.startswith("v_pk_") and x.endswith("_f32"):
            c["valu_pk"] += 1
        elif x.startswith("v_"):
            c["valu"] += 1
        elif x.startswith("ds_"):
            c["lds"] += 1
        elif x.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
        elif x.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_barrier", "s_sleep")):
            c["branch_wait"] += 1
        else:
            c["salu"] += 1
    return c


def step_mix(asm: str, kernel: str) -> dict:
    """The innermost loop holding a block of 18 v_mfma_f32_16x16x32_f16 (one tile-step): the
    instruction classes of that block (the MFMAs and the unmasked step's gates) plus the loop's
    bookkeeping blocks.  The masked step (t >= the tile's shortest length) is a second copy of the
    gates, one exec-guarded block per element, which a tile-step runs instead of, not besides, the
    unmasked gates: blocks with transcendentals other than the MFMA block are that copy and are left
    out (counting them too gave 1 526 cycles, more than the measured 1 291)."""
    bl = _blocks(asm, kernel)
    best = None
    for b in bl:
        if sum(1 for x in b["ins"] if x == "v_mfma_f32_16x16x32_f16") == 18 and b["loop"]:
            if best is None or b["depth"] > best["depth"]:
                best = b
    if best is None:
        raise RuntimeError("no 18-MFMA step loop in %s" % kernel)
    body = [x for b in bl if b["loop"] == best["loop"] and b["depth"] == best["depth"] and
            (b is best or classify(b["ins"])["trans"] == 0) for x in b["ins"]]
    c = classify(body)
    vec = c["valu"] * CYC["valu"] + c["valu_pk"] * CYC["valu_pk"] + c["trans"] * CYC["trans"] + \
        c["mfma16"] * CYC["mfma16_hold"]
    c["vector_issue_cycles"] = vec
    c["mfma_pipe_cycles"] = c["mfma16"] * CYC["mfma16_pipe"]
    c["cycles_per_tile_step"] = max(vec, c["mfma_pipe_cycles"])
    c["loop"] = best["loop"]
    return c


def main(argv):
    asm = open(argv[1]).read() if len(argv) > 1 else assemble()
    out = {"cycle_model": CYC, "kernels": {}}
    for name in re.findall(r"^(_Z23resident_forward_kernel\w*):", asm, re.M):
        out["kernels"][name] = step_mix(asm, name)
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    main(sys.argv)
