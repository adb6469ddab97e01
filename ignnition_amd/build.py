"""Build libignmp.so in-tree with hipcc for gfx950 (``python -m ignnition_amd.build``).

Every source compiles to its own object (in parallel, under build/), then one link.  kernels_bf.hip
(the split-bf16 kernels) is compiled with MFMA accumulators in VGPRs."""

from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "libignmp.so")
# the resident kernel's phase-A instruction mix (tools/isa_mix.py), read by bench.py's roofline.issue
ISA_MIX = os.path.join(HERE, "isa_mix.json")
SOURCES = ["engine.cpp", "devpool.cpp", "train.cpp", "readout.cpp", "dataset.cpp", "plan_json.cpp", "kernels.hip", "kernels_bf.hip",
           "train_kernels.hip", "readout_kernels.hip", "resident.hip", "readout_h32.hip", "train_csr.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-unused-value"]
EXTRA = {"kernels_bf.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"], "resident.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
         "readout_h32.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "ignmp.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not force and not needs_build():
        tool = os.path.join(HERE, "..", "tools", "isa_mix.py")
        if os.path.exists(tool) and (not os.path.exists(ISA_MIX) or os.path.getmtime(tool) > os.path.getmtime(ISA_MIX)):
            write_isa_mix(hipcc)   # the library is current, the instruction-mix tool is not
        return OUT
    os.makedirs(OBJ, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(OBJ, src + ".o")
        cmd = [hipcc] + FLAGS + EXTRA.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), os.cpu_count() or 1, 8))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = OUT + ".tmp"
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", tmp, "-lz", "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    write_isa_mix(hipcc)
    return OUT


def write_isa_mix(hipcc: str) -> None:
    """bench.py's roofline.issue input.  A diagnostic: a failure here (an asm or parser change, no
    hipcc) warns instead of failing build() -- bench.py runs without the file."""
    try:
        _write_isa_mix(hipcc)
    except Exception as e:   # noqa: BLE001
        print("ignnition_amd.build: warning: isa_mix.json not written (%s)" % e, file=sys.stderr)


def _write_isa_mix(hipcc: str) -> None:
    tool = os.path.join(HERE, "..", "tools", "isa_mix.py")
    if not os.path.exists(tool):
        return
    asm = os.path.join(OBJ, "resident.s")
    subprocess.run([hipcc] + FLAGS + EXTRA["resident.hip"] + ["--cuda-device-only", "-S", "-I", CSRC,
                                                               os.path.join(CSRC, "resident.hip"), "-o", asm], check=True)
    out = subprocess.run([sys.executable, tool, asm], check=True, capture_output=True, text=True).stdout
    with open(ISA_MIX + ".tmp", "w") as f:
        f.write(out)
    os.replace(ISA_MIX + ".tmp", ISA_MIX)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(OUT)
