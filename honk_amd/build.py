"""Build libhonk_hip.so (gfx950) in-tree with hipcc.  No torch in the ABI.

    python -m honk_amd.build          # or __graft_entry__.build()
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhonk_hip.so")
SOURCES = ["runtime.cpp", "res.hip", "res_vf.hip", "cnn.hip", "train.hip", "mfcc.hip", "head.hip", "augment.hip"]
# per-source extra flags / dependencies: res_vf.hip (the f16x2 pair and last-layer kernels)
# includes res.hip and takes the MFMA accumulators in VGPRs (see its header)
FLAGS = {"res_vf.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}
DEPS = {"res_vf.hip": ["res.hip"]}
ARCH = os.environ.get("HONK_OFFLOAD_ARCH", "gfx950")


def asm_path(build_dir, src):
    """The device assembly -save-temps=obj keeps for one source (the spill guard's input)."""
    return os.path.join(build_dir, src.rsplit(".", 1)[0] + f"-hip-amdgcn-amd-amdhsa-{ARCH}.s")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libhonk_hip.so)")


def needs_build():
    if not os.path.exists(LIB):
        return True
    tmp = os.path.join(HERE, "_build")
    for src in SOURCES:  # the device assembly the spill guard reads
        if src.endswith(".hip") and not os.path.exists(asm_path(tmp, src)):
            return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [
        os.path.join(HERE, "..", "include", "honk_hip.h")]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def check_spills(build_dir):
    """Fail the build on a SPLIT register spill (a reload that restores part of a tuple an
    MFMA or other instruction then reads whole: the shape of the LLVM miscompile that gave
    wrong bf16 logits in round 4) -- tools/check_spills.py over the device assembly."""
    sys.path.insert(0, os.path.join(HERE, "..", "tools"))
    try:
        import check_spills as cs
    finally:
        sys.path.pop(0)
    # exactly the current sources' assembly (not stale files of removed sources); every
    # .hip source must have produced one, or the guard would silently scan nothing
    paths = [asm_path(build_dir, src) for src in SOURCES if src.endswith(".hip")]
    missing = [p for p in paths if not os.path.exists(p)]
    if missing:
        raise RuntimeError("spill guard: no device assembly for " + ", ".join(map(os.path.basename, missing)))
    bad = cs.check_files(paths, verbose=False)
    if bad:
        raise RuntimeError("split register spills (tools/check_spills.py):\n" +
                           "\n".join(f"  {os.path.basename(p)}: {k}: {d}" for p, k, d in bad))


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    objs = []
    tmp = os.path.join(HERE, "_build")
    os.makedirs(tmp, exist_ok=True)
    # -save-temps=obj keeps each file's device assembly (<src>-hip-amdgcn-amd-amdhsa-gfx950.s in
    # _build/): the code the objects hold, which the spill guard below reads
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-save-temps=obj", "-I", os.path.join(HERE, "..", "include")]
    procs = []
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))] + [
        os.path.join(HERE, "..", "include", "honk_hip.h")]
    for src in SOURCES:
        obj = os.path.join(tmp, src.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        # incremental: an object newer than its source and every shared header is kept
        asm = asm_path(tmp, src)
        if not force and os.path.exists(obj) and (os.path.exists(asm) or not src.endswith(".hip")) and all(
                os.path.getmtime(obj) > os.path.getmtime(p)
                for p in [os.path.join(CSRC, f) for f in [src] + DEPS.get(src, [])] + headers):
            continue
        cmd = base + FLAGS.get(src, []) + (["-x", "hip"] if src.endswith(".cpp") else []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out}")
        if verbose and out.strip():
            print(out)
    check_spills(tmp)
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
