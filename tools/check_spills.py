"""Scan the gfx950 assembly of a csrc file for register spills, and flag PARTIAL
spills of register tuples ("12-byte Folded Spill", "Reload Reuse"): LLVM (ROCm 7.2)
miscompiled one such split in block16p_kernel<3, 1, 4, 4, 2> -- the reloaded MFMA
operand's last dword was never restored.  Whole-tuple spills are
listed for information.

    python tools/check_spills.py [res|cnn|train|...]     (compiles csrc/<name>.hip with -S)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "res"
    src = os.path.join(ROOT, "honk_amd", "csrc", name + ".hip")
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, name + ".s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-Wno-unused-function", "-I", os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                        src, "-o", out], check=True)
        s = open(out).read()
    bad = 0
    for m in re.finditer(r"\n(_Z\w+):", s):
        body = s[m.end():s.find(".Lfunc_end", m.end())]
        sizes = re.findall(r"(\d+)-byte Folded Spill", body)
        reuse = body.count("Reload Reuse")
        if not sizes and not reuse:
            continue
        dem = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        tuples = re.findall(r"scratch_store_dwordx(\d)", body)
        partial = reuse > 0 or any(sz in ("8", "12") for sz in sizes)
        bad += partial
        print(("PARTIAL " if partial else "spill   ") + f"{dem[:100]}: {len(sizes)} spills, sizes "
              f"{sorted(set(sizes))}, reload-reuse {reuse}, tuple stores {tuples}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
