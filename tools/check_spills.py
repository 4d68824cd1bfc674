"""Register-spill guard for the gfx950 kernels.

LLVM (ROCm 7.2) once miscompiled a PARTIAL spill of an MFMA operand in
block16p_kernel<3, 1, 4, 4, 2>: a 16-byte weight fragment went to scratch as 12 bytes
plus a "Reload Reuse" register that was never restored, and the MFMA read a stale
fourth dword.  A whole-tuple spill -- the value reloaded in full before
its consumer reads it -- is only slow; a split one is the miscompile's shape.

The check, per kernel of the device assembly (what ``honk_amd.build`` keeps from
``-save-temps``):
  * every ``... Folded Reload`` into registers D: the first later instruction that reads
    a register of D must read it through an operand that lies INSIDE D (the tuple the
    spill saved, or a part of it).  An operand reaching past D -- e.g. a 16-byte MFMA
    operand fed by a 12-byte reload -- was assembled from a partial restore: SPLIT;
  * any "Reload Reuse" annotation: SPLIT.
Whole-tuple spills are listed for information.  A SPLIT fails the build (honk_amd.build)
and the CPU test (tests/test_spills.py) unless the kernel is in WHITELIST with a reason.

    python tools/check_spills.py [file.s ...]     (default: honk_amd/_build/*-gfx950.s)
"""
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "honk_amd", "_build")

# kernel-name substring -> why a SPLIT there was reviewed and found benign (none today)
WHITELIST = {}

_REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def _regs(operands):
    out = []
    for m in _REG.finditer(operands):
        if m.group(1):
            out.append((m.group(1), int(m.group(2)), int(m.group(3))))
        else:
            out.append((m.group(4), int(m.group(5)), int(m.group(5))))
    return out


def _demangle(name):
    try:
        return subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip() or name
    except OSError:  # pragma: no cover
        return name


def scan_kernel(body):
    """(status, detail) of one kernel body: status None (no spill), "spill" or "SPLIT"."""
    lines = [ln.split(";", 1) for ln in body.split("\n")]
    sizes, splits = [], []
    if "Reload Reuse" in body:
        splits.append("Reload Reuse annotation")
    for i, parts in enumerate(lines):
        if len(parts) < 2:
            continue
        code, note = parts
        if "Folded Spill" in note:
            sizes.append(re.search(r"(\d+)-byte", note).group(1))
        if "Folded Reload" not in note:
            continue
        dst = _regs(code)
        if not dst:
            continue
        f, a, b = dst[0]
        for code2, *_ in lines[i + 1:]:
            c = code2.strip()
            if not c or c.startswith((".", "s_")):
                continue
            mnem, _, ops = c.partition(" ")
            regs = _regs(ops)
            # the first register operand is the destination, except for stores / LDS writes
            srcs = regs if ("store" in mnem or "write" in mnem) else regs[1:]
            hit = [r for r in srcs if r[0] == f and not (r[2] < a or r[1] > b)]
            if not hit:
                if regs and srcs is not regs and regs[0][0] == f and not (regs[0][2] < a or regs[0][1] > b):
                    break  # redefined before any read
                continue
            wide = [r for r in hit if r[1] < a or r[2] > b]
            if wide:
                splits.append(f"{b - a + 1}-dword reload {f}[{a}:{b}] feeds {f}[{wide[0][1]}:{wide[0][2]}] "
                              f"in `{c[:80]}`")
            break
    if splits:
        return "SPLIT", "; ".join(splits)
    if sizes:
        return "spill", f"{len(sizes)} whole-tuple spills of {sorted(set(sizes), key=int)} bytes"
    return None, ""


def scan_asm(text):
    """[(demangled kernel, status, detail)] for every kernel that spills."""
    out = []
    for m in re.finditer(r"\n(_Z\w+):", text):
        body = text[m.end():text.find(".Lfunc_end", m.end())]
        if "Folded" not in body and "Reload Reuse" not in body:
            continue
        st, detail = scan_kernel(body)
        if st:
            out.append((_demangle(m.group(1)), st, detail))
    return out


def check_files(paths, verbose=True):
    """Returns the SPLIT findings not covered by WHITELIST."""
    bad = []
    for p in paths:
        with open(p) as f:
            for kern, st, detail in scan_asm(f.read()):
                allowed = next((why for k, why in WHITELIST.items() if k in kern), None)
                if verbose:
                    tag = st if not (st == "SPLIT" and allowed) else "split (whitelisted)"
                    print(f"{tag:8s} {os.path.basename(p)}: {kern[:110]}: {detail}")
                if st == "SPLIT" and not allowed:
                    bad.append((p, kern, detail))
    return bad


def default_files():
    return sorted(glob.glob(os.path.join(BUILD, "*-hip-amdgcn-amd-amdhsa-gfx950.s")))


def main():
    paths = sys.argv[1:] or default_files()
    if not paths:
        sys.exit("no device assembly: run `python -m honk_amd.build` first")
    sys.exit(1 if check_files(paths) else 0)


if __name__ == "__main__":
    main()
