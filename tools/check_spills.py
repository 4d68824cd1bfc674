"""Register-spill guard for the gfx950 kernels.

LLVM (ROCm 7.2) once miscompiled a PARTIAL spill of an MFMA operand in
block16p_kernel<3, 1, 4, 4, 2>: a 16-byte weight fragment went to scratch as 12 bytes
plus a "Reload Reuse" register that was never restored, and the MFMA read a stale
fourth dword.  A whole-tuple spill -- the value reloaded in full before
its consumer reads it -- is only slow; a split one is the miscompile's shape.

The check, per kernel of the device assembly (what ``honk_amd.build`` keeps from
``-save-temps``):
  * every ``... Folded Reload`` into registers D: EVERY later read of a register of D
    while it still holds the reloaded value must go through an operand that lies INSIDE
    D (the tuple the spill saved, or a part of it).  An operand reaching past D -- e.g. a
    16-byte MFMA operand fed by a 12-byte reload -- was assembled from a partial restore:
    SPLIT.  A register stops being followed once an instruction writes it; the scan runs
    to the end of the kernel and, when the reload sits inside a loop (a backward branch
    over it), around the back edge from the loop head to the reload, so a reload at the
    bottom of a loop feeding the loop head is seen (paths are over-approximated:
    conservative);
  * any 8- or 12-byte ``Folded Spill`` of registers S (a part of a 16-byte MFMA operand
    is the miscompile's shape) whose registers some instruction of the kernel reads
    through an operand wider than S that overlaps it: SPLIT (a backstop; it can fire on
    an unrelated later use of the same registers -- then review and WHITELIST);
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


_STORE = ("ds_write", "ds_store", "buffer_store", "global_store", "scratch_store", "flat_store")


def _parse(line):
    """(mnemonic, destination registers, source registers) of one instruction line."""
    c = line.split(";", 1)[0].strip()
    if not c or c.startswith(".") or c.endswith(":"):
        return None
    mnem, _, ops = c.partition(" ")
    regs = _regs(ops)
    if mnem.startswith(_STORE) or "store" in mnem:
        return mnem, [], regs
    return mnem, regs[:1], regs[1:]


def _loops(lines):
    """[(head, branch)] line ranges of backward branches (s_branch / s_cbranch_* to a
    label above them)."""
    labels, out = {}, []
    for i, ln in enumerate(lines):
        t = ln.split(";", 1)[0].strip()
        if t.endswith(":"):
            labels[t[:-1]] = i
        elif t.startswith(("s_branch", "s_cbranch")):
            tgt = t.split()[-1]
            if tgt in labels:
                out.append((labels[tgt], i))
    return out


def scan_kernel(body):
    """(status, detail) of one kernel body: status None (no spill), "spill" or "SPLIT"."""
    lines = body.split("\n")
    parsed = [_parse(ln) for ln in lines]
    sizes, splits = [], []
    if "Reload Reuse" in body:
        splits.append("Reload Reuse annotation")
    loops = _loops(lines)
    for i, ln in enumerate(lines):
        note = ln.split(";", 1)[1] if ";" in ln else ""
        if "Folded Spill" in note:
            nb = int(re.search(r"(\d+)-byte", note).group(1))
            sizes.append(str(nb))
            src = parsed[i][2] if parsed[i] else []
            if nb in (8, 12) and src:
                f, a, b = src[0]
                for j, pr in enumerate(parsed):
                    wide = [r for r in (pr[1] + pr[2] if pr else []) if r[0] == f and
                            not (r[2] < a or r[1] > b) and (r[1] < a or r[2] > b)]
                    if wide:
                        splits.append(f"{nb}-byte spill of {f}[{a}:{b}]; {f}[{wide[0][1]}:{wide[0][2]}] is read "
                                      f"whole in `{lines[j].strip()[:80]}`")
                        break
        if "Folded Reload" not in note or not parsed[i] or not parsed[i][1]:
            continue
        f, a, b = parsed[i][1][0]
        # successors: the rest of the kernel, then around each enclosing loop's back edge
        order = list(range(i + 1, len(lines)))
        for head, br in loops:
            if head <= i <= br:
                order += list(range(head, i))
        live = set(range(a, b + 1))
        for j in order:
            pr = parsed[j]
            if pr is None:
                continue
            mnem, dst, srcs = pr
            hit = [r for r in srcs if r[0] == f and any(r[1] <= k <= r[2] for k in live)]
            wide = [r for r in hit if r[1] < a or r[2] > b]
            if wide:
                splits.append(f"{b - a + 1}-dword reload {f}[{a}:{b}] feeds {f}[{wide[0][1]}:{wide[0][2]}] "
                              f"in `{lines[j].strip()[:80]}`")
                break
            for r in dst:
                if r[0] == f:
                    live -= set(range(r[1], r[2] + 1))
            if not live:
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
