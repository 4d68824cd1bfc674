"""Condensed instruction flow of a kernel's biggest block: runs of VALU/SALU collapsed, waits and LDS ops shown."""
import re, subprocess, sys
text = open(sys.argv[1]).read()
for m in re.finditer(r"\n(_Z\w+):", text):
    name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
    if sys.argv[2] not in name:
        continue
    body = text[m.end():text.find(".Lfunc_end", m.end())]
    blocks = re.split(r"\n\.LBB\w+:", body)
    big = max(blocks, key=lambda b: b.count("v_mfma"))
    out, run = [], {}
    def flush():
        if run:
            out.append("   " + " ".join(f"{k}{v}" for k, v in run.items()))
            run.clear()
    nm = 0
    for ln in big.split("\n"):
        t = ln.strip().split(";")[0].strip()
        if not t or t.startswith("."):
            continue
        op = t.split()[0]
        if "mfma" in op:
            nm += 1
            run["M"] = run.get("M", 0) + 1
        elif op.startswith("v_"):
            run["v"] = run.get("v", 0) + 1
        elif op.startswith("s_") and "waitcnt" not in op and "barrier" not in op:
            run["s"] = run.get("s", 0) + 1
        else:
            flush()
            out.append(f"[{nm:3d}] {t[:70]}")
    flush()
    print("\n".join(out))
    break
