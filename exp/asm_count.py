"""Instruction mix of a kernel's MFMA blocks (each step body): python exp/asm_count.py FILE.s KERNEL_SUBSTR"""
import re, subprocess, sys
from collections import Counter
text = open(sys.argv[1]).read()
for m in re.finditer(r"\n(_Z\w+):", text):
    name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
    if sys.argv[2] not in name:
        continue
    body = text[m.end():text.find(".Lfunc_end", m.end())]
    blocks = re.split(r"\n\.LBB\w+:", body)
    print(name[:100])
    for big in sorted(blocks, key=lambda b: -b.count("v_mfma"))[:2]:
        c = Counter()
        vops = Counter()
        for ln in big.split("\n"):
            t = ln.strip().split(";")[0].split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            op = t[0]
            k = ("mfma" if "mfma" in op else "valu" if op.startswith("v_") else
                 "wait" if "waitcnt" in op else "bar" if "barrier" in op else
                 "salu" if op.startswith("s_") else "ds_r" if op.startswith("ds_read") else "ds_w" if op.startswith("ds_") else
                 "dma" if "lds" in ln and op.startswith("buffer") else "vmem" if op.startswith(("buffer", "global")) else op)
            c[k] += 1
            if k == "valu":
                vops[op] += 1
        print("  ", dict(c))
        print("     top VALU:", vops.most_common(14))
