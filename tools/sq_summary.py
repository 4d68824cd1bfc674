"""Summarise one `rocprofv3 --pmc <SQ counters> GRBM_GUI_ACTIVE` pass (tools/profile_sq_pair.sh)
into profiles/pmc_<tag>_pair_sq.json: per-launch means of every counter for the headline
kernels (res15 f16x2: the pair instances, the last layer, conv0m, tail_sum) and the derived
fractions, plus one entry that pools every `block16p_kernel` instance (the six tap-step
instances of a res15 chunk).

    python tools/sq_summary.py gpurun_out/prof/r5b_pairsq_counter_collection.csv r5b

Normalisation (MI355X_MICROARCH.md, SQ counters): MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); SQ_WAIT_ANY, SQ_WAIT_INST_ANY and SQ_ACTIVE_INST_ANY
over SQ_WAVE_CYCLES.
"""
import csv
import json
import os
import sys
from collections import defaultdict

TAGS = ("block16p_kernel", "block16k_kernel", "block16l_kernel", "conv0m_kernel", "tail_sum_kernel")


def derive(m):
    out = dict(m)
    g = m.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        out["_mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024)
    w = m.get("SQ_WAVE_CYCLES")
    for k, n in (("SQ_WAIT_ANY", "_wait_any_frac"), ("SQ_WAIT_INST_ANY", "_wait_inst_any_frac"),
                 ("SQ_ACTIVE_INST_ANY", "_active_inst_frac")):
        if w and k in m:
            out[n] = m[k] / w
    return out


def main(path, tag):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    with open(path) as fh:
        for rec in csv.DictReader(fh):
            name = rec["Kernel_Name"]
            if not any(t in name for t in TAGS):
                continue
            d = per[name][rec["Dispatch_Id"]]
            d[rec["Counter_Name"]] = d.get(rec["Counter_Name"], 0.0) + float(rec["Counter_Value"])
    kernels = {}
    pooled = defaultdict(list)
    for name, ds in sorted(per.items()):
        cs = defaultdict(list)
        for d in ds.values():
            for k, v in d.items():
                cs[k].append(v)
                if "block16p_kernel" in name:
                    pooled[k].append(v)
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        m["_launches"] = len(ds)
        kernels[name] = derive(m)
    if pooled:
        m = {k: sum(v) / len(v) for k, v in pooled.items()}
        m["_launches"] = sum(len(ds) for n, ds in per.items() if "block16p_kernel" in n)
        kernels["block16p_kernel (all instances)"] = derive(m)
    cmd = ("tools/profile_sq_pair.sh %s: rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
           "SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE "
           "--kernel-trace -- python3 bench.py --batch 16384 --steps 1 --warmup 1 --no-cpu-baseline --no-alt" % tag)
    out = {"command": cmd,
           "normalisation": "per-launch means; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 XCDs x 1024 "
                            "SIMDs); SQ_WAIT_*/SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint)",
           "kernels": kernels}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", f"pmc_{tag}_pair_sq.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    for n, m in kernels.items():
        print(f"{n[:80]:80s} launches {m['_launches']:4d}  MFMA busy {m.get('_mfma_busy_frac', 0):.3f}  "
              f"wait-inst {m.get('_wait_inst_any_frac', 0):.3f}")
    return dst


if __name__ == "__main__":
    print(main(sys.argv[1], sys.argv[2]))
