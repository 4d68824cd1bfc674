"""Summarise rocprofv3 kernel-trace stats + FETCH_SIZE/WRITE_SIZE passes into profiles/.

usage: python tools/pmc_summary.py gpurun_out/prof r1 [clips_per_launch] [model]
Writes profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_pmc_summary.json and
profiles/pmc_block_kernel.json (read by bench.py for roofline.traffic).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane)
coalesced streaming read -> doubled here.  Our block kernel reads with 16 B/lane
buffer_load...lds, so the correction applies; its stores are 4 B/lane
(uncalibrated width), reported raw.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d, tag = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    model = sys.argv[4] if len(sys.argv) > 4 else "res15"
    os.makedirs("profiles", exist_ok=True)
    shutil.copy(os.path.join(d, f"{tag}_trace_kernel_stats.csv"), f"profiles/{tag}_kernel_stats.csv")
    fetch = per_kernel(os.path.join(d, f"{tag}_fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, f"{tag}_write_counter_collection.csv"), "WRITE_SIZE")
    stats = {}
    with open(os.path.join(d, f"{tag}_trace_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = dict(calls=int(row["Calls"]), avg_ns=float(row["AverageNs"]),
                                      pct=float(row["Percentage"]))
    out = {"batch_clips_per_launch": batch, "kernels": {}}
    for name, s in stats.items():
        e = dict(s)
        if name in fetch:
            e["FETCH_SIZE_KiB_raw"] = fetch[name]
            e["hbm_read_bytes_corrected"] = fetch[name] * 1024 * 2
        if name in write:
            e["WRITE_SIZE_KiB_raw"] = write[name]
            e["hbm_write_bytes"] = write[name] * 1024
        out["kernels"][name] = e
    with open(f"profiles/{tag}_pmc_summary.json", "w") as f:
        json.dump(out, f, indent=1)
    # per kernel family (all template instances, weighted by launches) -> the
    # profiles/pmc_<family>.json that bench.py reads for roofline.traffic
    def family(k):
        for fam in ("block16r_kernel",):  # split by SP (3rd template argument): sp1 = bf16, sp2 = bf16x3
            if f"::{fam}<" in k:
                return f"{fam}_sp" + k.split("<")[1].split(",")[2].strip()
        for fam in ("block16w_kernel", "block16p_kernel"):  # SP is the 2nd template argument
            if f"::{fam}<" in k:
                return f"{fam}_sp" + k.split("<")[1].split(",")[1].strip()
        for fam in ("block_kernel", "conv_gemm_kernel"):
            if f"::{fam}<" in k:
                return fam
        return None

    fams = sorted({family(k) for k in out["kernels"]} - {None})
    for fam in fams:
        ks = [k for k in out["kernels"] if family(k) == fam and "hbm_read_bytes_corrected" in out["kernels"][k]]
        if not ks:
            continue
        calls = sum(out["kernels"][k]["calls"] for k in ks)
        rd = sum(out["kernels"][k]["hbm_read_bytes_corrected"] * out["kernels"][k]["calls"] for k in ks) / calls
        wr = sum(out["kernels"][k].get("hbm_write_bytes", 0.0) * out["kernels"][k]["calls"] for k in ks) / calls
        res = {"kernel": fam, "model": model, "instances": ks, "source": f"profiles/{tag}_pmc_summary.json",
               "batch_clips_per_launch": batch, "launches": calls,
               "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr}
        with open(f"profiles/pmc_{fam}.json", "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
