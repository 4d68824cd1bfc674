"""Summarise rocprofv3 kernel-trace stats + FETCH_SIZE/WRITE_SIZE passes into profiles/.

usage: python tools/pmc_summary.py gpurun_out/prof <tag> [clips_per_launch] [model] [steps]
Writes profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_pmc_summary.json and one
profiles/pmc_<family>_<model>.json per kernel family the trace holds (bench.py reads
them for roofline.traffic; res15's also under the legacy name pmc_<family>.json).
`clips_per_launch` is the batch key bench.py matches (for the cnn configs the clips of
the whole step, for the block kernels the 4096-clip chunk).  With `steps` (the number
of training steps the profiled command ran, warmup included) it also writes
profiles/pmc_train_step_<model>.json: the HBM bytes of every kernel of the run / steps.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide (16 B/lane)
coalesced streaming read -> doubled here.  The kernels summarised here stage with
16 B/lane buffer_load...lds or float4 loads, so the correction applies; stores are
reported raw.
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
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


# kernel families: a family pools every template instance of the named kernels
# (weighted by launches); the bf16-pipe res kernels are split by format (sp1 = bf16,
# sp2 = bf16x3, f16 = f16x2)
SP_ARG = {"block16r_kernel": 2, "block16w_kernel": 1, "block16p_kernel": 1, "block16l_kernel": 1}
# the operand-format template argument (2 = f16x2 -> family suffix "f16")
FM_ARG = {"block16w_kernel": 4, "block16p_kernel": 5, "block16l_kernel": 5}
POOLS = {"block_kernel": ("block_kernel",), "conv_gemm_kernel": ("conv_gemm_kernel",),
         "c2_f32_convs": ("conv1f_kernel", "conv2f_kernel"),
         "c2_bf16x3_convs": ("conv1x3_kernel", "conv2x3_kernel"),
         "conv3x3d_kernel": ("conv3x3d_kernel", "conv3x3s_kernel"),
         "wgrad3x3d_kernel": ("wgrad3x3d_kernel",)}


def families(k):
    out = []
    for fam, arg in SP_ARG.items():
        if f"::{fam}<" in k:
            args = [a.strip() for a in k.split("<")[1].split(">")[0].split(",")]
            fm = FM_ARG.get(fam)
            if fm is not None and len(args) > fm and args[fm] == "2":
                out.append(f"{fam}_f16")
            else:
                out.append(f"{fam}_sp" + args[arg])
    for fam, names in POOLS.items():
        if any(f"::{n}<" in k or f"::{n}(" in k for n in names):
            out.append(fam)
    return out


def main():
    d, tag = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    model = sys.argv[4] if len(sys.argv) > 4 else "res15"
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    os.makedirs("profiles", exist_ok=True)
    shutil.copy(os.path.join(d, f"{tag}_trace_kernel_stats.csv"), f"profiles/{tag}_kernel_stats.csv")
    fetch = per_kernel(os.path.join(d, f"{tag}_fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, f"{tag}_write_counter_collection.csv"), "WRITE_SIZE")
    stats = {}
    with open(os.path.join(d, f"{tag}_trace_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = dict(calls=int(row["Calls"]), avg_ns=float(row["AverageNs"]),
                                      pct=float(row["Percentage"]))
    out = {"batch_clips_per_launch": batch, "model": model, "kernels": {}}
    for name, s in stats.items():
        e = dict(s)
        if name in fetch:
            e["FETCH_SIZE_KiB_raw"] = fetch[name][0]
            e["hbm_read_bytes_corrected"] = fetch[name][0] * 1024 * 2
            e["pmc_launches"] = fetch[name][1]
        if name in write:
            e["WRITE_SIZE_KiB_raw"] = write[name][0]
            e["hbm_write_bytes"] = write[name][0] * 1024
        out["kernels"][name] = e
    with open(f"profiles/{tag}_pmc_summary.json", "w") as f:
        json.dump(out, f, indent=1)

    fams = sorted({f for k in out["kernels"] for f in families(k)})
    for fam in fams:
        ks = [k for k in out["kernels"] if fam in families(k) and "hbm_read_bytes_corrected" in out["kernels"][k]]
        if not ks:
            continue
        calls = sum(out["kernels"][k]["pmc_launches"] for k in ks)
        rd = sum(out["kernels"][k]["hbm_read_bytes_corrected"] * out["kernels"][k]["pmc_launches"] for k in ks) / calls
        wr = sum(out["kernels"][k].get("hbm_write_bytes", 0.0) * out["kernels"][k]["pmc_launches"] for k in ks) / calls
        res = {"kernel": fam, "model": model, "instances": ks, "source": f"profiles/{tag}_pmc_summary.json",
               "batch_clips_per_launch": batch, "launches": calls,
               "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr}
        names = [f"profiles/pmc_{fam}_{model}.json"] + ([f"profiles/pmc_{fam}.json"] if model == "res15" else [])
        for n in names:
            with open(n, "w") as f:
                json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))
    if steps:
        rd = sum(e.get("hbm_read_bytes_corrected", 0.0) * e.get("pmc_launches", 0) for e in out["kernels"].values())
        wr = sum(e.get("hbm_write_bytes", 0.0) * e.get("pmc_launches", 0) for e in out["kernels"].values())
        res = {"kernel": "train_step", "model": model, "source": f"profiles/{tag}_pmc_summary.json",
               "batch_clips_per_launch": batch, "steps": steps,
               "hbm_read_bytes_per_step": rd / steps, "hbm_write_bytes_per_step": wr / steps,
               "hbm_bytes_per_step": (rd + wr) / steps}
        with open(f"profiles/pmc_train_step_{model}.json", "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
