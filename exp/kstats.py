"""Print the res/cnn block kernels of rocprofv3 kernel_stats CSVs: name args, calls, average ms."""
import csv, sys
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if any(k in n for k in ("block16", "conv0", "block_kernel", "conv2x3", "conv1x3", "conv3x3", "wgrad")):
            short = n.split("(")[0].replace("void ", "").replace("honk::", "")
            print(f"  {short:60s} calls {r['Calls']:>5} avg {float(r['AverageNs']) / 1e6:.4f} ms")
