"""Print the top kernels of the newest rocprofv3 kernel_stats.csv under a directory."""
import csv, glob, os, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
f = max(glob.glob(os.path.join(d, "**/*kernel_stats.csv"), recursive=True), key=os.path.getmtime)
for x in list(csv.DictReader(open(f)))[:n]:
    print(f"{float(x['TotalDurationNs'])/1e6:9.3f} ms {int(x['Calls']):6d} {float(x['AverageNs'])/1e3:9.2f}us {x['Name'][:90]}")
