"""Prints a rocprofv3 kernel_stats.csv compactly."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof2/run_kernel_stats.csv")):
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>4} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
          f"tot_ms={float(r['TotalDurationNs']) / 1e6:8.3f}")
