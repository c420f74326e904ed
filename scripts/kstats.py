"""Per-step kernel time table from a rocprofv3 kernel_stats.csv: python scripts/kstats.py CSV STEPS [N]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows.sort(key=lambda x: -float(x['TotalDurationNs']))
for x in rows[:top]:
    n = x['Name'].replace('mh::(anonymous namespace)::', '').replace('void ', '')
    n = re.sub(r'rocprim::ROCPRIM_\w+::', 'rp::', n)
    n = re.sub(r'rp::detail::trampoline_kernel<.*?(onesweep_\w+|transform|histogram)\w*.*', r'rocprim \1', n)
    print(f"{float(x['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step  calls {int(x['Calls']) / steps:5.1f}  "
          f"avg {float(x['AverageNs']) / 1e3:8.1f} us  min {float(x['MinNs']) / 1e3:8.1f} us  {n[:70]}")
