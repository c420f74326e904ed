#!/usr/bin/env python3
"""Print per-launch averages of every counter found under gpurun_out/pmc/<tag>_*/run_counter_collection.csv."""
import csv
import glob
import sys

tag = sys.argv[1]
out = {}
for p in sorted(glob.glob('gpurun_out/pmc/{}_*/run_counter_collection.csv'.format(tag))):
  per = {}
  for r in csv.DictReader(open(p)):
    per.setdefault(r['Counter_Name'], {}).setdefault(r['Dispatch_Id'], 0.0)
    per[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
  for n, d in per.items():
    out[n] = sum(d.values()) / len(d)
for n in sorted(out):
  print('{:32s} {:16.1f}'.format(n, out[n]))
