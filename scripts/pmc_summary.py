#!/usr/bin/env python3
"""Summarise a gpu_pmc.sh run into profiles/pmc_<kernel>_<round>.json (read by bench.py for roofline.traffic).

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md § HBM: FETCH_SIZE and WRITE_SIZE are in KiB, from
separate passes; on gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane) streaming reads, so it is doubled.
The doubling is calibrated for the writer's own pattern too — 16-byte gathers of 150-byte windows at random
offsets read 1.97 x FETCH_SIZE bytes of distinct 128-byte lines (profiles/calib_fetch_size_r03.json,
scripts/calib_fetch.hip).  WRITE_SIZE is exact for 16-byte stores.
usage: pmc_summary.py <pmc dir> <tag> <kernel> <round> <rlen> <length> [algorithmic bytes per launch] [workload]
(workload: the bench workload the passes ran, 'chr1' or 'wgs'; bench.py takes traffic only from a matching file)
"""
import csv
import json
import os
import sys


def per_dispatch(path, name):
  vals = {}
  for r in csv.DictReader(open(path)):
    if r['Counter_Name'] == name:
      vals[r['Dispatch_Id']] = vals.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
  return list(vals.values())


def main():
  d, tag, kernel, rnd, rlen, length = sys.argv[1:7]
  alg = float(sys.argv[7]) if len(sys.argv) > 7 and sys.argv[7] != '-' else None
  out = {'kernel': kernel, 'rlen': int(rlen), 'length': int(length)}
  if len(sys.argv) > 8:
    out['workload'] = sys.argv[8]
  counters = {}
  for i in range(1, 6):
    p = os.path.join(d, '{}_{}'.format(tag, i), 'run_counter_collection.csv')
    if not os.path.exists(p):
      continue
    names = {r['Counter_Name'] for r in csv.DictReader(open(p))}
    for n in names:
      v = per_dispatch(p, n)
      counters[n] = sum(v) / len(v)
  out['counters_per_launch'] = counters
  if 'FETCH_SIZE' in counters and 'WRITE_SIZE' in counters:
    fetch = 2 * counters['FETCH_SIZE'] * 1024
    write = counters['WRITE_SIZE'] * 1024
    out['hbm_read_bytes_per_launch'] = fetch
    out['hbm_write_bytes_per_launch'] = write
    out['hbm_bytes_per_launch'] = fetch + write
    if alg:
      out['algorithmic_bytes_per_launch'] = alg
      out['traffic_over_algorithmic'] = (fetch + write) / alg
  if 'TCC_HIT_sum' in counters and 'TCC_MISS_sum' in counters:
    out['l2_hit_rate'] = counters['TCC_HIT_sum'] / max(counters['TCC_HIT_sum'] + counters['TCC_MISS_sum'], 1)
  dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'profiles',
                     'pmc_{}_{}.json'.format(kernel, rnd))
  with open(dst, 'w') as fp:
    json.dump(out, fp, indent=1)
  print(json.dumps(out, indent=1))


if __name__ == '__main__':
  main()
