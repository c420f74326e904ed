"""Device BGZF rate: a FASTQ-like buffer (the golden FASTQ repeated to --mb MB) deflated on the GPU through
mh_bgzf_compress_gpu (H2D, deflate, D2H), timed per call; run under rocprofv3 --kernel-trace --stats for the kernels'
own time.  python scripts/bgzf_rate.py [--mb 1024] [--reps 3]"""
import argparse
import gzip
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--mb', type=int, default=1024)
  ap.add_argument('--reps', type=int, default=3)
  a = ap.parse_args()
  from mitty_amd import _native
  fq = gzip.open(os.path.join(REPO, 'tests', 'golden', 'e2e_hiseq-X-v2.5-Garvan.r1.fq.gz')).read()
  n = a.mb << 20
  data = (fq * (n // len(fq) + 1))[:n]
  ctx = _native.Context(0)
  ts, z = [], b''
  for _ in range(a.reps):
    t0 = time.perf_counter()
    z = ctx.bgzf_compress(data)
    ts.append(time.perf_counter() - t0)
  print(json.dumps({'input_bytes': n, 'output_bytes': len(z), 'ratio': n / len(z), 'seconds': ts,
                    'GBps_incl_transfers': n / min(ts) / 1e9}))


if __name__ == '__main__':
  main()
