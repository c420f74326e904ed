"""The metric's full-size step byte-checked (BASELINE configs[3]'s genome at scale 1: the whole synthetic GRCh37,
30x, 2x150, 100 work units, 293 M templates, 216 GB of FASTQ): `bench.py --verify` runs one step of the bench's own
plan unit by unit and compares every unit's sha256 of both FASTQ ranges with the CPU oracle's digests of the same
unit (readgenerate.py:129-159 unit list, seeds and order).  Run as a child process (one GPU process, its own HIP
runtime); the oracle digests run in 16 worker processes beside the GPU work."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_wgs_full_step_every_unit_equals_oracle():
  from mitty_amd import _native
  if _native.device_count() == 0:
    pytest.fail('no HIP device: GPU tests must run on an MI355X')
  r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--steps', '1', '--warmup', '0',
                      '--no-cpu-baseline', '--no-e2e', '--verify'], cwd=REPO, capture_output=True, text=True,
                     timeout=850)
  assert r.returncode == 0, r.stderr[-3000:]
  line = [x for x in r.stdout.splitlines() if x.startswith('{')][-1]
  v = json.loads(line)['verify']
  assert v['units'] == 100 and v['units_equal'] == 100, v
  assert v['templates_kept'] > 280_000_000 and v['fastq_bytes'] > 200e9, v
