"""The BAI writer's host half (mh_bgzf.cpp bai_plan / bai_emit: per-record work on threads, then the virtual offsets)
against the oracle's BAI (oracle/god.py bai, a restatement of the SAM spec §5.2 index; it is a valid index of the
same file, not claimed byte-identical to what pysam.index (god_aligner.py:117-131) would write) on
synthetic sorted records: several references (one empty), runs of one bin cut across the thread pieces, records in
higher-level bins, windows without records, and record offsets on BGZF block boundaries.  The library's C++ is
compiled with a small driver (g++, zlib), no GPU."""
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import god

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, 'mitty_amd', 'csrc')

DRIVER = r'''
#include "mh_bgzf.h"
#include <cstdio>
#include <vector>
// stdin: n_refs n | n x (tid beg end bin) | n + 1 soff | nb coff   ->  argv[1] = the BAI
int main(int argc, char **argv) {
  int32_t n_refs; int64_t n, nb;
  if (fread(&n_refs, 4, 1, stdin) != 1 || fread(&n, 8, 1, stdin) != 1) return 2;
  std::vector<mh::BaiRec> recs(n + 1);
  std::vector<int64_t> soff(n + 1);
  if (fread(recs.data(), sizeof(mh::BaiRec), n, stdin) != (size_t)n) return 2;
  if (fread(soff.data(), 8, n + 1, stdin) != (size_t)(n + 1) || fread(&nb, 8, 1, stdin) != 1) return 2;
  std::vector<int64_t> coff(nb);
  if (fread(coff.data(), 8, nb, stdin) != (size_t)nb) return 2;
  std::string err;
  if (!mh::bai_write(argv[1], n_refs, n, recs.data(), soff.data(), coff, err)) {
    fprintf(stderr, "%s\n", err.c_str());
    return 1;
  }
  return 0;
}
'''


@pytest.fixture(scope='module')
def driver(tmp_path_factory):
  d = tmp_path_factory.mktemp('bai')
  src, exe = d / 'drv.cpp', d / 'drv'
  src.write_text(DRIVER)
  r = subprocess.run(['g++', '-O2', '-std=c++17', '-pthread', '-I', CSRC, str(src), os.path.join(CSRC, 'mh_bgzf.cpp'),
                      '-o', str(exe), '-lz'], capture_output=True, text=True)
  assert r.returncode == 0, r.stderr
  return str(exe), d


def _records(seed, n_refs, per_ref):
  rng = np.random.default_rng(seed)
  recs = []
  for tid in range(n_refs):
    n = per_ref[tid]
    if n == 0:
      continue
    beg = np.sort(rng.integers(0, 3_000_000, n))
    # mostly 150-250 bp; some long spans (higher-level bins); gaps leave windows without records
    ln = np.where(rng.random(n) < 0.02, rng.integers(20_000, 300_000, n), rng.integers(150, 251, n))
    for b, l in zip(beg.tolist(), ln.tolist()):
      recs.append((tid, b, b + l, god.reg2bin(b, b + l)))
  return recs


@pytest.mark.parametrize('seed,per_ref', [(1, [0]), (2, [5]), (3, [300_000, 0, 180_000]), (4, [0, 70_000, 1])])
def test_bai_matches_oracle(driver, seed, per_ref):
  exe, d = driver
  recs = _records(seed, len(per_ref), per_ref)
  n = len(recs)
  rng = np.random.default_rng(seed + 100)
  sizes = rng.integers(36, 400, n)
  if n > 10:   # a record ending exactly on a block boundary
    sizes[5] = 0xff00 - int(sizes[:5].sum())
  soff = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
  nb = int(soff[-1]) // 0xff00 + 2
  coff = np.concatenate([[1234], 1234 + np.cumsum(rng.integers(9000, 30000, nb - 1))]).astype(np.int64)
  blob = struct.pack('<iq', len(per_ref), n)
  blob += np.array(recs, dtype=np.int64).astype(np.int32).tobytes() if n else b''
  blob += soff.tobytes() + struct.pack('<q', nb) + coff.tobytes()
  out = d / 'x{}.bai'.format(seed)
  r = subprocess.run([exe, str(out)], input=blob, capture_output=True)
  assert r.returncode == 0, r.stderr

  def vo(u):
    b = u // 0xff00
    return (int(coff[b]) << 16) | (u - b * 0xff00)

  dec = [{'reference_id': t, 'pos': b, 'bin': bn, 'cigarstring': '{}M'.format(e - b)} for t, b, e, bn in recs]
  vos = [vo(int(u)) for u in soff[:-1]]
  assert out.read_bytes() == god.bai(len(per_ref), dec, vos, vo(int(soff[-1])))
