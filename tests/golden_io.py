"""Helpers to read the committed golden vectors (tests/golden, captured by make_golden.py)."""
import gzip
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
MODELS = ['hiseq-X-v2.5-Garvan', '1kg-pcr-free']


def path(*p):
  return os.path.join(GOLDEN, *p)


def load_json(name):
  if name.endswith('.gz'):
    with gzip.open(path(name), 'rt') as fp:
      return json.load(fp)
  with open(path(name)) as fp:
    return json.load(fp)


def fastq_bytes(name):
  with gzip.open(path(name), 'rb') as fp:
    return fp.read()


def templates():
  return np.load(path('templates.npz'), allow_pickle=False)


def model(name):
  from mitty_amd.readmodel import load_model_file
  return load_model_file(os.path.join(os.path.dirname(GOLDEN), '..', 'mitty_amd', 'data', 'readmodels', name + '.npz'))


def parse_fastq(b):
  lines = b.split(b'\n')
  recs = []
  for i in range(0, len(lines) - 3, 4):
    recs.append((lines[i][1:].decode(), lines[i + 1].decode(), lines[i + 3].decode()))
  return recs


def check_same(got, want, what='output'):
  """Byte-exact comparison that reports the first differing line (pytest's own diff of multi-MB bytes takes
  minutes)."""
  if got == want:
    return
  lg, lw = got.split(b'\n'), want.split(b'\n')
  for i, (x, y) in enumerate(zip(lg, lw)):
    if x != y:
      raise AssertionError('{} differs at line {}: got {!r} want {!r}'.format(what, i, x[:300], y[:300]))
  raise AssertionError('{} differs in length: {} vs {} lines ({} vs {} bytes)'.format(what, len(lg), len(lw),
                                                                                       len(got), len(want)))
