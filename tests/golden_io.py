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
