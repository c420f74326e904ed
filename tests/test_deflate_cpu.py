"""The single-thread parts of the device BGZF compressor (mitty_amd/csrc/mh_deflate.h) on the CPU: a sequential
restatement of its parse (tests/deflate_host.cpp) builds BGZF with the shared Huffman / header / CRC code, and zlib
inflates it back.  The device kernel itself is checked in tests/test_gpu_parity.py::test_device_bgzf_*."""
import gzip
import os
import subprocess

import pytest

from tests import golden_io as G

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope='module')
def tool(tmp_path_factory):
  out = str(tmp_path_factory.mktemp('df') / 'deflate_host')
  subprocess.check_call(['/opt/rocm/bin/hipcc', '-O2', '-std=c++17', '-x', 'hip', '--offload-arch=gfx950',
                         '-include', 'algorithm', '-o', out, os.path.join(HERE, 'deflate_host.cpp')])
  return out


@pytest.mark.parametrize('name', ['fastq', 'zeros', 'tiny', 'abc', 'text', 'multi'])
def test_bgzf_shared_code_round_trip(tool, tmp_path, name):
  data = {'fastq': lambda: G.fastq_bytes('e2e_hiseq-X-v2.5-Garvan.r1.fq.gz'),
          'zeros': lambda: b'\0' * 200000,
          'tiny': lambda: b'A',
          'abc': lambda: b'abcabcabcabc' * 7,
          'text': lambda: open(os.path.join(HERE, '..', 'DESIGN.md'), 'rb').read(),
          'multi': lambda: (G.fastq_bytes('e2e_1kg-pcr-free.r2.fq.gz') * 3)[:400_001]}[name]()
  src, dst = tmp_path / 'in', tmp_path / 'out'
  src.write_bytes(data)
  subprocess.check_call([tool, str(src), str(dst)])
  z = dst.read_bytes()
  assert gzip.decompress(z) == data
  if name in ('fastq', 'multi'):   # FASTQ compresses about as well as gzip -1 (~4x)
    assert len(z) < len(data) / 3.5


def test_bgzf_shared_code_incompressible_block_is_flagged(tool, tmp_path):
  src, dst = tmp_path / 'in', tmp_path / 'out'
  src.write_bytes(os.urandom(100000))
  assert subprocess.run([tool, str(src), str(dst)]).returncode == 3   # the device stores such a block
