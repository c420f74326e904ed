"""Inputs and outputs on FIFOs and process substitution, as the reference's pipeline runs them
(examples/reads/run.sh:13-16: generate-reads writes `>(tee > tf1 ...)`, corrupt-reads reads `<(cat < tf1)` and
`--fastq2-in <(cat < tf2)`).

* Every reader opens its file once and sniffs the gzip magic on the open stream (a second open of a FIFO with a
  single-open producer loses the records the first open swallowed; a reopened `/dev/fd` pipe loses the two sniffed
  bytes).
* The two files of a pair are read on a thread each and written on a thread each, so a producer that writes record
  by record (the reference's writer, readgenerate.py:233-253) or file by file, and a consumer that reads in lockstep
  (pysam.FastxFile pairs, readcorrupt.py:49-53), never wait on each other's other pipe.
"""
import gzip
import os
import threading

import pytest

from mitty_amd.lib import fastq_stream as FS
from mitty_amd.lib.openfile import open_input
from tests import golden_io as G

pytestmark = pytest.mark.timeout(120)


def _records(n, tag=b''):
  return [b'@t%d%s|1|0\n%s\n+\n%s\n' % (i, tag, b'ACGT' * (i % 7 + 1), b'~' * (4 * (i % 7 + 1))) for i in range(n)]


def _producer(path, chunks, started=None):
  """Open once, write the chunks, close (the shape of `tee > tf1`)."""
  def run():
    with open(path, 'wb') as fp:
      for c in chunks:
        fp.write(c)
        fp.flush()
  t = threading.Thread(target=run, daemon=True)
  t.start()
  return t


@pytest.mark.parametrize('gz', [False, True])
def test_open_input_fifo_single_open_producer(tmp_path, gz):
  data = b''.join(_records(3))
  payload = gzip.compress(data) if gz else data
  fifo = str(tmp_path / 'f')
  os.mkfifo(fifo)
  t = _producer(fifo, [payload[:1], payload[1:5], payload[5:]])   # the magic split across writes
  with open_input(fifo) as fp:
    got = fp.read()
  t.join()
  assert got == data


@pytest.mark.parametrize('gz', [False, True])
def test_open_input_dev_fd_pipe(gz):
  """`<(...)`: the path is /dev/fd/N of a pipe; opening it twice would continue the same pipe after the sniff."""
  data = b''.join(_records(50))
  payload = gzip.compress(data) if gz else data
  r, w = os.pipe()
  t = threading.Thread(target=lambda: (os.write(w, payload), os.close(w)), daemon=True)
  t.start()
  try:
    with open_input('/dev/fd/{}'.format(r)) as fp:
      got = fp.read()
  finally:
    os.close(r)
  t.join()
  assert got == data


def test_vcf_and_fasta_readers_over_fifos(tmp_path):
  from mitty_amd.lib import fasta as mfasta
  from mitty_amd.lib import vcfio
  c = G.load_json('e2e_config.json')['hiseq-X-v2.5-Garvan']
  vcf, fa, bed = G.path(c['vcf']), G.path(c['fasta']), G.path(c['bed'])
  want_py = vcfio.load_variant_file(vcf, c['sample'], bed)
  want_soa = vcfio.load_variants_soa(vcf, c['sample'], bed)
  want_fa = mfasta.read_fasta(fa)
  for k, (src, fn) in enumerate([(vcf, lambda p: vcfio.load_variant_file(p, c['sample'], bed)),
                                 (vcf, lambda p: vcfio.load_variants_soa(p, c['sample'], bed)),
                                 (fa, mfasta.read_fasta), (fa, mfasta.read_fasta_py)]):
    fifo = str(tmp_path / 'in{}'.format(k))
    os.mkfifo(fifo)
    raw = open(src, 'rb').read()
    t = _producer(fifo, [raw[:1], raw[1:]])
    got = fn(fifo)
    t.join()
    if k == 0:
      assert [[[v.tuple() for v in cp] for cp in r['v']] for r in got] == \
             [[[v.tuple() for v in cp] for cp in r['v']] for r in want_py]
    elif k == 1:
      assert len(got) == len(want_soa)
      for a, b in zip(got, want_soa):
        assert a['region'] == b['region'] and a['ploidy'] == b['ploidy']
        for ca, cb in zip(a['copies'], b['copies']):
          assert all(bytes(memoryview(ca[f])) == bytes(memoryview(cb[f])) for f in ca), a['region']
    else:
      assert got == want_fa


def _consume_into(out):
  """A host stand-in for the device parser: takes the complete templates present in both buffers."""
  def consume(b1, b2, want, done):
    def ends(b):
      e, k = [], 0
      lines = 0
      for i, ch in enumerate(b):
        if ch == 10:
          lines += 1
          if lines % 4 == 0:
            e.append(i + 1)
      return e
    e1 = ends(b1)
    e2 = ends(b2) if b2 is not None else e1
    t = min(len(e1), len(e2))
    if want >= 0:
      t = min(t, want)
    if t == 0:
      return 0, 0, 0
    out[0].append(b1[:e1[t - 1]])
    if b2 is not None:
      out[1].append(b2[:e2[t - 1]])
    return e1[t - 1], (e2[t - 1] if b2 is not None else 0), t
  return consume


@pytest.mark.parametrize('style', ['record_by_record', 'file_pieces'])
def test_stream_templates_fifo_pair(tmp_path, style):
  """A producer writing the pair record by record (the reference's writer) or in alternating 3 MB pieces per file
  (ours before threads): the lockstep consumer gets every template, in order, without a deadlock."""
  r1, r2 = _records(40000, b'/1'), _records(40000, b'/2')
  f1, f2 = str(tmp_path / 'tf1'), str(tmp_path / 'tf2')
  os.mkfifo(f1)
  os.mkfifo(f2)

  def produce():
    with open(f1, 'wb') as a, open(f2, 'wb') as b:
      if style == 'record_by_record':
        for x, y in zip(r1, r2):
          a.write(x)
          b.write(y)
      else:
        d1, d2 = b''.join(r1), b''.join(r2)
        for off in range(0, len(d1), 3 << 20):
          a.write(d1[off:off + (3 << 20)])
          a.flush()
          b.write(d2[off:off + (3 << 20)])
          b.flush()
  t = threading.Thread(target=produce, daemon=True)
  t.start()
  out = ([], [])
  n = FS.stream_templates(f1, f2, _consume_into(out), chunk=1 << 20, max_ahead=8 << 20)
  t.join()
  assert n == 40000
  assert b''.join(out[0]) == b''.join(r1) and b''.join(out[1]) == b''.join(r2)


def test_stream_templates_limit_releases_fifo_producer(tmp_path):
  """stream_templates returning early (limit, as god-aligner --max-templates): both readers stop and close their
  FIFOs, so a producer still writing gets EPIPE instead of blocking forever."""
  r1, r2 = _records(200000, b'/1'), _records(200000, b'/2')
  f1, f2 = str(tmp_path / 'lf1'), str(tmp_path / 'lf2')
  os.mkfifo(f1)
  os.mkfifo(f2)
  res = {}

  def produce():
    try:
      with open(f1, 'wb') as a, open(f2, 'wb') as b:
        for x, y in zip(r1, r2):
          a.write(x)
          b.write(y)
      res['end'] = 'finished'
    except BrokenPipeError:
      res['end'] = 'epipe'
  t = threading.Thread(target=produce, daemon=True)
  t.start()
  out = ([], [])
  n = FS.stream_templates(f1, f2, _consume_into(out), chunk=1 << 20, limit=1000, max_ahead=4 << 20)
  assert n == 1000
  t.join(30)
  assert not t.is_alive(), 'the FIFO producer is still blocked after the consumer stopped'
  assert res['end'] == 'epipe'


def test_write_pair_to_lockstep_fifo_reader(tmp_path):
  """Our producer side: 20 MB per file handed to write_pair, read by a consumer that alternates record by record
  between the two FIFOs (pysam.FastxFile zip, readcorrupt.py:49-53)."""
  r1, r2 = _records(150000, b'/1'), _records(150000, b'/2')
  d1, d2 = b''.join(r1), b''.join(r2)
  f1, f2 = str(tmp_path / 'o1'), str(tmp_path / 'o2')
  os.mkfifo(f1)
  os.mkfifo(f2)
  got = ([], [])

  def lockstep():
    with open(f1, 'rb') as a, open(f2, 'rb') as b:
      while True:
        x = b''.join(a.readline() for _ in range(4))
        y = b''.join(b.readline() for _ in range(4))
        if not x and not y:
          return
        got[0].append(x)
        got[1].append(y)
  t = threading.Thread(target=lockstep, daemon=True)
  t.start()
  s1, s2 = FS.FastqSink(f1), FS.FastqSink(f2)
  FS.write_pair([s1, s2], [d1, d2])
  s1.close()
  s2.close()
  t.join()
  assert b''.join(got[0]) == d1 and b''.join(got[1]) == d2


def test_pair_writer_chunks_in_order_to_lockstep_fifo_reader(tmp_path):
  """generate-reads' output side: chunks of both files handed to a PairWriter through two alternating staging slots
  (the slot is waited on before it is refilled, as readgenerate.process_multi_threaded does around its D2H copies),
  each FIFO drained by its own reader; file 2 shorter (fewer chunks)."""
  r1, r2 = _records(120000, b'/1'), _records(90000, b'/2')
  d1, d2 = b''.join(r1), b''.join(r2)
  f1, f2 = str(tmp_path / 'o1'), str(tmp_path / 'o2')
  os.mkfifo(f1)
  os.mkfifo(f2)
  got = ([], [])

  def reader(path, out):
    with open(path, 'rb') as a:
      out.append(a.read())
  ts = [threading.Thread(target=reader, args=(f, g), daemon=True) for f, g in zip((f1, f2), got)]
  for t in ts:
    t.start()
  s1, s2 = FS.FastqSink(f1), FS.FastqSink(f2)
  pw = FS.PairWriter([s1, s2])
  bufs = [[None, None], [None, None]]
  CH = 1 << 20
  for k, off in enumerate(range(0, max(len(d1), len(d2)), CH)):
    slot = k % 2
    pw.wait(slot)
    bufs[slot] = [bytearray(d1[off:off + CH]), bytearray(d2[off:off + CH])]   # a refilled staging slot
    pw.submit(slot, [bytes(b) if b else None for b in bufs[slot]])
  pw.close()
  s1.close()
  s2.close()
  for t in ts:
    t.join()
  assert got[0][0] == d1 and got[1][0] == d2


def test_pair_writer_reports_a_write_error(tmp_path):
  class Broken:
    gz = False

    def write(self, data):
      raise BrokenPipeError('reader went away')
  ok = FS.FastqSink(str(tmp_path / 'ok'))
  pw = FS.PairWriter([ok, Broken()])
  pw.submit(0, [b'@r\nA\n+\n~\n', b'@r\nC\n+\n~\n'])
  with pytest.raises(BrokenPipeError):
    pw.wait(0)
  with pytest.raises(BrokenPipeError):
    pw.close()
  ok.close()
  assert open(str(tmp_path / 'ok'), 'rb').read() == b'@r\nA\n+\n~\n'
