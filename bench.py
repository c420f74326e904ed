#!/usr/bin/env python3
"""Benchmark: paired 2x150 bp templates/s for `generate-reads` at 30x WGS on 1/2/4/8 MI355X.

Default workload (`--workload wgs`, BASELINE.json metric, configs[3]'s genome at every N): the whole synthetic GRCh37
(24 contigs + MT at their real lengths, one BED interval per contig, i.i.d. ACGT with N caps and a centromere gap,
~1.3 variants/kbp: SNV/INS/DEL, long insertions, deliberate overlaps, phased diploid), read model hiseq-X-v2.5-Garvan
(the built-in 2x150 model; SURVEY.md Finding 3), coverage 30, seed 7, perfect reads, rng=mitty (MT19937-exact).  The
reference's work-unit list (readgenerate.py:129-159: 25 regions x 2 copies x 2 passes = 100 units) is dealt to the
ranks by mitty_amd.distributed's LPT plan.  One step = the whole genome's job: every haplotype spliced on the device,
every unit sampled and emitted into the device FASTQ arenas, which are recycled per batch of units (the bytes of a
batch are complete in HBM before the next batch overwrites them; at N = 1 a whole genome's 229 GB of FASTQ would not
fit one GPU beside its inputs).  The same workload runs at every N (strong scaling: total work fixed), and at N > 1 an
RCCL all-reduce of the per-rank template and byte counts closes each step (the counts the file writer turns into
file offsets).  Inputs (contigs and variant arrays) are resident in HBM before timing.

`--workload chr1`: BASELINE configs[1] (one chr1-shaped contig, 4 units per step; N = 1 only).
`--tumor-normal`: BASELINE configs[4] on one GPU.

N ranks: `python bench.py --gpus N` starts N rank processes itself (before any GPU call); under torchrun WORLD_SIZE
must equal --gpus.  `MH_DIST_BACKEND=gloo` rehearses the plan with several ranks on one GPU.

Prints one JSON line (rank 0).  `roofline` is for the emission writer (k_emit_tiles): algorithmic bytes per launch =
sum over kept templates of 2*rlen (haplotype bases gathered) + FASTQ bytes written (both files), divided by the
launch's HIP-event duration on the writer's stream; `stage_ms` gives every stage per step.  At N = 1 the line also
carries `cpu_baseline` (the CPU oracle on the host cores, and the configs[0] CPU config beside it) and `end_to_end`
(the whole `generate-reads` command on chr1: files in, FASTQ to /dev/null).
"""
import argparse
import collections
import glob
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CHR1 = 249_250_621
PEAK_HBM_GBS = 8000.0
# stage timers that bracket other stages and cross streams (their intervals include queue waits behind earlier work):
# reported apart from the per-stage times
SPANS = ('emit', 'sample', 'splice')
STAGE_NOTE = ('stage_ms: per step, each stage = HIP events recorded on its own stream around its kernels (kernel '
              'time plus launch gaps; stages on different streams overlap, so they sum past ms_per_step); span_ms: '
              'the outer spans, which start on one stream and end on another and include queue waits')
METRIC = 'paired 2x150bp reads/sec at 30x WGS, 1/2/4/8 MI355X; qname POS/CIGAR bit-exact'


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=10)
  # (the first bench process on a fresh box ran 13 % slow with 2 warm-up steps in three calls, and at the rate of the
  # later processes with 40: profiles/r04/firstrun/)
  ap.add_argument('--warmup', type=int, default=30)
  ap.add_argument('--model', default='hiseq-X-v2.5-Garvan')
  ap.add_argument('--coverage', type=float, default=30.0)
  ap.add_argument('--length', type=int, default=CHR1)
  ap.add_argument('--seed', type=int, default=7)
  ap.add_argument('--rng', default='mitty', choices=['mitty', 'philox'])
  ap.add_argument('--corrupt', action='store_true', help='fused BQ corruption (BASELINE configs[2])')
  ap.add_argument('--cpu-baseline-mbp', type=float, default=100.0,
                  help='chr1 leg of the CPU baseline: the chr1 job\'s units on the first N Mbp of the contig (0 = skip)')
  ap.add_argument('--cpu-baseline-frac', type=float, default=0.25,
                  help='WGS leg of the CPU baseline: all 100 work units, each on the first FRAC of its region '
                       '(0 = skip)')
  ap.add_argument('--cpu-workers', type=int, default=0,
                  help='CPU baseline worker processes, the reference\'s --threads (SURVEY.md §8(d): min(host cores, '
                       '#units)); 0 = the CPU share this process may use, measured (affinity, cgroup cpu.max); a side '
                       'leg runs one process per unit (100) on that share, labelled')
  ap.add_argument('--verify', action='store_true',
                  help='wgs, N = 1: after the timed steps, run one more step unit by unit and compare every unit\'s '
                       'FASTQ bytes (sha256 of its arena range, both files) with the CPU oracle\'s digests')
  ap.add_argument('--no-cpu-baseline', action='store_true')
  ap.add_argument('--no-prime', action='store_true',
                  help='skip the HBM first-touch pass (scripts/prime_hbm.py) run before the GPU is used')
  ap.add_argument('--no-e2e', action='store_true', help='skip the end-to-end (files in, /dev/null out) leg')
  ap.add_argument('--e2e-gz', action=argparse.BooleanOptionalAction, default=True,
                  help='end-to-end leg: also with BGZF-compressed output (host deflate, level 1)')
  ap.add_argument('--stages', action='store_true', help='print per-stage timings to stderr')
  ap.add_argument('--tumor-normal', action='store_true',
                  help='BASELINE configs[4] on one GPU: tumor 60x + normal 30x, 2x250 model (1kg-pcr-free), mixed '
                       'into one FASTQ pair, + the god-aligner BAM records built and coordinate-sorted in HBM')
  ap.add_argument('--bam-hbm-gb', type=float, default=0.0,
                  help='--tumor-normal: bound the BAM store in HBM (GiB; 0 = unbounded): records past it spill to host '
                       'memory and the file is assembled window by window (mh_bam_set_capacity)')
  ap.add_argument('--tn-length', type=int, default=50_000_000,
                  help='--tumor-normal: contig length (a chr1 job at 90x of 2x250 does not fit one GPU with its BAM)')
  ap.add_argument('--tn-genome', action='store_true',
                  help='--tumor-normal --gpus N: the whole synthetic GRCh37 (lengths x --genome-scale) instead of one '
                       '--tn-length contig')
  ap.add_argument('--workload', default='wgs', choices=['wgs', 'chr1'],
                  help='wgs: whole synthetic GRCh37 at every N (the metric; configs[3]); chr1: configs[1], N = 1')
  ap.add_argument('--genome-scale', type=float, default=1.0,
                  help='wgs: contig lengths scaled by this (rehearsals of the plan; 1 = GRCh37)')
  ap.add_argument('--batch-draws', type=float, default=64e6,
                  help='wgs: units are sampled in batches of about this many template draws (a chr1 job is 30 M); '
                       'the FASTQ arenas are recycled per batch')
  ap.add_argument('--min-batches', type=int, default=2,
                  help='wgs: at least this many batches per rank and step (a rank\'s share at N = 8 is ~1/8 of the '
                       'genome: a second batch keeps its sampling beside its writers; rank 0\'s share timed alone, '
                       'two batches against four: +6.8 %% at N = 8, +4 %% at N = 4, equal at N = 2, round 4; N = 1 '
                       'has six by --batch-draws)')
  ap.add_argument('--plan-share', default=None, metavar='R/N',
                  help='wgs, one GPU, no process group: time only rank R\'s units of the N-rank LPT plan (a projection '
                       'of one rank of an N-GPU run; the JSON says so and is not the metric line)')
  ap.add_argument('--emit-mode', type=int, default=0, choices=[0, 2, 3],
                  help='0: every unit queued with no host readback (measure pass, tile scan, k_emit_tiles chained on '
                       'the device); 2: the host reads each unit\'s totals before its writer (round 5); 3: the '
                       'single-pass writer k_emit_fused (no measure pass)')
  ap.add_argument('--prefetch', action=argparse.BooleanOptionalAction, default=True,
                  help='wgs: splice the next batch\'s haplotypes and generate its MT19937 word streams while the '
                       'current batch is written (mh_prefetch_haplotypes_vset) instead of at the next batch\'s start '
                       '(+1.8 %%, 4 of 4 same-box alternations, profiles/r06/experiments/haplotype_prefetch_ab)')
  ap.add_argument('--prefetch-after', type=int, default=1,
                  help='--prefetch: once this unit of the batch is queued (-1: before the first; 1 measured best: '
                       '+2.2 %% over 0 and +0.6 %% over -1, 4 of 4 alternations, '
                       'profiles/r06/experiments/haplotype_prefetch_ab/placement)')
  ap.add_argument('--prefetch-last-after', type=int, default=-1,
                  help='--prefetch, the step\'s last batch (the next step\'s first batch prefetched): after this unit '
                       '(-1, before its first: the last batch is short and the next step\'s first batch has many '
                       'haplotypes; +1.2 %% over 0, profiles/r06/experiments/haplotype_prefetch_ab/words_last_batch)')
  ap.add_argument('--synth-workers', type=int, default=8, help='processes building the synthetic inputs')
  ap.add_argument('--cpu-config0', action=argparse.BooleanOptionalAction, default=True,
                  help='N = 1: also time the CPU oracle on BASELINE configs[0] (hg001.bed: 2 x 1 Mbp, 1kg-pcr-free, '
                       '--threads 2)')
  return ap.parse_args()


def roofline(stages, kept, b1, b2, rlen, kernel, steps, workload='chr1', world=1):
  agg = {}
  for name, ms in stages:
    agg.setdefault(name, [0.0, 0])
    agg[name][0] += ms
    agg[name][1] += 1
  ew_ms, ew_n = agg.get('emit_write', [0.0, 0])
  alg_bytes = 2 * rlen * kept + b1 + b2                       # this rank's algorithmic bytes over the timed steps
  achieved = alg_bytes / (ew_ms * 1e-3) / 1e9 if ew_ms > 0 else None
  traffic = None   # measured in separate rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE), see profiles/pmc_*.json
  pmc = sorted(glob.glob(os.path.join(REPO, 'profiles', 'pmc_{}_*.json'.format(kernel))))
  traffic_src = None
  for path in reversed(pmc if workload else []):   # the latest summary of this workload
    try:
      with open(path) as fp:
        d = json.load(fp)
    except Exception:
      continue
    if d.get('rlen') == rlen and d.get('workload', 'chr1' if d.get('length') == CHR1 else None) == workload:
      traffic = d.get('hbm_bytes_per_launch')
      traffic_src = os.path.relpath(path, REPO)
      break
  stage_ms = {k: round(v[0] / steps, 3) for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])
              if k not in SPANS}
  span_ms = {k: round(v[0] / steps, 3) for k, v in agg.items() if k in SPANS}
  hap_bytes = 2 * rlen * kept                                   # haplotype bases gathered (the read side alone)
  read_gbs = hap_bytes / (ew_ms * 1e-3) / 1e9 if ew_ms > 0 else None
  return {'kernel': kernel, 'bound': 'hbm', 'achieved': achieved, 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
          'frac': (achieved / PEAK_HBM_GBS) if achieved else None, 'traffic': traffic,
          'traffic_source': (('PMC passes (FETCH_SIZE, WRITE_SIZE) of this workload, ' if world == 1 else
                              'borrowed from the N = 1 PMC passes of this workload (not measured at this N), ') +
                             traffic_src) if traffic_src else None,
          'algorithmic_bytes_per_launch': alg_bytes / max(ew_n, 1),
          'avg_launch_ms': ew_ms / max(ew_n, 1),
          'read_bytes_per_launch': hap_bytes / max(ew_n, 1),
          'read_only_achieved': read_gbs,
          'read_only_frac': read_gbs / PEAK_HBM_GBS if read_gbs else None,
          # the north star's "HBM-read roofline" counts only the haplotype bytes read; the kernel also writes the FASTQ
          # (W per template against R = 2 rlen read), so at the full 8 TB/s for R + W its read-only fraction would be
          # R / (R + W): the highest read_only_frac this byte mix allows (DESIGN.md, round-6 performance)
          'read_only_ceiling': hap_bytes / alg_bytes if alg_bytes else None}, stage_ms, span_ms


def corrupt_roofline(stages, kept, b1, b2, rlen):
  """The corruption pass, timed by HIP events on the writer stream.  Default (corruption rows): k_cr_cols, stage
  'emit_corrupt_rows', before each writer — per 15-base block one 16-byte row slot and one 4-byte code word written
  (20 B per 15 bases); the writer (stage 'emit_write') lays them into the records.  In place (tables too large for
  the row pass's LDS, or the LDS-image writer): k_cr_recs + k_cr_inplace, stage 'emit_corrupt', after each writer — per base one read (the block's bases) and one quality
  written, the substituted bases written back (4.7 % under hiseq-X-v2.5-Garvan), 8 bytes of record word read and one
  '\n' per record.  Either is bound by VALU issue (Philox rounds and the table walk), not by HBM."""
  rows = any(k == 'emit_corrupt_rows' for k, _ in stages)
  name = 'emit_corrupt_rows' if rows else 'emit_corrupt'
  ms = sum(v for k, v in stages if k == name)
  n = sum(1 for k, _ in stages if k == name)
  bases = 2 * rlen * kept   # (upper bound: reads cut by the haplotype end are shorter)
  alg = bases * 20 / 15 if rows else bases * (2 + 0.047) + 2 * kept * 9
  gbs = alg / (ms * 1e-3) / 1e9 if ms > 0 else None
  return {'kernel': 'k_cr_cols' if rows else 'k_cr_inplace', 'bound': 'valu', 'avg_launch_ms': ms / max(n, 1),
          'algorithmic_bytes_per_launch': alg / max(n, 1), 'achieved_gbs': gbs,
          'hbm_frac': gbs / PEAK_HBM_GBS if gbs else None,
          'bases_per_s': bases / (ms * 1e-3) if ms > 0 else None}


class LazyCounts:
  """The (kept, bytes1, bytes2) of units queued with Engine.run_units(lazy=True), read after the timed region: a step
  returns getter(n) for its n units, so no step waits for its writers (the next step's splice and sampling run
  beside them, as the reference's worker pool runs the next units while earlier ones are written)."""

  def __init__(self, eng):
    self.eng = eng
    self.q = collections.deque()

  def getter(self, n):
    memo = []

    def get():   # (getters are called in step order; each reads its units once)
      if not memo:
        while len(self.q) < n:
          self.q.extend(self.eng.collect())
        res = [self.q.popleft() for _ in range(n)]
        memo.append((sum(r[1] for r in res), sum(r[2] for r in res), sum(r[3] for r in res)))
      return memo[0]
    return get


def timed(step, steps, warmup, eng, dist):
  def barrier():
    if dist is not None:
      dist.barrier()

  for _ in range(warmup):
    step()()
  eng.ctx.enable_timing(True)
  barrier()
  eng.ctx.sync()
  t0 = time.perf_counter()
  done = [step() for _ in range(steps)]   # each step's counts: read once its units have landed
  eng.ctx.sync()
  barrier()
  dt = time.perf_counter() - t0
  kept = b1 = b2 = 0
  for get in done:
    k, x1, x2 = get()
    kept += k
    b1 += x1
    b2 += x2
  stages = eng.ctx.stage_times()
  eng.ctx.enable_timing(False)
  return dt, kept, b1, b2, stages


def launch_ranks(n):
  """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
  MASTER_* as torchrun sets them) and exit with the worst exit status.  Nothing here touches the GPU (the ranks are
  children, not an exec)."""
  import signal
  import socket
  import subprocess
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  procs = []
  for r in range(n):
    env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
               MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
  rc = 0
  try:
    while procs:
      for p in list(procs):
        code = p.poll()
        if code is None:
          continue
        procs.remove(p)
        if code != 0:
          rc = rc or code
          for q in procs:   # one rank failed: the others would wait in a collective forever
            q.send_signal(signal.SIGTERM)
      time.sleep(0.05)
  finally:
    for q in procs:
      q.kill()
  return 1 if rc < 0 else rc


def main():
  a = parse()
  ws = os.environ.get('WORLD_SIZE')
  if ws is None and a.gpus > 1:
    sys.exit(launch_ranks(a.gpus))
  world = int(ws or '1')
  if world != a.gpus:
    sys.exit('bench.py: --gpus {} but WORLD_SIZE={}: the launcher and the flag disagree'.format(a.gpus, world))
  rank = int(os.environ.get('RANK', '0'))
  local = int(os.environ.get('LOCAL_RANK', '0'))
  global PRIME_S
  a.prime_s = PRIME_S = prime_hbm(a, local)
  if a.tumor_normal and world > 1:
    run_tumor_normal_ranks(a, rank, world, local)
    return
  if a.tumor_normal or a.workload == 'chr1':
    if world != 1:
      sys.exit('bench.py: --workload chr1 is a one-GPU config')
    run_tumor_normal(a) if a.tumor_normal else run_chr1(a)
    return
  run_genome(a, rank, world, local)


def prime_hbm(a, local):
  """Before this process touches the GPU: a child process writes most of the HBM of this rank's GPU once
  (scripts/prime_hbm.py).  On a fresh box the first process to use the HBM ran ~13 % slow throughout, warm-up steps
  or not; the bench then measures the steady state the later processes see.  The seconds go in the JSON line."""
  if a.no_prime:
    return None
  import subprocess
  t0 = time.perf_counter()
  r = subprocess.run([sys.executable, os.path.join(REPO, 'scripts', 'prime_hbm.py'), str(local)],
                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
  sys.stderr.write(r.stdout)
  return round(time.perf_counter() - t0, 2)


PRIME_S = None   # the priming pass's seconds in this process (None: it did not run)


def hbm_setup():
  """Whether this process's GPU was primed (scripts/prime_hbm.py in a child process before the first GPU call) and the
  pass's seconds: on a fresh box the first process to use the GPU ran 2-13 % slower throughout without it (DESIGN.md
  "the first process")."""
  return {'primed': PRIME_S is not None, 'prime_hbm_s': PRIME_S,
          'unprimed_first_process': 'a first GPU process on a newly taken box runs 0-10 % (median ~5 %) slower '
                                    'throughout without the pass: profiles/r05/fresh_box_ab.json'}

def run_chr1(a):
  import numpy as np
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from mitty_amd.readmodel import get_read_model

  _, model = get_read_model(a.model + '.pkl')
  rlen = int(model['mean_rlen'])
  p, passes = _native.read_model_params(rlen, a.coverage)
  seq = synth.contig(a.length, 1000)
  recs = synth.variants(seq, 2000)
  copies = synth.copies_soa(recs)
  units = _native.work_units(a.seed, [2], passes)

  eng = Engine(0, a.emit_mode)
  if a.corrupt:
    eng.ctx.set_corruption(True, model['cum_bq_mat'], 10 ** (-np.arange(100) / 10), a.seed)
  eng.load_region(0, ('1', 0, a.length), seq)
  for cpy in range(len(copies)):   # inputs resident in HBM before timing: contig and both copies' variants
    eng.upload_variants(0, cpy, copies[cpy])
  kernel = 'k_emit_tiles'

  counts = LazyCounts(eng)

  def step():
    # one chr1 job; consecutive jobs pipeline on the device (this job's splice and sampling run while the previous
    # job's last FASTQ writers drain); the timed region ends with a full synchronisation
    eng.drop_haplotypes()
    eng.ctx.reset_output()
    eng.run_units([(ps, ri, cpy, s) for ps, (ri, cpy, s) in enumerate(units)], lambda r, c: copies[c], p,
                  rlen, model['cum_tlen'], 'SYN', 0, True, a.rng, lazy=True)
    return counts.getter(len(units))

  dt, kept, b1, b2, stages = timed(step, a.steps, a.warmup, eng, None)
  eng.close()
  roof, stage_ms, span_ms = roofline(stages, kept, b1, b2, rlen, kernel, a.steps,
                                     'chr1_corrupt' if a.corrupt else 'chr1')
  if a.stages:
    print(json.dumps(stage_ms), file=sys.stderr)
  corrupt_pass = None
  if a.corrupt:
    corrupt_pass = corrupt_roofline(stages, kept, b1, b2, rlen)

  e2e = None
  if not a.no_e2e and not a.corrupt and a.rng == 'mitty':
    e2e = end_to_end(a, seq, recs, model, kept // a.steps)
  cpu = None
  if not a.no_cpu_baseline and a.cpu_baseline_mbp > 0:
    cpu = cpu_baseline(a, seq, recs, p, rlen, model, units)

  ms_per_step = dt / a.steps * 1e3
  out = {
    'metric': METRIC,
    'value': kept / dt,
    'unit': 'templates/s',
    'n_gpus': 1,
    'steps': a.steps,
    'warmup': a.warmup,
    'ms_per_step': ms_per_step,
    'higher_is_better': True,
    'scaling': 'weak',
    'vs_baseline': None,
    'dtype': 'int64+u8',
    'data': 'synthetic chr1-shaped contig + ~1.3/kbp phased diploid variants (mitty_amd.synth), seed-fixed',
    'config': {'workload': 'generate-reads chr1 (249,250,621 bp) diploid, {} 2x{} PE, {}x, rng={}{} '
                           '(BASELINE configs[{}])'.format(a.model, rlen, a.coverage, a.rng,
                                                           ', +BQ corruption' if a.corrupt else '',
                                                           2 if a.corrupt else 1),
               'read_model': a.model, 'coverage': a.coverage, 'contig_bp': a.length, 'units': len(units),
               'templates_per_step': kept // a.steps, 'parallelism': 'single GPU'},
    'roofline': roof,
    'corrupt_pass': corrupt_pass,
    'cpu_baseline': cpu,
    'end_to_end': e2e,
    'stage_ms': stage_ms,
    'span_ms': span_ms,
    'stage_note': STAGE_NOTE,
    'fastq_bytes_per_template': (b1 + b2) / max(kept, 1),
    'setup_s': hbm_setup(),
    'host_cpus': os.cpu_count(),
  }
  print(json.dumps(out), flush=True)


def run_tumor_normal(a):
  """BASELINE configs[4] (one GPU, a contig of --tn-length): per step, the normal sample at 30x and the tumor sample
  at 60x (2x250, 1kg-pcr-free) generated into the same FASTQ arenas — the mix — then the god-aligner's perfect BAM
  from the arenas: every record parsed and encoded (write_perfect_reads, god_aligner.py:153-183) and coordinate-sorted
  (samtools sort's order) in HBM.  The BAM file itself (host BGZF + BAI) is written once after the timed steps."""
  from mitty_amd import _native, synth
  from mitty_amd.engine import Engine
  from mitty_amd.readmodel import get_read_model

  _, model = get_read_model('1kg-pcr-free.pkl')
  rlen = int(model['mean_rlen'])
  L = a.tn_length
  seq = synth.contig(L, 1000)
  eng = Engine(0)
  cap = int(a.bam_hbm_gb * (1 << 30))
  eng.ctx.bam_set_capacity(cap)
  jobs = []
  # the tumor's variants: an independent synthetic set of the same density (its own haplotypes)
  for k, (name, cov, vseed) in enumerate((('NORMAL', 30.0, 2000), ('TUMOR', 60.0, 2001))):
    copies = synth.copies_soa(synth.variants(seq, vseed))
    eng.load_region(k, ('1', 0, L), seq)
    for cpy in range(2):
      eng.upload_variants(k, cpy, copies[cpy])
    p, passes = _native.read_model_params(rlen, cov)
    jobs.append((name, k, copies, p, _native.work_units(a.seed + k, [2], passes)))

  def step():
    eng.drop_haplotypes()
    eng.ctx.reset_output()
    tot = [0, 0, 0]
    for name, k, copies, p, units in jobs:
      res = eng.run_units([(ps, k, cpy, s) for ps, (_, cpy, s) in enumerate(units)],
                          lambda r, c, cp=copies: cp[c], p, rlen, model['cum_tlen'], name, 0, True, 'mitty')
      for r in res:
        tot[0] += r[1]
        tot[1] += r[2]
        tot[2] += r[3]
    eng.ctx.bam_set_refs(['1'], [L])
    eng.ctx.bam_add_output()
    eng.ctx.bam_sort()
    return lambda: tuple(tot)

  dt, kept, b1, b2, stages = timed(step, a.steps, a.warmup, eng, None)
  n_rec, bam_bytes = eng.ctx.bam_records()
  spilled = eng.ctx.bam_spilled()
  threads = min(16, os.cpu_count() or 1)
  bam_file_s = None
  if bam_bytes <= (16 << 30):   # (the host deflate leg: ~1 GB/s on 16 threads, skipped for chr1-size stores)
    t0 = time.perf_counter()
    eng.ctx.bam_write('/dev/null', '@HD\tVN:1.0\tSO:coordinate\n', level=1, threads=threads)
    bam_file_s = time.perf_counter() - t0
  # the same file with the record blocks deflated on the device (mh_bam_write_gpu) and its BAI: the whole configs[4]
  # pipeline per step is then the timed step + this
  # (twice: the first call also allocates the compressed-output buffer and the staging slots, which a per-step
  # pipeline keeps; the second is the steady state the per-step figure below uses)
  t0 = time.perf_counter()
  eng.ctx.bam_write_gpu('/dev/null', '@HD\tVN:1.0\tSO:coordinate\n', bai_path='/dev/null')
  bam_gpu_first_s = time.perf_counter() - t0
  t0 = time.perf_counter()
  _, _, bam_gpu_file_bytes = eng.ctx.bam_write_gpu('/dev/null', '@HD\tVN:1.0\tSO:coordinate\n', bai_path='/dev/null')
  bam_gpu_s = time.perf_counter() - t0
  eng.close()
  agg = {}
  for name, ms in stages:
    agg[name] = agg.get(name, 0.0) + ms
  ms_per_step = dt / a.steps * 1e3
  print(json.dumps({
    'metric': 'paired 2x250 templates/s, tumor 60x + normal 30x mixed, + god-aligner BAM records sorted in HBM',
    'value': kept / dt, 'unit': 'templates/s', 'n_gpus': 1, 'steps': a.steps, 'warmup': a.warmup,
    'ms_per_step': ms_per_step, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
    'dtype': 'int64+u8', 'data': 'synthetic contig + two independent synthetic variant sets (mitty_amd.synth)',
    'config': {'workload': 'generate-reads tumor/normal mix (BASELINE configs[4], one GPU, {} bp contig)'.format(L),
               'read_model': '1kg-pcr-free', 'coverage': {'TUMOR': 60, 'NORMAL': 30},
               'templates_per_step': kept // a.steps, 'bam_records_per_step': n_rec},
    'bam_bytes_per_step': bam_bytes, 'fastq_bytes_per_step': (b1 + b2) // a.steps,
    'bam_store': {'hbm_capacity_bytes': cap or None, 'spilled': spilled},
    'bam_file_after_timing': {'seconds': bam_file_s, 'level': 1, 'threads': threads, 'sink': '/dev/null'},
    'bam_file_gpu': {'seconds': bam_gpu_s, 'first_call_seconds': bam_gpu_first_s, 'file_bytes': bam_gpu_file_bytes,
                     'sink': '/dev/null', 'bai': True,
                     'note': 'the record blocks deflated on the device (mh_bam_write_gpu), D2H of the compressed '
                             'bytes, header block and BAI on the host; seconds = a second call (the buffers the '
                             'first one allocated are reused), first_call_seconds = the first'},
    'with_bam_file': {'seconds_per_step': ms_per_step / 1e3 + bam_gpu_s,
                      'value': (kept / a.steps) / (ms_per_step / 1e3 + bam_gpu_s), 'unit': 'templates/s',
                      'note': 'the timed step (mix + BAM records sorted in HBM) plus the BAM file with BAI written '
                              'from them (bam_file_gpu), per step'},
    'stage_ms': {k: round(v / a.steps, 3) for k, v in sorted(agg.items(), key=lambda kv: -kv[1])},
    'setup_s': hbm_setup(),
    'host_cpus': os.cpu_count()}), flush=True)


def run_tumor_normal_ranks(a, rank, world, local):
  """BASELINE configs[4] on N GPUs (one process per GPU, RCCL): the normal (30x) and tumor (60x) samples' work units
  (2x250, 1kg-pcr-free) dealt to the ranks by LPT; per step every rank generates its units into its arenas, turns
  them into BAM records on its GPU, partitions the records by coordinate range and the all-to-all (RCCL over xGMI)
  moves each to its range's rank, which sorts its range in HBM (mitty_amd.distributed: no rank merges the others'
  records).  After the timed steps the BAM and BAI are written once, every rank deflating its range's blocks on its
  GPU (the per-step file leg in the line)."""
  import torch
  import torch.distributed as tdist
  from mitty_amd import _native, synth
  from mitty_amd import distributed as D
  from mitty_amd.readmodel import get_read_model
  _, model = get_read_model('1kg-pcr-free.pkl')
  rlen = int(model['mean_rlen'])
  contigs = synth.genome_contigs(a.genome_scale) if a.tn_genome else [('1', a.tn_length)]
  samples = []
  units = []   # (sample, ri, cpy, seed, ps)
  for k, (name, cov) in enumerate((('NORMAL', 30.0), ('TUMOR', 60.0))):
    p, passes = _native.read_model_params(rlen, cov)
    samples.append((name, p))
    for ps, (ri, cpy, s) in enumerate(_native.work_units(a.seed + k, [2] * len(contigs), passes)):
      units.append((k, ri, cpy, s, ps))
  weights = [contigs[ri][1] * samples[k][1] for k, ri, _, _, _ in units]
  pieces = D.plan_pieces(weights, world, 'lpt')
  mine = [i for i, pc in enumerate(pieces) if pc[3] == rank]
  regions = sorted({units[i][1] for i in mine})
  t_synth = time.perf_counter()
  data = synth.genome_regions(contigs, regions, workers=max(1, a.synth_workers // world))
  tumor = {ri: synth.copies_soa(synth.variants(data[ri][0], 3000 + ri)) for ri in regions}
  t_synth = time.perf_counter() - t_synth
  local = local % max(1, torch.cuda.device_count())
  torch.cuda.set_device(local)
  tdist.init_process_group(os.environ.get('MH_DIST_BACKEND', 'nccl'))
  be = D.DeviceBackend(local)
  eng = be.eng
  for ri in regions:
    name, length = contigs[ri]
    seq, _, normal = data[ri]
    for k, copies in enumerate((normal, tumor[ri])):
      eng.load_region(2 * ri + k, (name, 0, length), seq)
      for cpy in (0, 1):
        eng.upload_variants(2 * ri + k, cpy, copies[cpy])
  soa = lambda r, c: (data[r // 2][2] if r % 2 == 0 else tumor[r // 2])[c]
  # this rank's batches: its units of one sample at a time (one read model per sampling batch), ~a.batch_draws each
  batches = []
  for k in (0, 1):
    cur, draws = [], 0
    for i in mine:
      sk, ri, cpy, s, ps = units[i]
      if sk != k:
        continue
      cur.append(i)
      draws += contigs[ri][1] * samples[k][1] * 1.2
      if draws >= a.batch_draws:
        batches.append((k, cur))
        cur, draws = [], 0
    if cur:
      batches.append((k, cur))
  rounds = int(D._allgather_i64([len(batches)], world, None)[:, 0].max())   # (the exchange is collective)
  refs = [(name, L) for name, L in contigs]
  splitters = D.range_splitters([(name, 0, L) for name, L in contigs], refs, world)
  cap = int(a.bam_hbm_gb * (1 << 30))
  stats = {}
  dev = 'cuda' if tdist.get_backend() == 'nccl' else 'cpu'
  counts = torch.zeros(3, dtype=torch.int64, device=dev)

  def step():
    eng.drop_haplotypes()
    be.bam_begin(refs, cap)
    kept = b1 = b2 = 0
    for r in range(rounds):
      part = None
      if r < len(batches):
        k, idx = batches[r]
        eng.ctx.reset_output()
        res = eng.run_units([(units[i][4], 2 * units[i][1] + k, units[i][2], units[i][3]) for i in idx], soa,
                            samples[k][1], rlen, model['cum_tlen'], samples[k][0], 0, True, 'mitty')
        kept += sum(x[1] for x in res)
        b1 += sum(x[2] for x in res)
        b2 += sum(x[3] for x in res)
        part = be.bam_partition(splitters, idx[0] << 32)
      D._bam_exchange(be, part, world, None, stats)
    be.rctx.bam_sort()
    counts.copy_(torch.tensor([kept, b1, b2], dtype=torch.int64))
    tdist.all_reduce(counts)
    return lambda: (kept, b1, b2)

  for _ in range(a.warmup):
    step()
  eng.ctx.sync()
  be.rctx.sync()
  torch.cuda.synchronize()
  tdist.barrier()
  t0 = time.perf_counter()
  kept = b1 = b2 = 0
  for _ in range(a.steps):
    k_, x1, x2 = step()()
    kept, b1, b2 = kept + k_, b1 + x1, b2 + x2
  eng.ctx.sync()
  be.rctx.sync()
  torch.cuda.synchronize()
  tdist.barrier()
  dt = time.perf_counter() - t0
  t = torch.tensor([dt], dtype=torch.float64, device=dev)
  tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
  dt = float(t.item())
  n_rec, nbytes = be.bam_range()
  tot = D.allreduce_i64([kept, b1, b2, n_rec, nbytes])
  # the BAM file and its BAI from the last step's ranges (each rank deflates its blocks on its GPU)
  path = os.path.join('/dev/shm' if os.path.isdir('/dev/shm') else tempfile.gettempdir(),
                      'mh_tn_{}.bam'.format(os.environ.get('MASTER_PORT', '0')))
  tdist.barrier()
  t1 = time.perf_counter()
  D._bam_write_ranges(be, rank, world, None, path, '@HD\tVN:1.0\tSO:coordinate\n', refs)
  tdist.barrier()
  file_s = time.perf_counter() - t1
  file_bytes = os.path.getsize(path) if rank == 0 else 0
  if rank == 0:
    os.remove(path)
    os.remove(path + '.bai')
  be.close()
  tdist.destroy_process_group()
  if rank != 0:
    return
  ms_per_step = dt / a.steps * 1e3
  per_step = tot[0] / a.steps
  print(json.dumps({
    'metric': 'paired 2x250 templates/s, tumor 60x + normal 30x mixed, + god-aligner BAM records sorted in HBM, '
              '{} GPUs'.format(world),
    'value': tot[0] / dt, 'unit': 'templates/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
    'ms_per_step': ms_per_step, 'higher_is_better': True, 'scaling': 'strong', 'vs_baseline': None,
    'dtype': 'int64+u8', 'data': 'synthetic contigs + two independent synthetic variant sets (mitty_amd.synth)',
    'config': {'workload': 'generate-reads tumor/normal mix (BASELINE configs[4]) on {} GPUs: {}'.format(
                   world, 'whole GRCh37 (lengths x{})'.format(a.genome_scale) if a.tn_genome
                   else '{} bp contig'.format(a.tn_length)),
               'read_model': '1kg-pcr-free', 'coverage': {'TUMOR': 60, 'NORMAL': 30}, 'units': len(units),
               'templates_per_step': per_step, 'bam_records_per_step': tot[3], 'rounds_per_step': rounds,
               'parallelism': 'unit-shard (LPT) x{}, BAM by coordinate range (all-to-all)'.format(world),
               'collective_backend': os.environ.get('MH_DIST_BACKEND', 'nccl')},
    'bam_bytes_per_step': tot[4], 'fastq_bytes_per_step': (tot[1] + tot[2]) // a.steps,
    'bam_store': {'hbm_capacity_bytes_per_rank': cap or None},
    'bam_file_ranges': {'seconds': file_s, 'file_bytes': file_bytes, 'bai': True,
                        'note': 'every rank deflates the blocks that start in its range on its GPU into a part file, '
                                'the parts are copied into one BAM at their offsets, the BAI joined on rank 0'},
    'with_bam_file': {'seconds_per_step': ms_per_step / 1e3 + file_s,
                      'value': per_step / (ms_per_step / 1e3 + file_s), 'unit': 'templates/s'},
    'setup_s': dict(synth_inputs=round(t_synth, 2), **hbm_setup()),
    'host_cpus': os.cpu_count()}), flush=True)


SPLIT_KEYS = ('setup_s', 'parse_s', 'run_s', 'gpu_s', 'flush_s', 'fetch_s', 'write_s', 'close_s')


def end_to_end(a, seq, recs, model, kept_per_job):
  """The whole generate-reads command on chr1: FASTA and VCF parsed by the host readers, the GPU job, FASTQ pulled to
  page-locked memory and written to /dev/null (readgenerate.process_multi_threaded).  Input files are written first
  (untimed) to a temp directory."""
  from mitty_amd import synth
  from mitty_amd.lib import fasta as mfasta
  from mitty_amd.lib import vcfio
  from mitty_amd.readmodel import get_read_model
  from mitty_amd.simulation import readgenerate
  d = tempfile.mkdtemp(prefix='mh_e2e_', dir='/tmp')
  try:
    fa, vcf, bed = os.path.join(d, 'chr1.fa'), os.path.join(d, 'chr1.vcf'), os.path.join(d, 'chr1.bed')
    synth.write_fasta(fa, [('1', seq)])
    synth.write_vcf(vcf, [('1', seq)], {'1': recs}, sample='SYN')
    with open(bed, 'w') as fp:
      fp.write('1\t0\t{}\n'.format(len(seq)))
    mod, mdl = get_read_model(a.model + '.pkl')
    t0 = time.perf_counter()
    mfasta.read_fasta(fa)
    t1 = time.perf_counter()
    vcfio.load_variants_soa(vcf, 'SYN', bed)
    t2 = time.perf_counter()
    st = readgenerate.process_multi_threaded(fa, vcf, 'SYN', bed, mod, mdl, a.coverage, '/dev/null', '/dev/null',
                                             seed=a.seed, stage_times=True)
    t3 = time.perf_counter()
    out = {'seconds': t3 - t2, 'value': st['kept'] / (t3 - t2), 'unit': 'templates/s', 'templates': st['kept'],
           'fastq_bytes': st['bytes1'] + st['bytes2'], 'fasta_parse_s': t1 - t0, 'vcf_parse_s': t2 - t1,
           'split_s': {k: round(st[k], 3) for k in SPLIT_KEYS}, 'stages_ms': st.get('stages_ms'),
           'primed': hbm_setup()['primed'],
           'note': 'generate-reads chr1 end to end: host FASTA (249 MB) + VCF parse, GPU job, FASTQ D2H to '
                   'page-locked memory, written to /dev/null; seconds = the whole command'}
    if a.e2e_gz:   # the same with both files BGZF-compressed (what `.gz` output names cost): on the GPU, then on host
      threads = min(16, os.cpu_count() or 1)
      for key, dev in (('gz', True), ('gz_host', False)):
        t4 = time.perf_counter()
        st = readgenerate.process_multi_threaded(fa, vcf, 'SYN', bed, mod, mdl, a.coverage, '/dev/null', '/dev/null',
                                                 seed=a.seed, compress=True, gz_level=1, gz_threads=threads,
                                                 gz_device=dev, stage_times=True)
        t5 = time.perf_counter()
        out[key] = {'seconds': t5 - t4, 'value': st['kept'] / (t5 - t4), 'unit': 'templates/s',
                    'gz_bytes': st['written1'] + st['written2'], 'primed': hbm_setup()['primed'],
                    'split_s': {k: round(st[k], 3) for k in SPLIT_KEYS}, 'stages_ms': st.get('stages_ms'),
                    'note': 'the same command with BGZF output, deflated ' +
                            ('on the GPU from the arenas (mh_output_bgzf), then D2H of the compressed bytes' if dev else
                             'by the host pool (level 1, {} threads) after D2H'.format(threads))}
    return out
  finally:
    for f in glob.glob(os.path.join(d, '*')):
      os.remove(f)
    os.rmdir(d)


def plan_batches(mine, draws_of_region, target, min_batches=1):
  """A rank's units [(ps, ri, cpy, seed)] in batches of about `target` template draws (draws_of_region[ri] per
  unit), in ps order; at least `min_batches` batches when the rank has that many units (so its sampling of one batch
  runs beside its writers of the previous one).  Returns (batches, the batch size used, the rank's draws)."""
  total = sum(int(draws_of_region[u[1]]) for u in mine)
  size = min(target, total / max(1, min_batches))
  batches, cur, draws = [], [], 0
  for u in mine:
    cur.append(u)
    draws += int(draws_of_region[u[1]])
    if draws >= size:
      batches.append(cur)
      cur, draws = [], 0
  if cur:
    batches.append(cur)
  return batches, size, total


def run_genome(a, rank, world, local):
  """The metric's workload at any N: whole synthetic GRCh37, the reference's unit list dealt to the ranks by LPT
  (mitty_amd.distributed.plan_pieces), every unit sampled and emitted by its owner, output in HBM (arenas recycled
  per batch), an all-reduce of the counts closing each step."""
  # a process group at N > 1, and at N = 1 when MH_DIST_BACKEND names one (the RCCL path exercised on one GPU)
  use_pg = world > 1 or bool(os.environ.get('MH_DIST_BACKEND'))
  if use_pg:
    # torch before libmitty_hip: a process holds ONE HIP runtime, and whichever library loads first provides it
    # (ours needs libamdhip64.so.7, which torch's copy satisfies; torch's own libamdhip64.so would not reuse ours)
    import torch  # noqa: F401
  from mitty_amd import _native, synth
  from mitty_amd import distributed as D
  from mitty_amd.readmodel import get_read_model

  _, model = get_read_model(a.model + '.pkl')
  rlen = int(model['mean_rlen'])
  p, passes = _native.read_model_params(rlen, a.coverage)
  contigs = synth.genome_contigs(a.genome_scale)
  units = _native.work_units(a.seed, [2] * len(contigs), passes)     # (region, copy, seed), reference order
  weights = [contigs[ri][1] for ri, _, _ in units]
  plan_world, plan_rank = world, rank
  if a.plan_share:   # projection: one rank's share of an N-rank plan, timed alone on this GPU
    plan_rank, plan_world = (int(x) for x in a.plan_share.split('/'))
    if world != 1 or not 0 <= plan_rank < plan_world:
      sys.exit('bench.py: --plan-share R/N runs in one process (0 <= R < N)')
  pieces = D.plan_pieces(weights, plan_world, 'lpt')                  # 100 units: whole units by LPT at any N
  mine = [(ps, ri, cpy, s) for ps, (ri, cpy, s) in enumerate(units) if pieces[ps][3] == plan_rank]
  regions = sorted({ri for _, ri, _, _ in mine})
  t_synth = time.perf_counter()
  data = synth.genome_regions(contigs, regions, workers=max(1, a.synth_workers // world))
  t_synth = time.perf_counter() - t_synth

  dist = None
  if use_pg:
    import torch
    import torch.distributed as tdist
    if world == 1:   # no launcher: a one-rank group on this host
      os.environ.setdefault('RANK', '0')
      os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
      if 'MASTER_PORT' not in os.environ:
        import socket
        with socket.socket() as sk:
          sk.bind(('127.0.0.1', 0))
          os.environ['MASTER_PORT'] = str(sk.getsockname()[1])
      os.environ['WORLD_SIZE'] = '1'
    local = local % max(1, torch.cuda.device_count())   # rehearsals: several ranks on one GPU
    torch.cuda.set_device(local)
    # MH_DIST_BACKEND=gloo: rehearsal of the multi-rank plan with several ranks on one GPU (RCCL needs one per GPU)
    tdist.init_process_group(os.environ.get('MH_DIST_BACKEND', 'nccl'))
    dist = tdist
    if dist.get_world_size() != world:
      sys.exit('bench.py: the process group has {} ranks, WORLD_SIZE={}'.format(dist.get_world_size(), world))
  from mitty_amd.engine import Engine
  eng = Engine(local, a.emit_mode)
  copies = {}
  for ri in regions:
    name, length = contigs[ri]
    seq, _, copies[ri] = data[ri]
    eng.load_region(ri, (name, 0, length), seq)
    for cpy in (0, 1):
      eng.upload_variants(ri, cpy, copies[ri][cpy])
  kernel = 'k_emit_tiles'
  batches, batch_draws, mine_draws = plan_batches(mine, [L * p * 1.2 for _, L in contigs], a.batch_draws,
                                                  a.min_batches)
  if dist is not None:
    import torch
    dev = 'cuda' if dist.get_backend() == 'nccl' else 'cpu'
    counts = torch.zeros(3, dtype=torch.int64, device=dev)

  lazy = LazyCounts(eng)
  n_mine = sum(len(b) for b in batches)
  prev = []

  def step():
    eng.drop_haplotypes()   # (with --prefetch: this step's first batch's haplotypes were built during the previous step)
    for i, batch in enumerate(batches):
      # the batch's writers append to empty arenas: they run after the previous batch's writers on the writer
      # stream, so a batch's FASTQ is complete in HBM before the next one overwrites it; no host wait on a writer
      # anywhere in the step (the totals are read after the timed region, or at the step's end with N > 1).  With
      # --prefetch the next batch's haplotypes are spliced while this one is written (for the last batch: the next
      # step's first batch, a fresh build kept for it) — every haplotype is still built once per step
      last = i + 1 == len(batches)
      nxt = batches[0] if last else batches[i + 1]
      eng.ctx.reset_output()
      eng.run_units(batch, lambda r, c: copies[r][c], p, rlen, model['cum_tlen'], 'SYN', 0, True, a.rng, lazy=True,
                    prefetch=nxt if a.prefetch else None, prefetch_next_step=last,
                    prefetch_after=a.prefetch_last_after if last else a.prefetch_after)
    get = lazy.getter(n_mine)
    if dist is not None:
      # RCCL over xGMI: the previous step's template / byte totals (file offsets in the file writer), all-reduced once
      # this step's units are queued — its writers have run beside this step's sampling, so no rank waits on them
      if prev:
        counts.copy_(torch.tensor(list(prev.pop()()), dtype=torch.int64))
        dist.all_reduce(counts)
      prev.append(get)
    return get

  steps, warmup = a.steps, a.warmup
  dt, kept, b1, b2, stages = timed(step, steps, warmup, eng, dist)
  verify = None
  if a.verify:
    if world != 1 or a.plan_share or a.rng != 'mitty':
      sys.exit('bench.py: --verify is the N = 1, rng=mitty WGS line')
    verify = verify_wgs(a, eng, batches, copies, contigs, data, units, p, rlen, model)
  live, peak = _native.device_live_bytes()   # the library's device blocks in use (not its block cache), and their peak
  eng.close()
  kept_all, b1_all, b2_all, n_units = kept, b1, b2, len(mine)
  backend, seen = None, 1
  if dist is not None:
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    c = torch.tensor([kept, b1, b2, len(mine)], dtype=torch.int64, device=dev)
    dist.all_reduce(c)
    kept_all, b1_all, b2_all, n_units = (int(x) for x in c.tolist())
    backend, seen = dist.get_backend(), dist.get_world_size()
  workload = 'wgs' if a.genome_scale == 1 else None
  roof, stage_ms, span_ms = roofline(stages, kept, b1, b2, rlen, kernel, steps, workload, world)
  cpu = e2e = None
  if world == 1 and not a.plan_share:
    seq1, recs1, _ = data[0]
    if not a.no_e2e and a.genome_scale == 1 and a.rng == 'mitty':
      e2e = end_to_end(a, seq1, recs1, model, None)
    if not a.no_cpu_baseline:
      legs = {}
      share = effective_cpus()
      if a.cpu_baseline_frac > 0:
        # headline: one worker per usable core (min(cores, units)); side leg: one process per unit on
        # the same share (time-shared), labelled
        w = a.cpu_workers or share[0]
        legs['wgs'] = cpu_baseline_wgs(a, contigs, data, units, p, rlen, model, w, share)
        if len(units) > w:
          side = cpu_baseline_wgs(a, contigs, data, units, p, rlen, model, len(units), share)
          side['note'] = 'one process per work unit, time-sharing the {} usable cores'.format(share[0])
          legs['wgs_process_per_unit'] = side
      if a.cpu_baseline_mbp > 0:
        legs['chr1'] = cpu_baseline(a, seq1, recs1, p, rlen, model, _native.work_units(a.seed, [2], passes))
      if a.cpu_config0:
        legs['configs0'] = cpu_baseline_config0(a, data)
      cpu = legs.pop('wgs', None) or legs.pop('chr1', None)   # the metric's workload when it ran
      if cpu is not None:
        cpu.update(legs)
        cpu['cpu_share'] = share[1]
        ref = dict(REFERENCE_MEASURED)
        if 'configs0' in legs:
          ref['port_over_reference_configs0'] = legs['configs0']['value'] / ref['configs0_shape_threads2_templates_per_s']
        cpu['reference_measured'] = ref
  if dist is not None:
    dist.destroy_process_group()
  if rank != 0:
    return
  ms_per_step = dt / steps * 1e3
  out = {
    'metric': METRIC,
    'value': kept_all / dt,
    'unit': 'templates/s',
    'n_gpus': world,
    'steps': steps,
    'warmup': warmup,
    'ms_per_step': ms_per_step,
    'higher_is_better': True,
    'scaling': 'strong',
    'vs_baseline': None,
    'dtype': 'int64+u8',
    'data': 'synthetic GRCh37-shaped genome (24 contigs + MT) + ~1.3/kbp phased diploid variants (mitty_amd.synth), '
            'seed-fixed',
    'config': {'workload': 'generate-reads 30x WGS: whole GRCh37{} diploid, {} 2x{} PE, {}x, rng={}, one BED '
                           'interval per contig, the 100 work units dealt by LPT over {} GPU(s) (BASELINE configs[3] '
                           'genome)'.format('' if a.genome_scale == 1 else ' (lengths x{})'.format(a.genome_scale),
                                            a.model, rlen, a.coverage, a.rng, world),
               'genome_bp': sum(L for _, L in contigs), 'read_model': a.model, 'coverage': a.coverage,
               'units': n_units, 'batches_rank0': len(batches), 'batch_draws': batch_draws,
               'templates_per_step': kept_all // steps,
               'parallelism': 'unit-shard (LPT) x{}'.format(world) if world > 1 else 'single GPU',
               'world_size_seen': seen, 'collective_backend': backend},
    'roofline': roof,
    'roofline_rank': 0,
    'verify': verify,
    'cpu_baseline': cpu,
    'end_to_end': e2e,
    'stage_ms': stage_ms,
    'span_ms': span_ms,
    'stage_note': STAGE_NOTE,
    'fastq_bytes_per_template': (b1_all + b2_all) / max(kept_all, 1),
    'device_peak_gib': round(peak / 2 ** 30, 1),
    'setup_s': dict(synth_inputs=round(t_synth, 2), **hbm_setup()),
    'host_cpus': os.cpu_count(),
  }
  if a.plan_share:   # not the metric line: one rank's share of an N-rank plan, timed alone
    out['metric'] = 'projection: one rank of an N-GPU run of [' + METRIC + ']'
    out['projection'] = {'plan_rank': plan_rank, 'plan_world': plan_world, 'units': len(mine),
                         'draws': mine_draws}
  print(json.dumps(out), flush=True)


def verify_wgs(a, eng, batches, copies, contigs, data, units, p, rlen, model):
  """One more step of the bench's own plan (same batches, engine and arenas), unit by unit: every unit's two FASTQ
  ranges fetched from the arenas before the next batch recycles them and hashed (sha256), against the CPU oracle's
  digests of the same unit (readgenerate.py:129-159 unit list, seeds and order; the oracle computes them in
  --cpu-workers processes while the GPU runs).  Untimed; fails the run on the first differing unit."""
  import hashlib
  import threading
  from concurrent.futures import ThreadPoolExecutor
  sys.path.insert(0, REPO)
  from oracle import oracle as O
  t0 = time.perf_counter()
  workers = max(1, a.cpu_workers or effective_cpus()[0])
  d = tempfile.mkdtemp(prefix='mh_verify_', dir='/dev/shm' if os.path.isdir('/dev/shm') else None)
  img = os.path.join(d, 'ref.bin')
  offs = {}
  try:
    with open(img, 'wb') as fp:
      for ri in sorted({u[0] for u in units}):
        offs[ri] = (fp.tell(), len(data[ri][0]))
        fp.write(bytes(data[ri][0]))
    # (ref bytes, region start, variants, p, rlen, cum_tlen, seed, stub, chrom, cpy): oracle._unit_digest's job
    jobs = [((img,) + offs[ri], 0, copies[ri][cpy], p, rlen, model['cum_tlen'], s, 'SYN:0:{}'.format(ps),
             contigs[ri][0], cpy) for ps, (ri, cpy, s) in enumerate(units)]
    ref = {}
    th = threading.Thread(target=lambda: ref.update(enumerate(O.digest_jobs(jobs, workers))), daemon=True)
    th.start()
    got = {}
    hpool = ThreadPoolExecutor(8)

    def sha(x):
      return hashlib.sha256(memoryview(x)).hexdigest()

    eng.ctx.sync()
    eng.drop_haplotypes()
    for batch in batches:
      eng.ctx.reset_output()
      res = eng.run_units(batch, lambda r, c: copies[r][c], p, rlen, model['cum_tlen'], 'SYN', 0, True, a.rng)
      eng.ctx.sync()
      o1 = o2 = 0
      for (ps, ri, cpy, _), (n, kept, x1, x2) in zip(batch, res):
        arr1, arr2 = eng.ctx.fetch_output_arrays(o1, x1, o2, x2)
        f1, f2 = hpool.submit(sha, arr1), hpool.submit(sha, arr2)
        got[ps] = (kept, x1, f1, x2, f2)   # (the oracle digest's first field is the kept-template count)
        o1, o2 = o1 + x1, o2 + x2
      for ps in [u[0] for u in batch]:   # hashed before the arenas are reused
        n, x1, f1, x2, f2 = got[ps]
        got[ps] = (n, x1, f1.result(), x2, f2.result())
    hpool.shutdown()
    t_gpu = time.perf_counter() - t0
    th.join()
  finally:
    for f in glob.glob(os.path.join(d, '*')):
      os.remove(f)
    os.rmdir(d)
  bad = [ps for ps in range(len(units)) if got.get(ps) != ref.get(ps)]
  out = {'units': len(units), 'units_equal': len(units) - len(bad), 'templates_kept': sum(v[0] for v in got.values()),
         'fastq_bytes': sum(v[1] + v[3] for v in got.values()), 'oracle_workers': workers,
         'gpu_fetch_hash_s': round(t_gpu, 1), 'seconds': round(time.perf_counter() - t0, 1),
         'method': 'per unit: sha256 of both FASTQ ranges of the arenas (D2H after the unit\'s batch) vs the CPU '
                   'oracle\'s sha256 of the same unit (oracle.digest_jobs)'}
  if bad:
    out['first_bad'] = {'ps': bad[0], 'gpu': list(got.get(bad[0], ())), 'oracle': list(ref.get(bad[0], ()))}
    print(json.dumps({'verify': out}), file=sys.stderr, flush=True)
    sys.exit('bench.py --verify: {} of {} units differ from the oracle'.format(len(bad), len(units)))
  return out


def _cpu_unit(args):
  """One work unit through the CPU oracle in a worker process; returns (templates, start, end) wall-clock stamps.
  The unit's reference bytes come from a file (a /dev/shm image the parent wrote before timing) when `ref` is
  (path, offset, length)."""
  ref, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy = args
  sys.path.insert(0, REPO)
  from oracle import oracle as O
  if isinstance(ref, tuple):
    path, off, n = ref
    with open(path, 'rb') as fp:
      fp.seek(off)
      ref = fp.read(n)
  t0 = time.time()
  n = O.generate_unit_soa(ref, 0, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy, keep_output=False)[0]
  return n, t0, time.time()


def _cpu_warm(_):
  sys.path.insert(0, REPO)
  from oracle import oracle as O
  O.lib()
  return os.getpid()


def _cpu_pool_run(jobs, workers):
  """The jobs through `workers` spawned oracle processes (warmed first: imports and the oracle library loaded before
  timing), longest first; returns (templates, seconds from the first unit's start to the last unit's end, per-core
  rate)."""
  import multiprocessing as mp
  pool = mp.get_context('spawn').Pool(workers)
  try:
    pool.map(_cpu_warm, range(workers), chunksize=1)
    res = pool.map(_cpu_unit, jobs, chunksize=1)
  except BaseException:
    pool.terminate()
    raise
  pool.close()
  pool.join()
  n = sum(r[0] for r in res)
  dt = max(r[2] for r in res) - min(r[1] for r in res)
  busy = sum(r[2] - r[1] for r in res)
  return n, dt, n / busy if busy > 0 else None


def effective_cpus():
  """The CPUs this process may actually use: the affinity mask, capped by the cgroup's CPU quota (cgroup v2
  cpu.max, or v1 cpu.cfs_quota_us / cpu.cfs_period_us); without a quota, OMP_NUM_THREADS when the launcher sets it
  (the GPU pool's per-job share).  Returns (cores, how) — `how` names what was read."""
  aff = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
  quota, src = None, None
  try:
    with open('/sys/fs/cgroup/cpu.max') as fp:
      q, per = fp.read().split()[:2]
    if q != 'max':
      quota, src = float(q) / float(per), 'cgroup v2 cpu.max {} {}'.format(q, per)
  except (OSError, ValueError):
    try:
      with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as fp:
        q = int(fp.read())
      with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as fp:
        per = int(fp.read())
      if q > 0:
        quota, src = q / per, 'cgroup v1 cfs quota {} / period {}'.format(q, per)
    except (OSError, ValueError):
      pass
  parts = ['sched_getaffinity: {} CPUs'.format(aff), src or 'no cgroup CPU quota']
  cores = aff
  if quota is not None:
    cores = max(1, min(aff, int(quota)))
  else:
    omp = os.environ.get('OMP_NUM_THREADS', '')
    if omp.isdigit() and 0 < int(omp) < aff:
      cores = int(omp)
      parts.append('OMP_NUM_THREADS={} (the launcher\'s per-job CPU share)'.format(omp))
  return cores, '; '.join(parts) + ' -> {} cores'.format(cores)


# The reference's own rates, measured in the survey container (8-vCPU Xeon, the reference with a
# pysam shim, synthetic 2 Mbp genome): the port's configs[0] leg is quoted against the first
REFERENCE_MEASURED = {
  'configs0_shape_threads2_templates_per_s': 60.0e3,   # 1kg-pcr-free 2x250, --threads 2 (119,868 templates, 2.03 s)
  'one_worker_templates_per_s': 43.7e3,                # hiseq-X-v2.5-Garvan 2x150, 1 worker (200,133 templates, 4.58 s)
  'hardware': '8-vCPU Intel Xeon (survey container), the reference itself under a test-side pysam shim',
  'source': 'SURVEY.md section 6'}


def cpu_baseline_wgs(a, contigs, data, units, p, rlen, model, n_workers, share=None):
  """The metric's workload on the CPU: the CPU oracle (oracle/mitty_oracle.c, a scalar port of the reference path)
  laid out like the reference's multiprocessing path (`readgenerate.process_multi_threaded`: worker processes pulling
  work units, readgenerate.py:76-126) over all 100 work units of the 30x WGS job, in --cpu-workers processes.  Bounded
  sample: each unit runs on the first --cpu-baseline-frac of its region (same variants, same seeds), so the sample
  has the full job's unit list and topology.  Rate = templates / (last unit's end - first unit's start)."""
  frac = a.cpu_baseline_frac
  workers = max(1, min(n_workers, len(units)))
  d = tempfile.mkdtemp(prefix='mh_cpu_', dir='/dev/shm' if os.path.isdir('/dev/shm') else None)
  img = os.path.join(d, 'ref.bin')
  try:
    offs, sub = {}, {}
    with open(img, 'wb') as fp:   # the regions' prefixes, written once before timing (workers read their own)
      for ri in sorted({u[0] for u in units}):
        seq, recs, _ = data[ri]
        L = max(1, int(len(seq) * frac))
        offs[ri] = (fp.tell(), L)
        fp.write(bytes(seq[:L]))
        sub[ri] = synth_copies(recs, L)
    jobs = [((img,) + offs[ri], sub[ri][cpy], p, rlen, model['cum_tlen'], s, 'SYN:0:{}'.format(ps), contigs[ri][0],
             cpy) for ps, (ri, cpy, s) in enumerate(units)]
    order = sorted(range(len(jobs)), key=lambda k: -offs[units[k][0]][1])   # longest first, as the GPU deal
    n, dt, per_core = _cpu_pool_run([jobs[k] for k in order], workers)
  finally:
    for f in glob.glob(os.path.join(d, '*')):
      os.remove(f)
    os.rmdir(d)
  cores, how = share if share else (workers, 'workers')
  return {'value': n / dt, 'unit': 'templates/s', 'cores': min(cores, workers), 'processes': workers, 'kind': 'port',
          'per_core': per_core, 'host_cpus': os.cpu_count(), 'workload': 'wgs',
          'sample': 'the 30x WGS job\'s {} work units (25 regions x 2 copies x 2 passes, the reference\'s unit order '
                    'and seeds), each on the first {:.0%} of its region, in {} oracle worker processes on this '
                    'process\'s CPU share ({}): {} templates in {:.2f} s'.format(len(jobs), frac, workers, how, n, dt)}


def synth_copies(recs, L):
  from mitty_amd import synth
  return synth.copies_soa(recs, 0, L)


def cpu_baseline(a, seq, recs, p, rlen, model, units):
  """chr1 leg (BASELINE configs[1]'s job): the oracle laid out like the reference's multiprocessing path, the job's
  4 work units side by side in 4 worker processes on the first `cpu_baseline_mbp` Mbp of the chr1 contig."""
  L = int(a.cpu_baseline_mbp * 1e6)
  sub = synth_copies(recs, L)
  ref = bytes(seq[:L])
  jobs = [(ref, sub[cpy], p, rlen, model['cum_tlen'], s, 'SYN:0:{}'.format(k), '1', cpy)
          for k, (ri, cpy, s) in enumerate(units)]
  n, dt, per_core = _cpu_pool_run(jobs, len(jobs))
  return {'value': n / dt, 'unit': 'templates/s', 'cores': len(jobs), 'kind': 'port',
          'per_core': per_core, 'host_cpus': os.cpu_count(), 'workload': 'chr1',
          'sample': '{} work units (2 copies x {} passes, one worker process each, {} host CPUs) on chr1[0:{:.0f} Mbp), '
                    '{} templates in {:.2f} s'.format(len(jobs), len(jobs) // 2, os.cpu_count(), a.cpu_baseline_mbp,
                                                     n, dt)}


HG001_BED = [('1', 20000, 1020000), ('10', 60000, 1060000)]   # reference examples/reads/hg001.bed


def _cpu_unit_region(args):
  """One configs[0] work unit through the CPU oracle (a worker of the 2-process pool)."""
  ref, s0, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy = args
  sys.path.insert(0, REPO)
  from oracle import oracle as O
  return O.generate_unit_soa(ref, s0, soa, p, rlen, cum_tlen, seed, stub, chrom, cpy, keep_output=False)[0]


def cpu_baseline_config0(a, data):
  """BASELINE configs[0] as stated: `mitty generate-reads` on hg001.bed (2 regions x 1 Mbp) with the 1kg-pcr-free
  model (2x250), 30x, seed 7, --threads 2 — here the CPU oracle in 2 worker processes that take the 8 work units in
  the reference's unit order (readgenerate.py:102-115), on the synthetic contigs 1 and 10."""
  import multiprocessing as mp
  from mitty_amd import _native, synth
  from mitty_amd.readmodel import get_read_model
  _, model = get_read_model('1kg-pcr-free.pkl')
  rlen = int(model['mean_rlen'])
  p, passes = _native.read_model_params(rlen, a.coverage)
  idx = {name: ri for ri, (name, _) in enumerate(synth.GRCH37)}
  units = _native.work_units(a.seed, [2] * len(HG001_BED), passes)
  jobs = []
  for ps, (ri, cpy, seed) in enumerate(units):
    chrom, s0, e = HG001_BED[ri]
    seq, recs, _ = data[idx[chrom]]
    soa = synth.copies_soa(recs, s0, e)[cpy]
    jobs.append((seq[s0:e], s0, soa, p, rlen, model['cum_tlen'], seed, 'SYN:{}:{}'.format(ps % 2, ps // 2), chrom,
                 cpy))
  pool = mp.get_context('spawn').Pool(2)
  try:
    pool.map(_cpu_unit_region, jobs[:2])   # workers warm (imports) before timing
    t0 = time.perf_counter()
    n = sum(pool.map(_cpu_unit_region, jobs, chunksize=1))
    dt = time.perf_counter() - t0
  except BaseException:
    pool.terminate()
    raise
  pool.close()
  pool.join()
  return {'value': n / dt, 'unit': 'templates/s', 'cores': 2, 'kind': 'port',
          'sample': 'BASELINE configs[0]: hg001.bed (1:20000-1020000, 10:60000-1060000) on the synthetic contigs, '
                    '1kg-pcr-free 2x{}, {}x, seed {}, 2 worker processes over the {} work units: {} templates in '
                    '{:.2f} s'.format(rlen, a.coverage, a.seed, len(jobs), n, dt)}


if __name__ == '__main__':
  main()
