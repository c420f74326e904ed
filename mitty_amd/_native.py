"""ctypes binding of libmitty_hip.so (include/mitty_hip.h).

There is no CPU fallback: if the library is missing or no HIP device is present, the product path raises.
"""
import ctypes
import os
import sys

import numpy as np

LIB_PATH = (os.environ.get('MH_LIB') or   # MH_LIB: another build of the library (A/B experiments)
            os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib', 'libmitty_hip.so'))

MH_OK, MH_E_ARG, MH_E_HIP, MH_E_OOM, MH_E_CAPACITY, MH_E_COMPLEX_VARIANT, MH_E_SEED, MH_E_STATE, MH_E_NO_DEVICE = \
  0, -1, -2, -3, -4, -5, -6, -7, -8
MH_RNG_MITTY, MH_RNG_PHILOX = 0, 1

# Every exported symbol of include/mitty_hip.h (tests check the library exports all of them).
EXPORTS = ['mh_version', 'mh_device_count', 'mh_create', 'mh_destroy', 'mh_last_error', 'mh_sync',
           'mh_selftest_scan_fault', 'mh_selftest_sort',
           'mh_read_model_params', 'mh_work_units', 'mh_upload_contig', 'mh_build_haplotype', 'mh_upload_variants', 'mh_build_haplotype_vset', 'mh_build_haplotypes_vset', 'mh_prefetch_haplotypes_vset', 'mh_release_variants', 'mh_get_nodes',
           'mh_release_haplotype', 'mh_expand_variant', 'mh_sample_templates', 'mh_sample_templates_span', 'mh_set_templates',
           'mh_get_templates', 'mh_templates_export', 'mh_templates_import', 'mh_emit_reads', 'mh_emit_prepare', 'mh_emit_reads_async', 'mh_emit_collect', 'mh_output_size', 'mh_output_fetch', 'mh_output_reset', 'mh_host_alloc', 'mh_host_free', 'mh_device_cache_trim', 'mh_device_live_bytes',
           'mh_read_batch', 'mh_set_corruption', 'mh_set_corruption_stream', 'mh_get_corruption_stream', 'mh_stage_times', 'mh_enable_timing', 'mh_sample_units', 'mh_sample_units_async', 'mh_templates_count',
           'mh_use_templates', 'mh_release_templates', 'mh_mt_window_at', 'mh_fixup_count', 'mh_set_emit_mode', 'mh_set_decode_mode',
           'mh_emit_reads_range', 'mh_emit_measure', 'mh_count_kept', 'mh_bam_set_refs', 'mh_bam_add_fastq', 'mh_bam_add_output',
           'mh_bam_records', 'mh_bam_set_capacity', 'mh_bam_set_spill_dir', 'mh_bam_spilled', 'mh_bam_export', 'mh_bam_import', 'mh_bam_sort', 'mh_bam_write', 'mh_bam_write_gpu', 'mh_bam_reset', 'mh_bam_partition', 'mh_bam_partition_fetch', 'mh_bam_import_tie', 'mh_bam_sorted_head', 'mh_bam_write_part', 'mh_bam_bai_runs', 'mh_corrupt_fastq', 'mh_bgzf_compress', 'mh_bgzf_eof', 'mh_bgzf_compress_device', 'mh_bgzf_compress_gpu', 'mh_output_bgzf',
           'mh_output_bgzf_range', 'mh_output_bgzf_pair', 'mh_output_bgzf_wait', 'mh_output_fetch_async',
           'mh_output_fetch_wait',
           'mh_vcf_open', 'mh_vcf_error', 'mh_vcf_close', 'mh_vcf_region', 'mh_vcf_copy', 'mh_vcf_filter',
           'mh_fasta_open', 'mh_fasta_error', 'mh_fasta_count', 'mh_fasta_contig', 'mh_fasta_copy', 'mh_fasta_close']


class NativeError(RuntimeError):
  pass


class NativeUnavailable(NativeError):
  pass


_lib = None

c_i32, c_i64, c_u64, c_dbl, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p
P_i64 = ctypes.POINTER(c_i64)


def _sig(L, name, args, res=c_i32):
  f = getattr(L, name)
  f.argtypes = args
  f.restype = res


def lib():
  """Load the library (raises NativeUnavailable when it has not been built)."""
  global _lib
  if _lib is not None:
    return _lib
  if not os.path.exists(LIB_PATH):
    raise NativeUnavailable('libmitty_hip.so not built ({}); run __graft_entry__.build() or make -C '
                            'mitty_amd/csrc'.format(LIB_PATH))
  if 'torch' not in sys.modules and int(os.environ.get('WORLD_SIZE', '1')) > 1:
    # a torch.distributed run: torch's HIP runtime must be the process's only one, so torch loads first (our
    # libamdhip64.so.7 dependency then binds to torch's copy; loaded the other way round, torch would bring a second
    # runtime, and whichever initialises second sees no GPU)
    import torch  # noqa: F401
  L = ctypes.CDLL(LIB_PATH)
  _sig(L, 'mh_version', [])
  _sig(L, 'mh_device_count', [ctypes.POINTER(c_i32)])
  _sig(L, 'mh_create', [c_i32, ctypes.POINTER(c_vp)])
  _sig(L, 'mh_destroy', [c_vp])
  _sig(L, 'mh_last_error', [c_vp], ctypes.c_char_p)
  _sig(L, 'mh_sync', [c_vp])
  _sig(L, 'mh_selftest_scan_fault', [c_vp])
  _sig(L, 'mh_selftest_sort', [c_vp, c_vp, c_i64, c_i32, c_vp, c_vp])
  _sig(L, 'mh_read_model_params', [c_i64, c_dbl, ctypes.POINTER(c_dbl), P_i64])
  _sig(L, 'mh_work_units', [c_u64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, P_i64])
  _sig(L, 'mh_upload_contig', [c_vp, c_i32, c_vp, c_i64])
  _sig(L, 'mh_upload_variants', [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64])
  _sig(L, 'mh_build_haplotype_vset', [c_vp, c_i32, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp])
  _sig(L, 'mh_release_variants', [c_vp, c_i32])
  _sig(L, 'mh_build_haplotype', [c_vp, c_i32, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                 P_i64, P_i64, P_i64])
  _sig(L, 'mh_get_nodes', [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, P_i64])
  _sig(L, 'mh_release_haplotype', [c_vp, c_i32])
  _sig(L, 'mh_bgzf_compress_device', [c_vp, c_vp, c_i64, c_vp, c_i64, P_i64])
  _sig(L, 'mh_bgzf_compress_gpu', [c_vp, c_vp, c_i64, c_vp, c_i64, P_i64])
  _sig(L, 'mh_output_bgzf', [c_vp, c_i32, c_vp, c_i64, P_i64])
  _sig(L, 'mh_output_bgzf_range', [c_vp, c_i32, c_i64, c_i64, c_vp, c_i64, P_i64])
  _sig(L, 'mh_output_bgzf_pair', [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, P_i64, P_i64,
                                  ctypes.POINTER(c_i32)])
  _sig(L, 'mh_output_bgzf_wait', [c_vp, c_i32])
  _sig(L, 'mh_output_fetch_async', [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, ctypes.POINTER(c_i32)])
  _sig(L, 'mh_output_fetch_wait', [c_vp, c_i32])
  _sig(L, 'mh_expand_variant', [c_i64, c_i64, c_i64, c_i64, c_i32, c_i64, P_i64, ctypes.POINTER(c_i32), P_i64, P_i64])
  _sig(L, 'mh_sample_templates', [c_vp, c_i32, c_dbl, c_i32, c_vp, c_i32, c_u64, c_i32, P_i64])
  _sig(L, 'mh_sample_templates_span', [c_vp, c_i64, c_i64, c_dbl, c_i32, c_vp, c_i32, c_u64, c_i32, P_i64])
  _sig(L, 'mh_set_templates', [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32])
  _sig(L, 'mh_get_templates', [c_vp, c_vp, c_vp, c_vp, c_i64, P_i64])
  _sig(L, 'mh_emit_reads', [c_vp, c_i32, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i32, c_u64, P_i64, P_i64, P_i64])
  _sig(L, 'mh_emit_prepare', [c_vp, c_i32, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i32, c_u64, P_i64, P_i64, P_i64])
  _sig(L, 'mh_emit_reads_async', [c_vp, c_i32, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i32, c_u64])
  _sig(L, 'mh_emit_collect', [c_vp, c_vp, c_i64, P_i64])
  _sig(L, 'mh_build_haplotypes_vset', [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp])
  _sig(L, 'mh_prefetch_haplotypes_vset', [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp, c_dbl])
  _sig(L, 'mh_emit_reads_range', [c_vp, c_i32, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i32, c_u64, c_i64, c_i64,
                                   c_i64, P_i64, P_i64, P_i64])
  _sig(L, 'mh_count_kept', [c_vp, c_i32, c_i64, c_i64, P_i64])
  _sig(L, 'mh_emit_measure', [c_vp, c_i32, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i32, c_u64, c_i64, c_i64, c_i64,
                              P_i64, P_i64, P_i64])
  _sig(L, 'mh_bam_set_refs', [c_vp, c_i32, ctypes.c_char_p, c_vp])
  _sig(L, 'mh_bam_add_fastq', [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, P_i64, P_i64, P_i64])
  _sig(L, 'mh_bam_add_output', [c_vp, c_i64, P_i64])
  _sig(L, 'mh_bam_records', [c_vp, P_i64, P_i64])
  _sig(L, 'mh_bam_set_capacity', [c_vp, c_i64])
  _sig(L, 'mh_bam_spilled', [c_vp, P_i64, P_i64])
  _sig(L, 'mh_bam_export', [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp])
  _sig(L, 'mh_bam_import', [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64])
  _sig(L, 'mh_bam_partition', [c_vp, c_vp, c_i32, ctypes.c_uint64, c_vp, c_vp, c_vp])
  _sig(L, 'mh_bam_set_spill_dir', [c_vp, ctypes.c_char_p])
  _sig(L, 'mh_bam_partition_fetch', [c_vp, c_vp, c_i64])
  _sig(L, 'mh_bam_import_tie', [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64])
  _sig(L, 'mh_bam_sorted_head', [c_vp, c_i64, c_vp])
  _sig(L, 'mh_bam_write_part', [c_vp, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i64, c_vp, c_i64, c_i32, P_i64,
                                P_i64, P_i64, c_vp, c_i64])
  _sig(L, 'mh_bam_bai_runs', [c_vp, P_i64, c_vp, c_i64, P_i64, c_vp, c_i64, c_vp])
  _sig(L, 'mh_bam_write', [c_vp, ctypes.c_char_p, ctypes.c_char_p, c_i64, c_i32, c_i32, ctypes.c_char_p, P_i64,
                           P_i64])
  _sig(L, 'mh_bam_write_gpu', [c_vp, ctypes.c_char_p, ctypes.c_char_p, c_i64, ctypes.c_char_p, P_i64, P_i64, P_i64])
  _sig(L, 'mh_bam_reset', [c_vp])
  _sig(L, 'mh_bam_sort', [c_vp])
  _sig(L, 'mh_corrupt_fastq', [c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, P_i64, P_i64, P_i64])
  _sig(L, 'mh_bgzf_compress', [c_vp, c_i64, c_i32, c_i32, c_vp, c_i64, P_i64])
  _sig(L, 'mh_bgzf_eof', [c_vp])
  _sig(L, 'mh_vcf_open', [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(c_vp)])
  _sig(L, 'mh_vcf_error', [c_vp], ctypes.c_char_p)
  _sig(L, 'mh_vcf_close', [c_vp])
  _sig(L, 'mh_vcf_region', [c_vp, ctypes.c_char_p, c_i64, c_i64, ctypes.POINTER(c_i32), c_vp, c_vp, c_i32])
  _sig(L, 'mh_vcf_copy', [c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp])
  _sig(L, 'mh_vcf_filter', [ctypes.c_char_p, ctypes.c_char_p, c_i32, c_vp, c_vp, c_vp, ctypes.c_char_p, c_i32, c_i32,
                            P_i64, P_i64, ctypes.c_char_p, c_i32])
  _sig(L, 'mh_fasta_open', [ctypes.c_char_p, c_vp, ctypes.POINTER(c_vp)])
  _sig(L, 'mh_fasta_error', [c_vp], ctypes.c_char_p)
  _sig(L, 'mh_fasta_count', [c_vp, ctypes.POINTER(c_i32)])
  _sig(L, 'mh_fasta_contig', [c_vp, c_i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_vp), P_i64])
  _sig(L, 'mh_fasta_copy', [c_vp, c_i32, c_vp])
  _sig(L, 'mh_fasta_close', [c_vp])
  _sig(L, 'mh_output_size', [c_vp, P_i64, P_i64])
  _sig(L, 'mh_output_fetch', [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64])
  _sig(L, 'mh_output_reset', [c_vp])
  _sig(L, 'mh_host_alloc', [c_i64, ctypes.POINTER(c_vp)])
  _sig(L, 'mh_host_free', [c_vp])
  _sig(L, 'mh_device_cache_trim', [ctypes.POINTER(c_i64)])
  _sig(L, 'mh_device_live_bytes', [ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_i32])
  _sig(L, 'mh_read_batch', [c_vp, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp,
                            c_vp, c_i64, c_vp, P_i64, c_vp, c_i64, c_vp, P_i64, c_vp, c_i64, c_vp, P_i64])
  _sig(L, 'mh_set_corruption', [c_vp, c_i32, c_vp, c_i32, c_i32, c_vp, c_u64])
  _sig(L, 'mh_templates_export', [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, P_i64])
  _sig(L, 'mh_templates_import', [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, c_i32])
  _sig(L, 'mh_set_corruption_stream', [c_vp, c_i32, c_u64, c_vp, c_i32])
  _sig(L, 'mh_get_corruption_stream', [c_vp, c_vp, ctypes.POINTER(c_i32), P_i64])
  _sig(L, 'mh_stage_times', [c_vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_dbl), c_i32,
                             ctypes.POINTER(c_i32)])
  _sig(L, 'mh_enable_timing', [c_vp, c_i32])
  _sig(L, 'mh_sample_units', [c_vp, c_i32, c_vp, c_vp, c_vp, c_dbl, c_i32, c_vp, c_i32, c_i32, c_vp])
  _sig(L, 'mh_sample_units_async', [c_vp, c_i32, c_vp, c_vp, c_vp, c_dbl, c_i32, c_vp, c_i32, c_i32])
  _sig(L, 'mh_templates_count', [c_vp, c_i32, c_vp])
  _sig(L, 'mh_use_templates', [c_vp, c_i32])
  _sig(L, 'mh_release_templates', [c_vp, c_i32])
  _sig(L, 'mh_mt_window_at', [ctypes.c_uint32, c_u64, c_vp])
  _sig(L, 'mh_fixup_count', [c_vp, P_i64])
  _sig(L, 'mh_set_emit_mode', [c_vp, c_i32])
  _sig(L, 'mh_set_decode_mode', [c_vp, c_i32])
  _lib = L
  return L


def mt_window_at(seed, offset):
  """Host jump-ahead: untempered MT19937 window (x_J .. x_{J+623}) of the stream seeded with `seed`."""
  out = np.empty(624, np.uint32)
  rc = lib().mh_mt_window_at(int(seed), int(offset), _ptr(out))
  if rc:
    _raise(rc, 'mh_mt_window_at failed')
  return out


def bgzf_compress(data, level=6, threads=8):
  """BGZF members for `data` (host-side deflate pool; no device needed).  Append bgzf_eof() at the end of a file."""
  n = len(data)
  src = np.frombuffer(data, np.uint8) if n else np.zeros(1, np.uint8)
  cap = n + (n // 0xff00 + 1) * 64 + 64
  out = np.empty(cap, np.uint8)
  used = c_i64()
  rc = lib().mh_bgzf_compress(_ptr(src), n, int(level), int(threads), _ptr(out), cap, ctypes.byref(used))
  if rc == MH_E_CAPACITY:
    out = np.empty(used.value, np.uint8)
    rc = lib().mh_bgzf_compress(_ptr(src), n, int(level), int(threads), _ptr(out), used.value, ctypes.byref(used))
  if rc:
    _raise(rc, 'mh_bgzf_compress failed')
  return out[:used.value].tobytes()


class VcfFile:
  """Host VCF reader (mh_vcf.cpp) for one sample: region(chrom, start0, end) -> (ploidy, [SoA per copy])."""

  def __init__(self, path, sample):
    L = lib()
    self._L = L
    self._h = c_vp()
    rc = L.mh_vcf_open(path.encode(), sample.encode(), ctypes.byref(self._h))
    if rc:
      msg = L.mh_vcf_error(self._h).decode() if self._h else 'mh_vcf_open failed'
      self.close()
      _raise(rc, msg)

  def close(self):
    if getattr(self, '_h', None):
      self._L.mh_vcf_close(self._h)
      self._h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  def region(self, chrom, start0, end):
    pl = c_i32()
    nv = np.zeros(64, np.int64)
    ab = np.zeros(64, np.int64)
    rc = self._L.mh_vcf_region(self._h, chrom.encode(), int(start0), int(end), ctypes.byref(pl), _ptr(nv), _ptr(ab),
                               64)
    if rc:
      _raise(rc, self._L.mh_vcf_error(self._h).decode())
    copies = []
    for c in range(pl.value):
      n, nb = int(nv[c]), int(ab[c])
      pos, oplen, aoff, alen = (np.empty(n, np.int64) for _ in range(4))
      op = np.empty(n, np.uint8)
      pool = np.empty(max(nb, 1), np.uint8)
      rc = self._L.mh_vcf_copy(self._h, c, _ptr(pos), _ptr(op), _ptr(oplen), _ptr(aoff), _ptr(alen), _ptr(pool))
      if rc:
        _raise(rc, self._L.mh_vcf_error(self._h).decode())
      copies.append({'pos': pos, 'op': op, 'oplen': oplen, 'alt_off': aoff, 'alt_len': alen,
                     'alt_pool': pool[:nb].tobytes()})
    return pl.value, copies


def vcf_filter(path_in, sample, regions, path_out, bgzf=False, threads=8):
  """filter-variants (mh_vcf_filter): regions [(chrom, start0, end)] in BED order.  Returns (written, filtered)."""
  L = lib()
  chroms = b''.join(c.encode() + b'\0' for c, _, _ in regions) or b'\0'
  s0 = np.array([r[1] for r in regions] or [0], np.int64)
  e = np.array([r[2] for r in regions] or [0], np.int64)
  cbuf = ctypes.create_string_buffer(chroms, len(chroms))
  w, f = c_i64(), c_i64()
  err = ctypes.create_string_buffer(1024)
  rc = L.mh_vcf_filter(path_in.encode(), sample.encode(), len(regions), ctypes.cast(cbuf, c_vp), _ptr(s0), _ptr(e),
                       path_out.encode(), 1 if bgzf else 0, int(threads), ctypes.byref(w), ctypes.byref(f), err, 1024)
  if rc:
    _raise(rc, err.value.decode())
  return w.value, f.value


class PinnedBuffer:
  """Page-locked host staging (mh_host_alloc), grown on demand."""

  def __init__(self):
    self.ptr, self.cap = None, 0

  def reserve(self, n):
    if n > self.cap:
      # page-locking costs ~0.1 s per GB: grow with headroom, so arenas of similar sizes reuse one allocation
      n = (int(n * 1.25) + (64 << 20) - 1) // (64 << 20) * (64 << 20)
      self.free()
      p = c_vp()
      rc = lib().mh_host_alloc(int(n), ctypes.byref(p))
      if rc:
        _raise(rc, 'mh_host_alloc failed')
      self.ptr, self.cap = p.value, int(n)

  def view(self, n):
    if n == 0:
      return memoryview(b'')
    return memoryview((ctypes.c_uint8 * n).from_address(self.ptr)).cast('B')

  def free(self):
    if self.ptr:
      lib().mh_host_free(c_vp(self.ptr))
    self.ptr, self.cap = None, 0

  def __del__(self):
    try:
      self.free()
    except Exception:
      pass


# an uninitialised bytes object of n bytes and its buffer (CPython's PyBytes_FromStringAndSize(NULL, n): filled once,
# before anything else sees it, as a C extension would)
_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_bytes_ptr = ctypes.pythonapi.PyBytes_AsString
_bytes_ptr.restype = ctypes.c_void_p
_bytes_ptr.argtypes = [ctypes.py_object]


def read_fasta(path, names=None):
  """Host FASTA reader (mh_fasta.cpp): {contig name: bytes}, only `names` when given."""
  L = lib()
  h = c_vp()
  sel = None
  if names is not None:
    sel = ctypes.create_string_buffer(b''.join(n.encode() + b'\0' for n in names) + b'\0')
  rc = L.mh_fasta_open(path.encode(), ctypes.cast(sel, c_vp) if sel is not None else None, ctypes.byref(h))
  try:
    if rc:
      _raise(rc, L.mh_fasta_error(h).decode() if h else 'mh_fasta_open failed')
    n = c_i32()
    L.mh_fasta_count(h, ctypes.byref(n))
    out = {}
    for i in range(n.value):
      nm, ln = ctypes.c_char_p(), c_i64()
      L.mh_fasta_contig(h, i, ctypes.byref(nm), None, ctypes.byref(ln))
      # the bytes object's own buffer filled by the library's threads (one pass over the file, no second copy)
      b = _new_bytes(None, ln.value) if ln.value else b''
      if ln.value:
        L.mh_fasta_copy(h, i, _bytes_ptr(b))
      out[nm.value.decode()] = b
    return out
  finally:
    if h:
      L.mh_fasta_close(h)


def device_cache_trim():
  """Free the device blocks the library keeps for reuse (mh_device_cache_trim); returns their bytes."""
  f = c_i64()
  lib().mh_device_cache_trim(ctypes.byref(f))
  return f.value


def device_live_bytes(reset_peak=False):
  """(live, peak) bytes of the library's device blocks in use (mh_device_live_bytes); reset_peak restarts the peak
  from the live value after reading it."""
  a, b = c_i64(), c_i64()
  lib().mh_device_live_bytes(ctypes.byref(a), ctypes.byref(b), 1 if reset_peak else 0)
  return a.value, b.value


def bgzf_eof():
  out = np.empty(28, np.uint8)
  lib().mh_bgzf_eof(_ptr(out))
  return out.tobytes()


def device_count():
  n = c_i32(0)
  lib().mh_device_count(ctypes.byref(n))
  return n.value


def bam_piece_layout(n, nbytes):
  """Byte offsets of a packed BAM store piece (n records, nbytes of records): records at 0, then (8-aligned) the
  n + 1 record offsets, the n sort keys and the n BAI infos (4 x int32); returns (o_roff, o_key, o_info, total)."""
  o_roff = (int(nbytes) + 7) & ~7
  o_key = o_roff + 8 * (n + 1)
  o_info = o_key + 8 * n
  return o_roff, o_key, o_info, o_info + 16 * n


def bam_part_layout(n, nbytes):
  """Byte offsets of one destination's segment of mh_bam_partition (n records, nbytes of records): the packed piece
  of bam_piece_layout, then n ties (uint64); returns (o_roff, o_key, o_info, o_tie, total)."""
  o_roff, o_key, o_info, o_tie = bam_piece_layout(n, nbytes)
  return o_roff, o_key, o_info, o_tie, o_tie + 8 * n


def _ptr(a):
  return a.ctypes.data_as(c_vp) if a is not None else None


def _raise(rc, msg):
  if rc in (MH_E_ARG, MH_E_COMPLEX_VARIANT, MH_E_SEED):
    raise ValueError(msg)
  if rc == MH_E_OOM:
    raise MemoryError(msg)
  if rc == MH_E_NO_DEVICE:
    raise NativeUnavailable('no HIP device visible: ' + msg)
  raise NativeError('libmitty_hip error {}: {}'.format(rc, msg))


def read_model_params(mean_rlen, coverage):
  p, passes = c_dbl(), c_i64()
  rc = lib().mh_read_model_params(int(mean_rlen), float(coverage), ctypes.byref(p), ctypes.byref(passes))
  if rc:
    _raise(rc, 'bad read model parameters')
  return p.value, passes.value


def work_units(seed, ploidy, passes):
  ploidy = np.ascontiguousarray(ploidy, dtype=np.int32)
  n = int(ploidy.sum()) * int(passes)
  r, c, s = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.uint32)
  nn = c_i64()
  rc = lib().mh_work_units(int(seed), _ptr(ploidy), len(ploidy), int(passes), _ptr(r), _ptr(c), _ptr(s),
                           ctypes.byref(nn))
  if rc:
    _raise(rc, 'Seed must be between 0 and 2**32 - 1')
  return [(int(a), int(b), int(x)) for a, b, x in zip(r[:n], c[:n], s[:n])]


class Context:
  """One device context (one GPU, one stream).  Wraps mh_ctx."""

  def __init__(self, device=0):
    L = lib()
    h = c_vp()
    rc = L.mh_create(int(device), ctypes.byref(h))
    if rc:
      _raise(rc, 'mh_create(device={}) failed'.format(device))
    self._h = h
    self._L = L
    self.device = device

  def close(self):
    if self._h:
      self._L.mh_destroy(self._h)
      self._h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  def _chk(self, rc):
    if rc:
      _raise(rc, self._L.mh_last_error(self._h).decode(errors='replace'))

  # ---- contigs / haplotypes ----------------------------------------------------------------------------
  def upload_contig(self, contig_id, seq):
    buf = np.frombuffer(seq, dtype=np.uint8) if len(seq) else np.zeros(1, np.uint8)
    self._chk(self._L.mh_upload_contig(self._h, contig_id, _ptr(buf), len(seq)))

  def build_haplotype(self, slot, contig_id, ref_start_pos, vsoa):
    """vsoa: dict with pos i64, op u8, oplen i64, alt_off i64, alt_len i64, alt_pool bytes."""
    n = len(vsoa['pos'])
    pool = vsoa['alt_pool']
    pool_arr = np.frombuffer(pool, dtype=np.uint8) if len(pool) else np.zeros(1, np.uint8)
    nn, pmin, pmax = c_i64(), c_i64(), c_i64()
    arrs = [np.ascontiguousarray(vsoa[k], dtype=dt) for k, dt in
            (('pos', np.int64), ('op', np.uint8), ('oplen', np.int64), ('alt_off', np.int64), ('alt_len', np.int64))]
    self._chk(self._L.mh_build_haplotype(self._h, slot, contig_id, int(ref_start_pos), *[_ptr(a) for a in arrs],
                                         _ptr(pool_arr), len(pool), n, ctypes.byref(nn), ctypes.byref(pmin),
                                         ctypes.byref(pmax)))
    return nn.value, pmin.value, pmax.value

  def upload_variants(self, vset, vsoa):
    """Keep one copy's variants resident on the device (same layout and checks as build_haplotype)."""
    n = len(vsoa['pos'])
    pool = vsoa['alt_pool']
    pool_arr = np.frombuffer(pool, dtype=np.uint8) if len(pool) else np.zeros(1, np.uint8)
    arrs = [np.ascontiguousarray(vsoa[k], dtype=dt) for k, dt in
            (('pos', np.int64), ('op', np.uint8), ('oplen', np.int64), ('alt_off', np.int64), ('alt_len', np.int64))]
    self._chk(self._L.mh_upload_variants(self._h, int(vset), *[_ptr(a) for a in arrs], _ptr(pool_arr), len(pool), n))

  def build_haplotype_vset(self, slot, contig_id, ref_start_pos, vset):
    nn, pmin, pmax = c_i64(), c_i64(), c_i64()
    self._chk(self._L.mh_build_haplotype_vset(self._h, slot, contig_id, int(ref_start_pos), int(vset),
                                              ctypes.byref(nn), ctypes.byref(pmin), ctypes.byref(pmax)))
    return nn.value, pmin.value, pmax.value

  def build_haplotypes_vset(self, slots, contig_ids, ref_starts, vsets):
    """Several resident-variant haplotypes at once (two side by side); [(n_nodes, p_min, p_max)] per slot."""
    n = len(slots)
    a = lambda xs, t: np.ascontiguousarray(np.asarray(xs, dtype=t))
    s, c, r, v = a(slots, np.int32), a(contig_ids, np.int32), a(ref_starts, np.int64), a(vsets, np.int32)
    nn, pmin, pmax = (np.zeros(max(n, 1), np.int64) for _ in range(3))
    self._chk(self._L.mh_build_haplotypes_vset(self._h, n, _ptr(s), _ptr(c), _ptr(r), _ptr(v), _ptr(nn), _ptr(pmin),
                                               _ptr(pmax)))
    return [(int(nn[i]), int(pmin[i]), int(pmax[i])) for i in range(n)]

  def prefetch_haplotypes_vset(self, slots, contig_ids, ref_starts, vsets, unit_slots=(), unit_seeds=(), p=1.0):
    """build_haplotypes_vset for the next batch, beside the current one (mh_prefetch_haplotypes_vset: returns at once;
    the splices run on the context's prefetch thread and stream, joined before the slots are used); the slots must be
    free.  unit_slots / unit_seeds / p: the next batch's units, whose MT19937 word streams the same thread generates
    for the sample_units call that matches them."""
    n, nu = len(slots), len(unit_slots)
    a = lambda xs, t: np.ascontiguousarray(np.asarray(xs, dtype=t))
    s, c, r, v = a(slots, np.int32), a(contig_ids, np.int32), a(ref_starts, np.int64), a(vsets, np.int32)
    us, ud = a(unit_slots, np.int32), a(unit_seeds, np.uint64)
    self._chk(self._L.mh_prefetch_haplotypes_vset(self._h, n, _ptr(s), _ptr(c), _ptr(r), _ptr(v), nu, _ptr(us),
                                                  _ptr(ud), float(p)))

  def release_variants(self, vset):
    self._chk(self._L.mh_release_variants(self._h, int(vset)))

  def get_nodes(self, slot, n_nodes, with_hap=True):
    ps, pr, ol = (np.empty(max(n_nodes, 1), np.int64) for _ in range(3))
    op = np.empty(max(n_nodes, 1), np.uint8)
    hl = c_i64()
    self._chk(self._L.mh_get_nodes(self._h, slot, None, None, None, None, None, 0, ctypes.byref(hl)))
    hap = np.empty(max(hl.value, 1), np.uint8) if with_hap else None
    self._chk(self._L.mh_get_nodes(self._h, slot, _ptr(ps), _ptr(pr), _ptr(op), _ptr(ol), _ptr(hap),
                                   hl.value if with_hap else 0, ctypes.byref(hl)))
    return ps[:n_nodes], pr[:n_nodes], op[:n_nodes], ol[:n_nodes], (hap[:hl.value].tobytes() if with_hap else None)

  def release_haplotype(self, slot):
    self._chk(self._L.mh_release_haplotype(self._h, slot))

  # ---- templates ---------------------------------------------------------------------------------------
  def sample_templates(self, slot, p, rlen, cum_tlen, seed, rng_mode=MH_RNG_MITTY):
    ct = np.ascontiguousarray(cum_tlen, dtype=np.float64)
    n = c_i64()
    self._chk(self._L.mh_sample_templates(self._h, slot, float(p), int(rlen), _ptr(ct), len(ct), int(seed),
                                          int(rng_mode), ctypes.byref(n)))
    return n.value

  def sample_templates_span(self, p_min, p_max, p, rlen, cum_tlen, seed, rng_mode=MH_RNG_MITTY):
    if not (0 <= int(seed) <= 0xffffffff):
      raise ValueError('Seed value {} is out of range 0 - {}'.format(seed, 0xffffffff))
    ct = np.ascontiguousarray(cum_tlen, dtype=np.float64)
    n = c_i64()
    self._chk(self._L.mh_sample_templates_span(self._h, int(p_min), int(p_max), float(p), int(rlen), _ptr(ct),
                                               len(ct), int(seed), int(rng_mode), ctypes.byref(n)))
    return n.value

  def sample_units(self, tpl_ids, slots, seeds, p, rlen, cum_tlen, rng_mode=MH_RNG_MITTY):
    """Batched sampling; returns templates kept per unit."""
    ids = np.ascontiguousarray(tpl_ids, dtype=np.int32)
    sl = np.ascontiguousarray(slots, dtype=np.int32)
    sd = np.ascontiguousarray(seeds, dtype=np.uint64)
    ct = np.ascontiguousarray(cum_tlen, dtype=np.float64)
    out = np.zeros(max(len(ids), 1), dtype=np.int64)
    self._chk(self._L.mh_sample_units(self._h, len(ids), _ptr(ids), _ptr(sl), _ptr(sd), float(p), int(rlen),
                                      _ptr(ct), len(ct), int(rng_mode), _ptr(out)))
    return out[:len(ids)]

  def sample_units_async(self, tpl_ids, slots, seeds, p, rlen, cum_tlen, rng_mode=MH_RNG_MITTY):
    """sample_units whose per-unit tails run on without a host wait; template_count(id) (or use_templates) waits
    for one unit."""
    ids = np.ascontiguousarray(tpl_ids, dtype=np.int32)
    sl = np.ascontiguousarray(slots, dtype=np.int32)
    sd = np.ascontiguousarray(seeds, dtype=np.uint64)
    ct = np.ascontiguousarray(cum_tlen, dtype=np.float64)
    self._chk(self._L.mh_sample_units_async(self._h, len(ids), _ptr(ids), _ptr(sl), _ptr(sd), float(p), int(rlen),
                                            _ptr(ct), len(ct), int(rng_mode)))
    return len(ids)

  def template_count(self, tpl_id):
    n = c_i64()
    self._chk(self._L.mh_templates_count(self._h, int(tpl_id), ctypes.byref(n)))
    return n.value

  def use_templates(self, tpl_id):
    self._chk(self._L.mh_use_templates(self._h, int(tpl_id)))

  def release_templates(self, tpl_id):
    self._chk(self._L.mh_release_templates(self._h, int(tpl_id)))

  def set_emit_mode(self, mode):
    """0: default (the single-pass writer for emit_async, measure pass + direct writer for emit_reads), 1: LDS-image
    writer, 2: never the single-pass writer (the two-pass path)."""
    self._chk(self._L.mh_set_emit_mode(self._h, int(mode)))

  def set_decode_mode(self, mode):
    """0: chunk-parallel shuffle decode (default), 1: block-sequential decode."""
    self._chk(self._L.mh_set_decode_mode(self._h, int(mode)))

  def fixup_count(self):
    n = c_i64()
    self._chk(self._L.mh_fixup_count(self._h, ctypes.byref(n)))
    return n.value

  def set_templates(self, fo0, pos0, pos1, rlen):
    fo0 = np.ascontiguousarray(fo0, dtype=np.int8)
    pos0 = np.ascontiguousarray(pos0, dtype=np.int64)
    pos1 = np.ascontiguousarray(pos1, dtype=np.int64)
    self._chk(self._L.mh_set_templates(self._h, _ptr(fo0), _ptr(pos0), _ptr(pos1), len(fo0), int(rlen)))

  def get_templates(self):
    n = c_i64()
    self._L.mh_get_templates(self._h, None, None, None, 0, ctypes.byref(n))
    m = n.value
    fo0, p0, p1 = np.empty(max(m, 1), np.int8), np.empty(max(m, 1), np.int64), np.empty(max(m, 1), np.int64)
    self._chk(self._L.mh_get_templates(self._h, _ptr(fo0), _ptr(p0), _ptr(p1), max(m, 1), ctypes.byref(n)))
    return fo0[:m], p0[:m], p1[:m]

  # ---- emission ----------------------------------------------------------------------------------------
  def emit_prepare(self, slot, serial_stub, chrom, cpy, write_fastq2=True, unit_key=0, wait=True):
    """The measure pass and record offsets of the current templates (the next emit_reads of the same unit only
    queues the writer).  Returns (kept, bytes1, bytes2); with wait=False it returns None at once, without waiting
    for the pass (emit_reads reads its totals)."""
    if not wait:
      self._chk(self._L.mh_emit_prepare(self._h, slot, serial_stub.encode(), chrom.encode(), int(cpy),
                                        1 if write_fastq2 else 0, int(unit_key), None, None, None))
      return None
    k, b1, b2 = c_i64(), c_i64(), c_i64()
    self._chk(self._L.mh_emit_prepare(self._h, slot, serial_stub.encode(), chrom.encode(), int(cpy),
                                      1 if write_fastq2 else 0, int(unit_key), ctypes.byref(k), ctypes.byref(b1),
                                      ctypes.byref(b2)))
    return k.value, b1.value, b2.value

  def emit_reads(self, slot, serial_stub, chrom, cpy, write_fastq2=True, unit_key=0, t_range=None, cnt_base=0):
    """Emit the current templates (or the slice t_range = (t_begin, t_end), kept ones numbered from cnt_base + 1).
    Returns (kept, bytes1, bytes2)."""
    k, b1, b2 = c_i64(), c_i64(), c_i64()
    if t_range is None:
      self._chk(self._L.mh_emit_reads(self._h, slot, serial_stub.encode(), chrom.encode(), int(cpy),
                                      1 if write_fastq2 else 0, int(unit_key), ctypes.byref(k), ctypes.byref(b1),
                                      ctypes.byref(b2)))
    else:
      self._chk(self._L.mh_emit_reads_range(self._h, slot, serial_stub.encode(), chrom.encode(), int(cpy),
                                            1 if write_fastq2 else 0, int(unit_key), int(t_range[0]),
                                            int(t_range[1]), int(cnt_base), ctypes.byref(k), ctypes.byref(b1),
                                            ctypes.byref(b2)))
    return k.value, b1.value, b2.value

  def emit_async(self, slot, serial_stub, chrom, cpy, write_fastq2=True, unit_key=0):
    """Queue the emission of the whole current template set (mh_emit_reads_async: the single-pass writer, no host
    wait); emit_collect returns its (kept, bytes1, bytes2) with those of the other queued units."""
    self._chk(self._L.mh_emit_reads_async(self._h, slot, serial_stub.encode(), chrom.encode(), int(cpy),
                                          1 if write_fastq2 else 0, int(unit_key)))

  def emit_collect(self):
    """Wait for the queued emissions; [(kept, bytes1, bytes2)] per unit, in queue order."""
    n = c_i64()
    self._chk(self._L.mh_emit_collect(self._h, None, 0, ctypes.byref(n)))
    out = np.zeros(3 * max(n.value, 1), np.int64)
    self._chk(self._L.mh_emit_collect(self._h, _ptr(out), n.value, ctypes.byref(n)))
    return [tuple(int(x) for x in out[3 * i:3 * i + 3]) for i in range(n.value)]

  def emit_measure(self, slot, serial_stub, chrom, cpy, write_fastq2=True, unit_key=0, t_range=None, cnt_base=0):
    """(kept, bytes1, bytes2) that emit_reads with the same arguments will produce, without writing anything."""
    k, b1, b2 = c_i64(), c_i64(), c_i64()
    t0, t1 = t_range if t_range is not None else (0, -1)
    self._chk(self._L.mh_emit_measure(self._h, slot, serial_stub.encode(), chrom.encode(), int(cpy),
                                      1 if write_fastq2 else 0, int(unit_key), int(t0), int(t1), int(cnt_base),
                                      ctypes.byref(k), ctypes.byref(b1), ctypes.byref(b2)))
    return k.value, b1.value, (b2.value if write_fastq2 else 0)

  def bgzf_range(self, f, off, n, pin):
    """Arena bytes [off, off + n) of file f BGZF-compressed on the GPU (mh_output_bgzf_range) into the page-locked
    buffer pin; returns the compressed bytes (no EOF marker)."""
    if n <= 0:
      return b''
    cap = n + (n // 0xff00 + 2) * 40 + 64
    pin.reserve(cap)
    used = c_i64()
    self._chk(self._L.mh_output_bgzf_range(self._h, int(f), int(off), int(n), c_vp(pin.ptr), cap, ctypes.byref(used)))
    return bytes(pin.view(used.value))

  def count_kept(self, slot, t_begin, t_end):
    """Templates of the current set in [t_begin, t_end) that pass the N filter."""
    k = c_i64()
    self._chk(self._L.mh_count_kept(self._h, slot, int(t_begin), int(t_end), ctypes.byref(k)))
    return k.value

  def output_size(self):
    a, b = c_i64(), c_i64()
    self._chk(self._L.mh_output_size(self._h, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value

  def fetch_output(self, off1=0, len1=None, off2=0, len2=None):
    u1, u2 = self.output_size()
    len1 = u1 - off1 if len1 is None else len1
    len2 = u2 - off2 if len2 is None else len2
    b1 = np.empty(max(len1, 1), np.uint8)
    b2 = np.empty(max(len2, 1), np.uint8)
    self._chk(self._L.mh_output_fetch(self._h, off1, _ptr(b1), len1, off2, _ptr(b2) if len2 > 0 else None, len2))
    return b1[:len1].tobytes(), b2[:len2].tobytes()

  def fetch_output_arrays(self, off1, len1, off2, len2):
    """The same ranges as uint8 arrays (no bytes copy)."""
    b1 = np.empty(max(len1, 1), np.uint8)
    b2 = np.empty(max(len2, 1), np.uint8)
    self._chk(self._L.mh_output_fetch(self._h, off1, _ptr(b1), len1, off2, _ptr(b2) if len2 > 0 else None, len2))
    return b1[:len1], b2[:len2]

  def stream_output(self, sinks, pin, chunk=256 << 20):
    """Both arenas to the sinks (file-like objects; None skips a file) through one page-locked staging buffer,
    `chunk` bytes per copy."""
    u = self.output_size()
    pin.reserve(min(chunk, max(u)) if max(u) else 1)
    for f in (0, 1):
      if sinks[f] is None:
        continue
      for off in range(0, u[f], chunk):
        n = min(chunk, u[f] - off)
        if f == 0:
          self._chk(self._L.mh_output_fetch(self._h, off, c_vp(pin.ptr), n, 0, None, 0))
        else:
          self._chk(self._L.mh_output_fetch(self._h, 0, None, 0, off, c_vp(pin.ptr), n))
        sinks[f].write(pin.view(n))

  def fetch_range_pinned(self, pins, off1, n1, off2, n2):
    """Arena bytes [off1, off1 + n1) of file 1 and [off2, off2 + n2) of file 2 into page-locked staging (pins:
    [PinnedBuffer, PinnedBuffer], grown as needed); returns memoryviews of them (valid until the next fetch)."""
    pins[0].reserve(max(n1, 1))
    pins[1].reserve(max(n2, 1))
    self._chk(self._L.mh_output_fetch(self._h, off1, c_vp(pins[0].ptr) if n1 > 0 else None, n1, off2,
                                      c_vp(pins[1].ptr) if n2 > 0 else None, n2))
    return pins[0].view(n1), pins[1].view(n2)

  def fetch_range_async(self, pins, off1, n1, off2, n2):
    """fetch_range_pinned without the wait: returns (ticket, memoryviews); the bytes are in after
    fetch_wait(ticket)."""
    pins[0].reserve(max(n1, 1))
    pins[1].reserve(max(n2, 1))
    t = c_i32()
    self._chk(self._L.mh_output_fetch_async(self._h, off1, c_vp(pins[0].ptr) if n1 > 0 else None, n1, off2,
                                            c_vp(pins[1].ptr) if n2 > 0 else None, n2, ctypes.byref(t)))
    return t.value, (pins[0].view(n1), pins[1].view(n2))

  def fetch_wait(self, ticket):
    self._chk(self._L.mh_output_fetch_wait(self._h, int(ticket)))

  def fetch_output_pinned(self, pins):
    """The whole arenas into page-locked staging (pins: [PinnedBuffer, PinnedBuffer], grown as needed); returns
    memoryviews of the bytes (valid until the next fetch)."""
    u1, u2 = self.output_size()
    pins[0].reserve(u1)
    pins[1].reserve(u2)
    self._chk(self._L.mh_output_fetch(self._h, 0, c_vp(pins[0].ptr), u1, 0, c_vp(pins[1].ptr) if u2 > 0 else None,
                                      u2))
    return pins[0].view(u1), pins[1].view(u2)

  def reset_output(self):
    self._chk(self._L.mh_output_reset(self._h))

  def bgzf_compress(self, data):
    """BGZF members of `data` deflated on the GPU (no EOF marker; mh_bgzf_compress_gpu)."""
    n = len(data)
    if n == 0:
      return b''
    src = np.frombuffer(data, np.uint8)
    out = np.empty(n + (n // 0xff00 + 2) * 40 + 64, np.uint8)
    used = c_i64()
    self._chk(self._L.mh_bgzf_compress_gpu(self._h, _ptr(src), n, _ptr(out), len(out), ctypes.byref(used)))
    return out[:used.value].tobytes()

  def output_bgzf_range_pinned(self, pins, off, n1, n2):
    """Arena bytes [off, off + n_f) of each file BGZF-compressed on the GPU into page-locked staging (pins:
    [PinnedBuffer, PinnedBuffer]); returns memoryviews of the compressed bytes (no EOF marker)."""
    out = []
    for f, n in enumerate((n1, n2)):
      if n <= 0:
        out.append(memoryview(b''))
        continue
      cap = n + (n // 0xff00 + 2) * 40 + 64   # every block stored, at worst
      pins[f].reserve(cap)
      used = c_i64()
      self._chk(self._L.mh_output_bgzf_range(self._h, f, off, n, c_vp(pins[f].ptr), cap, ctypes.byref(used)))
      out.append(pins[f].view(used.value))
    return out

  def output_bgzf_pair(self, pins, off, n1, n2):
    """Both arenas' [off, off + n_f) BGZF-compressed on the GPU, the compressed bytes copied into page-locked staging
    (pins: [PinnedBuffer, PinnedBuffer]) behind the deflates: returns (ticket, memoryviews) at once; the views hold
    the bytes after output_bgzf_wait(ticket)."""
    caps = []
    for f, n in enumerate((n1, n2)):
      cap = n + (n // 0xff00 + 2) * 40 + 64 if n > 0 else 0   # every block stored, at worst
      pins[f].reserve(max(cap, 1))
      caps.append(cap)
    u1, u2, t = c_i64(), c_i64(), c_i32()
    self._chk(self._L.mh_output_bgzf_pair(self._h, int(off), int(n1), int(n2), c_vp(pins[0].ptr) if n1 > 0 else None,
                                          caps[0], c_vp(pins[1].ptr) if n2 > 0 else None, caps[1], ctypes.byref(u1),
                                          ctypes.byref(u2), ctypes.byref(t)))
    return t.value, [pins[0].view(u1.value), pins[1].view(u2.value)]

  def output_bgzf_wait(self, ticket):
    self._chk(self._L.mh_output_bgzf_wait(self._h, int(ticket)))

  def output_bgzf_pinned(self, pins):
    """Both arenas BGZF-compressed on the GPU into page-locked staging (pins: [PinnedBuffer, PinnedBuffer]);
    returns memoryviews of the compressed bytes (no EOF marker)."""
    out = []
    for f, u in enumerate(self.output_size()):
      cap = u + (u // 0xff00 + 2) * 40 + 64   # every block stored, at worst
      pins[f].reserve(cap)
      used = c_i64()
      self._chk(self._L.mh_output_bgzf(self._h, f, c_vp(pins[f].ptr), cap, ctypes.byref(used)))
      out.append(pins[f].view(used.value))
    return out

  # ---- god-aligner BAM ----
  def bam_set_refs(self, names, lengths):
    blob = b''.join(n.encode() + b'\0' for n in names)
    ln = np.ascontiguousarray(lengths, dtype=np.int64)
    self._chk(self._L.mh_bam_set_refs(self._h, len(names), blob, _ptr(ln) if len(names) else None))

  def bam_add_fastq(self, fq1, fq2=None, max_templates=-1):
    """Parse the complete templates of FASTQ byte buffers into BAM records.  Returns (used1, used2, templates)."""
    u1, u2, t = c_i64(), c_i64(), c_i64()
    a1 = np.frombuffer(fq1, np.uint8) if len(fq1) else np.zeros(1, np.uint8)
    a2 = None if fq2 is None else (np.frombuffer(fq2, np.uint8) if len(fq2) else np.zeros(1, np.uint8))
    self._chk(self._L.mh_bam_add_fastq(self._h, _ptr(a1), len(fq1), None if a2 is None else _ptr(a2),
                                       0 if fq2 is None else len(fq2), int(max_templates), ctypes.byref(u1),
                                       ctypes.byref(u2), ctypes.byref(t)))
    return u1.value, u2.value, t.value

  def bam_add_output(self, max_templates=-1):
    t = c_i64()
    self._chk(self._L.mh_bam_add_output(self._h, int(max_templates), ctypes.byref(t)))
    return t.value

  def bam_set_capacity(self, nbytes):
    """HBM budget of the BAM record store (0: no limit); records past it spill to host memory."""
    self._chk(self._L.mh_bam_set_capacity(self._h, int(nbytes)))

  def bam_set_spill_dir(self, path):
    """Spill to unlinked temporary files in `path` (None: host memory)."""
    self._chk(self._L.mh_bam_set_spill_dir(self._h, None if path is None else path.encode()))

  def bam_spilled(self):
    """(bytes, host blocks) of the record store spilled to host memory."""
    b, k = c_i64(), c_i64()
    self._chk(self._L.mh_bam_spilled(self._h, ctypes.byref(b), ctypes.byref(k)))
    return b.value, k.value

  def bam_export(self, r0, r1, nbytes, ptr=None):
    """Records [r0, r1) of the store (nbytes of record bytes) packed (bam_piece_layout) at address ptr (host or
    device), or into a new uint8 array (returned)."""
    n = int(r1 - r0)
    o_roff, o_key, o_info, total = bam_piece_layout(n, nbytes)
    out = None
    if ptr is None:
      out = np.empty(max(total, 8), np.uint8)
      ptr = out.ctypes.data
    self._chk(self._L.mh_bam_export(self._h, int(r0), int(r1), c_vp(ptr), c_vp(ptr + o_roff), c_vp(ptr + o_key),
                                    c_vp(ptr + o_info)))
    return out

  def bam_import(self, n, nbytes, ptr):
    """Append a packed piece (bam_export's layout) at address ptr (host or device) to the store."""
    o_roff, o_key, o_info, _ = bam_piece_layout(n, nbytes)
    self._chk(self._L.mh_bam_import(self._h, c_vp(ptr), c_vp(ptr + o_roff), c_vp(ptr + o_key), c_vp(ptr + o_info),
                                    int(n)))

  def bam_records(self):
    n, b = c_i64(), c_i64()
    self._chk(self._L.mh_bam_records(self._h, ctypes.byref(n), ctypes.byref(b)))
    return n.value, b.value

  def bam_write(self, bam_path, header_text, level=6, threads=4, bai_path=None):
    n, b = c_i64(), c_i64()
    h = header_text.encode()
    self._chk(self._L.mh_bam_write(self._h, bam_path.encode(), h, len(h), int(level), int(threads),
                                   None if bai_path is None else bai_path.encode(), ctypes.byref(n), ctypes.byref(b)))
    return n.value, b.value

  def bam_write_gpu(self, bam_path, header_text, bai_path=None):
    """mh_bam_write with the record blocks deflated on the device.  Returns (records, record bytes, file bytes)."""
    n, b, fb = c_i64(), c_i64(), c_i64()
    h = header_text.encode()
    self._chk(self._L.mh_bam_write_gpu(self._h, bam_path.encode(), h, len(h),
                                       None if bai_path is None else bai_path.encode(), ctypes.byref(n),
                                       ctypes.byref(b), ctypes.byref(fb)))
    return n.value, b.value, fb.value

  def bam_reset(self):
    self._chk(self._L.mh_bam_reset(self._h))

  def bam_partition(self, splitters, tie_base):
    """The store's records by destination rank (mh_bam_partition): returns (segment offsets [n_dest + 1], records
    [n_dest], record bytes [n_dest]); the packed segments stay in the library until bam_partition_fetch."""
    sp = np.ascontiguousarray(splitters, dtype=np.uint64)
    nd = len(sp) + 1
    off, n, nb = np.zeros(nd + 1, np.int64), np.zeros(nd, np.int64), np.zeros(nd, np.int64)
    self._chk(self._L.mh_bam_partition(self._h, _ptr(sp) if len(sp) else None, nd, int(tie_base), _ptr(off), _ptr(n),
                                       _ptr(nb)))
    return off, n, nb

  def bam_partition_fetch(self, ptr, cap):
    """The packed segments to address ptr (host or device memory, cap bytes)."""
    self._chk(self._L.mh_bam_partition_fetch(self._h, c_vp(ptr), int(cap)))

  def bam_import_tie(self, n, nbytes, ptr):
    """Append a segment of mh_bam_partition (bam_part_layout) at address ptr (host or device) with its ties."""
    o_roff, o_key, o_info, o_tie, _ = bam_part_layout(n, nbytes)
    self._chk(self._L.mh_bam_import_tie(self._h, c_vp(ptr), c_vp(ptr + o_roff), c_vp(ptr + o_key),
                                        c_vp(ptr + o_info), c_vp(ptr + o_tie), int(n)))

  def bam_sorted_head(self, n):
    out = np.empty(max(int(n), 1), np.uint8)
    self._chk(self._L.mh_bam_sorted_head(self._h, int(n), _ptr(out)))
    return out[:int(n)].tobytes()

  def bam_write_part(self, path, header_text=None, skip=0, tail=b'', eof=False):
    """The sorted stream from `skip` plus `tail`, as BGZF blocks deflated on the device, to `path` (mh_bam_write_part).
    Returns (blocks, data_pos, file bytes, block offsets [blocks + 1] from data_pos)."""
    nb, dp, fb = c_i64(), c_i64(), c_i64()
    h = header_text.encode() if header_text is not None else b''
    t = np.frombuffer(tail, np.uint8) if len(tail) else None
    args = (self._h, path.encode(), h, len(h) if header_text is not None else -1, int(skip), _ptr(t), len(tail),
            1 if eof else 0, ctypes.byref(nb), ctypes.byref(dp), ctypes.byref(fb))
    n_bytes = self.bam_records()[1]
    cap = (n_bytes - int(skip) + len(tail)) // 0xff00 + 2
    boff = np.zeros(cap, np.int64)
    self._chk(self._L.mh_bam_write_part(*args, _ptr(boff), cap))
    return nb.value, dp.value, fb.value, boff[:nb.value + 1]

  def bam_bai_runs(self, n_refs):
    """The BAI's raw plan of the sorted store (mh_bam_bai_runs): (runs int64 [n_runs, 4], windows int64 [n_win],
    per-reference window counts)."""
    nr, nw = c_i64(), c_i64()
    self._chk(self._L.mh_bam_bai_runs(self._h, ctypes.byref(nr), None, 0, ctypes.byref(nw), None, 0, None))
    runs = np.zeros(max(4 * nr.value, 4), np.int64)
    win = np.zeros(max(nw.value, 1), np.int64)
    rn = np.zeros(max(n_refs, 1), np.int64)
    self._chk(self._L.mh_bam_bai_runs(self._h, ctypes.byref(nr), _ptr(runs), len(runs), ctypes.byref(nw), _ptr(win),
                                      len(win), _ptr(rn)))
    return runs[:4 * nr.value].reshape(-1, 4), win[:nw.value], rn[:n_refs]

  def bam_sort(self):
    """Coordinate-sort the record store in HBM (mh_bam_write reuses the result)."""
    self._chk(self._L.mh_bam_sort(self._h))

  def corrupt_fastq(self, fq1, fq2=None, t_base=0):
    """Corrupt the complete templates of FASTQ byte buffers into the arenas.  Returns (used1, used2, templates)."""
    u1, u2, t = c_i64(), c_i64(), c_i64()
    a1 = np.frombuffer(fq1, np.uint8) if len(fq1) else np.zeros(1, np.uint8)
    a2 = None if fq2 is None else (np.frombuffer(fq2, np.uint8) if len(fq2) else np.zeros(1, np.uint8))
    self._chk(self._L.mh_corrupt_fastq(self._h, _ptr(a1), len(fq1), None if a2 is None else _ptr(a2),
                                       0 if fq2 is None else len(fq2), int(t_base), ctypes.byref(u1),
                                       ctypes.byref(u2), ctypes.byref(t)))
    return u1.value, u2.value, t.value

  def read_batch(self, slot, p, l):
    p = np.ascontiguousarray(p, dtype=np.int64)
    l = np.ascontiguousarray(l, dtype=np.int64)
    n = len(p)
    pos, n0, n1 = (np.empty(max(n, 1), np.int64) for _ in range(3))
    offs = [np.empty(n + 1, np.int64) for _ in range(3)]
    used = [c_i64() for _ in range(3)]
    caps = [max(64, 64 * n), max(64, 16 * n), max(64, int(l.sum()) + 16 if n else 64)]
    for _ in range(2):
      bufs = [np.empty(c, np.uint8) for c in caps]
      rc = self._L.mh_read_batch(self._h, slot, _ptr(p), _ptr(l), n, _ptr(pos), _ptr(n0), _ptr(n1),
                                 _ptr(bufs[0]), caps[0], _ptr(offs[0]), ctypes.byref(used[0]),
                                 _ptr(bufs[1]), caps[1], _ptr(offs[1]), ctypes.byref(used[1]),
                                 _ptr(bufs[2]), caps[2], _ptr(offs[2]), ctypes.byref(used[2]))
      if rc == MH_E_CAPACITY:
        caps = [max(c, u.value + 16) for c, u in zip(caps, used)]
        continue
      self._chk(rc)
      break
    texts = [b[:u.value].tobytes().decode('latin-1') for b, u in zip(bufs, used)]
    return pos[:n], n0[:n], n1[:n], texts, offs

  def set_corruption(self, enable, cum_bq=None, phred_p=None, seed=0):
    if not enable:
      self._chk(self._L.mh_set_corruption(self._h, 0, None, 0, 0, None, 0))
      return
    cb = np.ascontiguousarray(cum_bq, dtype=np.float64)
    ph = np.ascontiguousarray(phred_p, dtype=np.float64)
    self._chk(self._L.mh_set_corruption(self._h, 1, _ptr(cb), cb.shape[1], cb.shape[2], _ptr(ph), int(seed)))

  def templates_export(self, tpl_id, fo0=None, pos0=None, pos1=None, cap=None):
    """Template set tpl_id's arrays.  With device pointers (ints) fo0/pos0/pos1 and cap: copied there on the device,
    returns n; without: returns host arrays (fo0, pos0, pos1)."""
    n = c_i64()
    if fo0 is not None:
      self._chk(self._L.mh_templates_export(self._h, int(tpl_id), 1, c_vp(fo0), c_vp(pos0), c_vp(pos1), int(cap),
                                            ctypes.byref(n)))
      return n.value
    self._L.mh_templates_export(self._h, int(tpl_id), 0, None, None, None, 0, ctypes.byref(n))
    m = n.value
    a, b, c = np.empty(max(m, 1), np.int8), np.empty(max(m, 1), np.int64), np.empty(max(m, 1), np.int64)
    self._chk(self._L.mh_templates_export(self._h, int(tpl_id), 0, _ptr(a), _ptr(b), _ptr(c), max(m, 1),
                                          ctypes.byref(n)))
    return a[:m], b[:m], c[:m]

  def templates_import(self, tpl_id, n, rlen, fo0, pos0, pos1, on_device=False):
    """Template set tpl_id := n templates from host arrays, or from device pointers (ints) with on_device."""
    if on_device:
      self._chk(self._L.mh_templates_import(self._h, int(tpl_id), 1, c_vp(fo0), c_vp(pos0), c_vp(pos1), int(n),
                                            int(rlen)))
      return
    a = np.ascontiguousarray(fo0, dtype=np.int8)
    b = np.ascontiguousarray(pos0, dtype=np.int64)
    c = np.ascontiguousarray(pos1, dtype=np.int64)
    self._chk(self._L.mh_templates_import(self._h, int(tpl_id), 0, _ptr(a), _ptr(b), _ptr(c), int(n), int(rlen)))

  def set_corruption_stream(self, rng_mode, seed=0, key=None, pos=624):
    """mh_corrupt_fastq's word source: MH_RNG_PHILOX, or MH_RNG_MITTY = the reference's exact MT19937 stream
    (RandomState(seed) from its first word, or continuing an explicit numpy state (key uint32[624], pos))."""
    k = None if key is None else np.ascontiguousarray(key, dtype=np.uint32)
    if k is not None and k.shape != (624,):
      raise ValueError('MT19937 key must hold 624 words')
    self._chk(self._L.mh_set_corruption_stream(self._h, int(rng_mode), int(seed), None if k is None else _ptr(k),
                                               int(pos)))

  def get_corruption_stream(self):
    """(key uint32[624], pos, words consumed or -1) of the exact corruption stream."""
    key = np.empty(624, np.uint32)
    pos, words = c_i32(), c_i64()
    self._chk(self._L.mh_get_corruption_stream(self._h, _ptr(key), ctypes.byref(pos), ctypes.byref(words)))
    return key, pos.value, words.value

  def enable_timing(self, on=True):
    self._chk(self._L.mh_enable_timing(self._h, 1 if on else 0))

  def stage_times(self):
    n = c_i32()
    self._L.mh_stage_times(self._h, None, None, 0, ctypes.byref(n))
    names = (ctypes.c_char_p * max(n.value, 1))()
    ms = (c_dbl * max(n.value, 1))()
    self._L.mh_stage_times(self._h, names, ms, n.value, ctypes.byref(n))
    return [(names[i].decode(), ms[i]) for i in range(n.value)]

  def sync(self):
    self._chk(self._L.mh_sync(self._h))

  def selftest_sort(self, keys, end_bit):
    """mh_selftest_sort: (sorted keys, input indices) of a u32 array by the library's LSD radix sort."""
    import numpy as np
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    ko, vo = np.empty_like(k), np.empty_like(k)
    self._chk(self._L.mh_selftest_sort(self._h, k.ctypes.data, k.size, int(end_bit), ko.ctypes.data, vo.ctypes.data))
    return ko, vo

  def selftest_scan_fault(self):
    """(return code, message) of mh_selftest_scan_fault: MH_E_STATE when a timed-out look-back scan is reported."""
    rc = self._L.mh_selftest_scan_fault(self._h)
    return rc, self._L.mh_last_error(self._h).decode(errors='replace')


def expand_variant(samp_pos, ref_pos, ref_start_pos, v_pos, op, oplen):
  """mh_expand_variant: ([(ps, pr, op, oplen, src)], samp_next, ref_next) for one variant at the given cursors."""
  out = (c_i64 * 10)()
  n, sn, rn = c_i32(), c_i64(), c_i64()
  rc = lib().mh_expand_variant(int(samp_pos), int(ref_pos), int(ref_start_pos), int(v_pos), ord(op), int(oplen), out,
                               ctypes.byref(n), ctypes.byref(sn), ctypes.byref(rn))
  if rc:
    _raise(rc, 'mh_expand_variant: bad variant (op {!r}, oplen {})'.format(op, oplen))
  return [(out[5 * j], out[5 * j + 1], chr(out[5 * j + 2]), out[5 * j + 3], out[5 * j + 4])
          for j in range(n.value)], sn.value, rn.value
